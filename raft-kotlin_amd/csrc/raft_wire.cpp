// raft_wire.cpp — batched proto3 wire codec of greeter.proto:16-44 (host code).
// See include/raft_wire.h for the contract.  Plain loops over the batch: the
// codec is a per-message byte scanner with no arithmetic worth a device.
#include "../../include/raft_wire.h"

#include <string>

int raft_internal_fail(int code, const std::string& msg);   // raft_engine.hip: sets raft_last_error()

namespace {

enum : uint32_t { WT_VARINT = 0, WT_I64 = 1, WT_LEN = 2, WT_SGROUP = 3, WT_EGROUP = 4, WT_I32 = 5 };

// ---- decoding --------------------------------------------------------------
struct Reader {
    const uint8_t* p;
    const uint8_t* end;
    bool ok = true;

    bool more() const { return ok && p < end; }
    uint64_t varint() {
        uint64_t v = 0;
        for (int s = 0; s < 70; s += 7) {
            if (p >= end) { ok = false; return 0; }
            const uint8_t b = *p++;
            if (s == 63 && b > 1) { ok = false; return 0; }        // more than 64 bits
            v |= (uint64_t)(b & 0x7F) << s;
            if (!(b & 0x80)) return v;
        }
        ok = false;
        return 0;
    }
    // skips the value of a field of wire type wt (unknown field)
    void skip(uint32_t wt) {
        switch (wt) {
            case WT_VARINT: varint(); break;
            case WT_I64: if (end - p < 8) ok = false; else p += 8; break;
            case WT_I32: if (end - p < 4) ok = false; else p += 4; break;
            case WT_LEN: {
                const uint64_t len = varint();
                if (!ok || len > (uint64_t)(end - p)) ok = false; else p += len;
                break;
            }
            default: ok = false;                                      // groups (deprecated) and 6/7
        }
    }
    // the next field's number and wire type; false at the end or on error
    bool field(uint32_t& num, uint32_t& wt) {
        if (!more()) return false;
        const uint64_t key = varint();
        if (!ok) return false;
        num = (uint32_t)(key >> 3);
        wt = (uint32_t)(key & 7);
        if (num == 0) { ok = false; return false; }
        return true;
    }
    // a length-delimited field's payload
    bool bytes(const uint8_t*& b, uint64_t& len) {
        len = varint();
        if (!ok || len > (uint64_t)(end - p)) { ok = false; return false; }
        b = p;
        p += len;
        return true;
    }
};

int32_t as_int32(uint64_t v) { return (int32_t)(uint32_t)v; }           // proto3 int32: low 32 bits

int bad_message(const char* what, int64_t m) {
    return raft_internal_fail(RAFT_EINVAL, std::string("malformed ") + what + " at message " + std::to_string(m));
}

int check_batch(const uint8_t* buf, const int64_t* off, int64_t n, const void* out) {
    if (n < 0) return raft_internal_fail(RAFT_EINVAL, "negative batch");
    if (n > 0 && (!buf || !off || !out)) return raft_internal_fail(RAFT_EINVAL, "null buffer");
    for (int64_t m = 0; m < n; ++m)
        if (off[m] < 0 || off[m + 1] < off[m])
            return raft_internal_fail(RAFT_EINVAL, "offsets must be non-decreasing from 0");
    return RAFT_OK;
}

// decodes messages whose fields are all varint scalars: setter(msg, field, value)
template <class T, class Set>
int decode_scalars(const uint8_t* buf, const int64_t* off, int64_t n, T* out, const char* what, Set set) {
    if (int rc = check_batch(buf, off, n, out)) return rc;
    for (int64_t m = 0; m < n; ++m) {
        T x{};
        Reader r{buf + off[m], buf + off[m + 1]};
        uint32_t num, wt;
        while (r.field(num, wt)) {
            if (wt == WT_VARINT && set(x, num, 0, false)) {
                const uint64_t v = r.varint();
                if (r.ok) set(x, num, v, true);
            } else {
                r.skip(wt);
            }
        }
        if (!r.ok) return bad_message(what, m);
        out[m] = x;
    }
    return RAFT_OK;
}

// ---- encoding --------------------------------------------------------------
int varint_size(uint64_t v) {
    int s = 1;
    while (v >= 0x80) { v >>= 7; ++s; }
    return s;
}
uint64_t int32_wire(int32_t v) { return (uint64_t)(int64_t)v; }          // negative: 10-byte sign extension

struct Writer {
    uint8_t* buf;
    int64_t cap, pos = 0;
    bool ok = true;

    void byte(uint8_t b) {
        if (pos < cap) buf[pos] = b; else ok = false;
        ++pos;
    }
    void varint(uint64_t v) {
        while (v >= 0x80) { byte((uint8_t)(v | 0x80)); v >>= 7; }
        byte((uint8_t)v);
    }
    void key(uint32_t num, uint32_t wt) { varint((uint64_t)num << 3 | wt); }
    void int32_field(uint32_t num, int32_t v) {                         // default 0 omitted
        if (v != 0) { key(num, WT_VARINT); varint(int32_wire(v)); }
    }
    void bool_field(uint32_t num, int32_t v) {
        if (v != 0) { key(num, WT_VARINT); byte(1); }
    }
    void bytes_field(uint32_t num, const uint8_t* b, int64_t len) {    // empty string omitted
        if (len <= 0) return;
        key(num, WT_LEN);
        varint((uint64_t)len);
        for (int64_t i = 0; i < len; ++i) byte(b[i]);
    }
};

int32_t int32_field_size(uint32_t num, int32_t v) {
    return v != 0 ? varint_size((uint64_t)num << 3) + varint_size(int32_wire(v)) : 0;
}

template <class T, class Emit>
int64_t encode_batch(const T* in, int64_t n, uint8_t* buf, int64_t cap, int64_t* off, Emit emit) {
    if (n < 0 || cap < 0) return raft_internal_fail(RAFT_EINVAL, "negative batch or capacity");
    if (n > 0 && (!in || !off || (cap > 0 && !buf))) return raft_internal_fail(RAFT_EINVAL, "null buffer");
    Writer w{buf, cap};
    for (int64_t m = 0; m < n; ++m) {
        off[m] = w.pos;
        emit(w, m);
    }
    if (n > 0) off[n] = w.pos;
    if (!w.ok) return raft_internal_fail(RAFT_ERANGE, "output buffer too small: " + std::to_string(w.pos) +
                                                          " bytes needed");
    return w.pos;
}

}  // namespace

extern "C" {

int raft_wire_decode_vote_req(const uint8_t* buf, const int64_t* off, int64_t n, raft_vote_req* out) {
    return decode_scalars(buf, off, n, out, "RequestVoteRPC", [](raft_vote_req& x, uint32_t f, uint64_t v, bool put) {
        int32_t* dst = f == 1 ? &x.term : f == 2 ? &x.candidate_id : f == 3 ? &x.last_log_index
                     : f == 4 ? &x.last_log_term : nullptr;
        if (put && dst) *dst = as_int32(v);
        return dst != nullptr;
    });
}

int raft_wire_decode_vote_resp(const uint8_t* buf, const int64_t* off, int64_t n, raft_vote_resp* out) {
    return decode_scalars(buf, off, n, out, "ResponseVoteRPC", [](raft_vote_resp& x, uint32_t f, uint64_t v, bool put) {
        if (put && f == 1) x.term = as_int32(v);
        if (put && f == 2) x.vote_granted = v != 0;
        return f == 1 || f == 2;
    });
}

int raft_wire_decode_append_resp(const uint8_t* buf, const int64_t* off, int64_t n, raft_append_resp* out) {
    return decode_scalars(buf, off, n, out, "ResponseAppendEntriesRPC",
                          [](raft_append_resp& x, uint32_t f, uint64_t v, bool put) {
        if (put && f == 1) x.term = as_int32(v);
        if (put && f == 2) x.success = v != 0;
        return f == 1 || f == 2;
    });
}

int raft_wire_decode_append_req(const uint8_t* buf, const int64_t* off, int64_t n, raft_append_req* out,
                                int64_t* cmd_off, int32_t* cmd_len, int32_t* n_entries) {
    if (int rc = check_batch(buf, off, n, out)) return rc;
    for (int64_t m = 0; m < n; ++m) {
        raft_append_req x{};
        int64_t co = off[m];
        int32_t cl = 0, ne = 0;
        Reader r{buf + off[m], buf + off[m + 1]};
        uint32_t num, wt;
        while (r.field(num, wt)) {
            if (wt == WT_VARINT && num >= 1 && num <= 6 && num != 5) {
                const int32_t v = as_int32(r.varint());
                if (num == 1) x.term = v;
                else if (num == 2) x.leader_id = v;
                else if (num == 3) x.prev_log_index = v;
                else if (num == 4) x.prev_log_term = v;
                else x.leader_commit = v;
            } else if (wt == WT_LEN && num == 5) {                      // one LogEntry
                const uint8_t* b;
                uint64_t len;
                if (!r.bytes(b, len)) break;
                Reader e{b, b + len};
                int32_t term = 0;
                const uint8_t* cb = b;
                uint64_t clen = 0;
                uint32_t en, ewt;
                while (e.field(en, ewt)) {
                    if (ewt == WT_VARINT && en == 1) term = as_int32(e.varint());
                    else if (ewt == WT_LEN && en == 2) e.bytes(cb, clen);
                    else e.skip(ewt);
                }
                if (!e.ok) { r.ok = false; break; }
                if (ne == 0) {                                          // entries[0] (RaftServer.kt:278)
                    x.has_entry = 1;
                    x.entry_term = term;
                    co = clen ? (int64_t)(cb - buf) : off[m];
                    cl = (int32_t)clen;
                }
                ++ne;
            } else {
                r.skip(wt);
            }
        }
        if (!r.ok) return bad_message("RequestAppendEntriesRPC", m);
        out[m] = x;
        if (cmd_off) cmd_off[m] = co;
        if (cmd_len) cmd_len[m] = cl;
        if (n_entries) n_entries[m] = ne;
    }
    return RAFT_OK;
}

int64_t raft_wire_encode_vote_req(const raft_vote_req* in, int64_t n, uint8_t* buf, int64_t cap, int64_t* off) {
    return encode_batch(in, n, buf, cap, off, [in](Writer& w, int64_t m) {
        w.int32_field(1, in[m].term);
        w.int32_field(2, in[m].candidate_id);
        w.int32_field(3, in[m].last_log_index);
        w.int32_field(4, in[m].last_log_term);
    });
}

int64_t raft_wire_encode_vote_resp(const raft_vote_resp* in, int64_t n, uint8_t* buf, int64_t cap, int64_t* off) {
    return encode_batch(in, n, buf, cap, off, [in](Writer& w, int64_t m) {
        w.int32_field(1, in[m].term);
        w.bool_field(2, in[m].vote_granted);
    });
}

int64_t raft_wire_encode_append_resp(const raft_append_resp* in, int64_t n, uint8_t* buf, int64_t cap,
                                     int64_t* off) {
    return encode_batch(in, n, buf, cap, off, [in](Writer& w, int64_t m) {
        w.int32_field(1, in[m].term);
        w.bool_field(2, in[m].success);
    });
}

int64_t raft_wire_encode_append_req(const raft_append_req* in, const uint8_t* cmd_bytes, const int64_t* cmd_off,
                                    int64_t n, uint8_t* buf, int64_t cap, int64_t* off) {
    if (n > 0 && !cmd_off) return raft_internal_fail(RAFT_EINVAL, "null command offsets");
    for (int64_t m = 0; m < n; ++m)
        if (cmd_off[m + 1] < cmd_off[m] || (cmd_off[m + 1] > cmd_off[m] && !cmd_bytes))
            return raft_internal_fail(RAFT_EINVAL, "bad command offsets");
    return encode_batch(in, n, buf, cap, off, [in, cmd_bytes, cmd_off](Writer& w, int64_t m) {
        const raft_append_req& x = in[m];
        w.int32_field(1, x.term);
        w.int32_field(2, x.leader_id);
        w.int32_field(3, x.prev_log_index);
        w.int32_field(4, x.prev_log_term);
        if (x.has_entry) {
            const int64_t clen = cmd_off[m + 1] - cmd_off[m];
            const int64_t body = int32_field_size(1, x.entry_term) +
                                 (clen > 0 ? varint_size((uint64_t)2 << 3) + varint_size((uint64_t)clen) + clen : 0);
            w.key(5, WT_LEN);
            w.varint((uint64_t)body);
            w.int32_field(1, x.entry_term);
            w.bytes_field(2, cmd_bytes + cmd_off[m], clen);
        }
        w.int32_field(6, x.leader_commit);
    });
}

}  // extern "C"
