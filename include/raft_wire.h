/*
 * raft_wire.h — batched proto3 wire codec for the reference's messages
 * (src/main/proto/greeter.proto:16-44), so that a gRPC-facing service can
 * hand RaftImplBase.vote()/append() traffic (RaftServer.kt:228, :253) to the
 * engine's batch entry points without a protobuf runtime in the data path.
 *
 * A batch of n messages is one byte buffer plus offsets: message m is
 * buf[off[m] .. off[m+1]), off has n + 1 entries.  Decoders accept any valid
 * proto3 encoding of the message: fields in any order, the last occurrence of
 * a scalar field wins, negative int32 as 10-byte varints, unknown fields (and
 * known field numbers with another wire type) are skipped.  A malformed
 * message (truncated varint or length, wire type 3/4/6/7) fails the call with
 * RAFT_EINVAL and raft_last_error() names the message index.  Encoders emit
 * the canonical encoding -- ascending field numbers, default values omitted --
 * which is byte-identical to protobuf's SerializeToString; they return the
 * bytes written, or RAFT_ERANGE (nothing usable written) if cap is too small.
 *
 * Commands.  LogEntry.command is a proto string (greeter.proto:31); the engine
 * stores a u32 command id (raft_append_req.entry_cmd).  Decoding reports the
 * string of entries[0] as (cmd_off, cmd_len) into buf, leaving entry_cmd = 0
 * for the caller's intern table; encoding takes the strings as cmd_bytes +
 * cmd_off[n + 1].  Only entries[0] is carried (the reference appends only
 * entries[0], RaftServer.kt:278; it sends at most one, :130-132); the decoder
 * reports every message's entry count in n_entries.
 */
#ifndef RAFT_WIRE_H
#define RAFT_WIRE_H

#include "raft_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* RequestVoteRPC (greeter.proto:16-21): term = 1, candidateId = 2, lastLogIndex = 3, lastLogTerm = 4 */
int raft_wire_decode_vote_req(const uint8_t* buf, const int64_t* off, int64_t n, raft_vote_req* out);
int64_t raft_wire_encode_vote_req(const raft_vote_req* in, int64_t n, uint8_t* buf, int64_t cap, int64_t* off);

/* ResponseVoteRPC (greeter.proto:23-26): term = 1, voteGranted = 2 */
int raft_wire_decode_vote_resp(const uint8_t* buf, const int64_t* off, int64_t n, raft_vote_resp* out);
int64_t raft_wire_encode_vote_resp(const raft_vote_resp* in, int64_t n, uint8_t* buf, int64_t cap, int64_t* off);

/* RequestAppendEntriesRPC (greeter.proto:28-39): term = 1, leaderId = 2,
 * prevLogIndex = 3, prevLogTerm = 4, repeated LogEntry entries = 5
 * (LogEntry: term = 1, command = 2), leaderCommit = 6.
 * cmd_off / cmd_len / n_entries: [n] each, nullable together with has_entry
 * messages carrying no command. */
int raft_wire_decode_append_req(const uint8_t* buf, const int64_t* off, int64_t n, raft_append_req* out,
                                int64_t* cmd_off, int32_t* cmd_len, int32_t* n_entries);
int64_t raft_wire_encode_append_req(const raft_append_req* in, const uint8_t* cmd_bytes, const int64_t* cmd_off,
                                    int64_t n, uint8_t* buf, int64_t cap, int64_t* off);

/* ResponseAppendEntriesRPC (greeter.proto:41-44): term = 1, success = 2.
 * raft_append_resp.status has no wire form: a handler that threw sends no
 * response at all (RaftServer.kt:170-172), so callers drop those messages;
 * the encoder emits them like any other and the decoder sets status = 0. */
int raft_wire_decode_append_resp(const uint8_t* buf, const int64_t* off, int64_t n, raft_append_resp* out);
int64_t raft_wire_encode_append_resp(const raft_append_resp* in, int64_t n, uint8_t* buf, int64_t cap, int64_t* off);

#ifdef __cplusplus
}
#endif
#endif /* RAFT_WIRE_H */
