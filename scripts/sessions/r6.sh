#!/bin/bash
# Round-6 GPU sessions, one named preset per call:
#   gpurun -- 'PRESET=a bash scripts/sessions/r6.sh'
# Every GPU step has its own time limit and a failure ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
P=${PRESET:?set PRESET}
OUT=gpurun_out/r6_$P${TAGS:-}; mkdir -p "$OUT"
step() {   # step NAME LIMIT CMD...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/status.txt"
  [ $rc -eq 0 ] || [ $rc -eq 1 -a "$name" = pytest ] || exit $rc
}
summ() {   # one line per log: value, wall, kernel, all-reduce
  for f in "$@"; do
    echo "$(basename $f) $(grep -o '"value": [0-9.e+]*' $f | head -1) $(grep -o '"wall_ms": [0-9.]*' $f | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1) $(grep -o '"allreduce_ms": [0-9.enul]*' $f | head -1)"
  done
}
Q="--no-cpu-baseline --handler-batch 0 --no-general-leg --stream-steps 0"
case $P in
  a)  # VALU issue cost per instruction class (scripts/ubench/valu_rate4.hip); the short shard's host-side
      # A/B (kernel timestamps on the launches; polling the last event before the closing sync), with the
      # one-rank native all-reduce inside the clock; the handler batches' scattered-access calibration
      step ubench4 120 ./scripts/ubench/valu_rate4
      for i in 1 2; do
        for ev in 1 0; do
          for sy in block spin; do
            tag=s8_ev${ev}_${sy}_$i
            RAFT_BENCH_NO_KERNEL_EVENTS=$([ $ev = 0 ] && echo 1 || echo 0) RAFT_BENCH_FORCE_COLLECTIVE=1 \
              step $tag 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 --sync $sy $Q
          done
        done
        step d20_block_$i 200 python -u bench.py --steps 20 --warmup 5 --sync block $Q
        step d20_spin_$i 200 python -u bench.py --steps 20 --warmup 5 --sync spin $Q
      done
      summ $OUT/s8_*.log $OUT/d20_*.log > $OUT/summary.txt
      TAG=r6_a step pmch 900 bash scripts/pmc_handler.sh
      ;;
  b)  # the state quads (handler batches: 2-3 sectors per message, HBM tail cache): the GPU suite, the
      # driver's command, the short shard's in-process A/B, the handler batches' calibrated traffic
      step pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
      step bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
      step shard_ab 300 python -u scripts/shard_ab.py --groups 125000 --reps 15 --collective
      TAG=r6_b step pmch 900 bash scripts/pmc_handler.sh
      ;;
  c)  # the SALU / mask hand-off costs (ubench parts 5, 6); row 22's bound on the quad-layout kernel (every
      # log store removed, results wrong, timing only) against production, interleaved; the driver's line
      step ubench5 120 ./scripts/ubench/valu_rate5
      step ubench6 120 ./scripts/ubench/valu_rate6
      step pytest 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 240 --timeout-method thread -k "multi_chunk or non_direct or traffic_probe"
      for i in 1 2; do
        step prod_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        RAFT_ENGINE_LIB=$PWD/raft-kotlin_amd/lib/libraft_engine_nostore.so step nostore_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        step prod_def_$i 200 python -u bench.py $Q
        RAFT_ENGINE_LIB=$PWD/raft-kotlin_amd/lib/libraft_engine_nostore.so step nostore_def_$i 200 python -u bench.py $Q
      done
      summ $OUT/prod_*.log $OUT/nostore_*.log > $OUT/summary.txt
      step bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
      ;;
  d)  # the VOP3 select rewrite (scripts/variants/cndmask_e64.py): the GPU suite on the rewritten build,
      # then production / the identity-rewrite control / the rewrite, interleaved, on the driver's command
      # and the default
      L=$PWD/raft-kotlin_amd/lib
      RAFT_ENGINE_LIB=$L/libraft_engine_e64.so step pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
      for i in 1 2 3; do
        step prod_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_asmid.so step asmid_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_e64.so step e64_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
      done
      for i in 1 2; do
        step prod_def_$i 200 python -u bench.py $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_asmid.so step asmid_def_$i 200 python -u bench.py $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_e64.so step e64_def_$i 200 python -u bench.py $Q
      done
      summ $OUT/prod_*.log $OUT/asmid_*.log $OUT/e64_*.log > $OUT/summary.txt
      ;;
  e)  # the short shard with no event inside the clock (replay timing) against the round-5 region timing,
      # in process; its timeline under the runtime trace; the driver's command
      step shard_ab 400 python -u scripts/shard_ab.py --groups 125000 --reps 15 --collective
      RAFT_BENCH_FORCE_COLLECTIVE=1 step trace_s8 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $OUT/trace_s8 -o run --output-format csv -- python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
      TIMELINE_STEP=-3 python scripts/trace_timeline.py $OUT/trace_s8 > $OUT/timeline_s8.json 2> $OUT/timeline_s8.err || true
      rm -rf $OUT/trace_s8
      for i in 1 2; do
        RAFT_BENCH_FORCE_COLLECTIVE=1 step s8_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        step d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
      done
      summ $OUT/s8_*.log $OUT/d20_*.log > $OUT/summary.txt
      ;;
  f)  # the handler batches with their requests staged by the tile kernel (gathered into LDS with the keys;
      # an append's log[prev] read with the state): the batch tests, then the bench's handler leg against
      # the previous batch design (prevh), interleaved
      L=$PWD/raft-kotlin_amd/lib
      H="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
      step pytest 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "handler or batch or ring_window or non_direct or wire or service"
      for i in 1 2 3; do
        step new_$i 200 python -u bench.py $H
        RAFT_ENGINE_LIB=$L/libraft_engine_prevh.so step prevh_$i 200 python -u bench.py $H
      done
      for f in $OUT/new_*.log $OUT/prevh_*.log; do
        python -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1])['handler_batch']; print('$(basename $f)', *('%s %.4e %.4f bad=%d' % (k, d[k]['messages_per_s_device'], d[k]['ms_per_batch_device'], d[k]['parity_mismatches']) for k in ('vote', 'append')))"
      done > $OUT/summary.txt
      ;;
  g)  # the untimed rehearsal and the occupancy cache: the GPU suite, standalone short-shard runs (the
      # driver's kind: one timed region per process) and the driver's command
      step pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
      for i in 1 2 3; do
        RAFT_BENCH_FORCE_COLLECTIVE=1 step s8_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        RAFT_BENCH_FORCE_COLLECTIVE=1 step s8norh_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 --no-rehearse $Q
      done
      for i in 1 2; do
        step d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
      done
      summ $OUT/s8_*.log $OUT/s8norh_*.log $OUT/d20_*.log > $OUT/summary.txt
      step bench_driver 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
      ;;
  h)  # the rehearsal's duration (GPU clocks out of idle before a short timed region), standalone runs as
      # the driver makes them; the tile kernel at 2,048 messages per tile (handler batches)
      L=$PWD/raft-kotlin_amd/lib
      for i in 1 2 3; do
        RAFT_BENCH_FORCE_COLLECTIVE=1 step s8_r50_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        RAFT_BENCH_FORCE_COLLECTIVE=1 step s8_r0_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 --rehearse-ms 0 $Q
      done
      for i in 1 2; do
        step d20_r50_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        step d20_r0_$i 200 python -u bench.py --steps 20 --warmup 5 --rehearse-ms 0 $Q
      done
      summ $OUT/s8_*.log $OUT/d20_*.log > $OUT/summary.txt
      H="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
      for i in 1 2; do
        step prod_$i 200 python -u bench.py $H
        RAFT_ENGINE_LIB=$L/libraft_engine_t512x4.so step t512x4_$i 200 python -u bench.py $H
        RAFT_ENGINE_LIB=$L/libraft_engine_t256x8.so step t256x8_$i 200 python -u bench.py $H
      done
      for f in $OUT/prod_*.log $OUT/t512x4_*.log $OUT/t256x8_*.log; do
        python -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1])['handler_batch']; print('$(basename $f)', *('%s %.4e %.4f bad=%d' % (k, d[k]['messages_per_s_device'], d[k]['ms_per_batch_device'], d[k]['parity_mismatches']) for k in ('vote', 'append')))"
      done > $OUT/handler_summary.txt
      ;;
  i)  # the rehearsal's length on the driver's command and the 1/8 shard; the N = 2 rehearsal (gloo ranks on
      # one GPU) through the rehearsal / replay path; the other workloads for the results table
      for i in 1 2; do
        for r in 0 50 200 1000; do
          step d20_r${r}_$i 200 python -u bench.py --steps 20 --warmup 5 --rehearse-ms $r $Q
        done
        for r in 50 200; do
          RAFT_BENCH_FORCE_COLLECTIVE=1 step s8_r${r}_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 --rehearse-ms $r $Q
        done
      done
      summ $OUT/d20_*.log $OUT/s8_*.log > $OUT/summary.txt
      TAG=r6_i/dist STEPS=512 step dist 900 bash scripts/dist_rehearsal.sh
      step cfg5 300 python -u bench.py --config 5 --groups 100000 --no-cpu-baseline --handler-batch 0
      step cfg2 300 python -u bench.py --config 2 --groups 10000 --no-cpu-baseline --handler-batch 0
      step textbook 300 python -u bench.py --mode textbook --no-cpu-baseline --handler-batch 0
      summ $OUT/cfg5.log $OUT/cfg2.log $OUT/textbook.log > $OUT/summary_other.txt
      ;;
  j)  # the scalar-compare fold (scripts/variants/scc_fold.py: an s_cmp of a mask the logic op before it
      # just computed, dropped, its branch inverted): the GPU suite on the rewritten build, then
      # production / the identity-rewrite control / the fold, interleaved, on the driver's command and
      # the default
      L=$PWD/raft-kotlin_amd/lib
      RAFT_ENGINE_LIB=$L/libraft_engine_scc.so step pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
      for i in 1 2 3; do
        step prod_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_asmid.so step asmid_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_scc.so step scc_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
      done
      for i in 1 2; do
        step prod_def_$i 200 python -u bench.py $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_asmid.so step asmid_def_$i 200 python -u bench.py $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_scc.so step scc_def_$i 200 python -u bench.py $Q
      done
      summ $OUT/prod_*.log $OUT/asmid_*.log $OUT/scc_*.log > $OUT/summary.txt
      ;;
  k)  # handler batches: runs found without the LDS sort in buckets of <= 2^11 replicas (the chunk kept in
      # batch order, a run led by its first position): the batch tests, then the handler leg against the
      # previous revision's library (hprev), interleaved
      L=$PWD/raft-kotlin_amd/lib
      step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
          -k "handler or batch or bucket or ring or gather"
      H="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
      for i in 1 2 3; do
        step prod_$i 200 python -u bench.py $H
        RAFT_ENGINE_LIB=$L/libraft_engine_hprev.so step hprev_$i 200 python -u bench.py $H
      done
      for f in $OUT/prod_*.log $OUT/hprev_*.log; do
        python -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1])['handler_batch']; print('$(basename $f)', *('%s %.4e %.4f bad=%d' % (k, d[k]['messages_per_s_device'], d[k]['ms_per_batch_device'], d[k]['parity_mismatches']) for k in ('vote', 'append')))"
      done > $OUT/handler_summary.txt
      ;;
  l)  # the tile kernel at 1,024 threads x 4 messages (16 waves, 4 per SIMD; same 4,096-message tile)
      # against production, interleaved, on the bench's handler leg
      L=$PWD/raft-kotlin_amd/lib
      H="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
      RAFT_ENGINE_LIB=$L/libraft_engine_t1024x4.so step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu \
          -x -v --timeout 300 --timeout-method thread -k "handler or batch or bucket or ring or gather"
      for i in 1 2 3; do
        step prod_$i 200 python -u bench.py $H
        RAFT_ENGINE_LIB=$L/libraft_engine_t1024x4.so step t1024x4_$i 200 python -u bench.py $H
      done
      for f in $OUT/prod_*.log $OUT/t1024x4_*.log; do
        python -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1])['handler_batch']; print('$(basename $f)', *('%s %.4e %.4f bad=%d' % (k, d[k]['messages_per_s_device'], d[k]['ms_per_batch_device'], d[k]['parity_mismatches']) for k in ('vote', 'append')))"
      done > $OUT/handler_summary.txt
      ;;
  m)  # the handler batch kernel's bucket size: ~640 messages per bucket (2^12 replicas, 1,221 buckets:
      # 1.2 rounds of the resident workgroups, two chunks each) and ~160 (2^10, 4,883 buckets) against
      # production's ~410 (2^11, 2,442 buckets: 2.4 rounds), interleaved
      L=$PWD/raft-kotlin_amd/lib
      H="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
      for i in 1 2 3; do
        step prod_$i 200 python -u bench.py $H
        RAFT_ENGINE_LIB=$L/libraft_engine_bm640.so step bm640_$i 200 python -u bench.py $H
        RAFT_ENGINE_LIB=$L/libraft_engine_bm160.so step bm160_$i 200 python -u bench.py $H
      done
      for f in $OUT/prod_*.log $OUT/bm640_*.log $OUT/bm160_*.log; do
        python -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1])['handler_batch']; print('$(basename $f)', *('%s %.4e %.4f bad=%d' % (k, d[k]['messages_per_s_device'], d[k]['ms_per_batch_device'], d[k]['parity_mismatches']) for k in ('vote', 'append')))"
      done > $OUT/handler_summary.txt
      ;;
  n)  # launch sub-ranges on the balanced schedule at the default (10^4 steps, 400-step launches): the
      # grid split over 2 or 3 streams whose launches overlap at the launch boundaries, against one
      for i in 1 2; do
        for sr in 1 2 3; do
          step def_sr${sr}_$i 200 python -u bench.py --subranges $sr $Q
        done
      done
      for sr in 2 3; do
        step d20_sr${sr} 200 python -u bench.py --steps 20 --warmup 5 --subranges $sr $Q
      done
      summ $OUT/def_*.log $OUT/d20_*.log > $OUT/summary.txt
      ;;
  o)  # launch length at the default (10^4 steps): 50 / 100 / 200 / 400 steps per launch, twice each,
      # interleaved -- how much of a launch's time is its boundary (tail, state in / out)
      for i in 1 2; do
        for k in 50 100 200 400; do
          step def_k${k}_$i 200 python -u bench.py --steps-per-launch $k $Q
        done
      done
      summ $OUT/def_*.log > $OUT/summary.txt
      ;;
  p)  # long launches, timing only (scripts/variants/long_launch_timing.patch: the counter rows wrap every
      # 400 steps in LDS, so a launch may run 2,000 steps; its counters are wrong): the default at 400 /
      # 1,000 / 2,000 steps per launch against production's 400
      L=$PWD/raft-kotlin_amd/lib
      for i in 1 2; do
        step prod_k400_$i 200 python -u bench.py $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_ll.so step ll_k400_$i 200 python -u bench.py $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_ll.so step ll_k1000_$i 200 python -u bench.py --steps-per-launch 1000 $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_ll.so step ll_k2000_$i 200 python -u bench.py --steps-per-launch 2000 $Q
      done
      summ $OUT/prod_*.log $OUT/ll_*.log > $OUT/summary.txt
      ;;
  q)  # counter rows in HBM for launches beyond the LDS rows (step_kernel HBM_ROWS): the GPU suite and smoke
      # on the new build, then the default (one 10^4-step launch) against the previous library (400-step
      # launches), and the driver's command, interleaved
      L=$PWD/raft-kotlin_amd/lib
      step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
      step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
      for i in 1 2; do
        step new_def_$i 200 python -u bench.py $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_prev.so step prev_def_$i 200 python -u bench.py --steps-per-launch 400 $Q
        step new_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_prev.so step prev_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
      done
      RAFT_BENCH_FORCE_COLLECTIVE=1 step s8_def 300 python -u bench.py --groups 125000 $Q
      summ $OUT/new_*.log $OUT/prev_*.log $OUT/s8_*.log > $OUT/summary.txt
      ;;
  r)  # one 10^4-step launch (counter rows in HBM) against 400-step launches at config 4's shard sizes
      # (10^6 / N groups), the default's 10^4 steps, interleaved
      for g in 125000 250000 500000; do
        for i in 1 2; do
          step g${g}_long_$i 200 python -u bench.py --groups $g $Q
          step g${g}_k400_$i 200 python -u bench.py --groups $g --steps-per-launch 400 $Q
        done
      done
      summ $OUT/g*.log > $OUT/summary.txt
      ;;
  s)  # counter rows in HBM with a per-wave LDS window (16 steps) flushed by atomics: the launch-length and
      # parity tests, then the default (one 10^4-step launch) against the previous library (400-step
      # launches) at 10^6 and at config 4's 1/8 shard, interleaved; the driver's command
      L=$PWD/raft-kotlin_amd/lib
      step pytest 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
          -k "steps_per_launch or full_size or config4 or subrange"
      for i in 1 2; do
        step new_def_$i 200 python -u bench.py $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_prev.so step prev_def_$i 200 python -u bench.py --steps-per-launch 400 $Q
        step new_s8_$i 200 python -u bench.py --groups 125000 $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_prev.so step prev_s8_$i 200 python -u bench.py --groups 125000 --steps-per-launch 400 $Q
      done
      step new_d20 200 python -u bench.py --steps 20 --warmup 5 $Q
      summ $OUT/new_*.log $OUT/prev_*.log > $OUT/summary.txt
      ;;
  t)  # the HBM-row kernel's launch length at the default: 1,000 / 2,000 / 5,000 / 10,000 steps per launch
      # against the previous library's 400, interleaved
      L=$PWD/raft-kotlin_amd/lib
      for i in 1 2; do
        for k in 1000 2000 5000 10000; do
          step new_k${k}_$i 200 python -u bench.py --steps-per-launch $k $Q
        done
        RAFT_ENGINE_LIB=$L/libraft_engine_prev.so step prev_k400_$i 200 python -u bench.py --steps-per-launch 400 $Q
      done
      summ $OUT/new_*.log $OUT/prev_*.log > $OUT/summary.txt
      ;;
  u)  # priority-band re-tune on this round's kernel (RAFT_BAND_ENDS / RAFT_AGE_SHIFTS builds): b1 later
      # band ends 600/800/930, b2 age shifts x1.5, b3 earlier ends 400/700/880, b4 age shifts /2, against
      # production (500/750/900, 80/40/20), interleaved on the driver's command and the 1/8 shard
      L=$PWD/raft-kotlin_amd/lib
      for i in 1 2 3; do
        step prod_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        for v in b1 b2 b3 b4; do
          RAFT_ENGINE_LIB=$L/libraft_engine_$v.so step ${v}_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        done
        step prod_s8_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        for v in b1 b2 b3 b4; do
          RAFT_ENGINE_LIB=$L/libraft_engine_$v.so step ${v}_s8_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        done
      done
      summ $OUT/*_d20_*.log $OUT/*_s8_*.log > $OUT/summary.txt
      ;;
  v)  # long launches as 400-step epochs (a workgroup barrier per epoch instead of a chip-wide launch
      # boundary): the launch-length / full-size parity tests, then the default (one 10^4-step launch)
      # against the previous library (400-step launches) at 10^6 and at config 4's shard sizes, interleaved
      L=$PWD/raft-kotlin_amd/lib
      step pytest 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
          -k "steps_per_launch or full_size or config4 or subrange"
      for i in 1 2; do
        for g in 1000000 125000 250000; do
          step new_g${g}_$i 200 python -u bench.py --groups $g $Q
          RAFT_ENGINE_LIB=$L/libraft_engine_prev.so step prev_g${g}_$i 200 python -u bench.py --groups $g --steps-per-launch 400 $Q
        done
      done
      step new_d20 200 python -u bench.py --steps 20 --warmup 5 $Q
      summ $OUT/new_*.log $OUT/prev_*.log > $OUT/summary.txt
      ;;
  w)  # the epochs build as the product (a separate kernel instantiation for epochs): the GPU suite and
      # smoke, then the driver's command (no epochs: must equal production) and the default / the 1/8
      # shard (one 10^4-step launch of epochs) against the previous library, interleaved
      L=$PWD/raft-kotlin_amd/lib
      step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
      step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
      for i in 1 2 3; do
        step new_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_prev.so step prev_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
      done
      for i in 1 2; do
        step new_def_$i 200 python -u bench.py $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_prev.so step prev_def_$i 200 python -u bench.py --steps-per-launch 400 $Q
      done
      RAFT_BENCH_FORCE_COLLECTIVE=1 step new_s8 200 python -u bench.py --groups 125000 $Q
      summ $OUT/new_*.log $OUT/prev_*.log > $OUT/summary.txt
      ;;
  x)  # PMC rows of the epochs build (kernel and batch sources changed): both bench commands, the 1/8
      # shard's and the handler batches'; merged back here into profiles/pmc_rows.json / pmc_handler.json
      TAG=r6_ep_d20 ARGS="--steps 20 --warmup 5" step pmc_d20 900 bash scripts/pmc_bench.sh
      TAG=r6_ep_def ARGS="" step pmc_def 900 bash scripts/pmc_bench.sh
      TAG=r6_ep_s8 ARGS="--groups 125000 --steps 20 --warmup 5" step pmc_s8 900 bash scripts/pmc_bench.sh
      TAG=r6_ep step pmch 900 bash scripts/pmc_handler.sh
      ;;
  y)  # short balanced launches as epochs too (RAFT_SHORT_EPOCH=E: a launch of more than E steps runs
      # E-step epochs, so every wave's share covers each step range equally -- the election storm's
      # heavy steps and the quiet ones): parity of the launch-length / full-size / config-4 tests at
      # E = 5, then the driver's command and the 1/8 shard at E = 0 / 5 / 10, interleaved
      RAFT_SHORT_EPOCH=5 step pytest 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
          --timeout-method thread -k "steps_per_launch or full_size or config4"
      for i in 1 2 3; do
        for E in 0 5 10; do
          RAFT_SHORT_EPOCH=$E step d20_e${E}_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
          RAFT_SHORT_EPOCH=$E RAFT_BENCH_FORCE_COLLECTIVE=1 \
            step s8_e${E}_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        done
      done
      summ $OUT/d20_*.log $OUT/s8_*.log > $OUT/summary.txt
      ;;
  z)  # per-step cost profile (scripts/step_profile.py): one-step launches from step 0 at full size and
      # at the 1/8 shard, and a steady-state window
      step prof_full 300 python -u scripts/step_profile.py --groups 1000000 --steps 40 --also 3000:3020
      step prof_s8 300 python -u scripts/step_profile.py --groups 125000 --steps 40 --also 3000:3020
      ;;
  fin)  # final verification of the committed tree: the GPU suite, smoke, the driver's command and the
      # default (every leg, CPU baseline included), the 1/8 shard with the one-rank RCCL all-reduce
      step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
      step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
      step bench_driver 600 python -u bench.py --steps 20 --warmup 5
      step bench_default 900 python -u bench.py
      RAFT_BENCH_FORCE_COLLECTIVE=1 step shard 300 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
      summ $OUT/bench_*.log $OUT/shard.log > $OUT/summary.txt
      ;;
  xcd) # XCD-aware bucket order in bucket_batch_kernel (XCD b % 8 takes a contiguous bucket range, so
      # neighbouring buckets share L2 lines of the segment table and the partitioned tiles): the batch
      # tests, then the handler leg against the previous library (rev HEAD), interleaved; its PMC rows
      L=$PWD/raft-kotlin_amd/lib
      H="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
      step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
          --timeout-method thread -k "batch or handler or service or wire"
      for i in 1 2 3; do
        step new_$i 300 python -u bench.py $H
        RAFT_ENGINE_LIB=$L/libraft_engine_prev.so step prev_$i 300 python -u bench.py $H
      done
      for f in $OUT/new_*.log $OUT/prev_*.log; do
        python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['handler_batch']; print(sys.argv[1].split('/')[-1], d['vote']['messages_per_s_device'], d['append']['messages_per_s_device'])" $f
      done > $OUT/summary.txt
      TAG=r6_xcd step pmch 900 bash scripts/pmc_handler.sh
      ;;
  spec) # the append handler's first log[prev] fetched beside the replica's fields (production) against
      # the previous tree (libraft_engine_base.so; not adopted, scripts/variants/append_prev_prefetch.patch): the batch tests on production, then 3 interleaved runs
      L=$PWD/raft-kotlin_amd/lib
      H="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
      step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
          -k "batch or handler or service or wire"
      for i in 1 2 3; do
        step prod_$i 300 python -u bench.py $H
        RAFT_ENGINE_LIB=$L/libraft_engine_base.so step base_$i 300 python -u bench.py $H
      done
      grep -ho '"handler_batch": {[^}]*' $OUT/prod_*.log $OUT/base_*.log > $OUT/summary.txt || true
      ;;
  rmaj) # the state as one 64-B record per replica (scripts/variants/replica_major_state.patch: a handler's
      # quads in one 64-B fetch; the step kernel's field loads 64 B apart per lane): the GPU suite on the
      # variant, then production / variant interleaved on the driver's command + handler leg, the default
      # and the 1/8 shard
      L=$PWD/raft-kotlin_amd/lib
      H="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
      RAFT_ENGINE_LIB=$L/libraft_engine_rmaj.so step pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 300 \
          --timeout-method thread
      for i in 1 2 3; do
        step prod_h_$i 300 python -u bench.py $H
        RAFT_ENGINE_LIB=$L/libraft_engine_rmaj.so step rmaj_h_$i 300 python -u bench.py $H
      done
      for i in 1 2; do
        step prod_def_$i 300 python -u bench.py $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_rmaj.so step rmaj_def_$i 300 python -u bench.py $Q
        RAFT_BENCH_FORCE_COLLECTIVE=1 step prod_s8_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_rmaj.so RAFT_BENCH_FORCE_COLLECTIVE=1 step rmaj_s8_$i 200 python -u bench.py \
            --groups 125000 --steps 20 --warmup 5 $Q
      done
      summ $OUT/prod_*.log $OUT/rmaj_*.log > $OUT/summary.txt
      for f in $OUT/prod_h_*.log $OUT/rmaj_h_*.log; do
        echo "$(basename $f) $(grep -o '"messages_per_s_device": [0-9.e+]*' $f | tr '\n' ' ')"
      done >> $OUT/summary.txt
      ;;
  sched) # LLVM's AMDGPU scheduling strategies on the step kernel (scripts/build_variants.sh "ilp:-mllvm
      # -amdgpu-sched-strategy=max-ilp", "memc:... =max-memory-clause"): the full-size digests on each, then
      # production / ilp / memc interleaved on the driver's command and the 1/8 shard
      L=$PWD/raft-kotlin_amd/lib
      for v in ilp memc; do
        RAFT_ENGINE_LIB=$L/libraft_engine_$v.so step pytest_$v 400 python -u -m pytest tests/test_gpu_parity.py -m gpu \
            -x -v --timeout 300 --timeout-method thread -k "full_size_digest"
      done
      for i in 1 2 3; do
        step prod_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        for v in ilp memc; do
          RAFT_ENGINE_LIB=$L/libraft_engine_$v.so step ${v}_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        done
      done
      for i in 1 2; do
        RAFT_BENCH_FORCE_COLLECTIVE=1 step prod_s8_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        for v in ilp memc; do
          RAFT_ENGINE_LIB=$L/libraft_engine_$v.so RAFT_BENCH_FORCE_COLLECTIVE=1 step ${v}_s8_$i 200 python -u bench.py \
              --groups 125000 --steps 20 --warmup 5 $Q
        done
      done
      summ $OUT/prod_*.log $OUT/ilp_*.log $OUT/memc_*.log > $OUT/summary.txt
      ;;
  ilp) # max-ilp scheduling on the whole library: production / ilp interleaved on the driver's command with
      # the handler leg, and on the default (one 10^4-step launch of epochs)
      L=$PWD/raft-kotlin_amd/lib
      H="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
      for i in 1 2 3; do
        step prod_h_$i 300 python -u bench.py $H
        RAFT_ENGINE_LIB=$L/libraft_engine_ilp.so step ilp_h_$i 300 python -u bench.py $H
      done
      for i in 1 2; do
        step prod_def_$i 300 python -u bench.py $Q
        RAFT_ENGINE_LIB=$L/libraft_engine_ilp.so step ilp_def_$i 300 python -u bench.py $Q
      done
      summ $OUT/prod_*.log $OUT/ilp_*.log > $OUT/summary.txt
      for f in $OUT/prod_h_*.log $OUT/ilp_h_*.log; do
        echo "$(basename $f) $(grep -o '"messages_per_s_device": [0-9.e+]*' $f | tr '\n' ' ')"
      done >> $OUT/summary.txt
      ;;
  occ) # the handler kernel's occupancy: bucket_batch_kernel at amdgpu_waves_per_eu 8 (vote: 61 VGPRs, 4
      # workgroups per CU instead of 3) and 6 / 8 (append: 80 VGPRs with 5 spills / 64 with 25; 3 or 4
      # workgroups instead of 2) against production; the batch tests on each variant first
      L=$PWD/raft-kotlin_amd/lib
      H="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
      for v in w86 w88; do
        RAFT_ENGINE_LIB=$L/libraft_engine_$v.so step pytest_$v 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x \
            -v --timeout 300 --timeout-method thread -k "batch or handler or service or wire"
      done
      for i in 1 2 3; do
        step prod_$i 300 python -u bench.py $H
        for v in w86 w88; do RAFT_ENGINE_LIB=$L/libraft_engine_$v.so step ${v}_$i 300 python -u bench.py $H; done
      done
      for f in $OUT/prod_*.log $OUT/w8*.log; do
        python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['handler_batch']; print(sys.argv[1].split('/')[-1], d['vote']['messages_per_s_device'], d['append']['messages_per_s_device'], d['vote']['parity_mismatches'], d['append']['parity_mismatches'])" $f
      done > $OUT/summary.txt
      ;;
  pre) # append requests loaded before the handler kernel's LDS sort (in flight across it) and staged in
      # LDS, the run's log[prev] read with the replica's fields; the vote kernel at 8 waves per SIMD: the
      # batch tests, then the handler leg against the previous library (rev HEAD), interleaved
      L=$PWD/raft-kotlin_amd/lib
      H="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
      step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
          --timeout-method thread -k "batch or handler or service or wire"
      for i in 1 2 3; do
        step new_$i 300 python -u bench.py $H
        RAFT_ENGINE_LIB=$L/libraft_engine_prev.so step prev_$i 300 python -u bench.py $H
      done
      for f in $OUT/new_*.log $OUT/prev_*.log; do
        python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['handler_batch']; print(sys.argv[1].split('/')[-1], d['vote']['messages_per_s_device'], d['append']['messages_per_s_device'], d['vote']['parity_mismatches'], d['append']['parity_mismatches'])" $f
      done > $OUT/summary.txt
      TAG=r6_pre step pmch 900 bash scripts/pmc_handler.sh
      ;;
  fin2) # final verification after the handler changes (XCD-aware bucket order, the vote kernel at 8 waves
      # per SIMD): the handler PMC rows of this build, then the GPU suite, smoke and both bench commands
      TAG=r6_fin2 step pmch 900 bash scripts/pmc_handler.sh
      step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
      step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
      step bench_driver 600 python -u bench.py --steps 20 --warmup 5
      step bench_default 900 python -u bench.py
      summ $OUT/bench_*.log > $OUT/summary.txt
      ;;
  tiles) # tile shapes again after the XCD-aware bucket order (each bucket's segment-table and message
      # lines now come through one L2, so more, smaller tiles cost the handler kernel less): 512 x 4 and
      # 1024 x 4 against production's 512 x 8, interleaved, after the batch tests on each
      L=$PWD/raft-kotlin_amd/lib
      H="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
      for v in t512x4 t1024x4; do
        RAFT_ENGINE_LIB=$L/libraft_engine_$v.so step pytest_$v 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x \
            -v --timeout 300 --timeout-method thread -k "batch or handler or service or wire"
      done
      for i in 1 2 3; do
        step prod_$i 300 python -u bench.py $H
        for v in t512x4 t1024x4; do RAFT_ENGINE_LIB=$L/libraft_engine_$v.so step ${v}_$i 300 python -u bench.py $H; done
      done
      for f in $OUT/prod_*.log $OUT/t*.log; do
        python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['handler_batch']; print(sys.argv[1].split('/')[-1], d['vote']['messages_per_s_device'], d['append']['messages_per_s_device'], d['vote']['parity_mismatches'], d['append']['parity_mismatches'])" $f
      done > $OUT/summary.txt
      ;;
  bands) # priority bands on the default's one launch of 400-step epochs (each epoch restarts the bands):
      # e0 no age shifts, e1 later band ends 600/800/930, e3 earlier 400/700/880, against production
      L=$PWD/raft-kotlin_amd/lib
      for i in 1 2; do
        step prod_def_$i 300 python -u bench.py $Q
        for v in e0 e1 e3; do RAFT_ENGINE_LIB=$L/libraft_engine_$v.so step ${v}_def_$i 300 python -u bench.py $Q; done
      done
      summ $OUT/*_def_*.log > $OUT/summary.txt
      ;;
  fin3) # the committed final tree: the GPU suite (C host and long-launch variants included), smoke, both
      # bench commands and the 1/8 shard with the one-rank RCCL all-reduce
      step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
      step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
      step bench_driver 600 python -u bench.py --steps 20 --warmup 5
      step bench_default 900 python -u bench.py
      RAFT_BENCH_FORCE_COLLECTIVE=1 step shard 300 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
      summ $OUT/bench_*.log $OUT/shard.log > $OUT/summary.txt
      ;;
  swg) # the 1/8 shard's 20 steps with fewer balanced workgroups (schedule_workgroups 1,536 / 1,280: 6 / 5
      # per CU, more chunk-steps per wave) against the resident 1,792, interleaved; the one-rank all-reduce
      for i in 1 2 3; do
        for w in 0 1536 1280; do
          RAFT_BENCH_FORCE_COLLECTIVE=1 step s8_w${w}_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 \
              --schedule-workgroups $w $Q
        done
      done
      summ $OUT/s8_*.log > $OUT/summary.txt
      ;;
  *) echo "unknown preset $P"; exit 2 ;;
esac
exit 0
