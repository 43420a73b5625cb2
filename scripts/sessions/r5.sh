#!/bin/bash
# Round-5 GPU sessions, one named preset per call:
#   gpurun -- 'PRESET=a bash scripts/sessions/r5.sh'
# Every GPU step has its own time limit and a failure ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
P=${PRESET:?set PRESET}
OUT=gpurun_out/r5_$P${TAGS:-}; mkdir -p "$OUT"
step() {   # step NAME LIMIT CMD...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/status.txt"
  [ $rc -eq 0 ] || [ $rc -eq 1 -a "$name" = pytest ] || exit $rc
}
Q="--no-cpu-baseline --handler-batch 0 --no-general-leg --stream-steps 0"
case $P in
  a)  # the collective inside the clock: forced one-rank RCCL beside the plain line, full size and 1/8 shard
      for i in 1 2; do
        step d20_plain_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        RAFT_BENCH_FORCE_COLLECTIVE=1 step d20_rccl_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        step s8_plain_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        RAFT_BENCH_FORCE_COLLECTIVE=1 step s8_rccl_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
      done
      for f in $OUT/*.log; do
        echo "$(basename $f) $(grep -o '"value": [0-9.e+]*' $f | head -1) $(grep -o '"allreduce_ms": [0-9.enul]*' $f | head -1) $(grep -o '"wall_ms": [0-9.]*' $f | head -1)"
      done > $OUT/summary.txt
      step pytest 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
      step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
      step bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
      TAG=r5_a/dist STEPS=512 step dist 900 bash scripts/dist_rehearsal.sh
      ;;
  b)  # issue costs of the Philox instructions; per-phase VALU / SALU budgets of the driver's launch
      # and of the default (steady-state) launch
      step ubench 200 scripts/ubench/valu_rate3
      # the handler batches: kernel trace of the claim path, and of the sorted path (rev d93a3b4)
      step htrace 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace -o run --output-format csv -- python scripts/handler_probe.py
      RAFT_BATCH_LOCALITY_BITS=0 step htrace_claim 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace_claim -o run --output-format csv -- python scripts/handler_probe.py
      RAFT_BATCH_LOCALITY_BITS=16 step htrace_loc16 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace_loc16 -o run --output-format csv -- python scripts/handler_probe.py
      RAFT_ENGINE_LIB=$PWD/raft-kotlin_amd/lib/libraft_engine_sorted.so step htrace_sorted 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace_sorted -o run --output-format csv -- python scripts/handler_probe.py
      TAG=r5_b_d20 step phase_d20 900 bash scripts/phase_budget.sh
      TAG=r5_b_def ARGS=" " step phase_def 900 bash scripts/phase_budget.sh
      ;;
  c)  # parity suite; branch frequencies (RAFT_BRANCH_STATS build) of the driver's launch and the default
      # bench; the driver's bench line; its PMC rows with the in-process traffic probes
      step pytest 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
      RAFT_ENGINE_LIB=$PWD/raft-kotlin_amd/lib/libraft_engine_bstats.so step bstats_d20 300 python -u bench.py --steps 20 --warmup 5 $Q
      RAFT_ENGINE_LIB=$PWD/raft-kotlin_amd/lib/libraft_engine_bstats.so step bstats_def 300 python -u bench.py $Q
      step bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
      TAG=r5_c_d20 ARGS="--steps 20 --warmup 5" step pmc_d20 900 bash scripts/pmc_bench.sh
      ;;
  d)  # the short shard's timeline: kernel + HIP runtime trace of the 1/8 shard's 20-step run, plain and
      # with the one-rank RCCL all-reduce inside the clock (scripts/trace_timeline.py)
      step trace_s8 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $OUT/trace_s8 -o run --output-format csv -- python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
      RAFT_BENCH_FORCE_COLLECTIVE=1 step trace_s8_rccl 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $OUT/trace_s8_rccl -o run --output-format csv -- python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
      python scripts/trace_timeline.py $OUT/trace_s8 > $OUT/timeline_s8.json
      python scripts/trace_timeline.py $OUT/trace_s8_rccl > $OUT/timeline_s8_rccl.json
      # row 22's upper bound: every log store sunk into one slot per wave (results differ; timing only)
      for i in 1 2; do
        step ab_prod_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        RAFT_ENGINE_LIB=$PWD/raft-kotlin_amd/lib/libraft_engine_sink.so step ab_sink_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        step ab_prod_def_$i 200 python -u bench.py $Q
        RAFT_ENGINE_LIB=$PWD/raft-kotlin_amd/lib/libraft_engine_sink.so step ab_sink_def_$i 200 python -u bench.py $Q
      done
      for f in $OUT/ab_*.log; do echo "$(basename $f) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1) $(grep -o '"value": [0-9.e+]*' $f | head -1)"; done > $OUT/ab_summary.txt
      ;;
  e)  # A/B of kernel variants (VARIANTS, built by scripts/build_variants.sh): dynamic VALU / SALU per
      # chunk-step (SQ_INSTS_* of the last step launch) and interleaved timings, driver's launch and default
      for v in prod ${VARIANTS:-}; do
        lib=$PWD/raft-kotlin_amd/lib/libraft_engine_$v.so; [ $v = prod ] && lib=$PWD/raft-kotlin_amd/lib/libraft_engine.so
        for a in d20 def; do
          A="--steps 20 --warmup 5"; [ $a = def ] && A=""
          RAFT_ENGINE_LIB=$lib step pmc_${v}_$a 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/pmc_${v}_$a -o run --output-format csv -- python bench.py $A $Q
        done
      done
      for i in 1 2; do
        for v in prod ${VARIANTS:-}; do
          lib=$PWD/raft-kotlin_amd/lib/libraft_engine_$v.so; [ $v = prod ] && lib=$PWD/raft-kotlin_amd/lib/libraft_engine.so
          RAFT_ENGINE_LIB=$lib step t_${v}_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
          RAFT_ENGINE_LIB=$lib step t_${v}_def_$i 200 python -u bench.py $Q
        done
      done
      for f in $OUT/t_*.log; do echo "$(basename $f) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1) $(grep -o '"value": [0-9.e+]*' $f | head -1)"; done > $OUT/timing.txt
      python scripts/pmc_valu.py $(for v in prod ${VARIANTS:-}; do echo $OUT/pmc_${v}_d20 $OUT/pmc_${v}_def; done) > $OUT/valu.json
      ;;
  f)  # parity suite (the native RCCL all-reduce included); the in-clock all-reduce through
      # raft_engine_allreduce_counters vs torch's, full size and 1/8 shard; row 22's bound (log
      # stores dropped); the default bench's PMC rows
      step pytest 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
      for i in 1 2; do
        step d20_plain_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        RAFT_BENCH_FORCE_COLLECTIVE=1 step d20_native_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        RAFT_BENCH_FORCE_COLLECTIVE=1 RAFT_BENCH_TORCH_ALLREDUCE=1 step d20_torch_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        step s8_plain_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        RAFT_BENCH_FORCE_COLLECTIVE=1 step s8_native_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        RAFT_BENCH_FORCE_COLLECTIVE=1 RAFT_BENCH_TORCH_ALLREDUCE=1 step s8_torch_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        RAFT_ENGINE_LIB=$PWD/raft-kotlin_amd/lib/libraft_engine_nostore.so step nostore_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $Q
        RAFT_ENGINE_LIB=$PWD/raft-kotlin_amd/lib/libraft_engine_nostore.so step nostore_def_$i 200 python -u bench.py $Q
        step prod_def_$i 200 python -u bench.py $Q
      done
      for f in $OUT/d20_*.log $OUT/s8_*.log $OUT/nostore_*.log $OUT/prod_*.log; do
        echo "$(basename $f) $(grep -o '"value": [0-9.e+]*' $f | head -1) $(grep -o '"allreduce_ms": [0-9.enul]*' $f | head -1) $(grep -o '"wall_ms": [0-9.]*' $f | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1)"
      done > $OUT/summary.txt
      TAG=r5_f_def ARGS="" step pmc_def 900 bash scripts/pmc_bench.sh
      ;;
  g)  # the round's evidence at the working tree's kernel: parity suite, smoke, the driver's and the
      # default bench lines, the 1/8 shard's timeline with the native in-clock all-reduce
      step pytest 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
      step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
      step bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
      step bench_default 600 python -u bench.py
      RAFT_BENCH_FORCE_COLLECTIVE=1 step trace_s8_native 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $OUT/trace_s8_native -o run --output-format csv -- python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
      python scripts/trace_timeline.py $OUT/trace_s8_native > $OUT/timeline_s8_native.json
      rm -rf $OUT/trace_s8_native
      ;;
  h)  # the bucketed handler-batch path: its parity tests, then a kernel trace of 5 vote + 5
      # append batches of 10^6 messages on each path, and the bench's handler leg
      step pytest 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "handler or batch" --timeout 300 --timeout-method thread
      for path in 1 2; do
        HANDLER_PATH=$path step htrace_p$path 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace_p$path -o run --output-format csv -- python -u scripts/handler_probe.py
      done
      step bench_handler 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0
      ;;
  h2)  # the bucketed handler path: its parity tests, a kernel trace of both paths, the bench's handler leg
      step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "handler or batch" --timeout 300 --timeout-method thread
      for mt in ${SWEEP:-}; do      # m:t = RAFT_BUCKET_MEAN:RAFT_BUCKET_THREADS (experiment switches)
        m=${mt%:*}; t=${mt#*:}
        RAFT_BUCKET_THREADS=$t step pytest_$t 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "handler or batch" --timeout 300 --timeout-method thread
        RAFT_BUCKET_MEAN=$m RAFT_BUCKET_THREADS=$t HANDLER_REPS=3 step htrace_${m}_$t 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace_${m}_$t -o run --output-format csv -- python -u scripts/handler_probe.py
      done
      HANDLER_REPS=3 step htrace_bucketed 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace_bucketed -o run --output-format csv -- python -u scripts/handler_probe.py
      if [ -n "${HPMC:-}" ]; then   # the bucketed kernels' counters (one pass per counter group)
        HANDLER_REPS=1 step hpmc_sq 300 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY --kernel-include-regex "bucket|batch_kernel" -d $OUT/hpmc_sq -o run --output-format csv -- python -u scripts/handler_probe.py
        HANDLER_REPS=1 step hpmc_fetch 300 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "bucket|batch_kernel" -d $OUT/hpmc_fetch -o run --output-format csv -- python -u scripts/handler_probe.py
      fi
      HANDLER_PATH=1 HANDLER_REPS=3 step htrace_sorted 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace_sorted -o run --output-format csv -- python -u scripts/handler_probe.py
      step bench_handler 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0
      ;;
  t2)  # handler batches: the tile kernel at 512 x 8 (the build) vs 256 x 16 (VARIANT tile256)
      step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "handler or batch" --timeout 300 --timeout-method thread
      for i in 1 2; do
        HANDLER_REPS=3 step htrace_prod_$i 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace_prod_$i -o run --output-format csv -- python -u scripts/handler_probe.py
        RAFT_ENGINE_LIB=$PWD/raft-kotlin_amd/lib/libraft_engine_tile256.so HANDLER_REPS=3 step htrace_tile256_$i 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace_tile256_$i -o run --output-format csv -- python -u scripts/handler_probe.py
      done
      step bench_handler 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0
      ;;
  t)  # the native all-reduce test; handler batches with tiles of 2,048 (VARIANT tile8) vs 4,096
      step pytest 600 python -u -m pytest tests/test_gpu_bench.py -m gpu -v -k "native" --timeout 300 --timeout-method thread
      for i in 1 2; do
        HANDLER_REPS=3 step htrace_prod_$i 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace_prod_$i -o run --output-format csv -- python -u scripts/handler_probe.py
        RAFT_ENGINE_LIB=$PWD/raft-kotlin_amd/lib/libraft_engine_tile8.so HANDLER_REPS=3 step htrace_tile8_$i 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace_tile8_$i -o run --output-format csv -- python -u scripts/handler_probe.py
      done
      ;;
  o)  # the other workloads at the final build (config 5, config 2, textbook config 3), the 1/8 shard
      # plain and with the native one-rank all-reduce, and the N = 2 rehearsal (gloo ranks on one GPU)
      step cfg5 300 python -u bench.py --config 5 --groups 100000 --no-cpu-baseline --handler-batch 0
      step cfg2 300 python -u bench.py --config 2 --groups 10000 --no-cpu-baseline --handler-batch 0
      step textbook 300 python -u bench.py --mode textbook --no-cpu-baseline --handler-batch 0
      for i in 1 2; do
        step s8_plain_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
        RAFT_BENCH_FORCE_COLLECTIVE=1 step s8_native_$i 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 $Q
      done
      TAG=r5_o/dist STEPS=512 step dist 900 bash scripts/dist_rehearsal.sh
      for f in $OUT/*.log; do
        echo "$(basename $f) $(grep -o '"value": [0-9.e+]*' $f | head -1) $(grep -o '"wall_ms": [0-9.]*' $f | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1) $(grep -o '"frac": [0-9.]*' $f | head -1)"
      done > $OUT/summary.txt
      ;;
  fin)  # the handler PMC rows at the working tree's batch sources, then the final checks (preset v)
      TAG=r5_${TAGP:-fin} step pmc_handler 600 bash scripts/pmc_handler.sh
      step pytest 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
      step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
      step bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
      ;;
  v)  # the committed tree as the driver will run it: the GPU suite, smoke, the driver's bench
      # command (every PMC-derived field attached?)
      [ -n "${NOTESTS:-}" ] || step pytest 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
      [ -n "${NOTESTS:-}" ] || step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
      step bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
      ;;
  ph)  # the handler batches' PMC rows alone (scripts/pmc_handler.sh) at the working tree's library
      TAG=r5_${TAGP:-ph} step pmc_handler 600 bash scripts/pmc_handler.sh
      ;;
  pmc)  # the PMC rows (scripts/pmc_bench.sh) of both bench commands at the working tree's kernel
      TAG=r5_${TAGP:-pmc}_d20 ARGS="--steps 20 --warmup 5" step pmc_d20 900 bash scripts/pmc_bench.sh
      TAG=r5_${TAGP:-pmc}_def ARGS="" step pmc_def 900 bash scripts/pmc_bench.sh
      TAG=r5_${TAGP:-pmc} step pmc_handler 600 bash scripts/pmc_handler.sh
      ;;
  *) echo "unknown preset $P"; exit 2 ;;
esac
exit 0
