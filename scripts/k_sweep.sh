cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/k512
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py::test_steps_per_launch_invariance tests/test_golden.py tests/test_gpu_parity.py::test_config3_drops_churn_reduced -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/k512/pytest.log 2>&1 || exit $?
for k in 64 128 256 512; do
  EXTRA="--steps-per-launch $k --reduce-every 512" STEPS=10000 TAG=k512 VARIANTS=base.k$k bash scripts/flag_sweep.sh || exit $?
done
