cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/ab13_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/ab13_pytest.log
TAG=ab13 VARIANTS="cpur base" ROUNDS=2 bash scripts/ab.sh && TAG=ab13c5 VARIANTS="cpur base" ROUNDS=2 ARGS="--steps 10000 --config 5 --groups 100000" bash scripts/ab.sh
