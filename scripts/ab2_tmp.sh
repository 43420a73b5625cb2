cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/ab11_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/ab11_pytest.log
TAG=ab11 VARIANTS="old base" ROUNDS=2 bash scripts/ab.sh && TAG=ab11flat VARIANTS="base" ROUNDS=2 ARGS="--steps 10000 --log-window 0" bash scripts/ab.sh
