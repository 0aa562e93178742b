cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_ab.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_env.sh "RT_LONG_BATCH=128" "RT_LONG_BATCH=192" "RT_LONG_BATCH=256" "RT_LONG_BATCH=320"
