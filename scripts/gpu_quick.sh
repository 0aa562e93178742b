cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/gpu_quick.py > gpurun_out/quick.log 2>&1; rc=$?; cat gpurun_out/quick.log | tail -20; exit $rc
