cd "$GRAFT_REPO_ROOT"
NOSELF=1 timeout -k 10 1000 bash scripts/rehearse_multi.sh > gpurun_out/reh_r4.log 2>&1; rc=$?; grep -v "^\[bench rank" gpurun_out/reh_r4.log | tail -12; exit $rc
