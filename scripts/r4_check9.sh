cd "$GRAFT_REPO_ROOT"
NOSELF=1 timeout -k 10 900 bash scripts/rehearse_multi.sh > gpurun_out/reh_r4.log 2>&1; rc=$?; grep -v "^\[bench rank" gpurun_out/reh_r4.log | tail -12; [ $rc -ne 0 ] && exit 1
ROUND=r04 STEPS=20 WARMUP=5 timeout -k 10 900 bash scripts/profile_round.sh > gpurun_out/prof_r04.log 2>&1; rc=$?; tail -8 gpurun_out/prof_r04.log; exit $rc
