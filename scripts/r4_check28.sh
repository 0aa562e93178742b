cd "$GRAFT_REPO_ROOT"
bash scripts/r4_check13.sh || exit 1
ROUND=r04 timeout -k 10 500 bash scripts/measure_configs.sh c2 c5 c1 > gpurun_out/cfg_r04.log 2>&1; rc=$?; grep -E "rc=" gpurun_out/cfg_r04.log; exit $rc
