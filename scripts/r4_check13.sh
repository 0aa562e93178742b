cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c13
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4c13/bench_driver.json 2> gpurun_out/r4c13/bench_driver.err || { tail -20 gpurun_out/r4c13/bench_driver.err; exit 1; }
tail -1 gpurun_out/r4c13/bench_driver.json | cut -c1-600
ROUND=r04 STEPS=20 WARMUP=5 timeout -k 10 700 bash scripts/profile_round.sh > gpurun_out/prof_r04.log 2>&1; rc=$?; tail -8 gpurun_out/prof_r04.log; exit $rc
