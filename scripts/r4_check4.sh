cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c4
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c4/tests.log 2>&1 || { tail -40 gpurun_out/r4c4/tests.log; exit 1; }
tail -1 gpurun_out/r4c4/tests.log
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 1,8 --lookahead 1 > gpurun_out/r4c4/sim_fused.log 2>&1 || { tail -5 gpurun_out/r4c4/sim_fused.log; exit 1; }
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 1,8 > gpurun_out/r4c4/sim_inline.log 2>&1 || { tail -5 gpurun_out/r4c4/sim_inline.log; exit 1; }
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 1 --depth 3 --frames 24 --ns 1 --lookahead 1 > gpurun_out/r4c4/sim_b1_fused.log 2>&1 || { tail -5 gpurun_out/r4c4/sim_b1_fused.log; exit 1; }
grep -h '"n"' gpurun_out/r4c4/sim_*.log
BENCH_ARGS="--steps 20 --warmup 5 --lookahead 1" bash scripts/ab_bench.sh RT_LIB_VARIANT= RT_LIB_VARIANT= || exit 1
BENCH_ARGS="--steps 20 --warmup 5 --lookahead 0" bash scripts/ab_bench.sh RT_LIB_VARIANT= RT_LIB_VARIANT= || exit 1
