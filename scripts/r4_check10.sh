cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c10
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c10/tests.log 2>&1 || { tail -40 gpurun_out/r4c10/tests.log; exit 1; }
tail -1 gpurun_out/r4c10/tests.log
for b in 20 10; do
  timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches $b --frames 20 --ns 1,8 --ranks first > gpurun_out/r4c10/sim_b$b.log 2>&1 || { tail -5 gpurun_out/r4c10/sim_b$b.log; exit 1; }
  grep -h '"n"' gpurun_out/r4c10/sim_b$b.log
done
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 20 --frames 20 --ns 4,2 --ranks first > gpurun_out/r4c10/sim_b20_n42.log 2>&1 && grep -h '"n"' gpurun_out/r4c10/sim_b20_n42.log
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 4,2 --ranks first > gpurun_out/r4c10/sim_b10_n42.log 2>&1 && grep -h '"n"' gpurun_out/r4c10/sim_b10_n42.log
BENCH_ARGS="--steps 20 --warmup 5 --batch 20" bash scripts/ab_bench.sh RT_LIB_VARIANT= RT_LIB_VARIANT= || exit 1
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/ab_bench.sh RT_LIB_VARIANT= RT_LIB_VARIANT= || exit 1
