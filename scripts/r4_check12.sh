cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c12
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c12/tests.log 2>&1 || { tail -40 gpurun_out/r4c12/tests.log; exit 1; }
tail -1 gpurun_out/r4c12/tests.log
for v in "" fifo; do
  timeout -k 10 200 python3 scripts/traffic_breakdown.py --batch 10 --groups bytes --variant "$v" --out gpurun_out/r4c12/tb_${v:-product}.json > gpurun_out/r4c12/tb_${v:-product}.log 2>&1 || { tail -5 gpurun_out/r4c12/tb_${v:-product}.log; exit 1; }
  grep -h "total FETCH" gpurun_out/r4c12/tb_${v:-product}.log
done
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/ab_bench.sh RT_LIB_VARIANT=fifo RT_LIB_VARIANT= RT_LIB_VARIANT=fifo RT_LIB_VARIANT= || exit 1
for v in "" fifo; do
  RT_LIB_VARIANT=$v timeout -k 10 300 python3 scripts/with_variant.py scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 1,8 --ranks first > gpurun_out/r4c12/sim_${v:-product}.log 2>&1 || { tail -5 gpurun_out/r4c12/sim_${v:-product}.log; exit 1; }
  grep -h '"n"' gpurun_out/r4c12/sim_${v:-product}.log
done
