cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c11
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c11/tests.log 2>&1 || { tail -40 gpurun_out/r4c11/tests.log; exit 1; }
tail -1 gpurun_out/r4c11/tests.log
for v in "" fifo; do
  timeout -k 10 200 python3 scripts/traffic_breakdown.py --batch 10 --groups bytes --variant "$v" --out gpurun_out/r4c11/tb_${v:-product}.json > gpurun_out/r4c11/tb_${v:-product}.log 2>&1 || { tail -5 gpurun_out/r4c11/tb_${v:-product}.log; exit 1; }
  grep -h "total FETCH" gpurun_out/r4c11/tb_${v:-product}.log
done
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/ab_bench.sh RT_LIB_VARIANT=fifo RT_LIB_VARIANT= RT_LIB_VARIANT=fifo RT_LIB_VARIANT= || exit 1
timeout -k 10 200 python3 scripts/shard_util.py 10 1,8 > gpurun_out/r4c11/shard_util.log 2>&1 || { tail -5 gpurun_out/r4c11/shard_util.log; exit 1; }
cat gpurun_out/r4c11/shard_util.log
timeout -k 10 600 bash scripts/pmc_shard.sh || exit 1
