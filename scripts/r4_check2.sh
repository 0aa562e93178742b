cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c2
for v in "" r3 skip1 skip2 skip4 skip8 skip16 skip64; do
  timeout -k 10 200 python3 scripts/traffic_breakdown.py --batch 10 --groups bytes --variant "$v" --out gpurun_out/r4c2/tb_${v:-product}.json > gpurun_out/r4c2/tb_${v:-product}.log 2>&1 || { tail -5 gpurun_out/r4c2/tb_${v:-product}.log; exit 1; }
  tail -1 gpurun_out/r4c2/tb_${v:-product}.log
done
timeout -k 10 400 python3 scripts/traffic_breakdown.py --batch 10 --out gpurun_out/r4c2/tb_full.json > gpurun_out/r4c2/tb_full.log 2>&1 || { tail -5 gpurun_out/r4c2/tb_full.log; exit 1; }
tail -6 gpurun_out/r4c2/tb_full.log
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/ab_bench.sh RT_LIB_VARIANT= RT_LIB_VARIANT=slots8 RT_LIB_VARIANT=slots4 RT_LIB_VARIANT= RT_LIB_VARIANT=slots8 || exit 1
bash scripts/pmc_lds.sh "" slots8 slots4
