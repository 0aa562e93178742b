cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c26
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ao or c5 or config or frame_bitexact" > gpurun_out/r4c26/tests.log 2>&1 || { tail -40 gpurun_out/r4c26/tests.log; exit 1; }
tail -1 gpurun_out/r4c26/tests.log
BENCH_ARGS="--config c5 --steps 8 --warmup 2" bash scripts/ab_bench.sh RT_LIB_VARIANT=nores RT_LIB_VARIANT= RT_LIB_VARIANT=nores RT_LIB_VARIANT= || exit 1
for v in "" nores; do
timeout -k 10 400 python3 scripts/traffic_breakdown.py --batch 4 --groups bytes --timeout 200 --variant "$v" --out gpurun_out/r4c26/tb_c5_${v:-product}.json --config c5 > gpurun_out/r4c26/tb_c5.log 2>&1 || { tail -5 gpurun_out/r4c26/tb_c5.log; exit 1; }
echo "C5 ${v:-product} $(grep -h 'total FETCH' gpurun_out/r4c26/tb_c5.log)"
done
