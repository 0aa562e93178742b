cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c36
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c36/tests.log 2>&1 || { tail -40 gpurun_out/r4c36/tests.log; exit 1; }
tail -1 gpurun_out/r4c36/tests.log
BENCH_ARGS="--config c5 --steps 8 --warmup 2" bash scripts/ab_bench.sh RT_LIB_VARIANT=head RT_LIB_VARIANT= RT_LIB_VARIANT=head RT_LIB_VARIANT= || exit 1
timeout -k 10 400 python3 scripts/traffic_breakdown.py --batch 4 --groups bytes --timeout 200 --out gpurun_out/r4c36/tb_c5.json --config c5 > gpurun_out/r4c36/tb_c5.log 2>&1 || { tail -5 gpurun_out/r4c36/tb_c5.log; exit 1; }
echo "C5 $(grep -h 'total FETCH' gpurun_out/r4c36/tb_c5.log)"
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/ab_bench.sh RT_LIB_VARIANT=head RT_LIB_VARIANT= || exit 1
