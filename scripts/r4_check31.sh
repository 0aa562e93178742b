cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c31
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c31/tests.log 2>&1 || { tail -40 gpurun_out/r4c31/tests.log; exit 1; }
tail -1 gpurun_out/r4c31/tests.log
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/ab_bench.sh RT_LIB_VARIANT=head RT_LIB_VARIANT= RT_LIB_VARIANT=head RT_LIB_VARIANT= || exit 1
BENCH_ARGS="--config c5 --steps 8 --warmup 2" bash scripts/ab_bench.sh RT_LIB_VARIANT=head RT_LIB_VARIANT= || exit 1
