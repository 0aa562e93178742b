cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c16
RT_LIB_VARIANT=refill16 timeout -k 10 300 python3 -u scripts/with_variant.py -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "frame or batch or fused or degenerate or config" > gpurun_out/r4c16/tests.log 2>&1 || { tail -40 gpurun_out/r4c16/tests.log; exit 1; }
tail -1 gpurun_out/r4c16/tests.log
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/ab_bench.sh RT_LIB_VARIANT= RT_LIB_VARIANT=refill8 RT_LIB_VARIANT=refill16 RT_LIB_VARIANT=refill32 RT_LIB_VARIANT= RT_LIB_VARIANT=refill16 || exit 1
