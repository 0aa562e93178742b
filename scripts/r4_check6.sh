cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c6
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c6/tests.log 2>&1 || { tail -40 gpurun_out/r4c6/tests.log; exit 1; }
tail -1 gpurun_out/r4c6/tests.log
for la in 1 0; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4c6/kt_la$la -o run -- python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 8 --ranks first --lookahead $la > gpurun_out/r4c6/kt_la$la.log 2>&1 || { tail -5 gpurun_out/r4c6/kt_la$la.log; exit 1; }
  f=$(find gpurun_out/r4c6/kt_la$la -name "*kernel_trace.csv" | head -1)
  python3 scripts/timeline.py $f 8 > gpurun_out/r4c6/timeline_la$la.txt
  grep '"n"' gpurun_out/r4c6/kt_la$la.log
done
rm -rf gpurun_out/r4c6/kt_la*/
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/ab_bench.sh RT_LIB_VARIANT= RT_LIB_VARIANT= || exit 1
