cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c14
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c14/tests.log 2>&1 || { tail -40 gpurun_out/r4c14/tests.log; exit 1; }
tail -1 gpurun_out/r4c14/tests.log
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/ab_bench.sh RT_LIB_VARIANT=static RT_LIB_VARIANT= RT_LIB_VARIANT=static RT_LIB_VARIANT= || exit 1
for v in static "" static ""; do
  RT_LIB_VARIANT=$v timeout -k 10 300 python3 scripts/with_variant.py scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 8 --ranks first > gpurun_out/r4c14/sim.log 2>&1 || { tail -5 gpurun_out/r4c14/sim.log; exit 1; }
  echo "${v:-product} $(grep -h '"n"' gpurun_out/r4c14/sim.log)"
done
for tu in 200 0 200; do
  timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 1,8 --ranks first --transport-us $tu > gpurun_out/r4c14/simt.log 2>&1 || { tail -5 gpurun_out/r4c14/simt.log; exit 1; }
  grep -h '"n"' gpurun_out/r4c14/simt.log
done
for v in "" res2 res8 "" res2 res8; do
  RT_LIB_VARIANT=$v timeout -k 10 300 python3 scripts/with_variant.py scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 8 --ranks first --transport-us 200 > gpurun_out/r4c14/sim.log 2>&1 || { tail -5 gpurun_out/r4c14/sim.log; exit 1; }
  echo "${v:-product} $(grep -h '"n"' gpurun_out/r4c14/sim.log)"
done
for v in "" res2; do
  RT_LIB_VARIANT=$v timeout -k 10 300 python3 scripts/with_variant.py scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 8 --ranks first > gpurun_out/r4c14/sim.log 2>&1 || { tail -5 gpurun_out/r4c14/sim.log; exit 1; }
  echo "no transport ${v:-product} $(grep -h '"n"' gpurun_out/r4c14/sim.log)"
done
