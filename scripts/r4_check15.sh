cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c15
for args in "--transport-us 200 --gate 1" "--transport-us 200" "--transport-us 200 --gate 1" "--transport-us 200" "--gate 1 --transport-us 1" ""; do
  timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 8 --ranks first $args > gpurun_out/r4c15/sim.log 2>&1 || { tail -5 gpurun_out/r4c15/sim.log; exit 1; }
  echo "[$args] $(grep -h '"n"' gpurun_out/r4c15/sim.log)"
done
