cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4simf
timeout -k 10 600 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 1,2,4,8 --ranks all > gpurun_out/r4simf/sim.log 2>&1 || { tail -5 gpurun_out/r4simf/sim.log; exit 1; }
grep -h '"n"' gpurun_out/r4simf/sim.log
timeout -k 10 600 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 8 --ranks first --transport-us 200 > gpurun_out/r4simf/simt.log 2>&1 || { tail -5 gpurun_out/r4simf/simt.log; exit 1; }
grep -h '"n"' gpurun_out/r4simf/simt.log
