cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ss; export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/shard_sim.py --ns 8 --steps 5 > gpurun_out/ss/split.log 2>&1 &&
RT_PIPELINE=staged timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ss/staged -- python3 scripts/shard_sim.py --ns 8 --steps 5 > gpurun_out/ss/staged.log 2>&1 &&
timeout -k 10 200 python3 scripts/shard_sim.py --ns 1,8 --steps 5 --max-steps 128 --ao 0 > gpurun_out/ss/cap128.log 2>&1 &&
timeout -k 10 200 python3 scripts/shard_sim.py --ns 1,8 --steps 5 --ao 0 > gpurun_out/ss/ao0.log 2>&1
