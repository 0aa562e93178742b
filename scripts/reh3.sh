#!/bin/bash
# One 3-rank rehearsal of bench.py's N>1 path on one GPU (gloo staging), progress on stderr.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/reh
export RT_BENCH_SAME_GPU=1 RT_DIST_BACKEND=gloo
timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \
  --master-port 29777 bench.py --gpus 3 --verify --no-cpu-baseline --traffic off --no-companions --steps 10 "$@" > gpurun_out/reh/r3.json 2> >(tee gpurun_out/reh/r3.err >&2)
rc=$?; echo "rc=$rc"; tail -1 gpurun_out/reh/r3.json; exit $rc
