#!/bin/bash
# Rehearsal of bench.py's N>1 path on ONE GPU box: every rank on cuda:0, collectives through
# gloo (host staging), --verify checks on rank 0 that each assembled frame of the last batch
# equals a whole-frame render.  Timings are meaningless (ranks share one GPU); correctness is not.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/reh
export RT_BENCH_SAME_GPU=1 RT_DIST_BACKEND=gloo RT_BENCH_WATCHDOG=60
PORT=29500
run() { local n=$1; shift; PORT=$((PORT + 1))
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $PORT bench.py --gpus $n --verify --no-cpu-baseline --traffic off "$@" > gpurun_out/reh/$PORT.json \
    2> >(tee gpurun_out/reh/$PORT.err | grep --line-buffered -E "bench rank|Thread|File" >&2) \
    || { echo "n=$n failed"; tail -20 gpurun_out/reh/$PORT.err; return 1; }
  tail -1 gpurun_out/reh/$PORT.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['config']['parallelism'], '->', d['config'].get('verify'))"
}
# `python bench.py --gpus N` without a launcher: bench starts the ranks under torch.distributed.run
selfrun() {
  timeout -k 10 300 python3 bench.py --gpus 2 --verify --no-cpu-baseline --traffic off --no-companions \
    > gpurun_out/reh/self.json 2> gpurun_out/reh/self.err || { echo "self-launch failed"; tail -20 gpurun_out/reh/self.err; return 1; }
  tail -1 gpurun_out/reh/self.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('self-launch', d['n_gpus'], '->', d['config'].get('verify'))"
}
run 2 --no-companions && run 2 --no-companions --lookahead 1 --steps 36 && run 3 --no-companions --steps 10 --split-prepass 1 && run 3 --batch 5 --steps 5 --no-companions && run 4 --split-prepass 1 --batch 5 --steps 5 --no-companions && selfrun  # run 4: split, 4 ranks x 2 frames: rank 3 has none
