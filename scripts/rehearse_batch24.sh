cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/reh24
export RT_BENCH_SAME_GPU=1 RT_DIST_BACKEND=gloo RT_BENCH_WATCHDOG=60
for n in 2 4; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --verify --no-cpu-baseline --traffic off --batch 24 --steps 20 --warmup 5 \
    > gpurun_out/reh24/n$n.json 2> gpurun_out/reh24/n$n.err || { echo "n=$n failed"; tail -20 gpurun_out/reh24/n$n.err; exit 1; }
  tail -1 gpurun_out/reh24/n$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['config'].get('global_batch', d['config'].get('batch')), d['config']['parallelism'], '->', d['config'].get('verify'))"
done
