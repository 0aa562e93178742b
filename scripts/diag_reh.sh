cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/reh
export RT_BENCH_SAME_GPU=1 RT_DIST_BACKEND=gloo
P=29600
for args in "2" "3 --steps 10" "2" "3 --steps 10" "3 --steps 12" "3 --steps 10" "4 --steps 10" "3 --steps 10"; do
  set -- $args; n=$1; shift; P=$((P+1))
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $P bench.py --gpus $n --verify --no-cpu-baseline --traffic off --no-companions "$@" > gpurun_out/reh/d$P.json 2> gpurun_out/reh/d$P.err || { echo fail; tail -5 gpurun_out/reh/d$P.err; exit 1; }
  echo "== $args"; tail -1 gpurun_out/reh/d$P.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['batches'], d['config'].get('verify'))"
done
