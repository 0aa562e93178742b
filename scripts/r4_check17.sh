cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c17
for c in c5 c2 c1; do
  timeout -k 10 500 python3 bench.py --config $c --steps 8 --warmup 2 --no-companions > gpurun_out/r4c17/bench_$c.json 2> gpurun_out/r4c17/bench_$c.err || { echo "$c failed"; tail -20 gpurun_out/r4c17/bench_$c.err; exit 1; }
  tail -1 gpurun_out/r4c17/bench_$c.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', d['value'], d['unit'], 'frac', r['frac'], 'x rgba8', d['config'].get('traffic_per_frame_vs_rgba8', r.get('traffic_per_frame_vs_rgba8')))"
done
