#!/bin/bash
# GPU parity tests, then per environment setting: the default bench (steady state, one-frame
# latency, isolated tracescreen launch) and the 8-way shard simulation (rank-max frame time).
# usage: ab_quick.sh "VAR=a" "VAR=b" ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/abq
timeout -k 10 400 python3 -m pytest tests -m gpu -x -q > gpurun_out/abq/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/abq/pytest.log; [ $rc -eq 0 ] || exit $rc
n=0
for setting in "$@"; do
  n=$((n+1))
  env $setting timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/abq/b$n.json 2> gpurun_out/abq/b$n.err || { echo "bench $n failed"; exit 1; }
  env $setting timeout -k 10 200 python3 scripts/shard_sim.py --ns 1,8 --steps 5 > gpurun_out/abq/s$n.log 2> gpurun_out/abq/s$n.err || { echo "shard_sim $n failed"; exit 1; }
  python3 - "$setting" gpurun_out/abq/b$n.json gpurun_out/abq/s$n.log <<'PY'
import json, sys
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
s = [json.loads(l) for l in open(sys.argv[3]) if l.startswith("{")]
n8 = [x for x in s if x.get("n") == 8][0]
print(f"== {sys.argv[1]}: {b['value']} Mray/s  {b['ms_per_step']} ms/frame  latency {b['config']['frame_latency_ms']}  "
      f"tracescreen {b['roofline']['kernel_avg_ms']}  | N=8 rank-max {n8['worst_frame_ms']} ms "
      f"(tracescreen {max(r['tracescreen_ms'] for r in n8['ranks'])})")
PY
done
