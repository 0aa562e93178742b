#!/bin/bash
# In-flight shard scaling (scripts/inflight_sim.py) once per environment setting.
# usage: inflight_ab.sh "DEPTHS" "VAR=a VAR2=b" ...   (first argument: the --depths list)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ifab
depths=$1; shift
n=0
for setting in "$@"; do
  n=$((n+1))
  env $setting timeout -k 10 300 python3 scripts/inflight_sim.py --depths $depths --ns 1,2,4,8 > gpurun_out/ifab/s$n.log 2>&1 || { echo "sim $n failed"; tail -5 gpurun_out/ifab/s$n.log; exit 1; }
  echo "== $setting"; grep '"depth"' gpurun_out/ifab/s$n.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('  depth', d['depth'], 'n', d['n'], 'frame_ms', d['worst_frame_ms'])"
done
