#!/bin/bash
# GPU parity tests, then the default bench once per argument string (A/B of bench flags).
# usage: ab_args.sh "--graph 1" "--graph 0" ...   (set NOTEST=1 to skip the tests)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/aba
if [ -z "$NOTEST" ]; then
  timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/aba/pytest.log 2>&1; rc=$?
  tail -1 gpurun_out/aba/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
n=0
for args in "$@"; do
  n=$((n+1))
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --traffic off $args > gpurun_out/aba/b$n.json 2> gpurun_out/aba/b$n.err || { echo "bench $n failed"; exit 1; }
  python3 - "$args" gpurun_out/aba/b$n.json <<'PY'
import json, sys
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"== {sys.argv[1]}: {b['value']} Mray/s  {b['ms_per_step']} ms/frame  latency {b['config']['frame_latency_ms']}  "
      f"tracescreen {b['roofline']['kernel_avg_ms']}")
PY
done
