#!/bin/bash
# Same-box A/B of the default bench: one run per environment setting, in the order given
# (repeat a setting to see the run-to-run spread).  usage: ab_bench.sh "VAR=a" "VAR=b" ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/abb
n=0
for setting in "$@"; do
  n=$((n+1))
  env $setting timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-companions $BENCH_ARGS > gpurun_out/abb/b$n.json 2> gpurun_out/abb/b$n.err || { echo "bench $n failed"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/abb/b$n.json').read().strip().splitlines()[-1]); print('== $setting:', d['value'], 'Mray/s', d['ms_per_step'], 'ms  latency', d['config']['frame_latency_ms'], ' tracescreen', d['roofline']['kernel_avg_ms'])"
done
