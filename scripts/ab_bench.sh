#!/bin/bash
# Same-box A/B of the default bench: one run per environment setting, in the order given
# (repeat a setting to see the run-to-run spread).  usage: ab_bench.sh "VAR=a" "VAR=b" ...
# Prints Mray/s, ms per frame, batch latency, the tracescreen launch (HIP events), the batch's
# noise3d count and its wave iterations (noise / (64 x lane utilisation)).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/abb
n=0
for setting in "$@"; do
  n=$((n+1))
  env $setting timeout -k 10 200 python3 scripts/with_variant.py bench.py --no-cpu-baseline --traffic off --no-companions $BENCH_ARGS > gpurun_out/abb/b$n.json 2> gpurun_out/abb/b$n.err || { echo "bench $n failed"; tail -3 gpurun_out/abb/b$n.err; exit 1; }
  python3 - "$setting" gpurun_out/abb/b$n.json <<'PY'
import json, re, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r, c = d["roofline"], d["config"]
noise = int(re.search(r"x (\d+) noise3d", r["work_unit"]).group(1))
u = c.get("noise_lane_utilisation") or 0
print("== %-28s %8.2f Mray/s %.4f ms/frame  latency %.3f  tracescreen %.3f ms  noise %d  wave-iters %.4g" % (
    sys.argv[1], d["value"], d["ms_per_step"], c["frame_latency_ms"], r["kernel_avg_ms"], noise, noise / (64 * u) if u else 0))
PY
done
