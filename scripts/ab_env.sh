#!/bin/bash
# A/B: kernel-trace the default bench under several environment settings.
# usage: ab_env.sh "VAR=a" "VAR=b" ...
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; rm -rf $O; mkdir -p $O
n=0
for setting in "$@"; do
  n=$((n+1))
  env $setting timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.log || { echo "run $n failed"; exit 1; }
  echo "== $setting"; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
  python3 - $O/$n <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "true>" in r["Name"] or "rocclr" in r["Name"]:
        continue
    print("   %-40s %8.4f" % (r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0], float(r["AverageNs"]) / 1e6))
PY
done
