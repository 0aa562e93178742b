#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over the FBM microbenchmark; per-kernel means.
# usage: bash scripts/ubench_pmc.sh [samples]
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ubpmc; rm -rf $O; mkdir -p $O
S=${1:-512}
pmc() { local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- scripts/_build/ubench_fbm $S > $O/$n.log 2>&1
  local rc=$?; echo "pmc $n rc=$rc"; return $rc; }
pmc a SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE && \
pmc b SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_ADDR_CONFLICT SQ_BUSY_CYCLES
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/ubpmc/*/*counter_collection.csv"):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        per[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), d in per.items():
        for c, v in d.items():
            acc[k.split("(")[0]][c].append(v)
for k in sorted(acc):
    print(k)
    for c in sorted(acc[k]):
        v = acc[k][c]
        print("  %-24s %.4g" % (c, sum(v) / len(v)))
PY
