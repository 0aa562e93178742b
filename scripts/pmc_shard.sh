#!/bin/bash
# k_trace counters of rank 0's share of 10-frame C3 batches at N = 1 and N = 8 (one-GPU shard
# simulation; rocprofv3 serialises the dispatches): VALU instructions per k_trace x N against N = 1
# (the same work?) and cycles per VALU instruction (the same issue efficiency?).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmcs; rm -rf $O; mkdir -p $O
for n in 1 8; do
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $O/n$n -o run -- python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns $n --ranks first > $O/n$n.log 2>&1 || { echo "pmc n$n failed"; tail -3 $O/n$n.log; exit 1; }
  python3 - $O/n$n $n <<'PY'
import csv, glob, re, sys, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        nm = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        if nm.startswith("k_trace") and not re.match(r"k_trace<\d+, true", nm):
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
n = int(sys.argv[2])
d = {c: sum(x[c] for x in per.values()) / len(per) for c in next(iter(per.values()))}
cyc = d["GRBM_GUI_ACTIVE"] / 8
print("== N=%d k_trace dispatches %d  cycles %.4g  VALU %.4g (x N %.4g)  SALU %.4g  LDS %.4g  wave-cycles %.4g  wait_any/wave %.3f  active_valu/wave %.3f  cyc/VALU %.3f" % (
    n, len(per), cyc, d["SQ_INSTS_VALU"], d["SQ_INSTS_VALU"] * n, d["SQ_INSTS_SALU"], d["SQ_INSTS_LDS"], d["SQ_WAVE_CYCLES"],
    d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"], d["SQ_ACTIVE_INST_VALU"] / d["SQ_WAVE_CYCLES"], cyc * 1024 / d["SQ_INSTS_VALU"]))
PY
done
