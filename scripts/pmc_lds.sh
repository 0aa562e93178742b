#!/bin/bash
# k_trace LDS counters of library variants (RT_LIB_VARIANT per argument, "" = default build): one --pmc
# pass per variant, one batch in flight; bank-conflict cycles / LDS-array cycles, LDS waits, cycles per
# VALU instruction.  usage: pmc_lds.sh v1 v2 ...
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmcl; rm -rf $O; mkdir -p $O
for v in "$@"; do
  tag=${v:-default}
  RT_LIB_VARIANT=$v timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d $O/$tag -o run -- python3 scripts/with_variant.py bench.py --steps 10 --warmup 1 --no-cpu-baseline --traffic off --no-companions --frames-in-flight 1 > $O/$tag.log 2>&1 || { echo "pmc $tag failed"; exit 1; }
  python3 - $O/$tag $tag <<'PY'
import csv, glob, re, sys, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        if n.startswith("k_trace") and not re.match(r"k_trace<\d+, true", n):
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
d = {c: sum(x[c] for x in per.values()) / len(per) for c in next(iter(per.values()))}
cyc = d["GRBM_GUI_ACTIVE"] / 8
print("== %-10s k_trace cycles %.4g  VALU %.4g  LDS instrs %.4g  bank-conflict/LDS-active %.3f  LDS-active/cycle/CU %.3f  wait_lds %.3f  cyc/VALU %.3f" % (
    sys.argv[2], cyc, d["SQ_INSTS_VALU"], d["SQ_INSTS_LDS"], d["SQ_LDS_BANK_CONFLICT"] / d["SQ_LDS_IDX_ACTIVE"],
    d["SQ_LDS_IDX_ACTIVE"] / (cyc * 256), d["SQ_WAIT_INST_LDS"] / d["SQ_WAVE_CYCLES"], cyc * 1024 / d["SQ_INSTS_VALU"]))
PY
done
