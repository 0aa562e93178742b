#!/bin/bash
# PMC passes on the default bench (one batch in flight), k_trace-focused counter groups:
# VALU issue (single / dual), wave cycles and waits, LDS latency and conflicts, instruction mix.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pv; rm -rf $O; mkdir -p $O
pmc() { local n=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- python3 bench.py --steps 12 --warmup 1 \
    --no-cpu-baseline --traffic off --no-companions --frames-in-flight 1 > $O/$n.log 2>&1; local rc=$?; echo "pmc $n rc=$rc"; return $rc; }
pmc a SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE && \
pmc b SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY && \
pmc c SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_SMEM
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob("gpurun_out/pv/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_trace" not in k or "true" in k.split("<")[1].split(",")[1]: continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    print(k[:60])
    for c in sorted(d): print("  %-26s %.4g" % (c, d[c]))
PY
