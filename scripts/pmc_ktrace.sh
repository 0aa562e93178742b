#!/bin/bash
# k_trace's issue counters for the product build, as profiles/r04/pmc.md took them: every tracescreen launch a
# 10-frame C3 batch with one batch in flight (the counters are chip-wide), two --pmc passes (8 SQ counters,
# then 7 SQ + GRBM_GUI_ACTIVE), each its own rocprofv3 run; tests/pmc_ratios.py prints the per-launch means of
# the product k_trace and the ratios (cycles per VALU instruction per SIMD, wait and LDS-conflict fractions).
#   gpurun -- bash scripts/pmc_ktrace.sh <tag> [<RT_LIB_VARIANT>]
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; mkdir -p $O
V=${2:-}
run() { local n=$1; shift
  RT_LIB_VARIANT=$V timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- python3 scripts/with_variant.py bench.py \
    --steps 10 --warmup 10 --batch 10 --frames-in-flight 1 --no-cpu-baseline --traffic off --no-companions > $O/$n.log 2>&1
  local rc=$?; echo "$n exit $rc"; return $rc; }
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY && \
run p2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE && \
python3 tests/pmc_ratios.py $O > $O/ratios.txt && cat $O/ratios.txt
