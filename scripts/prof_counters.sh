#!/bin/bash
# PMC passes (each its own rocprofv3 run, --pmc only) over a short bench; summary via tests/pmc_summary.py.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${PROF_TAG:-prof}; mkdir -p $O
run() { local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --traffic off > $O/$n.log 2>&1; local rc=$?; echo "$n exit $rc"; return $rc; }
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY && \
run p2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE && \
python3 tests/pmc_summary.py $O > $O/summary.txt && cat $O/summary.txt
