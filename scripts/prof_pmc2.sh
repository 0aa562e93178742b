#!/bin/bash
# profiling session 2: PMC counter passes (each its own run; no trace domains mixed in)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof2; mkdir -p $O
run() { # name counters...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > $O/$n.log 2>&1
  echo "$n exit $?"
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY && \
run p2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE && \
run p3 FETCH_SIZE && run p4 WRITE_SIZE && run p5 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS
