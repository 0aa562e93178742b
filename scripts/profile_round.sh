#!/bin/bash
# Round profile of the default bench command: kernel-trace stats, then PMC passes
# (one rocprofv3 run per pass, --pmc only, one frame in flight: the counters are chip-wide):
# HBM traffic (FETCH_SIZE, WRITE_SIZE) and SQ issue counters.  Summarised into $OUT (default profiles/$ROUND) by
# scripts/summarize_profiles.py (run where the repo is, after gpurun merged gpurun_out/).
cd /tmp && export TMPDIR=/tmp
# bench.py's hardware-queue count, here too: the profiler starts HIP first
export GPU_MAX_HW_QUEUES=8
cd "$GRAFT_REPO_ROOT"
ROUND=${ROUND:-r03}
# STEPS/WARMUP: the bench command profiled (STEPS=20 WARMUP=5: the driver's, two 10-frame launches);
# PMC=0 skips the counter passes (kernel trace only), PMC=only skips the kernel trace
STEPS=${STEPS:-24}; WARMUP=${WARMUP:-2}; PMC=${PMC:-1}
O=gpurun_out/prof_$ROUND${TAG:+_$TAG}; rm -rf $O; mkdir -p $O
BENCH="bench.py --steps $STEPS --warmup $WARMUP --no-cpu-baseline --traffic off --no-companions"
if [ "$PMC" != "only" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $BENCH > $O/kt_bench.json 2> $O/kt.log || exit 1
  echo "kernel trace ok"
fi
[ "$PMC" = "0" ] && exit 0
# PMC passes: every tracescreen launch of the run is one 10-frame batch (the driver's), one in
# flight, so the per-kernel means are per 10-frame launch
pmc() { local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- python3 bench.py --steps 10 --warmup 10 --batch 10 --no-cpu-baseline --traffic off --no-companions --frames-in-flight 1 > $O/$n.log 2>&1; local rc=$?; echo "pmc $n rc=$rc"; return $rc; }
pmc fetch FETCH_SIZE && pmc write WRITE_SIZE && pmc ea TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum && \
pmc sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE && \
pmc sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS
# summarised on the build host (only gpurun_out/ comes back): python3 scripts/summarize_profiles.py $O profiles/$ROUND
