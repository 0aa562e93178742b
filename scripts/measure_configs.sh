#!/bin/bash
# One GPU call: bench lines for the BASELINE GPU configs C2 / C5 (and C3 default, ref semantics),
# each under rocprofv3 --kernel-trace --stats (so --traffic off: no profiler inside the profiler),
# outputs under gpurun_out/cfg_$ROUND/.
# usage: ROUND=r02 bash scripts/measure_configs.sh [configs...]   (default: c2 c5 c3 ref)
cd /tmp && export TMPDIR=/tmp
# bench.py's hardware-queue count, here too: the profiler starts HIP first
export GPU_MAX_HW_QUEUES=8
cd "$GRAFT_REPO_ROOT"
ROUND=${ROUND:-r03}
O=gpurun_out/cfg_$ROUND; mkdir -p $O
CFGS=${*:-c2 c5 c3 ref}
for c in $CFGS; do
  extra=""
  [ "$c" = "c5" ] && extra="--cpu-row-step 16"
  [ "$c" = "c3" ] && extra="--cpu-row-step 8"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$c -o run -- \
    python3 bench.py --config $c --steps 24 --warmup 2 --traffic off $extra > $O/bench_$c.json 2> $O/bench_$c.log
  rc=$?; echo "$c rc=$rc"; tail -c 600 $O/bench_$c.json
  [ $rc -ne 0 ] && { tail -20 $O/bench_$c.log; exit $rc; }
done
exit 0
