#!/bin/bash
# Round 6 A/B of the segment march (post-drain long rays): per-wave timelines (trace builds) of one frame
# and of rank 0 of a 10-frame batch at N = 8, the N = 8 rank-0 shard simulation and the bench line with the
# single-frame companions, for each build named on the command line ("default" = the product build);
# output under gpurun_out/<out>/<variant>/.
#   gpurun -- bash scripts/ab_seg.sh <out> <variant> [<variant> ...]
cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; shift
for v in "$@"; do
  tv=trace; pv=$v
  [ "$v" = default ] && pv= || tv=trace_$v
  bash scripts/gpu_run.sh "$out/$v" "vpy=$tv:scripts/wave_trace.py --batch 1" \
    "vpy=$tv:scripts/wave_trace.py --batch 10 --n 8" \
    "vpy=$pv:scripts/batch_shard_sim.py --batches 10 --ns 8 --frames 20 --ranks first" \
    "vbench=$pv:--no-cpu-baseline --traffic off" || exit 1
done
