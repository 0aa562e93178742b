#!/bin/bash
# Re-tune k_trace's scheduler knobs at the default bench (RT_LONG_BATCH, RT_REFILL_IDLE,
# RT_COMPACT_LIVE): two passes over the settings below, each a quoted group of env assignments.
cd "$GRAFT_REPO_ROOT"
set -- "RT_REFILL_IDLE=8 RT_COMPACT_LIVE=40" "RT_REFILL_IDLE=4 RT_COMPACT_LIVE=48" \
  "RT_REFILL_IDLE=4 RT_COMPACT_LIVE=56" "RT_REFILL_IDLE=4 RT_COMPACT_LIVE=64" "RT_REFILL_IDLE=2 RT_COMPACT_LIVE=48" \
  "RT_REFILL_IDLE=8 RT_COMPACT_LIVE=56" "RT_REFILL_IDLE=4 RT_COMPACT_LIVE=48 RT_LONG_BATCH=96"
bash scripts/ab_bench.sh "$@" "$@"
