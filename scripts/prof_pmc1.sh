#!/bin/bash
# profiling session 1: kernel trace stats + counter list
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof1
timeout -k 10 120 rocprofv3 -L > gpurun_out/prof1/counters.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1/kt -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof1/bench.log 2>&1
echo "kt exit $?"
