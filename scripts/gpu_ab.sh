#!/bin/bash
# One GPU call for a candidate build against a variant (default: `base`, the previous build):
# optional microbenchmark binaries, the -m gpu tests on the candidate (the product library),
# then a same-box A/B of the default bench, alternating.  usage: gpu_ab.sh [variant] [ubench ...]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=${1:-base}; shift
for u in "$@"; do
  timeout -k 10 60 scripts/_build/$u > gpurun_out/$u.txt 2>&1 || { echo "$u failed"; exit 1; }
  cat gpurun_out/$u.txt
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
bash scripts/ab_bench.sh RT_LIB_VARIANT=$V RT_LIB_VARIANT= RT_LIB_VARIANT=$V RT_LIB_VARIANT=
