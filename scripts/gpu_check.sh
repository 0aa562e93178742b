#!/bin/bash
# One GPU call: the -m gpu tests, the default bench line (with CPU baseline, parity, companions),
# then the N>1 rehearsal (bench.py's multi-rank path on one GPU through gloo).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/check_tests.log 2>&1 || { tail -30 gpurun_out/check_tests.log; exit 1; }
tail -2 gpurun_out/check_tests.log
timeout -k 10 400 python3 bench.py > gpurun_out/check_bench.json 2> gpurun_out/check_bench.err \
  || { tail -20 gpurun_out/check_bench.err; exit 1; }
tail -c 3000 gpurun_out/check_bench.json
[ -n "$NOREH" ] && exit 0
bash scripts/rehearse_multi.sh
