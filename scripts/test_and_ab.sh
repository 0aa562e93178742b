#!/bin/bash
# GPU parity tests, then an A/B of the default bench under each environment setting given.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_ab.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_env.sh "$@"
