#!/bin/bash
# Round-end check of the default build: GPU tests, smoke(), the default bench line (with the CPU
# baseline), then the round profile (kernel trace + PMC passes) for profiles/$ROUND.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/final_tests.log 2>&1 || { tail -5 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 \
  || { tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err \
  || { tail -5 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.json
bash scripts/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -5 gpurun_out/profile_round.log; exit 1; }
tail -1 gpurun_out/profile_round.log
