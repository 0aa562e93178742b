cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4final
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4final/tests.log 2>&1 || { tail -40 gpurun_out/r4final/tests.log; exit 1; }
tail -1 gpurun_out/r4final/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4final/smoke.log 2>&1 || { tail -20 gpurun_out/r4final/smoke.log; exit 1; }
tail -1 gpurun_out/r4final/smoke.log
timeout -k 10 500 python3 bench.py > gpurun_out/r4final/bench_default.json 2> gpurun_out/r4final/bench_default.err || { tail -20 gpurun_out/r4final/bench_default.err; exit 1; }
tail -1 gpurun_out/r4final/bench_default.json | cut -c1-300
