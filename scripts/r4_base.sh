cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4base
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4base/tests.log 2>&1 || { tail -30 gpurun_out/r4base/tests.log; exit 1; }
tail -1 gpurun_out/r4base/tests.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4base/bench.json 2> gpurun_out/r4base/bench.err || { tail -20 gpurun_out/r4base/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4base/bench.json'));print(d['value'],d['roofline']['frac'],d['roofline'].get('traffic_per_frame_vs_rgba8'),d['config']['single_frame']['primary_plus_shadow_mrays'])"
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 1,8 > gpurun_out/r4base/sim.log 2>&1 || { tail -5 gpurun_out/r4base/sim.log; exit 1; }
tail -3 gpurun_out/r4base/sim.log
