cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c3
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c3/tests.log 2>&1 || { tail -40 gpurun_out/r4c3/tests.log; exit 1; }
tail -1 gpurun_out/r4c3/tests.log
timeout -k 10 200 python3 scripts/traffic_breakdown.py --batch 10 --out gpurun_out/r4c3/tb_full.json > gpurun_out/r4c3/tb_full.log 2>&1 || { tail -5 gpurun_out/r4c3/tb_full.log; exit 1; }
tail -6 gpurun_out/r4c3/tb_full.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4c3/bench.json 2> gpurun_out/r4c3/bench.err || { tail -20 gpurun_out/r4c3/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4c3/bench.json'));c=d['config'];print(d['value'],d['roofline']['frac'],d['roofline'].get('traffic_per_frame_vs_rgba8'),c['single_frame']['primary_plus_shadow_mrays'],c['noise_lane_utilisation'],c['timed_capture_check'],c['parity']['timed_frames_all_equal'])"
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 1 --depth 3 --frames 24 --ns 1 --lookahead 1 > gpurun_out/r4c3/sim_b1.log 2>&1 || { tail -5 gpurun_out/r4c3/sim_b1.log; exit 1; }
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 1 --depth 3 --frames 24 --ns 1 --no-prepass > gpurun_out/r4c3/sim_b1_noprepass.log 2>&1 || { tail -5 gpurun_out/r4c3/sim_b1_noprepass.log; exit 1; }
tail -1 gpurun_out/r4c3/sim_b1.log gpurun_out/r4c3/sim_b1_noprepass.log
