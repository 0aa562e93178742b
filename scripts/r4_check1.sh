cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r4c1/tests.log 2>&1 || { tail -40 gpurun_out/r4c1/tests.log; exit 1; }
tail -1 gpurun_out/r4c1/tests.log; grep "noise lane utilisation 64x48" gpurun_out/r4c1/tests.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4c1/bench.json 2> gpurun_out/r4c1/bench.err || { tail -20 gpurun_out/r4c1/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4c1/bench.json'));c=d['config'];print(d['value'],d['roofline']['frac'],d['roofline'].get('traffic_per_frame_vs_rgba8'),c['single_frame']['primary_plus_shadow_mrays'],c['noise_lane_utilisation'],c['timed_capture_check'],c['per_rank'])"
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/ab_bench.sh RT_LIB_VARIANT=r3 RT_LIB_VARIANT= RT_LIB_VARIANT=r3 RT_LIB_VARIANT=
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 1,8 > gpurun_out/r4c1/sim_inline.log 2>&1 || { tail -5 gpurun_out/r4c1/sim_inline.log; exit 1; }
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 1,8 --no-prepass > gpurun_out/r4c1/sim_noprepass.log 2>&1 || { tail -5 gpurun_out/r4c1/sim_noprepass.log; exit 1; }
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 1,8 --no-prepass --depth 1 > gpurun_out/r4c1/sim_noprepass_d1.log 2>&1 || { tail -5 gpurun_out/r4c1/sim_noprepass_d1.log; exit 1; }
tail -2 gpurun_out/r4c1/sim_inline.log gpurun_out/r4c1/sim_noprepass.log gpurun_out/r4c1/sim_noprepass_d1.log
