cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c5
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c5/tests.log 2>&1 || { tail -40 gpurun_out/r4c5/tests.log; exit 1; }
tail -1 gpurun_out/r4c5/tests.log
timeout -k 10 200 python3 scripts/traffic_breakdown.py --batch 10 --groups bytes --out gpurun_out/r4c5/tb_bytes.json > gpurun_out/r4c5/tb_bytes.log 2>&1 || { tail -5 gpurun_out/r4c5/tb_bytes.log; exit 1; }
tail -1 gpurun_out/r4c5/tb_bytes.log
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 1,8 --lookahead 1 > gpurun_out/r4c5/sim_fused.log 2>&1 || { tail -5 gpurun_out/r4c5/sim_fused.log; exit 1; }
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 1,8 > gpurun_out/r4c5/sim_inline.log 2>&1 || { tail -5 gpurun_out/r4c5/sim_inline.log; exit 1; }
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 1 --depth 3 --frames 24 --ns 1 --lookahead 1 > gpurun_out/r4c5/sim_b1_fused.log 2>&1 || { tail -5 gpurun_out/r4c5/sim_b1_fused.log; exit 1; }
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 1 --depth 3 --frames 24 --ns 1 --no-prepass > gpurun_out/r4c5/sim_b1_noprepass.log 2>&1 || { tail -5 gpurun_out/r4c5/sim_b1_noprepass.log; exit 1; }
grep -h '"n"' gpurun_out/r4c5/sim_*.log
BENCH_ARGS="--steps 20 --warmup 5 --lookahead 1" bash scripts/ab_bench.sh RT_LIB_VARIANT= RT_LIB_VARIANT= || exit 1
BENCH_ARGS="--steps 20 --warmup 5 --lookahead 0" bash scripts/ab_bench.sh RT_LIB_VARIANT= RT_LIB_VARIANT= || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4c5/bench.json 2> gpurun_out/r4c5/bench.err || { tail -20 gpurun_out/r4c5/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4c5/bench.json'));c=d['config'];print(d['value'],d['roofline']['frac'],d['roofline'].get('traffic_per_frame_vs_rgba8'),c['single_frame']['primary_plus_shadow_mrays'],c['noise_lane_utilisation'],c['timed_capture_check'],c['parity']['timed_frames_all_equal'])"
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/ab_bench.sh RT_LIB_VARIANT=octsmem RT_LIB_VARIANT= RT_LIB_VARIANT=octsmem RT_LIB_VARIANT= || exit 1
