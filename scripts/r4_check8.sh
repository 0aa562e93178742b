cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c8
for v in "" fprio1 fprio0; do
  RT_LIB_VARIANT=$v timeout -k 10 300 python3 scripts/with_variant.py scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 8 --ranks first --lookahead 1 > gpurun_out/r4c8/n8_${v:-p3}.log 2>&1 || { tail -5 gpurun_out/r4c8/n8_${v:-p3}.log; exit 1; }
  RT_LIB_VARIANT=$v timeout -k 10 300 python3 scripts/with_variant.py scripts/batch_shard_sim.py --batches 1 --depth 3 --frames 24 --ns 1 --lookahead 1 > gpurun_out/r4c8/b1_${v:-p3}.log 2>&1 || { tail -5 gpurun_out/r4c8/b1_${v:-p3}.log; exit 1; }
  echo "variant ${v:-p3}: $(grep -h '"n"' gpurun_out/r4c8/n8_${v:-p3}.log | python3 -c 'import json,sys;print([json.loads(l)["worst_frame_ms"] for l in sys.stdin])') B1 $(grep -h '"n"' gpurun_out/r4c8/b1_${v:-p3}.log | python3 -c 'import json,sys;print([json.loads(l)["worst_frame_ms"] for l in sys.stdin])')"
done
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 8 --ranks first --lookahead 0 > gpurun_out/r4c8/n8_inline.log 2>&1 && grep -h '"n"' gpurun_out/r4c8/n8_inline.log
