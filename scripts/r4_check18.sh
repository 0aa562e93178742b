cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c18
RT_LIB_VARIANT=hitpad timeout -k 10 300 python3 -u scripts/with_variant.py -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "frame_bitexact_device_path or config_batch_rows or mixed_cameras" > gpurun_out/r4c18/tests.log 2>&1 || { tail -40 gpurun_out/r4c18/tests.log; exit 1; }
tail -1 gpurun_out/r4c18/tests.log
for v in "" hitpad "" hitpad; do
  timeout -k 10 200 python3 scripts/traffic_breakdown.py --batch 10 --groups bytes --variant "$v" --out gpurun_out/r4c18/tb_${v:-product}.json > gpurun_out/r4c18/tb_${v:-product}.log 2>&1 || { tail -5 gpurun_out/r4c18/tb_${v:-product}.log; exit 1; }
  grep -h "total FETCH" gpurun_out/r4c18/tb_${v:-product}.log
done
