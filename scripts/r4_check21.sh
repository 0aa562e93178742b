cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c21
for v in "" skip4 skip8 skip16; do
  timeout -k 10 400 python3 scripts/traffic_breakdown.py --batch 4 --groups bytes --timeout 200 --variant "$v" --out gpurun_out/r4c21/tb_c5_${v:-product}.json --config c5 > gpurun_out/r4c21/tb_${v:-product}.log 2>&1 || { tail -5 gpurun_out/r4c21/tb_${v:-product}.log; exit 1; }
  grep -h "total FETCH" gpurun_out/r4c21/tb_${v:-product}.log
done
