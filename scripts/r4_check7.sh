cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c7
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/r4c7/ht -o run -- python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 8 --ranks first --lookahead 0 > gpurun_out/r4c7/ht.log 2>&1 || { tail -5 gpurun_out/r4c7/ht.log; exit 1; }
f=$(find gpurun_out/r4c7/ht -name "*hip_api_trace.csv" | head -1)
python3 - "$f" > gpurun_out/r4c7/api_summary.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
c = collections.Counter(r["Function"] for r in rows)
for k, v in c.most_common(40): print(v, k)
# the last 400 calls in order
t0 = int(rows[-400]["Start_Timestamp"]) if len(rows) > 400 else int(rows[0]["Start_Timestamp"])
for r in rows[-400:]:
    if "Memcpy" in r["Function"] or "Memset" in r["Function"] or "Launch" in r["Function"] or "Graph" in r["Function"]:
        print((int(r["Start_Timestamp"]) - t0) / 1e6, r["Function"], r.get("Args", "")[:120])
PY
head -60 gpurun_out/r4c7/api_summary.txt
rm -rf gpurun_out/r4c7/ht
mkdir -p gpurun_out/r4c8
for v in "" fprio1 fprio0; do
  RT_LIB_VARIANT=$v timeout -k 10 300 python3 scripts/with_variant.py scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 8 --ranks first --lookahead 1 > gpurun_out/r4c8/n8_${v:-p3}.log 2>&1 || { tail -5 gpurun_out/r4c8/n8_${v:-p3}.log; exit 1; }
  RT_LIB_VARIANT=$v timeout -k 10 300 python3 scripts/with_variant.py scripts/batch_shard_sim.py --batches 1 --depth 3 --frames 24 --ns 1 --lookahead 1 > gpurun_out/r4c8/b1_${v:-p3}.log 2>&1 || { tail -5 gpurun_out/r4c8/b1_${v:-p3}.log; exit 1; }
  echo "variant ${v:-p3}: $(grep -h '"n"' gpurun_out/r4c8/n8_${v:-p3}.log | python3 -c 'import json,sys;print([json.loads(l)["worst_frame_ms"] for l in sys.stdin])') B1 $(grep -h '"n"' gpurun_out/r4c8/b1_${v:-p3}.log | python3 -c 'import json,sys;print([json.loads(l)["worst_frame_ms"] for l in sys.stdin])')"
done
timeout -k 10 300 python3 scripts/batch_shard_sim.py --batches 10 --frames 20 --ns 8 --ranks first --lookahead 0 > gpurun_out/r4c8/n8_inline.log 2>&1 && grep -h '"n"' gpurun_out/r4c8/n8_inline.log
