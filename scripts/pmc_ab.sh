#!/bin/bash
# HBM traffic + speed of library variants: for each RT_LIB_VARIANT given ("" = the default build),
# one bench run, then FETCH_SIZE and WRITE_SIZE passes with one frame in flight; prints k_trace's means.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmcab; rm -rf $O; mkdir -p $O
for v in "$@"; do
  tag=${v:-default}
  RT_LIB_VARIANT=$v timeout -k 10 200 python3 scripts/with_variant.py bench.py --no-cpu-baseline --traffic off > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    RT_LIB_VARIANT=$v timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d $O/$tag-$c -o run -- python3 scripts/with_variant.py bench.py --steps 3 --warmup 1 --no-cpu-baseline --traffic off --frames-in-flight 1 > $O/$tag-$c.log 2>&1 || { echo "pmc $tag $c failed"; exit 1; }
  done
  python3 - $O $tag <<'PY'
import csv, glob, json, sys, collections
o, tag = sys.argv[1], sys.argv[2]
b = json.loads(open(f"{o}/{tag}.json").read().strip().splitlines()[-1])
out = [f"== {tag}: {b['value']} Mray/s, tracescreen {b['roofline']['kernel_avg_ms']} ms"]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{o}/{tag}-{c}/**/*counter_collection.csv", recursive=True)[0]
    d = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "k_trace" in r["Kernel_Name"] and "true>" not in r["Kernel_Name"]:
            d[r["Dispatch_Id"]] += float(r["Counter_Value"])
    out.append(f"k_trace {c} {sum(d.values()) / max(1, len(d)) / 1024:.1f} MiB")
print("  ".join(out))
PY
done
