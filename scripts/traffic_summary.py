"""HBM bytes per tracescreen launch from scripts/traffic_pass.sh (2*FETCH_SIZE + WRITE_SIZE, KiB
counters, MI355X_MICROARCH.md HBM rule), per kernel and per frame against the 8.3 MB RGBA8 frame.
usage: traffic_summary.py [dir] [frames per launch] [traffic.json to merge the launch into]
(the key is bench.py's: taken from the bench line in <dir>/fetch.log)"""
import collections
import csv
import glob
import json
import os
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/traffic"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 12
tot = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(src + "/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        per[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), cs in per.items():
        name = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        if "true" in name:
            continue  # the instrumented (STATS) frame
        for c, v in cs.items():
            tot[name][c].append(v)
s = 0.0
for k in sorted(tot):
    if any(k.startswith(x) for x in ("k_trace", "k_finish", "k_order")):
        d = {c: sum(v) / len(v) for c, v in tot[k].items()}
        b = (2 * d.get("FETCH_SIZE", 0) + d.get("WRITE_SIZE", 0)) * 1024
        s += b
        print("%-28s FETCH %8.1f MiB  WRITE %8.1f MiB  -> %7.1f MB" % (k, d.get("FETCH_SIZE", 0) / 1024,
                                                                     d.get("WRITE_SIZE", 0) / 1024, b / 1e6))
print("tracescreen launch %.1f MB = %.1f MB per frame = %.1fx the 8.3 MB RGBA8 frame" % (s / 1e6, s / frames / 1e6,
                                                                                         s / frames / 8.2944e6))

if len(sys.argv) > 3:
    bench = [line for line in open(os.path.join(src, "fetch.log")) if line.startswith("{")][-1]
    cf = json.loads(bench)["config"]
    key = (f"{cf['width']}x{cf['height']}_{cf['landscape']}_{cf['pose']}_ms{cf['max_steps']}_ao{cf.get('ao_samples', 0)}"
           f"_b{cf.get('batch', 1)}")
    fetch = sum(sum(v) / len(v) for k, cs in tot.items() for c, v in cs.items() if c == "FETCH_SIZE"
                and any(k.startswith(x) for x in ("k_trace", "k_finish", "k_order")))
    write = sum(sum(v) / len(v) for k, cs in tot.items() for c, v in cs.items() if c == "WRITE_SIZE"
                and any(k.startswith(x) for x in ("k_trace", "k_finish", "k_order")))
    tj = json.load(open(sys.argv[3])) if os.path.exists(sys.argv[3]) else {}
    tj[key] = {"hbm_bytes_per_launch": int(2 * fetch * 1024 + write * 1024), "fetch_size_kib": fetch,
               "write_size_kib": write,
               "kernels": "tracescreen launch: k_order + k_trace + k_finish (uninstrumented)",
               "rule": "2*FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section; calibrated, "
                       "profiles/r02/hbm_counter_calibration.txt)"}
    json.dump(tj, open(sys.argv[3], "w"), indent=1)
    print("merged", key, "into", sys.argv[3])
