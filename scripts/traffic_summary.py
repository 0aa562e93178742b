"""HBM bytes per tracescreen launch from scripts/traffic_pass.sh (2*FETCH_SIZE + WRITE_SIZE, KiB
counters, MI355X_MICROARCH.md HBM rule), per kernel and per frame against the 8.3 MB RGBA8 frame.
usage: traffic_summary.py [dir] [frames per launch]"""
import collections
import csv
import glob
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
    if any(k.startswith(x) for x in ("k_trace", "k_finish", "k_shade", "k_shadow", "k_order")):
        d = {c: sum(v) / len(v) for c, v in tot[k].items()}
        b = (2 * d.get("FETCH_SIZE", 0) + d.get("WRITE_SIZE", 0)) * 1024
        s += b
        print("%-28s FETCH %8.1f MiB  WRITE %8.1f MiB  -> %7.1f MB" % (k, d.get("FETCH_SIZE", 0) / 1024,
                                                                     d.get("WRITE_SIZE", 0) / 1024, b / 1e6))
print("tracescreen launch %.1f MB = %.1f MB per frame = %.1fx the 8.3 MB RGBA8 frame" % (s / 1e6, s / frames / 1e6,
                                                                                         s / frames / 8.2944e6))
