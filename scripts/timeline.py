"""Kernel timeline of the last stretch of a rocprofv3 --kernel-trace (kernel_trace.csv): every dispatch
of the last `n` k_trace launches' neighbourhood with start / end relative to the first shown, in ms,
and its queue, so batch boundaries (prepass, k_order waits, blits) can be read off.
  python3 scripts/timeline.py <kernel_trace.csv> [n_traces]"""
import csv
import sys


def short(name):
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]


rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Queue_Id", "?"))
              for r in csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
tr = [i for i, r in enumerate(rows) if r[2].startswith("k_trace")]
first = tr[-n] if len(tr) >= n else 0
t0 = rows[first][0]
for s, e, name, q in rows[max(0, first - 4):]:
    print(f"{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f}  q{q:>3}  {name}")
