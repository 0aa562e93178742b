"""Kernel timeline of scripts/serial_loop.py under `rocprofv3 --kernel-trace --output-format csv`: per k_trace
launch its start, end and the gap to the previous launch's end (negative = the two frames' traces overlap).
Usage: python scripts/serial_timeline.py <kernel_trace.csv>"""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows),
                key=lambda x: x[0])
    tr = [k for k in ks if "k_trace" in k[2]]
    print(f"{len(tr)} k_trace launches")
    prev = None
    gaps, spans = [], []
    for s, e, n in tr:
        if prev is not None:
            gaps.append((s - prev[1]) / 1e3)
            spans.append((s - prev[0]) / 1e3)
        prev = (s, e)
    for i, (s, e, n) in enumerate(tr):
        g = f"{gaps[i - 1]:9.1f}" if i else "        -"
        p = f"{spans[i - 1]:9.1f}" if i else "        -"
        print(f"  {i:3d} dur {(e - s) / 1e3:9.1f} us  start-to-start {p} us  gap after previous end {g} us")
    if gaps:
        print(f"mean start-to-start {sum(spans) / len(spans):.1f} us, mean gap {sum(gaps) / len(gaps):.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
