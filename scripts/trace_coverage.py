"""Batch-boundary view of a rocprofv3 --kernel-trace of a long bench run:
per-kernel spans, how much of the run k_trace covers (the union of its launches' intervals), and
the gaps between consecutive k_trace launches.  The spans of the short kernels include the time
they wait for CUs that the other batch's persistent k_trace holds.

  python3 scripts/trace_coverage.py <kernel_trace.csv> <out.md> [title]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


def main(path, out, title="kernel trace"):
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in csv.DictReader(open(path)))
    per = defaultdict(list)
    for s, e, n in ev:
        per[n].append((e - s) / 1e6)
    tr = [(s, e) for s, e, n in ev if n.startswith("k_trace") and not re.match(r"k_trace<\d+, true", n)]
    # the throughput loop: the longest stretch of k_trace launches separated by less than 2 ms
    # (the bench's warm-up, roofline and stats passes are separated by host work)
    runs, run = [], [tr[0]]
    for prev, x in zip(tr, tr[1:]):
        if x[0] - max(e for _, e in run) < 2_000_000:
            run.append(x)
        else:
            runs.append(run)
            run = [x]
    runs.append(run)
    tr = max(runs, key=len)
    t0, t1 = tr[0][0], max(e for _, e in tr)
    cover, cur_s, cur_e, gaps = 0, tr[0][0], tr[0][1], []
    for s, e in tr[1:]:
        if s > cur_e:
            cover += cur_e - cur_s
            gaps.append((s - cur_e) / 1e6)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    cover += cur_e - cur_s
    with open(out, "w") as f:
        f.write(f"# {title}\n\n| kernel | calls | mean span ms | max span ms | total ms |\n|---|---:|---:|---:|---:|\n")
        for n in sorted(per, key=lambda n: -sum(per[n])):
            v = per[n]
            f.write(f"| {n} | {len(v)} | {sum(v) / len(v):.4f} | {max(v):.4f} | {sum(v):.3f} |\n")
        span = (t1 - t0) / 1e6
        f.write(f"\nsteady-state stretch (k_trace launches less than 2 ms apart): {len(tr)} launches; first start to last end {span:.3f} ms; "
                f"covered by some k_trace {cover / 1e6:.3f} ms = {100.0 * cover / (t1 - t0):.2f}%\n")
        if gaps:
            gaps.sort()
            f.write(f"gaps between k_trace launches: {len(gaps)}, total {sum(gaps):.3f} ms, "
                    f"median {gaps[len(gaps) // 2]:.3f} ms, max {gaps[-1]:.3f} ms\n")
        f.write("\nShort kernels' spans include their wait for CUs: the other batch's persistent k_trace holds "
                "every CU until its blocks retire.\n")
    print(open(out).read())


if __name__ == "__main__":
    main(*sys.argv[1:])
