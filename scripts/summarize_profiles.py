"""Summarise a scripts/profile_round.sh run into profiles/<round>/:
kernel_stats.csv (rocprofv3 --stats, verbatim), kernels.md (per-kernel table),
pmc.md (per-kernel counter means over the non-instrumented dispatches) and
traffic.json (HBM bytes per tracescreen launch for bench.py's roofline.traffic).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) doubled for gfx950's
half-counted wide streaming reads, WRITE_SIZE (KiB) as reported; TCC_EA0_* request
counts are kept alongside as the raw cross-check."""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

TRACESCREEN = ("k_order", "k_trace", "k_finish")


def instrumented(name):
    """STATS instantiations (the untimed counting frame): k_x<L, true, ..> / k_x<true>."""
    return re.search(r"<(\d+, )?true", name) is not None


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


def pmc_means(d):
    per = defaultdict(lambda: defaultdict(float))
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            per[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            agg[short(k)][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    ks = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)
    rows = list(csv.DictReader(open(ks[0])))
    shutil.copy(ks[0], os.path.join(dst, "kernel_stats.csv"))
    bench = open(os.path.join(src, "kt_bench.json")).read().strip().splitlines()[-1]
    with open(os.path.join(dst, "kernels.md"), "w") as f:
        bj = json.loads(bench)
        f.write(f"# rocprofv3 --kernel-trace --stats: `python3 bench.py --steps {bj['steps']} --warmup {bj['warmup']} "
                "--no-cpu-baseline --traffic off --no-companions`\n\n"
                "All launches of the run.  The timed loop keeps several batches of frames in flight, so those\n"
                "launches share the GPU and each one spans longer than it would alone; the per-launch cost the\n"
                "roofline uses is the bench's one-batch-in-flight pass, tabulated at the end from the same trace.\n"
                "One tracescreen launch traces a whole batch (config.batch frames).\n\n")
        f.write("| kernel | calls | avg ms | total ms |\n|---|---:|---:|---:|\n")
        for r in rows:
            f.write(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e6:.4f} | "
                    f"{float(r['TotalDurationNs']) / 1e6:.3f} |\n")
        plain = {short(r["Name"]): float(r["AverageNs"]) / 1e6 for r in rows}
        ts = sum(v for k, v in plain.items() if any(k.startswith(t) for t in TRACESCREEN) and not instrumented(k))
        f.write(f"\ntracescreen (uninstrumented k_order + k_trace + k_finish) avg sum: {ts:.4f} ms\n")
        f.write(f"\nbench line of the same run:\n\n```\n{bench}\n```\n")
    # the bench's roofline pass = its last K tracescreen launches (one frame in flight): per-kernel
    # means and the launch span (k_order start -> k_finish end) over exactly those dispatches
    kt = glob.glob(os.path.join(src, "kt", "**", "*kernel_trace.csv"), recursive=True)
    b0 = json.loads(bench)
    K = int(b0["roofline"].get("kernel_launches", 0))
    if kt and K:
        disp = sorted(((short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                       for r in csv.DictReader(open(kt[0]))), key=lambda x: x[1])
        ts_disp = [d for d in disp if any(d[0].startswith(t) for t in TRACESCREEN) and not instrumented(d[0])]
        starts = [i for i, d in enumerate(ts_disp) if d[0].startswith(("k_order", "k_tracescreen", "k_march"))]
        last = ts_disp[starts[-K]:] if len(starts) >= K else []
        per = defaultdict(list)
        for n, t0, t1 in last:
            per[n].append((t1 - t0) / 1e6)
        spans, cur = [], None
        for n, t0, t1 in last:
            if n.startswith(("k_order", "k_tracescreen", "k_march")):
                cur = t0
            if n.startswith(("k_finish", "k_tracescreen")) and cur is not None:
                spans.append((t1 - cur) / 1e6)
        with open(os.path.join(dst, "kernels.md"), "a") as f:
            f.write(f"\n## Roofline pass: the last {K} tracescreen launches (one batch in flight)\n\n")
            f.write("| kernel | calls | avg ms |\n|---|---:|---:|\n")
            for n in sorted(per, key=lambda n: -sum(per[n])):
                f.write(f"| {n} | {len(per[n])} | {sum(per[n]) / len(per[n]):.4f} |\n")
            if spans:
                f.write(f"\ntracescreen launch span (k_order start -> k_finish end), mean of {len(spans)}: "
                        f"{sum(spans) / len(spans):.4f} ms; bench.py HIP-event kernel_avg_ms: "
                        f"{b0['roofline']['kernel_avg_ms']} ms\n")
    m = pmc_means(src)
    with open(os.path.join(dst, "pmc.md"), "w") as f:
        f.write("# rocprofv3 --pmc per-kernel means (one pass per counter group, "
                "`bench.py --steps 10 --warmup 10 --batch 10 --frames-in-flight 1`: the counters are chip-wide, so no "
                "batch may overlap; every tracescreen launch is one 10-frame batch)\n\n")
        for k in sorted(m):
            f.write(f"## {k}\n\n")
            for c in sorted(m[k]):
                f.write(f"- {c}: {m[k][c]:.6g}\n")
            f.write("\n")
    tr = {}
    fetch = write = rd = wr = 0.0
    for k, cs in m.items():
        if any(k.startswith(t) for t in TRACESCREEN) and not instrumented(k):
            fetch += cs.get("FETCH_SIZE", 0.0)
            write += cs.get("WRITE_SIZE", 0.0)
            rd += cs.get("TCC_EA0_RDREQ_sum", 0.0)
            wr += cs.get("TCC_EA0_WRREQ_sum", 0.0)
    b = json.loads(bench)
    cf = b["config"]
    key = (f"{cf['width']}x{cf['height']}_{cf['landscape']}_{cf['pose']}_ms{cf['max_steps']}_ao{cf.get('ao_samples', 0)}"
           f"_b{cf.get('batch', 1)}")
    tr[key] = {"hbm_bytes_per_launch": int(2 * fetch * 1024 + write * 1024),
               "fetch_size_kib": fetch, "write_size_kib": write,
               "tcc_ea0_rdreq": rd, "tcc_ea0_wrreq": wr,
               "kernels": "tracescreen launch: k_order + k_trace + k_finish (uninstrumented)",
               "rule": "2*FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section)"}
    if fetch == 0.0 and write == 0.0:  # a kernel-trace-only profile (PMC=0): no traffic to record
        print(open(os.path.join(dst, "kernels.md")).read())
        return
    tpath = os.path.join(dst, "traffic.json")
    old = json.load(open(tpath)) if os.path.exists(tpath) else {}
    old.update(tr)  # other configs' launches (traffic_summary.py merges) stay
    json.dump(old, open(tpath, "w"), indent=1)
    print(open(os.path.join(dst, "kernels.md")).read())
    print(json.dumps(tr, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
