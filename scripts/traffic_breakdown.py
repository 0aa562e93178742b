#!/usr/bin/env python3
"""Per-kernel L2 / fabric counters of ONE measured tracescreen launch (the launch bench.py's
roofline.traffic measures), one rocprofv3 --pmc pass per counter group over
`bench.py --traffic-child` child processes.  Used to attribute HBM bytes to k_trace's intermediates
(VERDICT r2 weak #6).

  python3 scripts/traffic_breakdown.py [--batch 10] [--out gpurun_out/traffic_breakdown.json] [bench args...]

Groups respect the per-pass limits (<= 4 TCC counters; FETCH_SIZE uses 3, WRITE_SIZE 2)."""
import argparse
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GROUPS = [
    ["FETCH_SIZE"],
    ["WRITE_SIZE"],
    ["TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"],
    ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum"],
    ["TCC_HIT_sum", "TCC_MISS_sum"],
    ["TCC_READ_sum", "TCC_WRITE_sum"],
    ["TCC_ATOMIC_sum", "TCC_WRITEBACK_sum"],
]
KERNELS = ("k_order", "k_trace", "k_finish", "k_camerarays")


def short(name):
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=10)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "traffic_breakdown.json"))
    ap.add_argument("--timeout", type=int, default=120)
    ap.add_argument("--variant", default="", help="experiment build librt_hip_<variant>.so (scripts/with_variant.py)")
    ap.add_argument("--groups", default="all", help="'all' or 'bytes' (FETCH_SIZE and WRITE_SIZE only)")
    a, rest = ap.parse_known_args()
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    child = [sys.executable, os.path.join(ROOT, "scripts", "with_variant.py"), os.path.join(ROOT, "bench.py"),
             "--traffic-child", "--batch", str(a.batch)] + rest
    env = dict(os.environ, TMPDIR="/tmp", RT_LIB_VARIANT=a.variant)
    groups = GROUPS if a.groups == "all" else GROUPS[:2]
    result = {"batch": a.batch, "variant": a.variant, "child": " ".join(child[1:]), "kernels": {}}
    for g in groups:
        work = tempfile.mkdtemp(prefix="tb_", dir="/tmp")
        cmd = ["timeout", "-s", "KILL", str(a.timeout), prof, "--pmc"] + g + ["--output-format", "csv", "-d", work,
                                                                               "-o", "run", "--"] + child
        r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        if r.returncode != 0:
            print(f"group {g}: rc={r.returncode} {r.stderr.decode(errors='replace')[-300:]}", flush=True)
            result.setdefault("failed", []).append(g)
            shutil.rmtree(work, ignore_errors=True)
            continue
        per = {}
        for f in glob.glob(work + "/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                key = (int(row["Dispatch_Id"]), short(row["Kernel_Name"]), row["Counter_Name"])
                per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        shutil.rmtree(work, ignore_errors=True)
        orders = sorted({d for d, n, _ in per if n.startswith("k_order")})
        if len(orders) < 2:
            print(f"group {g}: {len(orders)} launches", flush=True)
            continue
        last = orders[len(orders) // 2]
        # the measured launch: its prepass (the camerarays dispatch just before its k_order) and the
        # tracescreen kernels from its k_order on
        cam = max((d for d, n, _ in per if n.startswith("k_camerarays") and d < last), default=last)
        for (d, n, c), v in per.items():
            if re.match(r"k_trace<\d+, true|k_camerarays_group<true", n) or not n.startswith(KERNELS):  # STATS kernels
                continue
            if d >= last or d == cam:
                kk = n.split("<")[0]
                result["kernels"].setdefault(kk, {})
                result["kernels"][kk][c] = result["kernels"][kk].get(c, 0.0) + v
        print(f"group {g}: ok", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(result, open(a.out, "w"), indent=1)
    for k, cs in result["kernels"].items():
        print(k, {c: round(v) for c, v in sorted(cs.items())})
    tot = {c: sum(cs.get(c, 0.0) for cs in result["kernels"].values() if c in cs) for c in ("FETCH_SIZE", "WRITE_SIZE")}
    print(f"variant={a.variant or 'product'} total FETCH_SIZE {tot['FETCH_SIZE'] / 1024:.1f} MiB, WRITE_SIZE "
          f"{tot['WRITE_SIZE'] / 1024:.1f} MiB, 2F+W {(2 * tot['FETCH_SIZE'] + tot['WRITE_SIZE']) / 1024:.1f} MiB", flush=True)


if __name__ == "__main__":
    main()
