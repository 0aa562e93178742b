"""Per-launch means of the product k_trace (k_trace<0, false, false>) over the --pmc passes of
scripts/pmc_ktrace.sh, and the ratios profiles/r04/pmc.md reported: cycles per VALU instruction per SIMD
(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs / SQ_INSTS_VALU), SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES and
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.  (A diagnostic for profiles/; not a test module.)"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    per = defaultdict(lambda: defaultdict(float))
    for p in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            k = r.get("Kernel_Name", "")
            if "k_trace<0, false, false>" not in k:
                continue
            per[(p, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    means = defaultdict(list)
    for cs in per.values():
        for c, v in cs.items():
            means[c].append(v)
    m = {c: sum(v) / len(v) for c, v in means.items()}
    print(f"k_trace<0, false, false>: {len(per)} dispatches over the passes (10-frame C3 batches)")
    for c in sorted(m):
        print(f"  {c:24s} {m[c]:.4g}")
    if "GRBM_GUI_ACTIVE" in m and "SQ_INSTS_VALU" in m:
        print(f"cycles per VALU instruction per SIMD: {m['GRBM_GUI_ACTIVE'] / 8 * 1024 / m['SQ_INSTS_VALU']:.3f}")
    if "SQ_WAIT_INST_ANY" in m:
        print(f"SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES: {m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
    if "SQ_LDS_BANK_CONFLICT" in m:
        print(f"SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE: {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.3f}")
        print(f"LDS-array busy per CU cycle: {m['SQ_LDS_IDX_ACTIVE'] / 256 / (m['GRBM_GUI_ACTIVE'] / 8):.3f}")
    if "SQ_ACTIVE_INST_VALU" in m:
        print(f"VALU lane utilisation (SQ_THREAD_CYCLES_VALU / 64 SQ_ACTIVE_INST_VALU): "
              f"{m['SQ_THREAD_CYCLES_VALU'] / 64 / m['SQ_ACTIVE_INST_VALU']:.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
