"""FETCH_SIZE / WRITE_SIZE against known byte counts (scripts/ubench_hbm.hip).
GPU box: O=gpurun_out/hbmcal; scripts/_build/ubench_hbm > $O/expected.txt;
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- scripts/_build/ubench_hbm
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- scripts/_build/ubench_hbm
then: python3 scripts/hbm_calibration.py [gpurun_out/hbmcal]"""
import collections
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/hbmcal"
exp = [line.split() for line in open(d + "/expected.txt")]
names, mib = [e[2] for e in exp], [float(e[4]) for e in exp]
for tag, cn in (("f", "FETCH_SIZE"), ("w", "WRITE_SIZE")):
    per = collections.OrderedDict()
    for r in csv.DictReader(open(f"{d}/{tag}/run_counter_collection.csv")):
        if "k_read" in r["Kernel_Name"] or "k_write" in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])] = per.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    vals = [per[k] for k in sorted(per)]
    print(cn)
    for n, m, v in zip(names, mib, vals):
        print("  %-14s expected %7.1f MiB  counter %7.1f MiB  ratio %.3f" % (n, m, v / 1024, v / 1024 / m))
