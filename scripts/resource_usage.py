"""Per-kernel VGPR / scratch / occupancy / LDS of the HIP kernels (compile-time report).
usage: python3 scripts/resource_usage.py [-DKNOB=value ...]  (an A/B build's rt_variants.h overrides)"""
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpgpuraytrace_amd", "csrc")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
       "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-fast-math", "--cuda-device-only", "-c", "rt_kernels.hip",
       "-o", "/tmp/rt_kernels_dev.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
out = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = {"name": re.sub(r"\(anonymous namespace\)::", "", name).split("(")[0]}
        rows.append(cur)
        continue
    for key, tag in (("VGPRs", "vgpr"), (r"ScratchSize \[bytes/lane\]", "scratch"),
                     (r"Occupancy \[waves/SIMD\]", "occ"), (r"LDS Size \[bytes/block\]", "lds")):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[tag] = m.group(1)
for r in rows:
    print("%-44s vgpr=%-4s scratch=%-4s occ=%-2s lds=%s" % (r["name"], r.get("vgpr"), r.get("scratch"), r.get("occ"),
                                                           r.get("lds")))
