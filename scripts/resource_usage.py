"""Per-kernel VGPR / SGPR (+ SGPR spills to VGPR lanes) / scratch / occupancy / LDS / code size of the HIP
kernels (compile-time report; the code size is the kernel symbol's size in the gfx950 code object).
usage: python3 scripts/resource_usage.py [-DKNOB=value ...]  (an A/B build's rt_variants.h overrides)"""
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpgpuraytrace_amd", "csrc")
CO = "/tmp/rt_kernels_dev.hsaco"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
       "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-fast-math", "--cuda-device-only", "--no-gpu-bundle-output",
       "-c", "rt_kernels.hip", "-o", CO, "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
out = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True).stderr


def demangle(sym):
    name = subprocess.run(["c++filt", sym], capture_output=True, text=True).stdout.strip()
    return re.sub(r"\(anonymous namespace\)::", "", name).split("(")[0]


sizes = {}
syms = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-s", "--wide", CO], capture_output=True, text=True).stdout
for line in syms.splitlines():
    f = line.split()
    if len(f) >= 8 and f[3] == "FUNC":
        sizes[f[7]] = int(f[2])
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": demangle(m.group(1)), "code": sizes.get(m.group(1))}
        rows.append(cur)
        continue
    for key, tag in (("VGPRs", "vgpr"), ("TotalSGPRs", "sgpr"), ("SGPRs Spill", "sspill"),
                     (r"ScratchSize \[bytes/lane\]", "scratch"), (r"Occupancy \[waves/SIMD\]", "occ"),
                     (r"LDS Size \[bytes/block\]", "lds")):
        m = re.search("remark:\\s+" + key + r": (\d+)", line)
        if m and cur is not None:
            cur[tag] = m.group(1)
for r in rows:
    print("%-48s vgpr=%-4s sgpr=%-4s sgpr_spill=%-4s scratch=%-4s occ=%-2s lds=%-7s code=%s" % (
        r["name"], r.get("vgpr"), r.get("sgpr"), r.get("sspill"), r.get("scratch"), r.get("occ"), r.get("lds"),
        r.get("code")))
