#!/usr/bin/env python3
"""Diagnostic: would speculative multi-sample marching shorten the prepass?

A wave marching one prepass ray could evaluate W consecutive samples per pass (W x 18 octave values
over 64 lanes) if each next position were known in advance; it is only when the previous sample's
density lies in the unit-step band [-5, 0].  This runs the oracle's camerarays (single-threaded,
tests/tools/prepass_band_study.c) for the C3 frame's two poses and reports, for the longest ray (the
prepass's latency), the passes a W-wide speculation would need against its steps.

  python3 tests/tools/prepass_band_study.py
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402

SO = os.path.join(ROOT, "tests", "tools", "_build", "libprepass_band_study.so")


def main():
    import gpgpuraytrace_amd as G
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["gcc", "-O2", "-std=c11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-shared", "-o", SO,
                    os.path.join(ROOT, "tests", "tools", "prepass_band_study.c"), "-lm"], check=True)
    L = C.CDLL(SO)
    fp = C.POINTER(C.c_float)
    L.ro_noise_generate.argtypes = [C.POINTER(O.Noise), C.c_uint32, C.c_int]
    L.ro_camerarays.argtypes = [C.POINTER(O.Noise), C.POINTER(O.Frame), fp, C.POINTER(O.Stats)]
    L.pp_n.restype = C.c_int64
    L.pp_flags.restype = C.POINTER(C.c_uint8)
    L.pp_starts.restype = C.POINTER(C.c_int32)
    nz = O.Noise()
    L.ro_noise_generate(C.byref(nz), 300, O.RAND_MSVC)
    for pose, euler in (("reset", G.camera.INITIAL_ROTATION_EULER), ("lookdown", G.camera.LOOKDOWN_ROTATION_EULER)):
        fr = O.make_frame(G.frame_constants(1920, 1080, euler=euler), landscape=0, max_steps=512, ao=1, rows=(0, 0, 1))
        L.pp_reset()
        cr = np.zeros(4096, np.float32)
        L.ro_camerarays(C.byref(nz), C.byref(fr), cr.ctypes.data_as(fp), None)
        n, rays = L.pp_n(), L.pp_rays()
        fl = np.ctypeslib.as_array(L.pp_flags(), (n,)).copy()
        st = list(np.ctypeslib.as_array(L.pp_starts(), (rays,))) + [n]
        steps = np.diff(st)
        print(f"{pose}: {rays} rays, {n} samples, longest ray {steps.max()} steps (mean {steps.mean():.1f}), "
              f"samples in the unit-step band {(fl & 1).mean():.3f}")
        for w in (2, 3, 4, 8):
            passes = []
            for r in range(rays):
                f, i, p = fl[st[r]:st[r + 1]], 0, 0
                while i < len(f):
                    p, k = p + 1, 1
                    while k < w and i + k < len(f) and f[i + k - 1]:
                        k += 1
                    i += k
                passes.append(p)
            print(f"  W={w}: longest ray {max(passes)} passes (against {steps.max()} steps): "
                  f"{max(passes) / steps.max():.3f} of the prepass latency")


if __name__ == "__main__":
    main()
