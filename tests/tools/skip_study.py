#!/usr/bin/env python3
"""Diagnostic: potential of an exact FBM early exit (tests/tools/skip_study.c) at a BASELINE config.

Renders bands of 8 rows with the oracle instrumented per march sample, then emulates the GPU's
wave64 lockstep: a primary unit (8x8 pixels) pays, per march iteration, the max over its live
lanes of the octaves evaluated; long rays (shadow / AO) refill lanes, so they are modelled as
random groups of 64 samples.  Prints octave-iteration totals now vs with the early exit.

  python tests/tools/skip_study.py [--config c3] [--nb 1.0] [--band-every 64]
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402

SO = os.path.join(ROOT, "tests", "tools", "_build", "libskip_study.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = os.path.join(ROOT, "tests", "tools", "skip_study.c")
    subprocess.run(["gcc", "-O2", "-std=c11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fopenmp",
                    "-shared", "-o", SO, src, "-lm"], check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--nb", type=float, default=1.0)
    ap.add_argument("--margin", type=float, default=0.02)
    ap.add_argument("--band-every", type=int, default=64)
    ap.add_argument("--pose", default="reset")
    a = ap.parse_args()
    import gpgpuraytrace_amd as G
    cfg = {"c2": (1280, 720, 256, 0), "c3": (1920, 1080, 512, 1), "c5": (3840, 2160, 1024, 4),
           "ref": (1920, 1080, 0, 0)}[a.config]
    W, H, ms, ao = cfg
    build()
    L = C.CDLL(SO)
    L.st_config.argtypes = [C.c_float, C.c_float, C.c_int64]
    for n in ("st_pixel_len",):
        getattr(L, n).argtypes = [C.c_int64]
        getattr(L, n).restype = C.c_int64
    L.st_pixel_data.argtypes = [C.c_int64]
    L.st_pixel_data.restype = C.c_void_p
    L.st_long_len.argtypes = [C.c_int, C.c_int]
    L.st_long_len.restype = C.c_int64
    L.st_long_data.argtypes = [C.c_int, C.c_int]
    L.st_long_data.restype = C.c_void_p
    L.st_check_err.restype = C.c_double
    fp = C.POINTER(C.c_float)
    L.ro_noise_generate.argtypes = [C.POINTER(O.Noise), C.c_uint32, C.c_int]
    L.ro_camerarays.argtypes = [C.POINTER(O.Noise), C.POINTER(O.Frame), fp, C.POINTER(O.Stats)]
    L.ro_set_target_depths.argtypes = [fp, fp]
    L.ro_tracescreen.argtypes = [C.POINTER(O.Noise), C.POINTER(O.Frame), fp, fp, C.POINTER(C.c_uint8), fp,
                                 C.POINTER(O.Stats)]
    nz = O.Noise()
    L.ro_noise_generate(C.byref(nz), 300, O.RAND_MSVC)
    euler = G.camera.INITIAL_ROTATION_EULER if a.pose == "reset" else G.camera.LOOKDOWN_ROTATION_EULER
    consts = G.frame_constants(W, H, euler=euler)
    L.st_config(a.nb, a.margin, W * H)
    cr = np.zeros(4096, np.float32)
    cd = np.zeros(2048, np.float32)
    fr = O.make_frame(consts, landscape=0, max_steps=ms, ao=ao, rows=(0, 0, 1))
    L.ro_camerarays(C.byref(nz), C.byref(fr), cr.ctypes.data_as(fp), None)
    L.ro_set_target_depths(cr.ctypes.data_as(fp), cd.ctypes.data_as(fp))
    bands = list(range(0, H - 7, a.band_every))
    rgba = np.zeros((H, W, 4), np.float32)
    for y0 in bands:
        fr = O.make_frame(consts, landscape=0, max_steps=ms, ao=ao, rows=(y0, y0 + 8, 1))
        L.ro_tracescreen(C.byref(nz), C.byref(fr), cd.ctypes.data_as(fp), rgba.ctypes.data_as(fp), None, None, None)
    print(f"sanity max |d recomputed - d| = {L.st_check_err():.3g}")

    def pix(i):
        n = L.st_pixel_len(i)
        if n == 0:
            return np.zeros((0, 2), np.uint8)
        return np.ctypeslib.as_array(C.cast(L.st_pixel_data(i), C.POINTER(C.c_uint8)), (n,)).reshape(-1, 2).copy()

    base_lane = skip_lane = base_wave = skip_wave = 0
    for y0 in bands:
        for x0 in range(0, W - 7, 8):
            seqs = [pix((y0 + j // 8) * W + x0 + j % 8) for j in range(64)]
            T = max(len(s) for s in seqs)
            nmat = np.zeros((64, T), np.int64)
            kmat = np.zeros((64, T), np.int64)
            for j, s in enumerate(seqs):
                nmat[j, :len(s)] = s[:, 0]
                kmat[j, :len(s)] = s[:, 1]
            base_lane += nmat.sum()
            skip_lane += kmat.sum()
            base_wave += nmat.max(axis=0).sum()
            skip_wave += kmat.max(axis=0).sum()
    print(f"primary ({len(bands)} bands of 8 rows): octave lane-evals {base_lane} -> {skip_lane} "
          f"({skip_lane / max(1, base_lane):.3f}); wave octave-iterations {base_wave} -> {skip_wave} "
          f"({skip_wave / max(1, base_wave):.3f})")
    rng = np.random.default_rng(1)
    for kind, name in ((0, "prepass"), (1, "shadow"), (2, "AO")):
        parts = []
        for t in range(256):
            n = L.st_long_len(kind, t)
            if n:
                parts.append(np.ctypeslib.as_array(C.cast(L.st_long_data(kind, t), C.POINTER(C.c_uint8)),
                                                   (n,)).reshape(-1, 2).copy())
        if not parts:
            continue
        s = np.concatenate(parts).astype(np.int64)
        if kind != 0:
            s = s[rng.permutation(len(s))]
        g = len(s) // 64 * 64
        bw = s[:g, 0].reshape(-1, 64).max(axis=1).sum()
        sw = s[:g, 1].reshape(-1, 64).max(axis=1).sum()
        print(f"{name}: samples {len(s)}, octave lane-evals {s[:, 0].sum()} -> {s[:, 1].sum()} "
              f"({s[:, 1].sum() / max(1, s[:, 0].sum()):.3f}); random-64 wave {bw} -> {sw} ({sw / max(1, bw):.3f})")


if __name__ == "__main__":
    main()
