#!/usr/bin/env python3
"""How far the reference's unknowable arithmetic conventions can move a frame: the error bar on
"parity unpinned" (BASELINE.md:32-35).

The GPU path is bit-identical to oracle/rt_oracle.c, which fixes ONE reading of the HLSL (R2 mad
fusion, R3 div = a * rcp(b), R5 polynomial transcendentals).  fxc + a D3D driver may read it
another way.  This renders the same frames with convention variants of the oracle
(rt_oracle.c RO_CONV_*: unfused mads, IEEE division, libm transcendentals, all three) and reports,
against the default oracle (= the GPU):

  * the fraction of pixels whose primary march took a different number of steps, and the fraction
    where any of the pixel's rays (primary, shadow, AO) did (divergent),
  * max |delta| of the float32 colour over the step-agreeing pixels (all rays agree; BASELINE.md's
    parity bound is 1e-4 there) and the fraction of step-agreeing pixels above 1e-4,
  * the UNORM8 histogram of the largest channel difference over all pixels.

Cases: every committed golden frame (tests/golden, small) and row samples of BASELINE C2 and C3.
Writes profiles/r03/parity_sensitivity.{json,md}.
  python tests/tools/parity_sensitivity.py [--row-step 8] [--threads 0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden_index as GI  # noqa: E402
import oracle_lib as O  # noqa: E402

VARIANTS = ["unfused", "ieeediv", "libm", "all"]
TOL = 1e-4
BINS = [(0, 0), (1, 1), (2, 3), (4, 15), (16, 255)]


def compare(ref, ref8, ref_steps, var, var8, var_steps, rows=slice(None)):
    """*_steps: (primary, secondary) per-pixel march iterations.  A pixel AGREES when all its rays
    (primary, shadow, AO) took the same number of steps under both conventions."""
    a, b = ref[rows][..., :3].astype(np.float64), var[rows][..., :3].astype(np.float64)
    prim = ref_steps[0][rows] == var_steps[0][rows]
    agree = prim & (ref_steps[1][rows] == var_steps[1][rows])
    d = np.abs(a - b).max(axis=-1)
    d8 = np.abs(ref8[rows][..., :3].astype(np.int32) - var8[rows][..., :3].astype(np.int32)).max(axis=-1)
    n = d.size
    out = {
        "pixels": int(n),
        "divergent_primary_fraction": float(1.0 - prim.mean()),
        "divergent_fraction": float(1.0 - agree.mean()),
        "max_abs_delta_agreeing": float(d[agree].max()) if agree.any() else 0.0,
        "agreeing_above_tol_fraction": float((d[agree] > TOL).mean()) if agree.any() else 0.0,
        "max_abs_delta_all": float(d.max()),
        "bitexact_fraction": float((d == 0).mean()),
        "unorm8_hist": {f"{lo}-{hi}" if lo != hi else f"{lo}": int(((d8 >= lo) & (d8 <= hi)).sum()) for lo, hi in BINS},
    }
    return out


def render(L, consts, land, aa, ms, ao, rows, threads):
    h, w = consts["height"], consts["width"]
    fr = O.make_frame(consts, landscape=O.LANDSCAPES[land], aa=aa, max_steps=ms, ao=ao, rows=rows, threads=threads)
    steps, sec = np.zeros((h, w), np.float32), np.zeros((h, w), np.float32)
    rgba, rgba8, _, _, _ = O.render_rows(O.noise_tables(), fr, L=L, steps=steps, secondary_steps=sec)
    return rgba, rgba8, (steps, sec)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--row-step", type=int, default=8)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03", "parity_sensitivity"))
    a = ap.parse_args()
    import gpgpuraytrace_amd.camera as cam
    cases = []
    for spec in GI.FRAMES:
        land, pose, w, h, aa, ms, ao = GI.unpack(spec)
        cases.append((GI.frame_key(*spec), GI.consts(w, h, pose), land, aa, ms, ao, (0, h, 1)))
    for name, (w, h, ms, ao) in {"C2_1280x720_ms256": (1280, 720, 256, 0),
                                 "C3_1920x1080_ms512_ao1": (1920, 1080, 512, 1)}.items():
        for pose, eul in (("reset", cam.INITIAL_ROTATION_EULER), ("lookdown", cam.LOOKDOWN_ROTATION_EULER)):
            cases.append((f"{name}_{pose}_rows0::{a.row_step}", cam.frame_constants(w, h, euler=eul), "nomadplains", 1,
                          ms, ao, (0, h, a.row_step)))
    result = {"tolerance": TOL, "variants": {}, "cases": [c[0] for c in cases]}
    base = {}
    t0 = time.time()
    for key, consts, land, aa, ms, ao, rows in cases:
        base[key] = render(O.lib(), consts, land, aa, ms, ao, rows, a.threads)
    print(f"default oracle: {len(cases)} cases in {time.time() - t0:.1f} s", flush=True)
    for v in VARIANTS:
        L = O.variant(v)
        per = {}
        for key, consts, land, aa, ms, ao, rows in cases:
            r = base[key]
            x = render(L, consts, land, aa, ms, ao, rows, a.threads)
            sl = slice(rows[0], rows[1], rows[2])
            per[key] = compare(r[0], r[1], r[2], x[0], x[1], x[2], rows=sl)
        result["variants"][v] = per
        worst = max(per.values(), key=lambda c: c["max_abs_delta_agreeing"])
        print(f"{v}: worst agreeing max|d| {worst['max_abs_delta_agreeing']:.3g}; divergent up to "
              f"{max(c['divergent_fraction'] for c in per.values()):.4f}", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out + ".json", "w") as f:
        json.dump(result, f, indent=1)
    with open(a.out + ".md", "w") as f:
        f.write(report(result))
    print("wrote", a.out + ".{json,md}")


def report(r):
    lines = ["# Parity sensitivity to the HLSL arithmetic conventions (generated by tests/tools/parity_sensitivity.py)",
             "",
             "Each variant re-renders the case with oracle/rt_oracle.c built under another equally valid reading",
             "of the HLSL (RO_CONV_UNFUSED: every mad / lerp / dot / mul unfused, tracing.hlsl:54 included;",
             "RO_CONV_IEEEDIV: IEEE division instead of a * rcp(b), normalize = v / length; RO_CONV_LIBM: glibc",
             "powf / expf / exp2f / log2f / sinf / cosf instead of the R5 polynomials; all: the three together),",
             "and compares it with the default oracle, which the GPU matches bit for bit.",
             "",
             "Columns: div. primary = pixels whose primary march took a different step count; divergent = pixels",
             "where any of their rays (primary, shadow, AO) did; agreeing max|d| = largest float32 channel",
             f"difference over the other (step-agreeing) pixels (BASELINE.md bound {r['tolerance']});",
             "> tol = fraction of step-agreeing pixels above the bound; UNORM8 = histogram of the largest",
             "channel difference of the RGBA8 output over all pixels (0 / 1 / 2-3 / 4-15 / 16+ LSB).", ""]
    for v, per in r["variants"].items():
        lines += [f"## {v}", "", "| case | pixels | div. primary | divergent | agreeing max\\|d\\| | > tol | all max\\|d\\| | UNORM8 0 / 1 / 2-3 / 4-15 / 16+ |",
                  "|---|---:|---:|---:|---:|---:|---:|---|"]
        for k, c in per.items():
            h = c["unorm8_hist"]
            lines.append(f"| {k} | {c['pixels']} | {c['divergent_primary_fraction']:.3%} | {c['divergent_fraction']:.3%} | "
                         f"{c['max_abs_delta_agreeing']:.3g} | "
                         f"{c['agreeing_above_tol_fraction']:.4%} | {c['max_abs_delta_all']:.3g} | "
                         f"{' / '.join(str(x) for x in h.values())} |")
        lines.append("")
    return "\n".join(lines) + "\n"


if __name__ == "__main__":
    main()
