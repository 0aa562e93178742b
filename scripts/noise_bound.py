#!/usr/bin/env python3
"""The amplitude bound behind the RT_FBM_EXIT A/B build (rt_shader.h kNoiseBound).

noise3d (noise.hlsl:153-179, oracle/rt_oracle.c noise3d) blends the eight corner terms
g_c . (f - c) with the quintic fade weights w_c(f) (non-negative, summing to 1).  The gradient
table holds the {-1, 0, 1} edge vectors (two +-1 components and one 0, Graphics/Noise.cpp:6-24), so
|g_c . (f - c)| <= the sum of the two largest |f_a - c_a|, and

    |noise3d(p)| <= max over f in [0,1]^3 of  sum_c w_c(f) * (two largest |f_a - c_a|).

The bound is symmetric under f_a -> 1 - f_a, so [0, 0.5]^3 covers the cube.  This evaluates it on
a 257^3 grid of that octant: 1.0364 (at f ~ (0.355, 0.482, 0.5)).  The kernel uses 1.05: the
grid maximum plus slack for the function's variation between grid points (its gradient is
a few units at most; half a grid diagonal is 0.0017).

    python3 scripts/noise_bound.py
"""
import numpy as np


def fade(t):
    return t * t * t * (t * (t * 6 - 15) + 10)


def main(n=257):
    t = np.linspace(0.0, 0.5, n)
    best, arg = 0.0, None
    fy, fz = np.meshgrid(t, t, indexing="ij")
    for fx in t:
        f = [np.full_like(fy, fx), fy, fz]
        u = [fade(a) for a in f]
        tot = np.zeros_like(fy)
        for c in range(8):
            cs = [(c >> k) & 1 for k in range(3)]
            w = np.ones_like(fy)
            d = []
            for a in range(3):
                w = w * (u[a] if cs[a] else 1 - u[a])
                d.append(np.abs(f[a] - cs[a]))
            d = np.sort(np.stack(d), axis=0)
            tot += w * (d[1] + d[2])
        m = float(tot.max())
        if m > best:
            k = np.unravel_index(tot.argmax(), tot.shape)
            best, arg = m, (float(fx), float(t[k[0]]), float(t[k[1]]))
    print(f"max sum_c w_c * (two largest |f - c|) = {best:.6f} at f = {arg}")


if __name__ == "__main__":
    main()
