"""CPU tests of the oracle (oracle/rt_oracle.c): pinned against the reference's
own Noise.cpp output, the MSVC-rand golden values, analytic known answers, and
regression fixtures.  No GPU needed."""
import os

import numpy as np
import pytest

import oracle_lib as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fnv1a32(b):
    h = 0x811C9DC5
    for x in bytes(b):
        h = ((h ^ x) * 0x01000193) & 0xFFFFFFFF
    return h


def tables(nz):
    return (np.frombuffer(bytes(nz.perm2d), np.uint8).copy(), np.frombuffer(bytes(nz.grad), np.float32).copy())


# --- tables: Graphics/Noise.cpp:39-94 -------------------------------------------------
def test_noise_tables_match_reference_build():
    """glibc rand: bit-identical to the reference's own Noise.cpp compiled and run here
    (tests/golden/noise_reference_glibc_seed300.npz, made by oracle/_ref/ref_noise_dump)."""
    ref = np.load(os.path.join(GOLDEN, "noise_reference_glibc_seed300.npz"))
    p2, g = tables(O.noise_tables(300, O.RAND_GLIBC))
    assert np.array_equal(p2, ref["perm2d"])
    assert np.array_equal(g, ref["grad"])


def test_noise_tables_match_reference_build_msvc():
    """MSVC CRT rand (the reference's platform): bit-identical to the reference's own Noise.cpp
    built here with the MSVC rand/srand interposed (oracle/msvc_rand.cpp;
    tests/golden/noise_reference_msvc_seed300.npz, made by oracle/_ref/ref_noise_dump_msvc)."""
    ref = np.load(os.path.join(GOLDEN, "noise_reference_msvc_seed300.npz"))
    p2, g = tables(O.noise_tables(300, O.RAND_MSVC))
    assert np.array_equal(p2, ref["perm2d"])
    assert np.array_equal(g, ref["grad"])


@pytest.mark.parametrize("exe,kind", [("ref_noise_dump", O.RAND_GLIBC), ("ref_noise_dump_msvc", O.RAND_MSVC)])
def test_noise_tables_reference_binary_if_present(exe, kind):
    exe = os.path.join(O.ORACLE_DIR, "_ref", exe)
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    import subprocess
    raw = subprocess.run([exe], capture_output=True, check=True).stdout
    p2, g = tables(O.noise_tables(300, kind))
    assert raw[:65536] == p2.tobytes() and raw[65536:] == g.tobytes()


def test_noise_tables_msvc_golden():
    """MSVC CRT rand: SURVEY.md §8c measured values."""
    p2, g = tables(O.noise_tables(300, O.RAND_MSVC))
    assert list(p2[:8]) == [25, 53, 121, 90, 121, 90, 7, 19]
    assert fnv1a32(p2) == 0x6067CD85
    g = g.reshape(128, 4)
    assert g[:4, :3].tolist() == [[-1, 1, 0], [-1, 1, 0], [-1, -1, 0], [1, 1, 0]]
    assert np.all(g[:, 3] == 0)


@pytest.mark.parametrize("kind", [O.RAND_MSVC, O.RAND_GLIBC])
def test_noise_tables_structure(kind):
    nz = O.noise_tables(12345, kind)
    perm = np.array(nz.perm)
    assert sorted(perm.tolist()) == list(range(128))
    p2 = np.frombuffer(bytes(nz.perm2d), np.uint8).reshape(128, 128, 4)  # [y][x][c]
    P = lambda i: perm[i % 128]
    for x, y in ((0, 0), (5, 77), (127, 127), (64, 3)):
        a, b = P(x) + y, P(x + 1) + y
        assert p2[y, x].tolist() == [P(a), P(a + 1), P(b), P(b + 1)]


# --- numeric primitives ---------------------------------------
def ulp_err(y, ref):
    ref32 = ref.astype(np.float32)
    sp = np.spacing(np.abs(ref32)).astype(np.float64)
    return np.abs(y.astype(np.float64) - ref) / sp


def test_exp2_log2_accuracy():
    rng = np.random.default_rng(1)
    x = rng.uniform(-60, 60, 200000).astype(np.float32)
    assert ulp_err(O.unary(0, x), np.exp2(x.astype(np.float64))).max() <= 2.0
    x = np.exp(rng.uniform(-80, 80, 200000)).astype(np.float32)
    x = x[(x > 0) & np.isfinite(x)]
    y = O.unary(1, x)
    ref = np.log2(x.astype(np.float64))
    # absolute error near log2(x) = 0, relative elsewhere
    err = np.abs(y - ref) / np.maximum(np.spacing(np.abs(ref.astype(np.float32))), 2 ** -24)
    assert err.max() <= 3.0


def test_sin_cos_accuracy():
    rng = np.random.default_rng(2)
    x = rng.uniform(-600, 600, 200000).astype(np.float32)
    for op, fn in ((3, np.sin), (4, np.cos)):
        y = O.unary(op, x)
        assert np.abs(y - fn(x.astype(np.float64))).max() < 2e-7


def test_exact_special_values():
    k = np.arange(-100, 100, dtype=np.float32)
    assert np.array_equal(O.unary(0, k), np.ldexp(np.float32(1), k.astype(int)).astype(np.float32))
    assert np.array_equal(O.unary(1, np.ldexp(np.float32(1), k.astype(int)).astype(np.float32)), k)
    n = np.arange(1, 30, dtype=np.float32)
    assert np.array_equal(O.binary(0, np.full_like(n, 2.0), n), 2.0 ** n)  # pow(2, N) exact (greenrocks FBM)
    assert O.unary(0, np.array([-np.inf], np.float32))[0] == 0.0
    assert O.binary(0, np.array([0.0], np.float32), np.array([0.35], np.float32))[0] == 0.0  # pow(0, y>0)
    assert np.isnan(O.unary(1, np.array([-1.0], np.float32))[0])


def test_max_min_semantics():
    a = np.array([-0.0, 0.0, np.nan, 1.0, np.nan], np.float32)
    b = np.array([0.0, -0.0, 2.0, np.nan, np.nan], np.float32)
    mx, mn = O.binary(1, a, b), O.binary(2, a, b)
    assert [np.signbit(v) for v in mx[:2]] == [False, False]
    assert [np.signbit(v) for v in mn[:2]] == [True, True]
    assert mx[2] == 2.0 and mx[3] == 1.0 and np.isnan(mx[4])


# --- noise3d: Media/common/shaders/noise.hlsl:153-179 -----------------------------------
def test_noise3d_zero_on_lattice():
    nz = O.noise_tables()
    rng = np.random.default_rng(3)
    p = rng.integers(-1000, 1000, (5000, 3)).astype(np.float32)
    assert np.all(O.noise3d(nz, p) == 0.0)


def test_noise3d_range_continuity_periodicity():
    nz = O.noise_tables()
    rng = np.random.default_rng(4)
    p = rng.uniform(-300, 300, (20000, 3)).astype(np.float32)
    n = O.noise3d(nz, p)
    assert np.abs(n).max() < 1.2 and np.abs(n).mean() > 0.05
    # C2-continuous across cell faces
    face = np.floor(p).astype(np.float32)
    face[:, 1:] = p[:, 1:]
    eps = np.float32(1e-4)
    a = O.noise3d(nz, face - np.array([eps, 0, 0], np.float32))
    b = O.noise3d(nz, face + np.array([eps, 0, 0], np.float32))
    assert np.abs(a - b).max() < 1e-2
    # 128-periodic lattice (perm tables are 128-entry)
    q = rng.integers(-200, 200, (2000, 3)).astype(np.float32) + np.float32(0.25)
    assert np.array_equal(O.noise3d(nz, q), O.noise3d(nz, q + np.float32(128)))


# --- setTargetDepths: Graphics/Terrain.cpp:356-439 -------------------------------------
def set_target_depths_numpy(cr):
    """Independent float32 restatement (Terrain.cpp:356-439) for the oracle check."""
    d = cr.reshape(32, 32, 4)[:, :, 3]  # [y][x]
    f = np.float32

    def gd(x, y):
        return d[min(max(y, 0), 31), min(max(x, 0), 31)]

    def gi(x, y):
        if x < 0:
            m = gd(x + 1, y); return f(m - f(gd(x + 2, y) - m))
        if x >= 32:
            m = gd(x - 1, y); return f(m - f(gd(x - 2, y) - m))
        if y < 0:
            m = gd(x, y + 1); return f(m - f(gd(x, y + 2) - m))
        if y >= 32:
            m = gd(x, y - 1); return f(m - f(gd(x, y - 2) - m))
        return gd(x, y)

    out = np.zeros((1024, 2), np.float32)
    for i in range(1024):
        x, y = i % 32, i // 32
        lo = hi = gi(x, y)
        for xp in range(-2, 3):
            for yp in range(-2, 3):
                v = gi(x + xp, y + yp)
                lo = lo if lo < v else v
                hi = hi if v < hi else v
        lo = f(f(lo * f(0.96)) - f(0.01))
        hi = f(f(hi * f(1.22)) + f(0.4))
        out[i] = (lo if f(0.01) < lo else f(0.01), hi if hi < f(5000) else f(5000))
    return out


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_set_target_depths(seed):
    rng = np.random.default_rng(seed)
    cr = rng.uniform(0, 6000, (1024, 4)).astype(np.float32)
    cr[rng.random(1024) < 0.3, 3] = 5000.0  # sky cells
    cd = np.zeros(2048, np.float32)
    O.lib().ro_set_target_depths(O._fp(cr), O._fp(cd))
    assert np.array_equal(cd.reshape(1024, 2), set_target_depths_numpy(cr))


# --- analytic known answers: Media/testing (d = -y + 10 sin(.1x) cos(.1z)) ---------------
def test_testing_landscape_prepass_hits_surface():
    import scene
    c = scene.frame_constants(64, 48, euler=scene.LOOKDOWN_EULER)
    fr = O.make_frame(c, landscape=O.TESTING)
    nz = O.noise_tables()
    cr = np.zeros(4096, np.float32)
    st = O.Stats()
    import ctypes as C
    O.lib().ro_camerarays(C.byref(nz), C.byref(fr), O._fp(cr), C.byref(st))
    cr = cr.reshape(1024, 4)
    hit = cr[:, 3] < 5000.0
    assert hit.sum() > 100
    x, y, z = cr[hit, 0].astype(np.float64), cr[hit, 1], cr[hit, 2]
    surf = 10 * np.sin(0.1 * x) * np.cos(0.1 * z)
    # skiprefine march: first sample inside (d > 0) -> below the surface by at most one step
    assert np.all(surf - y > 0)
    assert np.median(surf - y) < 2.0


# --- regression fixtures (self-generated, tests/golden/make_golden.py) ------------------
@pytest.mark.parametrize("spec", __import__("golden_index").FRAMES)
def test_oracle_frames_regression(spec):
    import golden_index as GI
    gold = GI.load()
    land, pose, w, h, aa, ms, ao = GI.unpack(spec)
    key = GI.frame_key(*spec)
    fr = O.make_frame(GI.consts(w, h, pose), landscape=O.LANDSCAPES[land], aa=aa, max_steps=ms, ao=ao)
    r = O.render(O.noise_tables(), fr)
    assert np.array_equal(r["rgba32f"].view(np.uint32), gold[key + "_rgba32f"].view(np.uint32))
    assert np.array_equal(r["rgba8"], gold[key + "_rgba8"])
    assert np.array_equal(r["cell_distance"], gold[key + "_cell_distance"])
