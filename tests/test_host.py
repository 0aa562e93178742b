"""CPU tests of the product's host side: the C-ABI library loads and exports every
symbol include/frosttrace.h declares, and the host-side engine code (noise
tables, setTargetDepths, tile sizes, camera, shard mapping) agrees with the
oracle / reference formulas.  No GPU compute is issued."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import oracle_lib as O
import scene

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "frosttrace.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import _native
    L = G.lib()
    names = header_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # the ctypes binding covers the whole header
    assert set(names) <= set(_native.SIGNATURES), set(names) - set(_native.SIGNATURES)
    assert L.rt_abi_version() == _native.ABI_VERSION == 9


def test_product_reads_no_environment_and_has_no_experiment_switches():
    """The product's loader takes no environment variable (experiment builds are selected by
    scripts/with_variant.py) and the kernels carry no work-skipping experiment switch."""
    src = open(os.path.join(ROOT, "gpgpuraytrace_amd", "_native.py")).read()
    assert "os.environ" not in src
    kern = open(os.path.join(ROOT, "gpgpuraytrace_amd", "csrc", "rt_kernels.hip")).read()
    assert "SKIP_PREPASS" not in kern


def test_stats_sized_never_writes_past_a_short_struct():
    """rt_device_stats_sized (ABI 4) on a null device fails before touching the buffer; the ctypes
    binding refuses a library older than itself (ABI-1 callers and the 8-byte overrun)."""
    import ctypes as C
    import gpgpuraytrace_amd as G
    buf = (C.c_ubyte * 64)(*([0xAB] * 64))
    assert G.lib().rt_device_stats_sized(None, C.cast(buf, C.POINTER(G._native.RtStats)), 48, 0) != 0
    assert bytes(buf) == b"\xab" * 64


def test_product_loads_only_in_tree_library():
    import gpgpuraytrace_amd as G
    assert os.path.abspath(G.LIB_PATH).startswith(ROOT)
    assert os.path.exists(G.LIB_PATH)


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("seed", [300, 1, 123456789])
def test_product_noise_generator_matches_oracle(kind, seed):
    import gpgpuraytrace_amd as G
    n = G.Noise()
    n.generate(seed=seed, rand_kind=kind)
    o = O.noise_tables(seed, kind)
    assert np.array_equal(n.permutations2D, np.frombuffer(bytes(o.perm2d), np.uint8))
    assert np.array_equal(n.permutations1D, np.frombuffer(bytes(o.grad), np.float32))


@pytest.mark.parametrize("crt,kind", [("msvc", 0), ("glibc", 1)])
def test_product_noise_generator_matches_reference_build(crt, kind):
    """The product's table generator (rt_noise.cpp) against the reference's own Noise.cpp built
    here with each CRT's rand (tests/golden/noise_reference_<crt>_seed300.npz, make_golden.py)."""
    import gpgpuraytrace_amd as G
    ref = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                               f"noise_reference_{crt}_seed300.npz"))
    n = G.Noise()
    n.generate(seed=300, rand_kind=kind)
    assert np.array_equal(n.permutations2D, ref["perm2d"])
    assert np.array_equal(n.permutations1D, ref["grad"])


@pytest.mark.parametrize("seed", [0, 7])
def test_product_host_set_target_depths_matches_oracle(seed):
    import gpgpuraytrace_amd as G
    rng = np.random.default_rng(seed)
    cr = rng.uniform(0, 6000, (1024, 4)).astype(np.float32)
    cr[rng.random(1024) < 0.4, 3] = 5000.0
    cd = np.zeros(2048, np.float32)
    O.lib().ro_set_target_depths(O._fp(cr), O._fp(cd))
    assert np.array_equal(G.set_target_depths_host(cr), cd.reshape(1024, 2))


@pytest.mark.parametrize("res,expect", [
    # SURVEY.md §2 launch table, replayed from Terrain::calculateTileSizes (Terrain.cpp:208-242)
    ((256, 256), (1, 1, 256, 256, 16, 16, 16, 16)),
    ((480, 270), (1, 1, 480, 270, 16, 18, 30, 15)),
    ((1280, 720), (2, 2, 640, 360, 16, 18, 40, 20)),
    ((1920, 1080), (2, 3, 960, 360, 16, 18, 60, 20)),
    ((3840, 2160), (4, 5, 960, 432, 16, 16, 60, 27)),
])
def test_terrain_tile_sizes(res, expect):
    from gpgpuraytrace_amd.engine import Terrain

    class FakeDevice:
        width, height = res
    t = Terrain.__new__(Terrain)
    t.device, t.record_mode = FakeDevice(), False
    t.calculate_tile_sizes()
    assert (t.tiles_x, t.tiles_y, t.tile_x, t.tile_y, t.thread_x, t.thread_y, t.dispatch_x, t.dispatch_y) == expect


@pytest.mark.parametrize("euler", [scene.RESET_EULER, scene.LOOKDOWN_EULER])
def test_camera_matches_independent_restatement(euler):
    from gpgpuraytrace_amd import camera
    a = camera.frame_constants(1920, 1080, euler=euler)
    b = scene.frame_constants(1920, 1080, euler=euler)
    for k in ("eye", "view_inverse", "projection", "sun"):
        assert np.allclose(a[k], b[k], rtol=1e-6, atol=1e-6), k


def test_reset_pose_geometry():
    """Camera.cpp:9-20: eye (0,100,0), FOV 80, near/far 0.01/5000, LH projection."""
    from gpgpuraytrace_amd import camera
    c = camera.Camera(1920, 1080)
    p = c.projection_hlsl()
    assert np.isclose(p[1, 1], 1 / np.tan(np.radians(40)), rtol=1e-6)
    assert np.isclose(p[0, 0], p[1, 1] / (1920 / 1080), rtol=1e-6)
    assert p[2, 3] == 1.0 and np.isclose(p[3, 2], -0.01 * 5000 / (5000 - 0.01), rtol=1e-6)
    vi = c.view_inverse_hlsl()
    assert np.allclose(vi[3, :3], [0, 100, 0], atol=1e-4)  # translation row = eye
    assert np.allclose(vi[:3, :3] @ vi[:3, :3].T, np.eye(3), atol=1e-6)


@pytest.mark.parametrize("w,h,world", [(1920, 1080, 2), (1920, 1080, 8), (100, 70, 3), (64, 48, 4)])
def test_shard_mapping_partitions_frame(w, h, world):
    from gpgpuraytrace_amd import parallel as P
    tiles = np.concatenate([P.shard_tiles(w, h, r, world) for r in range(world)])
    tx, ty = P.tiles_xy(w, h)
    assert sorted(tiles.tolist()) == list(range(tx * ty))
    rng = np.random.default_rng(0)
    frame = rng.integers(0, 2 ** 32, (h, w), dtype=np.uint64).astype(np.uint32)
    out = np.zeros_like(frame)
    for r in range(world):
        P.unpack_host(out, P.pack_host(frame, r, world), r, world)
    assert np.array_equal(out, frame)


def test_shard_bytes_match_library():
    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import parallel as P
    # rt_shard_bytes needs a device handle; compare against the kernel-side formula instead
    for (w, h, world) in ((1920, 1080, 8), (333, 77, 3)):
        tx, ty = P.tiles_xy(w, h)
        for r in range(world):
            n = (tx * ty - r + world - 1) // world
            assert P.shard_bytes(w, h, r, world) == n * 32 * 32 * 4
    assert G.lib().rt_shard_bytes(None, 0, 1) == 0  # null device -> 0, no crash


REF_SRC = "/root/reference/gpuraytrace"


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference headers not present (GPU box)")
def test_cpp_adapter_compiles_against_reference_headers():
    """integration/hip_adapter.cpp implements the reference's IDevice/ICompute/IShaderVariable/
    IShaderArray/ITexture over include/frosttrace.h; compile it against the reference's own headers."""
    import subprocess
    r = subprocess.run(["g++", "-std=c++11", "-fsyntax-only", "-I", REF_SRC, "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "integration", "hip_adapter.cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_capi_errors_are_reported_not_crashes():
    import gpgpuraytrace_amd as G
    L = G.lib()
    assert L.rt_device_present(None) < 0
    assert b"null" in L.rt_last_error()
    assert L.rt_compute_get_variable(None, b"Eye") is None
    assert L.rt_array_map(None) is None
    assert L.rt_compute_run(None, 1, 1, 1) < 0
    out = C.c_void_p()
    assert L.rt_device_create(0, 0, 0, 0, C.byref(out)) < 0


def header_enum(name):
    txt = open(os.path.join(ROOT, "include", "frosttrace.h")).read()
    m = re.search(r"\b" + name + r"\s*=\s*(\d+)u?\b", txt)
    assert m, name
    return int(m.group(1))


def test_deferred_device_binding():
    """ABI 9's deferred submission as the binding sees it, without a GPU: the flag value matches the header,
    Device(deferred=True) sets it (and only it beside the others asked for), rt_device_defer_batch and
    rt_debug_defer_slot reject a null device, and the info key matches the header."""
    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import _native
    assert _native.RT_DEVICE_DEFERRED == header_enum("RT_DEVICE_DEFERRED") == 1024
    assert header_enum("RT_INFO_DEFERRED_FUSED") == 3
    d = G.engine.Device(64, 48, deferred=True)
    assert d.flags == _native.RT_DEVICE_DEFERRED
    d2 = G.engine.Device(64, 48, float_output=True, deferred=True)
    assert d2.flags == _native.RT_DEVICE_DEFERRED | _native.RT_DEVICE_FLOAT_OUTPUT
    assert G.engine.Device(64, 48).flags & _native.RT_DEVICE_DEFERRED == 0
    assert _native.RT_DEVICE_DEBUG_DEFER_SMALL == header_enum("RT_DEVICE_DEBUG_DEFER_SMALL") == 2048
    d3 = G.engine.Device(64, 48, deferred=True, debug_defer_small=True)
    assert d3.flags == _native.RT_DEVICE_DEFERRED | _native.RT_DEVICE_DEBUG_DEFER_SMALL
    L = G.lib()
    assert L.rt_device_defer_batch(None, 2) < 0 and b"null" in L.rt_last_error()
    p = C.c_void_p()
    assert L.rt_debug_defer_slot(None, 0, C.byref(p), C.byref(p), C.byref(p)) < 0
