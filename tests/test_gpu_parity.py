"""GPU parity tests (MI355X): the HIP path through the C-ABI vs the oracle /
golden fixtures.  Bar: bit-exact float32 colours and UNORM8 pixels, identical
step / noise3d counts.  Run on the GPU box with `pytest -m gpu`."""
import ctypes as C
import os

import numpy as np
import pytest

import golden_index as GI
import oracle_lib as O

pytestmark = pytest.mark.gpu


class FixedCamera:
    """Feeds the fixture's frame constants through the Terrain/ShaderVariable path."""

    def __init__(self, consts):
        self.c = consts
        self.width, self.height = consts["width"], consts["height"]

    def view_inverse_hlsl(self):
        return np.asarray(self.c["view_inverse"], np.float32)

    def projection_hlsl(self):
        return np.asarray(self.c["projection"], np.float32)

    def eye(self):
        return np.asarray(self.c["eye"], np.float32)


def make(consts, land="nomadplains", aa=1, recording=False, max_steps=0, seed=300, rand_kind=0, stats=False,
         ao=0, graph=False, small_rings=False, float_output=True, gated=False, **dev_kw):
    """float_output=False: the product's device (RGBA8 only), where one sample per pixel with at most one
    AO ray finishes hit pixels in k_trace (UnitMap::fit) instead of through per-sample colours."""
    import gpgpuraytrace_amd as G
    dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, consts["width"], consts["height"], float_output=float_output,
                                    stats=stats, graph=graph, small_rings=small_rings, gated=gated, **dev_kw)
    assert dev is not None, G.lib().rt_last_error()
    ter = G.Terrain(dev, land, record_mode=recording, aa_samples=aa, max_steps=max_steps, noise_seed=seed,
                    rand_kind=rand_kind, ao_samples=ao)
    ter.create()
    assert ter.reload(), G.lib().rt_last_error()
    ter.set_camera(FixedCamera(consts))
    ter.set_time_of_day_vec(consts["sun"])
    ter.update_shaders()
    return dev, ter


def bits_equal(a, b):
    a32, b32 = np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32)
    both_nan = np.isnan(np.asarray(a, np.float32)) & np.isnan(np.asarray(b, np.float32))
    return np.all((a32 == b32) | both_nan)


# --- numeric primitives -----------------------------------------------------------------
def _special():
    return np.array([0.0, -0.0, 1.0, -1.0, 0.5, 2.0, 1e-38, 1e-45, 3.4e38, np.inf, -np.inf, np.nan, 127.5, -149.9,
                     1.41421354, 0.70710677], np.float32)


@pytest.mark.parametrize("gop,oop,rng_lo,rng_hi,logspace", [
    (0, 0, -160, 140, False), (1, 1, -90, 90, True), (2, 2, -100, 90, False), (3, 3, -3e3, 3e3, False),
    (4, 4, -3e3, 3e3, False), (5, 5, -90, 90, True), (6, 6, -90, 90, True), (7, 7, -90, 90, True)])
def test_unary_primitives_bitexact(gop, oop, rng_lo, rng_hi, logspace):
    import gpgpuraytrace_amd as G
    dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, 8, 8)
    rng = np.random.default_rng(gop)
    x = rng.uniform(rng_lo, rng_hi, 200000)
    x = (np.exp(x) if logspace else x).astype(np.float32)
    x = np.concatenate([x, _special(), -_special()])
    y = np.empty_like(x)
    assert G.lib().rt_debug_math(dev._h, gop, x.ctypes.data, None, y.ctypes.data, x.size) == 0
    assert bits_equal(y, O.unary(oop, x))
    dev.destroy()


@pytest.mark.parametrize("gop,oop", [(8, 0), (9, 1), (10, 2), (11, 0)])
def test_binary_primitives_bitexact(gop, oop):
    import gpgpuraytrace_amd as G
    dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, 8, 8)
    rng = np.random.default_rng(10 + gop)
    a = np.exp(rng.uniform(-40, 40, 200000)).astype(np.float32)
    b = rng.uniform(-4, 41, 200000).astype(np.float32)
    if gop != 11:
        a = np.concatenate([a * np.sign(rng.uniform(-1, 1, a.size)).astype(np.float32), _special()])
        b = np.concatenate([b, _special()[::-1]])
    else:
        b = np.abs(b) + np.float32(0.01)  # pow for x >= 0, y > 0 (the hot-path form)
    y = np.empty_like(a)
    assert G.lib().rt_debug_math(dev._h, gop, a.ctypes.data, b.ctypes.data, y.ctypes.data, a.size) == 0
    assert bits_equal(y, O.binary(oop, a, b))
    dev.destroy()


def test_octave_estimate_exhaustive():
    """nomadplains' octave count from the hardware log/exp estimate (rt_shader.h np_octaves)
    equals the rule-R5 count (sqrt + polynomial pow, the oracle's) for EVERY finite float
    d2 >= 0 the estimate does not flag as near an integer."""
    import gpgpuraytrace_amd as G
    dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, 8, 8)

    def sweep(start, end):
        total = [0, 0, 0]
        while start < end:
            n = min(end - start, 1 << 30)
            a = np.array([start], np.uint32).view(np.float32)
            out = np.zeros(3, np.uint32)
            assert G.lib().rt_debug_math(dev._h, 12, a.ctypes.data, None, out.ctypes.data, n) == 0
            total = [t + int(o) for t, o in zip(total, out)]
            start += n
        return total

    every = sweep(0, 0x7F800000)  # +0 .. largest finite
    lo, hi = (int(np.array([v], np.float32).view(np.uint32)[0]) for v in (1e-4, 4e7))
    scene = sweep(lo, hi)         # distances 0.01 .. 6300: where the march samples
    dev.destroy()
    assert every[2] == 0x7F800000 and scene[2] == hi - lo
    assert every[0] == 0, f"{every[0]} unflagged estimates differ from the exact octave count"
    assert scene[1] < scene[2] // 200, scene  # the exact fallback stays rare


# --- noise3d and getDensity ---------------------------------------------------------------
@pytest.mark.parametrize("seed,kind", [(300, 0), (777, 1)])
def test_noise3d_bitexact(seed, kind):
    import gpgpuraytrace_amd as G
    consts = GI.consts(64, 48, "reset")
    dev, ter = make(consts, seed=seed, rand_kind=kind)
    rng = np.random.default_rng(5)
    p = np.concatenate([rng.uniform(-500, 500, (100000, 3)), rng.uniform(-2e6, 2e6, (20000, 3)),
                        rng.integers(-300, 300, (2000, 3))]).astype(np.float32)
    out = np.empty(len(p), np.float32)
    assert G.lib().rt_debug_noise(ter.compute._h, p.ctypes.data, out.ctypes.data, len(p), 0) == 0
    assert bits_equal(out, O.noise3d(O.noise_tables(seed, kind), p))
    dev.destroy()


def test_noise3d_z0_equals_noise3d_at_z0():
    """noise3d_z0(x, y), nomadplains' steep noise in k_trace (rt_shader.h), equals the oracle's
    noise3d(x, y, 0) bit for bit up to the sign of a zero (lattice points included, where the
    value is a zero); the density tests cover its only use, sat((n - 0.2) * 6)."""
    import gpgpuraytrace_amd as G
    dev, ter = make(GI.consts(64, 48, "reset"))
    rng = np.random.default_rng(10)
    p = np.concatenate([rng.uniform(-500, 500, (100000, 3)), rng.uniform(-2e6, 2e6, (20000, 3)),
                        rng.integers(-300, 300, (2000, 3))]).astype(np.float32)
    p[:, 2] = 0.0
    out = np.empty(len(p), np.float32)
    assert G.lib().rt_debug_noise(ter.compute._h, p.ctypes.data, out.ctypes.data, len(p), 2) == 0
    ref = O.noise3d(O.noise_tables(), p)
    assert np.array_equal(out, ref)  # +0 == -0
    assert bits_equal(out[ref != 0], ref[ref != 0])
    assert (ref == 0).sum() >= 2000
    dev.destroy()


@pytest.mark.parametrize("land", ["nomadplains", "testing", "simple", "greenrocks"])
def test_density_bitexact(land):
    import gpgpuraytrace_amd as G
    consts = GI.consts(64, 48, "reset")
    dev, ter = make(consts, land=land)
    rng = np.random.default_rng(6)
    p = np.concatenate([rng.uniform(-3000, 3000, (30000, 3)) * [1, 0.05, 1] + [0, 50, 0],
                        rng.uniform(-20, 20, (5000, 3)) + [0, 100, 0]]).astype(np.float32)
    out = np.empty(len(p), np.float32)
    assert G.lib().rt_debug_noise(ter.compute._h, p.ctypes.data, out.ctypes.data, len(p), 1) == 0
    fr = O.make_frame(consts, landscape=O.LANDSCAPES[land])
    assert bits_equal(out, O.density(O.noise_tables(), fr, p))
    dev.destroy()


# --- whole frames vs the golden oracle frames ----------------------------------------------
@pytest.mark.parametrize("kernels", ["stats", "product", "spill", "fit", "fit_spill"])
@pytest.mark.parametrize("spec", GI.FRAMES, ids=[GI.frame_key(*s) for s in GI.FRAMES])
def test_frame_bitexact_device_path(spec, kernels):
    """stats: the instrumented kernels (their counts equal the oracle's too); product: the
    uninstrumented kernels the bench times; spill: the product kernels with a 64-entry LDS long ring
    and an 8-slot fin pool (RT_DEVICE_DEBUG_SMALL_RINGS), so queued long rays go through the
    per-block spill rings and long shadows through the fin[t] fallback; fit / fit_spill: the same
    without float output, the bench's device (one sample per pixel and <= 1 AO ray: hit pixels
    finished in k_trace, UnitMap::fit), UNORM8 against the golden frame."""
    gold = GI.load()
    land, pose, w, h, aa, ms, ao = GI.unpack(spec)
    key = GI.frame_key(*spec)
    fit = kernels.startswith("fit")
    dev, ter = make(GI.consts(w, h, pose), land=land, aa=aa, max_steps=ms, stats=kernels == "stats", ao=ao,
                    small_rings=kernels.endswith("spill"), float_output=not fit)
    ter.render_device()
    dev.present()
    img8 = dev.readback()
    assert np.array_equal(img8, gold[key + "_rgba8"])
    dev.check()
    if fit:
        assert np.array_equal(_device_cells(ter), gold[key + "_cell_distance"])
        dev.destroy()
        return
    img = dev.readback_float()
    assert bits_equal(img, gold[key + "_rgba32f"])
    if kernels != "stats":
        assert np.array_equal(_device_cells(ter), gold[key + "_cell_distance"])
        dev.destroy()
        return
    st = dev.stats()
    ref = gold[key + "_stats"]  # noise3d, prepass, primary, shadow, rays, hits, ao
    assert (st["noise_calls"], st["prepass_steps"], st["primary_steps"], st["shadow_steps"], st["hits"],
            st["ao_steps"]) == (ref[0], ref[1], ref[2], ref[3], ref[5], ref[6])
    # wave iterations of the noise work (ABI 2): every one has at least one lane
    assert 0 < st["noise_wave_iters"] <= st["noise_calls"]
    assert np.array_equal(_device_cells(ter), gold[key + "_cell_distance"])
    dev.destroy()


def test_noise_wave_iterations_bound_lane_utilisation():
    """rt_stats.noise_wave_iters (ABI 2): over a tracescreen (the prepass's lane-only counts
    subtracted), 64 * wave iterations >= noise evaluations, i.e. lane utilisation in (0, 1]."""
    dev, ter = make(GI.consts(64, 48, "reset"), stats=True, max_steps=0, ao=1)
    ter.update_shaders()
    ter.camera_compute.run(2, 2, 1)
    pre = dev.stats(reset=True)
    ter.render_device()
    st = dev.stats(reset=True)
    calls = st["noise_calls"] - pre["noise_calls"]
    waves = st["noise_wave_iters"] - pre["noise_wave_iters"]
    assert pre["noise_wave_iters"] == 0 and waves > 0
    util = calls / (64.0 * waves)
    # a 64x48 frame is mostly partial units (its 8x8 units straddle the horizon): measured 0.449 with
    # the product's primary segment tail (ABI 6); far too many counted wave iterations fall below this
    assert 0.35 < util <= 1.0, util
    dev.destroy()


def _device_cells(ter):
    """CellDistance as computed on the device (SRV arrays have no map(), so copy directly)."""
    import gpgpuraytrace_amd as G
    p = ter.var_cell_distance.device_pointer()
    out = np.empty((1024, 2), np.float32)
    G.lib().rt_device_synchronize(ter.device._h)
    lib = C.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert lib.hipMemcpy(out.ctypes.data, p, out.nbytes, 2) == 0  # hipMemcpyDeviceToHost
    return out


@pytest.mark.parametrize("spec", [GI.FRAMES[0], GI.FRAMES[1], GI.FRAMES[4]], ids=["np_reset", "np_down", "testing"])
def test_frame_bitexact_reference_call_sequence(spec):
    """Terrain::render's own sequence: run(2,2,1) -> CameraResults map/unmap -> host
    setTargetDepths -> CellDistance write -> per-tile ThreadOffset write + run + flush."""
    gold = GI.load()
    land, pose, w, h, aa, ms, ao = GI.unpack(spec)
    key = GI.frame_key(*spec)
    dev, ter = make(GI.consts(w, h, pose), land=land, aa=aa, max_steps=ms, ao=ao)
    ter.render()
    dev.present()
    assert bits_equal(dev.readback_float(), gold[key + "_rgba32f"])
    assert np.array_equal(ter.camera_view, gold[key + "_camera_results"])
    dev.destroy()


DRIVER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "integration", "_build",
                      "terrain_driver")


@pytest.mark.parametrize("mode", ["ref", "device", "deferred"])
@pytest.mark.parametrize("spec", [GI.FRAMES[0], GI.FRAMES[1], GI.FRAMES[4], GI.FRAMES[9]],
                         ids=["np_reset", "np_down", "testing", "np_down_ms512_ao4"])
def test_cpp_adapter_terrain_sequence(spec, mode, tmp_path):
    """The C++ adapter (integration/hip_adapter.cpp: DeviceHIP, ComputeHIP, ShaderVariableHIP,
    ShaderArrayHIP, TextureHIP) driven through the reference's own interfaces by
    integration/terrain_driver.cpp, which replays Terrain::create / reload / updateShaders /
    render (Terrain.cpp:55-206: run(2,2,1) -> CameraResults map/unmap -> setTargetDepths ->
    CellDistance write -> per tile ThreadOffset write + run + flush -> present), the one-call
    device path, or that path on an RT_DEVICE_DEFERRED device (DeviceHIP::setFlags) over three frames;
    the RGBA8 readback and CameraResults equal the golden frame's."""
    assert os.path.exists(DRIVER), "integration/_build/terrain_driver not built (make -C integration, needs " \
                                   "the reference headers: __graft_entry__.build() in the build container)"
    import subprocess
    gold = GI.load()
    land, pose, w, h, aa, ms, ao = GI.unpack(spec)
    key = GI.frame_key(*spec)
    c = GI.consts(w, h, pose)
    cin, cout = tmp_path / "consts.bin", tmp_path / "out.bin"
    with open(cin, "wb") as f:  # the cbuffer bytes Terrain writes (XMMatrixTranspose of the matrices)
        f.write(np.array([w, h], np.int32).tobytes())
        f.write(np.ascontiguousarray(np.asarray(c["view_inverse"], np.float32).T).tobytes())
        f.write(np.asarray(c["eye"], np.float32).tobytes())
        f.write(np.ascontiguousarray(np.asarray(c["projection"], np.float32).T).tobytes())
        f.write(np.asarray(c["sun"], np.float32).tobytes())
    r = subprocess.run([DRIVER, str(cin), str(cout), land, str(aa), str(ms), str(ao), mode],
                       capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    raw = np.fromfile(cout, np.uint8)
    img8 = raw[:w * h * 4].reshape(h, w, 4)
    cam = raw[w * h * 4:].view(np.float32).reshape(1024, 4)
    assert np.array_equal(img8, gold[key + "_rgba8"])
    assert np.array_equal(cam, gold[key + "_camera_results"])


def test_tiled_dispatch_1280x720_rows():
    """2x2 tiles of 640x360 with 16x18 groups (Terrain.cpp:208-242) through the compat path."""
    consts = _consts_1080p_like(1280, 720)
    dev, ter = make(consts)
    assert (ter.tiles_x, ter.tiles_y, ter.thread_x, ter.thread_y) == (2, 2, 16, 18)
    ter.render()
    img = dev.readback_float()
    fr = O.make_frame(consts, rows=(0, 720, 48))
    ref = np.zeros((720, 1280, 4), np.float32)
    cd = np.zeros(2048, np.float32)
    cr = np.zeros(4096, np.float32)
    O.lib().ro_camerarays(C.byref(O.noise_tables()), C.byref(fr), O._fp(cr), None)
    O.lib().ro_set_target_depths(O._fp(cr), O._fp(cd))
    O.lib().ro_tracescreen(C.byref(O.noise_tables()), C.byref(fr), O._fp(cd), O._fp(ref), None, None, None)
    assert bits_equal(img[0::48], ref[0::48])
    dev.destroy()


def _consts_1080p_like(w, h, pose="reset"):
    from gpgpuraytrace_amd import camera
    euler = camera.INITIAL_ROTATION_EULER if pose == "reset" else camera.LOOKDOWN_ROTATION_EULER
    return camera.frame_constants(w, h, euler=euler)


@pytest.mark.parametrize("pose", ["reset", "lookdown"])
def test_1080p_full_frame_rows_and_properties(pose):
    """BASELINE size: bit-exact on a row sample vs the oracle, plus whole-frame properties
    (prepass + cells exact, every pixel written, alpha 255)."""
    gold_scene = GI.consts(1920, 1080, pose)
    dev, ter = make(gold_scene, stats=True)
    ter.render_device()
    img = dev.readback_float()
    img8 = dev.readback()
    st = dev.stats()
    fr = O.make_frame(gold_scene, rows=(0, 1080, 54))
    ref = np.zeros((1080, 1920, 4), np.float32)
    cr = np.zeros(4096, np.float32)
    cd = np.zeros(2048, np.float32)
    ost = O.Stats()
    O.lib().ro_camerarays(C.byref(O.noise_tables()), C.byref(fr), O._fp(cr), C.byref(ost))
    O.lib().ro_set_target_depths(O._fp(cr), O._fp(cd))
    O.lib().ro_tracescreen(C.byref(O.noise_tables()), C.byref(fr), O._fp(cd), O._fp(ref), None, None, C.byref(ost))
    assert bits_equal(img[0::54], ref[0::54])
    assert np.array_equal(_device_cells(ter), cd.reshape(1024, 2))
    assert np.all(img8[..., 3] == 255) and np.all(img[..., 3] == 1.0)
    assert st["prepass_steps"] == ost.prepass_steps
    dev.destroy()


@pytest.mark.parametrize("aa", [1, 4])
def test_max_ao_bitexact(aa):
    """RT_AO_SAMPLES=16, the most the AO extension takes: k_trace counts each sample's occluded AO
    rays in one byte, four samples to a word (16 fits; neighbours' counts must not bleed), and
    k_finish applies them -- bit-exact against the oracle's whole frame, one and four samples per
    pixel (the look-down pose: most pixels hit, many AO rays occluded)."""
    consts = GI.consts(64, 48, "lookdown")
    fr = O.make_frame(consts, aa=aa, max_steps=128, ao=16)
    ref = O.render(O.noise_tables(), fr)
    dev, ter = make(consts, aa=aa, max_steps=128, ao=16, stats=True)
    ter.render_device()
    assert bits_equal(dev.readback_float(), ref["rgba32f"])
    assert np.array_equal(dev.readback(), ref["rgba8"])
    st = dev.stats()
    assert st["ao_steps"] == ref["stats"]["ao_steps"] and st["hits"] == ref["stats"]["primary_hits"]
    dev.destroy()


# BASELINE.json GPU configs at their full sizes (configs[1], [2], [4]): the product path vs the
# oracle on a row sample (rows r0::step; the oracle renders only those rows).  C3 is the
# bench's headline workload, C5 the 4K / 1024-step / 4-AO one.
BASELINE_CONFIGS = {  # name: (W, H, max_steps, ao, row_step)
    "c1": (256, 256, 64, 0, 1),
    "c2": (1280, 720, 256, 0, 8),
    "c3": (1920, 1080, 512, 1, 8),
    "c5": (3840, 2160, 1024, 4, 36),
}


def _config_rows(name, pose, r0):
    w, h, ms, ao, step = BASELINE_CONFIGS[name]
    consts = _consts_1080p_like(w, h, pose)
    fr = O.make_frame(consts, max_steps=ms, ao=ao, rows=(r0, h, step))
    return consts, O.render_rows(O.noise_tables(), fr), slice(r0, h, step)


@pytest.mark.parametrize("pose", ["reset", "lookdown"])
@pytest.mark.parametrize("name", sorted(BASELINE_CONFIGS))
def test_baseline_config_rows_bitexact(name, pose):
    """rt_terrain_render (the device path: prepass -> device setTargetDepths -> k_trace) at the
    config's full size, step cap and AO count: float32 colour and UNORM8 bit-exact against the
    oracle on the row sample, the whole CameraResults / CellDistance exact, every pixel written."""
    w, h, ms, ao, step = BASELINE_CONFIGS[name]
    consts, (ref, ref8, cr, cd, _), rows = _config_rows(name, pose, 5)
    dev, ter = make(consts, max_steps=ms, ao=ao)
    ter.render_device()
    img, img8 = dev.readback_float(), dev.readback()
    assert bits_equal(img[rows], ref[rows])
    assert np.array_equal(img8[rows], ref8[rows])
    assert np.array_equal(_device_cells(ter), cd)
    ter.get_camera_results()
    assert np.array_equal(ter.camera_view, cr)
    assert np.all(img8[..., 3] == 255) and np.all(img[..., 3] == 1.0)
    dev.destroy()


def test_c5_batched_graph_frame_loop_rows_bitexact():
    """BASELINE C5's frame loop as `bench.py --config c5` runs it: a FrameRing of 2-frame batches,
    2 batches in flight, every batch a replay of its slot group's captured hipGraphs, at 3840x2160
    with the 1024-step cap and 4 AO rays per hit.  Three batches (group 0 captures, then replays),
    every frame of the last two float32- and UNORM8-bit-exact against the oracle's row sample."""
    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E
    w, h, ms, ao, step = BASELINE_CONFIGS["c5"]
    ring = E.FrameRing(w, h, depth=2, camera=G.Camera(w, h), time_of_day=0.3, max_steps=ms, ao_samples=ao,
                       graph=True, batch=2, float_output=True)
    for _ in range(3):
        ring.render_batch()
    ring.synchronize()
    fr = O.make_frame(_consts_1080p_like(w, h, "reset"), max_steps=ms, ao=ao, rows=(11, h, step))
    ref, ref8, _, _, _ = O.render_rows(O.noise_tables(), fr)
    rows = slice(11, h, step)
    for dev, _ in ring.slots:
        assert bits_equal(dev.readback_float()[rows], ref[rows])
        assert np.array_equal(dev.readback()[rows], ref8[rows])
    cap0, launch0 = ring.slots[0][0].graph_info()
    cap1, launch1 = ring.slots[2][0].graph_info()
    # group 0 replayed its graphs: one per batch with the gated launch (tracescreen runs the prepass), two
    # with a prepass launch of its own
    per = _graphs_per_render(ring.slots[0][0])
    assert cap0 == cap1 == per and launch0 == 2 * launch1 > 0
    ring.destroy()


@pytest.mark.parametrize("land,ao", [("testing", 0), ("simple", 1), ("greenrocks", 1)])
def test_other_landscapes_720p_rows_bitexact(land, ao):
    """The other live landscapes (analytic testing, simple, greenrocks with its fog live) at the
    C2 size and step cap, with and without AO, through rt_terrain_render: float32 colour and
    UNORM8 bit-exact against the oracle on every 24th row, CellDistance exact."""
    w, h, ms, step = 1280, 720, 256, 24
    consts = _consts_1080p_like(w, h, "reset")
    fr = O.make_frame(consts, landscape=O.LANDSCAPES[land], max_steps=ms, ao=ao, rows=(7, h, step))
    ref, ref8, _, cd, _ = O.render_rows(O.noise_tables(), fr)
    rows = slice(7, h, step)
    dev, ter = make(consts, land=land, max_steps=ms, ao=ao)
    ter.render_device()
    assert bits_equal(dev.readback_float()[rows], ref[rows])
    assert np.array_equal(dev.readback()[rows], ref8[rows])
    assert np.array_equal(_device_cells(ter), cd)
    dev.destroy()


@pytest.mark.parametrize("name,small_rings,fit", [("c2", False, False), ("c3", False, False), ("c3", True, False),
                                                  ("c2", False, True), ("c3", False, True), ("c3", True, True)])
def test_baseline_config_batch_rows_bitexact(name, small_rings, fit):
    """The bench's entry point: one rt_terrain_render_batch of 4 frames (reset, look-down,
    reset, look-down) at the config's size; every frame equals the oracle on its row sample.
    small_rings: the C3 batch with 64-entry LDS rings, so most queued work spills to HBM.  fit: the
    bench's RGBA8-only devices (hit pixels finished in k_trace; C2 has no k_finish at all)."""
    from gpgpuraytrace_amd import engine as E
    w, h, ms, ao, step = BASELINE_CONFIGS[name]
    poses = ["reset", "lookdown", "reset", "lookdown"]
    refs = {p: _config_rows(name, p, 3) for p in ("reset", "lookdown")}
    frames = [make(refs[p][0], max_steps=ms, ao=ao, small_rings=small_rings, float_output=not fit) for p in poses]
    E.render_batch([t for _, t in frames])
    for (dev, _), p in zip(frames, poses):
        _, (ref, ref8, _, _, _), rows = refs[p]
        if not fit:
            assert bits_equal(dev.readback_float()[rows], ref[rows])
        assert np.array_equal(dev.readback()[rows], ref8[rows])
        dev.check()
    for d, _ in frames:
        d.destroy()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_shards_assemble_to_full_frame(world):
    import torch

    from gpgpuraytrace_amd import engine as E
    consts = GI.consts(256, 256, "reset")
    full_dev, full_ter = make(consts)
    full_ter.render_device()
    full = full_dev.readback()
    devs = [make(consts) for _ in range(world)]
    maxb = max(E.shard_bytes(d, r, world) for r, (d, _) in enumerate(devs))
    bufs = [torch.zeros(maxb, dtype=torch.uint8, device="cuda:0") for _ in range(world)]
    torch.cuda.synchronize()  # the fill (torch's stream) before the devices' non-blocking streams
    for r, (d, t) in enumerate(devs):
        t.render_device(r, world)
        E.shard_pack(d, r, world, bufs[r].data_ptr())
        d.synchronize()
    d0 = devs[0][0]
    for r in range(1, world):
        E.shard_unpack(d0, r, world, bufs[r].data_ptr())
    assert np.array_equal(d0.readback(), full)
    for d, _ in devs:
        d.destroy()
    full_dev.destroy()


@pytest.mark.parametrize("w,h,world,frames", [(1920, 1080, 8, 12), (50, 36, 3, 5), (64, 48, 3, 4)])
def test_shard_batch_pack_unpack_roundtrip(w, h, world, frames):
    """rt_shard_pack_batch / rt_shard_unpack_batch (one launch for a batch's frames, devices on
    separate streams) against the host tile mapping (parallel.pack_host): random framebuffers
    are packed with frame f's rotated shard (f % N) into offsets of one buffer, which must hold
    exactly pack_host's tiles; unpacked into fresh devices, every shard's pixels come back and no
    other pixel is touched.  1920x1080 takes the 16-byte path (its last tile row is partial),
    50x36 the per-pixel one (W % 4 != 0), 64x48 ragged shards of 2/1/1 tiles."""
    import torch

    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E
    from gpgpuraytrace_amd import parallel as P
    rng = np.random.default_rng(11)
    devs = [G.DeviceFactory.construct(G.DeviceAPI.HIP, w, h) for _ in range(frames)]
    imgs = [rng.integers(0, 2**32, (h, w), dtype=np.uint32) for _ in range(frames)]
    # fill each framebuffer through the single-job unpack of every shard from host-packed tiles
    for d, img in zip(devs, imgs):
        for s in range(world):
            src = torch.from_numpy(P.pack_host(img, s, world).view(np.int32)).to("cuda:0")
            if src.numel():
                E.shard_unpack(d, s, world, src.data_ptr())
        d.synchronize()
        assert np.array_equal(d.readback().view(np.uint32).reshape(h, w), img)
    plan = P.BatchPlan(w, h, frames, world)
    packed = torch.zeros(plan.packed_bytes(), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()  # the fill (torch's stream) before the devices' non-blocking streams
    items = [(f, f % world, plan.pack_offset(f)) for f in range(frames)]
    E.shard_pack_batch([devs[f] for f, _, _ in items], [s for _, s, _ in items], world,
                       [packed.data_ptr() + off for _, _, off in items])
    devs[0].synchronize()
    got = packed.cpu().numpy().view(np.uint32)
    for f, s, off in items:
        want = P.pack_host(imgs[f], s, world)
        inside = P.pack_host(np.ones((h, w), np.uint32), s, world) == 1  # pixels of the frame
        part = got[off // 4:off // 4 + want.size]
        assert np.array_equal(part[inside], want[inside]), (f, s)
        assert not part[~inside].any(), (f, s)  # padding pixels of partial tiles are not written
    fresh = [G.DeviceFactory.construct(G.DeviceAPI.HIP, w, h) for _ in range(frames)]
    E.shard_unpack_batch([fresh[f] for f, _, _ in items], [s for _, s, _ in items], world,
                         [packed.data_ptr() + off for _, _, off in items])
    for f, s, _ in items:
        img = fresh[f].readback().view(np.uint32).reshape(h, w)
        mine = P.unpack_host(np.zeros((h, w), np.uint32), P.pack_host(imgs[f], s, world), s, world)
        assert np.array_equal(img, mine), (f, s)
    with pytest.raises(Exception):
        E.shard_pack_batch([devs[0]], [world], world, [packed.data_ptr()])  # shard out of range
    for d in devs + fresh:
        d.destroy()


@pytest.mark.parametrize("w,h,world,frames,pose,ao,land", [
    (1920, 1080, 8, 3, "reset", 1, "nomadplains"),    # the bench's C3 shard: fit + k_finish
    (64, 48, 3, 4, "lookdown", 4, "nomadplains"),     # fitm (AO slots + colour pool), ragged shards
    (64, 48, 2, 2, "reset", 0, "nomadplains"),        # fit with no k_finish
    (48, 32, 3, 3, "reset", 2, "greenrocks"),         # fog live
])
def test_render_batch_packed_equals_render_then_pack(w, h, world, frames, pose, ao, land):
    """rt_terrain_render_batch_packed (ABI 7, parallel.run_batch's direct pack): every rank's shards
    rendered straight into the packed buffer are byte-identical to render_batch + rt_shard_pack_batch of
    the same rank (padding of partial tiles untouched), and the framebuffers are not written."""
    import torch

    from gpgpuraytrace_amd import engine as E
    from gpgpuraytrace_amd import parallel as P
    consts = _consts_1080p_like(w, h, pose) if w >= 1280 else GI.consts(w, h, pose)
    plan = P.BatchPlan(w, h, frames, world)
    ms = 512 if w >= 1280 else 0
    direct = [make(consts, land, max_steps=ms, ao=ao, float_output=False) for _ in range(frames)]
    ref = [make(consts, land, max_steps=ms, ao=ao, float_output=False) for _ in range(frames)]
    for rank in range(world):
        a = torch.zeros(plan.packed_bytes(), dtype=torch.uint8, device="cuda:0")
        b = torch.zeros_like(a)
        torch.cuda.synchronize()
        E.render_batch_packed([t for _, t in direct], rank, world, a.data_ptr(), plan.max_bytes)
        E.render_batch([t for _, t in ref], rank, world)
        items = plan.packs(rank)
        E.shard_pack_batch([ref[f][0] for f, _, _ in items], [s for _, s, _ in items], world,
                           [b.data_ptr() + off for _, _, off in items])
        for d, _ in direct + ref:
            d.synchronize()
        assert torch.equal(a, b), rank
        for d, _ in direct:  # never written: still the cleared framebuffer
            assert not d.readback().any()
        for d, _ in direct + ref:
            d.check()
    for d, _ in direct + ref:
        d.destroy()


@pytest.mark.parametrize("land", ["nomadplains", "greenrocks"])
def test_recording_macro_bitexact(land):
    consts = GI.consts(48, 32, "reset")
    dev, ter = make(consts, land=land, recording=True)
    ter.render_device()
    r = O.render(O.noise_tables(), O.make_frame(consts, landscape=O.LANDSCAPES[land], recording=1))
    assert bits_equal(dev.readback_float(), r["rgba32f"])
    dev.destroy()


def test_random_seed_tables_bitexact():
    consts = GI.consts(48, 32, "lookdown")
    dev, ter = make(consts, seed=424242, rand_kind=1)
    ter.render_device()
    r = O.render(O.noise_tables(424242, 1), O.make_frame(consts))
    assert bits_equal(dev.readback_float(), r["rgba32f"])
    dev.destroy()


def test_reference_error_behaviour():
    import gpgpuraytrace_amd as G
    consts = GI.consts(64, 48, "reset")
    dev, ter = make(consts)
    cs = dev.create_compute()
    assert not cs.create("shaders", "nosuch.hlsl", "CSMain", (16, 16, 1))
    assert not cs.create("shaders", "tracescreen.hlsl", "CSMain", (16, 16, 1), [("AA_SAMPLES", "3")])
    assert cs.create("shaders", "tracescreen.hlsl", "CSMain", (16, 16, 1))
    cs.run(1, 1, 1)  # no current shader before swap(): silent no-op (ComputeDirect3D.cpp:532)
    assert cs.swap() and not cs.swap()
    assert cs.get_variable("NoSuchVar") is None and cs.get_buffer("CBFrame") is None
    assert cs.get_array("CellDistance").map() is None       # SRV: map unsupported
    cam = ter.camera_compute.get_array("CameraResults")
    assert cam.write(np.zeros((1024, 4), np.float32)) is False  # UAV: write unsupported
    with pytest.raises(G.NativeError):
        cs.run(1, 1, 1)  # texture stage 0 not bound
    G.vfs_add_path("Media/benchmark")
    assert not cs.create("shaders", "tracescreen.hlsl", "CSMain", (16, 16, 1))  # benchmark does not compile
    G.vfs_add_path("Media/nomadplains")
    dev.destroy()


def test_frame_ring_in_flight_bitexact():
    """engine.FrameRing (bench.py's frames in flight): 6 frames over 3 slots, the camera switching
    every frame while the other slots' frames are still running; each slot's last frame equals
    the golden frame of its camera."""
    import gpgpuraytrace_amd as G
    gold = GI.load()
    specs = [GI.FRAMES[0], GI.FRAMES[1]]  # nomadplains 64x48, reset / lookdown
    cams = []
    for spec in specs:
        land, pose, w, h, aa, ms, ao = GI.unpack(spec)
        cams.append((FixedCamera(GI.consts(w, h, pose)), GI.frame_key(*spec)))
    w, h = cams[0][0].width, cams[0][0].height
    ring = G.FrameRing(w, h, depth=3, camera=cams[0][0])
    for _, ter in ring.slots:
        ter.set_time_of_day_vec(cams[0][0].c["sun"])
    last = {}
    for i in range(6):
        cam, key = cams[i % 2]
        dev = ring.render(camera=cam)
        last[id(dev)] = key
    ring.synchronize()
    for dev, _ in ring.slots:
        assert np.array_equal(dev.readback(), gold[last[id(dev)] + "_rgba8"]), last[id(dev)]
    ring.destroy()


def test_frame_ring_lookahead_bitexact():
    """FrameRing(lookahead=True) (bench.py's default frame loop): each batch's prepass queued on
    the side stream before the previous batch's trace (rt_terrain_prepass_ahead), two slot groups
    so the ahead prepass rewrites CameraResults the batch before it in the same group read; every
    batch equals the golden frames of its cameras, including a batch whose cameras change after
    its prepass was queued (rt_terrain_trace_ahead prepasses again) and a partial batch."""
    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E
    gold = GI.load()
    cams = []
    for spec in (GI.FRAMES[0], GI.FRAMES[1]):  # nomadplains 64x48, reset / lookdown
        land, pose, w, h, aa, ms, ao = GI.unpack(spec)
        cams.append((FixedCamera(GI.consts(w, h, pose)), GI.frame_key(*spec)))
    w, h = cams[0][0].width, cams[0][0].height
    ring = G.FrameRing(w, h, depth=2, batch=3, camera=cams[0][0], lookahead=True)
    for _, ter in ring.slots:
        ter.set_time_of_day_vec(cams[0][0].c["sun"])

    def set_group(g, seq):
        keys = []
        for (dev, ter), c in zip(ring.slots[g * 3:(g + 1) * 3], seq):
            ter.set_camera(cams[c][0])
            ter.update_terrain()
            keys.append((dev, cams[c][1]))
        return keys

    def check(keys, n=3):
        for dev, key in keys[:n]:
            assert np.array_equal(dev.readback(), gold[key + "_rgba8"]), key

    seqs = [(0, 1, 0), (1, 0, 0), (1, 1, 0), (0, 0, 1), (0, 1, 1), (1, 0, 1)]
    expect = [set_group(0, seqs[0])]
    for b in range(len(seqs)):
        if b + 1 < len(seqs):  # the next batch's cameras, before its prepass is queued below
            expect.append(set_group((b + 1) % 2, seqs[b + 1]))
        n = 2 if b == 4 else 3  # batch 4: a partial batch (the ahead prepass covered 3 frames)
        ring.render_batch(frames=n, ahead=b + 1 < len(seqs))
        if b == 2:  # batch 3's cameras change after its ahead prepass was queued
            expect[3] = set_group(1, (1, 0, 1))
        if b >= 1:  # the previous batch (the other group), while this one runs
            check(expect[b - 1], 2 if b - 1 == 4 else 3)
    ring.synchronize()
    check(expect[-1])
    # one ahead prepass per leading device at a time; none on hipGraph devices
    ters = [t for _, t in ring.slots[:3]]
    E.prepass_ahead(ters)
    with pytest.raises(RuntimeError):
        E.prepass_ahead(ters)
    E.trace_ahead(ters)
    ring.synchronize()
    ring.destroy()
    dev, ter = make(GI.consts(w, h, "reset"), graph=True)
    with pytest.raises(RuntimeError):
        E.prepass_ahead([ter])
    dev.destroy()


def test_trace_ahead_uses_the_ahead_prepass_unless_a_camera_changed():
    """rt_terrain_trace_ahead consumes the pending ahead prepass (one prepass in the stats) when the
    camera constants were only rewritten with the same bytes (rt_variable_write skips unchanged
    bytes), and prepasses again in line after a real camera change; the frames are golden both ways."""
    from gpgpuraytrace_amd import engine as E
    gold = GI.load()
    s0, s1 = GI.FRAMES[0], GI.FRAMES[1]  # nomadplains 64x48, reset / lookdown
    land, pose0, w, h, aa, ms, ao = GI.unpack(s0)
    pose1 = GI.unpack(s1)[1]
    dev, ter = make(GI.consts(w, h, pose0), stats=True)
    one = gold[GI.frame_key(*s0) + "_stats"][1]  # prepass steps of one frame
    dev.stats(reset=True)
    E.prepass_ahead([ter])
    ter.update_terrain()  # the same camera written again
    E.trace_ahead([ter])
    dev.synchronize()
    assert dev.stats(reset=True)["prepass_steps"] == one
    assert np.array_equal(dev.readback(), gold[GI.frame_key(*s0) + "_rgba8"])
    E.prepass_ahead([ter])
    ter.set_camera(FixedCamera(GI.consts(w, h, pose1)))
    ter.update_terrain()  # a real change after the ahead prepass was queued
    E.trace_ahead([ter])
    dev.synchronize()
    assert dev.stats(reset=True)["prepass_steps"] == one + gold[GI.frame_key(*s1) + "_stats"][1]
    assert np.array_equal(dev.readback(), gold[GI.frame_key(*s1) + "_rgba8"])
    dev.destroy()


@pytest.mark.parametrize("spec", GI.FRAMES, ids=[GI.frame_key(*s) for s in GI.FRAMES])
def test_graph_replay_bitexact(spec):
    """RT_DEVICE_GRAPH (the C5 hipGraph frame loop): frames replayed from the captured graphs
    equal the golden frames, stats included; replays capture once."""
    gold = GI.load()
    land, pose, w, h, aa, ms, ao = GI.unpack(spec)
    key = GI.frame_key(*spec)
    dev, ter = make(GI.consts(w, h, pose), land=land, aa=aa, max_steps=ms, stats=True, ao=ao, graph=True)
    for _ in range(3):
        ter.render_device()
        dev.present()
        img, img8 = dev.readback_float(), dev.readback()
        st = dev.stats()
        assert bits_equal(img, gold[key + "_rgba32f"])
        assert np.array_equal(img8, gold[key + "_rgba8"])
        ref = gold[key + "_stats"]
        assert (st["noise_calls"], st["primary_steps"], st["shadow_steps"], st["ao_steps"]) == \
            (ref[0], ref[2], ref[3], ref[6])
    assert dev.graph_info() == (2, 6)
    dev.destroy()


def _graphs_per_render(dev):
    """hipGraphs one render of `dev` captures / replays: the tracescreen graph, plus the prepass graph when
    the prepass is its own launch (not the gated launch of ABI 7)."""
    gated, inline = dev.launch_info()
    assert (gated > 0) != (inline > 0)
    return 1 if gated else 2


def test_graph_constants_shards_and_swap():
    """A replay reads the constants uploaded before it (camera switch: no re-capture); a new
    shard or a shader swap re-captures; shards replayed from graphs assemble to the frame."""
    import torch

    from gpgpuraytrace_amd import engine as E
    gold = GI.load()
    ka, kb = GI.frame_key(*GI.FRAMES[0]), GI.frame_key(*GI.FRAMES[1])  # 64x48 reset / lookdown
    ca, cb = GI.consts(64, 48, "reset"), GI.consts(64, 48, "lookdown")
    dev, ter = make(ca, graph=True)
    for consts, key in ((ca, ka), (cb, kb), (ca, ka)):
        ter.set_camera(FixedCamera(consts))
        ter.set_time_of_day_vec(consts["sun"])
        ter.update_terrain()
        ter.render_device()
        assert np.array_equal(dev.readback(), gold[key + "_rgba8"]), key
    per = _graphs_per_render(dev)
    assert dev.graph_info() == (per, 3 * per)
    # two shards replayed on one device, packed, then assembled
    bufs = [torch.zeros(E.shard_bytes(dev, r, 2), dtype=torch.uint8, device="cuda:0") for r in range(2)]
    torch.cuda.synchronize()  # the fill (torch's stream) before the device's non-blocking stream
    for r in (1, 0):
        ter.render_device(r, 2)
        E.shard_pack(dev, r, 2, bufs[r].data_ptr())
    E.shard_unpack(dev, 1, 2, bufs[1].data_ptr())
    assert np.array_equal(dev.readback(), gold[ka + "_rgba8"])
    assert dev.graph_info()[0] == per + 2  # tracescreen re-captured per shard (a prepass graph is reused)
    # Terrain.reload + swap: new shaders, new graphs
    assert ter.reload()
    ter.render_device()
    assert np.array_equal(dev.readback(), gold[ka + "_rgba8"])
    assert dev.graph_info()[0] >= per + 3  # (a key equal in every baked pointer may reuse a graph)
    dev.destroy()


def test_frame_ring_graphs_bitexact():
    import gpgpuraytrace_amd as G
    gold = GI.load()
    spec = GI.FRAMES[1]
    land, pose, w, h, aa, ms, ao = GI.unpack(spec)
    cam = FixedCamera(GI.consts(w, h, pose))
    ring = G.FrameRing(w, h, depth=3, camera=cam, graph=True)
    for _, ter in ring.slots:
        ter.set_time_of_day_vec(cam.c["sun"])
    for _ in range(7):
        ring.render()
    ring.synchronize()
    for dev, _ in ring.slots:
        assert np.array_equal(dev.readback(), gold[GI.frame_key(*spec) + "_rgba8"])
        assert dev.graph_info()[0] == _graphs_per_render(dev)
    ring.destroy()


# --- frame batches (rt_terrain_render_batch) ----------------------------------------------
def _batch(specs, stats=False, graph=False):
    """One (Device, Terrain) per spec, made as the single-frame tests make them."""
    out = []
    for spec in specs:
        land, pose, w, h, aa, ms, ao = GI.unpack(spec)
        out.append(make(GI.consts(w, h, pose), land=land, aa=aa, max_steps=ms, stats=stats, ao=ao, graph=graph))
    return out


def _check_frames(frames, specs):
    gold = GI.load()
    for (dev, _), spec in zip(frames, specs):
        key = GI.frame_key(*spec)
        assert bits_equal(dev.readback_float(), gold[key + "_rgba32f"]), key
        assert np.array_equal(dev.readback(), gold[key + "_rgba8"]), key


@pytest.mark.parametrize("n", [2, 3, 5, 8, 17, 24])
def test_batch_mixed_cameras_bitexact(n):
    """n frames of two cameras in one batch (hits and long rays of different frames share
    the kernel's shading batches and rings): every frame equals its golden frame, and the
    batch's stats are the sum of the frames' oracle counts."""
    from gpgpuraytrace_amd import engine as E
    specs = [GI.FRAMES[i % 2] for i in range(n)]  # nomadplains 64x48 reset / lookdown
    frames = _batch(specs, stats=True)
    E.render_batch([t for _, t in frames])
    _check_frames(frames, specs)
    st = frames[0][0].stats()
    gold = GI.load()
    ref = sum(gold[GI.frame_key(*s) + "_stats"].astype(np.int64) for s in specs)
    prepass = sum(gold[GI.frame_key(*s) + "_stats"][1] for s in specs)
    assert (st["noise_calls"], st["primary_steps"], st["shadow_steps"], st["hits"], st["prepass_steps"]) == \
        (ref[0], ref[2], ref[3], ref[5], prepass)
    for d, _ in frames:
        d.destroy()


@pytest.mark.parametrize("idx", [2, 3, 4, 6, 7, 8, 9, 10, 11, 12], ids=lambda i: GI.frame_key(*GI.FRAMES[i]))
def test_batch_every_landscape_and_macro_set(idx):
    """Three frames of one spec per batch: AA 4/8/16, step cap, the other landscapes (greenrocks'
    fog), AO 1/2/4."""
    from gpgpuraytrace_amd import engine as E
    specs = [GI.FRAMES[idx]] * 3
    frames = _batch(specs)
    E.render_batch([t for _, t in frames])
    _check_frames(frames, specs)
    for d, _ in frames:
        d.destroy()


def test_batch_shards_graphs_and_ring():
    """Batches of 2 frames on 2 tile shards, replayed from graphs, assemble to the golden
    frames; FrameRing(batch=3) over 2 slot groups."""
    import torch

    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E
    specs = [GI.FRAMES[0], GI.FRAMES[1]]
    ranks = [_batch(specs, graph=True) for _ in range(2)]
    bufs = {}
    for _ in range(2):  # second pass: graph replay
        for r, frames in enumerate(ranks):
            E.render_batch([t for _, t in frames], r, 2)
            for f, (d, _) in enumerate(frames):
                # frame f of a batch traces shard (r + f) % 2 (the per-frame rotation)
                bufs[r, f] = torch.zeros(E.shard_bytes(d, (r + f) % 2, 2), dtype=torch.uint8, device="cuda:0")
                torch.cuda.synchronize()  # the fill (torch's stream) before the device's stream
                E.shard_pack(d, (r + f) % 2, 2, bufs[r, f].data_ptr())
                d.synchronize()
        for f, (d, _) in enumerate(ranks[0]):
            E.shard_unpack(d, (1 + f) % 2, 2, bufs[1, f].data_ptr())
        for (d, _), spec in zip(ranks[0], specs):  # the shard transport moves the RGBA8 frame
            assert np.array_equal(d.readback(), GI.load()[GI.frame_key(*spec) + "_rgba8"])
    per = _graphs_per_render(ranks[0][0][0])
    assert ranks[0][0][0].graph_info() == (per, 2 * per)
    for frames in ranks:
        for d, _ in frames:
            d.destroy()
    cam = FixedCamera(GI.consts(64, 48, "lookdown"))
    ring = G.FrameRing(64, 48, depth=2, batch=3, camera=cam)
    for _, ter in ring.slots:
        ter.set_time_of_day_vec(cam.c["sun"])
    for _ in range(3):
        ring.render_batch()
    ring.synchronize()
    for dev, _ in ring.slots:
        assert np.array_equal(dev.readback(), GI.load()[GI.frame_key(*GI.FRAMES[1]) + "_rgba8"])
    ring.destroy()


@pytest.mark.parametrize("w,h,world,split", [(64, 48, 3, True), (64, 48, 3, False), (50, 36, 3, True),
                                             (64, 48, 2, True)])
def test_batch_ragged_rotated_shards_bitexact(w, h, world, split):
    """bench.py's N>1 batch on one GPU, following parallel.BatchPlan: 3-frame batches whose tile
    count is not a multiple of N (64x48 and 50x36: 4 tiles, shards of 2/1/1), so rotated frames
    trace shards smaller than the launch's unit count and the trailing units map past the tile
    range.  Each rank runs its prepass range (split) into its slice of a shared CameraResults
    buffer (what the all-gather produces) and traces from it, or renders the whole batch
    (unsplit); packs frame f's shard (r + f) % N at the plan's offsets; rank 0 unpacks every
    other rank's frames.  Every assembled frame equals its golden frame."""
    import torch

    from gpgpuraytrace_amd import engine as E
    from gpgpuraytrace_amd import parallel as P
    specs = [("nomadplains", "reset", w, h, 1, 0), ("nomadplains", "lookdown", w, h, 1, 0),
             ("nomadplains", "reset", w, h, 1, 0)]
    gold = GI.load()
    have = all(GI.frame_key(*s) + "_rgba8" in gold for s in specs)
    consts = {p: GI.consts(w, h, p) if have else _consts_1080p_like(w, h, p) for p in ("reset", "lookdown")}
    # 50x36 has no golden frame: the oracle renders the reference frames here
    want = {p: gold[GI.frame_key("nomadplains", p, w, h, 1, 0) + "_rgba8"] if have
            else O.render(O.noise_tables(), O.make_frame(consts[p]))["rgba8"] for p in consts}
    plan = P.BatchPlan(w, h, len(specs), world, split_prepass=split)
    ranks = [[make(consts[s[1]]) for s in specs] for _ in range(world)]
    cams = torch.full((plan.camera_floats(),), float("nan"), dtype=torch.float32, device="cuda:0")
    packed = [torch.zeros(plan.packed_bytes(), dtype=torch.uint8, device="cuda:0") for _ in range(world)]
    # the fills run on torch's stream; the devices' streams are non-blocking (no implicit order)
    torch.cuda.synchronize()
    if split:
        for r, frames in enumerate(ranks):
            first, count = plan.prepass_range(r)
            # frame f's CameraResults land at f * 16 KiB: rank r's frames fill its plan.camera_slice(r)
            E.prepass_batch([t for _, t in frames], first, count, cams.data_ptr())
        # every rank's prepass is complete before any rank traces (bench.py: the all-gather); a
        # rank's trace reads the other ranks' frames' CameraResults
        for frames in ranks:
            for d, _ in frames:
                d.synchronize()
    for r, frames in enumerate(ranks):
        ters = [t for _, t in frames]
        if split:
            E.trace_batch(ters, r, world, cams.data_ptr())
        else:
            E.render_batch(ters, r, world)
        items = plan.packs(r)  # one rt_shard_pack_batch launch, as bench.py's run_batch does
        E.shard_pack_batch([frames[f][0] for f, _, _ in items], [s for _, s, _ in items], world,
                           [packed[r].data_ptr() + off for _, _, off in items])
        for d, _ in frames:
            d.synchronize()
    items = plan.unpacks()
    E.shard_unpack_batch([ranks[0][f][0] for _, f, _, _ in items], [s for _, _, s, _ in items], world,
                         [packed[src].data_ptr() + off for src, _, _, off in items])
    for (d, _), s in zip(ranks[0], specs):
        assert np.array_equal(d.readback(), want[s[1]]), s
    for frames in ranks:
        for d, _ in frames:
            d.destroy()


@pytest.mark.parametrize("world", [2, 8])
def test_c4_sharded_batch_1080p_assembles_whole_frames(world):
    """BASELINE configs[3] (C4: 1920x1080 tiled over 2/4/8 GPUs, RCCL gather) emulated on one GPU
    at full size with the C3 settings (512-step cap, shadow, 1 AO): N ranks each trace their
    rotated shard (r + f) % N of every frame of a 4-frame batch mixing both poses
    (rt_terrain_render_batch), pack it at the plan's offsets (rt_shard_pack_batch); rank 0 unpacks
    every other rank's frames (rt_shard_unpack_batch), exactly bench.py's run_batch at N > 1 with
    the gather's copy done by hand.  Every assembled RGBA8 frame equals the whole-frame render of
    its pose (itself checked against the oracle by test_baseline_config_rows_bitexact)."""
    import torch

    from gpgpuraytrace_amd import engine as E
    from gpgpuraytrace_amd import parallel as P
    poses = ["reset", "lookdown", "reset", "lookdown"]
    want = {}
    for pose in ("reset", "lookdown"):
        dev, ter = make(GI.consts(1920, 1080, pose), max_steps=512, ao=1)
        ter.render_device()
        want[pose] = dev.readback()
        dev.destroy()
    plan = P.BatchPlan(1920, 1080, len(poses), world)
    ranks = [[make(GI.consts(1920, 1080, pose), max_steps=512, ao=1) for pose in poses] for _ in range(world)]
    packed = [torch.zeros(plan.packed_bytes(), dtype=torch.uint8, device="cuda:0") for _ in range(world)]
    torch.cuda.synchronize()  # the fills (torch's stream) before the devices' non-blocking streams
    for r, frames in enumerate(ranks):
        E.render_batch([t for _, t in frames], r, world)
        items = plan.packs(r)
        E.shard_pack_batch([frames[f][0] for f, _, _ in items], [s for _, s, _ in items], world,
                           [packed[r].data_ptr() + off for _, _, off in items])
        for d, _ in frames:
            d.synchronize()
    items = plan.unpacks()
    E.shard_unpack_batch([ranks[0][f][0] for _, f, _, _ in items], [s for _, _, s, _ in items], world,
                         [packed[src].data_ptr() + off for src, _, _, off in items])
    for f, ((d, _), pose) in enumerate(zip(ranks[0], poses)):
        got = d.readback()
        assert np.array_equal(got, want[pose]), (world, f, pose, int((got != want[pose]).any(-1).sum()))
    for frames in ranks:
        for d, _ in frames:
            d.destroy()


def test_batch_split_prepass_bitexact():
    """rt_terrain_prepass_batch in three ranks' shares into one buffer (what the all-gather
    produces), then rt_terrain_trace_batch from it: the golden frames, and every frame's
    CameraResults array holds its golden prepass."""
    import torch

    from gpgpuraytrace_amd import engine as E
    specs = [GI.FRAMES[i % 2] for i in range(5)]
    frames = _batch(specs, stats=True)
    ters = [t for _, t in frames]
    buf = torch.full((len(specs), 1024, 4), float("nan"), dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()  # the fill (torch's stream) before the devices' non-blocking streams
    # (5, 0) and (6, 0): ranks past the last frame (bench.py at N = 8 with 12-frame batches)
    for first, count in ((0, 2), (2, 2), (4, 1), (5, 0), (6, 0)):
        E.prepass_batch(ters, first, count, buf.data_ptr())
    E.trace_batch(ters, 0, 1, buf.data_ptr())
    _check_frames(frames, specs)
    gold = GI.load()
    for (d, t), spec in zip(frames, specs):
        t.get_camera_results()
        assert np.array_equal(t.camera_view, gold[GI.frame_key(*spec) + "_camera_results"])
    st = frames[0][0].stats()
    assert st["prepass_steps"] == sum(gold[GI.frame_key(*s) + "_stats"][1] for s in specs)
    for d, _ in frames:
        d.destroy()


@pytest.mark.parametrize("ao,ms", [(1, 512), (0, 0)], ids=["c3", "ref"])
def test_batch_1080p_equals_single_frames(ao, ms):
    """Full-size frames (the bench's workload, overflow lists in use): a 3-frame batch mixing
    the reset and look-down poses equals the same frames rendered one at a time, pixel for
    pixel, and the batch's counts are the sum of theirs."""
    from gpgpuraytrace_amd import engine as E
    poses = ["reset", "lookdown", "reset"]
    singles, ref_stats = [], []
    for pose in poses:
        dev, ter = make(GI.consts(1920, 1080, pose), max_steps=ms, ao=ao, stats=True)
        ter.render_device()
        singles.append((dev.readback_float(), dev.readback()))
        ref_stats.append(dev.stats())
        dev.destroy()
    frames = [make(GI.consts(1920, 1080, pose), max_steps=ms, ao=ao, stats=True) for pose in poses]
    E.render_batch([t for _, t in frames])
    for (dev, _), (f32, f8) in zip(frames, singles):
        assert bits_equal(dev.readback_float(), f32)
        assert np.array_equal(dev.readback(), f8)
    st = frames[0][0].stats()
    for key in ("noise_calls", "primary_steps", "shadow_steps", "ao_steps", "hits", "prepass_steps"):
        assert st[key] == sum(r[key] for r in ref_stats), key
    for d, _ in frames:
        d.destroy()


@pytest.mark.parametrize("ao", [0, 1])
def test_edge_scenes_all_sky_and_eye_in_terrain(ao):
    """Degenerate frames, single and batched (64x48, C3 step cap): a camera pitched up (every
    prepass ray and every pixel misses: no hit records, no long rays, an all-zero hit ballot for
    k_finish) and eyes inside the terrain at y = 30 and y = 12 (every ray hits within a few steps:
    every pixel goes through the hit stack, shading and shadow / AO rays).  Each frame equals the
    oracle's bit for bit and the march counts equal the oracle's."""
    from gpgpuraytrace_amd import camera
    from gpgpuraytrace_amd import engine as E
    scenes = [camera.frame_constants(64, 48, euler=(-2.0, -4.6, 0.0)),
              camera.frame_constants(64, 48, position=(0.0, 30.0, 0.0)),
              camera.frame_constants(64, 48, position=(0.0, 12.0, 0.0))]
    nz = O.noise_tables()
    refs = [O.render(nz, O.make_frame(c, max_steps=512, ao=ao)) for c in scenes]
    assert refs[0]["stats"]["primary_hits"] == 0 and refs[1]["stats"]["primary_hits"] == 64 * 48
    for c, ref in zip(scenes, refs):
        dev, ter = make(c, max_steps=512, ao=ao, stats=True)
        ter.render_device()
        assert bits_equal(dev.readback_float(), ref["rgba32f"])
        assert np.array_equal(dev.readback(), ref["rgba8"])
        st = dev.stats()
        for key, okey in (("hits", "primary_hits"), ("primary_steps", "primary_steps"),
                          ("shadow_steps", "shadow_steps"), ("prepass_steps", "prepass_steps")):
            assert st[key] == ref["stats"][okey], key
        dev.destroy()
    frames = [make(c, max_steps=512, ao=ao) for c in scenes + scenes[::-1]]
    E.render_batch([t for _, t in frames])
    for (d, _), ref in zip(frames, refs + refs[::-1]):
        assert np.array_equal(d.readback(), ref["rgba8"])
    for d, _ in frames:
        d.destroy()


def test_batch_rejects_mixed_macro_sets():
    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E
    frames = _batch([GI.FRAMES[0]]) + [make(GI.consts(64, 48, "reset"), max_steps=64)]
    with pytest.raises(G.NativeError):
        E.render_batch([t for _, t in frames])
    for d, _ in frames:
        d.destroy()


# --- output path: GPU swizzle + recorder --------------------------
@pytest.mark.parametrize("w,h", [(64, 48), (50, 36)])
def test_bgrx_readback_bitexact(w, h):
    """k_bgrx (rt_device_readback_bgrx) == RecorderWinAPI::write's conversion (oracle) of the
    same frame's RGBA8 readback; odd widths take the per-pixel tail path."""
    import gpgpuraytrace_amd as G
    dev, ter = make(GI.consts(64, 48, "lookdown") if (w, h) == (64, 48) else G.frame_constants(w, h))
    ter.render_device()
    dev.present()
    rgba = dev.readback()
    got = dev.readback_bgrx()
    assert np.array_equal(got, O.bgrx(rgba))
    if (w, h) == (64, 48):
        assert np.array_equal(got, O.bgrx(GI.load()[GI.frame_key(*GI.FRAMES[1]) + "_rgba8"]))
    dev.destroy()


def test_recorder_present_and_write(tmp_path):
    """IRecorder over the raw-video sink: present() while recording writes the GPU-swizzled frame
    with RecorderWinAPI's sample time stamps; write() on host rows gives the same bytes; nothing
    is written when not recording or after Finalize."""
    import gpgpuraytrace_amd as G
    w, h = 64, 48
    dev, ter = make(GI.consts(w, h, "reset"))
    path = str(tmp_path / "out.rgb32")
    rec = G.RecorderFactory.construct(dev, 25, True, path)
    assert rec is not None and not rec.is_recording()
    ter.render_device()
    dev.present()  # not recording: no sample
    rec.start()
    frames = []
    for i in range(3):
        ter.set_time_of_day(0.3 + 0.05 * i)
        ter.render_device()
        dev.present()
        frames.append(dev.readback())
    rec.write(frames[0])  # host path, fixed speed
    info = rec.info()
    assert info["frames"] == 4 and info["frame_duration"] == 400000
    rec.stop()
    assert not rec.is_recording()
    dev.present()  # after stop: no sample
    with pytest.raises(Exception):
        rec.start()  # BeginWriting after Finalize
    rec.destroy()
    vid, samples = G.read_recording(path, w, h)
    assert vid.shape == (4, h, w)
    for i in range(3):
        assert np.array_equal(vid[i], O.bgrx(frames[i]))
    assert np.array_equal(vid[3], vid[0])
    t, d = O.sample_times(25, True, np.zeros(4, np.float32))
    assert samples[:, 0].tolist() == [0, 1, 2, 3]
    assert samples[:, 1].tolist() == t.tolist() and samples[:, 2].tolist() == d.tolist()
    # timer-driven durations (not fixed speed)
    path2 = str(tmp_path / "out2.rgb32")
    rec2 = G.RecorderFactory.construct(dev, 25, False, path2)
    rec2.start()
    fts = np.array([0.04, 0.0333333, 0.1], np.float32)
    for ft in fts:
        rec2.set_frame_time(ft)
        ter.render_device()
        dev.present()
    rec2.stop()
    rec2.destroy()
    _, s2 = G.read_recording(path2, w, h)
    t2, d2 = O.sample_times(25, False, fts)
    assert s2[:, 1].tolist() == t2.tolist() and s2[:, 2].tolist() == d2.tolist()
    dev.destroy()


# --- Flyby fed by the device prepass ------------------------------
def test_fly_through_device_feed_matches_oracle_feed():
    """Flyby steering from the GPU's CameraResults (rt_terrain_render_feed) follows exactly the
    path it follows from the oracle's camerarays, one frame at a time and with 3 frames in flight."""
    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import camera as CAM
    from gpgpuraytrace_amd.flyby import Flyby, fly_through
    W, H, frames, dt = 64, 48, 6, 1.0 / 25.0
    cam = CAM.Camera(W, H)
    dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H)
    ter = G.Terrain(dev, "nomadplains")
    ter.create()
    assert ter.reload()
    ter.set_camera(cam)
    ter.set_time_of_day(0.3)
    ter.update_shaders()
    path_dev = fly_through(ter, cam, frames, dt)
    dev.destroy()
    cam2 = CAM.Camera(W, H)
    ring = G.FrameRing(W, H, depth=3, camera=cam2)
    path_ring = fly_through(ring, cam2, frames, dt)
    ring.destroy()
    nz = O.noise_tables()
    cam3 = CAM.Camera(W, H)
    fly = Flyby(cam3)
    view = np.zeros((1024, 4), np.float32)
    path = []
    for _ in range(frames):
        fly.fly(dt, view)
        cam3.update()
        path.append((cam3.position.copy(), np.asarray(cam3.front, float).copy()))
        fr = O.make_frame(CAM.camera_constants(cam3))
        cr = np.zeros(1024 * 4, np.float32)
        st = O.Stats()
        O.lib().ro_camerarays(C.byref(nz), C.byref(fr), O._fp(cr), C.byref(st))
        view = cr.reshape(1024, 4)
    path = np.array(path)
    assert np.array_equal(path_dev, path)
    assert np.array_equal(path_ring, path)


# --- VariableManager: a live SunDirection tweak reaches the frame ----
def test_variable_manager_live_tweak_changes_frame():
    import socket

    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import camera as CAM
    from gpgpuraytrace_amd import varclient as VC
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    consts = GI.consts(64, 48, "reset")
    G.VariableManager.start(port)
    try:
        dev, ter = make(consts)  # reload: tracescreen then camerarays -> registry cleared again
        assert G.VariableManager.count() == 0  # the reference's order leaves nothing registered
        G.VariableManager.register_compute(ter.compute)
        assert G.VariableManager.count() == 1
        cl = VC.VariableClient("127.0.0.1", port)
        assert cl.poll() == "add"
        assert cl.variables["SunDirection"][0] == "float3"
        assert np.array_equal(cl.value("SunDirection"), np.asarray(consts["sun"], np.float32))
        sun = CAM.sun_direction(0.36)
        cl.send("SunDirection", sun)
        cl.close()
        cl2 = VC.VariableClient("127.0.0.1", port)  # served after the first client is done
        assert cl2.poll() == "add" and np.array_equal(cl2.value("SunDirection"), sun)
        cl2.close()
        ter.render_device()
        dev.present()
        img = dev.readback_float()
        c2 = dict(consts, sun=sun)
        ref = O.render(O.noise_tables(), O.make_frame(c2))
        assert bits_equal(img, ref["rgba32f"])
        dev.destroy()
    finally:
        G.VariableManager.stop()


# --- stream ownership (frosttrace.h rt_device_set_stream / rt_stream_refs, ABI 4) -------------
def test_stream_owner_destroyed_before_borrower():
    """A device borrowing another device's stream keeps it alive: destroying the owner first (the
    order that hung FrameRing.destroy in round 2's multi-rank rehearsals) leaves the borrower a live
    stream it renders a bit-exact frame on, and the stream goes with its last user."""
    import gpgpuraytrace_amd as G
    gold = GI.load()
    key = GI.frame_key("nomadplains", "reset", 64, 48, 1, 0)
    owner, _ = make(GI.consts(64, 48, "reset"))
    dev, ter = make(GI.consts(64, 48, "reset"))
    s = owner.stream()
    assert G.lib().rt_stream_refs(s) == 1
    dev.set_stream(s)
    assert G.lib().rt_stream_refs(s) == 2
    owner.destroy()
    assert G.lib().rt_stream_refs(s) == 1  # the borrower's reference keeps it
    ter.render_device()
    dev.present()
    assert bits_equal(dev.readback_float(), gold[key + "_rgba32f"])
    dev.set_stream(None)  # back to its own stream: the loan ends and the lent stream is destroyed
    assert G.lib().rt_stream_refs(s) == 0
    ter.render_device()
    assert np.array_equal(dev.readback(), gold[key + "_rgba8"])
    dev.destroy()


# --- sky known answers (SURVEY 8c iv; tests/test_sky_kat.py pins the oracle to float64) ----------
@pytest.mark.parametrize("eye_i", [0, 1, 2])
def test_sky_known_answers_device(eye_i):
    """rt_debug_sky: the device's getRayleighMieColor / getSpaceColor at the KAT directions, sun
    angles and eye positions, bit-identical to the oracle (which test_sky_kat.py holds within 1e-4
    of the float64 restatement of sky.hlsl)."""
    import gpgpuraytrace_amd as G
    import test_sky_kat as K
    d = K.directions()
    for t in K.TIMES:
        consts = dict(GI.consts(64, 48, "reset"))
        consts["eye"] = np.array(list(K.EYES[eye_i]) + [1.0], np.float32)
        consts["sun"] = K.sun(t)
        dev, ter = make(consts)
        ter.update_shaders()
        out = np.empty((len(d), 7), np.float32)
        assert G.lib().rt_debug_sky(ter.compute._h, d.ctypes.data, out.ctypes.data, len(d)) == 0
        assert bits_equal(out, O.sky(O.noise_tables(), K.frame(K.EYES[eye_i], t), d))
        dev.destroy()


# --- stream handoff (ABI 6 rt_device_wait_event / rt_device_record_event) -----------------------------
def _hip():
    lib = C.CDLL("libamdhip64.so")
    lib.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    return lib


def test_event_handoff_without_host_sync():
    """A buffer filled on torch's stream (behind a ~20 ms spin kernel, so an unordered reader would
    see the old contents) is handed to a device by event, no host synchronisation: rt_shard_unpack on
    the device stream reads the filled bytes.  The other way, a rendered frame is handed to torch's
    stream by rt_device_record_event and copied there: the golden frame."""
    import torch
    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E
    gold = GI.load()
    key = GI.frame_key("nomadplains", "reset", 64, 48, 1, 0)
    dev, ter = make(GI.consts(64, 48, "reset"))
    n = E.shard_bytes(dev, 0, 1)
    buf = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    pattern = (torch.arange(n, device="cuda:0") % 251).to(torch.uint8)
    torch.cuda._sleep(50_000_000)  # ~20 ms on the torch stream before the fill
    buf.copy_(pattern)
    filled = torch.cuda.Event()
    filled.record(torch.cuda.current_stream())
    dev.wait_event(filled.cuda_event)
    E.shard_unpack(dev, 0, 1, buf.data_ptr())  # tiles -> framebuffer (64x48: 2x2 tiles, partly outside)
    got = dev.readback().view(np.uint32).reshape(48, 64)
    want = np.zeros((48, 64), np.uint32)
    from gpgpuraytrace_amd import parallel as P
    P.unpack_host(want, pattern.cpu().numpy().view(np.uint32), 0, 1)
    assert np.array_equal(got, want)
    # device -> torch: the frame, recorded on the device stream, copied on torch's stream
    torch.cuda.synchronize()
    ter.render_device()
    done = torch.cuda.Event()
    done.record()  # torch creates its events on first record; the device then re-records it on its stream
    dev.record_event(done.cuda_event)
    torch.cuda.current_stream().wait_event(done)
    out = torch.empty(64 * 48 * 4, dtype=torch.uint8, device="cuda:0")
    assert _hip().hipMemcpyAsync(out.data_ptr(), dev.framebuffer_pointer(), out.numel(), 3,
                                 torch.cuda.current_stream().cuda_stream) == 0  # device to device
    assert np.array_equal(out.cpu().numpy().reshape(48, 64, 4), gold[key + "_rgba8"])
    dev.check()
    dev.destroy()


def test_device_flags_retired_and_check():
    """ABI 6: the retired flags 8 and 16 (ABI <= 5 RT_DEVICE_SEG_TAIL_*) and any unknown flag are
    rejected; rt_device_check is RT_OK after frames through the spill rings (no dropped push)."""
    import gpgpuraytrace_amd as G
    h = C.c_void_p()
    for bad in (8, 16, 256, 1 << 20):
        assert G.lib().rt_device_create(0, 64, 48, bad, C.byref(h)) == -1  # RT_ERR_INVALID
    dev, ter = make(GI.consts(64, 48, "lookdown"), small_rings=True, ao=4)
    for _ in range(3):
        ter.render_device()
    dev.check()
    dev.destroy()


def test_graph_ring_phase_marks_readable():
    """bench.py's timed loop on a hipGraph FrameRing (C5's frame loop, 2 slot groups of 2 frames):
    run_batch's phase marks (torch events on each batch's stream) read right after the loop, with no
    graph capture inside it after warm-up and no mark recorded on a capturing stream -- every pair
    readable (round 3 read them after the ring's streams were destroyed and lost C5 marks)."""
    import torch
    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E
    from gpgpuraytrace_amd import parallel as P
    import bench
    gold = GI.load()
    spec = GI.FRAMES[1]
    land, pose, w, h, aa, ms, ao = GI.unpack(spec)
    cam = FixedCamera(GI.consts(w, h, pose))
    ring = G.FrameRing(w, h, depth=2, batch=2, camera=cam, graph=True)
    for _, ter in ring.slots:
        ter.set_time_of_day_vec(cam.c["sun"])
    plan = P.BatchPlan(w, h, 2, 1)

    class Ops:
        def __init__(self):
            self.group = ring.group()

        def render(self):
            E.render_batch([t for _, t in self.group], 0, 1)

        def present(self):
            for d, _ in self.group:
                d.present()

    streams = [torch.cuda.ExternalStream(ring.slots[g * 2][0].stream(), device="cuda:0") for g in range(2)]
    for _ in range(3):  # warm-up: both groups capture their graphs
        P.run_batch(plan, 0, Ops())
        ring.frame += 2
    torch.cuda.synchronize()
    caps = sum(d.graph_info()[0] for d, _ in ring.slots)
    marks, capturing = [], 0
    for _ in range(4):
        g = (ring.frame // 2) % 2
        mk = []

        def mark(name, mk=mk, s=streams[g]):
            nonlocal capturing
            capturing += bench.stream_capturing(s)
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(s)
            mk.append((name, ev))
        P.run_batch(plan, 0, Ops(), mark=mark)
        marks.append(mk)
        ring.frame += 2
    torch.cuda.synchronize()
    assert sum(d.graph_info()[0] for d, _ in ring.slots) == caps  # no capture in the timed loop
    assert capturing == 0
    summary = P.phase_summary(marks, lambda a, b: a.elapsed_time(b))
    assert summary["batches"] == 4 and len(summary["phase_ms"]) == 1 and summary["phase_ms"]["trace"] > 0
    for d, _ in ring.slots:
        assert np.array_equal(d.readback(), gold[GI.frame_key(*spec) + "_rgba8"])
    ring.destroy()


# --- the next batch's prepass fused into this batch's k_trace (FusedPrepass, ABI 6) ----------------
def test_fused_prepass_frame_ring_bitexact():
    """FrameRing(lookahead=True) on RGBA8 devices (the bench's single-frame companion and --lookahead 1):
    each batch's camerarays prepass runs inside the previous batch's k_trace as 8-ray tasks, and its
    k_order waits for the rays.  Over 8 batches of 2 frames, 2 slot groups, cameras alternating per
    batch: every frame equals its golden frame, and the CameraResults / CellDistance the fused prepass
    produced equal the golden ones; rt_device_check reports no flag (no k_order wait timed out)."""
    import gpgpuraytrace_amd as G
    gold = GI.load()
    specs = [GI.FRAMES[0], GI.FRAMES[1]]  # nomadplains 64x48, reset / lookdown
    cams = [(FixedCamera(GI.consts(*GI.unpack(s)[2:4], GI.unpack(s)[1])), GI.frame_key(*s)) for s in specs]
    w, h = cams[0][0].width, cams[0][0].height
    ring = G.FrameRing(w, h, depth=2, batch=2, camera=cams[0][0], lookahead=True)
    for _, ter in ring.slots:
        ter.set_time_of_day_vec(cams[0][0].c["sun"])

    def set_group(g, c):
        for _, ter in ring.slots[g * 2:(g + 1) * 2]:
            ter.set_camera(cams[c][0])
            ter.update_terrain()

    set_group(0, 0)
    for b in range(8):
        if b + 1 < 8:
            set_group((b + 1) % 2, (b + 1) % 2)  # the next batch's cameras before its prepass is staged
        ring.render_batch(ahead=b + 1 < 8)
        if b >= 1:  # the previous batch (the other group) while this one runs
            key = cams[(b - 1) % 2][1]
            for dev, ter in ring.slots[((b - 1) % 2) * 2:((b - 1) % 2 + 1) * 2]:
                assert np.array_equal(dev.readback(), gold[key + "_rgba8"]), (b, key)
    ring.synchronize()
    for dev, ter in ring.slots[2:4]:  # batch 7: group 1, camera 1
        assert np.array_equal(dev.readback(), gold[cams[1][1] + "_rgba8"])
        assert np.array_equal(_device_cells(ter), gold[cams[1][1] + "_cell_distance"])
        ter.get_camera_results()
        assert np.array_equal(ter.camera_view, gold[cams[1][1] + "_camera_results"])
    for dev, ter in ring.slots[0:2]:  # batch 6: group 0, camera 0 (its prepass fused into batch 5's k_trace)
        assert np.array_equal(_device_cells(ter), gold[cams[0][1] + "_cell_distance"])
        ter.get_camera_results()
        assert np.array_equal(ter.camera_view, gold[cams[0][1] + "_camera_results"])
    for dev, _ in ring.slots:
        dev.check()
    ring.destroy()


# --- the gated launch (ABI 7): the prepass inside the trace kernel, units gated on their cells' rays ----------
GATED_SPECS = [GI.FRAMES[0], GI.FRAMES[1], GI.FRAMES[2], GI.FRAMES[3], GI.FRAMES[8], GI.FRAMES[9]]


@pytest.mark.parametrize("float_output", [True, False], ids=["f32", "rgba8"])
@pytest.mark.parametrize("spec", GATED_SPECS, ids=[GI.frame_key(*s) for s in GATED_SPECS])
def test_gated_launch_golden(spec, float_output):
    """With RT_DEVICE_GATED a render of a nomadplains frame is ONE gated launch (rt_device_info): k_trace runs the
    1024 prepass rays as 8-ray tasks, each unit starts once its cells' 5x5 prepass rays have flagged and
    derives its cells' setTargetDepths bracket from them, the frame's last task writes CellDistance.
    The unit order comes from the PREVIOUS CellDistance, poisoned here with NaN / inf / garbage: frames,
    CameraResults and CellDistance still equal the golden ones; a second frame (a real previous order)
    too; and the default device (the prepass as its own launch) gives the same bits."""
    import gpgpuraytrace_amd as G
    gold = GI.load()
    land, pose, w, h, aa, ms, ao = GI.unpack(spec)
    key = GI.frame_key(*spec)
    consts = GI.consts(w, h, pose)
    dev, ter = make(consts, land, aa=aa, max_steps=ms, ao=ao, float_output=float_output, gated=True)
    rng = np.random.default_rng(7)
    junk = rng.uniform(-1e3, 1e3, (1024, 2)).astype(np.float32)
    junk[::7] = np.nan
    junk[3::11, 1] = np.inf
    junk[5::13, 0] = 0.0
    ter.var_cell_distance.write(junk)
    for rep in range(2):
        ter.render_device()
        assert dev.launch_info() == (rep + 1, 0)
        assert np.array_equal(dev.readback(), gold[key + "_rgba8"]), rep
        if float_output:
            assert bits_equal(dev.readback_float(), gold[key + "_rgba32f"]), rep
        assert np.array_equal(_device_cells(ter), gold[key + "_cell_distance"]), rep
        ter.get_camera_results()
        assert np.array_equal(ter.camera_view, gold[key + "_camera_results"]), rep
    dev.check()
    dev.destroy()
    idev = G.DeviceFactory.construct(G.DeviceAPI.HIP, w, h, float_output=float_output)
    iter_ = G.Terrain(idev, land, aa_samples=aa, max_steps=ms, ao_samples=ao)
    iter_.create()
    assert iter_.reload()
    iter_.set_camera(FixedCamera(consts))
    iter_.set_time_of_day_vec(consts["sun"])
    iter_.render_device()
    assert idev.launch_info() == (0, 1)
    assert np.array_equal(idev.readback(), gold[key + "_rgba8"])
    idev.destroy()


def test_gated_launch_c3_batch_rows():
    """The gated launch at full size: a batch of 3 C3 frames (1920x1080, 512-step cap, AO 1; both poses
    and the reset pose moved), the units of 3 x 2040 tiles deferred while 384 prepass tasks march, against
    the oracle on row samples; then as an 8-way rotated shard of one rank (most of the batch's units wait
    for rays of cells it does not trace)."""
    from gpgpuraytrace_amd import engine as E
    W, H = 1920, 1080
    cams = [_consts_1080p_like(W, H, "reset"), _consts_1080p_like(W, H, "lookdown")]
    cams.append(_moved_consts(cams[0], (60.0, -20.0, 35.0)))
    rows = (0, H, 67)
    nz = O.noise_tables()
    refs = []
    for c in cams:
        rgba, rgba8, cr, cd, _ = O.render_rows(nz, O.make_frame(c, max_steps=512, ao=1, rows=rows, threads=0))
        refs.append((rgba8, cr, cd))
    pairs = [make(c, max_steps=512, ao=1, float_output=False, gated=True) for c in cams]
    E.render_batch([t for _, t in pairs])
    for (dev, ter), (rgba8, cr, cd) in zip(pairs, refs):
        img = dev.readback()
        assert np.array_equal(img[0:H:67], rgba8[0:H:67])
        assert np.array_equal(_device_cells(ter), cd)
        ter.get_camera_results()
        assert np.array_equal(ter.camera_view, cr)
    assert pairs[0][0].launch_info() == (1, 0)
    for dev, _ in pairs:
        dev.check()
    # one rank of an 8-way shard: its tiles of every frame against the whole-frame rows
    E.render_batch([t for _, t in pairs], 3, 8)
    tiles_x = (W + 31) // 32
    for f, ((dev, _), (rgba8, _, _)) in enumerate(zip(pairs, refs)):
        img = dev.readback()
        shard = (3 + f) % 8
        for y in range(0, H, 67):
            for tx in range(tiles_x):
                if ((y // 32) * tiles_x + tx) % 8 == shard:
                    x0, x1 = tx * 32, min(W, tx * 32 + 32)
                    assert np.array_equal(img[y, x0:x1], rgba8[y, x0:x1]), (f, y, tx)
    for dev, _ in pairs:
        dev.check()
        dev.destroy()


def _moved_consts(consts, d):
    """The fixture's camera moved by d (eye and ViewInverse's translation row): a third pose whose
    oracle frame the test renders itself."""
    c = dict(consts)
    c["eye"] = np.asarray(consts["eye"], np.float32).copy()
    c["eye"][:3] += np.asarray(d, np.float32)
    vi = np.asarray(consts["view_inverse"], np.float32).copy().reshape(4, 4)
    vi[3, :3] += np.asarray(d, np.float32)
    c["view_inverse"] = vi
    return c


def test_fused_prepass_cameras_change_every_batch():
    """a batch must never trace from its group's PREVIOUS fused CameraResults.  Three cameras
    cycle over two slot groups (group g renders cameras g, g + 2, g + 4, ... mod 3), so every group's
    camera changes from one fused batch to its next; every frame, its CameraResults and CellDistance
    equal the oracle's for that batch's own camera.  (With a fixed camera per group, a k_order that
    passed on the previous round's count would still have matched.)"""
    import gpgpuraytrace_amd as G
    gold = GI.load()
    specs = [GI.FRAMES[0], GI.FRAMES[1]]
    base = [GI.consts(*GI.unpack(s)[2:4], GI.unpack(s)[1]) for s in specs]
    consts = base + [_moved_consts(base[0], (40.0, -30.0, 25.0))]
    refs = [{"rgba8": gold[GI.frame_key(*specs[0]) + "_rgba8"],
             "camera_results": gold[GI.frame_key(*specs[0]) + "_camera_results"],
             "cell_distance": gold[GI.frame_key(*specs[0]) + "_cell_distance"]},
            {"rgba8": gold[GI.frame_key(*specs[1]) + "_rgba8"],
             "camera_results": gold[GI.frame_key(*specs[1]) + "_camera_results"],
             "cell_distance": gold[GI.frame_key(*specs[1]) + "_cell_distance"]}]
    refs.append(O.render(O.noise_tables(), O.make_frame(consts[2])))
    assert not np.array_equal(refs[2]["camera_results"], refs[0]["camera_results"])
    cams = [FixedCamera(c) for c in consts]
    w, h = cams[0].width, cams[0].height
    ring = G.FrameRing(w, h, depth=2, batch=2, camera=cams[0], lookahead=True)
    for _, ter in ring.slots:
        ter.set_time_of_day_vec(cams[0].c["sun"])

    def set_group(g, c):
        for _, ter in ring.slots[g * 2:(g + 1) * 2]:
            ter.set_camera(cams[c])
            ter.update_terrain()

    def check_group(g, c, b, arrays):
        for dev, ter in ring.slots[g * 2:(g + 1) * 2]:
            assert np.array_equal(dev.readback(), refs[c]["rgba8"]), (b, g, c)
            assert np.array_equal(_device_cells(ter), refs[c]["cell_distance"]), (b, g, c)
            if arrays:  # (mid-run, the group's NEXT prepass is already fused into the running trace)
                ter.get_camera_results()
                assert np.array_equal(ter.camera_view, refs[c]["camera_results"]), (b, g, c)

    n = 9
    set_group(0, 0)
    for b in range(n):
        if b + 1 < n:
            set_group((b + 1) % 2, (b + 1) % 3)  # the next batch's camera, before its prepass is staged
        ring.render_batch(ahead=b + 1 < n)
        if b >= 1:  # the previous batch (the other group), while this one runs
            check_group((b - 1) % 2, (b - 1) % 3, b - 1, False)
    ring.synchronize()
    check_group((n - 1) % 2, (n - 1) % 3, n - 1, True)
    check_group((n - 2) % 2, (n - 2) % 3, n - 2, True)
    for dev, _ in ring.slots:
        dev.check()
    ring.destroy()


@pytest.mark.parametrize("recording", [False, True], ids=["plain", "recording"])
def test_fused_prepass_timeout_fails_safe(recording, tmp_path):
    """a batch whose fused prepass never runs (RT_DEVICE_DEBUG_WITHHOLD_FUSE on the
    fusing device) times out in k_order; from then on every call that launches on or reads a device of
    the GPU fails with RT_ERR_STATE (a reference-shaped host that never calls rt_device_check cannot
    read the frame), rt_device_check reports and clears it, and the next frames are bit-exact again.
    recording: a present() right after the trace -- before the asynchronous timeout fired --
    still fails and writes no frame to the recorder's video."""
    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E
    gold = GI.load()
    spec = GI.FRAMES[0]
    consts = GI.consts(*GI.unpack(spec)[2:4], GI.unpack(spec)[1])
    key = GI.frame_key(*spec)
    pairs = [make(consts, float_output=False)]
    a_dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, consts["width"], consts["height"], debug_withhold_fuse=True)
    assert a_dev is not None
    a_ter = G.Terrain(a_dev, "nomadplains")
    a_ter.create()
    assert a_ter.reload()
    a_ter.set_camera(FixedCamera(consts))
    a_ter.set_time_of_day_vec(consts["sun"])
    a_ter.update_shaders()
    b_dev, b_ter = pairs[0]
    E.prepass_ahead([a_ter])   # staged; traced before any other trace: in line
    E.prepass_ahead([b_ter])   # staged, then "fused" into a's trace, which withholds its tasks
    E.trace_ahead([a_ter])
    rec = None
    if recording:
        rec = G.RecorderFactory.construct(b_dev, 25, True, str(tmp_path / "out.rgb32"))
        rec.start()
    E.trace_ahead([b_ter])     # k_order waits 0.5 s for rays no kernel computes, then flags
    if recording:
        with pytest.raises(G.NativeError):
            b_dev.present()    # the recorder's sync sees the flag: no frame written
        assert rec.info()["frames"] == 0
    with pytest.raises(G.NativeError):
        b_dev.synchronize()
    with pytest.raises(G.NativeError):
        b_dev.readback()
    with pytest.raises(G.NativeError):
        a_ter.render_device()  # every device of the GPU refuses until the check
    with pytest.raises(G.NativeError, match="timed out"):
        b_dev.check()
    b_dev.check()              # cleared
    b_ter.render_device()
    assert np.array_equal(b_dev.readback(), gold[key + "_rgba8"])
    if rec is not None:
        b_dev.present()
        assert rec.info()["frames"] == 1
        rec.stop()
        rec.destroy()
    a_dev.destroy()
    b_dev.destroy()


def test_fused_prepass_camera_change_and_partial_batch():
    """A batch whose prepass was already fused into the running k_trace gets a new camera before its own
    trace: it waits for that kernel and prepasses again in line (golden frames of the new camera); a
    partial batch traces from a fused prepass of the full group; a staged batch traced before any other
    trace prepasses in line."""
    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E
    gold = GI.load()
    specs = [GI.FRAMES[0], GI.FRAMES[1]]
    cams = [(FixedCamera(GI.consts(*GI.unpack(s)[2:4], GI.unpack(s)[1])), GI.frame_key(*s)) for s in specs]
    w, h = cams[0][0].width, cams[0][0].height
    ring = G.FrameRing(w, h, depth=2, batch=3, camera=cams[0][0], lookahead=True)
    for _, ter in ring.slots:
        ter.set_time_of_day_vec(cams[0][0].c["sun"])
    g0 = [t for _, t in ring.slots[:3]]
    g1 = [t for _, t in ring.slots[3:]]
    E.prepass_ahead(g0)            # staged, no trace before its own: in line
    E.prepass_ahead(g1)            # staged, then fused into g0's k_trace
    E.trace_ahead(g0)
    for t in g1:                    # a real camera change after the fusing trace was queued
        t.set_camera(cams[1][0])
        t.update_terrain()
    E.trace_ahead(g1)               # waits for g0's k_trace, prepasses again
    ring.synchronize()
    for dev, _ in ring.slots[:3]:
        assert np.array_equal(dev.readback(), gold[cams[0][1] + "_rgba8"])
    for dev, _ in ring.slots[3:]:
        assert np.array_equal(dev.readback(), gold[cams[1][1] + "_rgba8"])
    E.prepass_ahead(g0)            # g0 fused into g1's next trace, traced as a partial batch of 2
    E.trace_ahead(g1)
    E.trace_ahead(g0[:2])
    ring.synchronize()
    for dev, _ in ring.slots[:2]:
        assert np.array_equal(dev.readback(), gold[cams[0][1] + "_rgba8"])
    for dev, _ in ring.slots:
        dev.check()
    ring.destroy()


# --- rt_terrain_render's prepass stream (round 5): frame i+1's prepass in frame i's trace tail ----------------
@pytest.mark.parametrize("pair", [(0, 1), (4, 5)], ids=["nomadplains", "testing"])
def test_render_serial_prepass_stream_frames_in_flight(pair):
    """Frames rendered back to back on ONE device with no host synchronisation, the camera alternating
    between two golden poses: each rt_terrain_render queues its prepass on the device's prepass stream
    behind the previous frame's k_order only (so it overlaps that frame's trace) and its trace behind the
    prepass.  A copy of every frame queued on the device's stream right after it (rt_shard_pack, one shard)
    equals that pose's golden frame, and the last frame's CameraResults and CellDistance equal its golden
    arrays: no prepass overwrote CameraResults before the previous k_order read them."""
    import torch
    from gpgpuraytrace_amd import engine as E
    from gpgpuraytrace_amd import parallel as P
    gold = GI.load()
    specs = [GI.FRAMES[i] for i in pair]
    land, _, w, h, aa, ms, ao = GI.unpack(specs[0])
    cams = [GI.consts(w, h, GI.unpack(s)[1]) for s in specs]
    keys = [GI.frame_key(*s) for s in specs]
    dev, ter = make(cams[0], land, aa=aa, max_steps=ms, ao=ao, float_output=False)
    nbytes = P.shard_bytes(w, h, 0, 1)
    bufs = [torch.zeros(nbytes, dtype=torch.uint8, device="cuda:0") for _ in range(7)]
    torch.cuda.synchronize()
    for k, buf in enumerate(bufs):
        ter.set_camera(FixedCamera(cams[k % 2]))
        ter.update_terrain()
        ter.set_time_of_day_vec(cams[k % 2]["sun"])
        ter.render_device()
        E.shard_pack(dev, 0, 1, buf.data_ptr())
    dev.synchronize()
    assert dev.launch_info() == (0, len(bufs))  # every render ran its prepass launch (the first in line)
    assert dev.prestream_renders() == len(bufs) - 1  # ... and every render after the first on the prepass stream
    for k, buf in enumerate(bufs):
        frame = P.unpack_host(np.zeros((h, w), np.uint32), buf.cpu().numpy().view(np.uint32), 0, 1)
        assert np.array_equal(frame.view(np.uint8).reshape(h, w, 4), gold[keys[k % 2] + "_rgba8"]), k
    last = keys[(len(bufs) - 1) % 2]
    assert np.array_equal(_device_cells(ter), gold[last + "_cell_distance"])
    ter.get_camera_results()
    assert np.array_equal(ter.camera_view, gold[last + "_camera_results"])
    dev.check()
    dev.destroy()


def test_render_wait_event_orders_prepass_stream():
    """rt_device_wait_event orders EVERY later launch of the device, the next rt_terrain_render's
    prepass included.  Frames A (reset pose) and B (look-down, its prepass on the prepass stream) render back
    to back; the caller's stream waits for B (rt_device_record_event), spins ~20 ms, then copies B's
    CameraResults, and hands back by rt_device_wait_event.  Frame C (reset pose) must not prepass into
    CameraResults before that copy: the copy equals B's golden CameraResults, C equals its golden frame, and
    C prepassed in line (the prepass-stream count stays at 1)."""
    import torch
    gold = GI.load()
    specs = [GI.FRAMES[0], GI.FRAMES[1]]
    land, _, w, h, aa, ms, ao = GI.unpack(specs[0])
    cams = [GI.consts(w, h, GI.unpack(s)[1]) for s in specs]
    keys = [GI.frame_key(*s) for s in specs]
    dev, ter = make(cams[0], land, aa=aa, max_steps=ms, ao=ao, float_output=False)
    torch.cuda.synchronize()

    def render(i):
        ter.set_camera(FixedCamera(cams[i]))
        ter.update_terrain()
        ter.set_time_of_day_vec(cams[i]["sun"])
        ter.render_device()

    render(0)
    render(1)
    assert dev.prestream_renders() == 1
    done_b = torch.cuda.Event()
    done_b.record()
    dev.record_event(done_b.cuda_event)
    stream = torch.cuda.current_stream()
    stream.wait_event(done_b)
    torch.cuda._sleep(50_000_000)  # ~20 ms on the caller's stream before it reads CameraResults
    copy = torch.empty(1024 * 16, dtype=torch.uint8, device="cuda:0")
    assert _hip().hipMemcpyAsync(copy.data_ptr(), ter.var_cam_results.device_pointer(), copy.numel(), 3,
                                 stream.cuda_stream) == 0
    read = torch.cuda.Event()
    read.record(stream)
    dev.wait_event(read.cuda_event)
    render(0)
    assert dev.prestream_renders() == 1  # C prepassed in line, behind the caller's event
    got = copy.cpu().numpy().view(np.float32).reshape(1024, 4)
    assert np.array_equal(got, gold[keys[1] + "_camera_results"])
    assert np.array_equal(dev.readback(), gold[keys[0] + "_rgba8"])
    dev.check()
    dev.destroy()



@pytest.mark.parametrize("reserve", [1, 200])
def test_reserve_cus_golden(reserve):
    """rt_device_reserve_cus (ABI 8): the trace kernel launches (CUs - n) persistent blocks, leaving n CUs to
    other streams' kernels (rank 0's receive at N > 1): the same frames bit for bit, at 1 and 200 CUs left out;
    out-of-range counts are rejected."""
    import gpgpuraytrace_amd as G
    gold = GI.load()
    spec = GI.FRAMES[1]
    land, pose, w, h, aa, ms, ao = GI.unpack(spec)
    key = GI.frame_key(*spec)
    dev, ter = make(GI.consts(w, h, pose), land, aa=aa, max_steps=ms, ao=ao)
    for bad in (-1, 1 << 16):
        with pytest.raises(G.NativeError):
            dev.reserve_cus(bad)
    dev.reserve_cus(reserve)
    for _ in range(2):
        ter.render_device()
        assert bits_equal(dev.readback_float(), gold[key + "_rgba32f"])
        assert np.array_equal(dev.readback(), gold[key + "_rgba8"])
    dev.check()
    dev.destroy()


@pytest.mark.parametrize("spec", [GI.FRAMES[0], GI.FRAMES[1]], ids=["reset", "lookdown"])
def test_gated_cells_handoff_l1_warm_late(spec):
    """the gated launch's cross-CU CellDistance hand-off (the frame's last prepass task stores
    it with 8-B sc1 stores, waits, then stores an sc1 flag; units poll the flag and read their cell with 4-B sc1
    loads -- MI355X_MICROARCH.md's first hand-off row) under RT_DEVICE_DEBUG_GATE_STRESS: every trace wave
    first reads the previous CellDistance with plain loads, so the consumers' L1 holds the old lines, and the
    last task stores the new ones ~200 us late.  The previous CellDistance is poisoned; frames, CellDistance and
    CameraResults equal the golden ones, twice (the second over the first's cells)."""
    gold = GI.load()
    land, pose, w, h, aa, ms, ao = GI.unpack(spec)
    key = GI.frame_key(*spec)
    dev, ter = make(GI.consts(w, h, pose), land, aa=aa, max_steps=ms, ao=ao, gated=True, debug_gate_stress=True)
    junk = np.random.default_rng(11).uniform(-1e3, 1e3, (1024, 2)).astype(np.float32)
    ter.var_cell_distance.write(junk)
    for rep in range(2):
        ter.render_device()
        assert dev.launch_info()[0] == rep + 1
        assert bits_equal(dev.readback_float(), gold[key + "_rgba32f"]), rep
        assert np.array_equal(dev.readback(), gold[key + "_rgba8"]), rep
        assert np.array_equal(_device_cells(ter), gold[key + "_cell_distance"]), rep
        ter.get_camera_results()
        assert np.array_equal(ter.camera_view, gold[key + "_camera_results"]), rep
    dev.check()
    dev.destroy()
