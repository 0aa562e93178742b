"""GPU tests of RT_DEVICE_DEFERRED (ABI 9): rt_terrain_render's setTargetDepths + trace launch with the next
rt_terrain_render, whose own frame's prepass runs inside that trace kernel (FusedPrepass on one stream), and
every other call that launches on or reads the device launches a pending frame first.  Bar: the same bits as
the golden frames / the oracle, for every frame of a serial loop, whichever call ends the deferral."""
import ctypes as C

import numpy as np
import pytest

import golden_index as GI
from test_gpu_parity import FixedCamera, _config_rows, _device_cells, _hip, make

pytestmark = pytest.mark.gpu

# the one-frame deferral at every frame size (RT_DEVICE_DEBUG_DEFER_SMALL): without it a device under 1280x720
# pixels renders as without RT_DEVICE_DEFERRED at one frame to a launch (test_deferred_small_frames_serial)
DEFER = dict(deferred=True, debug_defer_small=True)


def _pose(ter, consts):
    ter.set_camera(FixedCamera(consts))
    ter.update_terrain()
    ter.set_time_of_day_vec(consts["sun"])


def _golden_pair(i=0, j=1):
    gold = GI.load()
    specs = [GI.FRAMES[i], GI.FRAMES[j]]
    land, _, w, h, aa, ms, ao = GI.unpack(specs[0])
    cams = [GI.consts(w, h, GI.unpack(s)[1]) for s in specs]
    keys = [GI.frame_key(*s) for s in specs]
    return gold, land, w, h, aa, ms, ao, cams, keys


@pytest.mark.parametrize("float_output", [False, True], ids=["rgba8", "rgba32f"])
def test_deferred_serial_frames_golden(float_output):
    """Seven frames back to back on one deferred device, the camera alternating between two golden poses, no
    host synchronisation.  Right after render k returns, frame k-1's trace (with frame k's prepass inside it)
    is on the device's stream: a copy queued there (through the stream and framebuffer pointers taken before
    the loop, so no C-ABI call ends the deferral) holds frame k-1, and equals that pose's golden frame.  The
    last frame comes out through rt_device_readback; its CameraResults and CellDistance equal the golden
    arrays.  Six of the seven prepasses ran fused, one (the first) as its own launch."""
    import torch
    import gpgpuraytrace_amd as G
    gold, land, w, h, aa, ms, ao, cams, keys = _golden_pair()
    dev, ter = make(cams[0], land, aa=aa, max_steps=ms, ao=ao, float_output=float_output, **DEFER)
    stream = G.lib().rt_device_stream(dev._h)
    fb = G.lib().rt_device_framebuffer(dev._h)
    assert stream and fb
    n = 7
    bufs = [torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda:0") for _ in range(n - 1)]
    torch.cuda.synchronize()
    hip = _hip()
    for k in range(n):
        _pose(ter, cams[k % 2])
        ter.render_device()
        if k >= 1:
            assert hip.hipMemcpyAsync(bufs[k - 1].data_ptr(), fb, w * h * 4, 3, stream) == 0
    last = dev.readback()
    assert dev.deferred_fused() == n - 1
    assert dev.launch_info() == (0, 1)
    for k, buf in enumerate(bufs):
        got = buf.cpu().numpy().reshape(h, w, 4)
        assert np.array_equal(got, gold[keys[k % 2] + "_rgba8"]), k
    kl = keys[(n - 1) % 2]
    assert np.array_equal(last, gold[kl + "_rgba8"])
    if float_output:
        f32 = dev.readback_float()
        assert np.array_equal(f32.view(np.uint32), gold[kl + "_rgba32f"].view(np.uint32))
    assert np.array_equal(_device_cells(ter), gold[kl + "_cell_distance"])
    ter.get_camera_results()
    assert np.array_equal(ter.camera_view, gold[kl + "_camera_results"])
    dev.check()
    dev.destroy()


def test_deferred_flush_points():
    """Each way a pending frame is launched: a readback, rt_device_synchronize, a map of CameraResults, an
    event recorded for the caller's stream, rt_device_flush, a render of another kind, and the device's
    destruction.  Every frame read equals its pose's golden frame; renders that followed a pending frame fused
    their prepass into its trace, the others launched their own."""
    import torch
    import gpgpuraytrace_amd as G
    gold, land, w, h, aa, ms, ao, cams, keys = _golden_pair()
    dev, ter = make(cams[0], land, aa=aa, max_steps=ms, ao=ao, float_output=False, **DEFER)
    A, B = 0, 1

    def render(i):
        _pose(ter, cams[i])
        ter.render_device()

    render(A)
    assert np.array_equal(dev.readback(), gold[keys[A] + "_rgba8"])     # readback
    assert dev.deferred_fused() == 0
    render(B)
    render(A)
    dev.synchronize()                                                   # synchronize
    assert dev.deferred_fused() == 1
    assert np.array_equal(dev.readback(), gold[keys[A] + "_rgba8"])
    render(B)
    ter.get_camera_results()                                            # map of CameraResults
    assert np.array_equal(ter.camera_view, gold[keys[B] + "_camera_results"])
    assert np.array_equal(dev.readback(), gold[keys[B] + "_rgba8"])
    render(A)
    ev = torch.cuda.Event()
    ev.record()  # (torch creates the HIP event at its first record)
    dev.record_event(ev.cuda_event)                                     # an event for the caller's stream
    stream = torch.cuda.current_stream()
    stream.wait_event(ev)
    fb = torch.empty(w * h * 4, dtype=torch.uint8, device="cuda:0")
    assert _hip().hipMemcpyAsync(fb.data_ptr(), G.lib().rt_device_framebuffer(dev._h), fb.numel(), 3,
                                 stream.cuda_stream) == 0
    assert np.array_equal(fb.cpu().numpy().reshape(h, w, 4), gold[keys[A] + "_rgba8"])
    render(B)
    render(A)
    dev.flush()                                                         # rt_device_flush
    assert dev.deferred_fused() == 2
    assert np.array_equal(dev.readback(), gold[keys[A] + "_rgba8"])
    render(B)
    ter.render_device(feed=True)                                        # a render of another kind
    ter.camera_feed()
    assert np.array_equal(dev.readback(), gold[keys[B] + "_rgba8"])
    assert dev.deferred_fused() == 2
    render(A)
    dev.check()                                                         # rt_device_check launches it too
    assert np.array_equal(dev.readback(), gold[keys[A] + "_rgba8"])
    render(B)
    render(A)
    dev.destroy()                                                       # destruction with a frame pending


def test_deferred_other_landscape_renders_in_line():
    """A landscape whose trace kernel has no fused prepass (testing): a deferred device renders every frame in
    line (a flush, then the full render), so each frame is complete when the call returns."""
    gold, land, w, h, aa, ms, ao, cams, keys = _golden_pair(4, 5)
    dev, ter = make(cams[0], land, aa=aa, max_steps=ms, ao=ao, float_output=False, **DEFER)
    for k in range(3):
        _pose(ter, cams[k % 2])
        ter.render_device()
    assert np.array_equal(dev.readback(), gold[keys[0] + "_rgba8"])
    assert dev.deferred_fused() == 0 and dev.launch_info() == (0, 3)
    dev.destroy()


def test_deferred_small_frames_serial():
    """A deferred device under 1280x720 pixels at one frame to a launch (the product setting, no
    RT_DEVICE_DEBUG_DEFER_SMALL) renders as a plain device: no prepass fused, every render after the first with
    its prepass on the prepass stream.  Five frames alternating between two golden poses, each read back equal to
    its golden frame, then two frames to a launch (fused) and back to one (serial again)."""
    gold, land, w, h, aa, ms, ao, cams, keys = _golden_pair()
    assert w * h < 1280 * 720
    dev, ter = make(cams[0], land, aa=aa, max_steps=ms, ao=ao, float_output=False, deferred=True)
    for k in range(5):
        _pose(ter, cams[k % 2])
        ter.render_device()
        if k % 2:
            assert np.array_equal(dev.readback(), gold[keys[1] + "_rgba8"]), k
    assert np.array_equal(dev.readback(), gold[keys[0] + "_rgba8"])
    assert dev.deferred_fused() == 0
    assert dev.launch_info() == (0, 5) and dev.prestream_renders() == 4
    dev.defer_batch(2)
    for k in range(3):
        _pose(ter, cams[k % 2])
        ter.render_device()
    assert np.array_equal(dev.readback(), gold[keys[0] + "_rgba8"])
    assert dev.deferred_fused() == 1
    dev.defer_batch(1)
    for k in range(3):
        _pose(ter, cams[(k + 1) % 2])
        ter.render_device()
    assert np.array_equal(dev.readback(), gold[keys[1] + "_rgba8"])
    assert dev.deferred_fused() == 1 and dev.prestream_renders() == 6  # (the first after the batch: in line)
    ter.get_camera_results()
    assert np.array_equal(ter.camera_view, gold[keys[1] + "_camera_results"])
    assert np.array_equal(_device_cells(ter), gold[keys[1] + "_cell_distance"])
    dev.check()
    dev.destroy()


def test_deferred_c3_rows_bitexact():
    """BASELINE C3 at full size (1920x1080, 512-step cap, 1 AO ray, RGBA8 device) on a deferred device: the
    look-down frame, then the reset frame whose prepass runs inside the look-down frame's trace.  The
    look-down frame (copied on the device's stream right after the second render) and the reset frame (read
    back) are UNORM8-bit-exact against the oracle's row sample; the reset frame's CameraResults and
    CellDistance are exact."""
    import torch
    import gpgpuraytrace_amd as G
    c_ld, (_, ref8_ld, _, _, _), rows = _config_rows("c3", "lookdown", 5)
    c_rs, (_, ref8_rs, cr_rs, cd_rs, _), _ = _config_rows("c3", "reset", 5)
    w, h = c_rs["width"], c_rs["height"]
    dev, ter = make(c_ld, max_steps=512, ao=1, float_output=False, deferred=True)
    stream, fb = G.lib().rt_device_stream(dev._h), G.lib().rt_device_framebuffer(dev._h)
    buf = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    ter.render_device()
    _pose(ter, c_rs)
    ter.render_device()
    assert _hip().hipMemcpyAsync(buf.data_ptr(), fb, w * h * 4, 3, stream) == 0
    img8 = dev.readback()
    assert dev.deferred_fused() == 1
    ld = buf.cpu().numpy().reshape(h, w, 4)
    assert np.array_equal(ld[rows], ref8_ld[rows])
    assert np.array_equal(img8[rows], ref8_rs[rows])
    assert np.all(img8[..., 3] == 255) and np.all(ld[..., 3] == 255)
    assert np.array_equal(_device_cells(ter), cd_rs)
    ter.get_camera_results()
    assert np.array_equal(ter.camera_view, cr_rs)
    dev.destroy()


@pytest.mark.parametrize("k", [2, 3])
def test_deferred_batch_sequences_golden(k):
    """rt_device_defer_batch(k): frames queue in the device's frame slots and trace k to a launch, each group's
    prepasses inside the previous group's trace.  For every sequence length L = 1 .. 2k+1 (so the last frame
    sits at every position of a group, its prepass standalone or fused, its trace alone or beside other frames),
    L renders with the camera alternating between two golden poses, then a readback: the last frame's RGBA8
    frame, CameraResults and CellDistance equal its pose's golden arrays.  All but the first k frames of a
    sequence prepass inside a trace; each sequence launches one prepass of its own."""
    gold, land, w, h, aa, ms, ao, cams, keys = _golden_pair()
    dev, ter = make(cams[0], land, aa=aa, max_steps=ms, ao=ao, float_output=False, **DEFER)
    dev.defer_batch(k)
    fused = 0
    for L in range(1, 2 * k + 2):
        for i in range(L):
            _pose(ter, cams[(L - 1 - i) % 2])  # the last frame is pose 0
            ter.render_device()
        assert np.array_equal(dev.readback(), gold[keys[0] + "_rgba8"]), L
        fused += max(0, L - k)
        assert dev.deferred_fused() == fused, L
        assert np.array_equal(_device_cells(ter), gold[keys[0] + "_cell_distance"]), L
        ter.get_camera_results()
        assert np.array_equal(ter.camera_view, gold[keys[0] + "_camera_results"]), L
    assert dev.launch_info() == (0, 2 * k + 1)
    dev.defer_batch(1)
    _pose(ter, cams[1])
    ter.render_device()
    assert np.array_equal(dev.readback(), gold[keys[1] + "_rgba8"])
    dev.check()
    dev.destroy()


def test_deferred_batch_c3_rows_bitexact():
    """BASELINE C3 at full size on a deferred device tracing 2 frames to a launch: look-down, reset, look-down,
    reset, then a readback.  The last reset frame (its prepass inside the first pair's trace, its trace beside
    the third frame's) is UNORM8-bit-exact against the oracle's row sample, its CameraResults and CellDistance
    exact."""
    c_ld = _config_rows("c3", "lookdown", 5)[0]
    c_rs, (_, ref8_rs, cr_rs, cd_rs, _), rows = _config_rows("c3", "reset", 5)
    dev, ter = make(c_ld, max_steps=512, ao=1, float_output=False, deferred=True)
    dev.defer_batch(2)
    for c in (c_ld, c_rs, c_ld, c_rs):
        _pose(ter, c)
        ter.render_device()
    img8 = dev.readback()
    assert dev.deferred_fused() == 2
    assert np.array_equal(img8[rows], ref8_rs[rows])
    assert np.all(img8[..., 3] == 255)
    assert np.array_equal(_device_cells(ter), cd_rs)
    ter.get_camera_results()
    assert np.array_equal(ter.camera_view, cr_rs)
    dev.destroy()


def test_deferred_batch_intermediate_frames_golden():
    """Every frame of a deferred-batch sequence, not only the flush's last: 2 frames to a launch, seven frames
    alternating between two golden poses, then a readback.  Frame i takes slot i % 4 (rt_debug_defer_slot), so
    after the flush slots 0 and 1 hold frames 4 and 5, slot 3 frame 3, and slot 2 frame 2's framebuffer and
    CellDistance beside frame 6's CameraResults (the flush's last frame prepasses into its slot, then traces into
    the device's own buffers; frames 2 and 6 share a pose).  Every one equals its pose's golden arrays."""
    import gpgpuraytrace_amd as G
    gold, land, w, h, aa, ms, ao, cams, keys = _golden_pair()
    dev, ter = make(cams[0], land, aa=aa, max_steps=ms, ao=ao, float_output=False, **DEFER)
    dev.defer_batch(2)
    n = 7
    for i in range(n):
        _pose(ter, cams[i % 2])
        ter.render_device()
    assert np.array_equal(dev.readback(), gold[keys[(n - 1) % 2] + "_rgba8"])
    lib = C.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    for slot, frame in ((0, 4), (1, 5), (2, 2), (3, 3)):
        fb, cr, cd = C.c_void_p(), C.c_void_p(), C.c_void_p()
        assert G.lib().rt_debug_defer_slot(dev._h, slot, C.byref(fb), C.byref(cr), C.byref(cd)) == 0
        img = np.empty((h, w, 4), np.uint8)
        cam = np.empty((1024, 4), np.float32)
        cells = np.empty((1024, 2), np.float32)
        for dst, src in ((img, fb), (cam, cr), (cells, cd)):
            assert lib.hipMemcpy(dst.ctypes.data, src, dst.nbytes, 2) == 0
        key = keys[frame % 2]
        assert np.array_equal(img, gold[key + "_rgba8"]), (slot, frame)
        assert np.array_equal(cam, gold[key + "_camera_results"]), (slot, frame)
        assert np.array_equal(cells, gold[key + "_cell_distance"]), (slot, frame)
    assert dev.deferred_fused() == n - 2
    dev.destroy()


@pytest.mark.parametrize("small", [True, False], ids=["fused-small", "serial-small"])
def test_deferred_differential_sequence(small):
    """A seeded random sequence of 60 operations, applied to a plain device and to a deferred one: renders
    with the camera, sun and time changing, readbacks, CameraResults maps, CellDistance reads, flushes,
    synchronisations and changes of the frames traced to a launch (1, 2, 3, 4).  At every observation the
    deferred device shows what the plain device shows, bit for bit (RGBA8 and RGBA32F).  Without
    RT_DEVICE_DEBUG_DEFER_SMALL the small frame's one-frame renders take the serial path (prepass on the prepass
    stream), interleaved with the K >= 2 launches."""
    gold, land, w, h, aa, ms, ao, cams, keys = _golden_pair()
    suns = [np.asarray(cams[0]["sun"], np.float32), np.asarray(cams[1]["sun"], np.float32),
            np.asarray([0.3, 0.8, -0.52], np.float32)]
    dp, tp = make(cams[0], land, aa=aa, max_steps=ms, ao=1, float_output=True)
    dd, td = make(cams[0], land, aa=aa, max_steps=ms, ao=1, float_output=True, deferred=True, debug_defer_small=small)
    rng = np.random.default_rng(7)
    renders = observed = 0
    for step in range(60):
        op = rng.choice(["render"] * 7 + ["readback", "float", "map", "cells", "flush", "sync", "k"])
        if op == "render":
            pose, sun = cams[int(rng.integers(2))], suns[int(rng.integers(3))]
            for ter in (tp, td):
                ter.set_camera(FixedCamera(pose))
                ter.update_terrain(float(rng.integers(4)))
                ter.set_time_of_day_vec(sun)
                ter.render_device()
            renders += 1
        elif renders == 0:
            continue
        elif op == "readback":
            assert np.array_equal(dd.readback(), dp.readback()), step
            observed += 1
        elif op == "float":
            assert np.array_equal(dd.readback_float().view(np.uint32), dp.readback_float().view(np.uint32)), step
            observed += 1
        elif op == "map":
            tp.get_camera_results()
            td.get_camera_results()
            assert np.array_equal(td.camera_view, tp.camera_view), step
            observed += 1
        elif op == "cells":
            assert np.array_equal(_device_cells(td), _device_cells(tp)), step
            observed += 1
        elif op == "flush":
            dd.flush()
        elif op == "sync":
            dd.synchronize()
        else:
            dd.defer_batch(int(rng.integers(1, 5)))
    assert np.array_equal(dd.readback(), dp.readback())
    assert observed >= 8 and renders >= 20, (observed, renders)
    assert dd.deferred_fused() > 0 or not small
    assert small or dd.prestream_renders() > 0
    dd.check()
    dp.destroy()
    dd.destroy()


@pytest.mark.parametrize("k", [1, 2])
def test_deferred_recorder_frames(tmp_path, k):
    """The recorder on a deferred device: present() while recording launches the pending frames first, so every
    recorded frame is the one just rendered.  Four frames alternating between two golden poses, 1 or 2 frames to
    a launch: the video holds the four golden frames in order (the recorder's BGRX rows)."""
    import gpgpuraytrace_amd as G
    import oracle_lib as O
    gold, land, w, h, aa, ms, ao, cams, keys = _golden_pair()
    dev, ter = make(cams[0], land, aa=aa, max_steps=ms, ao=ao, float_output=False, **DEFER)
    dev.defer_batch(k)
    path = str(tmp_path / "out.rgb32")
    rec = G.RecorderFactory.construct(dev, 25, True, path)
    rec.start()
    for i in range(4):
        _pose(ter, cams[i % 2])
        ter.render_device()
        dev.present()
    rec.stop()
    rec.destroy()
    vid, _ = G.read_recording(path, w, h)
    assert vid.shape == (4, h, w)
    for i in range(4):
        assert np.array_equal(vid[i], O.bgrx(gold[keys[i % 2] + "_rgba8"])), i
    dev.destroy()


@pytest.mark.parametrize("k", [1, 2])
@pytest.mark.parametrize("spec", [2, 3, 8, 9, 11, 12, 10], ids=["aa4", "ms64", "ao1", "ms512-ao4", "aa8", "aa16-ao1",
                                                                  "greenrocks-aa2-ao2"])
@pytest.mark.parametrize("float_output", [False, True], ids=["rgba8", "rgba32f"])
def test_deferred_golden_specs(spec, k, float_output):
    """The golden frames of every macro set on a deferred device: AA 4/8/16 (k_finish's per-sample sums), a
    64- and a 512-step cap, 1 and 4 AO rays (fit, fitm), and a landscape without a fused prepass (greenrocks,
    rendered in line).  Three renders of the frame, 1 or 2 to a launch, then a readback: the golden RGBA8 (and
    RGBA32F) frame."""
    gold = GI.load()
    land, pose, w, h, aa, ms, ao = GI.unpack(GI.FRAMES[spec])
    key = GI.frame_key(land, pose, w, h, aa, ms, ao)
    c = GI.consts(w, h, pose)
    dev, ter = make(c, land, aa=aa, max_steps=ms, ao=ao, float_output=float_output, **DEFER)
    dev.defer_batch(k)
    for _ in range(3):
        _pose(ter, c)
        ter.render_device()
    assert np.array_equal(dev.readback(), gold[key + "_rgba8"])
    if float_output:
        assert np.array_equal(dev.readback_float().view(np.uint32), gold[key + "_rgba32f"].view(np.uint32))
    if land == "nomadplains":  # all but the first k frames prepass inside a trace
        assert dev.deferred_fused() == 3 - k
    dev.destroy()


@pytest.mark.parametrize("small", [True, False], ids=["fused-small", "serial-small"])
@pytest.mark.parametrize("k", [1, 2])
def test_deferred_sharded_renders_match_plain(k, small):
    """Sharded renders on a deferred device and on a plain one, the camera alternating: shards 1 and 2 of 3, shard
    7 of 9 (past the 64x48 frame's 6 tiles: no trace kernel, so nothing may be fused into it) and the whole frame.
    Every readback is equal.  A sharded render on a device tracing K >= 2 frames to a launch takes the one-frame
    deferral; without RT_DEVICE_DEBUG_DEFER_SMALL the small frame's one-frame renders (sharded too) take the
    serial path, mixed with the K = 2 batches."""
    gold, land, w, h, aa, ms, ao, cams, keys = _golden_pair()
    dp, tp = make(cams[0], land, aa=aa, max_steps=ms, ao=ao, float_output=False)
    dd, td = make(cams[0], land, aa=aa, max_steps=ms, ao=ao, float_output=False, deferred=True, debug_defer_small=small)
    dd.defer_batch(k)
    for i, (r, n) in enumerate([(1, 3), (2, 3), (1, 3), (7, 9), (0, 1), (2, 3)]):
        for ter in (tp, td):
            _pose(ter, cams[i % 2])
            ter.render_device(r, n)
        if i % 2:
            assert np.array_equal(dd.readback(), dp.readback()), (i, r, n)
    assert np.array_equal(dd.readback(), dp.readback())
    dd.check()
    dp.destroy()
    dd.destroy()
