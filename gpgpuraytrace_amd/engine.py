"""Host-side mirror of the reference engine's dispatch-and-readback surface over
the C-ABI (include/frosttrace.h).

Class/method names follow the reference interfaces so an engine-side caller
reads the same:  DeviceFactory.construct -> Device (IDevice, Factories/IDevice.h),
Device.create_compute -> Compute (ICompute, Factories/ICompute.h), ShaderVariable /
ShaderArray (Graphics/IShaderVariable.h), Texture (Factories/ITexture.h), Noise
(Graphics/Noise.cpp), Terrain (Graphics/Terrain.cpp).  Errors follow the
reference: bool returns / None for missing names; HIP failures raise.
"""
import ctypes as C
import os
import warnings

import numpy as np

from . import _native
from ._native import check, lib

CAMERA_VIEW_RES = 32    # Gameplay/Flyby.h:6
CAMERA_THREAD_RES = 16  # Gameplay/Flyby.h:7


class DeviceAPI:
    NONE, DIRECT3D, OPENGL, HIP = 0, 1, 2, 3   # IDevice.h:5-10 + the HIP slot


def vfs_add_path(path):
    """VFS::addPath (Common/VFS.cpp); "Media/<landscape>" selects the landscape."""
    check(lib().rt_vfs_add_path(path.encode()), "vfs_add_path")


def vfs_clear():
    lib().rt_vfs_clear()


class ShaderVariable:
    """IShaderVariable: write() copies exactly the reflected size into the cbuffer shadow."""

    def __init__(self, handle, compute):
        self._h, self._compute = handle, compute
        self.name = lib().rt_variable_name(handle).decode()
        self.size = int(lib().rt_variable_size(handle))

    def write(self, data):
        buf = bytes(np.ascontiguousarray(data).tobytes() if not isinstance(data, (bytes, bytearray)) else data)
        if len(buf) < self.size:
            raise ValueError(f"{self.name}: need {self.size} bytes, got {len(buf)}")
        check(lib().rt_variable_write(self._h, buf), f"write {self.name}")


class ShaderArray:
    """IShaderArray: create(n), map()/unmap() on UAV arrays, write() on SRV arrays."""

    def __init__(self, handle, compute):
        self._h, self._compute = handle, compute
        self.stride = int(lib().rt_array_stride(handle))
        self.elements = 0

    def create(self, elements):
        rc = lib().rt_array_create(self._h, int(elements))
        if rc == 0:
            self.elements = int(elements)
        return rc == 0

    def map(self):
        """Blocking device->host copy; returns a float32 view (elements x stride/4) or None."""
        p = lib().rt_array_map(self._h)
        if not p:
            return None
        n = self.elements * self.stride // 4
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), shape=(n,)).reshape(self.elements, -1)

    def unmap(self):
        check(lib().rt_array_unmap(self._h), "unmap")

    def write(self, data):
        a = np.ascontiguousarray(data)
        if a.nbytes < self.elements * self.stride:
            raise ValueError("array write smaller than the array")
        return lib().rt_array_write(self._h, a.ctypes.data) == 0

    def device_pointer(self):
        return lib().rt_array_device_pointer(self._h)


class Texture:
    """ITexture over a device allocation."""

    def __init__(self, device):
        h = C.c_void_p()
        check(lib().rt_texture_create(device._h, C.byref(h)), "texture_create")
        self._h = h.value
        self._device = device

    def create(self, dimensions, fmt, width, height, data, binding=0, cpu_flags=0):
        a = np.ascontiguousarray(data)
        return lib().rt_texture_init(self._h, dimensions, fmt, width, height, a.ctypes.data, binding, cpu_flags) == 0

    def __del__(self):
        try:
            if self._h and self._device._h:   # a destroyed device already freed its textures
                lib().rt_texture_destroy(self._h)
        except Exception:
            pass


class Compute:
    """ICompute (Factories/ICompute.h:16-59)."""

    def __init__(self, device):
        self.device = device
        h = C.c_void_p()
        check(lib().rt_compute_create(device._h, C.byref(h)), "compute_create")
        self._h = h.value
        self.thread_size = (0, 0, 0)

    def create(self, directory, file_name, main, thread_size, macros=()):
        names = (C.c_char_p * max(1, len(macros)))(*[k.encode() for k, _ in macros])
        vals = (C.c_char_p * max(1, len(macros)))(*[str(v).encode() for _, v in macros])
        tx, ty, tz = thread_size
        rc = lib().rt_compute_load(self._h, directory.encode(), file_name.encode(), main.encode(), tx, ty, tz,
                                   names, vals, len(macros))
        if rc == 0:
            self.thread_size = (tx, ty, tz)
        return rc == 0

    def swap(self):
        return lib().rt_compute_swap(self._h) == 1

    def run(self, dx, dy, dz=1):
        check(lib().rt_compute_run(self._h, dx, dy, dz), "run")

    def get_variable(self, name):
        h = lib().rt_compute_get_variable(self._h, name.encode())
        return ShaderVariable(h, self) if h else None

    def get_array(self, name):
        h = lib().rt_compute_get_array(self._h, name.encode())
        return ShaderArray(h, self) if h else None

    def get_buffer(self, name):
        return None  # the reference's getBuffer always returns nullptr (ComputeDirect3D.cpp:138-141)

    def set_texture(self, stage, texture):
        check(lib().rt_compute_set_texture(self._h, stage, texture._h if texture else None), "set_texture")

    def get_thread_size(self):
        return self.thread_size

    def __del__(self):
        try:
            if self._h and self.device._h:    # a destroyed device already freed its computes
                lib().rt_compute_destroy(self._h)
        except Exception:
            pass


class Device:
    """IDevice over rt_device (DeviceDirect3D's role)."""

    def __init__(self, width, height, gpu=0, float_output=False, stats=False, graph=False, small_rings=False,
                 debug_withhold_fuse=False, gated=False, debug_gate_stress=False, deferred=False,
                 debug_defer_small=False):
        """small_rings: diagnostic RT_DEVICE_DEBUG_SMALL_RINGS (k_trace's LDS long-ray ring holds 64
        entries and its fin pool 8 slots, so queued long rays take the per-block spill rings and long
        shadows the fin[t] fallback; same bits).  debug_withhold_fuse: diagnostic
        RT_DEVICE_DEBUG_WITHHOLD_FUSE (a trace this device leads runs none of the next batch's fused
        prepass tasks, so that batch's wait times out: the fail-safe's test).  gated:
        RT_DEVICE_GATED (the gated launch: the prepass inside the trace kernel instead of its own launch
        before it; same bits, measured slower).  deferred: RT_DEVICE_DEFERRED (ABI 9; a render's trace
        launches with the next render, which runs its own frame's prepass inside that trace kernel; every
        other call that launches on or reads the device launches a pending frame first; one frame to a launch, a
        device under 1280x720 pixels renders as without it).  debug_defer_small: diagnostic
        RT_DEVICE_DEBUG_DEFER_SMALL (the one-frame deferral at every size, for tests on small frames)."""
        self.width, self.height, self.gpu = int(width), int(height), int(gpu)
        self.flags = ((_native.RT_DEVICE_FLOAT_OUTPUT if float_output else 0) | (_native.RT_DEVICE_STATS if stats else 0)
                      | (_native.RT_DEVICE_GRAPH if graph else 0)
                      | (_native.RT_DEVICE_DEBUG_SMALL_RINGS if small_rings else 0)
                      | (_native.RT_DEVICE_DEBUG_WITHHOLD_FUSE if debug_withhold_fuse else 0)
                      | (_native.RT_DEVICE_GATED if gated else 0)
                      | (_native.RT_DEVICE_DEBUG_GATE_STRESS if debug_gate_stress else 0)
                      | (_native.RT_DEVICE_DEFERRED if deferred else 0)
                      | (_native.RT_DEVICE_DEBUG_DEFER_SMALL if debug_defer_small else 0))
        self._h = None

    def create(self):
        h = C.c_void_p()
        rc = lib().rt_device_create(self.gpu, self.width, self.height, self.flags, C.byref(h))
        if rc != 0:
            return False
        self._h = h.value
        return True

    def present(self):
        check(lib().rt_device_present(self._h), "present")

    def flush(self):
        check(lib().rt_device_flush(self._h), "flush")

    def synchronize(self):
        check(lib().rt_device_synchronize(self._h), "synchronize")

    def create_compute(self):
        return Compute(self)

    def create_texture(self):
        return Texture(self)

    def readback(self):
        out = np.empty((self.height, self.width, 4), np.uint8)
        check(lib().rt_device_readback(self._h, out.ctypes.data, self.width * 4), "readback")
        return out

    def readback_float(self):
        out = np.empty((self.height, self.width, 4), np.float32)
        check(lib().rt_device_readback_float(self._h, out.ctypes.data), "readback_float")
        return out

    def readback_bgrx(self):
        """The recorder's view of the frame: (H, W) uint32 (B, G, R, 0) rows, swizzled on the GPU
        (DeviceDirect3D.cpp:242-256 + RecorderWinAPI.cpp:244-253)."""
        out = np.empty((self.height, self.width), np.uint32)
        check(lib().rt_device_readback_bgrx(self._h, out.ctypes.data, self.width * 4), "readback_bgrx")
        return out

    def stats(self, reset=True):
        s = _native.RtStats()
        check(lib().rt_device_stats_sized(self._h, C.byref(s), C.sizeof(s), 1 if reset else 0), "stats")
        return {n: int(getattr(s, n)) for n, _ in s._fields_}

    def launch_info(self):
        """(gated launches, prepass launches) of the renders this device led (rt_device_info, ABI 7): the
        gated launch runs the prepass inside the trace kernel, a prepass launch is the ABI <= 6 sequence."""
        return self._info((0, 1))

    def prestream_renders(self):
        """Renders whose prepass ran on the device's prepass stream, behind the previous frame's k_order
        (rt_terrain_render with a frame in flight; RT_INFO_PRESTREAM_RENDERS)."""
        return self._info((2,))[0]

    def deferred_fused(self):
        """RT_DEVICE_DEFERRED renders whose prepass ran inside the previous frame's trace kernel
        (RT_INFO_DEFERRED_FUSED, ABI 9)."""
        return self._info((3,))[0]

    def defer_batch(self, frames):
        """rt_device_defer_batch (ABI 9, RT_DEVICE_DEFERRED devices): trace `frames` (1..4) frames to a launch, the
        next group's prepasses inside it; a flush launches all queued frames, the last into the device's buffers."""
        check(lib().rt_device_defer_batch(self._h, int(frames)), "defer_batch")

    def reserve_cus(self, n):
        """rt_device_reserve_cus (ABI 8): this device's trace kernels leave n CUs free for other streams'
        kernels (rank 0's RCCL receive at N > 1)."""
        check(lib().rt_device_reserve_cus(self._h, int(n)), "reserve_cus")

    def _info(self, keys):
        out = []
        for key in keys:
            v = C.c_ulonglong()
            check(lib().rt_device_info(self._h, key, C.byref(v)), "device info")
            out.append(int(v.value))
        return tuple(out)

    def graph_info(self):
        """RT_DEVICE_GRAPH: (graphs captured, graph launches) since creation."""
        cap, lau = C.c_ulonglong(), C.c_ulonglong()
        check(lib().rt_device_graph_info(self._h, C.byref(cap), C.byref(lau)), "graph_info")
        return int(cap.value), int(lau.value)

    def wait_event(self, hip_event):
        """rt_device_wait_event (ABI 6): the device's later work waits for `hip_event` (a hipEvent_t
        handle, e.g. torch.cuda.Event.cuda_event recorded after the caller's fills on its stream)."""
        check(lib().rt_device_wait_event(self._h, int(hip_event)), "wait_event")

    def record_event(self, hip_event):
        """rt_device_record_event (ABI 6): record `hip_event` after the device's queued work (the
        caller's stream then waits for it before reading the device's outputs)."""
        check(lib().rt_device_record_event(self._h, int(hip_event)), "record_event")

    def check(self):
        """rt_device_check (ABI 6): synchronise and raise NativeError if a k_trace queue push was
        dropped at its bound since the last check (never expected: rt_spill_caps)."""
        check(lib().rt_device_check(self._h), "device check")

    def framebuffer_pointer(self):
        return lib().rt_device_framebuffer(self._h)

    def stream(self):
        return lib().rt_device_stream(self._h)

    def set_stream(self, stream_ptr):
        check(lib().rt_device_set_stream(self._h, stream_ptr), "set_stream")

    def destroy(self):
        if self._h:
            lib().rt_device_destroy(self._h)
            self._h = None


class DeviceFactory:
    @staticmethod
    def construct(api, width, height, gpu=0, **kw):
        """DeviceFactory::construct (DeviceFactory.cpp:6-29): nullptr (None) on failure."""
        if api != DeviceAPI.HIP:
            return None
        d = Device(width, height, gpu, **kw)
        return d if d.create() else None


class Recorder:
    """IRecorder / RecorderWinAPI (Factories/IRecorder.h, Adapters/RecorderWinAPI.cpp) over the
    raw-video sink of rt_recorder_create: frames as raw (B, G, R, 0) rows in `path`, sample time
    stamps in `path`.txt.  Attached to its device: Device.present() writes each frame while
    recording, as DeviceDirect3D::present does."""

    def __init__(self, handle, device, path):
        self._h, self.device, self.path = handle, device, path

    def start(self):
        check(lib().rt_recorder_start(self._h), "recorder start")

    def stop(self):
        check(lib().rt_recorder_stop(self._h), "recorder stop")

    def is_recording(self):
        return lib().rt_recorder_is_recording(self._h) == 1

    def set_frame_time(self, seconds):
        """Timer::getConstant() of the next frame (used when not fixed speed)."""
        check(lib().rt_recorder_set_frame_time(self._h, float(seconds)), "recorder frame time")

    def write(self, frame, stride=None):
        """IRecorder::write(frame, stride) with host RGBA8 rows (an (H, W, 4) uint8 array)."""
        a = np.ascontiguousarray(frame)
        check(lib().rt_recorder_write(self._h, a.ctypes.data, int(stride or a.strides[0])), "recorder write")

    def info(self):
        f, t, d = C.c_ulonglong(), C.c_ulonglong(), C.c_ulonglong()
        check(lib().rt_recorder_info(self._h, C.byref(f), C.byref(t), C.byref(d)), "recorder info")
        return {"frames": f.value, "next_sample_time": t.value, "frame_duration": d.value}

    def destroy(self):
        if self._h:
            lib().rt_recorder_destroy(self._h)
            self._h = None


class RecorderFactory:
    @staticmethod
    def construct(device, frame_rate, fixed_speed, path="output.rgb32"):
        """RecorderFactory::construct (RecorderFactory.cpp:6-19): None on failure."""
        h = C.c_void_p()
        if lib().rt_recorder_create(device._h, int(frame_rate), 1 if fixed_speed else 0, path.encode(), C.byref(h)):
            return None
        return Recorder(h.value, device, path)


def read_recording(path, width, height):
    """(frames (F, H, W) uint32 BGRX, samples (F, 3) uint64 [frame, time, duration]) of a recording."""
    raw = np.fromfile(path, np.uint32)
    frames = raw.reshape(-1, height, width)
    rows = [ln.split() for ln in open(path + ".txt") if ln.strip() and not ln.startswith("#")]
    return frames, np.array(rows, np.uint64).reshape(-1, 3)


class VariableManager:
    """Common/VariableManager (the live-tweak TCP server, main.cpp:99 `-m`), native in the runtime:
    start() serves the protocol of varclient.VariableClient on a thread."""

    @staticmethod
    def start(port=10666, bind_address="127.0.0.1"):
        check(lib().rt_varmgr_start(int(port), bind_address.encode()), "variable manager start")

    @staticmethod
    def stop():
        check(lib().rt_varmgr_stop(), "variable manager stop")

    @staticmethod
    def count():
        return int(lib().rt_varmgr_count())

    @staticmethod
    def register_compute(compute):
        check(lib().rt_varmgr_register_compute(compute._h), "variable manager register")


class Noise:
    """Graphics/Noise.cpp:39-94 via rt_noise_generate (seed 300 unless random)."""
    TEXTURE_SIZE = 128
    RAND_MSVC, RAND_GLIBC = 0, 1

    def __init__(self):
        self.permutations2D = None
        self.permutations1D = None

    def generate(self, random=False, seed=None, rand_kind=RAND_MSVC):
        import time
        if seed is None:
            seed = int(time.time()) & 0xFFFFFFFF if random else 300
        p2 = np.empty(128 * 128 * 4, np.uint8)
        g = np.empty(128 * 4, np.float32)
        check(lib().rt_noise_generate(seed, rand_kind, p2.ctypes.data, g.ctypes.data), "noise_generate")
        self.permutations2D, self.permutations1D = p2, g


def set_target_depths_host(camera_results):
    cr = np.ascontiguousarray(camera_results, np.float32).reshape(1024, 4)
    cd = np.empty((1024, 2), np.float32)
    check(lib().rt_terrain_set_target_depths(cr.ctypes.data, cd.ctypes.data), "set_target_depths")
    return cd


class Terrain:
    """Graphics/Terrain.{h,cpp}: creates the two computes, binds variables by name after
    swap, and renders a frame.  render() keeps the reference's call sequence (prepass ->
    CameraResults map/unmap -> host setTargetDepths -> CellDistance write -> tiled runs);
    render_device() is the same frame with the round trip kept on the GPU."""

    def __init__(self, device, theme="nomadplains", record_mode=False, aa_samples=1, max_steps=0,
                 noise_seed=300, rand_kind=Noise.RAND_MSVC, ao_samples=0):
        vfs_add_path("Media/" + theme)  # Terrain.cpp:23
        self.device, self.theme, self.record_mode = device, theme, record_mode
        # max_steps / ao_samples: build extensions (BASELINE configs), 0 = reference semantics
        self.aa_samples, self.max_steps, self.ao_samples = aa_samples, max_steps, ao_samples
        self.noise_seed, self.rand_kind = noise_seed, rand_kind
        self.compute = self.camera_compute = None
        self.camera = None
        self.camera_view = np.zeros((CAMERA_VIEW_RES * CAMERA_VIEW_RES, 4), np.float32)
        self.sun = np.zeros(3, np.float32)

    def create(self):  # Terrain.cpp:69-89
        self.calculate_tile_sizes()
        self.compute = self.device.create_compute()
        self.camera_compute = self.device.create_compute()
        self.noise = Noise()
        self.noise.generate(seed=self.noise_seed, rand_kind=self.rand_kind)
        self.tex_noise_2d = self.device.create_texture()
        ok = self.tex_noise_2d.create(_native.RT_TEXTURE_2D, _native.RT_FORMAT_R8G8B8A8_UINT, 128, 128,
                                      self.noise.permutations2D)
        if not ok:
            raise RuntimeError("texture create failed: " + lib().rt_last_error().decode())

    def reload(self):  # Terrain.cpp:91-103
        macros = [("RECORDING", "1")] if self.record_mode else []
        if self.aa_samples != 1:
            macros.append(("AA_SAMPLES", str(self.aa_samples)))
        if self.max_steps:
            macros.append(("RT_MAX_STEPS", str(self.max_steps)))
        screen_macros = macros + ([("RT_AO_SAMPLES", str(self.ao_samples))] if self.ao_samples else [])
        ok1 = self.compute.create("shaders", "tracescreen.hlsl", "CSMain", (self.thread_x, self.thread_y, 1),
                                  screen_macros)
        ok2 = self.camera_compute.create("shaders", "camerarays.hlsl", "CSMain",
                                         (CAMERA_THREAD_RES, CAMERA_THREAD_RES, 1), macros)
        return ok1 and ok2

    def calculate_tile_sizes(self):  # Terrain.cpp:208-242
        resx, resy = self.device.width, self.device.height
        divisor = 4 if self.record_mode else 1
        tpx, tpy = 1024 // divisor, 512 // divisor
        self.tiles_x = -(-resx // tpx)
        self.tiles_y = -(-resy // tpy)
        self.tile_x, self.tile_y = resx // self.tiles_x, resy // self.tiles_y
        self.thread_x = self.thread_y = 16
        while self.tile_x % self.thread_x:
            self.thread_x += 1
        while self.tile_y % self.thread_y:
            self.thread_y += 1
        self.dispatch_x, self.dispatch_y = self.tile_x // self.thread_x, self.tile_y // self.thread_y

    def set_camera(self, camera):
        self.camera = camera

    def update_shaders(self):  # Terrain.cpp:138-206
        cam = self.camera
        proj = _cbuffer_matrix(cam.projection_hlsl())
        screen = np.array([cam.width, cam.height], np.float32)
        if self.compute.swap():
            self.var_view = self.compute.get_variable("ViewInverse")
            self.var_eye = self.compute.get_variable("Eye")
            self.var_sun = self.compute.get_variable("SunDirection")
            self.var_thread_offset = self.compute.get_variable("ThreadOffset")
            self.var_cell_distance = self.compute.get_array("CellDistance")
            if self.var_cell_distance:
                self.var_cell_distance.create(CAMERA_VIEW_RES * CAMERA_VIEW_RES)
            for name, val in (("Projection", proj), ("ScreenSize", screen), ("permGradients", self.noise.permutations1D)):
                v = self.compute.get_variable(name)
                if v:
                    v.write(val)
            self.compute.set_texture(0, self.tex_noise_2d)
            self._write_frame_vars()
        if self.camera_compute.swap():
            self.var_cam_view = self.camera_compute.get_variable("ViewInverse")
            self.var_cam_eye = self.camera_compute.get_variable("Eye")
            self.var_cam_results = self.camera_compute.get_array("CameraResults")
            if self.var_cam_results:
                self.var_cam_results.create(CAMERA_VIEW_RES * CAMERA_VIEW_RES)
            for name, val in (("Projection", proj), ("ScreenSize", screen), ("permGradients", self.noise.permutations1D)):
                v = self.camera_compute.get_variable(name)
                if v:
                    v.write(val)
            self.camera_compute.set_texture(0, self.tex_noise_2d)
            self._write_frame_vars()

    def _write_frame_vars(self):
        """Variables set before the first dispatch (avoids the frame-1 zero-constant
        artefact of the reference)."""
        if self.camera is None:
            return
        self.update_terrain()
        self.set_time_of_day_vec(self.sun)

    def update_terrain(self, time=0.0):  # Terrain.cpp:302-311
        vinv = _cbuffer_matrix(self.camera.view_inverse_hlsl())
        eye = self.camera.eye()
        for v in (getattr(self, "var_view", None), getattr(self, "var_cam_view", None)):
            if v:
                v.write(vinv)
        for v in (getattr(self, "var_eye", None), getattr(self, "var_cam_eye", None)):
            if v:
                v.write(eye)

    def set_time_of_day(self, time_of_day):  # Terrain.cpp:285-300
        from .camera import sun_direction
        self.set_time_of_day_vec(sun_direction(time_of_day))

    def set_time_of_day_vec(self, sun):
        self.sun = np.asarray(sun, np.float32)
        v = getattr(self, "var_sun", None)
        if v:
            v.write(self.sun)

    def get_camera_results(self):  # Terrain.cpp:441-452
        fd = self.var_cam_results.map()
        if fd is None:
            return
        self.camera_view[:] = fd
        self.var_cam_results.unmap()
        if self.var_cell_distance:
            self.var_cell_distance.write(set_target_depths_host(self.camera_view))

    def render(self):  # Terrain.cpp:105-136 (reference call sequence)
        self.update_shaders()
        n = -(-CAMERA_VIEW_RES // CAMERA_THREAD_RES)
        self.camera_compute.run(n, n, 1)
        self.get_camera_results()
        if self.var_thread_offset:
            for x in range(self.tiles_x):
                for y in range(self.tiles_y):
                    off = np.array([x * self.dispatch_x * self.thread_x, y * self.dispatch_y * self.thread_y], np.uint32)
                    self.var_thread_offset.write(off)
                    self.compute.run(self.dispatch_x, self.dispatch_y, 1)
                    self.device.flush()
        else:
            self.compute.run(self.dispatch_x * self.tiles_x, self.dispatch_y * self.tiles_y, 1)

    def render_device(self, shard_rank=0, shard_count=1, feed=False):
        """Terrain::render with setTargetDepths on the GPU: no host round trip, all on one stream.
        feed=True also sends this frame's CameraResults to the host right after the prepass
        (camera_feed() collects them) -- what Flyby reads, without waiting for the whole frame."""
        self.update_shaders()
        fn = lib().rt_terrain_render_feed if feed else lib().rt_terrain_render
        check(fn(self.camera_compute._h, self.compute._h, shard_rank, shard_count), "terrain_render")

    def camera_feed(self):
        """Wait for the feed of the last render_device(feed=True); it becomes the camera view
        (Terrain::getCameraView, Terrain.cpp:441-452) and is returned, (1024, 4) float32."""
        out = np.empty((CAMERA_VIEW_RES * CAMERA_VIEW_RES, 4), np.float32)
        check(lib().rt_terrain_feed_wait(self.camera_compute._h, out.ctypes.data), "camera feed")
        self.camera_view[:] = out
        return self.camera_view


def render_batch(terrains, shard_rank=0, shard_count=1):
    """rt_terrain_render_batch: Terrain.render_device for up to 24 Terrains at once (RT_MAX_BATCH) (one GPU,
    one resolution, landscape, macro set and noise).  Each frame lands in its own Device's
    framebuffer; the work is enqueued on the first terrain's device stream and the others'
    streams wait for it."""
    n = len(terrains)
    for t in terrains:
        t.update_shaders()
    cams = (C.c_void_p * n)(*[t.camera_compute._h for t in terrains])
    scrs = (C.c_void_p * n)(*[t.compute._h for t in terrains])
    check(lib().rt_terrain_render_batch(cams, scrs, n, shard_rank, shard_count), "terrain_render_batch")


def render_batch_packed(terrains, shard_rank, shard_count, dst_ptr, frame_stride):
    """rt_terrain_render_batch_packed (ABI 7): the batch's shard (frame f traces shard (rank + f) % count)
    with its pixels stored straight into the packed device buffer dst_ptr + f * frame_stride (rt_shard_pack's
    layout) instead of the framebuffers: no pack launch before the gather (RGBA8-only devices)."""
    n, cams, scrs = _batch_handles(terrains)
    check(lib().rt_terrain_render_batch_packed(cams, scrs, n, shard_rank, shard_count, dst_ptr, frame_stride),
          "terrain_render_batch_packed")


def _batch_handles(terrains):
    n = len(terrains)
    for t in terrains:
        t.update_shaders()
    return n, (C.c_void_p * n)(*[t.camera_compute._h for t in terrains]), (C.c_void_p * n)(*[t.compute._h for t in terrains])


def prepass_batch(terrains, first, count, camera_out_ptr):
    """rt_terrain_prepass_batch: the prepass of frames [first, first + count) of the batch, frame
    f's CameraResults to camera_out_ptr + f * 16 KiB (device memory)."""
    n, cams, scrs = _batch_handles(terrains)
    check(lib().rt_terrain_prepass_batch(cams, scrs, n, first, count, camera_out_ptr), "terrain_prepass_batch")


def trace_batch(terrains, shard_rank, shard_count, camera_in_ptr):
    """rt_terrain_trace_batch: setTargetDepths + tracescreen of the batch from gathered
    CameraResults (frame f at camera_in_ptr + f * 16 KiB)."""
    n, cams, scrs = _batch_handles(terrains)
    check(lib().rt_terrain_trace_batch(cams, scrs, n, shard_rank, shard_count, camera_in_ptr), "terrain_trace_batch")


def prepass_ahead(terrains):
    """rt_terrain_prepass_ahead (ABI 5): queue the batch's prepass on the GPU's side stream, after
    the last setTargetDepths of the batches the first terrain's device leads.  Issue it before
    the previous batch's trace_ahead / render_batch; trace_ahead(terrains) consumes it."""
    n, cams, scrs = _batch_handles(terrains)
    check(lib().rt_terrain_prepass_ahead(cams, scrs, n), "terrain_prepass_ahead")


def trace_ahead(terrains, shard_rank=0, shard_count=1):
    """rt_terrain_trace_ahead (ABI 5): setTargetDepths + tracescreen after the batch's ahead
    prepass (the full render_batch when none covers these frames or a camera changed since)."""
    n, cams, scrs = _batch_handles(terrains)
    check(lib().rt_terrain_trace_ahead(cams, scrs, n, shard_rank, shard_count), "terrain_trace_ahead")


def _cbuffer_matrix(m):
    """Bytes of XMMatrixTranspose(M) -- what the engine writes for a float4x4 cbuffer variable."""
    return np.ascontiguousarray(np.asarray(m, np.float32).T)


def shard_bytes(device, rank, count):
    return int(lib().rt_shard_bytes(device._h, rank, count))


def shard_pack(device, rank, count, dst_ptr):
    check(lib().rt_shard_pack(device._h, rank, count, dst_ptr), "shard_pack")


def shard_unpack(device, rank, count, src_ptr):
    check(lib().rt_shard_unpack(device._h, rank, count, src_ptr), "shard_unpack")


def _shard_batch(fn, what, devices, shards, count, ptrs):
    n = len(devices)
    if not (n == len(shards) == len(ptrs)):
        raise ValueError(f"{what}: devices, shards and buffers differ in length")
    if n == 0:
        return
    hs = (C.c_void_p * n)(*[d._h for d in devices])
    ss = (C.c_int * n)(*[int(s) for s in shards])
    ps = (C.c_void_p * n)(*[int(p) for p in ptrs])
    check(fn(hs, ss, count, ps, n), what)


def shard_pack_batch(devices, shards, count, dst_ptrs):
    """rt_shard_pack_batch: device i's shard shards[i] -> dst_ptrs[i], one launch on devices[0]'s stream."""
    _shard_batch(lib().rt_shard_pack_batch, "shard_pack_batch", devices, shards, count, dst_ptrs)


def shard_unpack_batch(devices, shards, count, src_ptrs):
    """rt_shard_unpack_batch: src_ptrs[i] -> device i's shard shards[i], one launch on devices[0]'s stream."""
    _shard_batch(lib().rt_shard_unpack_batch, "shard_unpack_batch", devices, shards, count, src_ptrs)


class FrameRing:
    """Frames in flight: `depth` complete frame contexts (Device + Terrain: own constants,
    CameraResults/CellDistance, ray buffers and framebuffer), each on its own non-blocking HIP
    stream, with frames dealt round-robin.  This is the D3D swap chain's queued frames
    (IDevice::present with a frame-latency queue, DeviceDirect3D.cpp:234-257) made explicit:
    frame i+1's camerarays prepass and primary phase run on the CUs that frame i's ray tail
    leaves idle, instead of waiting for it.  Every frame is still computed in full and
    independently; a slot is reused only after its previous frame (i - depth) has completed on
    that slot's stream.  depth=1 is the reference's one-frame-at-a-time behaviour.
    graph=True: each slot replays its frame as captured hipGraphs (RT_DEVICE_GRAPH).
    batch=B: a slot is B frames rendered by one rt_terrain_render_batch (B devices, the
    batch on the first one's stream); render_batch() queues the next B frames.
    lookahead=True (not with graph): render_batch(ahead=True) also queues the NEXT group's prepass
    on the GPU's side stream before this batch's trace (rt_terrain_prepass_ahead), so it runs
    beside this trace instead of in front of the next one; set the next frames' cameras before
    that call (a camera written after it makes the next batch prepass again, in line)."""

    def __init__(self, width, height, depth=3, gpu=0, theme="nomadplains", camera=None, time_of_day=0.3,
                 graph=False, batch=1, float_output=False, lookahead=False, gated=False, **terrain_kw):
        self.depth, self.frame, self.batch = int(depth), 0, int(batch)
        if lookahead and graph:
            raise ValueError("lookahead runs the prepass on a side stream: not with graph=True")
        self.lookahead, self._ahead = bool(lookahead), set()  # groups with an ahead prepass queued
        # one HIP hardware queue per busy stream: the groups', the side stream, torch's default
        # (DESIGN.md section 7); fewer make two groups share one and their batches serialise
        want = self.depth + 1 + int(self.lookahead)
        try:
            have = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
        except ValueError:
            have = 4
        if self.depth > 1 and have < want:
            warnings.warn(f"FrameRing: {want} busy streams but GPU_MAX_HW_QUEUES={have}; set it to >= {want} "
                          "before HIP starts, or the batches in flight may run one after the other", stacklevel=2)
        self.slots = []
        for _ in range(self.depth * self.batch):
            dev = DeviceFactory.construct(DeviceAPI.HIP, width, height, gpu=gpu, graph=graph,
                                          float_output=float_output, gated=gated)
            if dev is None:
                raise RuntimeError("device create failed: " + lib().rt_last_error().decode())
            ter = Terrain(dev, theme, **terrain_kw)
            ter.create()
            if not ter.reload():
                raise RuntimeError("shader load failed: " + lib().rt_last_error().decode())
            if camera is not None:
                ter.set_camera(camera)
            ter.set_time_of_day(time_of_day)
            ter.update_shaders()
            if len(self.slots) % self.batch:  # a batch's devices share the first one's stream
                dev.set_stream(self.slots[len(self.slots) - len(self.slots) % self.batch][0].stream())
            self.slots.append((dev, ter))

    def next_slot(self):
        return self.slots[self.frame % self.depth]

    def group(self, frames=None):
        """The next slot group (its first `frames` slots, default all `batch`)."""
        g = (self.frame // self.batch) % self.depth
        n = self.batch if frames is None else int(frames)
        if not 1 <= n <= self.batch:
            raise ValueError("frames must be 1..batch")
        return self.slots[g * self.batch:g * self.batch + n]

    def render_batch(self, shard_rank=0, shard_count=1, present=True, frames=None, ahead=True):
        """Queue the next `batch` frames (or the first `frames` of them: a partial batch) as one
        batch on the next slot group; returns their Devices in frame order (each complete once
        its stream reaches this point).  With lookahead, ahead=False skips queueing the next
        group's prepass (the last batch of a run)."""
        group = self.group(frames)
        terrains = [t for _, t in group]
        if not self.lookahead:
            render_batch(terrains, shard_rank, shard_count)
        else:
            g = (self.frame // self.batch) % self.depth
            if g not in self._ahead:
                prepass_ahead(terrains)
            self._ahead.discard(g)
            nxt = (g + 1) % self.depth
            if ahead and nxt != g:
                prepass_ahead([t for _, t in self.slots[nxt * self.batch:(nxt + 1) * self.batch]])
                self._ahead.add(nxt)
            trace_ahead(terrains, shard_rank, shard_count)
        devs = [d for d, _ in group]
        if present:
            for d in devs:
                d.present()
        self.frame += self.batch
        return devs

    def render(self, shard_rank=0, shard_count=1, camera=None, present=True):
        """Queue one frame on the next slot; returns its Device (the frame is complete once
        that device's stream reaches this point: Device.synchronize / readback)."""
        dev, ter = self.next_slot()
        if camera is not None:
            ter.set_camera(camera)
            ter.update_terrain()
        ter.render_device(shard_rank, shard_count)
        if present:
            dev.present()
        self.frame += 1
        return dev

    def synchronize(self):
        for dev, _ in self.slots:
            dev.synchronize()

    def set_profiling(self, on):
        for dev, _ in self.slots:
            check(lib().rt_device_set_profiling(dev._h, 1 if on else 0), "set_profiling")

    def kernel_time(self):
        """(total ms, launches) of tracescreen launches recorded since the last call, all slots."""
        tot, n = 0.0, 0
        for dev, _ in self.slots:
            kms, kn = C.c_double(), C.c_int()
            check(lib().rt_device_kernel_time(dev._h, C.byref(kms), C.byref(kn)), "kernel_time")
            tot, n = tot + kms.value, n + kn.value
        return tot, n

    def destroy(self):
        # any order is safe: a group's devices borrow its first device's stream, and the runtime
        # keeps a lent stream alive until its last user is destroyed (rt_stream_refs)
        for dev, _ in reversed(self.slots):
            dev.destroy()
        self.slots = []
