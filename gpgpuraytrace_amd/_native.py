"""ctypes binding of the in-tree C-ABI library (include/frosttrace.h).

The product path has no fallback: if librt_hip.so is missing this module
raises, loudly, instead of computing anything on the CPU.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# the product loads this library only (experiment builds are selected by scripts/with_variant.py,
# outside the package, before the first lib() call)
LIB_PATH = os.path.join(HERE, "_build", "librt_hip.so")
ROOT = os.path.dirname(HERE)
HEADER = os.path.join(ROOT, "include", "frosttrace.h")

RT_OK = 0
RT_DEVICE_FLOAT_OUTPUT = 1
RT_DEVICE_STATS = 2
RT_DEVICE_GRAPH = 4
RT_DEVICE_DEBUG_SMALL_RINGS = 32  # ABI 4: k_trace's long ring holds 64 entries, its fin pool 8 (spill / fallback tests)
RT_DEVICE_DEBUG_WITHHOLD_FUSE = 64  # ABI 7: a fusing trace runs none of the next batch's prepass tasks (timeout test)
RT_DEVICE_GATED = 128  # ABI 7 (opt-in): the prepass inside the trace kernel, units gated on their cells' rays
RT_DEVICE_DEBUG_GATE_STRESS = 512  # ABI 8, diagnostic: L1-warm consumers and a late CellDistance (gated hand-off test)
RT_DEVICE_DEFERRED = 1024  # ABI 9: a render's trace launches with the next render (which fuses its prepass into it)
RT_DEVICE_DEBUG_DEFER_SMALL = 2048  # ABI 9, diagnostic: the one-frame deferral below 1280x720 pixels too (tests)
ABI_VERSION = 9  # include/frosttrace.h RT_ABI_VERSION this binding's structs and signatures match
RT_TEXTURE_2D = 1
RT_FORMAT_R8G8B8A8_UINT = 3


class RtStats(C.Structure):
    _fields_ = [("primary_steps", C.c_ulonglong), ("shadow_steps", C.c_ulonglong),
                ("prepass_steps", C.c_ulonglong), ("hits", C.c_ulonglong), ("noise_calls", C.c_ulonglong),
                ("ao_steps", C.c_ulonglong), ("noise_wave_iters", C.c_ulonglong)]


class NativeError(RuntimeError):
    pass


_lib = None

# name -> (restype, argtypes)
_vp, _i, _u, _sz, _cp = C.c_void_p, C.c_int, C.c_uint, C.c_size_t, C.c_char_p
SIGNATURES = {
    "rt_last_error": (_cp, []),
    "rt_abi_version": (_i, []),
    "rt_vfs_add_path": (_i, [_cp]),
    "rt_vfs_clear": (_i, []),
    "rt_device_create": (_i, [_i, _i, _i, _u, C.POINTER(_vp)]),
    "rt_device_destroy": (None, [_vp]),
    "rt_device_present": (_i, [_vp]),
    "rt_device_flush": (_i, [_vp]),
    "rt_device_synchronize": (_i, [_vp]),
    "rt_device_readback": (_i, [_vp, _vp, _sz]),
    "rt_device_readback_float": (_i, [_vp, _vp]),
    "rt_device_readback_bgrx": (_i, [_vp, _vp, _sz]),
    "rt_device_size": (_i, [_vp, C.POINTER(_i), C.POINTER(_i)]),
    "rt_device_framebuffer": (_vp, [_vp]),
    "rt_device_stream": (_vp, [_vp]),
    "rt_device_set_stream": (_i, [_vp, _vp]),
    "rt_device_stats": (_i, [_vp, C.POINTER(RtStats), _i]),
    "rt_device_stats_sized": (_i, [_vp, C.POINTER(RtStats), _sz, _i]),
    "rt_stream_refs": (_i, [_vp]),
    "rt_device_set_profiling": (_i, [_vp, _i]),
    "rt_device_kernel_time": (_i, [_vp, C.POINTER(C.c_double), C.POINTER(_i)]),
    "rt_device_graph_info": (_i, [_vp, C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]),
    "rt_device_info": (_i, [_vp, _i, C.POINTER(C.c_ulonglong)]),
    "rt_device_reserve_cus": (_i, [_vp, _i]),
    "rt_device_defer_batch": (_i, [_vp, _i]),
    "rt_debug_spin": (_i, [_vp, _vp, C.c_ulonglong, C.c_ulonglong, _vp]),
    "rt_debug_defer_slot": (_i, [_vp, _i, _vp, _vp, _vp]),
    "rt_device_wait_event": (_i, [_vp, _vp]),
    "rt_device_record_event": (_i, [_vp, _vp]),
    "rt_device_check": (_i, [_vp]),
    "rt_texture_create": (_i, [_vp, C.POINTER(_vp)]),
    "rt_texture_init": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i]),
    "rt_texture_destroy": (None, [_vp]),
    "rt_compute_create": (_i, [_vp, C.POINTER(_vp)]),
    "rt_compute_destroy": (None, [_vp]),
    "rt_compute_load": (_i, [_vp, _cp, _cp, _cp, _i, _i, _i, C.POINTER(_cp), C.POINTER(_cp), _i]),
    "rt_compute_swap": (_i, [_vp]),
    "rt_compute_run": (_i, [_vp, _u, _u, _u]),
    "rt_compute_set_texture": (_i, [_vp, _i, _vp]),
    "rt_compute_thread_size": (_i, [_vp, C.POINTER(_i), C.POINTER(_i), C.POINTER(_i)]),
    "rt_compute_get_variable": (_vp, [_vp, _cp]),
    "rt_compute_get_array": (_vp, [_vp, _cp]),
    "rt_compute_get_buffer": (_vp, [_vp, _cp]),
    "rt_variable_write": (_i, [_vp, _vp]),
    "rt_variable_size": (_sz, [_vp]),
    "rt_variable_name": (_cp, [_vp]),
    "rt_array_create": (_i, [_vp, _u]),
    "rt_array_map": (_vp, [_vp]),
    "rt_array_unmap": (_i, [_vp]),
    "rt_array_write": (_i, [_vp, _vp]),
    "rt_array_stride": (_sz, [_vp]),
    "rt_array_device_pointer": (_vp, [_vp]),
    "rt_terrain_render": (_i, [_vp, _vp, _i, _i]),
    "rt_terrain_render_feed": (_i, [_vp, _vp, _i, _i]),
    "rt_terrain_render_batch": (_i, [C.POINTER(_vp), C.POINTER(_vp), _i, _i, _i]),
    "rt_terrain_render_batch_packed": (_i, [C.POINTER(_vp), C.POINTER(_vp), _i, _i, _i, _vp, _sz]),
    "rt_terrain_prepass_batch": (_i, [C.POINTER(_vp), C.POINTER(_vp), _i, _i, _i, _vp]),
    "rt_terrain_trace_batch": (_i, [C.POINTER(_vp), C.POINTER(_vp), _i, _i, _i, _vp]),
    "rt_terrain_prepass_ahead": (_i, [C.POINTER(_vp), C.POINTER(_vp), _i]),
    "rt_terrain_trace_ahead": (_i, [C.POINTER(_vp), C.POINTER(_vp), _i, _i, _i]),
    "rt_terrain_feed_wait": (_i, [_vp, _vp]),
    "rt_shard_bytes": (_sz, [_vp, _i, _i]),
    "rt_shard_pack": (_i, [_vp, _i, _i, _vp]),
    "rt_shard_unpack": (_i, [_vp, _i, _i, _vp]),
    "rt_shard_pack_batch": (_i, [C.POINTER(_vp), C.POINTER(_i), _i, C.POINTER(_vp), _i]),
    "rt_shard_unpack_batch": (_i, [C.POINTER(_vp), C.POINTER(_i), _i, C.POINTER(_vp), _i]),
    "rt_noise_generate": (_i, [C.c_uint32, _i, _vp, _vp]),
    "rt_terrain_set_target_depths": (_i, [_vp, _vp]),
    "rt_recorder_create": (_i, [_vp, _i, _i, _cp, C.POINTER(_vp)]),
    "rt_recorder_start": (_i, [_vp]),
    "rt_recorder_stop": (_i, [_vp]),
    "rt_recorder_is_recording": (_i, [_vp]),
    "rt_recorder_set_frame_time": (_i, [_vp, C.c_float]),
    "rt_recorder_write": (_i, [_vp, _vp, _i]),
    "rt_recorder_info": (_i, [_vp, C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]),
    "rt_recorder_destroy": (None, [_vp]),
    "rt_varmgr_start": (_i, [_i, _cp]),
    "rt_varmgr_stop": (_i, []),
    "rt_varmgr_count": (_i, []),
    "rt_varmgr_register_compute": (_i, [_vp]),
    "rt_debug_math": (_i, [_vp, _i, _vp, _vp, _vp, _i]),
    "rt_debug_noise": (_i, [_vp, _vp, _vp, _i, _i]),
    "rt_debug_sky": (_i, [_vp, _vp, _vp, _i]),
}


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"gpgpuraytrace_amd: native library missing at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (make -C gpgpuraytrace_amd/csrc)")
        L = C.CDLL(LIB_PATH)
        # the version first: an older library lacks later exports, and binding those would fail
        # with a bare AttributeError before this message could say what to do
        L.rt_abi_version.restype, L.rt_abi_version.argtypes = _i, []
        if L.rt_abi_version() < ABI_VERSION:  # an older library: its structs are shorter than ours
            raise ImportError(f"gpgpuraytrace_amd: {LIB_PATH} has ABI {L.rt_abi_version()}, this binding "
                              f"needs >= {ABI_VERSION}; rebuild it (make -C gpgpuraytrace_amd/csrc)")
        for name, (res, args) in SIGNATURES.items():
            try:
                f = getattr(L, name)
            except AttributeError:
                raise ImportError(f"gpgpuraytrace_amd: {LIB_PATH} does not export {name}; rebuild it "
                                  "(make -C gpgpuraytrace_amd/csrc)") from None
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc, what=""):
    if rc != RT_OK:
        msg = lib().rt_last_error().decode(errors="replace")
        raise NativeError(f"{what}: rc={rc}: {msg}")
    return rc
