"""ctypes bindings to the CPU oracle (oracle/_build/librt_oracle.so).

TEST INFRASTRUCTURE: used only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker (see oracle/rt_oracle.h).
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "_build", "librt_oracle.so")

NOMADPLAINS, TESTING, SIMPLE, GREENROCKS = 0, 1, 2, 3
LANDSCAPES = {"nomadplains": 0, "testing": 1, "simple": 2, "greenrocks": 3}
RAND_MSVC, RAND_GLIBC = 0, 1


class Noise(C.Structure):
    _fields_ = [("perm2d", C.c_uint8 * (128 * 128 * 4)), ("grad", C.c_float * 512), ("perm", C.c_int32 * 128)]


class Frame(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32), ("landscape", C.c_int32), ("aa_samples", C.c_int32),
        ("recording", C.c_int32), ("max_steps", C.c_int32), ("eye", C.c_float * 4),
        ("view_inverse", C.c_float * 16), ("projection", C.c_float * 16), ("sun", C.c_float * 3),
        ("row_begin", C.c_int32), ("row_end", C.c_int32), ("row_step", C.c_int32), ("threads", C.c_int32),
        ("ao_samples", C.c_int32),
    ]


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("noise3d_calls", "prepass_steps", "primary_steps", "shadow_steps",
                                          "primary_rays", "primary_hits", "density_calls", "ao_steps", "ao_rays")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "all"], check=True)


_variants = {}


def variant(name):
    """An arithmetic-convention variant of the checker (oracle/rt_oracle.c RO_CONV_*: "unfused",
    "ieeediv", "libm", "all"), for the parity-sensitivity study; same API as lib()."""
    if name not in _variants:
        path = os.path.join(ORACLE_DIR, "_build", f"librt_oracle_{name}.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", ORACLE_DIR, "variants"], check=True)
        _variants[name] = _configure(C.CDLL(path))
    return _variants[name]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = _configure(C.CDLL(LIB_PATH))
    return _lib


def _configure(L):
    if True:
        fp = C.POINTER(C.c_float)
        L.ro_noise_generate.argtypes = [C.POINTER(Noise), C.c_uint32, C.c_int]
        for n in ("ro_exp2", "ro_log2", "ro_exp", "ro_sin", "ro_cos"):
            getattr(L, n).argtypes = [C.c_float]
            getattr(L, n).restype = C.c_float
        for n in ("ro_pow", "ro_max", "ro_min"):
            getattr(L, n).argtypes = [C.c_float, C.c_float]
            getattr(L, n).restype = C.c_float
        L.ro_batch_unary.argtypes = [C.c_int, fp, fp, C.c_int64]
        L.ro_batch_binary.argtypes = [C.c_int, fp, fp, fp, C.c_int64]
        L.ro_noise3d.argtypes = [C.POINTER(Noise), C.c_float, C.c_float, C.c_float]
        L.ro_noise3d.restype = C.c_float
        L.ro_noise3d_batch.argtypes = [C.POINTER(Noise), fp, fp, C.c_int64]
        L.ro_get_density_batch.argtypes = [C.POINTER(Noise), C.POINTER(Frame), fp, fp, C.c_int64]
        L.ro_camerarays.argtypes = [C.POINTER(Noise), C.POINTER(Frame), fp, C.POINTER(Stats)]
        L.ro_camerarays_steps.argtypes = [C.POINTER(Noise), C.POINTER(Frame), fp, fp, C.POINTER(Stats)]
        L.ro_set_target_depths.argtypes = [fp, fp]
        L.ro_tracescreen.argtypes = [C.POINTER(Noise), C.POINTER(Frame), fp, fp, C.POINTER(C.c_uint8), fp,
                                     C.POINTER(Stats)]
        L.ro_tracescreen2.argtypes = [C.POINTER(Noise), C.POINTER(Frame), fp, fp, C.POINTER(C.c_uint8), fp, fp,
                                      C.POINTER(Stats)]
        L.ro_render_frame.argtypes = [C.POINTER(Noise), C.POINTER(Frame), fp, fp, fp, C.POINTER(C.c_uint8), fp,
                                      C.POINTER(Stats)]
        L.ro_bgrx.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.ro_sky.argtypes = [C.POINTER(Noise), C.POINTER(Frame), fp, fp, C.c_int64]
        L.ro_sample_times.argtypes = [C.c_int, C.c_int, fp, C.c_int, C.c_void_p, C.c_void_p]
    return L


def bgrx(frame):
    """RecorderWinAPI::write's conversion of (H, W, 4) uint8 RGBA rows -> (H, W) uint32."""
    f = np.ascontiguousarray(frame, np.uint8)
    h, w = f.shape[:2]
    out = np.empty((h, w), np.uint32)
    lib().ro_bgrx(f.ctypes.data, w, h, f.strides[0], out.ctypes.data)
    return out


def sample_times(frame_rate, fixed_speed, frame_times):
    ft = np.ascontiguousarray(frame_times, np.float32)
    n = len(ft)
    t, d = np.empty(n, np.uint64), np.empty(n, np.uint64)
    lib().ro_sample_times(frame_rate, 1 if fixed_speed else 0, _fp(ft), n, t.ctypes.data, d.ctypes.data)
    return t, d


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def noise_tables(seed=300, rand_kind=RAND_MSVC):
    nz = Noise()
    lib().ro_noise_generate(C.byref(nz), seed, rand_kind)
    return nz


def unary(op, x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty_like(x)
    lib().ro_batch_unary(op, _fp(x), _fp(y), x.size)
    return y


def binary(op, a, b):
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    y = np.empty_like(a)
    lib().ro_batch_binary(op, _fp(a), _fp(b), _fp(y), a.size)
    return y


def noise3d(nz, xyz):
    xyz = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
    out = np.empty(len(xyz), np.float32)
    lib().ro_noise3d_batch(C.byref(nz), _fp(xyz), _fp(out), len(xyz))
    return out


def make_frame(consts, landscape=NOMADPLAINS, aa=1, recording=0, max_steps=0, rows=None, threads=0, ao=0):
    """consts: dict with width, height, eye(4), view_inverse(16), projection(16), sun(3) (HLSL matrices)."""
    fr = Frame()
    fr.width, fr.height = int(consts["width"]), int(consts["height"])
    fr.landscape, fr.aa_samples, fr.recording, fr.max_steps = landscape, aa, recording, max_steps
    fr.eye[:] = [float(v) for v in consts["eye"]]
    fr.view_inverse[:] = [float(v) for v in np.asarray(consts["view_inverse"], np.float32).ravel()]
    fr.projection[:] = [float(v) for v in np.asarray(consts["projection"], np.float32).ravel()]
    fr.sun[:] = [float(v) for v in consts["sun"]]
    if rows is None:
        rows = (0, fr.height, 1)
    fr.row_begin, fr.row_end, fr.row_step = rows
    fr.threads = threads
    fr.ao_samples = ao
    return fr


def sky(nz, fr, dirs):
    """(n, 7) float32: getRayleighMieColor (mie rgb, rayleigh rgb) and getSpaceColor per direction."""
    d = np.ascontiguousarray(dirs, dtype=np.float32).reshape(-1, 3)
    out = np.empty((len(d), 7), np.float32)
    lib().ro_sky(C.byref(nz), C.byref(fr), _fp(d), _fp(out), len(d))
    return out


def density(nz, fr, xyz):
    xyz = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
    out = np.empty(len(xyz), np.float32)
    lib().ro_get_density_batch(C.byref(nz), C.byref(fr), _fp(xyz), _fp(out), len(xyz))
    return out


def render(nz, fr, L=None):
    """Full frame (prepass + setTargetDepths + tracescreen). Returns dict of arrays + stats.
    L: a variant() library instead of the checker."""
    L = L or lib()
    W, H = fr.width, fr.height
    cr = np.zeros(1024 * 4, np.float32)
    cd = np.zeros(1024 * 2, np.float32)
    rgba = np.zeros((H, W, 4), np.float32)
    rgba8 = np.zeros((H, W, 4), np.uint8)
    steps = np.zeros((H, W), np.float32)
    st = Stats()
    L.ro_render_frame(C.byref(nz), C.byref(fr), _fp(cr), _fp(cd), _fp(rgba),
                          rgba8.ctypes.data_as(C.POINTER(C.c_uint8)), _fp(steps), C.byref(st))
    return {"camera_results": cr.reshape(1024, 4), "cell_distance": cd.reshape(1024, 2), "rgba32f": rgba,
            "rgba8": rgba8, "primary_steps": steps, "stats": st.as_dict()}


def render_rows(nz, fr, L=None, steps=None, secondary_steps=None):
    """Prepass + setTargetDepths + tracescreen on fr's rows (row_begin::row_step) only.
    Returns (rgba32f, rgba8, camera_results, cell_distance, stats); rows outside the sample
    stay zero.  L: a variant() library; steps / secondary_steps: (H, W) float32 arrays that
    receive each pixel's primary / shadow + AO march iterations."""
    L = L or lib()
    W, H = fr.width, fr.height
    cr = np.zeros(1024 * 4, np.float32)
    cd = np.zeros(1024 * 2, np.float32)
    rgba = np.zeros((H, W, 4), np.float32)
    rgba8 = np.zeros((H, W, 4), np.uint8)
    st = Stats()
    L.ro_camerarays(C.byref(nz), C.byref(fr), _fp(cr), C.byref(st))
    L.ro_set_target_depths(_fp(cr), _fp(cd))
    L.ro_tracescreen2(C.byref(nz), C.byref(fr), _fp(cd), _fp(rgba), rgba8.ctypes.data_as(C.POINTER(C.c_uint8)),
                      _fp(steps) if steps is not None else None,
                      _fp(secondary_steps) if secondary_steps is not None else None, C.byref(st))
    return rgba, rgba8, cr.reshape(1024, 4), cd.reshape(1024, 2), st.as_dict()
