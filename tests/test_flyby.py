"""Flyby autopilot on the CPU: the vectorised product form
(gpgpuraytrace_amd/flyby.py) against the scalar restatement of Flyby.cpp (oracle/flyby_ref.py),
on synthetic views that hit each rule and on a short fly-through fed by the oracle's own
camerarays prepass (the CameraResults the GPU path reproduces bit for bit)."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import oracle_lib as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
from flyby_ref import FlybyRef  # noqa: E402

from gpgpuraytrace_amd import camera as CAM  # noqa: E402
from gpgpuraytrace_amd.flyby import Flyby  # noqa: E402


def _pair(position=(0.0, 100.0, 0.0), euler=CAM.INITIAL_ROTATION_EULER):
    cam = CAM.Camera(64, 48, position, euler)
    return cam, Flyby(cam), FlybyRef(cam.position, cam.front)


def _step(cam, fly, ref, dt, view):
    fly.fly(dt, view)
    p, f = ref.fly(dt, view)
    np.testing.assert_array_equal(np.asarray(cam.position, np.float32), p)
    np.testing.assert_array_equal(np.asarray(cam.front, np.float32), f)
    np.testing.assert_array_equal(fly.target, ref.target)


def _view(rng, depth_lo=0.5, depth_hi=60.0, sky_rows=()):
    v = np.zeros((1024, 4), np.float32)
    v[:, :3] = rng.normal(0, 30, (1024, 3)).astype(np.float32) + np.array([0, 95, 0], np.float32)
    v[:, 3] = rng.uniform(depth_lo, depth_hi, 1024).astype(np.float32)
    for r in sky_rows:
        v[r * 32 + 5:(r + 1) * 32, 3] = 5000.0  # unusable from x = 5: the row's scan breaks there
    return v


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_flyby_matches_scalar_restatement_synthetic(seed):
    rng = np.random.default_rng(seed)
    cam, fly, ref = _pair()
    for i in range(12):
        view = _view(rng, sky_rows=range(0, 32, 3 + i % 4))
        if i == 5:
            view[:, 3] = 1.0  # 20% depth in (0.01, 1.4): direction blocked, score dropped
        if i == 7:
            view[:, 3] = 0.0  # nothing usable: no target
        _step(cam, fly, ref, 1.0 / 25.0, view)


def test_flyby_no_target_turns_around():
    cam, fly, ref = _pair()
    empty = np.zeros((1024, 4), np.float32)  # Terrain's zero view: every row breaks at x = 0
    logs = []
    for _ in range(130):  # > 5 s of 1/25 steps without a target
        _step(cam, fly, ref, 1.0 / 25.0, empty)
        logs += fly.log
    assert sum("Turning around cause of no target" in m for m in logs) == 1


def test_fly_through_on_oracle_prepass():
    """8 frames: Flyby steers from the oracle's camerarays results of the previous camera."""
    nz = O.noise_tables()
    cam, fly, ref = _pair()
    view = np.zeros((1024, 4), np.float32)
    for _ in range(8):
        _step(cam, fly, ref, 1.0 / 25.0, view)
        cam.update()
        fr = O.make_frame(CAM.camera_constants(cam))
        cr = np.zeros(1024 * 4, np.float32)
        st = O.Stats()
        O.lib().ro_camerarays(C.byref(nz), C.byref(fr), O._fp(cr), C.byref(st))
        view = cr.reshape(1024, 4)
    assert np.isfinite(cam.position).all() and (view[:, 3] > 0).any()
