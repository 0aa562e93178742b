"""Sky known-answer vectors: the oracle's getRayleighMieColor and
getSpaceColor (oracle/rt_oracle.c get_rayleigh_mie / get_space_color, float32 under rules R1-R9)
against tests/sky_ref.py, an independent float64 restatement of Media/common/shaders/sky.hlsl
with exact exp / pow, at fixed view directions, sun angles and eye positions.  The bound is
BASELINE.md's parity tolerance, 1e-4 per channel; the measured worst case is 5.8e-5 (the star
field: float32 rounding of dir * 500 before the lattice) and 1.2e-5 for the scattering.  The GPU's
sky equals the oracle's bit for bit (tests/test_gpu_parity.py::test_sky_known_answers_device)."""
import numpy as np
import pytest

import oracle_lib as O
import sky_ref as R

TOL = 1e-4  # BASELINE.md parity bound, per channel


def directions():
    az = np.radians(np.arange(0, 360, 30))
    el = np.radians([-30, -5, 0, 2, 5, 15, 30, 60, 89.5])
    d = [[np.cos(e) * np.cos(a), np.sin(e), np.cos(e) * np.sin(a)] for e in el for a in az]
    return np.array(d + [[0.0, 1.0, 0.0], [0.3, 0.0, -0.7]], np.float32)


def sun(t):
    """Terrain::setTimeOfDay (Terrain.cpp:292-298): normalize(-sin 2 pi t, -cos 2 pi t, 0.1)."""
    s = np.array([-np.sin(2 * np.pi * t), -np.cos(2 * np.pi * t), 0.1])
    return (s / np.linalg.norm(s)).astype(np.float32)


EYES = [(0.0, 100.0, 0.0), (1234.0, 350.0, -987.0), (-50.0, 2.0, 75.0)]
TIMES = [0.05, 0.2, 0.25, 0.3, 0.45, 0.7, 0.9]


def frame(eye, t):
    c = {"width": 64, "height": 48, "eye": list(eye) + [1.0], "view_inverse": np.eye(4), "projection": np.eye(4),
         "sun": sun(t)}
    return O.make_frame(c)


@pytest.mark.parametrize("eye", EYES)
@pytest.mark.parametrize("t", TIMES)
def test_sky_oracle_matches_float64_restatement(eye, t):
    nz = O.noise_tables()
    perm2d = np.frombuffer(bytes(nz.perm2d), np.uint8)
    grad = np.array(nz.grad[:], np.float32).reshape(128, 4)
    d = directions()
    got = O.sky(nz, frame(eye, t), d).astype(np.float64)
    mie, ray = R.rayleigh_mie(d, np.array(eye, np.float32), sun(t))
    space = R.space_color(perm2d, grad, d, sun(t))
    assert np.all(np.isfinite(got))
    assert np.abs(got[:, 0:3] - mie).max() <= TOL
    assert np.abs(got[:, 3:6] - ray).max() <= TOL
    assert np.abs(got[:, 6] - space).max() <= TOL


def test_sky_known_answer_properties():
    """Structure the restatements share with the HLSL: below-horizon directions see the horizon's
    sky (modRayDir saturates y) and no stars; the day hack adds (0.3, 0.4, 0.6) * saturate(sun.y)."""
    nz = O.noise_tables()
    d = np.array([[0.6, -0.4, 0.2], [0.6, 0.0, 0.2]], np.float32)
    got = O.sky(nz, frame(EYES[0], 0.3), d)
    assert np.array_equal(got[0, :3], got[1, :3])  # mie of the clamped direction
    assert got[0, 6] == 0.0 and got[1, 6] == 0.0  # getSpaceColor: dir.y <= 0 -> 0
    noon = O.sky(nz, frame(EYES[0], 0.5), np.array([[0.0, 1.0, 0.0]], np.float32))[0]
    assert np.all(noon[3:6] >= np.array([0.3, 0.4, 0.6], np.float32) * sun(0.5)[1] - 1e-6)
