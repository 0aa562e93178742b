"""Access to the committed golden fixtures (tests/golden/*.npz, made by
tests/golden/make_golden.py).  Frame constants come from the fixture, so parity
checks never depend on the host camera maths."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

FRAMES = [  # (landscape, pose, W, H, aa, max_steps[, ao_samples]) -- keep in sync with make_golden.py
    ("nomadplains", "reset", 64, 48, 1, 0),
    ("nomadplains", "lookdown", 64, 48, 1, 0),
    ("nomadplains", "reset", 48, 32, 4, 0),
    ("nomadplains", "reset", 64, 48, 1, 64),
    ("testing", "reset", 64, 48, 1, 0),
    ("testing", "lookdown", 64, 48, 1, 0),
    ("simple", "reset", 48, 32, 1, 0),
    ("greenrocks", "reset", 48, 32, 1, 0),
    # AO build extension (BASELINE configs C3/C5): (..., ao_samples)
    ("nomadplains", "reset", 64, 48, 1, 0, 1),
    ("nomadplains", "lookdown", 48, 32, 1, 512, 4),
    ("greenrocks", "reset", 48, 32, 2, 0, 2),
    # AA_SAMPLES 8 and 16 (antialiasing.hlsl, D3D11 standard sample patterns)
    ("nomadplains", "reset", 32, 24, 8, 0),
    ("nomadplains", "lookdown", 24, 16, 16, 0, 1),
]

_cache = {}


def frame_key(land, pose, w, h, aa, ms, ao=0):
    return f"{land}_{pose}_{w}x{h}_aa{aa}_ms{ms}" + (f"_ao{ao}" if ao else "")


def unpack(spec):
    """(landscape, pose, W, H, aa, max_steps[, ao_samples]) -> 7-tuple"""
    return tuple(spec) + (0,) * (7 - len(spec))


def load():
    if "frames" not in _cache:
        _cache["frames"] = dict(np.load(os.path.join(GOLDEN, "oracle_frames.npz")))
    return _cache["frames"]


def scene():
    if "scene" not in _cache:
        _cache["scene"] = dict(np.load(os.path.join(GOLDEN, "scene_constants.npz")))
    return _cache["scene"]


def consts(w, h, pose):
    s = scene()
    p = f"{pose}_{w}x{h}_"
    return {"width": w, "height": h, "eye": s[p + "eye"], "view_inverse": s[p + "view_inverse"],
            "projection": s[p + "projection"], "sun": s[p + "sun"]}
