"""Output path on the CPU: the oracle's restatement of
RecorderWinAPI::write (pixel conversion, sample time stamps) against known answers and an
independent numpy statement, and the PPM / PNG frame writers."""
import numpy as np

import oracle_lib as O
from gpgpuraytrace_amd import output as OUT


def test_bgrx_known_answers():
    # dwc = 0x80402010 (R 0x10, G 0x20, B 0x40, A 0x80) -> 0x00102040: bytes B G R 0 (MFVideoFormat_RGB32)
    px = np.array([[[0x10, 0x20, 0x40, 0x80], [0xFF, 0x00, 0x00, 0xFF], [0x00, 0x00, 0xFF, 0x00]]], np.uint8)
    assert O.bgrx(px).tolist() == [[0x00102040, 0x00FF0000, 0x000000FF]]


def test_bgrx_matches_numpy_statement_with_stride():
    rng = np.random.default_rng(7)
    big = rng.integers(0, 256, (37, 64, 4), dtype=np.uint8)
    frame = big[:, :61]  # rows 256 B apart, 61 pixels used (odd width, padded stride)
    got = O.bgrx(frame)
    d = np.ascontiguousarray(frame).view(np.uint32)[..., 0]
    want = (d & 0x0000FF00) | ((d & 0x000000FF) << 16) | ((d & 0x00FF0000) >> 16)
    assert np.array_equal(got, want)
    assert np.array_equal(OUT.bgrx_to_rgb(got), frame[..., :3])


def test_sample_times_fixed_and_timer_driven():
    t, d = O.sample_times(25, True, np.zeros(4, np.float32))
    assert d.tolist() == [400000] * 4 and t.tolist() == [0, 400000, 800000, 1200000]
    ft = np.array([0.04, 0.0333333, 0.1, 1.0 / 60.0], np.float32)
    t, d = O.sample_times(25, False, ft)
    want = (np.float32(10000000.0) * ft).astype(np.uint64)  # (UINT64)(10000000.0f * modifier)
    assert d.tolist() == want.tolist()
    assert t.tolist() == np.concatenate([[0], np.cumsum(want)[:-1]]).tolist()


def test_ppm_png_round_trip(tmp_path):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (21, 34, 4), dtype=np.uint8)
    OUT.write_ppm(tmp_path / "a.ppm", img)
    assert np.array_equal(OUT.read_ppm(tmp_path / "a.ppm"), img[..., :3])
    OUT.write_png(tmp_path / "a.png", img)
    assert np.array_equal(OUT.read_png(tmp_path / "a.png"), img)
