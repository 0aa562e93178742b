"""Frame files: the step after the framebuffer readback.

The reference shows frames in a window and records video through Media Foundation
(RecorderWinAPI.cpp); neither exists here.  These writers turn a readback into image files:
binary PPM (P6) and PNG (8-bit RGBA, zlib from the standard library), plus the converter
from the recorder's raw (B, G, R, 0) rows back to RGB for viewing.  Pure host code over
numpy arrays; the GPU side is Device.readback / readback_bgrx.
"""
import struct
import zlib

import numpy as np


def write_ppm(path, rgba):
    """(H, W, 4|3) uint8 -> binary PPM (alpha dropped)."""
    a = np.ascontiguousarray(np.asarray(rgba, np.uint8)[..., :3])
    h, w = a.shape[:2]
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(a.tobytes())


def read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(maxsplit=4)
    if parts[0] != b"P6" or parts[3] != b"255":
        raise ValueError("not an 8-bit binary PPM")
    w, h = int(parts[1]), int(parts[2])
    return np.frombuffer(parts[4][:w * h * 3], np.uint8).reshape(h, w, 3)


def _chunk(tag, body):
    return struct.pack(">I", len(body)) + tag + body + struct.pack(">I", zlib.crc32(tag + body) & 0xFFFFFFFF)


def write_png(path, rgba, level=6):
    """(H, W, 4) uint8 -> 8-bit RGBA PNG (filter 0 on every row)."""
    a = np.ascontiguousarray(np.asarray(rgba, np.uint8))
    h, w = a.shape[:2]
    raw = np.zeros((h, 1 + w * 4), np.uint8)
    raw[:, 1:] = a.reshape(h, w * 4)
    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(_chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)))
        f.write(_chunk(b"IDAT", zlib.compress(raw.tobytes(), level)))
        f.write(_chunk(b"IEND", b""))


def read_png(path):
    """Reader for the files write_png produces (8-bit RGBA, filter 0)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError("not a PNG")
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        tag, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", body[:10])
            if depth != 8 or ctype != 6:
                raise ValueError("only 8-bit RGBA")
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + w * 4)
    if raw[:, 0].any():
        raise ValueError("only filter 0")
    return raw[:, 1:].reshape(h, w, 4).copy()


def bgrx_to_rgb(bgrx):
    """(H, W) uint32 (B, G, R, 0) rows -> (H, W, 3) uint8 RGB."""
    b = np.ascontiguousarray(bgrx, np.uint32).view(np.uint8).reshape(*bgrx.shape, 4)
    return b[..., 2::-1].copy()
