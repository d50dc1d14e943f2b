"""Host tone mapping (reference: main_taichi.py:53-78 finish/tonemap/finishing_tonemap,
tone_map.py:5-43).  Inputs are mean radiance frames (W, H, 3) [x][y]."""
import struct
import zlib

import numpy as np


def finish(mean):
    """buffer = sqrt(pixels / samples) (main_taichi.py:61-64)."""
    return np.sqrt(np.asarray(mean, np.float32))


def luminance(mean):
    """main_taichi.py:53-58 (NaN pixels skipped → 0)."""
    m = np.asarray(mean, np.float32)
    lum = m[..., 0] * np.float32(0.2126) + m[..., 1] * np.float32(0.7152) + m[..., 2] * np.float32(0.0722)
    return np.where(np.isnan(lum), np.float32(0), lum)


def reinhard_extended(mean):
    """finishing_tonemap (main_taichi.py:67-78) on the mean radiance."""
    m = np.asarray(mean, np.float32)
    lum = luminance(m)
    max_white = np.max(lum)
    num = lum * (1.0 + lum / (max_white * max_white))
    l_new = num / (1.0 + lum)
    with np.errstate(divide="ignore", invalid="ignore"):
        scale = np.where(lum > 0, l_new / lum, 0.0)
    return (m * scale[..., None]).astype(np.float32)


def to_uint8(img):
    return (np.clip(np.asarray(img), 0.0, 1.0) * 255.0 + 0.5).astype(np.uint8)


def write_png(path, rows_rgb_u8):
    """Minimal RGB PNG writer (no imaging dependency). rows: (H, W, 3) uint8, top row first."""
    a = np.ascontiguousarray(rows_rgb_u8, np.uint8)
    h, w, _ = a.shape
    raw = b"".join(b"\x00" + a[r].tobytes() for r in range(h))

    def chunk(tag, data):
        c = struct.pack(">I", len(data)) + tag + data
        return c + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as fh:
        fh.write(png)
