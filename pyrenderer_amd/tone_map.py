"""Host tone mapping (reference: main_taichi.py:53-78 finish/tonemap/finishing_tonemap,
tone_map.py:5-43).  Inputs are mean radiance frames (W, H, 3) [x][y]."""
import struct
import zlib

import numpy as np


def finish(mean):
    """buffer = sqrt(pixels / samples) (main_taichi.py:61-64)."""
    return np.sqrt(np.asarray(mean, np.float32))


def save_hdr(directory, sums, samples):
    """The reference's HDR pair (main_taichi.py:120-123): `hdr.npy` = the per-pixel radiance SUMS
    (`pixels.to_numpy()`, (W, H, 3) float32 [x][y]) and `spp.npy` = the per-pixel sample counts
    (`samples.to_numpy()`, (W, H) float32), the input of the reference's offline tone_map.py:5-9.
    Returns the two paths."""
    import os
    os.makedirs(directory, exist_ok=True)
    sums = np.asarray(sums, np.float32)
    hdr, spp = os.path.join(directory, "hdr.npy"), os.path.join(directory, "spp.npy")
    np.save(hdr, sums)
    np.save(spp, np.full(sums.shape[:2], np.float32(samples), np.float32))
    return hdr, spp


def finish_hdr(hdr_mat, spp_mat):
    """tone_map.py:5-9 on the pair: NaN sums -> 0, then sqrt(hdr / spp[0, 0]) — finish() of the
    mean (main_taichi.py:61-64) computed from the saved files."""
    h = np.array(hdr_mat, np.float32)
    h[np.isnan(h)] = 0
    return np.sqrt(h / np.asarray(spp_mat, np.float32)[0, 0])


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
