"""The oracle's own RNG path (PCG stream, draws at the closest hit only) against
the statistical reference image: main_taichi.py's render() run by the
reference code itself (tests/golden/image_d{4,8}.npz: 32x32, 256 spp)."""
import numpy as np
import pytest

from conftest import golden
from oracle import oracle as O


@pytest.mark.parametrize("depth", [4, 8])
def test_statistical_image(oracle_scene, cornell, depth):
    g = golden(f"image_d{depth}.npz")
    ref, se = g["mean"], g["se"]
    cam = cornell[1].convert_to_taichi_camera().packed()
    spp = 2048
    a = oracle_scene.render(cam, 32, 32, spp, depth, seed=11) / spp
    b = oracle_scene.render(cam, 32, 32, spp, depth, seed=12) / spp
    img = 0.5 * (a + b)
    se_o = 0.5 * np.abs(a - b)
    # whole-image relative L2 difference is at the noise level of the reference image
    rel = np.sqrt(((img - ref) ** 2).sum() / (ref ** 2).sum())
    noise = np.sqrt((se ** 2 + se_o ** 2).sum() / (ref ** 2).sum())
    assert rel < 1.5 * noise, (rel, noise)
    # per-channel image mean within 4 sigma
    n = ref.shape[0] * ref.shape[1]
    zg = (img.mean((0, 1)) - ref.mean((0, 1))) / (np.sqrt((se ** 2 + se_o ** 2).sum((0, 1))) / n)
    assert np.all(np.abs(zg) < 4), zg
    # well-sampled pixels (mean > 0.01): per-pixel |z| < 6, and < 2% beyond 4 sigma
    z = (img - ref) / np.sqrt(se ** 2 + se_o ** 2 + 1e-12)
    well = ref > 0.01
    assert np.abs(z[well]).max() < 6, np.abs(z[well]).max()
    assert (np.abs(z[well]) > 4).mean() < 0.02
