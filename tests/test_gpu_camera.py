"""camera_kernel's primary rays (prt_camera_rays) against the host gen_ray of the converted camera
(VERDICT r04 item 4): for every item the (u, v) of main_taichi.py:93-94 from the sample's keyed
stream, then PackedCamera.gen_ray — bit for bit, pinhole (the kernel's shortcut), thin-lens (the two
lens draws that follow the jitter) and projective cameras, 4096 rays each."""
import copy

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _host_rays(pc, W, H, tile, tiles, spp, seed, lens):
    from oracle import oracle as O
    f = np.float32
    tx = (W + tile - 1) // tile
    uv, xi = [], []
    for s in range(spp):
        for t in tiles:
            for r in range(tile * tile):
                x = (t % tx) * tile + r % tile
                y = (t // tx) * tile + r // tile
                dr = O.rng_draws(O.rng_key(seed, y * W + x, s), 4)
                uv.append(((f(x) + dr[0]) / f(W - 1), (f(y) + dr[1]) / f(H - 1)))
                xi.append((dr[2], dr[3]))
    uv = np.array(uv, f)
    return pc.gen_ray(uv[:, 0], uv[:, 1], lens=np.array(xi, f) if lens else None)


@pytest.mark.parametrize("mod", ["pinhole", "aperture", "projective"])
def test_camera_kernel_rays_equal_host_gen_ray(gpu_scene, cornell, mod):
    pc = copy.deepcopy(cornell[1].convert_to_taichi_camera())
    if mod == "aperture":
        pc.sensor_dim = pc.sensor_dim.copy()
        pc.sensor_dim[3] = np.float32(1.0)
    elif mod == "projective":
        pc.iview_cols = pc.iview_cols.copy()
        pc.iview_cols[3, 0] = np.float32(1e-3)
    W, H, tile, spp, seed = 64, 48, 16, 2, 11
    tiles = [0, 2, 5, 7, 9, 11, 1, 4]                 # 8 tiles x 256 px x 2 samples = 4096 rays
    go, gd, _ = gpu_scene.camera_rays(pc.packed(), W, H, tile, tile, tiles, 3, spp, seed=seed)
    # prt_camera_rays' first sample is 3: the host keys the same global samples
    ho, hd = _host_rays(pc, W, H, tile, tiles, spp + 3, seed, mod == "aperture")
    n = len(tiles) * tile * tile
    ho, hd = ho[3 * n:], hd[3 * n:]
    assert go.shape == ho.shape == (4096, 3)
    np.testing.assert_array_equal(gd, hd)
    np.testing.assert_array_equal(go, ho)


def test_camera_rays_of_partial_edge_tiles(gpu_scene, cornell):
    """a frame whose size is not a multiple of the tile (40 x 36, 16-pixel tiles): rows of
    slots whose pixel lies outside the frame come back as zeros (origin, RNG state and direction — the
    camera kernel gives them no ray), the in-frame rows still equal the host gen_ray.  Also keys each
    sample as enqueue_render does (frame_spp = spp, frame_stride = 0)."""
    pc = cornell[1].convert_to_taichi_camera()
    W, H, tile, spp, seed = 40, 36, 16, 3, 5
    tiles = list(range(9))                              # 3 x 3 tiles, the last row and column partial
    go, gd, gs = gpu_scene.camera_rays(pc.packed(), W, H, tile, tile, tiles, 0, spp, seed=seed)
    ho, hd = _host_rays(pc, W, H, tile, tiles, spp, seed, False)
    tx = (W + tile - 1) // tile
    inside = np.array([((t % tx) * tile + r % tile < W) and ((t // tx) * tile + r // tile < H)
                       for _ in range(spp) for t in tiles for r in range(tile * tile)])
    assert inside.sum() == W * H * spp and (~inside).sum() > 0
    np.testing.assert_array_equal(gd[inside], hd[inside])
    np.testing.assert_array_equal(go[inside], ho[inside])
    assert not go[~inside].any() and not gd[~inside].any() and not gs[~inside].any()
