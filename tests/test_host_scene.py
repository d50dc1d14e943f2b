"""Host API parity: the Tungsten loader, transforms, camera and flattening
reproduce what the reference loads (tests/golden/scene_cornell.npz)."""
import numpy as np

from conftest import golden


def test_transforms_vertices_normals_exact(cornell):
    scene, cam, flat = cornell
    g = golden("scene_cornell.npz")
    np.testing.assert_array_equal(np.stack([p.trans_mat for p in scene.primitives]), g["trans_mat"])
    np.testing.assert_array_equal(np.concatenate([p.vertices for p in scene.primitives]), g["vertices_f64"])
    np.testing.assert_array_equal(np.concatenate([p.faces for p in scene.primitives]), g["faces"])
    np.testing.assert_array_equal(flat.tri_n, g["normals"])
    v32 = g["vertices_f32"]
    f = g["faces"] + np.repeat(g["prim_vert_off"][:-1], np.diff(g["prim_face_off"]))[:, None]
    np.testing.assert_array_equal(flat.tri_v, v32[f].reshape(-1, 9))


def test_bsdfs_and_lights(cornell):
    scene, cam, flat = cornell
    g = golden("scene_cornell.npz")
    np.testing.assert_array_equal(flat.mat[flat.tri_mat[g["prim_face_off"][:-1]], :3], g["rho"])
    np.testing.assert_array_equal(flat.mat[flat.tri_mat[g["prim_face_off"][:-1]], 3].astype(int), g["emit"])
    np.testing.assert_array_equal(flat.mat[flat.tri_mat[g["prim_face_off"][:-1]], 4].astype(int), g["sided"])
    assert flat.n_light == 1
    np.testing.assert_array_equal(flat.light_tri, [34, 35])  # Light quad, last primitive
    np.testing.assert_array_equal(flat.prim_lo, g["bounds_min"].astype(np.float32))
    np.testing.assert_array_equal(flat.prim_hi, g["bounds_max"].astype(np.float32))


def test_camera_record(cornell):
    scene, cam, flat = cornell
    g = golden("scene_cornell.npz")
    pc = cam.convert_to_taichi_camera()
    np.testing.assert_array_equal(pc.iview_cols, g["cam_iview_cols"])
    np.testing.assert_array_equal(pc.sensor_dim, g["cam_sensor_dim"])
    packed = pc.packed()
    assert packed.shape == (24,) and packed.dtype == np.float32
    np.testing.assert_array_equal(packed[[3, 7, 11]], np.float32([0, 1, 6.8]))  # eye, test.py:39 first origin


def test_bsdf_factory_errors():
    import pytest
    from pyrenderer_amd.core.bsdf import BSDF
    with pytest.raises(NotImplementedError):
        BSDF({"type": "plastic", "albedo": 1})
    with pytest.raises(NotImplementedError):
        BSDF({"type": "metal", "albedo": 1}, strict=True)   # reference factory semantics
    assert BSDF({"type": "metal", "albedo": [1, 1, 1]}).get_distribution().type_id == 2


def test_no_light_raises():
    import pytest
    from pyrenderer_amd.core.bsdf import BSDF
    from pyrenderer_amd.core.scene import Scene
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.mathematics.affine_transformation import make_transformation_matrix
    from pyrenderer_amd.mathematics.shapes import Quad
    s = Scene()
    s.add_primitive(Quad(make_transformation_matrix({}), BSDF({"type": "lambert", "albedo": [1, 1, 1]}).get_distribution()))
    with pytest.raises(ValueError):
        flatten_scene(s)


def test_obj_loader_and_tile_unpack():
    import os
    from conftest import ROOT
    from pyrenderer_amd.device_scene import interleaved_tiles, unpack_tiles
    from pyrenderer_amd.io_utils.read_tungsten import load_obj
    v, f = load_obj(os.path.join(ROOT, "pyrenderer_amd", "media", "cube.obj"))
    assert v.shape == (8, 3) and f.shape == (12, 3) and f.min() == 0 and f.max() == 7
    # tiles: 100x70 frame, 32x32 tiles -> 4x3 tiles; interleave over 3 ranks covers all once
    ids = [interleaved_tiles(100, 70, 32, r, 3) for r in range(3)]
    allids = np.sort(np.concatenate(ids))
    np.testing.assert_array_equal(allids, np.arange(12))
    frame = np.zeros((100, 70, 3), np.float32)
    for r in range(3):
        slots = np.zeros((len(ids[r]) * 32 * 32, 3), np.float32)
        for k, t in enumerate(ids[r]):
            tx, ty = t % 4, t // 4
            ly, lx = np.divmod(np.arange(32 * 32), 32)
            slots[k * 1024:(k + 1) * 1024, 0] = tx * 32 + lx
            slots[k * 1024:(k + 1) * 1024, 1] = ty * 32 + ly
        unpack_tiles(slots, 100, 70, 32, 32, ids[r], frame)
    xs, ys = np.meshgrid(np.arange(100), np.arange(70), indexing="ij")
    np.testing.assert_array_equal(frame[..., 0], xs)
    np.testing.assert_array_equal(frame[..., 1], ys)


def test_cli_arguments():
    """The CLI's flags (python -m pyrenderer_amd): parsing only, no device work."""
    from pyrenderer_amd.main import DEFAULT_SCENE, parse
    a = parse([])
    assert a.scene == DEFAULT_SCENE and a.samples == 64 and a.depth == 16 and a.devices == [0]
    a = parse(["x.json", "--samples", "8", "--devices", "0", "1", "--nee", "mis", "--resolution", "64", "32"])
    assert a.samples == 8 and a.devices == [0, 1] and a.nee == "mis" and a.resolution == [64, 32]


def test_tone_maps_restate_the_reference():
    """finish = sqrt(pixels / samples) (main_taichi.py:61-64); reinhard_extended = the
    extended Reinhard of main_taichi.py:67-78 / tone_map.py:17-35 on the mean radiance
    (luminance 0.2126 / 0.7152 / 0.0722, white point = max luminance, zero-luminance pixels
    stay black as tone_map.py:31-32 leaves them)."""
    from pyrenderer_amd.tone_map import finish, luminance, reinhard_extended
    rng = np.random.default_rng(5)
    spp = 16
    pixels = (rng.random((24, 20, 3)) * 40).astype(np.float32)
    pixels[3, 4] = 0.0
    mean = pixels / np.float32(spp)
    np.testing.assert_array_equal(finish(mean), np.sqrt(pixels / np.float32(spp)))
    lum = (mean[..., 0] * np.float32(0.2126) + mean[..., 1] * np.float32(0.7152)) + mean[..., 2] * np.float32(0.0722)
    np.testing.assert_allclose(luminance(mean), lum, rtol=1e-6)
    ref = np.zeros_like(mean, dtype=np.float64)
    mw = float(lum.max())
    for i in range(mean.shape[0]):
        for j in range(mean.shape[1]):
            li = float(lum[i, j])
            if li == 0.0:
                continue
            l_new = li * (1.0 + li / (mw * mw)) / (1.0 + li)
            ref[i, j] = pixels[i, j].astype(np.float64) * (l_new / li) / spp
    np.testing.assert_allclose(reinhard_extended(mean), ref, rtol=2e-6, atol=1e-7)
    assert not reinhard_extended(mean)[3, 4].any()
