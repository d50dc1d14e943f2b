"""Config 3 host + oracle checks on CPU: the specular scene loads, the oracle's
specular path is finite, energy-bounded and deterministic, and the scene
renders differently from the Lambertian box (the BSDFs are really used)."""
import json
import os

import numpy as np

from conftest import ROOT
from oracle import oracle as O


def test_specular_scene_oracle():
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import process_primitives, read_file
    d = json.load(open(os.path.join(ROOT, "pyrenderer_amd", "media", "cornell-box", "scene_specular.json")))
    scene, cam = process_primitives(d)
    flat = flatten_scene(scene)
    assert flat.sph.shape == (1, 4)
    np.testing.assert_allclose(flat.sph[0], [0.33, 0.9, 0.37, 0.3], rtol=1e-6)
    c = cam.convert_to_taichi_camera().packed()
    a = O.OracleScene.from_flat(flat).render(c, 32, 32, 8, 8, seed=1)
    b = O.OracleScene.from_flat(flat).render(c, 32, 32, 8, 8, seed=1)
    np.testing.assert_array_equal(a, b)
    assert np.isfinite(a).all() and a.min() >= 0
    s2, c2 = read_file(os.path.join(ROOT, "pyrenderer_amd", "media", "cornell-box", "scene.json"))
    lam = O.OracleScene.from_flat(flatten_scene(s2)).render(c, 32, 32, 8, 8, seed=1)
    assert not np.array_equal(a, lam)
    # the image mean stays within the Lambertian box's order of magnitude
    assert 0.2 < a.mean() / lam.mean() < 5
