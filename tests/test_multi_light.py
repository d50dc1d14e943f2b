"""Scenes with several emitters: World.sample_a_light's randInt over lights
(intersection_taichi.py:194-207) then Quad/Cube.sample_a_point's randInt over the
chosen light's faces (shapes.py:62-71, :188-197).  The Cornell box has one light, so
these paths are exercised here with a second emitting quad and an emitting cube added
to the Tungsten JSON (read_file -> flatten -> kernel / oracle / NumPy path)."""
import copy
import json

import numpy as np
import pytest

from conftest import CORNELL_JSON
from oracle import oracle as O
from oracle import numpy_path as NP


def _scene_json(tmp_path):
    d = json.load(open(CORNELL_JSON))
    lights = [p for p in d["primitives"] if p.get("bsdf") == "Light"]
    q = copy.deepcopy(lights[0])
    q["transform"]["position"] = [0.45, 1.6, 0.2]          # a second, lower light quad
    c = {"transform": {"position": [-0.6, 1.7, 0.5], "scale": [0.1, 0.1, 0.1], "rotation": [0, 30, 0]},
         "type": "cube", "bsdf": "Light"}                 # and an emitting cube (12 faces)
    d["primitives"] += [q, c]
    p = tmp_path / "scene.json"
    p.write_text(json.dumps(d))
    return str(p)


@pytest.fixture
def multi(tmp_path):
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    scene, cam = read_file(_scene_json(tmp_path))
    return scene, cam, flatten_scene(scene)


def test_three_lights_are_flattened(multi):
    flat = multi[2]
    assert flat.n_light == 3
    assert np.diff(flat.light_off).tolist() == [2, 2, 12]


def test_numpy_path_matches_oracle_with_three_lights(multi):
    cam = multi[1].convert_to_taichi_camera().packed()
    ids = np.arange(16, dtype=np.int32)
    a = NP.NumpyScene(multi[2]).render_tiles(cam, 32, 32, 8, 8, ids, 4, 8, seed=3)
    b = O.OracleScene.from_flat(multi[2]).render_tiles(cam, 32, 32, 8, 8, ids, 4, 8, seed=3)
    np.testing.assert_array_equal(a, b)
    one = O.OracleScene.from_flat(_one_light_reference()).render_tiles(cam, 32, 32, 8, 8, ids, 4, 8, seed=3)
    assert not np.array_equal(b, one)


def _one_light_reference():
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    return flatten_scene(read_file(CORNELL_JSON)[0])


@pytest.mark.gpu
def test_gpu_matches_oracle_with_three_lights(multi):
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    cam = multi[1].convert_to_taichi_camera().packed()
    ds = DeviceScene(multi[2], 0)
    osc = O.OracleScene.from_flat(multi[2])
    ids = np.arange(6, dtype=np.int32)
    o = osc.render_tiles(cam, 96, 64, 32, 32, ids, 4, 8, seed=8)
    g, _ = ds.render_tiles(cam, 96, 64, 32, 32, ids, 4, 8, 8)
    np.testing.assert_array_equal(g, o)
    # the global-scene kernel and the MIS estimator over the same lights
    g2, _ = ds.render_tiles(cam, 96, 64, 32, 32, ids, 4, 8, 8, N.VAR_GLOBAL << 8)
    np.testing.assert_array_equal(g2, o)
    O.set_nee_mode(True)
    try:
        om = osc.render_tiles(cam, 96, 64, 32, 32, ids, 2, 8, seed=8)
    finally:
        O.set_nee_mode(False)
    gm, _ = ds.render_tiles(cam, 96, 64, 32, 32, ids, 2, 8, 8, N.PRT_FLAG_MIS_NEE)
    np.testing.assert_array_equal(gm, om)
    ds.close()
