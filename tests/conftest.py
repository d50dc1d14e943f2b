import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
CORNELL_JSON = os.path.join(ROOT, "pyrenderer_amd", "media", "cornell-box", "scene.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libprt's HIP path)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def cornell():
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    scene, cam = read_file(CORNELL_JSON)
    flat = flatten_scene(scene)
    return scene, cam, flat


@pytest.fixture(scope="session")
def oracle_scene(cornell):
    from oracle import oracle as O
    return O.OracleScene.from_flat(cornell[2])


@pytest.fixture(scope="session")
def gpu_scene(cornell):
    from pyrenderer_amd.device_scene import DeviceScene
    return DeviceScene(cornell[2], 0)
