"""The traversal stacks are sized to the BVH4's exact bound (prt_bvh.cpp collapse_bvh4: 1 + the
pushed siblings of the deepest node's ancestors + the <= 3 slots a visit writes above the top), and
the pooled kernel's LDS stack is exactly that bound with nothing bounds-checked behind it — an
overflow would silently overwrite the shadow pool.  Here the measured maximum depth (diag word 13,
PRT_FLAG_STATS) of a full render stays within the bound for both BVH4 collapses (SAH-optimal dynamic
program, PRT_BVH4_DP=1, the default, and the greedy one, PRT_BVH4_DP=0) on the LDS-resident scenes
(ADVICE r03)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dp", ["1", "0"])
@pytest.mark.parametrize("name", ["cornell", "specular"])
def test_stack_depth_within_the_collapse_bound(name, dp, monkeypatch):
    from pyrenderer_amd import _native as N
    from pyrenderer_amd import scenes
    from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    monkeypatch.setenv("PRT_BVH4_DP", dp)    # read at scene creation
    scene, cam = read_file(scenes.CORNELL if name == "cornell" else scenes.CORNELL_SPECULAR)
    ds = DeviceScene(flatten_scene(scene), 0)
    try:
        packed = cam.convert_to_taichi_camera().packed()
        W = H = 256
        tiles = interleaved_tiles(W, H, 64)
        for var in N.VAR_POOL + (N.VAR_LDS,):
            flags = N.PRT_FLAG_STATS | (var << 8)
            info = ds.kernel_info(n_items=W * H * 32, flags=flags)
            assert info["variant"] == var
            ds.render_tiles(packed, W, H, 64, 64, tiles, 32, 8, seed=1, flags=flags)
            deepest = int(ds.diag_stats()[13])
            assert 1 <= deepest <= info["stack"], (name, dp, var, deepest, info)
    finally:
        ds.close()
