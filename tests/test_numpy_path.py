"""The NumPy restatement of main.py's path (oracle/numpy_path.py, bench.py's cpu_numpy
baseline) against the C oracle: identical per-pixel sums, to the last bit, on the same
seeded inputs (the C oracle is itself pinned to the reference's vectors)."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import numpy_path as NP


@pytest.mark.parametrize("W,H,spp,depth,seed", [(128, 128, 4, 4, 0),   # config 1 (BASELINE configs[0])
                                                (48, 40, 4, 8, 3),     # config 2's estimator, ragged tiles
                                                (24, 24, 2, 16, 7)])   # reference default depth
def test_numpy_path_matches_c_oracle(cornell, oracle_scene, W, H, spp, depth, seed):
    cam = cornell[1].convert_to_taichi_camera().packed()
    tiles = np.arange(((W + 7) // 8) * ((H + 7) // 8), dtype=np.int32)
    a = NP.NumpyScene(cornell[2]).render_tiles(cam, W, H, 8, 8, tiles, spp, depth, seed)
    b = oracle_scene.render_tiles(cam, W, H, 8, 8, tiles, spp, depth, seed)
    assert np.isfinite(a).all() and a.any()
    np.testing.assert_array_equal(a, b)


def test_rng_streams_match_c_oracle():
    keys = NP.rng_key(5 | (9 << 32), np.arange(64, dtype=np.uint32), 3)
    for k in (0, 17, 63):
        assert int(keys[k]) == int(O.rng_key(5 | (9 << 32), k, 3))
        st = np.array([keys[k]], np.uint32)
        got = [float(NP._rng_next(st, np.array([0]))[0]) for _ in range(6)]
        np.testing.assert_array_equal(np.float32(got), O.rng_draws(int(keys[k]), 6))


def test_timed_sample_in_worker_processes(cornell, oracle_scene):
    cam = cornell[1].convert_to_taichi_camera().packed()
    ids, sums, wall = NP.timed_sample(cornell[2], cam, 64, 64, 2, 4, 1, 0.2, 2)
    assert wall > 0 and sums.shape == (len(ids) * 64, 3)
    np.testing.assert_array_equal(sums, oracle_scene.render_tiles(cam, 64, 64, 8, 8, ids, 2, 4, seed=1))


def test_scope_is_enforced():
    flat = dict(tri_v=np.zeros((1, 9), np.float32), tri_n=np.zeros((1, 3), np.float32),
                tri_mat=np.zeros(1, np.int32), mat=np.array([[1, 1, 1, 0, 0, 2, 1.5, 0]], np.float32),
                light_tri=np.zeros(1, np.int32), light_off=np.array([0, 1], np.int32),
                direct_rgb=np.ones(3, np.float32))
    with pytest.raises(NotImplementedError):
        NP.NumpyScene(flat)


def test_large_scenes_are_out_of_scope():
    big = dict(tri_v=np.zeros((NP.MAX_TRIANGLES + 1, 9), np.float32), tri_n=np.zeros((NP.MAX_TRIANGLES + 1, 3), np.float32),
               tri_mat=np.zeros(NP.MAX_TRIANGLES + 1, np.int32), mat=np.array([[1, 1, 1, 0, 0, 0, 1.5, 0]], np.float32),
               light_tri=np.zeros(1, np.int32), light_off=np.array([0, 1], np.int32), direct_rgb=np.ones(3, np.float32))
    with pytest.raises(NotImplementedError):
        NP.NumpyScene(big)
