"""world_size 2 / 3 / 8 gloo runs of the tile-shard + gather path on CPU (the oracle
stands in for the GPU renderer): the gathered frame equals the single-process
frame bit for bit — including the driver's N = 8 layout and a frame with fewer tiles
than ranks (ranks with no tile still join the gather with an empty shard)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import CORNELL_JSON, ROOT

W, H, TILE, SPP, DEPTH, SEED = 40, 36, 16, 2, 4, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path, W=W, H=H):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    from pyrenderer_amd.distributed import TileShard
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    scene, cam = read_file(CORNELL_JSON)
    osc = O.OracleScene.from_flat(flatten_scene(scene))
    shard = TileShard(W, H, TILE, rank, world, torch.device("cpu"))
    sums = osc.render_tiles(cam.convert_to_taichi_camera().packed(), W, H, TILE, TILE, shard.tiles, SPP, DEPTH,
                            seed=SEED, nthreads=1)
    shard.buf[:sums.size] = torch.from_numpy(sums.reshape(-1))
    shard.gather()
    if rank == 0:
        np.save(out_path, shard.assemble())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world, W, H", [(2, W, H), (3, W, H), (8, W, H), (8, 32, 24)])
def test_gather_matches_single_process(tmp_path, world, W, H):
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), out, W, H), nprocs=world, join=True)
    frame = np.load(out)
    from oracle import oracle as O
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    scene, cam = read_file(CORNELL_JSON)
    ref = O.OracleScene.from_flat(flatten_scene(scene)).render(cam.convert_to_taichi_camera().packed(), W, H, SPP,
                                                                DEPTH, seed=SEED, tile=TILE)
    np.testing.assert_array_equal(frame, ref)
    assert frame.sum() > 0


def _frames_worker(rank, world, port, out_path, n_frames, coll=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    from pyrenderer_amd.distributed import TileShard
    shard = TileShard(W, H, TILE, rank, world, torch.device("cpu"), frames=n_frames, collective=coll)
    assert shard.coll == (world > 1 or coll) and (shard.gathered is not None) == (rank == 0 and shard.coll)
    # frame f's sums of pixel (x, y): a value that names both, so a mixed-up frame or tile shows
    n = len(shard.tiles) * TILE * TILE
    for f in range(n_frames):
        vals = np.zeros((n, 3), np.float32)
        for k, t in enumerate(shard.tiles):
            tx, ty = t % ((W + TILE - 1) // TILE), t // ((W + TILE - 1) // TILE)
            for j in range(TILE * TILE):
                x, y = tx * TILE + j % TILE, ty * TILE + j // TILE
                vals[k * TILE * TILE + j] = (x, y, f) if (x < W and y < H) else 0.0
        shard.bufs[f, :n * 3] = torch.from_numpy(vals.reshape(-1))
    shard.gather(n_frames=n_frames)
    if rank == 0:
        np.save(out_path, np.stack([shard.assemble(f=f) for f in range(n_frames)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world, coll", [(1, True), (2, False), (3, False)])
def test_multi_frame_gathers(tmp_path, world, coll):
    """bench.py's multi-frame groups: F frames' tile sums per rank, one gather per frame, each
    frame assembled from its own gathered buffer.  World 1 with `collective` is bench.py
    --force-collective's path: a one-rank group still gathers into rank 0's buffer and assembles
    from it."""
    out = str(tmp_path / "frames.npy")
    F = 3
    mp.spawn(_frames_worker, args=(world, _free_port(), out, F, coll), nprocs=world, join=True)
    frames = np.load(out)
    assert frames.shape == (F, W, H, 3)
    x, y = np.meshgrid(np.arange(W), np.arange(H), indexing="ij")
    for f in range(F):
        np.testing.assert_array_equal(frames[f][..., 0], x)
        np.testing.assert_array_equal(frames[f][..., 1], y)
        assert np.all(frames[f][..., 2] == f)
