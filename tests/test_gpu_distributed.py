"""The torch.distributed path with the HIP renderer, and failure
detection on the device-output path.

* world_size 2 over gloo: both ranks build their own scene handle on device 0, render
  their latin-interleaved tiles with the HIP kernel into device buffers
  (pyrenderer_amd.distributed.render_distributed), stage them through host memory and
  gather to rank 0.  The frame must equal the single-process render and the oracle bit
  for bit (random numbers are keyed by the global pixel, so sharding cannot change a bit).
* The traversal watchdog (prt_device.h traverse_ww4) lowered to one traversal phase per
  query with PRT_GUARD_TRIPS=1 trips on any real scene: every entry point must report it —
  the host-output render, prt_check_faults after a device-output render, and
  render_distributed (which previously returned the frame unchecked).
"""
import os
import socket

import numpy as np
import pytest

from conftest import CORNELL_JSON, ROOT

pytestmark = pytest.mark.gpu

W, H, TILE, SPP, DEPTH, SEED = 160, 96, 32, 4, 8, 21


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pyrenderer_amd.device_scene import DeviceScene
    from pyrenderer_amd.distributed import render_distributed
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    scene, cam = read_file(CORNELL_JSON)
    ds = DeviceScene(flatten_scene(scene), 0)
    img = render_distributed(ds, cam.convert_to_taichi_camera().packed(), W, H, SPP, DEPTH, seed=SEED, tile=TILE)
    if rank == 0:
        np.save(out_path, img)
    else:
        assert img is None
    dist.barrier()
    dist.destroy_process_group()
    ds.close()


def test_two_ranks_over_gloo_equal_one_process(tmp_path, gpu_scene, oracle_scene, cornell):
    import torch.multiprocessing as mp
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    frame = np.load(out)
    cam = cornell[1].convert_to_taichi_camera().packed()
    ref = oracle_scene.render(cam, W, H, SPP, DEPTH, seed=SEED) / np.float32(SPP)
    np.testing.assert_array_equal(frame, ref)
    from pyrenderer_amd.distributed import render_distributed
    np.testing.assert_array_equal(render_distributed(gpu_scene, cam, W, H, SPP, DEPTH, seed=SEED, tile=TILE), ref)
    assert frame.sum() > 0


def test_render_distributed_under_a_side_stream(gpu_scene, oracle_scene, cornell):
    """A caller-provided stream that is not torch's current stream: the render and the read-back
    are both ordered on it (the gather ran on the current stream)."""
    import torch
    from pyrenderer_amd.distributed import render_distributed
    cam = cornell[1].convert_to_taichi_camera().packed()
    side = torch.cuda.Stream(torch.device("cuda", 0))
    img = render_distributed(gpu_scene, cam, 128, 64, 8, 8, seed=2, tile=64, stream=side)
    np.testing.assert_array_equal(img, oracle_scene.render(cam, 128, 64, 8, 8, seed=2) / np.float32(8))


def test_watchdog_is_reported_on_every_path(cornell, monkeypatch):
    import torch
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    from pyrenderer_amd.distributed import render_distributed
    cam = cornell[1].convert_to_taichi_camera().packed()
    ids = np.arange(4, dtype=np.int32)
    monkeypatch.setenv("PRT_GUARD_TRIPS", "1")
    ds = DeviceScene(cornell[2], 0)
    with pytest.raises(N.PrtError, match="watchdog"):
        ds.render_tiles(cam, 64, 64, 32, 32, ids, 4, 8, 0)
    buf = torch.empty(4 * 32 * 32 * 3, dtype=torch.float32, device="cuda:0")
    ds.render_tiles_device(cam, 64, 64, 32, 32, ids, 4, 8, buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
    with pytest.raises(N.PrtError) as e:
        ds.check_faults()
    assert e.value.code == N.PRT_ERR_INTERNAL
    with pytest.raises(N.PrtError, match="watchdog"):
        render_distributed(ds, cam, 64, 64, 4, 8)
    ds.close()
    # the default limit never trips on a sound tree: same calls, no error
    monkeypatch.delenv("PRT_GUARD_TRIPS")
    ok = DeviceScene(cornell[2], 0)
    ok.render_tiles_device(cam, 64, 64, 32, 32, ids, 4, 8, buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
    ok.check_faults()
    assert render_distributed(ok, cam, 64, 64, 4, 8).sum() > 0
    ok.close()


def test_watchdog_flags_are_reported_once(cornell, monkeypatch):
    """a fault is reported by the call that checks the launch that raised it, then
    cleared — a device-output render on a fresh scene reports its own fault, and a clean
    device-output render after a faulted one (on another stream, or after a faulted hit query)
    is not blamed for it."""
    import torch
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    cam = cornell[1].convert_to_taichi_camera().packed()
    ids = np.arange(4, dtype=np.int32)
    buf = torch.empty(4 * 32 * 32 * 3, dtype=torch.float32, device="cuda:0")
    monkeypatch.setenv("PRT_GUARD_TRIPS", "1")
    ds = DeviceScene(cornell[2], 0)
    side = torch.cuda.Stream(torch.device("cuda", 0))
    # only a device-output render on the fresh scene: its fault is reported
    ds.render_tiles_device(cam, 64, 64, 32, 32, ids, 4, 8, buf.data_ptr(), side.cuda_stream)
    with pytest.raises(N.PrtError) as e:
        ds.check_faults()
    assert e.value.code == N.PRT_ERR_INTERNAL
    ds.check_faults()                     # reported once: nothing new since
    # a faulted render on one stream, then a clean (no-work) render on another
    ds.render_tiles_device(cam, 64, 64, 32, 32, ids, 4, 8, buf.data_ptr(), side.cuda_stream)
    with pytest.raises(N.PrtError):
        ds.check_faults()
    ds.render_tiles_device(cam, 64, 64, 32, 32, ids, 0, 8, buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
    ds.check_faults()
    # a faulted hit query (reported by the query itself), then a clean device-output render
    rng = np.random.default_rng(0)
    o = rng.uniform((-0.9, 0.1, -0.9), (0.9, 1.9, 0.9), (4096, 3)).astype(np.float32)
    d = rng.normal(size=(4096, 3)).astype(np.float32)
    with pytest.raises(N.PrtError, match="watchdog"):
        ds.closest_hits(o, d, 1e-5, 99999.9)
    ds.render_tiles_device(cam, 64, 64, 32, 32, ids, 0, 8, buf.data_ptr(), side.cuda_stream)
    ds.check_faults()
    ds.close()
