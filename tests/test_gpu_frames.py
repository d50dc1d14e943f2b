"""Multi-frame launches (prt_render_frames_device): several frames' (pixel, sample) items run
through the same persistent trace launches — the progressive frame loop of main_taichi.py:108-118
without a launch drain between frames.  Every frame must equal, bit for bit, the render of its own
samples (prt_render_tiles for repeated frames, prt_render_tiles_accumulate from zero sums for
progressive ones) and, on a sample, the CPU oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frames(ds, packed, W, H, tile, tiles, spp, depth, n, stride, seed, flags=0):
    import torch
    from pyrenderer_amd import _native as N
    n_slots = len(tiles) * tile * tile
    out = torch.full((n, n_slots * 3), float("nan"), dtype=torch.float32, device="cuda:0")
    ds.kernel_timing()                              # reset the launch events
    ds.render_frames_device(packed, W, H, tile, tile, tiles, spp, depth, n, out.data_ptr(), None, seed=seed,
                            frame_stride=stride, flags=flags | N.PRT_FLAG_TIME)
    _, launches = ds.kernel_timing()                # synchronises, checks the watchdog
    return out.cpu().numpy().reshape(n, n_slots, 3), launches


@pytest.mark.parametrize("stride", [0, "spp"])
def test_frames_in_one_launch_match_single_renders(gpu_scene, cornell, oracle_scene, stride):
    from pyrenderer_amd.device_scene import interleaved_tiles
    scene, cam, flat = cornell
    packed = cam.convert_to_taichi_camera().packed()
    W, H, tile, spp, depth, n, seed = 128, 96, 16, 8, 8, 5, 3
    stride = spp if stride == "spp" else 0
    tiles = interleaved_tiles(W, H, tile, 1, 3)     # a ragged shard: the latin tiles of rank 1 of 3
    frames, launches = _frames(gpu_scene, packed, W, H, tile, tiles, spp, depth, n, stride, seed)
    assert launches == 1                            # all five frames in one persistent launch
    for f in range(n):
        if stride == 0:
            ref, _ = gpu_scene.render_tiles(packed, W, H, tile, tile, tiles, spp, depth, seed=seed)
        else:
            ref = np.zeros_like(frames[f])
            gpu_scene.render_tiles_accumulate(packed, W, H, tile, tile, tiles, f * stride, spp, depth, ref, seed=seed)
        assert np.array_equal(frames[f], ref), f
    if stride:
        assert not np.array_equal(frames[0], frames[1])   # progressive frames: new samples each
    # frame 0 against the CPU oracle on a few tiles
    ids = tiles[:6]
    cpu = oracle_scene.render_tiles(packed, W, H, tile, tile, ids, spp, depth, seed=seed)
    assert np.array_equal(frames[0][:len(ids) * tile * tile], cpu)


def test_frames_split_across_launches_by_the_buffer_budget(cornell, monkeypatch):
    """A per-launch budget smaller than the frames' buffers splits them over several launches, with
    launch boundaries inside frames (partial reduces that continue a frame's sums): same frames."""
    from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles
    scene, cam, flat = cornell
    packed = cam.convert_to_taichi_camera().packed()
    W, H, tile, spp, depth, n, seed = 64, 64, 8, 6, 4, 4, 9
    tiles = interleaved_tiles(W, H, tile)
    # 28 B per sample of a 4096-pixel frame: 1 MiB holds 9 samples, so 24 samples take 3 launches of 8
    monkeypatch.setenv("PRT_CHUNK_BYTES", str(1 << 20))
    ds = DeviceScene(flat, 0)
    try:
        frames, launches = _frames(ds, packed, W, H, tile, tiles, spp, depth, n, spp, seed)
        assert launches == 3
        for f in range(n):
            ref = np.zeros_like(frames[f])
            ds.render_tiles_accumulate(packed, W, H, tile, tile, tiles, f * spp, spp, depth, ref, seed=seed)
            assert np.array_equal(frames[f], ref), f
    finally:
        ds.close()


def test_frames_argument_checks(gpu_scene, cornell):
    import torch
    from pyrenderer_amd._native import PrtError
    scene, cam, flat = cornell
    packed = cam.convert_to_taichi_camera().packed()
    out = torch.zeros(2 * 64 * 3, dtype=torch.float32, device="cuda:0")
    for n, stride, pitch in ((0, 0, 0), (2, -1, 0), (2, 1, 64 * 3 - 1)):
        with pytest.raises(PrtError):
            gpu_scene.render_frames_device(packed, 8, 8, 8, 8, [0], 1, 1, n, out.data_ptr(), frame_stride=stride,
                                           out_pitch=pitch)


@pytest.mark.parametrize("world", [3, 5])
def test_ragged_shard_frames_land_in_their_gather_rows(gpu_scene, cornell, oracle_scene, world):
    """a rank owning fewer tiles than the gather slot (max_tiles) renders F > 1
    frames straight into TileShard.bufs at the slot's pitch (bench.py's call): every frame f sits in
    row f, equal to the render of its own samples, and the padding after the rank's tiles is untouched."""
    import torch
    from pyrenderer_amd.distributed import TileShard
    scene, cam, flat = cornell
    packed = cam.convert_to_taichi_camera().packed()
    W = H = 128
    tile, spp, depth, F, seed = 16, 4, 4, 4, 5
    sh = None
    for r in range(world):
        s = TileShard(W, H, tile, r, world, torch.device("cuda", 0), frames=F)
        if len(s.tiles) < s.max_tiles:
            sh = s
            break
    assert sh is not None, "no ragged rank"
    sh.bufs.fill_(float("nan"))
    n = len(sh.tiles) * tile * tile * 3
    gpu_scene.render_frames_device(packed, W, H, tile, tile, sh.tiles, spp, depth, F, sh.bufs.data_ptr(), None,
                                   seed=seed, frame_stride=spp, out_pitch=sh.pitch)
    gpu_scene.check_faults()
    bufs = sh.bufs.cpu().numpy()
    for f in range(F):
        ref = np.zeros((len(sh.tiles) * tile * tile, 3), np.float32)
        gpu_scene.render_tiles_accumulate(packed, W, H, tile, tile, sh.tiles, f * spp, spp, depth, ref, seed=seed)
        assert np.array_equal(bufs[f, :n].reshape(-1, 3), ref), f
        assert np.isnan(bufs[f, n:]).all(), f          # the slot's padding is not written
    cpu = oracle_scene.render_tiles(packed, W, H, tile, tile, sh.tiles[:2], spp, depth, seed=seed)
    assert np.array_equal(bufs[0, :2 * tile * tile * 3].reshape(-1, 3), cpu)


def test_in_kernel_camera_flag_is_rejected(gpu_scene, cornell):
    """PRT_FLAG_NO_PRIMARY_KERNEL is gone from the trace kernels (round 4): an explicit error, not a
    silently different path."""
    import torch
    from pyrenderer_amd._native import PrtError, PRT_FLAG_NO_PRIMARY_KERNEL, PRT_ERR_UNSUP
    scene, cam, flat = cornell
    packed = cam.convert_to_taichi_camera().packed()
    out = torch.zeros(64 * 3, dtype=torch.float32, device="cuda:0")
    with pytest.raises(PrtError) as e:
        gpu_scene.render_frames_device(packed, 8, 8, 8, 8, [0], 1, 1, 1, out.data_ptr(),
                                       flags=PRT_FLAG_NO_PRIMARY_KERNEL)
    assert e.value.code == PRT_ERR_UNSUP
