"""GPU parity of the SURVEY.md §8(b) window / multi-device entry points of the C-ABI:
prt_render (one window of the frame) and prt_render_multi (tiles over the devices of
one process, RCCL send/recv group to the root).

Both must equal the CPU oracle (oracle/prt_oracle.c) and the tile renders of the same
frame bit for bit: random numbers are keyed by (seed, global pixel, sample), so neither
the window nor the device count may change a pixel.  The one-GPU box exercises
prt_render_multi with one device, whose root still moves its tiles through RCCL (a
send/recv self-loop), so the communicator, the group and the root's scatter all run.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _full(ds, cam, W, H, spp, depth, seed):
    from pyrenderer_amd.device_scene import interleaved_tiles, unpack_tiles
    ids = interleaved_tiles(W, H, 64)
    sums, _ = ds.render_tiles(cam, W, H, 64, 64, ids, spp, depth, seed)
    return unpack_tiles(sums, W, H, 64, 64, ids)


@pytest.mark.parametrize("x0,y0,w,h", [(0, 0, 100, 70),      # whole (ragged) frame
                                       (13, 5, 37, 50),      # unaligned window
                                       (99, 69, 1, 1),       # last pixel
                                       (8, 16, 64, 8)])      # tile-aligned strip
def test_window_is_crop_of_frame_and_oracle(gpu_scene, oracle_scene, cornell, x0, y0, w, h):
    cam = cornell[1].convert_to_taichi_camera().packed()
    W, H, spp, depth, seed = 100, 70, 3, 8, 11
    full = _full(gpu_scene, cam, W, H, spp, depth, seed)
    win, _ = gpu_scene.render_window(cam, W, H, x0, y0, w, h, spp, depth, seed)
    assert win.shape == (w, h, 3)
    np.testing.assert_array_equal(win, full[x0:x0 + w, y0:y0 + h])
    ora = oracle_scene.render(cam, W, H, spp, depth, seed=seed)
    np.testing.assert_array_equal(win, ora[x0:x0 + w, y0:y0 + h])


def test_window_stats_and_errors(gpu_scene, cornell):
    from pyrenderer_amd._native import PRT_FLAG_STATS, PrtError
    cam = cornell[1].convert_to_taichi_camera().packed()
    _, st = gpu_scene.render_window(cam, 64, 64, 0, 0, 64, 64, 2, 8, 3, PRT_FLAG_STATS)
    assert st[2] >= 64 * 64 * 2 and st[0] > 0
    z, _ = gpu_scene.render_window(cam, 64, 64, 4, 4, 9, 9, 0, 8)
    assert not z.any()
    for x0, y0, w, h in [(0, 0, 65, 64), (-1, 0, 4, 4), (0, 0, 0, 4), (60, 60, 5, 1)]:
        with pytest.raises(PrtError):
            gpu_scene.render_window(cam, 64, 64, x0, y0, w, h, 1, 1)


@pytest.mark.parametrize("W,H,tile,spp,depth", [(128, 128, 64, 4, 4),   # config 1
                                                (100, 70, 16, 3, 8),    # ragged tiles
                                                (512, 512, 64, 2, 8)])  # config 2 frame
def test_render_multi_one_device_through_rccl(gpu_scene, oracle_scene, cornell, W, H, tile, spp, depth):
    from pyrenderer_amd.device_scene import render_multi
    cam = cornell[1].convert_to_taichi_camera().packed()
    m = render_multi([gpu_scene], cam, W, H, tile, spp, depth, seed=5)
    np.testing.assert_array_equal(m, _full(gpu_scene, cam, W, H, spp, depth, 5))
    if W * H <= 128 * 128:
        np.testing.assert_array_equal(m, oracle_scene.render(cam, W, H, spp, depth, seed=5))


def test_render_multi_rejects_shared_device(gpu_scene, cornell):
    from pyrenderer_amd._native import PrtError
    from pyrenderer_amd.device_scene import DeviceScene, render_multi
    other = DeviceScene(cornell[2], 0)
    cam = cornell[1].convert_to_taichi_camera().packed()
    with pytest.raises(PrtError, match="distinct devices"):
        render_multi([gpu_scene, other], cam, 64, 64, 64, 1, 1)
    other.close()


def test_tracing_render_all_devices(cornell, oracle_scene):
    """core.tracing.render over every visible device (prt_render_multi when > 1) equals the
    oracle's mean image."""
    from pyrenderer_amd._native import device_count
    from pyrenderer_amd.core.tracing import render
    scene, camera, _ = cornell
    devs = tuple(range(device_count()))
    mean = render(scene, camera, spp=2, depth=8, seed=9, resolution=(96, 64), devices=devs)
    cam = camera.convert_to_taichi_camera().packed()
    np.testing.assert_array_equal(mean, oracle_scene.render(cam, 96, 64, 2, 8, seed=9) / np.float32(2))


def test_cli_progressive_resume_equals_one_render(tmp_path, cornell):
    """python -m pyrenderer_amd (main_taichi.py's loop without the GUI): progressive passes
    with a saved / resumed accumulation give the one-shot render's image bit for bit, and
    the PNG is written."""
    from pyrenderer_amd.core.tracing import render
    from pyrenderer_amd.main import main
    state = str(tmp_path / "acc.npz")
    common = ["--resolution", "48", "32", "--depth", "8", "--seed", "3"]
    main(common + ["--samples", "3", "--interval", "2", "--state", state, "--out", ""])
    mean = main(common + ["--samples", "6", "--interval", "2", "--state", state,
                          "--out", str(tmp_path / "o.png"), "--hdr", str(tmp_path / "hdr")])
    ref = render(cornell[0], cornell[1], spp=6, depth=8, seed=3, resolution=(48, 32))
    np.testing.assert_array_equal(mean, ref)
    # the reference's HDR pair: radiance sums + per-pixel sample counts (main_taichi.py:120-123)
    hdr, spp = np.load(tmp_path / "hdr" / "hdr.npy"), np.load(tmp_path / "hdr" / "spp.npy")
    assert hdr.shape == (48, 32, 3) and spp.shape == (48, 32) and (spp == 6).all()
    np.testing.assert_array_equal(hdr / spp[0, 0], ref)
    m1 = main(common + ["--samples", "5", "--out", "", "--hdr", str(tmp_path / "one")])
    np.testing.assert_array_equal(np.load(tmp_path / "one" / "hdr.npy") / np.float32(5), m1)
    assert (tmp_path / "o.png").read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"
    m2 = main(common + ["--samples", "2", "--nee", "mis", "--out", "", "--tonemap", "reinhard"])
    assert np.isfinite(m2).all() and not np.array_equal(m2, render(cornell[0], cornell[1], spp=2, depth=8, seed=3,
                                                                     resolution=(48, 32)))


def test_cli_resume_state_path_and_mismatches(tmp_path, cornell):
    """a --state path without '.npz' must resume (np.savez appends the suffix),
    a resumed run must refuse other --depth / --seed / --resolution / --nee, and
    Accumulator.load must refuse another camera or scene."""
    import pytest
    from pyrenderer_amd.core.tracing import Accumulator, render
    from pyrenderer_amd.main import main
    state = str(tmp_path / "acc")                      # no suffix
    common = ["--resolution", "48", "32", "--depth", "6", "--seed", "4"]
    main(common + ["--samples", "2", "--state", state, "--out", ""])
    assert (tmp_path / "acc.npz").exists()
    mean = main(common + ["--samples", "5", "--state", state, "--out", ""])
    np.testing.assert_array_equal(mean, render(cornell[0], cornell[1], spp=5, depth=6, seed=4, resolution=(48, 32)))
    for bad in (["--depth", "7"], ["--seed", "5"], ["--nee", "mis"]):
        args = common + ["--samples", "8", "--state", state, "--out", ""] + bad
        with pytest.raises(SystemExit, match="other settings"):
            main(args)
    with pytest.raises(SystemExit, match="other settings"):
        main(["--resolution", "32", "32", "--depth", "6", "--seed", "4", "--samples", "8", "--state", state,
              "--out", ""])
    scene, camera, _ = cornell
    import copy
    moved = copy.deepcopy(camera)
    moved.iview = moved.iview.copy()
    moved.iview[0, 3] += 0.25
    with pytest.raises(ValueError, match="camera"):
        Accumulator.load(state, scene, moved)
    from test_multi_light import _scene_json
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    other, ocam = read_file(_scene_json(tmp_path))
    with pytest.raises(ValueError, match="scene"):
        Accumulator.load(state, other, camera)
