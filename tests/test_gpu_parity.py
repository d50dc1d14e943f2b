"""GPU parity: libprt's HIP path (through the C-ABI) against the CPU oracle on the
same seeded inputs.

Tolerance (north star): per-pixel L2 of mean linear radiance, RMSE < 1e-3.
The arithmetic contract makes the two bit-identical, which is
asserted too: >= 99.9% of pixels identical to the last bit (measured: 100%).
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

TOL_RMSE = 1e-3


def _gpu_frame(ds, cam, W, H, spp, depth, seed=0, tile=64, flags=0):
    from pyrenderer_amd.device_scene import interleaved_tiles, unpack_tiles
    ids = interleaved_tiles(W, H, tile)
    sums, _ = ds.render_tiles(cam, W, H, tile, tile, ids, spp, depth, seed, flags=flags)
    return unpack_tiles(sums, W, H, tile, tile, ids)


def _compare(gpu_sum, ora_sum, spp):
    g = gpu_sum / np.float32(spp)
    o = ora_sum / np.float32(spp)
    rmse = float(np.sqrt(np.mean((g - o) ** 2)))
    same = np.all(gpu_sum == ora_sum, axis=-1).mean()
    return rmse, same


@pytest.mark.parametrize("W,H,spp,depth", [(128, 128, 4, 4),     # config 1 (BASELINE.json configs[0])
                                           (64, 64, 8, 8),       # config 2's estimator at small size
                                           (100, 70, 3, 16)])    # ragged tiles, reference default depth
def test_cornell_matches_oracle(gpu_scene, oracle_scene, cornell, W, H, spp, depth):
    cam = cornell[1].convert_to_taichi_camera().packed()
    g = _gpu_frame(gpu_scene, cam, W, H, spp, depth, seed=7)
    o = oracle_scene.render(cam, W, H, spp, depth, seed=7)
    assert np.isfinite(g).all()
    rmse, same = _compare(g, o, spp)
    assert rmse < TOL_RMSE, rmse
    assert same >= 0.999, same


def test_counters_match_oracle(gpu_scene, oracle_scene, cornell):
    """Extension / shadow query counts are a deterministic function of the paths."""
    from pyrenderer_amd._native import PRT_FLAG_STATS
    cam = cornell[1].convert_to_taichi_camera().packed()
    ids = np.arange(4, dtype=np.int32)
    _, st = gpu_scene.render_tiles(cam, 64, 64, 32, 32, ids, 4, 8, 3, PRT_FLAG_STATS)
    _, oc = oracle_scene.render_tiles(cam, 64, 64, 32, 32, ids, 4, 8, seed=3, counters=True)
    assert st[2] == oc[2] and st[3] == oc[3], (st, oc)
    assert st[0] > 0 and st[1] > 0


def test_tiling_and_sharding_invariance(gpu_scene, cornell):
    """RNG keyed by global pixel: tile size and tile order do not change a bit."""
    from pyrenderer_amd.device_scene import interleaved_tiles, unpack_tiles
    cam = cornell[1].convert_to_taichi_camera().packed()
    a = _gpu_frame(gpu_scene, cam, 96, 80, 4, 8, seed=5, tile=64)
    b = _gpu_frame(gpu_scene, cam, 96, 80, 4, 8, seed=5, tile=16)
    np.testing.assert_array_equal(a, b)
    # 3 "ranks" with interleaved 16x16 tiles, rendered separately, reassembled
    frame = np.zeros_like(a)
    for r in range(3):
        ids = interleaved_tiles(96, 80, 16, r, 3)[::-1].copy()
        s, _ = gpu_scene.render_tiles(cam, 96, 80, 16, 16, ids, 4, 8, 5)
        unpack_tiles(s, 96, 80, 16, 16, ids, frame)
    np.testing.assert_array_equal(frame, a)
    # determinism: same call twice
    np.testing.assert_array_equal(_gpu_frame(gpu_scene, cam, 96, 80, 4, 8, seed=5), a)
    # a different seed changes the image
    assert not np.array_equal(_gpu_frame(gpu_scene, cam, 96, 80, 4, 8, seed=6), a)


def test_edge_cases(gpu_scene, oracle_scene, cornell):
    cam = cornell[1].convert_to_taichi_camera().packed()
    z, _ = gpu_scene.render_tiles(cam, 8, 8, 8, 8, np.array([0], np.int32), 0, 8)
    assert not z.any()
    z, _ = gpu_scene.render_tiles(cam, 8, 8, 8, 8, np.array([0], np.int32), 4, 0)
    assert not z.any()
    e, _ = gpu_scene.render_tiles(cam, 8, 8, 8, 8, np.zeros(0, np.int32), 4, 4)
    assert e.shape == (0, 3)
    t, _ = gpu_scene.render_tiles(cam, 2, 2, 8, 8, np.array([0], np.int32), 2, 3)
    t = t.reshape(8, 8, 3)                              # [ly][lx]
    np.testing.assert_array_equal(t[:2, :2].transpose(1, 0, 2), oracle_scene.render(cam, 2, 2, 2, 3, seed=0))
    assert not t[2:].any() and not t[:, 2:].any()       # outside the 2x2 frame stays 0
    from pyrenderer_amd._native import PrtError
    with pytest.raises(PrtError):
        gpu_scene.render_tiles(cam, 8, 8, 8, 8, np.array([5], np.int32), 1, 1)   # tile id out of range
    with pytest.raises(PrtError):
        gpu_scene.render_tiles(cam, 1, 8, 8, 8, np.array([0], np.int32), 1, 1)   # W - 1 == 0


def test_depth1_is_direct_light_only(gpu_scene, oracle_scene, cornell):
    cam = cornell[1].convert_to_taichi_camera().packed()
    g = _gpu_frame(gpu_scene, cam, 48, 48, 4, 1, seed=1)
    o = oracle_scene.render(cam, 48, 48, 4, 1, seed=1)
    np.testing.assert_array_equal(g, o)


def _soup_scene(cornell, n_extra, seed):
    """Cornell + a random triangle soup inside the box (config 4's shape, small)."""
    from pyrenderer_amd.flatten import FlatScene
    f = cornell[2]
    rng = np.random.default_rng(seed)
    c = np.stack([rng.uniform(-0.9, 0.9, n_extra), rng.uniform(0.05, 1.8, n_extra), rng.uniform(-0.9, 0.9, n_extra)], 1)
    tv = (c[:, None, :] + rng.normal(0, 0.03, (n_extra, 3, 3))).astype(np.float32).reshape(-1, 9)
    e1 = tv[:, 3:6] - tv[:, 0:3]
    e2 = tv[:, 6:9] - tv[:, 0:3]
    nn = np.cross(e1.astype(np.float64), e2.astype(np.float64))
    nn = (nn / np.linalg.norm(nn, axis=1, keepdims=True)).astype(np.float32)
    # extra triangles first so the light's triangle ids move
    tri_v = np.concatenate([tv, f.tri_v])
    tri_n = np.concatenate([nn, f.tri_n])
    tri_mat = np.concatenate([np.full(n_extra, 0, np.int32), f.tri_mat])
    tri_prim = np.concatenate([np.zeros(n_extra, np.int32), f.tri_prim + 1])
    lo = np.concatenate([tv.reshape(-1, 3, 3).min(1).min(0)[None], f.prim_lo])
    hi = np.concatenate([tv.reshape(-1, 3, 3).max(1).max(0)[None], f.prim_hi])
    return FlatScene(tri_v, tri_n, tri_mat, tri_prim, lo, hi, f.mat, f.light_tri + n_extra, f.light_off, f.direct_rgb)


@pytest.mark.parametrize("n_extra", [0, 6, 12, 20, 28, 40])
def test_default_variant_reaches_its_occupancy(cornell, n_extra):
    """The default kernel is chosen by how many blocks' LDS fit one CU: the >= 7-waves LDS build
    (variant 1) must actually get 7 blocks per CU, the >= 6-waves one (variant 6) 6, the global
    scene kernel (3) 6 — otherwise an occupancy target would be paid for in registers and not
    collected; an LDS copy too large for six blocks takes the untargeted build (2, <= 5 blocks).
    Each scene also renders bit-identically to the oracle with that variant."""
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    flat = _soup_scene(cornell, n_extra, 11) if n_extra else cornell[2]
    ds = DeviceScene(flat, 0)
    var = ds.kernel_info()["variant"]
    want = {N.VAR_LDS_POOL: (7,), N.VAR_LDS: (7,), N.VAR_LDS6: (6,), N.VAR_GLOBAL: (6,),
            N.VAR_LDS_ANY_OCC: (1, 2, 3, 4, 5)}
    assert var in want, var
    assert ds.blocks_per_cu in want[var], (n_extra, var, ds.blocks_per_cu)
    osc = O.OracleScene.from_flat(flat)
    cam = cornell[1].convert_to_taichi_camera().packed()
    g = _gpu_frame(ds, cam, 32, 32, 2, 6, seed=5)
    o = osc.render(cam, 32, 32, 2, 6, seed=5)
    np.testing.assert_array_equal(g, o)
    ds.close()


def test_default_variants_cover_the_lds_builds(cornell):
    """Among the scenes above, the pooled-shadow kernel (Cornell) and the phase-aligned LDS builds
    (scenes whose pool copy no longer fits seven blocks) are each the default somewhere."""
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    seen = set()
    for n_extra in (0, 6, 12, 20, 28, 40):
        ds = DeviceScene(_soup_scene(cornell, n_extra, 11) if n_extra else cornell[2], 0)
        seen.add(ds.kernel_info()["variant"])
        ds.close()
    assert N.VAR_LDS_POOL in seen and ({N.VAR_LDS, N.VAR_LDS6} & seen), seen


def test_triangle_soup_matches_oracle(cornell):
    from pyrenderer_amd.device_scene import DeviceScene
    flat = _soup_scene(cornell, 3000, 9)
    ds = DeviceScene(flat, 0)
    assert ds.bvh_depth > 5
    osc = O.OracleScene.from_flat(flat)
    cam = cornell[1].convert_to_taichi_camera().packed()
    g = _gpu_frame(ds, cam, 48, 48, 2, 6, seed=2)
    o = osc.render(cam, 48, 48, 2, 6, seed=2)
    rmse, same = _compare(g, o, 2)
    assert rmse < TOL_RMSE, rmse
    assert same >= 0.999, same


def test_lds_soup_deep_stack_matches_oracle(cornell):
    """A scene still LDS-resident but with a deeper BVH4 than the Cornell box: the octant
    node copies and the 16-bit traversal stack (16 entries) of the LDS kernels, against the
    oracle and against the global-scene kernel on the same scene."""
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    flat = _soup_scene(cornell, 12, 11)
    ds = DeviceScene(flat, 0)
    k = ds.kernel_info()
    assert k["lds_scene"] and k["stack"] >= 16 and ds.bvh_depth > 4, (k, ds.bvh_depth)
    osc = O.OracleScene.from_flat(flat)
    cam = cornell[1].convert_to_taichi_camera().packed()
    g = _gpu_frame(ds, cam, 64, 64, 4, 8, seed=4)
    o = osc.render(cam, 64, 64, 4, 8, seed=4)
    np.testing.assert_array_equal(g, o)
    from pyrenderer_amd.device_scene import interleaved_tiles
    ids = interleaved_tiles(64, 64, 32)
    a, _ = ds.render_tiles(cam, 64, 64, 32, 32, ids, 4, 8, 4, N.VAR_LDS << 8)
    b, _ = ds.render_tiles(cam, 64, 64, 32, 32, ids, 4, 8, 4, N.VAR_GLOBAL << 8)
    np.testing.assert_array_equal(a, b)
    ds.close()


def test_full_size_config2_matches_oracle(gpu_scene, oracle_scene, cornell):
    """BASELINE config 2 at full size (512^2 x 64 spp, depth 8), the WHOLE frame
    against the oracle (brute-force closest hits, all host threads).  At this size
    rare events (e.g. a direction component of exactly 0, ~2^-24 per draw) occur a
    few times, so a sampled check is not enough."""
    import os
    cam = cornell[1].convert_to_taichi_camera().packed()
    W = H = 512
    full = _gpu_frame(gpu_scene, cam, W, H, 64, 8, seed=0)
    assert np.isfinite(full).all() and full.mean() > 0
    nthreads = min(16, len(os.sched_getaffinity(0)))
    o = oracle_scene.render(cam, W, H, 64, 8, seed=0, nthreads=nthreads)
    diff = np.any(full != o, axis=-1)
    assert not diff.any(), (int(diff.sum()), np.argwhere(diff)[:5])


def _specular_scene(rough=0.0, spheres=True):
    import json
    import os
    from conftest import ROOT
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import process_primitives
    d = json.load(open(os.path.join(ROOT, "pyrenderer_amd", "media", "cornell-box", "scene_specular.json")))
    for b in d["bsdfs"]:
        if b["type"] == "metal":
            b["roughness"] = rough
    if not spheres:
        d["primitives"] = [p for p in d["primitives"] if p["type"] != "sphere"]
    scene, cam = process_primitives(d)
    return scene, cam, flatten_scene(scene)


@pytest.mark.parametrize("rough,kernel", [(0.0, "default"), (0.35, "default"), (0.35, "phase")])
def test_specular_scene_matches_oracle(rough, kernel):
    """Config 3's materials (metal, dielectric, sphere) through the C-ABI vs the oracle: the default
    (the pooled kernel's full build) and, forced, the phase-aligned LDS kernel."""
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    scene, cam, flat = _specular_scene(rough)
    assert flat.sph.shape[0] == 1 and (flat.mat[:, 5] == 2).any() and (flat.mat[:, 5] == 3).any()
    ds = DeviceScene(flat, 0)
    osc = O.OracleScene.from_flat(flat)
    c = cam.convert_to_taichi_camera().packed()
    flags = (N.VAR_LDS << 8) if kernel == "phase" else 0
    g = _gpu_frame(ds, c, 64, 64, 4, 8, seed=4, flags=flags)
    o = osc.render(c, 64, 64, 4, 8, seed=4)
    assert np.isfinite(g).all() and g.sum() > 0
    rmse, same = _compare(g, o, 4)
    assert rmse < TOL_RMSE, rmse
    assert same >= 0.999, same


def test_pool_variants_identical_on_the_specular_scene():
    """Both builds of the pooled kernel's full instantiation (spheres, metal, dielectric; 7 and 6 waves
    per SIMD) render the same bits on config 3's materials, and those bits match the oracle as
    test_specular_scene_matches_oracle requires."""
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    scene, cam, flat = _specular_scene(0.35)
    ds = DeviceScene(flat, 0)
    c = cam.convert_to_taichi_camera().packed()
    imgs = {v: _gpu_frame(ds, c, 64, 64, 4, 8, seed=6, flags=v << 8) for v in N.VAR_POOL}
    first = imgs[N.VAR_LDS_POOL]
    for v, g in imgs.items():
        assert np.array_equal(g, first), v
    o = O.OracleScene.from_flat(flat).render(c, 64, 64, 4, 8, seed=6)
    rmse, same = _compare(first, o, 4)
    assert rmse < TOL_RMSE, rmse
    assert same >= 0.999, same


def test_specular_boxes_without_spheres_take_the_full_pooled_build():
    """Metal / dielectric boxes but no sphere: the pooled kernel's lean build (TraceParams::plain)
    must not be chosen — it has no specular code — so the image still matches the oracle."""
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    scene, cam, flat = _specular_scene(0.35, spheres=False)
    assert flat.sph.shape[0] == 0 and (flat.mat[:, 5] == 2).any() and (flat.mat[:, 5] == 3).any()
    ds = DeviceScene(flat, 0)
    osc = O.OracleScene.from_flat(flat)
    c = cam.convert_to_taichi_camera().packed()
    g = _gpu_frame(ds, c, 64, 64, 4, 8, seed=5, flags=N.VAR_LDS_POOL << 8)
    o = osc.render(c, 64, 64, 4, 8, seed=5)
    rmse, same = _compare(g, o, 4)
    assert rmse < TOL_RMSE, rmse
    assert same >= 0.999, same


def test_all_kernel_variants_bit_identical(gpu_scene, oracle_scene, cornell):
    """Every trace-kernel variant of the reference estimator (LDS scene with and without the
    occupancy target, global scene: quantised nodes, spill stack, suspended tails) renders
    the same bits as the oracle."""
    from pyrenderer_amd.device_scene import interleaved_tiles
    cam = cornell[1].convert_to_taichi_camera().packed()
    ids = interleaved_tiles(64, 64, 32)
    o = oracle_scene.render_tiles(cam, 64, 64, 32, 32, ids, 4, 8, seed=2)
    from pyrenderer_amd import _native as N
    for v in N.VAR_REFERENCE:
        g, _ = gpu_scene.render_tiles(cam, 64, 64, 32, 32, ids, 4, 8, 2, v << 8)
        assert np.array_equal(g, o), v


def test_frames_in_flight_on_two_streams(gpu_scene, oracle_scene, cornell):
    """Two renders enqueued on two HIP streams (one render context each) overlap on the
    device and both return the oracle's frame (bench.py --streams 2)."""
    import torch
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import interleaved_tiles, unpack_tiles
    cam = cornell[1].convert_to_taichi_camera().packed()
    W, spp, tile = 128, 8, 64
    ids = interleaved_tiles(W, W, tile)
    o = oracle_scene.render_tiles(cam, W, W, tile, tile, ids, spp, 8, seed=7)
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    outs = [torch.empty(len(ids) * tile * tile * 3, dtype=torch.float32, device=dev) for _ in range(4)]
    for k in range(4):
        v = (N.VAR_GLOBAL if k % 2 else 0) << 8
        gpu_scene.render_tiles_device(cam, W, W, tile, tile, ids, spp, 8, outs[k].data_ptr(),
                                      streams[k % 2].cuda_stream, seed=7, flags=v)
    torch.cuda.synchronize(dev)
    for k in range(4):
        assert np.array_equal(outs[k].cpu().numpy().reshape(-1, 3), o), k


def test_progressive_accumulation_matches_one_render(cornell, oracle_scene, tmp_path):
    """Accumulator (main_taichi.py's progressive loop): samples added over several calls,
    across a save / load, give the sums of one render of all samples, bit for bit."""
    from pyrenderer_amd.core.tracing import Accumulator, render
    scene, camera, _ = cornell
    W, H, depth, seed = 96, 64, 6, 11
    acc = Accumulator(scene, camera, depth=depth, seed=seed, resolution=(W, H))
    acc.add(2).add(3).add(0).add(1)
    assert acc.samples == 6
    cam = camera.convert_to_taichi_camera().packed()
    o6 = oracle_scene.render(cam, W, H, 6, depth, seed=seed)
    assert np.array_equal(acc.sums(), o6)
    assert np.array_equal(acc.mean(), render(scene, camera, spp=6, depth=depth, seed=seed, resolution=(W, H),
                                             world=acc.world))
    path = str(tmp_path / "acc.npz")
    acc.save(path)
    resumed = Accumulator.load(path, scene, camera, world=acc.world)
    resumed.add(2)
    assert resumed.samples == 8
    assert np.array_equal(resumed.sums(), oracle_scene.render(cam, W, H, 8, depth, seed=seed))


def test_tile_set_changes_on_one_stream(gpu_scene, oracle_scene, cornell):
    """A render context re-uploads its tile origins only when the tile set changes:
    alternating tile sets (and sizes) on one stream must each match the oracle."""
    import torch
    from pyrenderer_amd.device_scene import interleaved_tiles
    cam = cornell[1].convert_to_taichi_camera().packed()
    W, spp = 128, 4
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    sets = [(64, interleaved_tiles(W, W, 64, 0, 2)), (64, interleaved_tiles(W, W, 64, 1, 2)),
            (32, interleaved_tiles(W, W, 32, 1, 3)), (64, interleaved_tiles(W, W, 64, 0, 2))]
    outs = []
    for tile, ids in sets:
        buf = torch.empty(len(ids) * tile * tile * 3, dtype=torch.float32, device=dev)
        gpu_scene.render_tiles_device(cam, W, W, tile, tile, ids, spp, 6, buf.data_ptr(), stream.cuda_stream, seed=4)
        outs.append(buf)
    torch.cuda.synchronize(dev)
    for (tile, ids), buf in zip(sets, outs):
        o = oracle_scene.render_tiles(cam, W, W, tile, tile, ids, spp, 6, seed=4)
        assert np.array_equal(buf.cpu().numpy().reshape(-1, 3), o), (tile, list(ids))


@pytest.mark.parametrize("mod", ["aperture", "projective"])
def test_general_camera_matches_oracle(gpu_scene, oracle_scene, cornell, mod):
    """The kernel's pinhole/affine camera shortcut must not change a bit, and the
    general gen_ray (thin-lens draws, non-affine matrix) must match too."""
    cam = cornell[1].convert_to_taichi_camera().packed().copy()
    if mod == "aperture":
        cam[19] = 1.0          # sensor_dim.w > 0: lens sample (camera_taichi.py:57-60)
    else:
        cam[12] = 1e-3         # last matrix row != (0, 0, 0, 1)
    g = _gpu_frame(gpu_scene, cam, 40, 40, 2, 4, seed=3)
    o = oracle_scene.render(cam, 40, 40, 2, 4, seed=3)
    np.testing.assert_array_equal(g, o)


def test_spill_stack_matches_oracle(cornell, oracle_scene, monkeypatch):
    """The global-scene kernel with a 4-entry LDS stack (PRT_SPILL_LDS=4): the Cornell box's
    traversal stack reaches 8 entries, so the global spill area is exercised."""
    from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles
    monkeypatch.setenv("PRT_SPILL_LDS", "4")
    ds = DeviceScene(cornell[2], 0)
    cam = cornell[1].convert_to_taichi_camera().packed()
    ids = interleaved_tiles(64, 64, 32)
    o = oracle_scene.render_tiles(cam, 64, 64, 32, 32, ids, 4, 8, seed=2)
    from pyrenderer_amd import _native as N
    g, _ = ds.render_tiles(cam, 64, 64, 32, 32, ids, 4, 8, 2, N.VAR_GLOBAL << 8)
    assert np.array_equal(g, o)


@pytest.mark.parametrize("variant", ["lds", "global"])
def test_bvh4_collapse_choice_keeps_the_image(cornell, oracle_scene, monkeypatch, variant):
    """The SAH-optimal BVH4 collapse (default) and the greedy one (PRT_BVH4_DP=0) give the
    oracle's image bit for bit, and the optimal one visits no more nodes."""
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene, interleaved_tiles
    cam = cornell[1].convert_to_taichi_camera().packed()
    ids = interleaved_tiles(64, 64, 32)
    o = oracle_scene.render_tiles(cam, 64, 64, 32, 32, ids, 4, 8, seed=5)
    flags = N.PRT_FLAG_STATS | ((N.VAR_GLOBAL << 8) if variant == "global" else 0)
    visits = {}
    for dp in ("0", "1"):
        monkeypatch.setenv("PRT_BVH4_DP", dp)
        ds = DeviceScene(cornell[2], 0)
        g, st = ds.render_tiles(cam, 64, 64, 32, 32, ids, 4, 8, 5, flags)
        assert np.array_equal(g, o), dp
        visits[dp] = int(st[0])
        ds.close()
    assert visits["1"] <= visits["0"], visits


def test_large_frame_matches_oracle(gpu_scene, oracle_scene, cornell):
    """1024^2 x 32 spp (33.5 M samples): contains shadow rays with t_max = NaN
    (p2.x == p.x), which once made BVH4 empty slots (then ref = root) 'hit' and the
    traversal loop forever.  Whole frame against the oracle."""
    import os
    cam = cornell[1].convert_to_taichi_camera().packed()
    W = H = 1024
    g = _gpu_frame(gpu_scene, cam, W, H, 32, 8, seed=0)
    o = oracle_scene.render(cam, W, H, 32, 8, seed=0, nthreads=min(16, len(os.sched_getaffinity(0))))
    diff = np.any(g != o, axis=-1)
    assert not diff.any(), (int(diff.sum()), np.argwhere(diff)[:5])


def test_mis_direct_lighting_variant_matches_oracle(gpu_scene, oracle_scene, cornell):
    """The reference's unused MIS estimator (sample_direct_lighting2, core/tracing.py:57-90)
    as the optional NEE variant: LDS-scene kernel (variant 32) bit-identical to the oracle's
    MIS mode, and different from the default estimator's image."""
    from pyrenderer_amd import _native as N
    cam = cornell[1].convert_to_taichi_camera().packed()
    W, H, spp, depth = 64, 48, 4, 8
    ids = np.arange(((W + 31) // 32) * ((H + 31) // 32), dtype=np.int32)
    O.set_nee_mode(True)
    try:
        o = oracle_scene.render_tiles(cam, W, H, 32, 32, ids, spp, depth, seed=4)
        oc = oracle_scene.render_tiles(cam, W, H, 32, 32, ids, 2, depth, seed=4, counters=True)[1]
    finally:
        O.set_nee_mode(False)
    g, _ = gpu_scene.render_tiles(cam, W, H, 32, 32, ids, spp, depth, 4, N.PRT_FLAG_MIS_NEE)
    assert np.isfinite(g).all() and g.any()
    np.testing.assert_array_equal(g, o)
    _, st = gpu_scene.render_tiles(cam, W, H, 32, 32, ids, 2, depth, 4, N.PRT_FLAG_MIS_NEE | N.PRT_FLAG_STATS)
    assert st[2] == oc[2] and st[3] == oc[3], (st, oc)
    ref, _ = gpu_scene.render_tiles(cam, W, H, 32, 32, ids, spp, depth, 4)
    assert not np.array_equal(g, ref)
    # the global-scene MIS kernel (quantised BVH4, spill stack, resume) gives the same bits
    g2, _ = gpu_scene.render_tiles(cam, W, H, 32, 32, ids, spp, depth, 4, N.PRT_FLAG_MIS_NEE | (N.VAR_MIS[1] << 8))
    np.testing.assert_array_equal(g2, o)
    # flag and variant must agree
    with pytest.raises(N.PrtError):
        gpu_scene.render_tiles(cam, W, H, 32, 32, ids, 1, depth, 4, N.VAR_MIS[0] << 8)
    with pytest.raises(N.PrtError):
        gpu_scene.render_tiles(cam, W, H, 32, 32, ids, 1, depth, 4, N.PRT_FLAG_MIS_NEE | (N.VAR_LDS << 8))
    with pytest.raises(N.PrtError):
        gpu_scene.render_tiles(cam, W, H, 32, 32, ids, 1, depth, 4, (N.VAR_LAST + 1) << 8)   # unknown id


def test_mis_variant_on_a_global_scene_matches_oracle(cornell):
    """MIS estimator on a scene too large for LDS (default global MIS kernel, variant 33)."""
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    flat = _soup_scene(cornell, 3000, 11)
    ds = DeviceScene(flat, 0)
    osc = O.OracleScene.from_flat(flat)
    cam = cornell[1].convert_to_taichi_camera().packed()
    ids = np.arange(4, dtype=np.int32)
    O.set_nee_mode(True)
    try:
        o = osc.render_tiles(cam, 64, 64, 32, 32, ids, 2, 8, seed=6)
    finally:
        O.set_nee_mode(False)
    g, _ = ds.render_tiles(cam, 64, 64, 32, 32, ids, 2, 8, 6, N.PRT_FLAG_MIS_NEE)
    np.testing.assert_array_equal(g, o)
    ds.close()


def test_nonfinite_sample_counter(gpu_scene, cornell):
    """Failure detection: the STATS pass counts samples whose radiance is NaN or
    infinite — none for the Cornell box; every sample that reaches a wall whose albedo is
    NaN once the NaN guard cannot help (tracing.py:146-148 retries only with pdf = 1e-4)."""
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    from pyrenderer_amd.flatten import FlatScene
    cam = cornell[1].convert_to_taichi_camera().packed()
    ids = np.arange(4, dtype=np.int32)
    gpu_scene.render_tiles(cam, 64, 64, 32, 32, ids, 2, 8, 1, N.PRT_FLAG_STATS)
    assert gpu_scene.diag_stats()[14] == 0
    f = cornell[2]
    mat = f.mat.copy()
    mat[f.tri_mat[0], 0] = np.nan                  # the floor's red albedo
    bad = FlatScene(f.tri_v, f.tri_n, f.tri_mat, f.tri_prim, f.prim_lo, f.prim_hi, mat, f.light_tri, f.light_off,
                    f.direct_rgb)
    ds = DeviceScene(bad, 0)
    s, _ = ds.render_tiles(cam, 64, 64, 32, 32, ids, 2, 8, 1, N.PRT_FLAG_STATS)
    n_bad = int(ds.diag_stats()[14])
    px_bad = int((~np.isfinite(s)).any(axis=1).sum())
    assert n_bad > 0 and n_bad >= px_bad > 0, (n_bad, px_bad)
    ds.close()


def test_mis_variant_on_the_specular_scene():
    """MIS estimator with config 3's materials: its closest-hit visibility queries also land
    on the analytic sphere (hit ids >= n_tri, sphere material lookup) and on specular boxes."""
    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    scene, cam, flat = _specular_scene(0.35)
    ds = DeviceScene(flat, 0)
    osc = O.OracleScene.from_flat(flat)
    c = cam.convert_to_taichi_camera().packed()
    ids = np.arange(4, dtype=np.int32)
    O.set_nee_mode(True)
    try:
        o = osc.render_tiles(c, 64, 64, 32, 32, ids, 4, 8, seed=12)
    finally:
        O.set_nee_mode(False)
    g, _ = ds.render_tiles(c, 64, 64, 32, 32, ids, 4, 8, 12, N.PRT_FLAG_MIS_NEE)
    assert np.isfinite(g).all() and g.sum() > 0
    rmse, same = _compare(g, o, 4)
    assert rmse < TOL_RMSE, rmse
    assert same >= 0.999, same
    ds.close()


def test_launch_size_selects_the_pooled_kernel(gpu_scene):
    """prt_launch_kernel: on the Cornell box every launch takes the block-pooled shadow kernel (round 6:
    config 1's 65 k items and an 8-rank shard of config 2 too, now that it is faster there than the
    phase-aligned one); explicit variant flags win."""
    from pyrenderer_amd import _native as N
    assert gpu_scene.kernel_info()["variant"] == N.VAR_LDS_POOL
    assert gpu_scene.kernel_info(n_items=512 * 512 * 64)["variant"] == N.VAR_LDS_POOL
    assert gpu_scene.kernel_info(n_items=128 * 128 * 4)["variant"] == N.VAR_LDS_POOL
    assert gpu_scene.kernel_info(n_items=512 * 512 * 64 // 8)["variant"] == N.VAR_LDS_POOL   # an 8-rank shard
    assert gpu_scene.kernel_info(n_items=128 * 128 * 4, flags=N.VAR_LDS << 8)["variant"] == N.VAR_LDS
    assert gpu_scene.kernel_info(n_items=512 * 512 * 64, flags=N.PRT_FLAG_MIS_NEE)["variant"] == N.VAR_MIS[0]
