"""Benchmark: Msamples/s of the path-tracing hot path, Cornell box 512x512 x 64 spp,
depth 8 (BASELINE.json configs[1]), on N GPUs of one node.

One step = one full frame: every rank renders its interleaved tiles (64x64 on one GPU, 16x16 on several)
(device_scene.tile_owner, 'latin' scheme) through libprt's HIP path into a device
buffer, then the per-tile radiance sums are gathered to rank 0 over RCCL
(torch.distributed 'nccl' backend).  Total work is fixed as N grows ("scaling":
"strong").  Consecutive frames alternate between --streams HIP streams, each with
its own buffers, so the drain of frame k (the last paths of a persistent launch,
~0.3 ms at any frame size) and its gather overlap the start of frame k+1 (auto: 3
streams when a rank renders < 8 M samples per frame, else 2 on several GPUs and
serial frames on one, where the per-launch roofline is measured).

    python bench.py --gpus 1 --steps 10 --warmup 3
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

Rank 0 prints ONE JSON line with `roofline` (trace kernel, per launch: the counted
traversal work ÷ the kernel's average duration measured with HIP events on its stream,
against the resource that serves it — SURVEY.md §8(d)'s FLOP accounting against the FP32
vector peak for LDS-resident scenes, whose scene bytes never reach HBM, and §8(d)'s
algorithmic bytes against the HBM peak for scenes read from HBM) and
`cpu_baseline` (the C oracle port with OpenMP, timed on this host on a bounded
sample), plus `cpu_numpy` (N = 1): the NumPy restatement of main.py's path,
one spawned process per core, on its own bounded sample, with its per-pixel
comparison against the GPU frame.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
LDS_PEAK_GBS = 150000.0  # MI355X_MICROARCH.md §LDS: ~150 TB/s aggregate for ds_read_b128 at ~2.4 GHz
VALU_PEAK_TFLOPS = 157.3
SIMDS, PEAK_CLOCK_GHZ = 1024, 2.4   # 256 CUs x 4 SIMD-32; a wave64 VALU instruction holds its SIMD 2 cycles
# Algorithmic bytes per sample, SURVEY.md §8(d) (the roofline's `achieved`):
#   B_sample = 32 N_node + 48 N_tri + 48 N_lightpt + 16 N_ray + 12 / spp_per_launch
# N_node = BVH node visits (one BVH4 visit counted as one 32-B node fetch, as §8(d)'s
# per-visit figure; the BVH4 visits replace ~2-3 BVH2 visits each, so this is the
# conservative side), N_tri = triangle tests, N_lightpt = NEE light samples that issue a
# shadow query, N_ray = 0 (one persistent kernel: no ray state passes between stages),
# 12 B per pixel = the framebuffer write.
S8_NODE, S8_TRI, S8_LIGHT, S8_PIXEL = 32, 48, 48, 12
# Logical bytes the kernel actually reads per unit (the `lds` block for LDS-resident scenes):
# 112 B per f32 BVH4 node (4 boxes SoA + refs), 64 B per quantised node, 48 B per triangle,
# 64 B per light record.
B_NODE4, B_NODE4Q, B_TRI, B_LIGHT = 112, 64, 48, 64
# SURVEY.md §8(d)'s fixed FLOP accounting for the VALU roofline: ~30 FLOP per AABB test (a
# BVH4 node visit tests 4 boxes) and ~40 per Moller-Trumbore test.
F_BOX, F_TRI = 30, 40


DATA_NOTES = {
    "cornell": "synthetic (Cornell box scene.json shipped with the reference)",
    "specular": "synthetic (Cornell box + build-added metal/dielectric boxes and a glass sphere)",
    "cubes": "synthetic (Cornell box + 83,334 jittered instances of cube.obj, seed 1234)",
}

# BASELINE.json configs; the bench line is quoted on config 2.
CONFIGS = {
    1: dict(scene="cornell", res=128, spp=4, depth=4),
    2: dict(scene="cornell", res=512, spp=64, depth=8),
    3: dict(scene="specular", res=1024, spp=256, depth=8),
    4: dict(scene="cubes", res=512, spp=64, depth=8),
    5: dict(scene="cornell", res=4096, spp=256, depth=8),
}


SCENE_NAMES = {"cornell": "Cornell box (Lambertian)", "specular": "Cornell box + metal/dielectric + sphere",
               "cubes": "Cornell box + 1M-triangle instanced cube.obj"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--scene", default=None, help="cornell | specular | cubes (overrides --config)")
    ap.add_argument("--res", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--tile", type=int, default=None,
                    help="tile side in pixels (default 64 on one GPU, 16 on several: the finer latin "
                         "interleave balances 8 ranks best, profiles/r01/shard_sim_c2_tiles_streams3.jsonl)")
    ap.add_argument("--streams", type=int, default=0,
                    help="frames in flight (1 = strictly serial frames; 0 = auto: 3 when a rank renders < 8 M "
                         "samples per frame, else 2 on several GPUs and 1 on one)")
    ap.add_argument("--scheme", default="latin", help="tile assignment: latin | mod")
    ap.add_argument("--frames-per-launch", type=int, default=0,
                    help="frames per render call (prt_render_frames_device: their items share the persistent "
                         "launches, one ramp-up and drain per call); 0 = auto: enough frames for >= ~16 M items "
                         "per launch, 16..256, at most the steps; 1 for frames of > 64 M samples per rank")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="torch.distributed backend for N > 1: nccl (= RCCL over xGMI, the default) or gloo "
                         "(tile sums staged through host memory; rehearses the N > 1 path with several ranks "
                         "on one GPU)")
    ap.add_argument("--force-collective", action="store_true",
                    help="take the N > 1 step's collective path even at --gpus 1: a process group of one rank "
                         "under torch.distributed.run (started by bench.py itself), the device-tensor "
                         "all_gather_object / all_reduce, the async gather into rank 0's device buffer and the "
                         "root's scatter from it — the RCCL branch of the 8-GPU run, exercised on one GPU")
    ap.add_argument("--single-frame-steps", type=int, default=5,
                    help="extra timed leg after the main one: this many steps of ONE frame per launch (what a "
                         "caller's one-shot render of one frame costs), reported as `single_frame`; 0 = skip "
                         "(also skipped when the main leg already runs one frame per launch)")
    ap.add_argument("--variant", type=int, default=0, help="trace-kernel variant id (0 = the library's default)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU time of the baseline sample")
    ap.add_argument("--numpy-seconds", type=float, default=8.0,
                    help="target wall time of the NumPy-path CPU sample (main.py counterpart); 0 = skip")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc.json"),
                    help="PMC summaries per workload (tools/pmc_summary.py): HBM bytes per trace launch, "
                         "VALU issue / lane utilisation; traffic is null for a workload without an entry")
    a = ap.parse_args()
    for k, v in CONFIGS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    return a


def load_scene(name):
    from pyrenderer_amd import scenes
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    if name == "cornell":
        return read_file(scenes.CORNELL)
    if name == "specular":
        return read_file(scenes.CORNELL_SPECULAR)
    if name == "cubes":
        return scenes.instanced_cubes()
    raise SystemExit(f"unknown scene {name}")


def host_cpu():
    """(threads used, affinity cores, CPU model): the CPU legs use every core this process
    may run on, capped by OMP_NUM_THREADS when the environment sets it (the GPU box sets it to
    the box's CPU share, 16 per GPU, while its affinity mask shows the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "").strip()
    threads = min(aff, int(omp)) if omp.isdigit() and int(omp) > 0 else aff
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return threads, aff, model


def cpu_sample(flat, cam, args, seconds):
    """Oracle (C restatement of PathTracer.trace, OpenMP) on a bounded sample of the
    same workload: random 8x8 tiles of the frame at the full spp/depth, sized to about
    `seconds` of CPU time.  Closest hits by stack traversal of the same BVH2 (oracle
    BACKEND_BVH, bit-identical to the brute-force and reference-structure backends and
    the fastest of the three).  Returns (tile ids, per-slot sums, seconds, threads)."""
    from oracle import oracle as O
    from pyrenderer_amd._native import Bvh
    osc = O.OracleScene.from_flat(flat)
    nodes, _, order = Bvh(flat.tri_v).export()
    osc.set_bvh(nodes, order)
    cores = host_cpu()[0]
    W = H = args.res
    n_tiles_total = (W // 8) * (H // 8)
    rng = np.random.default_rng(1)
    perm = rng.permutation(n_tiles_total).astype(np.int32)
    # calibrate on 4 tiles, then size the sample for ~args.cpu_seconds
    t0 = time.perf_counter()
    osc.render_tiles(cam, W, H, 8, 8, perm[:4], args.spp, args.depth, seed=args.seed, nthreads=cores,
                     backend=O.BACKEND_BVH)
    dt = max(time.perf_counter() - t0, 1e-3)
    n = int(min(n_tiles_total, max(8, 4 * seconds / dt)))
    ids = np.sort(perm[:n])
    t0 = time.perf_counter()
    sums = osc.render_tiles(cam, W, H, 8, 8, ids, args.spp, args.depth, seed=args.seed, nthreads=cores,
                            backend=O.BACKEND_BVH)
    dt = time.perf_counter() - t0
    return ids, sums, dt, cores


def cpu_baseline(ids, dt, cores, args):
    W = H = args.res
    n = len(ids)
    samples = n * 64 * args.spp
    _, aff, model = host_cpu()
    return {"value": round(samples / dt / 1e6, 4), "unit": "Msamples/s", "cores": cores, "kind": "port",
            "cpu_model": model, "affinity_cores": aff,
            "sample": f"{n} random 8x8 tiles of the {W}x{H} frame at {args.spp} spp, depth {args.depth} "
                      f"({samples} samples, {dt:.1f} s); oracle/prt_oracle.c (C port of PathTracer.trace), "
                      f"BVH2 closest hit, OpenMP {cores} threads"}


def numpy_baseline(flat, cam, args, seconds, procs=None):
    """main.py's NumPy path counterpart (oracle/numpy_path.py: PathTracer.trace as array code
    over ray batches, bit-identical to the C oracle), one spawned process per core like
    main.py's joblib workers (or `procs` of them: main.py:52 itself uses n_jobs=4), on random
    8x8 tiles sized to ~`seconds`.  Returns (report, tile ids, sums) or (note, None, None) for
    scenes outside its scope (config 3, 4)."""
    from oracle import numpy_path as NP
    cores = procs or host_cpu()[0]
    W = H = args.res
    try:
        ids, sums, dt = NP.timed_sample(flat, cam, W, H, args.spp, args.depth, args.seed, seconds, cores)
    except NotImplementedError as e:
        return {"value": None, "note": str(e)}, None, None
    samples = len(ids) * 64 * args.spp
    return ({"value": round(samples / dt / 1e6, 5), "unit": "Msamples/s", "cores": cores, "kind": "port",
             "sample": f"{len(ids)} random 8x8 tiles of the {W}x{H} frame at {args.spp} spp, depth {args.depth} "
                       f"({samples} samples, {dt:.1f} s); oracle/numpy_path.py (NumPy restatement of "
                       f"PathTracer.trace over ray batches, brute-force closest hit), {cores} spawned processes"},
            ids, sums)


def l2_vs_cpu(gpu_sums, ids, cpu_sums, args):
    """Per-pixel comparison of the timed frame (rank 0's gathered sums) with the CPU
    oracle on the sampled 8x8 tiles: mean radiance = sums / spp on both sides; the
    north-star tolerance is a per-pixel L2 < 1e-3."""
    W = H = args.res
    tx = W // 8
    c = np.asarray(cpu_sums, np.float64).reshape(len(ids), 8, 8, 3)
    g = np.stack([gpu_sums[(t % tx) * 8:(t % tx) * 8 + 8, (t // tx) * 8:(t // tx) * 8 + 8].transpose(1, 0, 2)
                  for t in ids]).astype(np.float64)
    diff = (g - c) / args.spp
    pix_l2 = np.sqrt((diff ** 2).sum(axis=-1))
    same = np.all(g.astype(np.float32) == c.astype(np.float32), axis=-1)
    return {"pixels": int(pix_l2.size), "rmse": float(np.sqrt((diff ** 2).mean())),
            "max_pixel_l2": float(pix_l2.max()), "identical_pixels": round(float(same.mean()), 6),
            "tolerance": 1e-3, "pass": bool(pix_l2.max() < 1e-3),
            "reference": "oracle/prt_oracle.c (C port of PathTracer.trace), same seed, random 8x8 tiles"}


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_check(args, env=None):
    """The N-GPU launch contract, checked before anything touches a GPU (torch.cuda.device_count()
    does not initialise the device on this image).  Returns None when this process should
    render, else an exit code: a child launcher's, or 2 for a mislaunch.

    * `--gpus N > 1` (or `--force-collective`) without a launcher (no WORLD_SIZE): start
      `torch.distributed.run` with N ranks on this node as a CHILD process (never exec: the parent
      has not touched the GPU, but the child must own it), forward its output and exit with its code.
    * under a launcher: WORLD_SIZE must equal --gpus, and for --backend nccl (RCCL: one rank per
      device) N must not exceed the visible devices — either mismatch would print a plausible
      line for the wrong N."""
    env = os.environ if env is None else env
    import torch
    n_dev = torch.cuda.device_count()
    if args.gpus < 1:
        print(f"bench.py: --gpus must be >= 1 (got {args.gpus})", file=sys.stderr)
        return 2
    if args.backend == "nccl" and args.gpus > 1 and args.gpus > n_dev:
        print(f"bench.py: --gpus {args.gpus} with --backend nccl needs {args.gpus} devices, "
              f"{n_dev} visible", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in env:
        if args.gpus == 1 and not getattr(args, "force_collective", False):
            return None
        import subprocess
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
               os.path.abspath(__file__)] + sys.argv[1:]
        child_env = dict(env, HSA_ENABLE_IPC_MODE_LEGACY=env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        sys.stdout.flush()
        return subprocess.run(cmd, env=child_env).returncode
    world = int(env["WORLD_SIZE"])
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch N ranks for --gpus N",
              file=sys.stderr)
        return 2
    return None


def rank_identity(dev, rank=0, local_rank=0):
    """This rank's GPU, as the line reports it (config.ranks): rank, local rank, torch device index,
    the device's PCI address (domain:bus:device) and UUID — what makes an N-GPU line self-proving
    (N distinct PCI addresses = N distinct GPUs rendered)."""
    import torch
    p = torch.cuda.get_device_properties(dev)
    return {"rank": int(rank), "local_rank": int(local_rank), "device": int(dev.index),
            "pci": f"{int(p.pci_domain_id):04x}:{int(p.pci_bus_id):02x}:{int(p.pci_device_id):02x}",
            "uuid": str(getattr(p, "uuid", ""))}


def shared_devices(ranks):
    """{pci address: [ranks]} for every physical device that more than one rank runs on."""
    by = {}
    for r in ranks:
        by.setdefault(r["pci"], []).append(r["rank"])
    return {k: v for k, v in by.items() if len(v) > 1}


def check_rank_devices(ranks, backend):
    """None, or why this launch is refused: under nccl (RCCL) every rank must own its own GPU — two
    ranks on one device would make an N-GPU line that N GPUs did not produce.  The gloo rehearsal
    (several ranks on one GPU, tile sums staged through host memory) may share devices."""
    shared = shared_devices(ranks)
    if backend == "nccl" and shared:
        return "ranks share a GPU under nccl: " + ", ".join(f"{k} <- ranks {v}" for k, v in sorted(shared.items()))
    return None


def main():
    args = parse()
    rc = launch_check(args)
    if rc is not None:
        sys.exit(rc)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; with more ranks than visible GPUs (a gloo rehearsal on a one-GPU box)
    # ranks share devices round-robin
    n_dev = max(1, torch.cuda.device_count())
    dev = torch.device("cuda", local % n_dev if world > 1 else 0)
    # the collective path (process group, gather to rank 0's buffer, the root's scatter): every N > 1
    # run, and N = 1 with --force-collective (the same code on a world of one rank)
    coll = world > 1 or args.force_collective
    gloo = coll and args.backend == "gloo"
    if coll:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(dev)
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    else:
        torch.cuda.set_device(0)
    coll_dev = torch.device("cpu") if gloo else dev   # where collective operands live
    # which GPU every rank renders on (config.ranks): gathered before any work, and a launch whose
    # nccl ranks share a device is refused (exit 2) on every rank alike
    ident = rank_identity(dev, rank, local)
    ranks = [ident]
    if coll:
        ranks = [None] * world
        dist.all_gather_object(ranks, ident)
        why = check_rank_devices(ranks, args.backend)
        if why:
            if rank == 0:
                print(f"bench.py: {why}", file=sys.stderr)
            dist.destroy_process_group()
            sys.exit(2)

    from pyrenderer_amd import _native as N
    from pyrenderer_amd.device_scene import DeviceScene
    from pyrenderer_amd.distributed import TileShard
    from pyrenderer_amd.flatten import flatten_scene

    scene, camera = load_scene(args.scene)
    flat = flatten_scene(scene)
    cam = camera.convert_to_taichi_camera().packed()
    t_build = time.perf_counter()
    ds = DeviceScene(flat, dev.index)
    t_build = time.perf_counter() - t_build
    W = H = args.res
    T = args.tile if args.tile else (64 if world == 1 else 16)
    rank_samples = W * H * args.spp / world
    # frames per render call (prt_render_frames_device): F frames' (pixel, sample) items run through
    # the same persistent launches, so a launch ramps up and drains once per F frames instead of once
    # per frame; each frame is still rendered, reduced, gathered and scattered whole
    F = args.frames_per_launch
    if F <= 0:
        # enough frames for a launch of >= ~16 M items (one C2 frame), at least 16 and at most 256:
        # 16 for C2 on 1-8 GPUs, 256 for config 1's 65 k-sample frames; frames above 64 M samples
        # (C3, C5) already fill their launches
        F = min(256, max(16, -(-int(16.8e6) // max(int(rank_samples), 1)))) if rank_samples <= 64e6 else 1
    F = max(1, min(F, args.steps))
    n_streams = args.streams
    if n_streams <= 0:
        # measured (profiles/r01/shard_sim_*, streams_ab): for a whole C2 frame on one GPU,
        # overlapping frames gains ~2 % (5.15 vs 5.26 ms) but makes every launch's event span
        # include time shared with the next frame, so the roofline's kernel duration (and the
        # rocprof average it is checked against) would no longer be the kernel's own; serial
        # frames keep them equal.  For the 1/4 and 1/8 frames of 4- and 8-rank runs the launch
        # tail is a larger share: 3 frames in flight (0.741 vs 0.777 ms per frame at 1/8).
        # On several GPUs the per-launch roofline is not the headline, and overlap pays more (a
        # half frame at N = 2: 2.55 vs 2.65 ms with 2 streams, profiles/r01/shard_sim_c2_streams_t16.jsonl).
        # Multi-frame launches already amortise the drain: serial launches.
        n_streams = 1 if F > 1 else (3 if rank_samples < 8e6 else (2 if world > 1 else 1))
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(n_streams - 1)]
    shards = [TileShard(W, H, T, rank, world, dev, args.scheme, host_staging=gloo, frames=F, collective=coll)
              for _ in range(n_streams)]
    my_tiles = shards[0].tiles
    n_step = [0]
    rflags = args.variant << 8

    def steps(nf, flags=0):
        """nf (<= F) steps: nf frames rendered by one render call, then one gather of them to rank 0
        and (root) its device scatter into the (W, H, 3) frame."""
        k = n_step[0] % n_streams
        n_step[0] += 1
        shard, stream = shards[k], streams[k]
        if nf == 1:
            ds.render_tiles_device(cam, W, H, T, T, my_tiles, args.spp, args.depth, shard.buf.data_ptr(),
                                   stream.cuda_stream, seed=args.seed, flags=flags | rflags)
        else:
            # consecutive progressive frames (main_taichi.py:108-118): frame f of the group renders
            # samples f * spp .. (f + 1) * spp - 1, so no two frames of a launch repeat work
            # frame f -> shard.bufs[f]: the rows are padded to the largest shard (the gather's slot), so
            # the render writes at that pitch (a ragged shard's frames would otherwise shift)
            ds.render_frames_device(cam, W, H, T, T, my_tiles, args.spp, args.depth, nf, shard.bufs.data_ptr(),
                                    stream.cuda_stream, seed=args.seed, frame_stride=args.spp, flags=flags | rflags,
                                    out_pitch=shard.pitch)
        with torch.cuda.stream(stream):
            shard.gather(n_frames=nf)    # RCCL gathers of per-tile radiance sums to rank 0 (ordered after the frames)
            if coll and rank == 0:
                # root: every rank's tiles of the group's frames into the (W, H, 3) device frames
                # (SURVEY.md §8(e)), one launch, inside the step
                shard.scatter_frames(ds, stream, nf)

    def run(n):
        # equal groups of <= F frames (equal launches: the per-launch roofline averages like sizes)
        groups = -(-n // F)
        for g in range(groups):
            nf = n // groups + (1 if g < n % groups else 0)
            steps(nf, N.PRT_FLAG_TIME if timing[0] else 0)

    timing = [False]
    # counted traversal work of one frame (deterministic: same RNG as the timed steps)
    steps(1, N.PRT_FLAG_STATS)
    torch.cuda.synchronize(dev)
    st = np.append(ds.last_stats().astype(np.float64), float(ds.diag_stats()[14]))
    cnt = torch.tensor(st, dtype=torch.float64, device=coll_dev)
    if coll:
        dist.all_reduce(cnt)
    nodes, tris, ext, shadow, nonfinite = cnt.tolist()

    # warmup: the W steps, and at least one full group of F frames (its buffers are then allocated)
    run(max(args.warmup, F))
    if coll:
        dist.barrier()
    torch.cuda.synchronize(dev)
    timing[0] = True
    t0 = time.perf_counter()
    run(args.steps)
    if coll:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms, launches = ds.kernel_timing()   # HIP events on `stream` around every trace launch
    # the frame is split into chunks of <= PRT chunk bytes of per-sample radiance (several
    # trace launches per step at C5); the roofline is per launch
    launches_per_step = max(launches, 1) / args.steps
    t = torch.tensor([elapsed, kern_ms / max(launches, 1)], dtype=torch.float64, device=coll_dev)
    # every rank's own timed-region wall time (imbalance shows as max / min)
    per_rank = [t[0:1].clone() for _ in range(world)]
    if coll:
        dist.all_gather(per_rank, t[0:1].clone())
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_avg_ms = t.tolist()
    rank_ms = [float(x.item()) * 1e3 / args.steps for x in per_rank]
    groups_timed = -(-args.steps // F)
    f_group = -(-args.steps // groups_timed)   # frames of the timed groups (the first ones; equal groups)

    # the accuracy sample comes from the headline's own launches: rank 0 copies frame 0 of
    # the last timed group (samples 0 .. spp - 1, rendered inside a multi-frame launch, gathered and, at
    # N > 1 or with --force-collective, scattered from the gather buffer) before any other leg renders
    timed_frame = None
    if rank == 0 and not args.no_cpu_baseline:
        last = shards[(n_step[0] - 1) % n_streams]
        timed_frame = last.assemble(ds, streams[(n_step[0] - 1) % n_streams])

    # what batching buys: the same step with ONE frame per persistent launch, timed the
    # same way (barrier + synchronize on both sides, max over ranks), after the main leg
    single = None
    if F > 1 and args.single_frame_steps > 0:
        steps(1, 0)                                  # warm the single-frame buffers and launch shape
        if coll:
            dist.barrier()
        torch.cuda.synchronize(dev)
        ds.kernel_timing()
        t1 = time.perf_counter()
        for _ in range(args.single_frame_steps):
            steps(1, N.PRT_FLAG_TIME)
        if coll:
            dist.barrier()
        torch.cuda.synchronize(dev)
        el1 = time.perf_counter() - t1
        k1_ms, k1_n = ds.kernel_timing()
        t1v = torch.tensor([el1, k1_ms / max(k1_n, 1)], dtype=torch.float64, device=coll_dev)
        if coll:
            dist.all_reduce(t1v, op=dist.ReduceOp.MAX)
        el1, k1_avg = t1v.tolist()
        ms1 = el1 * 1e3 / args.single_frame_steps
        single = {"frames_per_launch": 1, "steps": args.single_frame_steps, "ms_per_step": round(ms1, 4),
                  "value": round(W * H * args.spp / (ms1 * 1e-3) / 1e6, 3),
                  "kernel_avg_ms": round(k1_avg, 4), "launches_per_step": round(k1_n / args.single_frame_steps, 3),
                  "note": "one frame per persistent launch (a one-shot render() of this frame); `value` above "
                          "batches frames_per_launch frames per launch, each still rendered, reduced, gathered "
                          "and scattered whole"}

    if rank == 0:
        samples_per_step = W * H * args.spp
        ms_per_step = elapsed * 1e3 / args.steps
        value = samples_per_step / (elapsed / args.steps) / 1e6
        # roofline of the dominant kernel (trace_kernel) on rank 0 (per launch)
        share = 1.0 / world
        n_px_rank = len(my_tiles) * T * T
        # the variant of this workload's launches (DeviceScene.kernel_info: the default rule for its size)
        kinfo = ds.kernel_info(n_items=int(round(n_px_rank * args.spp / launches_per_step)))
        if args.variant:
            kinfo = dict(kinfo, variant=args.variant)
        # SURVEY.md §8(d) algorithmic bytes per launch (module constants S8_*)
        work_launch = share / launches_per_step
        bytes_launch = ((S8_NODE * nodes + S8_TRI * tris + S8_LIGHT * shadow) * work_launch
                        + S8_PIXEL * n_px_rank / launches_per_step)
        kern_s = kern_avg_ms * 1e-3
        achieved = bytes_launch / kern_s / 1e9
        # what the kernel really reads per launch from its scene copy (LDS for LDS-resident scenes)
        b_node = B_NODE4Q if kinfo["quantized"] else B_NODE4
        scene_gbs = (b_node * nodes + B_TRI * tris + B_LIGHT * shadow) * work_launch / kern_s / 1e9
        flops_launch = (F_BOX * 4 * nodes + F_TRI * tris) * work_launch
        # counter figures (PMC passes, tools/profile_bench.sh -> tools/pmc_summary.py) only when
        # they were measured on this exact kernel build and variant
        from pyrenderer_amd.build import kernel_sha
        sha = kernel_sha()
        pmc, pmc_state = {}, "no entry"
        if args.pmc_json and os.path.exists(args.pmc_json) and world == 1:
            try:
                e = json.load(open(args.pmc_json)).get(f"{args.scene}_{W}x{H}x{args.spp}spp_d{args.depth}")
            except (OSError, ValueError):
                e = None
            if e:
                if e.get("kernel_sha") == sha and e.get("variant") == kinfo["variant"]:
                    pmc, pmc_state = e, "this build"
                else:
                    pmc_state = f"stale (measured on kernel {e.get('kernel_sha')} variant {e.get('variant')})"
        traffic = pmc.get("hbm_bytes_per_launch")
        issue = pmc.get("valu_issue_util")
        lane = pmc.get("valu_lane_util")
        cpu, l2, cpu_np = None, None, None
        if not args.no_cpu_baseline and world == 1 and args.numpy_seconds > 0:
            cpu_np, np_ids, np_sums = numpy_baseline(flat, cam, args, args.numpy_seconds)
            if np_ids is not None:
                cmp = l2_vs_cpu(timed_frame, np_ids, np_sums, args)
                cpu_np["l2_vs_gpu"] = {k: cmp[k] for k in ("pixels", "rmse", "max_pixel_l2", "identical_pixels")}
                # main.py:52's own parallelism (joblib n_jobs=4), on a shorter sample
                n4, _, _ = numpy_baseline(flat, cam, args, args.numpy_seconds / 2, procs=4)
                cpu_np["n_jobs_4"] = {k: n4.get(k) for k in ("value", "cores", "sample")}
        if not args.no_cpu_baseline:
            # at N = 1 the baseline sample (~cpu_seconds) doubles as the accuracy sample; at
            # N > 1 only a short accuracy sample of the gathered frame is rendered on the CPU
            ids, cpu_sums, dt, cores = cpu_sample(flat, cam, args, args.cpu_seconds if world == 1 else 2.0)
            if world == 1:
                cpu = cpu_baseline(ids, dt, cores, args)
            l2 = l2_vs_cpu(timed_frame, ids, cpu_sums, args)
            l2.update({"source": "timed group", "frame": 0, "frames_per_launch": f_group,
                       "gathered": bool(coll)})
        hbm_measured = round(traffic / kern_s / 1e9 / HBM_PEAK_GBS, 4) if traffic else None
        flops_tf = flops_launch / kern_s / 1e12
        # the dominant kernel's name as rocprofv3 reports it (profiles/*/kernel_stats.csv)
        kname = "trace_kernel_pool" if kinfo["variant"] in N.VAR_POOL else "trace_kernel"
        common = {"traffic": traffic, "hbm_measured_frac": hbm_measured, "valu_issue_util": issue,
                  "valu_lane_util": lane, "kernel": kname, "kernel_avg_ms": round(kern_avg_ms, 4),
                  "launches_per_step": round(launches_per_step, 3), "variant": kinfo, "kernel_sha": sha,
                  "pmc": pmc_state}
        hbm_logical = {"achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(achieved / HBM_PEAK_GBS, 4), "bytes_per_launch": int(bytes_launch)}
        if kinfo["lds_scene"]:
            # the scene sits in LDS: §8(d)'s algorithmic bytes are LDS reads, not HBM traffic, and
            # what binds is VALU issue under divergence
            roofline = dict({"bound": "valu", "achieved": round(flops_tf, 3), "peak": VALU_PEAK_TFLOPS,
                             "unit": "TFLOP/s", "frac": round(flops_tf / VALU_PEAK_TFLOPS, 4),
                             "flops_per_launch": int(flops_launch)}, **common)
            # §8(d)'s byte accounting, kept as a rate only: priced against the HBM peak it would read
            # above 1 although none of these bytes reach HBM (the `lds` block prices them correctly)
            roofline["s8d_bytes_from_lds"] = {
                "rate": round(achieved, 2), "unit": "GB/s", "bytes_per_launch": int(bytes_launch),
                "note": "SURVEY.md §8(d) algorithmic bytes (32 B per node visit, 48 per triangle test, 48 per "
                        "shadow query's light point, 12 per pixel) over the kernel duration; served from the "
                        "LDS scene copy, so not an HBM figure (HBM: traffic / hbm_measured_frac)"}
            roofline["lds"] = {"achieved": round(scene_gbs, 2), "peak": LDS_PEAK_GBS, "unit": "GB/s",
                               "frac": round(scene_gbs / LDS_PEAK_GBS, 4),
                               "note": "bytes read from the LDS scene copy (112 B per f32 BVH4 node, 48 per "
                                       "triangle, 64 per light record) against the aggregate ds_read_b128 rate"}
            roofline["note"] = ("achieved/frac: SURVEY.md §8(d) FLOP accounting (30 per box test, 4 boxes per BVH4 "
                                "visit; 40 per Moller-Trumbore test) over the HIP-event kernel duration against the "
                                "157.3 TFLOP/s FP32 vector peak. The kernel is VALU-issue bound (valu_issue_util = 2 "
                                "cycles x SQ_INSTS_VALU / (1024 SIMDs x dispatch cycles)); the gap to the FLOP peak "
                                "is divergence (valu_lane_util = active lanes per VALU instruction / 64) and the "
                                "exact-arithmetic contract's compares, selects and divisions. traffic / "
                                "hbm_measured_frac: PMC FETCH_SIZE x 2 + WRITE_SIZE per launch (profiles/pmc.json, "
                                "only when measured on this kernel_sha and variant, else null).")
        else:
            roofline = dict({"bound": "hbm"}, **hbm_logical, **common)
            roofline["valu_tflops"] = round(flops_tf, 3)
            roofline["note"] = ("achieved/frac: SURVEY.md §8(d) algorithmic bytes (32 B per node visit, 48 per "
                                "triangle test, 48 per shadow query's light point, 12 per pixel) over the HIP-event "
                                "kernel duration against the 8 TB/s HBM peak; the scene is read through L2 and the "
                                "256 MB MALL (traffic / hbm_measured_frac: PMC FETCH_SIZE x 2 + WRITE_SIZE per "
                                "launch, profiles/pmc.json, only for this kernel_sha and variant). Latency-bound "
                                "on the dependent node-fetch chain: neither HBM nor VALU issue saturates.")
        line = {
            "metric": "Msamples/sec Cornell box 512²×64spp at 1/2/4/8 GPU; per-pixel L2 vs CPU",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": DATA_NOTES[args.scene],
            "config": {"workload": f"{SCENE_NAMES[args.scene]} {W}x{H}, {args.spp} spp, depth {args.depth}",
                       "baseline_config": args.config, "triangles": int(flat.n_tri), "spheres": int(flat.sph.shape[0]),
                       "global_batch": W * H * args.spp, "parallelism": f"tiles{world}",
                       "backend": (args.backend if coll else None), "collective": bool(coll),
                       "tile_scheme": args.scheme, "frames_in_flight": n_streams, "frames_per_launch": -(-args.steps // -(-args.steps // F)),
                       "tile": T, "bvh_depth": ds.bvh_depth, "bvh_nodes": ds.n_nodes, "scene_build_s": round(t_build, 3),
                       "ranks": ranks},
            # each rank's own wall time per step over the timed steps (value uses the max)
            "rank_ms_per_step": {"min": round(min(rank_ms), 4), "max": round(max(rank_ms), 4),
                                 "per_rank": [round(x, 4) for x in rank_ms]},
            "single_frame": single,
            "roofline": roofline,
            "work_per_sample": {"nodes": round(nodes / samples_per_step, 2), "tris": round(tris / samples_per_step, 2),
                                "ext_queries": round(ext / samples_per_step, 3),
                                "shadow_queries": round(shadow / samples_per_step, 3),
                                "nonfinite_samples": int(nonfinite)},
            # the same counts summed over the ranks (independent of the tile split for the queries)
            "work_totals": {"nodes": int(nodes), "tris": int(tris), "ext_queries": int(ext),
                            "shadow_queries": int(shadow)},
            "cpu_baseline": cpu,
            "cpu_numpy": cpu_np,
            "l2_vs_cpu": l2,
        }
        print(json.dumps(line), flush=True)
    if coll:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
