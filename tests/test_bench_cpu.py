"""bench.py's host-side contract, checked without a GPU: defaults (config 2 = BASELINE's
configs[1]), the CPU legs' report formats and the per-pixel comparison arithmetic."""
import sys
import types

import numpy as np

from conftest import ROOT

if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_defaults_are_the_baseline_workload(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.config, a.scene, a.res, a.spp, a.depth) == (2, "cornell", 512, 64, 8)
    assert a.steps > 0 and a.warmup >= 0 and a.tile is None and a.streams == 0
    assert sorted(bench.CONFIGS) == [1, 2, 3, 4, 5]
    assert bench.CONFIGS[5]["res"] == 4096 and bench.CONFIGS[5]["spp"] == 256


def test_l2_vs_cpu_arithmetic():
    args = types.SimpleNamespace(res=16, spp=4)
    ids = np.array([0, 3], np.int32)
    rng = np.random.default_rng(0)
    frame = rng.random((16, 16, 3)).astype(np.float32)
    tx = 16 // 8
    cpu = np.stack([frame[(t % tx) * 8:(t % tx) * 8 + 8, (t // tx) * 8:(t // tx) * 8 + 8].transpose(1, 0, 2)
                    for t in ids]).reshape(-1, 3)
    r = bench.l2_vs_cpu(frame, ids, cpu, args)
    assert r["identical_pixels"] == 1.0 and r["rmse"] == 0.0 and r["pass"]
    cpu2 = cpu.copy()
    cpu2[5, 1] += 0.04                      # one pixel off by 0.01 in mean radiance
    r = bench.l2_vs_cpu(frame, ids, cpu2, args)
    assert r["pixels"] == 128 and abs(r["max_pixel_l2"] - 0.01) < 1e-6 and not r["pass"]


def test_cpu_leg_reports():
    args = types.SimpleNamespace(res=64, spp=2, depth=4, seed=1)
    c = bench.cpu_baseline(np.arange(10000), 2.0, 4, args)
    assert c["kind"] == "port" and c["cores"] == 4 and c["unit"] == "Msamples/s"
    assert c["value"] == round(10000 * 64 * 2 / 2.0 / 1e6, 4)
    scene, cam = bench.load_scene("cornell")
    from pyrenderer_amd.flatten import flatten_scene
    rep, ids, sums = bench.numpy_baseline(flatten_scene(scene), cam.convert_to_taichi_camera().packed(), args, 0.2)
    assert rep["kind"] == "port" and rep["value"] > 0 and sums.shape == (len(ids) * 64, 3)


def test_host_cpu_and_kernel_sha(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    t, aff, model = bench.host_cpu()
    assert t == min(3, aff) and aff >= 1
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.host_cpu()[0] == aff
    from pyrenderer_amd.build import kernel_sha
    assert kernel_sha() == kernel_sha() and len(kernel_sha()) == 16


def _args(monkeypatch, argv):
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    return bench.parse()


def test_launch_check_spawns_the_launcher_as_a_child(monkeypatch):
    """`bench.py --gpus N` without WORLD_SIZE starts torch.distributed.run with N ranks as a child
    process (subprocess, never exec) and exits with its code."""
    import subprocess
    seen = {}

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return types.SimpleNamespace(returncode=7)

    monkeypatch.setattr(subprocess, "run", fake_run)
    args = _args(monkeypatch, ["--gpus", "2", "--backend", "gloo", "--steps", "3"])
    rc = bench.launch_check(args, env={"PATH": "/usr/bin"})
    assert rc == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=2" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-6:] == ["--gpus", "2", "--backend", "gloo", "--steps", "3"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # one GPU, or already under a launcher with the matching world size: render in this process
    assert bench.launch_check(_args(monkeypatch, []), env={}) is None
    assert bench.launch_check(args, env={"WORLD_SIZE": "2"}) is None
    # --force-collective at one GPU: a one-rank launcher, then the collective path
    fc = _args(monkeypatch, ["--force-collective", "--steps", "3"])
    assert fc.force_collective and fc.gpus == 1
    assert bench.launch_check(fc, env={"PATH": "/usr/bin"}) == 7
    assert "--nproc-per-node=1" in seen["cmd"] and seen["cmd"][-3:] == ["--force-collective", "--steps", "3"]
    assert bench.launch_check(fc, env={"WORLD_SIZE": "1"}) is None


def _run_bench(argv, **env):
    import os
    import subprocess
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, "bench.py"] + argv, cwd=ROOT, env=e, capture_output=True, text=True,
                          timeout=120)


def test_mislaunch_exits_nonzero_before_any_gpu_call():
    # WORLD_SIZE != --gpus under a launcher
    r = _run_bench(["--gpus", "4", "--backend", "gloo"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2 and "WORLD_SIZE=2 but --gpus 4" in r.stderr, r.stderr
    # nccl (one rank per device) with more ranks than visible devices (none in this container)
    import torch
    n = torch.cuda.device_count() + 1
    r = _run_bench(["--gpus", str(max(n, 2)), "--backend", "nccl"])
    assert r.returncode == 2 and "needs" in r.stderr and "visible" in r.stderr, r.stderr
    r = _run_bench(["--gpus", "0"])
    assert r.returncode == 2


def test_ranks_sharing_a_gpu_are_refused_under_nccl():
    """an N-GPU line must prove N distinct GPUs rendered.  bench.py gathers every
    rank's (rank, local rank, device, PCI address) into config.ranks and refuses (exit 2) an nccl
    launch whose ranks share a physical device; the gloo rehearsal may share one."""
    r = [{"rank": 0, "local_rank": 0, "device": 0, "pci": "0000:05:00"},
         {"rank": 1, "local_rank": 1, "device": 1, "pci": "0000:15:00"}]
    assert bench.check_rank_devices(r, "nccl") is None
    dup = [dict(r[0]), dict(r[1], device=0, pci="0000:05:00"), dict(r[1], rank=2, pci="0000:25:00")]
    why = bench.check_rank_devices(dup, "nccl")
    assert why and "0000:05:00" in why and "[0, 1]" in why
    assert bench.check_rank_devices(dup, "gloo") is None
    assert bench.shared_devices(dup) == {"0000:05:00": [0, 1]}
