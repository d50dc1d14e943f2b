"""bench.py's N > 1 code path, rehearsed on one GPU: plain `python bench.py --gpus 2 --backend gloo`
as a fresh subprocess — bench.py starts torch.distributed.run itself (both ranks render
their latin-interleaved tiles on device 0 with the HIP kernel, the tile sums are staged through
host memory, gathered to rank 0 and scattered into the frame on the device by libprt's scatter
kernel inside every timed step).  The line must report 2 GPUs, a frame bit-identical to the CPU oracle on its sample, and
per-rank work counters that sum to the one-process counts.  The only piece of the driver's
8-GPU run this leaves untested is the RCCL transport itself.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

ARGS = ["--res", "128", "--spp", "8", "--depth", "8", "--tile", "16", "--steps", "2", "--warmup", "1",
        "--numpy-seconds", "0", "--cpu-seconds", "2"]


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


@pytest.mark.timeout(400)
def test_bench_two_ranks_over_gloo_on_one_gpu():
    # plain `bench.py --gpus 2` (the driver's command form): bench.py starts torch.distributed.run
    # with two ranks itself, as a child process
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--backend", "gloo"] + ARGS
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    two = _line(r.stdout)
    assert two["n_gpus"] == 2 and two["config"]["backend"] == "gloo"
    assert two["l2_vs_cpu"]["identical_pixels"] == 1.0 and two["l2_vs_cpu"]["pass"]
    assert two["value"] > 0 and two["steps"] == 2
    # the line names the device of every rank and each rank's own step time
    ranks = two["config"]["ranks"]
    assert len(ranks) == 2 and sorted(r["rank"] for r in ranks) == [0, 1]
    assert all(set(r) >= {"rank", "local_rank", "device", "pci", "uuid"} for r in ranks)
    assert len({r["pci"] for r in ranks}) == 1          # gloo rehearsal: both ranks on the one GPU
    rm = two["rank_ms_per_step"]
    assert len(rm["per_rank"]) == 2 and 0 < rm["min"] <= rm["max"]
    assert abs(rm["max"] - two["ms_per_step"]) <= 1e-3 * rm["max"] + 1e-3
    # the one-frame-per-launch leg
    sf = two["single_frame"]
    assert sf["frames_per_launch"] == 1 and sf["ms_per_step"] > 0 and sf["kernel_avg_ms"] > 0
    r1 = subprocess.run([sys.executable, "bench.py"] + ARGS + ["--no-cpu-baseline"], cwd=ROOT, env=env,
                        capture_output=True, text=True, timeout=200)
    assert r1.returncode == 0, r1.stdout[-3000:] + r1.stderr[-3000:]
    one = _line(r1.stdout)
    assert one["n_gpus"] == 1 and len(one["config"]["ranks"]) == 1
    a, b = two["work_totals"], one["work_totals"]
    # path queries depend only on the (seed, pixel, sample) streams: exact for any tile split
    assert a["ext_queries"] == b["ext_queries"] and a["shadow_queries"] == b["shadow_queries"], (a, b)
    # node / triangle counts also depend on which lanes share a wave (leaf-phase thresholds)
    for k in ("nodes", "tris"):
        assert abs(a[k] - b[k]) <= 0.01 * b[k], (k, a, b)


@pytest.mark.timeout(400)
def test_bench_three_ranks_ragged_multi_frame_over_gloo():
    """ADVICE r04 (medium) end to end: three gloo ranks on the one GPU, 64 tiles of 16 x 16 (ranks of
    22 / 21 / 21 tiles: two ragged shards) and 4 frames per launch — the ranks render into their padded
    gather rows at the slot pitch, rank 0 scatters the group in one launch; the gathered frame equals the
    CPU oracle and the counters sum to the one-process counts."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONUNBUFFERED="1")
    args = ["--res", "128", "--spp", "4", "--depth", "6", "--tile", "16", "--steps", "4", "--warmup", "1",
            "--numpy-seconds", "0", "--cpu-seconds", "1", "--frames-per-launch", "4", "--single-frame-steps", "0"]
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--backend", "gloo"] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    three = _line(r.stdout)
    assert three["n_gpus"] == 3 and three["config"]["frames_per_launch"] == 4
    assert len(three["config"]["ranks"]) == 3 and len(three["rank_ms_per_step"]["per_rank"]) == 3
    assert three["l2_vs_cpu"]["identical_pixels"] == 1.0


@pytest.mark.timeout(400)
def test_bench_force_collective_nccl_world_one():
    """the RCCL branch of the N > 1 step, executed on the one GPU.  `bench.py --gpus 1
    --backend nccl --force-collective` starts torch.distributed.run with ONE rank itself, runs
    init_process_group("nccl", device_id=dev), the device-tensor all_gather_object / all_reduce / all_gather,
    the async dist.gather of every multi-frame group into rank 0's DEVICE `gathered` buffer with
    work.wait() ordering the stream, and prt_scatter_frames from that buffer — the code the driver's 8-GPU
    line runs, minus the xGMI transport between distinct GPUs.  The gathered frame of a timed group must
    equal the CPU oracle bit for bit."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONUNBUFFERED="1")
    args = ["--res", "128", "--spp", "8", "--depth", "8", "--tile", "16", "--steps", "8", "--warmup", "1",
            "--numpy-seconds", "0", "--cpu-seconds", "2", "--frames-per-launch", "4", "--single-frame-steps", "2"]
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--backend", "nccl", "--force-collective"] + args,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = _line(r.stdout)
    c = line["config"]
    assert line["n_gpus"] == 1 and c["backend"] == "nccl" and c["collective"] is True
    assert len(c["ranks"]) == 1 and c["ranks"][0]["rank"] == 0 and c["frames_per_launch"] == 4
    l2 = line["l2_vs_cpu"]
    assert l2["source"] == "timed group" and l2["gathered"] is True and l2["frames_per_launch"] == 4
    assert l2["identical_pixels"] == 1.0 and l2["rmse"] == 0.0 and l2["pass"]
    assert line["single_frame"]["ms_per_step"] > 0 and line["value"] > 0
