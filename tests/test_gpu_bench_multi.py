"""bench.py's N > 1 code path, rehearsed on one GPU: `python -m torch.distributed.run
--nproc-per-node 2 bench.py --gpus 2 --backend gloo` as a fresh subprocess (both ranks render
their latin-interleaved tiles on device 0 with the HIP kernel, the tile sums are staged through
host memory, gathered to rank 0 and scattered into the frame on the device by libprt's scatter
kernel).  The line must report 2 GPUs, a frame bit-identical to the CPU oracle on its sample, and
per-rank work counters that sum to the one-process counts.  The only piece of the driver's
8-GPU run this leaves untested is the RCCL transport itself.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

ARGS = ["--res", "128", "--spp", "8", "--depth", "8", "--tile", "16", "--steps", "2", "--warmup", "1",
        "--numpy-seconds", "0", "--cpu-seconds", "2"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


@pytest.mark.timeout(400)
def test_bench_two_ranks_over_gloo_on_one_gpu():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--backend", "gloo"] + ARGS
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    two = _line(r.stdout)
    assert two["n_gpus"] == 2 and two["config"]["backend"] == "gloo"
    assert two["l2_vs_cpu"]["identical_pixels"] == 1.0 and two["l2_vs_cpu"]["pass"]
    assert two["value"] > 0 and two["steps"] == 2
    r1 = subprocess.run([sys.executable, "bench.py"] + ARGS + ["--no-cpu-baseline"], cwd=ROOT, env=env,
                        capture_output=True, text=True, timeout=200)
    assert r1.returncode == 0, r1.stdout[-3000:] + r1.stderr[-3000:]
    one = _line(r1.stdout)
    assert one["n_gpus"] == 1
    a, b = two["work_totals"], one["work_totals"]
    # path queries depend only on the (seed, pixel, sample) streams: exact for any tile split
    assert a["ext_queries"] == b["ext_queries"] and a["shadow_queries"] == b["shadow_queries"], (a, b)
    # node / triangle counts also depend on which lanes share a wave (leaf-phase thresholds)
    for k in ("nodes", "tris"):
        assert abs(a[k] - b[k]) <= 0.01 * b[k], (k, a, b)
