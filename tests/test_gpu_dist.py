"""The bench's multi-GPU code path on real hardware: one process
under torch.distributed.run with the nccl backend (RCCL), i.e. the process-group
init, the barriers around the timed steps, the max-over-ranks all-reduce of the
wall time and, with --scatter, rank 0's grouped send / receive of the channel
blocks -- at world size 1, the only size a one-GPU box can run (RCCL needs one
GPU per rank; world size 2 runs on CPU with gloo in test_bench_dist.py) -- and
two libldsp processes sharing the one GPU over a gloo process group.  The
children are separate processes started by torch.distributed.run (no exec)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("scatter", [False, True])
def test_bench_rccl_world1(scatter):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--dist", "--steps", "3",
           "--warmup", "1", "--no-cpu-baseline", "--no-components", "--iq-samples", str(1 << 22)]
    if scatter:
        cmd.append("--scatter")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 1 and res["steps"] == 3 and res["value"] > 0
    assert res["config"]["parallelism"].startswith("channel-per-gpu x1")
    assert ("rank0-scatter/gather" in res["config"]["parallelism"]) == scatter


def test_bench_two_ranks_one_gpu_gloo(tmp_path):
    """Two libldsp processes on one GPU: torch.distributed.run
    starts two ranks (gloo process group; both on cuda:0), each demodulates its
    own channel with its own streams, stream pools and object handles.  Each
    rank's PCM must equal, bit for bit, a single-process run of that channel with
    the same call sequence, and the line's value must be the whole-job figure
    (both ranks' samples over the max-over-ranks wall time)."""
    import numpy as np
    n, steps = 1 << 22, 3
    common = ["bench.py", "--steps", str(steps), "--warmup", "1", "--no-cpu-baseline", "--no-components",
              "--iq-samples", str(n)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + common + \
          ["--backend", "gloo", "--dump-pcm", str(tmp_path / "two")]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == steps
    assert "gloo" in res["config"]["parallelism"]
    # value = 2 ranks x n x steps / (max wall time), ms_per_step = that time / steps
    assert abs(res["value"] - 2 * n / (res["ms_per_step"] * 1e-3) / 1e6) <= 1e-3 * res["value"] + 0.01
    for ch in (0, 1):
        s1 = subprocess.run([sys.executable] + common + ["--channel", str(ch), "--dump-pcm", str(tmp_path / f"one{ch}")],
                            cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
        assert s1.returncode == 0, s1.stderr[-3000:]
        a = np.load(tmp_path / f"two.rank{ch}.npy")
        b = np.load(tmp_path / f"one{ch}.rank0.npy")
        assert a.shape == b.shape and a.size > 90_000
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), ch
