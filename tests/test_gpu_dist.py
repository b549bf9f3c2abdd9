"""The bench's multi-GPU code path on real hardware: one process
under torch.distributed.run with the nccl backend (RCCL), i.e. the process-group
init, the barriers around the timed steps, the max-over-ranks all-reduce of the
wall time and, with --scatter, rank 0's grouped send / receive of the channel
blocks -- at world size 1, the only size a one-GPU box can run (RCCL needs one
GPU per rank; world size 2 runs on CPU with gloo in test_bench_dist.py).  The
child is a separate process started by torch.distributed.run (no exec)."""
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
