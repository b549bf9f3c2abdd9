"""The bench's multi-rank path (one independent AM channel per rank, no
data-path collective; max-over-ranks wall time; whole-job throughput) on CPU
with the gloo backend at world size 2.  The per-rank step is the CPU
restatement of the chain (oracle/, allowed in tests) on that rank's channel, so
the test also checks that every rank's synthetic channel is a lockable AM
signal that demodulates to its message.
"""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, outdir):
    sys.path.insert(0, REPO)
    import bench
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1 << 18
    x = bench.synth_channel(n, rank, torch.device("cpu")).numpy()
    radio = O.AMRadio()
    outs = []

    def step(k, w=None):
        outs.append(np.concatenate([radio(x[i:i + 65536]) for i in range(0, n, 65536)]))

    mine = bench.timed_steps(step, 2, 1, lambda: None, dist.barrier)
    job = bench.reduce_max(mine, torch.device("cpu"))
    y = outs[-1]
    # the message (400/1000/2500 Hz tones) survives demodulation: correlate the
    # PCM output with the tones at 48 kS/s after the AGC / PLL settle
    t = np.arange(y.size) / 48000.0
    msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t) + np.sin(2 * np.pi * 2500 * t)) / 3
    tail = slice(y.size // 2, None)
    best = max(abs(np.corrcoef(np.roll(msg, d)[tail], y[tail])[0, 1]) for d in range(0, 80))
    res = {"rank": rank, "mine": mine, "job": job, "n_out": int(y.size), "corr": float(best),
           "value": bench.aggregate_value(world, n, 2, job), "carrier": bench.CARRIERS[rank % len(bench.CARRIERS)]}
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
        json.dump(res, fh)
    dist.destroy_process_group()


def test_two_rank_gloo_weak_scaling(tmp_path):
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    # max over ranks: every rank sees the same job time, no smaller than its own
    assert rs[0]["job"] == rs[1]["job"]
    assert all(r["job"] >= r["mine"] for r in rs)
    # whole-job throughput = samples of all ranks / job time
    assert rs[0]["value"] == pytest.approx(world * (1 << 18) * 2 / rs[0]["job"] / 1e6)
    # independent channels (different carriers), each demodulated correctly
    assert rs[0]["carrier"] != rs[1]["carrier"]
    assert all(r["n_out"] == rs[0]["n_out"] for r in rs)
    assert all(r["corr"] > 0.8 for r in rs), [r["corr"] for r in rs]     # de-emphasis shapes the tones


def _scatter_main(rank, world, port, outdir):
    sys.path.insert(0, REPO)
    import bench
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1 << 17
    dev = torch.device("cpu")
    x_all = torch.stack([bench.synth_channel(n, r, dev) for r in range(world)]) if rank == 0 else None
    mine = bench.scatter_channels(x_all, n, dev)
    local = bench.synth_channel(n, rank, dev)          # what this rank would synthesise itself
    y = torch.from_numpy(np.concatenate([O.AMRadio()(mine.numpy()[i:i + 65536]) for i in range(0, n, 65536)]))
    outs = bench.gather_pcm(y)
    res = {"rank": rank, "same_block": bool(torch.equal(mine, local)), "n_out": int(y.numel())}
    if rank == 0:
        # rank 0 holds every channel's PCM; recompute each here and compare bitwise
        ok = []
        for r in range(world):
            ref = np.concatenate([O.AMRadio()(x_all[r].numpy()[i:i + 65536]) for i in range(0, n, 65536)])
            ok.append(bool(np.array_equal(outs[r].numpy().view(np.uint32), ref.view(np.uint32))))
        res["gathered_ok"] = ok
    with open(os.path.join(outdir, f"s{rank}.json"), "w") as fh:
        json.dump(res, fh)
    dist.destroy_process_group()


def test_two_rank_gloo_scatter_gather(tmp_path):
    """SURVEY 8(e) scatter / gather mode (bench.py --scatter): rank 0's blocks
    reach their ranks intact and every rank's PCM comes back to rank 0."""
    world = 2
    mp.spawn(_scatter_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rs = [json.load(open(tmp_path / f"s{r}.json")) for r in range(world)]
    assert all(r["same_block"] for r in rs)
    assert rs[0]["gathered_ok"] == [True] * world
