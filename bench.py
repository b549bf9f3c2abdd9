"""Benchmark: the AMRadio receive chain (README.md:41-58 of the reference):
ComplexIIRFilter(cheby2, order 8) -> ComplexResampler(48k/2M) -> AGC ->
AmpModem(dsb, carrier) -> DeemphasisFilter, on synthetic 2 MS/s AM IQ.

One step = one __call__ of the chain on a block of N complex64 samples that is
already resident in HBM (torch tensor on the GPU).  One process per GPU: every
rank demodulates its own independent channel (weak scaling, no data-path
collective).  Prints ONE JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n SAMPLES]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
# HIP hardware queues per process (read at HIP init, before torch loads it): the
# chain rotates 4 streams and the multi-channel component 2 per channel (16); with
# HIP's default of 4 (also the GPU box's setting) those streams share queues and
# serialise.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 32:
    os.environ["GPU_MAX_HW_QUEUES"] = "32"
# LDSP_PKG_DIR: load the liquiddsp package from another build of it (e.g. the
# tuning build of python-liquiddsp_amd/Makefile); default: the in-tree product.
PKG_DIR = os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "python-liquiddsp_amd")
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
# Serial floor of one PLL-walk repair, derived from the hardware's hop latencies and
# fixed across rounds (it no longer follows the walker's own loop).  A repair is at
# least the dependent chain  s_ff1 (next event lane j) -> v_readlane (lane j's kicks)
# -> v_mad (offsets of the later lanes) -> v_add -> v_cmp (their events, into VCC)
# -> s_ff1.  scripts/ubench/chain_lat.hip measured on MI355X (profiles/r04d_chain_lat.txt):
# C3  s_ff1 -> v_readlane -> v_add -> v_cmp -> s_and (-> s_ff1)  72 clocks per iteration;
# the repair has one more VALU -> VALU hop (C5: 56 / 4 = 14 clocks) and no s_and
# (C0: SALU -> SALU 56 / 4 = 14 clocks), so 72 + 14 - 14 = 72 shader clocks at the
# 2384 MHz s_memtime clock of the same run = 30.2 ns.  (The walker's loop itself runs
# a repair in 89 clocks = 37.3 ns, scripts/ubench/walk_loop.hip V10; the walk also
# pays its lane-block transitions, which this floor does not count.)
REPAIR_FLOOR_NS = 30.2
FP32_PEAK_TFLOPS = 157.3       # MI355X FP32 vector spec


# Carrier offset per rank.  Rank 0 is SURVEY C4 exactly (+1.2 kHz, seed 4).  The
# other channels use offsets inside the AmpModem PLL's lock range: its phase
# detector sits behind a 51-tap fc = 0.01 lowpass (480 Hz at 48 kS/s), and
# measured on the CPU restatement the loop locks up to ~1.2 kHz but never at
# +-3.5 kHz (SURVEY C5's offsets), where it cycle-slips indefinitely.
CARRIERS = [1200.0, -1200.0, 900.0, -900.0, 600.0, -600.0, 300.0, -300.0]


def synth_channel(n, rank, device):
    """AM DSB with carrier at 2 MS/s: 0.1 (1 + 0.5 m(t)) e^{j(2 pi f t + phi)} + AWGN (30 dB SNR)."""
    g = torch.Generator(device=device)
    g.manual_seed(4 if rank == 0 else 10 + rank)
    fs = 2.0e6
    fcar = CARRIERS[rank % len(CARRIERS)]
    t = torch.arange(n, device=device, dtype=torch.float64) / fs
    msg = (torch.sin(2 * np.pi * 400 * t) + torch.sin(2 * np.pi * 1000 * t) + torch.sin(2 * np.pi * 2500 * t)) / 3
    ph = 2 * np.pi * fcar * t + 0.3 * (rank + 1)
    amp = 0.1 * (1 + 0.5 * msg)
    sig = torch.complex((amp * torch.cos(ph)).float(), (amp * torch.sin(ph)).float())
    sigma = 0.1 * 10 ** (-30 / 20) / np.sqrt(2)
    noise = torch.complex(torch.randn(n, generator=g, device=device), torch.randn(n, generator=g, device=device))
    return (sig + sigma * noise).contiguous()


class AMRadio:
    """The reference README's AMRadio callback, on the MI355X classes."""

    def __init__(self, L, bandwidth=15000, iq_rate=2000000, pcm_rate=48000, fused_front=False):
        # fused_front: the IIR and the resampler as one call (liquiddsp.filter_resample,
        # same bits; the filter's outputs stay on chip) -- the multi-channel component
        self.L = L
        self.fused_front = fused_front
        self.bandpass = L.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=bandwidth / iq_rate)
        self.resample = L.ComplexResampler(rate=pcm_rate / iq_rate, Fc=pcm_rate / iq_rate)
        self.am = L.AmpModem(modulation=0.5, type="dsb", carrier=True)
        self.audio_filter = L.DeemphasisFilter(pcm_rate)
        self.agc = L.AGC()
        self.agc.lock = False
        self.agc.scale = 0.01

    def stages(self):
        return [("iir", self.bandpass), ("resamp", self.resample), ("agc", self.agc), ("ampmodem", self.am),
                ("deemph", self.audio_filter)]

    def __call__(self, iq, events=None, front_done=None):
        # front_done: a torch event recorded once the resampler's call is enqueued
        # (the next step's chain waits for it, bench.py main: pipeline depth)
        x = iq
        if self.fused_front and events is None:
            x = self.L.filter_resample(self.bandpass, self.resample, x)
            if front_done is not None:
                front_done.record()
            for st in (self.agc, self.am, self.audio_filter):
                x = st(x)
            return x
        for i, (name, st) in enumerate(self.stages()):
            if events is not None:
                events[i][0].record()
            x = st(x)
            if events is not None:
                events[i][1].record()
            if name == "resamp" and front_done is not None:
                front_done.record()
        return x


def timed_steps(step, steps, warmup, sync, barrier):
    """W untimed warmup steps, then exactly K steps bracketed by a barrier and a
    device synchronize on both sides; returns this rank's wall time (s).
    step(k, w) gets the timed index k (None while warming up) and the warmup index w."""
    for w in range(warmup):
        step(None, w)
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k, None)
    sync()
    barrier()
    return time.perf_counter() - t0


def reduce_max(elapsed, device):
    """Max of the per-rank wall times (the job takes as long as its slowest rank).
    gloo reduces host tensors: the value travels on the CPU then."""
    import torch.distributed as tdist
    if tdist.is_initialized() and tdist.get_backend() == "gloo":
        device = torch.device("cpu")
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())


def aggregate_value(world, n_per_rank, steps, elapsed):
    """Whole-job throughput: IQ samples all ranks processed / max wall time (Msamples/s)."""
    return world * n_per_rank * steps / elapsed / 1e6


def scatter_channels(x_all, n, device):
    """SURVEY 8(e) input scatter: rank 0 holds every channel's IQ block and
    sends channel r to rank r with grouped point-to-point sends (RCCL has no
    scatter primitive; over xGMI every peer has its own link).  Complex
    blocks travel as their float32 (re, im) view.  Returns this rank's block."""
    import torch.distributed as tdist
    rank, world = tdist.get_rank(), tdist.get_world_size()
    if rank == 0:
        mine = x_all[0]
        ops = [tdist.P2POp(tdist.isend, torch.view_as_real(x_all[r]), r) for r in range(1, world)]
    else:
        mine = torch.empty(n, dtype=torch.complex64, device=device)
        ops = [tdist.P2POp(tdist.irecv, torch.view_as_real(mine), 0)]
    if ops:
        for req in tdist.batch_isend_irecv(ops):
            req.wait()
    return mine


def gather_pcm(y):
    """SURVEY 8(e) output gather: every rank's PCM block (same length on all
    ranks: same rates, same block size) to rank 0.  Returns the list on rank 0."""
    import torch.distributed as tdist
    rank, world = tdist.get_rank(), tdist.get_world_size()
    if rank != 0:
        for req in tdist.batch_isend_irecv([tdist.P2POp(tdist.isend, y, 0)]):
            req.wait()
        return None
    outs = [y] + [torch.empty_like(y) for _ in range(1, world)]
    ops = [tdist.P2POp(tdist.irecv, outs[r], r) for r in range(1, world)]
    if ops:
        for req in tdist.batch_isend_irecv(ops):
            req.wait()
    return outs


def host_info():
    """the box's host CPU next to the CPU baseline (nproc, model, clock)."""
    info = {"nproc": os.cpu_count()}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name") and "model" not in info:
                    info["model"] = line.split(":", 1)[1].strip()
                elif line.startswith("cpu MHz") and "mhz" not in info:
                    info["mhz"] = float(line.split(":", 1)[1])
    except OSError:
        pass
    return info


def _cpu_block(n, carrier, seed):
    """synth_channel's AM signal, in numpy, for the CPU legs."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 2e6
    msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t) + np.sin(2 * np.pi * 2500 * t)) / 3
    return (0.1 * (1 + 0.5 * msg) * np.exp(1j * (2 * np.pi * carrier * t))
            + 0.00224 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)


def _cpu_run(radio, x, seconds):
    """README-style 65,536-sample callbacks over x, repeated for about `seconds`;
    returns (IQ samples done, elapsed s).  The oracle's ctypes calls release the GIL."""
    done = 0
    t0 = time.perf_counter()
    while True:
        for i in range(0, len(x), 65536):
            radio(x[i:i + 65536])
        done += len(x)
        el = time.perf_counter() - t0
        if el >= seconds:
            return done, el


def cpu_baseline(n_iq, seconds=10.0, c5_seconds=5.0):
    """Time the CPU restatement (oracle/, -O3) on bounded samples: one channel on
    one thread (BASELINE config 4, the reported value) and SURVEY 8(d)'s C5 leg,
    8 independent channels on min(8, nproc) threads."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    n = 1 << 22
    x = _cpu_block(n, 1200.0, 4)
    done, el = _cpu_run(O.AMRadio(), x, seconds)
    res = {"value": round(done / el / 1e6, 3), "unit": "Msamples/s", "cores": 1, "kind": "port",
           "sample": f"{done} IQ samples ({done // n} passes over a {n}-sample synthetic AM block) through the "
                     f"oracle AMRadio chain in 65536-sample calls, single thread, {el:.1f} s"}
    if c5_seconds > 0:
        threads = max(1, min(8, os.cpu_count() or 1))
        nc = 1 << 20
        blocks = [_cpu_block(nc, CARRIERS[c], 10 + c) for c in range(8)]

        def channel(c):
            return _cpu_run(O.AMRadio(), blocks[c], c5_seconds)
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            outs = list(ex.map(channel, range(8)))
        wall = time.perf_counter() - t0
        tot = sum(d for d, _ in outs)
        res["c5_channels"] = {
            "value": round(tot / wall / 1e6, 3), "unit": "Msamples/s", "channels": 8, "cores": threads,
            "sample": f"8 channels (carriers {CARRIERS}, seeds 10-17), {nc} IQ samples each, repeated "
                      f"~{c5_seconds:.0f} s per channel in 65536-sample calls, {threads} threads, {wall:.1f} s wall"}
    return res


def _divergence(y, ref):
    """|y - ref| / max|ref| over the PCM samples (tests/test_gpu_chain.py)."""
    d = np.abs(np.asarray(y, np.float64) - np.asarray(ref, np.float64)) / np.max(np.abs(ref))
    return {"maxrel": float(d.max()), "p999": float(np.quantile(d, 0.999)), "n_diff": int(np.sum(d > 0)),
            "frac_gt_1e-5": float(np.mean(d > 1e-5))}


def parity_check(L, device, n=4 << 20):
    """The headline chain's measured divergence, next to `value`,
    outside the timed region and part of the CPU leg (the oracle is the checker
    here, never the thing measured): on the first n samples of the bench channel
    (C4, seed 4), the benchmarked fast chain and the exact chain against the CPU
    restatement (float32, = liquid's arithmetic) and against the restatement with
    a float64 IIR (the truth the fast IIR approximates).  The gates are those of
    tests/test_gpu_chain.py: IIR stage <= 1e-6 and <= the float32 recursion's own
    error; chain p999 / samples off <= the float32 restatement's; largest single
    deviation <= the spread of liquid's build variants (tests/golden/variants.json)."""
    from oracle import oracle as O
    xd = synth_channel(n, 0, device)
    x = xd.cpu().numpy()
    fast = AMRadio(L)
    y_fast = fast(xd).cpu().numpy()
    ex = AMRadio(L)
    ex.bandpass.exact = True
    y_exact = ex(xd).cpu().numpy()
    iir = L.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2000000)
    y_iir = iir(xd).cpu().numpy()
    o = O.IIRFilter(prototype=("cheby2", "lowpass", 1, 8, np.float32(15000 / 2000000), 0.3, 0.7, 60.0))
    t_iir = o.execute_f64(x)
    o.reset()
    f32_iir = o(x)

    def maxrel(a, b):
        return float(np.max(np.abs(np.asarray(a, np.complex128) - b)) / np.max(np.abs(b)))
    e_gpu, e_f32 = maxrel(y_iir, t_iir), maxrel(f32_iir, t_iir)
    truth = O.AMRadio(iir_f64=True)(x)
    f32 = O.AMRadio()(x)
    dg, df, dr = _divergence(y_fast, truth), _divergence(f32, truth), _divergence(y_fast, f32)
    with open(os.path.join(REPO, "tests", "golden", "variants.json")) as f:
        spread = json.load(f)["chain_variant_spread_maxrel"]
    exact_bits = bool(y_exact.shape == f32.shape and np.array_equal(y_exact.view(np.uint32), f32.view(np.uint32)))
    gates = {"iir_stage_le_1e-6": e_gpu <= 1e-6, "iir_stage_le_f32_recursion": e_gpu <= e_f32,
             "chain_p999_le_f32": dg["p999"] <= df["p999"], "chain_n_diff_le_f32": dg["n_diff"] <= df["n_diff"],
             "chain_maxrel_le_variant_spread": dg["maxrel"] <= spread, "exact_chain_bitwise": exact_bits}
    return {"prefix_iq_samples": n, "pcm_samples": int(f32.size),
            "mode": "fast (default: modal float64 IIR scan; every later stage exact given its input)",
            "fast_vs_restatement_f32": dr, "fast_vs_f64_iir_truth": dg, "restatement_f32_vs_f64_iir_truth": df,
            "iir_stage_maxrel_vs_f64": {"gpu_fast": e_gpu, "restatement_f32": e_f32},
            "variant_spread_maxrel": spread, "exact_mode_bitwise_vs_restatement": exact_bits,
            "gates": gates, "all_gates_pass": all(gates.values())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    # (--iq-samples under torch.distributed.run, whose parser takes "--n" for a prefix of its own options)
    ap.add_argument("--n", "--iq-samples", dest="n", type=int, default=64 * 1024 * 1024)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-components", action="store_true")
    ap.add_argument("--streams", type=int, default=4,
                    help="HIP streams the steps rotate over (1 = every step on torch's current stream). "
                         "Each object orders its own calls across streams (libldsp StreamMark), so step k+1's "
                         "IIR/resampler/AGC/candidate kernels overlap step k's serial PLL walk")
    ap.add_argument("--channel", type=int, default=None,
                    help="synthetic channel (carrier offset / seed) this rank demodulates; default: its rank")
    ap.add_argument("--no-kprof", action="store_true",
                    help="no per-kernel HIP events inside the timed steps (kernel times then come from a separate "
                         "profiled pass)")
    ap.add_argument("--dist", action="store_true",
                    help="initialise torch.distributed (RCCL) even at world size 1: the multi-GPU code path "
                         "(nccl init, barriers, max-over-ranks all-reduce) on a one-GPU box under torch.distributed.run")
    ap.add_argument("--scatter", action="store_true",
                    help="rank 0 holds all channels: every step scatters the IQ blocks and gathers the PCM "
                         "(SURVEY 8e) instead of each rank reading a resident channel")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process-group backend for world size > 1: nccl (RCCL, one GPU per rank) or gloo, which "
                         "also runs several ranks on one GPU (rank r on device r mod the device count) -- the "
                         "multi-process libldsp path on a one-GPU box (tests/test_gpu_dist.py)")
    ap.add_argument("--walk-early", type=int, choices=(0, 1), default=1,
                    help="the PLL walker's early hand-off (default on); 0: each walker waits in stream order, so a "
                         "rocprofv3 kernel trace times the walk itself (the walk-duration cross-check)")
    ap.add_argument("--dump-pcm", default=None,
                    help="write each rank's last PCM block to <prefix>.rank<r>.npy (parity checks)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1 or (args.dist and "RANK" in os.environ)
    if args.backend == "gloo":
        if args.scatter:
            ap.error("--scatter sends device tensors: nccl only")
        local = local % max(1, torch.cuda.device_count())     # (counting devices does not initialise HIP)
    if dist:
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if args.backend == "gloo":
            tdist.init_process_group("gloo")
        else:
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    import liquiddsp as L
    if not args.walk_early:
        L._debug_walk_early(0)
    x = synth_channel(args.n, rank if args.channel is None else args.channel, device)
    x_all = None
    if args.scatter and dist and rank == 0:
        x_all = torch.stack([x] + [synth_channel(args.n, r, device) for r in range(1, world)])
    radio = AMRadio(L)
    nst = len(radio.stages())

    events = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nst)]
              for _ in range(args.steps)]
    out = {}

    nstreams = 1 if (args.scatter and dist) else max(1, args.streams)
    streams = [torch.cuda.current_stream(device)] + [torch.cuda.Stream(device) for _ in range(nstreams - 1)]
    barrier = tdist.barrier if dist else (lambda: None)

    host = {"t": 0.0, "max": 0.0}
    # Pipeline depth: each step's chain waits (on the GPU, no host sync) until the
    # previous step's resampler call is done.  Without it the rotating streams start
    # every step's IIR at once and the first step's resampler and AGC kernels wait
    # behind three other full-GPU filter launches (1.1 ms for a
    # 0.12 ms resampler); with it the filters still run one step ahead of the walks.
    front = {"ev": None}

    def step(k, w=None, prof=False, rot=nstreams, walk_only=False):
        # warmup steps rotate over the streams too: the first use of a stream makes torch's
        # caching allocator map fresh 512 MB blocks for it, which must not land in the timed steps
        h0 = time.perf_counter()
        if k == 0 and (prof or walk_only):
            L._profile_reset()                 # HIP events over exactly these steps
            L._profile_only("k_pll_walk" if walk_only else "")
            L._profile_enable(True)
        xin = scatter_channels(x_all, args.n, device) if (args.scatter and dist) else x
        with torch.cuda.stream(streams[(k if k is not None else (w or 0)) % rot]):
            if front["ev"] is not None and rot > 1:
                torch.cuda.current_stream().wait_event(front["ev"])
            ev = torch.cuda.Event() if rot > 1 else None
            out["y"] = radio(xin, events[k] if (k is not None and prof) else None, front_done=ev)
            front["ev"] = ev
        if args.scatter and dist:
            gather_pcm(out["y"])
        if k is not None:
            dt = time.perf_counter() - h0
            host["t"] += dt
            host["max"] = max(host["max"], dt)

    kp = not args.no_kprof
    # setup, before the W warm-up steps: one chain call per stream, so torch's caching
    # allocator holds blocks for every stream whatever W the caller asks for
    if not (args.scatter and dist):
        for si in range(nstreams):
            with torch.cuda.stream(streams[si]):
                radio(x)
        torch.cuda.synchronize()
    # The timed steps carry HIP events around the dominant kernel's launches only (the
    # PLL walk: 2 events per step, on its launch stream, for roofline.ms_per_launch);
    # per-kernel and per-stage times come from a separate profiled pass over the same
    # steps right after (events around every launch cost ~0.03 ms per step).
    act0 = radio.am._walk_active()      # walker device clocks (ticks, walks) so far (synchronises)
    elapsed = timed_steps(lambda k, w: step(k, w, walk_only=kp), args.steps, args.warmup, torch.cuda.synchronize,
                          barrier)
    act1 = radio.am._walk_active()
    host_ms = host["t"] / args.steps * 1e3
    host_max_ms = host["max"] * 1e3
    L._profile_enable(False)
    walk_timed = L._profile_report().get("k_pll_walk")
    timed_steps(lambda k, w: step(k, w, prof=True), args.steps, 0, torch.cuda.synchronize, barrier)
    L._profile_enable(False)
    L._profile_only("")
    kprof = L._profile_report()
    # the same chain with every step on one stream (no overlap between steps), for reference
    single = timed_steps(lambda k, w: step(k, w, prof=False, rot=1), min(args.steps, 5), 1, torch.cuda.synchronize,
                         barrier)
    single_steps = min(args.steps, 5)
    if dist:
        elapsed = reduce_max(elapsed, device)
        single = reduce_max(single, device)
    y = out["y"]

    stage_ms = {name: float(np.mean([events[k][i][0].elapsed_time(events[k][i][1]) for k in range(args.steps)]))
                for i, (name, _) in enumerate(radio.stages())}
    n_pcm = int(y.numel())
    value = aggregate_value(world, args.n, args.steps, elapsed)

    # Algorithmic bytes per launch (read the stage input once, write
    # its output once; complex64 = 8 B, float32 = 4 B).  Multi-kernel stages
    # attribute the stage minimum to the kernel that produces the stage output.
    n = args.n
    alg = {"k_iir_modal": 16 * n, "k_iir_scan_local": 8 * n, "k_iir_scan_carry": 0, "k_iir_scan_final": 16 * n,
           "k_iir_blk_local": 8 * n, "k_iir_blk_final": 16 * n,
           "k_resamp": 8 * n + 8 * n_pcm, "k_agc_chunks": 16 * n_pcm, "k_agc_verify": 0,
           "k_fir_exact": 8 * n_pcm + 8 * n_pcm, "k_pll_cand": 12 * n_pcm, "k_pll_walk": 12 * n_pcm,
           "k_iir_spec_chunks": 8 * n_pcm, "k_iir_spec_verify": 0, "k_delay_hist": 0}
    kernels = {}
    for name, (calls, tot) in kprof.items():
        per = tot / calls
        ab = alg.get(name, 0)
        kernels[name] = {"calls_per_step": round(calls / args.steps, 2), "ms": round(per, 4),
                         "alg_GBs": round(ab / (per * 1e-3) / 1e9, 2) if ab else None}
    dom = max(kprof, key=lambda k: kprof[k][1])
    dom_ms = kprof[dom][1] / kprof[dom][0]
    dom_src = "profiled pass after the timed steps"
    walk_events_ms = None
    if dom == "k_pll_walk" and walk_timed:
        dom_ms = walk_events_ms = walk_timed[1] / walk_timed[0]
        dom_src = "HIP events around its launches inside the timed steps"
    if dom == "k_pll_walk" and act1[1] > act0[1]:
        # a walker is dispatched as soon as its candidates are ready and waits on the
        # device for the previous walk's state (capi.cpp amp_pll_stage): its launch
        # (HIP events, rocprof) spans that wait; the walk itself is timed by its own
        # clock from the hand-off to its end, over every walk of the W + K steps
        dom_ms = (act1[0] - act0[0]) * 1e-5 / (act1[1] - act0[1])
        dom_src = ("walker device clock (s_memrealtime) from the hand-off to the end, mean over the "
                   f"{act1[1] - act0[1]} walks of the warm-up and timed steps; HIP events around the launches, "
                   "which include the early-dispatched walker's wait: " +
                   (f"{walk_events_ms:.4f} ms" if walk_events_ms else "n/a"))
    achieved = alg.get(dom, 0) / (dom_ms * 1e-3) / 1e9
    entries, repairs, fallbacks = radio.am._walk_stats()       # the last call's walk (synchronises)
    res = {
        "metric": "Msamples/s on AM chain (IIR->resample->AGC->demod), 2 MS/s IQ; HBM GB/s vs roofline",
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": "AMRadio chain (cheby2 IIR ord8 -> resampler 48k/2M -> AGC -> AmpModem dsb+carrier "
                               "-> de-emphasis), one independent channel per GPU",
                   "samples_per_step_per_gpu": args.n, "iq_rate": 2000000, "pcm_rate": 48000,
                   "pcm_samples_per_step": n_pcm,
                   "carrier_hz": CARRIERS[(rank if args.channel is None else args.channel) % len(CARRIERS)],
                   "seed": 4 if (rank if args.channel is None else args.channel) == 0 else 10 + (rank if args.channel is None else args.channel),
                   "parallelism": f"channel-per-gpu x{world}" + (" rank0-scatter/gather" if args.scatter and dist else "")
                   + (" (gloo, ranks sharing GPUs)" if dist and args.backend == "gloo" else "")},
        "roofline": dict(roofline(dom, dom_ms, achieved, entries, repairs, fallbacks), ms_source=dom_src),
        "streams": nstreams,
        "walk_early_handoff": bool(args.walk_early),
        "host_ms_per_step": round(host_ms, 4),
        "host_ms_max_step": round(host_max_ms, 4),
        "kernel_events_in_timed_steps": "k_pll_walk only" if kp else False,
        "pipeline": "each step waits for the previous step's resampler call (GPU event)" if nstreams > 1 else None,
        "single_stream_ms_per_step": round(single / single_steps * 1e3, 4),
        "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
        "kernels": kernels,
    }
    if rank == 0 and world == 1 and not args.no_components:
        res["components"] = components(L, device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:      # the CPU leg runs at N = 1 only
        res["cpu_baseline"] = cpu_baseline(args.n, args.cpu_seconds)
        res["cpu_baseline"]["host"] = host_info()
        res["parity"] = parity_check(L, device)
    if args.dump_pcm:
        np.save(f"{args.dump_pcm}.rank{rank}.npy", y.cpu().numpy())
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist:
        tdist.destroy_process_group()


def roofline(dom, dom_ms, achieved, entries, repairs, fallbacks):
    """The dominant kernel against the roof that bounds it.  The PLL walk is one
    serial chain of dependent repairs: its roof is the
    measured per-repair floor (scripts/ubench/walk_loop.hip), so the primary
    figures are repairs per ms against that floor; its HBM view is kept beside
    (12 B per PCM sample, a tiny fraction by construction)."""
    hbm = {"bound": "hbm", "kernel": dom, "ms_per_launch": round(dom_ms, 4), "achieved": round(achieved, 2),
           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
           "traffic": pmc_traffic("bench", dom), "traffic_source": PMC_SOURCE}
    if dom != "k_pll_walk":
        return hbm
    peak = 1e6 / REPAIR_FLOOR_NS                        # dependent repairs per ms at the floor
    ach = repairs / dom_ms if dom_ms else 0.0
    return {"bound": "serial", "kernel": dom, "ms_per_launch": round(dom_ms, 4),
            "achieved": round(ach, 1), "peak": round(peak, 1), "unit": "dependent repairs/ms",
            "frac": round(ach / peak, 3) if peak else None,
            "traffic": hbm["traffic"], "traffic_source": PMC_SOURCE,
            "serial_chain": {"entries": int(entries), "repairs": int(repairs), "fallback_lane_blocks": int(fallbacks),
                             "floor_ns_per_repair": REPAIR_FLOOR_NS,
                             "floor_ms": round(repairs * REPAIR_FLOOR_NS * 1e-6, 4)},
            "hbm": {k: hbm[k] for k in ("achieved", "peak", "unit", "frac")},
            "note": "the PLL recurrence is one serial walker wave: bounded by the dependent-repair latency "
                    "(floor_ns_per_repair), not by HBM (alg bytes 12 B per PCM sample)"}


def _pmc_summary():
    """Latest committed rocprofv3 PMC summary (scripts/prof_round.sh ->
    profiles/rNN_pmc_summary.json): per-kernel HBM bytes per launch from
    FETCH_SIZE (x2, gfx950 correction) + WRITE_SIZE, measured on the same
    commands in separate --pmc passes."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_summary.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        return json.load(f), os.path.relpath(files[-1], REPO)


PMC, PMC_SOURCE = _pmc_summary()


def rocprof_kernel(run, pattern):
    """Mean / min / max launch duration of the first kernel whose name contains
    `pattern` in the latest committed rocprofv3 --stats summary of `run`
    (profiles/rNN_<run>_kernel_stats.csv, scripts/prof_round.sh): the spread beside
    the mean (DVFS moves a sustained kernel's clock by ~20 %)."""
    import csv
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_{run}_kernel_stats.csv")))
    if not files:
        return None
    with open(files[-1]) as f:
        for r in csv.DictReader(f):
            if pattern in r["Name"]:
                return {"calls": int(r["Calls"]), "avg_ms": round(float(r["AverageNs"]) * 1e-6, 4),
                        "min_ms": round(float(r["MinNs"]) * 1e-6, 4), "max_ms": round(float(r["MaxNs"]) * 1e-6, 4),
                        "source": os.path.relpath(files[-1], REPO)}
    return None


def pmc_traffic(run, kernel):
    """HBM bytes per launch of `kernel` (a profiling label; the rocprof name may
    carry a variant suffix, e.g. k_fir_fft512x for the k_fir_fft512 label)."""
    try:
        d = PMC[run]
        k = kernel if kernel in d else next(n for n in sorted(d) if n.startswith(kernel))
        return round(d[k]["hbm_bytes"])
    except (TypeError, KeyError, StopIteration):
        return None


def components(L, device, reps=5):
    """The north-star kernel (127-tap ComplexFIRFilter on 64 Mi samples, target
    >= 50 % of the HBM roofline) and BASELINE config 3 (NCO.mix_down + 255-tap
    ComplexFIRFilter on 256 Mi samples), per-kernel HIP-event times."""
    g = torch.Generator(device=device)
    g.manual_seed(1)

    def kaiser(n, fc, As):
        beta = 0.1102 * (As - 8.7)
        t = np.arange(n) - (n - 1) / 2
        r = 2 * t / n
        return (np.sinc(2 * fc * t) * np.i0(beta * np.sqrt(1 - r * r)) / np.i0(beta)).astype(np.float32)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        L._profile_reset()
        L._profile_enable(True)
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        L._profile_enable(False)
        return {k: v[1] / v[0] for k, v in L._profile_report().items()}

    out = {}
    n = 64 << 20
    xs = torch.complex(torch.randn(n, generator=g, device=device), torch.randn(n, generator=g, device=device))
    for mode in ("fast", "direct"):
        f = L.ComplexFIRFilter(kaiser(127, 0.1, 60.0))
        f.mode = mode
        t = timed(lambda: f(xs))
        (kn, ms), = t.items()
        out[f"fir127_64Mi_{mode}"] = {"kernel": kn, "ms": round(ms, 4), "GBs": round(16 * n / ms / 1e6, 1),
                                      "hbm_frac": round(16 * n / ms / 1e6 / HBM_PEAK_GBS, 4),
                                      "direct_form_TFLOPs": round(4 * 127 * n / ms / 1e9, 2)}
        if mode == "fast":      # north-star roofline line: 16 B per complex sample (read + write once)
            out["north_star_roofline"] = {
                "kernel": "k_fir_fft512", "bound": "hbm", "achieved": round(16 * n / ms / 1e6, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(16 * n / ms / 1e6 / HBM_PEAK_GBS, 4),
                "traffic": pmc_traffic("fir", "k_fir_fft512"), "traffic_source": PMC_SOURCE,
                "alg_bytes": 16 * n, "target_frac": 0.5, "rocprof": rocprof_kernel("fir", "k_fir_fft512x")}
    # BASELINE config 2: ComplexResampler(rate = 48 k / 2 M) on 64 Mi samples, as one
    # call and as the README's 65 536-sample blocks (device tensors, one stream)
    rs = L.ComplexResampler(rate=48000 / 2000000, Fc=48000 / 2000000)
    t = timed(lambda: rs(xs))
    nout = int(rs(xs[:65536]).numel())
    rb = L.ComplexResampler(rate=48000 / 2000000, Fc=48000 / 2000000)
    blocks = [xs[i:i + 65536] for i in range(0, 1 << 22, 65536)]
    for b in blocks[:4]:
        rb(b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in blocks:
        rb(b)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kr = [k for k in t if k.startswith("k_resamp")][0]
    ab = 8 * n + 8 * round(n * 0.024)
    out["resampler_64Mi"] = {"kernel": kr, "ms": round(t[kr], 4), "Msamples_s": round(n / t[kr] / 1e3, 1),
                             "alg_GBs": round(ab / t[kr] / 1e6, 1), "hbm_frac": round(ab / t[kr] / 1e6 / HBM_PEAK_GBS, 4),
                             "blocks_65536_Msamples_s": round(len(blocks) * 65536 / el / 1e6, 1),
                             "outputs_per_65536": nout}
    del xs, blocks
    # the chain's first filter fed the SDR wire format.  Two
    # calls (bytes_to_iq, then the cheby2 IIR) against ComplexIIRFilter.from_bytes,
    # which converts int16 IQ in the blocked scan's loads (4 B / sample per pass).
    raw = torch.randint(-32768, 32768, (2 * n,), generator=g, device=device, dtype=torch.int32).to(torch.int16)
    iir = dict(filter_type="cheby2", order=8, Fc=15000 / 2000000)
    fa, fb = L.ComplexIIRFilter(**iir), L.ComplexIIRFilter(**iir)
    ta = timed(lambda: fa(L.bytes_to_iq(raw)))
    tb = timed(lambda: fb.from_bytes(raw))
    out["iq16_iir_64Mi"] = {"two_calls_ms": round(sum(ta.values()), 4), "fused_ms": round(sum(tb.values()), 4),
                            "two_calls_kernels": {k: round(v, 4) for k, v in ta.items()},
                            "fused_kernels": {k: round(v, 4) for k, v in tb.items()},
                            "alg_bytes_fused": 12 * n, "alg_bytes_two_calls": 24 * n}
    del raw
    out["exact_chain_64Mi"] = exact_chain(L, device, n)
    out["exact_channels_batched_8"] = exact_channels_batched(L, device)
    n = 256 << 20
    xs = torch.complex(torch.randn(n, generator=g, device=device), torch.randn(n, generator=g, device=device))
    nco = L.NCO("nco")
    nco.freq = float(2 * np.pi * 0.05)
    f2 = L.ComplexFIRFilter(kaiser(255, 0.05, 60.0))
    t = timed(lambda: f2(nco.mix_down(xs)))
    fk = [k for k in t if k.startswith("k_fir")][0]
    out["nco_fir255_256Mi"] = {"nco_ms": round(t["k_nco_mix"], 4), "fir_kernel": fk, "fir_ms": round(t[fk], 4),
                               "nco_GBs": round(16 * n / t["k_nco_mix"] / 1e6, 1),
                               "fir_GBs": round(16 * n / t[fk] / 1e6, 1),
                               "Msamples_s": round(n / (t["k_nco_mix"] + t[fk]) / 1e3, 1)}
    # the same chain fused (liquiddsp.mix_down_filter: the mix happens in the FIR's
    # window loads): 16 B per sample of HBM traffic instead of 32
    nco_f = L.NCO("nco")
    nco_f.freq = float(2 * np.pi * 0.05)
    f3 = L.ComplexFIRFilter(kaiser(255, 0.05, 60.0))
    t = timed(lambda: L.mix_down_filter(nco_f, f3, xs))
    (fk, ms), = t.items()
    rp = rocprof_kernel("fir", "k_fir_fft1024x<true")
    if rp:
        for k in ("avg_ms", "min_ms", "max_ms"):
            rp[k.replace("_ms", "_hbm_frac")] = round(16 * n / rp[k] / 1e6 / HBM_PEAK_GBS, 4)
    out["nco_fir255_256Mi_fused"] = {"kernel": fk, "ms": round(ms, 4), "Msamples_s": round(n / ms / 1e3, 1),
                                     "alg_GBs": round(16 * n / ms / 1e6, 1),
                                     "hbm_frac": round(16 * n / ms / 1e6 / HBM_PEAK_GBS, 4),
                                     "roof_ms": round(16 * n / HBM_PEAK_GBS / 1e6, 4), "rocprof": rp}
    del xs
    out["host_buffers"] = host_path(L, device)
    # both configurations on the same 16 streams: torch hands out streams from a
    # pool of 32 per device, so a second set of 16 (after the chain's 4) would wrap
    # onto streams the first set used and put two channels on one stream
    strm = [[torch.cuda.Stream(device) for _ in range(2)] for _ in range(8)]
    out["channels_per_gpu"] = multi_channel(L, device, fused=True, strm=strm)
    out["channels_per_gpu_unfused"] = multi_channel(L, device, strm=strm)
    # 4 rotating streams (112.7 GS/s vs 108.8 on 3, r05h), taken from the 16 above: every
    # new stream that a process uses takes the next of GPU_MAX_HW_QUEUES (32) hardware
    # queues, and past 32 streams share queues, i.e. run in order -- new streams here
    # (after ~27 used) gave 96-100 GS/s against 125-128 in a fresh process (r05zz, r05zw2)
    bs = [strm[c][0] for c in range(4)]
    out["channels_per_gpu_batched"] = multi_channel_batched(L, device, 8, strm=bs)
    out["channels_per_gpu_batched_16"] = multi_channel_batched(L, device, 16, n=32 << 20, strm=bs)
    return out


def exact_chain(L, device, n):
    """The benchmarked chain with bandpass.exact = True -- the configuration whose
    output is bit-identical to the restatement (tests/test_gpu_chain.py) -- one
    64 Mi step on one stream.  Its cheby2 IIR is the float32 DF-II recursion run
    in order, one wave per section and component (k_iir_sect): float32
    trajectories of this filter started early from another state do not coalesce
    bit for bit (scripts/analysis/iir_coalesce.py), so no
    chunk-parallel exact form exists for it."""
    x = synth_channel(n, 0, device)
    r = AMRadio(L)
    r.bandpass.exact = True
    r(x[:65536])
    torch.cuda.synchronize()
    L._profile_reset()
    L._profile_enable(True)
    t0 = time.perf_counter()
    r(x)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    L._profile_enable(False)
    kern = {k: round(v[1] / v[0], 3) for k, v in L._profile_report().items()}
    del x
    return {"ms_per_step": round(el * 1e3, 2), "Msamples_s": round(n / el / 1e6, 2), "kernels_ms": kern,
            "iir_kernel": "k_iir_sect", "note": "exact (bit-identical) mode: the IIR is one sequential recursion "
                                                "per section and component, a wave each"}


def exact_channels_batched(L, device, channels=8, n=64 << 20):
    """C independent exact (bit-identical) AMRadio chains on one GPU, one 64 Mi step
    each: the exact IIRs of all channels in ONE merged launch (execute_many ->
    k_iir_sect, one workgroup per channel and component), the resamplers per
    channel, the AGC / AmpModem / de-emphasis back half batched.  Same bits per
    channel as its own exact chain (tests/test_gpu_many.py)."""
    xs = [synth_channel(n, c % 8, device) for c in range(channels)]
    radios = [AMRadio(L) for _ in range(channels)]
    for r in radios:
        r.bandpass.exact = True

    def step(m):
        ys = L.execute_many([r.bandpass for r in radios], [x[:m] for x in xs])
        zs = [r.resample(y) for r, y in zip(radios, ys)]
        a = L.execute_many([r.agc for r in radios], zs)
        b = L.execute_many([r.am for r in radios], a)
        return L.execute_many([r.audio_filter for r in radios], b)
    step(65536)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step(n)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    del xs
    return {"channels": channels, "iq_samples_per_channel": n, "ms_per_step": round(el * 1e3, 2),
            "Msamples_s": round(channels * n / el / 1e6, 1), "iir_kernel": "k_iir_sect (merged, one launch)"}


def multi_channel_batched(L, device, channels=8, steps=10, n=64 << 20, per=4, strm=None):
    """The same C channels stepped with the many-calls (liquiddsp.filter_resample_many /
    execute_many): one kernel launch per stage for all channels, each step on one of
    `per` rotating streams (steps overlap: step k+1's filters run under step k's walks).
    Same bits per channel as the per-channel calls (tests/test_gpu_many.py)."""
    xs = [synth_channel(n, r % 8, device) for r in range(channels)]
    radios = [AMRadio(L) for _ in range(channels)]
    if strm is None:
        strm = [torch.cuda.Stream(device) for _ in range(per)]
    iirs, rss = [r.bandpass for r in radios], [r.resample for r in radios]
    agcs, ams, des = [r.agc for r in radios], [r.am for r in radios], [r.audio_filter for r in radios]

    def step(k, w=None):
        kk = k if k is not None else w
        with torch.cuda.stream(strm[kk % len(strm)]):
            a = L.filter_resample_many(iirs, rss, xs)
            L.execute_many(des, L.execute_many(ams, L.execute_many(agcs, a)))

    t = timed_steps(step, steps, max(2, len(strm)), torch.cuda.synchronize, lambda: None)
    del xs
    return {"channels": channels, "batched": True, "streams": len(strm), "steps": steps,
            "ms_per_step": round(t / steps * 1e3, 3), "Msamples_s": round(channels * n * steps / t / 1e6, 1),
            "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default")}


def multi_channel(L, device, channels=8, steps=10, n=64 << 20, per=2, split=False, fused=False, strm=None,
                  prio=False):
    """SURVEY 8(e)'s caveat: independent channels also share one GPU -- each
    channel's serial PLL walk / AGC repair occupy one CU, so C channels on C
    stream pairs overlap.  Aggregate IQ Msamples/s of `channels` AMRadio chains
    (BASELINE config 4 each, carriers as the ranks of config 5) on this GPU."""
    xs = [synth_channel(n, r, device) for r in range(channels)]
    radios = [AMRadio(L, fused_front=fused) for _ in range(channels)]
    if strm is None:
        strm = [[torch.cuda.Stream(device) for _ in range(per)] for _ in range(channels)]
    # split: the front stages (IIR, resampler, AGC) and the back stages (AmpModem,
    # de-emphasis) of a step on different streams, so that stream order never
    # holds a step's front behind an earlier step's walk
    # prio: the back stages' streams at high priority (the serial walk is each channel's long pole)
    back = [[torch.cuda.Stream(device, priority=-1 if prio else 0) for _ in range(per)] for _ in range(channels)] \
        if split else None

    def step(k, w=None):
        kk = k if k is not None else w
        for c in range(channels):
            if not split:
                with torch.cuda.stream(strm[c][kk % per]):
                    radios[c](xs[c])
                continue
            r = radios[c]
            with torch.cuda.stream(strm[c][kk % per]):
                a = r.agc(r.resample(r.bandpass(xs[c])))
                ev = torch.cuda.Event()
                ev.record()
            with torch.cuda.stream(back[c][kk % per]):
                torch.cuda.current_stream().wait_event(ev)
                r.audio_filter(r.am(a))

    # warm-up steps cover every stream (torch's caching allocator maps fresh blocks
    # for a stream's first use, which must not land in the timed steps)
    t = timed_steps(step, steps, max(2, per), torch.cuda.synchronize, lambda: None)
    del xs
    return {"channels": channels, "streams_per_channel": per * (2 if split else 1), "split_front_back": split,
            "fused_front": fused, "back_priority_high": bool(split and prio),
            "steps": steps, "ms_per_step": round(t / steps * 1e3, 3),
            "Msamples_s": round(channels * n * steps / t / 1e6, 1),
            "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default")}


def host_path(L, device, n=16 << 20, reps=3):
    """PCIe-inclusive rates of the AM chain when the caller hands over host
    buffers (never `value`): (a) one H2D copy of the IQ block, the chain on the
    device, one D2H copy of the PCM; (b) the README callback on numpy arrays,
    where every stage stages its input to HBM and its output back."""
    xh = synth_channel(n, 0, device).cpu().numpy()
    res = {"iq_samples": n}
    for name, fn in (("h2d_chain_d2h", lambda r: r(torch.from_numpy(xh).to(device)).cpu()),
                     ("numpy_every_stage", lambda r: r(xh))):
        radio = AMRadio(L)
        fn(radio)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn(radio)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / reps
        res[name] = {"ms": round(el * 1e3, 2), "Msamples_s": round(n / el / 1e6, 1)}
    # the README's SDR callback block: 65 536 IQ samples per numpy call (the
    # reference's own loop), and the same blocks as device tensors
    blk, nblk = 65536, 64
    for name, mk in (("readme_65536_numpy", lambda i: xh[i * blk:(i + 1) * blk]),
                     ("readme_65536_device", lambda i, xd=torch.from_numpy(xh[:blk * nblk]).to(device):
                      xd[i * blk:(i + 1) * blk])):
        for nst in ((1,) if name.endswith("numpy") else (1, 3)):
            radio = AMRadio(L)
            strm = [torch.cuda.current_stream(device)] + [torch.cuda.Stream(device) for _ in range(nst - 1)]
            for i in range(4):
                with torch.cuda.stream(strm[i % nst]):
                    radio(mk(i))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(nblk):
                with torch.cuda.stream(strm[i % nst]):
                    radio(mk(i))
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            res[name + ("" if nst == 1 else f"_{nst}streams")] = {"ms_per_block": round(el / nblk * 1e3, 3),
                                                                  "Msamples_s": round(blk * nblk / el / 1e6, 1)}
    return res


if __name__ == "__main__":
    main()
