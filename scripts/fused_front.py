"""IIR -> resampler fusion (liquiddsp.filter_resample) at the bench size: per-kernel
HIP-event times of the fused front against the two calls on 64 Mi samples
(`front`), or the multi-channel component (8 AMRadio chains on one GPU) with or
without it (`channels fused|unfused`; one per process: a second run's streams
would share hardware queues with the first's).
    python fused_front.py front | channels fused|unfused [streams per channel] [split] [prio] [c=<channels>]
(split: front and back stages on separate streams; prio: the back streams at high priority)"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR", os.path.join(REPO, "python-liquiddsp_amd"))]
import bench  # noqa: E402  (sets GPU_MAX_HW_QUEUES before torch initialises HIP)
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402

dev = torch.device("cuda", 0)
n = 64 << 20
mode = sys.argv[1] if len(sys.argv) > 1 else "front"
if mode == "channels":
    per = int(sys.argv[3]) if len(sys.argv) > 3 else 2       # streams per channel
    ch = [int(a[2:]) for a in sys.argv[4:] if a.startswith("c=")]      # channel count (default 8)
    print(json.dumps(bench.multi_channel(L, dev, channels=ch[0] if ch else 8, fused=(sys.argv[2] == "fused"), per=per,
                                         split="split" in sys.argv[4:], prio="prio" in sys.argv[4:])), flush=True)
    sys.exit(0)
x = bench.synth_channel(n, 0, dev)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    L._profile_reset()
    L._profile_enable(True)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    L._profile_enable(False)
    return {k: round(v[1] / v[0], 4) for k, v in L._profile_report().items()}


r1, r2 = bench.AMRadio(L), bench.AMRadio(L)
out = {"two_calls": timed(lambda: r1.resample(r1.bandpass(x))),
       "fused": timed(lambda: L.filter_resample(r2.bandpass, r2.resample, x))}
for k in ("two_calls", "fused"):
    out[k + "_ms"] = round(sum(out[k].values()), 4)
print(json.dumps(out), flush=True)
