"""In-kernel re-runs of small AGC calls on the README chain's AGC input
(65 536-IQ blocks -> ~1 573 samples per call): calls, chunks re-run, time per call."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "python-liquiddsp_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
import liquiddsp as L  # noqa: E402

dev = torch.device("cuda", 0)
blk, nblk = 65536, 64
x = bench.synth_channel(blk * nblk, 0, dev)
radio = bench.AMRadio(L)
ins = []
for i in range(nblk):
    v = radio.resample(radio.bandpass(x[i * blk:(i + 1) * blk]))
    ins.append(v.clone())
torch.cuda.synchronize()
agc = L.AGC()
agc.lock = False
agc.scale = 0.01
t0 = time.perf_counter()
for v in ins:
    agc(v)
torch.cuda.synchronize()
el = time.perf_counter() - t0
print(json.dumps({"calls": nblk, "samples_per_call": int(ins[0].numel()), "reruns": agc._tsa_reruns(),
                  "us_per_call": round(el / nblk * 1e6, 1)}))
