"""The AGC stage alone on the bench channel's AGC input (64 Mi IQ -> 1.6 M
samples): per-kernel device time with nothing else running, against the same
calls inside the chain (bench.py's kernels)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-liquiddsp_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
import liquiddsp as L  # noqa: E402

dev = torch.device("cuda", 0)
radio = bench.AMRadio(L)
x = bench.synth_channel(64 << 20, 0, dev)
ins = []
for k in range(6):
    ins.append(radio.resample(radio.bandpass(x)).clone())
torch.cuda.synchronize()
agc = L.AGC()
agc.lock = False
agc.scale = 0.01
for k in range(2):
    agc(ins[k])
torch.cuda.synchronize()
L._profile_reset()
L._profile_enable(True)
for k in range(2, 6):
    agc(ins[k])
    torch.cuda.synchronize()
L._profile_enable(False)
print(json.dumps({k: round(v[1] / v[0], 4) for k, v in L._profile_report().items()}))
