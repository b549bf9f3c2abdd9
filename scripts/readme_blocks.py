"""The README's SDR callback granularity (65 536 IQ samples per call): per-kernel
device time per block and wall time per block, numpy and device-tensor inputs
(diagnostic for small-call latency)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-liquiddsp_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
import liquiddsp as L  # noqa: E402

dev = torch.device("cuda", 0)
blk, nblk = int(os.environ.get("BLK", "65536")), 64
x = bench.synth_channel(blk * nblk, 0, dev)
radio = bench.AMRadio(L)
for i in range(4):
    radio(x[i * blk:(i + 1) * blk])
torch.cuda.synchronize()
L._profile_reset()
L._profile_enable(True)
t0 = time.perf_counter()
for i in range(nblk):
    radio(x[i * blk:(i + 1) * blk])
torch.cuda.synchronize()
el = time.perf_counter() - t0
L._profile_enable(False)
kp = {k: round(v[1] / nblk * 1e3, 1) for k, v in L._profile_report().items()}
print(json.dumps({"block": blk, "ms_per_block": round(el / nblk * 1e3, 3), "kernel_us_per_block": kp}))
