"""The README's SDR callback granularity (65 536 IQ samples per call): per-kernel
device time per block and wall time per block, numpy and device-tensor inputs
(diagnostic for small-call latency)."""
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
blk, nblk = int(os.environ.get("BLK", "65536")), 64
x = bench.synth_channel(blk * nblk, 0, dev)
res = {"block": blk}
for nst in (1, 2, 3, 4):
    radio = bench.AMRadio(L)
    strm = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nst - 1)]
    for i in range(4):
        with torch.cuda.stream(strm[i % nst]):
            radio(x[i * blk:(i + 1) * blk])
    torch.cuda.synchronize()
    if nst == 1:
        L._profile_reset()
        L._profile_enable(True)
    t0 = time.perf_counter()
    for i in range(nblk):
        with torch.cuda.stream(strm[i % nst]):
            radio(x[i * blk:(i + 1) * blk])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if nst == 1:
        L._profile_enable(False)
        res["kernel_us_per_block"] = {k: round(v[1] / nblk * 1e3, 1) for k, v in L._profile_report().items()}
    res[f"streams{nst}"] = {"ms_per_block": round(el / nblk * 1e3, 3), "Msamples_s": round(blk * nblk / el / 1e6, 1)}
print(json.dumps(res))
