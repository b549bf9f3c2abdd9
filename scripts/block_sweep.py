"""AMRadio chain throughput vs call size (device tensors; 1 stream, and 4
rotating streams): where the chunk-parallel paths take over from the one-lane
loops.  Prints one JSON line."""
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
total = 1 << 26
x = bench.synth_channel(total, 0, dev)
res = {}
for lg in range(16, 27, 2):
    blk = 1 << lg
    nblk = max(4, min(64, (1 << 28) // blk // 4))
    for nst in (1, 4):
        radio = bench.AMRadio(L)
        strm = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nst - 1)]
        blocks = [x[(i * blk) % total:(i * blk) % total + blk] for i in range(nblk + nst)]
        for i in range(nst):
            with torch.cuda.stream(strm[i % nst]):
                radio(blocks[i])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(nblk):
            with torch.cuda.stream(strm[i % nst]):
                radio(blocks[nst + i])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        res[f"2^{lg}_streams{nst}"] = {"ms_per_call": round(el / nblk * 1e3, 3), "Msamples_s": round(blk * nblk / el / 1e6, 1)}
        print(f"2^{lg} streams {nst}", res[f"2^{lg}_streams{nst}"], flush=True)
print(json.dumps(res))
