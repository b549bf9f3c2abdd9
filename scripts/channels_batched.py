"""Multi-channel throughput on one GPU: C AMRadio chains (bench.py) per step,
batched (liquiddsp many-calls, one launch per stage for all channels) against the
per-channel calls (2 streams per channel, fused front).
    python scripts/channels_batched.py [C ...]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402

dev = torch.device("cuda", 0)
for C in [int(a) for a in sys.argv[1:]] or [8]:
    for per in (2, 3, 4):
        r = bench.multi_channel_batched(L, dev, C, n=(64 << 20) if C <= 8 else (32 << 20), per=per)
        print(json.dumps(r), flush=True)
    if C == 8:
        print(json.dumps(bench.multi_channel(L, dev, fused=True)), flush=True)
