"""The bench's batched channel components alone (8 channels x 64 Mi and 16
channels x 32 Mi IQ per step, many-call launches on 4 rotating streams), for
A/B runs of the tuning knobs:
    LDSP_PKG_DIR=build_tuning LDSP_AGC_WMUL=5 python3 scripts/batched_run.py"""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR", os.path.join(REPO, "python-liquiddsp_amd"))]
import torch  # noqa: E402
import bench  # noqa: E402
import liquiddsp as L  # noqa: E402

dev = torch.device("cuda", 0)
bs = [torch.cuda.Stream(dev) for _ in range(int(os.environ.get("BATCHED_STREAMS", "4")))]
print(json.dumps({"batched_8": bench.multi_channel_batched(L, dev, 8, strm=bs),
                  "batched_16": bench.multi_channel_batched(L, dev, 16, n=32 << 20, strm=bs)}))
