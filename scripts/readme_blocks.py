"""The README callback's rates (bench.host_path): 65 536-sample blocks as numpy
arrays through every stage, the same blocks as device tensors (1 and 3 streams),
and the PCIe-inclusive whole-buffer paths."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR", os.path.join(REPO, "python-liquiddsp_amd"))]
import bench  # noqa: E402
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402

for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    print(json.dumps(bench.host_path(L, torch.device("cuda", 0))), flush=True)
