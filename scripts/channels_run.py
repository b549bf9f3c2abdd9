"""The bench's channels_per_gpu component alone (8 AMRadio chains, 2 streams
each, 64 Mi IQ per channel per step), for a rocprofv3 kernel trace:
    rocprofv3 --kernel-trace --output-format csv -d DIR -o ch -- python3 scripts/channels_run.py
then scripts/trace_summary.py DIR."""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR", os.path.join(REPO, "python-liquiddsp_amd"))]
os.environ.setdefault("GPU_MAX_HW_QUEUES", "32")
import torch
import bench
import liquiddsp as L

steps = int(os.environ.get("STEPS", "6"))
ch = int(os.environ.get("CHANNELS", "8"))
print(json.dumps(bench.multi_channel(L, torch.device("cuda", 0), channels=ch, steps=steps, per=int(os.environ.get("PER", "2")),
                                        split=os.environ.get("SPLIT", "0") == "1")))
