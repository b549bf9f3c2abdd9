"""One AMRadio call alone on one stream (the bench chain, 64 Mi IQ), kernel by
kernel: start / end relative to the call's first kernel, from a tuning-build
LDSP_PROF_TIMELINE dump (LDSP_PKG_DIR=build_tuning, LDSP_PROF_TIMELINE=<file>).
Prints the last of 4 calls (the first ones warm the objects up)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "build_tuning")]
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402
from bench import AMRadio, synth_channel  # noqa: E402

tl = os.environ["LDSP_PROF_TIMELINE"]
dev = torch.device("cuda", 0)
x = synth_channel(64 << 20, 0, dev)
r = AMRadio(L)
for _ in range(3):
    r(x)
torch.cuda.synchronize()
open(tl, "w").close()
L._profile_reset()
L._profile_enable(True)
r(x)
torch.cuda.synchronize()
L._profile_enable(False)
L._profile_report()          # collects the launches' events (and appends them to the timeline)
rows = [l.split() for l in open(tl) if l.strip()]
rows = sorted(((n, float(a), float(b)) for n, s, a, b in rows), key=lambda t: t[1])
t0 = rows[0][1]
out = [{"kernel": n, "start_ms": round(a - t0, 4), "end_ms": round(b - t0, 4), "ms": round(b - a, 4)} for n, a, b in rows]
for o in out:
    print(f"{o['kernel']:24s} {o['start_ms']:8.4f} {o['end_ms']:8.4f} {o['ms']:8.4f}")
print(json.dumps({"call_ms": round(rows[-1][2] - t0, 4), "kernels": out}))
