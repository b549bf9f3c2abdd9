"""Round-3 advice: a filter with a long look-back (Butterworth order 8 at Fc =
0.001: J = 28 units) at the bench size -- the modal scan (forced, _scan_path 2)
against the blocked scan (_scan_path 1) and the default choice (IirObj::modal_pays),
64 Mi complex samples, per-kernel HIP-event times, and the two outputs' agreement."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-liquiddsp_amd")]
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402

dev = torch.device("cuda", 0)
n = 64 << 20
g = torch.Generator(device=dev)
g.manual_seed(3)
x = torch.complex(torch.randn(n, generator=g, device=dev), torch.randn(n, generator=g, device=dev))
out = {}
ys = {}
for name, path in (("modal", 2), ("blocked", 1), ("default", 0)):
    f = L.ComplexIIRFilter(filter_type="butter", order=8, Fc=0.001)
    f._scan_path(path)
    out["J"] = f._modal_info()[2]
    f(x[:65536])
    torch.cuda.synchronize()
    f.reset()
    L._profile_reset()
    L._profile_enable(True)
    ys[name] = f(x)
    torch.cuda.synchronize()
    L._profile_enable(False)
    out[name] = {k: round(v[1] / v[0], 4) for k, v in L._profile_report().items()}
d = (ys["modal"] - ys["blocked"]).abs().max().item() / ys["blocked"].abs().max().item()
out["modal_vs_blocked_maxrel"] = d
print(json.dumps(out), flush=True)
