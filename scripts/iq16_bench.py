"""bytes_to_iq + ComplexIIRFilter (two calls) against ComplexIIRFilter.from_bytes
(fused) at 64 Mi samples: per-kernel device times (libldsp HIP events)."""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-liquiddsp_amd")]
import torch
import liquiddsp as L

dev = torch.device("cuda", 0)
n = 64 << 20
g = torch.Generator(device=dev)
g.manual_seed(1)
raw = torch.randint(-32768, 32768, (2 * n,), generator=g, device=dev, dtype=torch.int32).to(torch.int16)
iir = dict(filter_type="cheby2", order=8, Fc=15000 / 2000000)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    L._profile_reset()
    L._profile_enable(True)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    L._profile_enable(False)
    return {k: round(v[1] / v[0], 4) for k, v in L._profile_report().items()}


fa, fb, fc = (L.ComplexIIRFilter(**iir) for _ in range(3))
xc = L.bytes_to_iq(raw)
res = {"complex_in": timed(lambda: fc(xc)), "two_calls": timed(lambda: fa(L.bytes_to_iq(raw))),
       "fused": timed(lambda: fb.from_bytes(raw))}
for k in list(res):
    res[k + "_ms"] = round(sum(res[k].values()), 4)
print(json.dumps(res))
