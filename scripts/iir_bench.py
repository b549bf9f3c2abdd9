"""Fast-mode ComplexIIRFilter at 64 Mi samples (the chain's first stage, cheby2
order 8): the modal single-pass scan against the blocked scan, complex64 and
int16 IQ (from_bytes) input; per-kernel device times from libldsp's HIP events.
LDSP_PKG_DIR selects another build of the package (A/B runs)."""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "python-liquiddsp_amd")]
import torch
import liquiddsp as L

dev = torch.device("cuda", 0)
n = 64 << 20
g = torch.Generator(device=dev)
g.manual_seed(1)
raw = torch.randint(-32768, 32768, (2 * n,), generator=g, device=dev, dtype=torch.int32).to(torch.int16)
xc = L.bytes_to_iq(raw)
iir = dict(filter_type="cheby2", order=8, Fc=15000 / 2000000)
reps = int(os.environ.get("REPS", "10"))


def timed(fn):
    fn()
    torch.cuda.synchronize()
    L._profile_reset()
    L._profile_enable(True)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    L._profile_enable(False)
    return {k: round(v[1] / v[0], 4) for k, v in L._profile_report().items()}


res = {}
for path, name in ((2, "modal"), (1, "blocked")):
    f = L.ComplexIIRFilter(**iir)
    f._scan_path(path)
    res[name] = timed(lambda: f(xc))
    f2 = L.ComplexIIRFilter(**iir)
    f2._scan_path(path)
    res[name + "_iq16"] = timed(lambda: f2.from_bytes(raw))
for k in list(res):
    res[k + "_ms"] = round(sum(res[k].values()), 4)
alg = 16 * n
res["modal_alg_GBs"] = round(alg / res["modal_ms"] / 1e6, 1)
res["modal_hbm_frac"] = round(alg / res["modal_ms"] / 1e6 / 8000, 4)
print(json.dumps(res))
