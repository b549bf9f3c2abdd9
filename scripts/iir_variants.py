"""Timing decomposition of k_iir_modal (tuning build, LDSP_PKG_DIR=build_tuning):
LDSP_IIR_VARIANT bit 0 drops the look-back, bit 1 pass 2, bit 2 pass 1 + scan
(wrong outputs; timing only); bit 3 staggers the first round of workgroups by
(variant >> 4) x ~3.4 us steps (outputs unchanged).  64 Mi complex samples,
cheby2 order 8.  python iir_variants.py [v,v,...]"""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR", os.path.join(REPO, "python-liquiddsp_amd"))]
import torch
import liquiddsp as L

n = 64 << 20
x = (torch.randn(n, dtype=torch.complex64, device="cuda"))
f = L.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2000000)
f._scan_path(2)
res = {}
vs = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1, 2, 4, 3, 5, 6, 7, 0]
for v in vs:
    os.environ["LDSP_IIR_VARIANT"] = str(v)
    f(x)
    torch.cuda.synchronize()
    L._profile_reset()
    L._profile_enable(True)
    for _ in range(10):
        f(x)
    torch.cuda.synchronize()
    L._profile_enable(False)
    r = L._profile_report()
    res[str(v)] = round(r["k_iir_modal"][1] / r["k_iir_modal"][0], 4)
print(json.dumps(res))
