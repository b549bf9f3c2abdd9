"""Record how far the build variants of the CPU restatement diverge from each
other (tests/golden/variants.json) and freeze each variant's outputs on the
golden inputs (tests/golden/variants.npz).

Why: the reference's arithmetic lives in liquid-dsp, which is absent here and
unpinned.  Two platform choices of a real liquid-dsp build move
its output and are not knowable from the reference:
  * the libm its feedback loops call (agc_crcf expf/logf, src/agc.hpp:115;
    ampmodem cargf, src/demod.hpp:294; Costas tanhf);
  * the order its SIMD dotprod sums in (firfilt / firpfb / iirfilt TF,
    src/firfilter.hpp:33, src/resampler.hpp:165).
The restatement builds four variants (oracle/Makefile): fdlibm + portable order
("default", which the GPU exact mode reproduces bit for bit), glibc ("libm"),
8-lane SIMD order ("simd") and both ("libm_simd").  The divergence between them
bounds what "parity with liquid-dsp" can mean for each stage; the GPU tests
(tests/test_gpu_variants.py) check the GPU outputs against every variant with
the tolerances derived here.

Run from the repository root:   python tests/golden/make_variants.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from oracle import oracle as O  # noqa: E402
from make_golden import am_signal  # noqa: E402


def divergence(y, ref):
    """max|y - ref| / max|ref|, its 99.9th percentile and the fractions of samples above 1e-6 / 1e-5."""
    d = np.abs(np.asarray(y).astype(np.complex128) - np.asarray(ref).astype(np.complex128))
    d /= max(float(np.max(np.abs(ref))), 1e-30)
    return {"maxrel": float(d.max()), "p999": float(np.quantile(d, 0.999)),
            "frac_gt_1e-6": float(np.mean(d > 1e-6)), "frac_gt_1e-5": float(np.mean(d > 1e-5))}


def stage_outputs(M, g):
    """Every stage of the AMRadio path on the golden inputs, evaluated by variant module M."""
    out = {}
    out["fir127_y"] = M.FIRFilter(g["fir127_h"], cplx=True)(g["fir127_x"])
    out["resamp_y"] = M.Resampler(float(np.float32(48000 / 2000000)), m=20, fc=0.024, As=60.0, npfb=13,
                                  cplx=True)(g["resamp_x"])
    agc = M.AGC()
    agc.lock(False)
    agc.scale = 0.01
    out["agc_y"] = agc(g["agc_x"])
    out["ampmodem_y"] = M.AmpModem(0.5, "dsb", True)(out["agc_y"])
    out["ampmodem_costas_y"] = M.AmpModem(0.75, "dsb", False)(out["agc_y"])
    out["chain_y"] = M.AMRadio()(g["chain_x"])
    return out


def main():
    g = dict(np.load(os.path.join(HERE, "golden.npz")))
    fix, meta = {}, {"generator": "tests/golden/make_variants.py",
                     "variants": {"default": "fdlibm transcendentals, portable dotprod order (= GPU exact mode)",
                                  "libm": "system libm (glibc) in the feedback loops",
                                  "simd": "8-lane SIMD dotprod order (partial sums, pairwise reduction, sequential tail)",
                                  "libm_simd": "glibc + SIMD order (a typical Linux x86-64 liquid-dsp build)"},
                     "golden_inputs": {}, "long_chain": {}}
    outs = {v: stage_outputs(O.variant(v), g) for v in O.VARIANTS}
    for v, o in outs.items():
        for k, y in o.items():
            fix[f"{v}__{k}"] = y
    for k in outs["default"]:
        meta["golden_inputs"][k] = {v: divergence(outs[v][k], outs["default"][k]) for v in O.VARIANTS
                                    if v != "default"}
    # the chain over 4 Mi IQ samples of SURVEY C4 (seed 4): divergence between every pair of variants
    x = am_signal(1 << 22)
    ys = {v: O.variant(v).AMRadio()(x) for v in O.VARIANTS}
    ys["f64_iir"] = O.AMRadio(iir_f64=True)(x)
    names = list(ys)
    for i, a in enumerate(names):
        for b in names[i + 1:]:
            meta["long_chain"][f"{a} vs {b}"] = divergence(ys[a], ys[b])
    meta["long_chain_input"] = "make_golden.am_signal(4194304) (SURVEY C4, seed 4): 100664 PCM samples"
    spread = max(d["maxrel"] for k, d in meta["long_chain"].items() if "f64_iir" not in k)
    meta["chain_variant_spread_maxrel"] = spread
    np.savez(os.path.join(HERE, "variants.npz"), **fix)
    with open(os.path.join(HERE, "variants.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    print(json.dumps(meta["golden_inputs"], indent=1))
    print(json.dumps(meta["long_chain"], indent=1))
    print(f"wrote variants.npz ({os.path.getsize(os.path.join(HERE, 'variants.npz')) / 1e6:.2f} MB)")


if __name__ == "__main__":
    main()
