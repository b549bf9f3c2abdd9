"""AmpModem short-call loop (k_pll_seqc) on the README chain's AmpModem input:
per-call kernel time and the batches with a directly evaluated step.  One JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "python-liquiddsp_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
import liquiddsp as L  # noqa: E402

dev = torch.device("cuda", 0)
blk, nblk = int(os.environ.get("BLK", "65536")), 48
x = bench.synth_channel(blk * nblk, 0, dev)
radio = bench.AMRadio(L)
ins = []
for i in range(nblk):
    ins.append(radio.agc(radio.resample(radio.bandpass(x[i * blk:(i + 1) * blk]))).clone())
torch.cuda.synchronize()
am = L.AmpModem(modulation=0.5, type="dsb", carrier=True)
for v in ins[:4]:
    am(v)
torch.cuda.synchronize()
b0, r0 = am._seq_stats()
L._profile_reset()
L._profile_enable(True)
for v in ins[4:]:
    am(v)
torch.cuda.synchronize()
L._profile_enable(False)
b1, r1 = am._seq_stats()
rep = {k: round(v[1] / v[0] * 1e3, 1) for k, v in L._profile_report().items()}
print(json.dumps({"samples_per_call": int(ins[0].numel()),
                  "kernel_us": rep, "batches": b1 - b0, "redone": r1 - r0,
                  "redone_frac": round((r1 - r0) / max(1, b1 - b0), 4)}))
