"""PLL walk: time spent redoing walker blocks whose interval test failed (the
tuning build's product walker accumulates s_memrealtime ticks around each block
redo into the walk statistics).  Bench chain (bench.py AMRadio, 64 Mi IQ per
call), one stream; per call: entries, repairs, fallback lane-blocks, redone
blocks and their device time.
    LDSP_PKG_DIR=build_tuning python scripts/walk_fallback_cost.py [calls]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (sets the package path, GPU_MAX_HW_QUEUES)
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda", 0)
x = bench.synth_channel(64 << 20, 0, dev)
r = bench.AMRadio(L)
rows = []
for i in range(calls):
    L._profile_reset()
    L._profile_only("k_pll_walk")
    L._profile_enable(True)
    r(x)
    torch.cuda.synchronize()
    L._profile_enable(False)
    walk = L._profile_report()["k_pll_walk"]
    e, rep, fb = r.am._walk_stats()
    ticks, packed = r.am._walk_clocks()
    blocks, undo, fbt = packed & 0xffff, (packed >> 16) & 0xffffff, (packed >> 40) & 0xffffff
    rows.append({"walk_ms": round(walk[1] / walk[0], 4), "entries": e, "repairs": rep, "fallback_lane_blocks": fb,
                 "redone_blocks": blocks, "redo_ms": round(ticks * 1e-5, 4), "undo_ms": round(undo * 1e-5, 4),
                 "fallback_lb_ms": round(fbt * 1e-5, 4)})
L._profile_only("")
print(json.dumps({"calls": rows,
                  "mean_redo_ms": round(sum(r_["redo_ms"] for r_ in rows[1:]) / max(1, len(rows) - 1), 4),
                  "mean_walk_ms": round(sum(r_["walk_ms"] for r_ in rows[1:]) / max(1, len(rows) - 1), 4)}))
