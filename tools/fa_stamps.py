"""Per-phase cycle breakdown of the assembly flash-attention dK/dV kernel from a timestamp build
(PIAMD_FA_STAMP=1 fa_gen.py → an .hsaco given by PIAMD_FA_HSACO): every wave writes s_memtime at
6 points of every tile over the dV output ([wg][wave][tile][8] u64):
  0 tile start, 1 after A0 (MFMA 15), 2 after A1 (31), 3 after C0 (47), 4 after the barrier,
  5 tile end (after MFMA 63). The stamp itself drains lgkmcnt (adds a little to each phase).

  PIAMD_FA_HSACO=.../fa_stamp.hsaco python tools/fa_stamps.py [B,S,H,D]
"""
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_infer_amd  # noqa: E402,F401
from paddle_infer_amd.ops import attention  # noqa: E402


def main():
    B, S, H, D = map(int, (sys.argv[1] if len(sys.argv) > 1 else "96,1024,16,128").split(","))
    torch.manual_seed(0)
    q, k, v, do = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(4))
    sc = 1 / math.sqrt(D)
    o, lse = attention._fwd(q, k, v, True, sc)
    dq, dk = torch.empty_like(q), torch.empty_like(k)
    for _ in range(3):
        dv = torch.zeros_like(v)
        attention._bwd(q, k, v, o, lse, do, dq, dk, dv, True, sc)
    torch.cuda.synchronize()
    st = dv.view(-1).view(torch.int64)[: 256 * 4 * 256 * 8].cpu().numpy().reshape(256, 4, 256, 8)
    res = {}
    ph = ["A0", "A1", "C0", "barrier", "C1", "between"]
    rows = []
    for wg in range(256):
        for w in range(4):
            t = st[wg, w]
            n = int((t[:, 0] != 0).sum())
            if n < 3:
                continue
            t = t[:n, :6].astype(np.int64)
            d = np.diff(t, axis=1)                       # 5 in-tile phases
            between = t[1:, 0] - t[:-1, 5]               # end of tile → start of next
            rows.append((d[1:], between, t[-1, 5] - t[0, 0], n))
    dd = np.concatenate([r[0] for r in rows])
    bt = np.concatenate([r[1] for r in rows])
    for i, name in enumerate(ph[:5]):
        res[name] = dict(mean=float(dd[:, i].mean()), median=float(np.median(dd[:, i])),
                         p90=float(np.percentile(dd[:, i], 90)))
    res["between"] = dict(mean=float(bt.mean()), median=float(np.median(bt)), p90=float(np.percentile(bt, 90)),
                          p99=float(np.percentile(bt, 99)), max=float(bt.max()))
    tile = dd.sum(1)
    res["tile_total"] = dict(mean=float(tile.mean()), median=float(np.median(tile)))
    res["tiles_per_wave"] = float(np.mean([r[3] for r in rows]))
    res["wave_span_cycles"] = float(np.mean([r[2] for r in rows]))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
