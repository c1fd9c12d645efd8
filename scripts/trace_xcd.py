"""Per-XCD view of the kNN pass phase trace: each block records its XCD (HW_REG_XCC_ID, trace
slot 15).  Prints, per XCD, the median / max stream-end and arrival times (us from the earliest
start), to tell XCD-level imbalance from CU-level imbalance (GPU box measurement)."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from spatialflink_amd import Context, _abi, synth  # noqa: E402

n, K, R, GN = 10_000_000, 50, 0.5, 100
ctx = Context(0)
bj, q = synth.BEIJING, synth.README_QUERY
grid = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / GN, GN)
xs, ys = [], []
for w in range(4):
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    ctx.synth_uniform_async(x, y, 0, 2 + 7919 * w, bj)
    xs.append(x)
    ys.append(y)
torch.cuda.synchronize()
acc_se, acc_ar, acc_x = [], [], []
for rep in range(8):
    for w in range(4):
        ctx.knn_pp(grid, xs[w], ys[w], q[0], q[1], R, K)
    tr = ctx.debug_knn_pass_trace(grid, xs[rep % 4], ys[rep % 4], q[0], q[1], R, K, 0).astype(np.int64)
    t0 = tr[:, 0].min()
    rel = (tr - t0) / 100.0
    acc_se.append(rel[:, 1])
    acc_ar.append(rel[:, 4])
    acc_x.append(tr[:, 15] & 0xF)
se = np.stack(acc_se)  # [rep, block]
ar = np.stack(acc_ar)
nb = se.shape[1]
print("blocks", nb)
xid = np.stack(acc_x)
print("block -> XCC id consistent across reps:", bool((xid == xid[0]).all()), "| b % 8 == id (up to a rotation):",
      len({int((xid[0, b] - b) % 8) for b in range(nb)}) == 1)
for x in range(8):
    sel = xid == x
    se_x = np.where(sel, se, np.nan)
    ar_x = np.where(sel, ar, np.nan)
    print(f"xcc {x}: blocks {int(sel[0].sum()):3d} stream_end med {np.nanmedian(se_x):6.2f} max "
          f"{np.nanmax(se_x, 1).mean():6.2f}  arrived med {np.nanmedian(ar_x):6.2f} max {np.nanmax(ar_x, 1).mean():6.2f}")
# correlation of a block's lateness across reps (a slow CU stays slow?)
z = se - se.mean(1, keepdims=True)
c = np.corrcoef(z)
print("rep-to-rep correlation of per-block stream end (mean off-diagonal):", float((c.sum() - len(c)) / (len(c) ** 2 - len(c))))
print("stream_end spread per rep (max - median):", np.round(se.max(1) - np.median(se, 1), 2).tolist())
