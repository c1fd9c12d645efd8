"""Per-XCD view of the kNN pass phase trace: block b runs on XCD b % 8 (round-robin dispatch).
Prints, per XCD, the median / max stream-end and arrival times (us from the earliest start), to
tell XCD-level imbalance from CU-level imbalance (GPU box measurement)."""
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
acc_se, acc_ar = [], []
for rep in range(8):
    for w in range(4):
        ctx.knn_pp(grid, xs[w], ys[w], q[0], q[1], R, K)
    tr = ctx.debug_knn_pass_trace(grid, xs[rep % 4], ys[rep % 4], q[0], q[1], R, K, 0).astype(np.int64)
    t0 = tr[:, 0].min()
    rel = (tr - t0) / 100.0
    acc_se.append(rel[:, 1])
    acc_ar.append(rel[:, 4])
se = np.stack(acc_se)  # [rep, block]
ar = np.stack(acc_ar)
nb = se.shape[1]
print("blocks", nb)
for x in range(8):
    b = np.arange(x, nb, 8)
    print(f"xcd {x}: stream_end med {np.median(se[:, b]):6.2f} max {se[:, b].max(1).mean():6.2f}  "
          f"arrived med {np.median(ar[:, b]):6.2f} max {ar[:, b].max(1).mean():6.2f}")
# correlation of a block's lateness across reps (a slow CU stays slow?)
z = se - se.mean(1, keepdims=True)
c = np.corrcoef(z)
print("rep-to-rep correlation of per-block stream end (mean off-diagonal):", float((c.sum() - len(c)) / (len(c) ** 2 - len(c))))
print("stream_end spread per rep (max - median):", np.round(se.max(1) - np.median(se, 1), 2).tolist())
