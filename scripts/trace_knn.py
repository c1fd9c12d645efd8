"""Phase timeline of one kNN scan launch (MODE 6 timestamps, 100 MHz clock): per-block start,
stream-loop end, flush end, list written, ticket; then the last block's final-selection
phases.  Prints percentiles in microseconds relative to the earliest block start."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from spatialflink_amd import Context, _abi, synth  # noqa: E402

n = 10_000_000
W = 4
shapes = [tuple(int(v) for v in s.split(",")) for s in sys.argv[1:]] or [(4, 1, 32), (16, 1, 16)]
ctx = Context(0)
bj = synth.BEIJING
q = synth.README_QUERY
x = torch.empty(W * n, dtype=torch.float64, device="cuda")
y = torch.empty(W * n, dtype=torch.float64, device="cuda")
for w in range(W):
    ctx.synth_uniform_async(x[w * n:(w + 1) * n], y[w * n:(w + 1) * n], 0, 2 + 7919 * w, bj)
torch.cuda.synchronize()
grid = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / 100, 100)
names = ["start", "loop_end", "flush_end", "compacted", "list_written", "ticket"]
cols = [0, 1, 2, 7, 3, 4]
fin = ["acquired", "heads", "T", "gathered", "written", "hist_landed", "dry_start", "dry_end"]
for shape in shapes:
    _abi.debug_set_knn_config(*shape)
    out = {}
    for rep in range(3):
        ctx.debug_knn_scan_variant(0, grid, x, y, n, W, q[0], q[1], 0.5, 50, reps=8)
        ctx.debug_knn_scan_variant(6, grid, x, y, n, W, q[0], q[1], 0.5, 50, reps=1)
        tr = ctx.debug_knn_trace().astype(np.int64)
        nb = tr.shape[0] - 1
        blk = tr[:nb][:, cols]
        t0 = blk[:, 0].min()
        rel = (blk - t0) / 100.0  # us
        row = {}
        for j, nm in enumerate(names):
            v = rel[:, j]
            row[nm] = [round(float(np.percentile(v, p)), 2) for p in (0, 10, 50, 90, 100)]
        f = (tr[nb, :8] - t0) / 100.0
        row["final"] = {nm: round(float(v), 2) for nm, v in zip(fin, f)}
        out[f"rep{rep}"] = row
    print("shape", shape, "nblocks", nb)
    print(json.dumps(out, indent=1))
_abi.debug_set_knn_config()

# per-XCC / per-CU view of the stream phase for the default shape
_abi.debug_set_knn_config(*shapes[0])
ctx.debug_knn_scan_variant(0, grid, x, y, n, W, q[0], q[1], 0.5, 50, reps=8)
ctx.debug_knn_scan_variant(6, grid, x, y, n, W, q[0], q[1], 0.5, 50, reps=1)
tr = ctx.debug_knn_trace().astype(np.int64)
nb = tr.shape[0] - 1
t0 = tr[:nb, 0].min()
le = (tr[:nb, 1] - t0) / 100.0
hw = tr[:nb, 5]
xcc = tr[:nb, 6] & 0xF
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
print("loop_end by xcc:", {int(v): [round(float(le[xcc == v].mean()), 2), round(float(le[xcc == v].max()), 2), int((xcc == v).sum())] for v in np.unique(xcc)})
print("block%8 == xcc fraction:", float(np.mean((np.arange(nb) % 8) == xcc)))
cid = ((xcc * 8 + se) * 2 + sh) * 16 + cu
u, inv = np.unique(cid, return_inverse=True)
per_cu_max = np.array([le[inv == i].max() for i in range(len(u))])
per_cu_min = np.array([le[inv == i].min() for i in range(len(u))])
cnt = np.bincount(inv)
print("CUs used", len(u), "blocks per CU", np.bincount(cnt).tolist())
print("per-CU last loop_end pct (0,10,50,90,100):", [round(float(np.percentile(per_cu_max, p)), 2) for p in (0, 10, 50, 90, 100)])
print("per-CU first loop_end pct:", [round(float(np.percentile(per_cu_min, p)), 2) for p in (0, 10, 50, 90, 100)])
print("loop_end vs block id (deciles of id):", [round(float(le[i * nb // 10:(i + 1) * nb // 10].mean()), 2) for i in range(10)])
_abi.debug_set_knn_config()
