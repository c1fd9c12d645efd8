"""Phase timeline of one kNN pass launch (100 MHz timestamps): per-block start, stream end,
flush (block barrier), stores drained, arrived; the last block's acquire, gather and write.
Percentiles (0, 10, 50, 90, 100) in microseconds relative to the earliest block start (GPU box
measurement)."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from spatialflink_amd import Context, _abi, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
R = float(sys.argv[3]) if len(sys.argv) > 3 else 0.5
GN = int(sys.argv[4]) if len(sys.argv) > 4 else 100
ABL = int(sys.argv[5]) if len(sys.argv) > 5 else 0
W = 4
ctx = Context(0)
bj, q = synth.BEIJING, synth.README_QUERY
grid = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / GN, GN)
xs, ys = [], []
for w in range(W):
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    ctx.synth_uniform_async(x, y, 0, 2 + 7919 * w, bj)
    xs.append(x)
    ys.append(y)
torch.cuda.synchronize()
names = ["start", "stream_end", "flush", "drained", "arrived"] + (["lookback", "emitted"] if ABL < 0 else [])
blk = {"hist": 8, "listed": 9, "heads": 10}
fin = {"acquired": 5, "loaded": 11, "T": 12, "taken": 13, "gathered": 6, "written": 7}
out = {}
for rep in range(4):
    for w in range(W):  # warm the path, cycle windows
        ctx.knn_pp(grid, xs[w], ys[w], q[0], q[1], R, K)
    tr = ctx.debug_knn_pass_trace(grid, xs[rep % W], ys[rep % W], q[0], q[1], R, K, ABL).astype(np.int64)
    t0 = tr[:, 0].min()
    rel = (tr - t0) / 100.0
    row = {nm: [round(float(np.percentile(rel[:, j], p)), 2) for p in (0, 10, 50, 90, 100)] for j, nm in enumerate(names)}
    # blocks that reached the stamp (0 = not reached: the slot-complete end stamps 8 and 10 but
    # not 9, the list path all three) -- their median and their number
    row["block_median"] = {nm: (round(float(np.median(rel[tr[:, j] != 0, j])), 2) if (tr[:, j] != 0).any() else None)
                           for nm, j in blk.items()}
    row["blocks_reached"] = {nm: int((tr[:, j] != 0).sum()) for nm, j in blk.items()}
    last = int(np.argmax(tr[:, 7]))
    row["final"] = {nm: round(float(rel[last, j]), 2) for nm, j in fin.items()}
    row["last_block"] = last
    row["stats"] = ctx.debug_knn_pass_stats()
    out[f"rep{rep}"] = row
print(json.dumps({"shape": dict(n=n, k=K, r=R, grid=GN, ablation=ABL), **out}))
