"""Attribute knn_scan time: ablation variants timed in one process, interleaved rounds
(MODE 1 loads only, 2 + classification, 3 + staging/distances, 7 no block tail, 8 block lists
only (no fused final), 9 = 8 + separate knn_final, 0 full incl. the fused final selection), plus a plain
streaming-read reference (torch sum) on the same 4-window ring."""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from spatialflink_amd import Context, _abi, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
W = 4
ctx = Context(0)
bj = synth.BEIJING
q = synth.README_QUERY
x = torch.empty(W * n, dtype=torch.float64, device="cuda")
y = torch.empty(W * n, dtype=torch.float64, device="cuda")
for w in range(W):
    ctx.synth_uniform_async(x[w * n:(w + 1) * n], y[w * n:(w + 1) * n], 0, 2 + 7919 * w, bj)
torch.cuda.synchronize()
grid = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / 100, 100)
res = {m: [] for m in (1, 2, 3, 7, 8, 9, 0)}
for rnd in range(5):
    for m in (1, 2, 3, 7, 8, 9, 0):
        res[m].append(ctx.debug_knn_scan_variant(m, grid, x, y, n, W, q[0], q[1], 0.5, 50, reps=20) * 1e3)
out = {f"mode{m}_us": sorted(v)[len(v) // 2] for m, v in res.items()}
t5, nsurv, nspill = ctx.debug_knn_scan_variant(5, grid, x, y, n, W, q[0], q[1], 0.5, 50, reps=5)
out["mode5_us"] = t5 * 1e3
out["survivors_total"] = nsurv
out["spilled_total"] = nspill
# knn_final cost: merge of P sorted lists of 64 (P = 1 and P = 1024) into k = 50
for P in (1, 1024):
    d = torch.sort(torch.rand(P, 64, dtype=torch.float64, device="cuda"), dim=1).values
    ii = torch.arange(P * 64, dtype=torch.int32, device="cuda").view(P, 64)
    oi = torch.empty(50, dtype=torch.int32, device="cuda")
    od = torch.empty(50, dtype=torch.float64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        ctx.knn_merge_async(d, ii, P, 64, 50, oi, od, cnt)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        ctx.knn_merge_async(d, ii, P, 64, 50, oi, od, cnt)
    e1.record()
    torch.cuda.synchronize()
    out[f"final_P{P}_us"] = e0.elapsed_time(e1) / 50 * 1e3
    ctx.set_stream(None)
# torch streaming read of the same bytes (sum of x and y windows), cycling windows
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
acc = torch.zeros((), dtype=torch.float64, device="cuda")
ev0.record()
for i in range(20):
    w = i % W
    acc += x[w * n:(w + 1) * n].sum() + y[w * n:(w + 1) * n].sum()
ev1.record()
torch.cuda.synchronize()
out["torch_sum_read_us"] = ev0.elapsed_time(ev1) / 20 * 1e3
for k_, v in list(out.items()):
    if k_.endswith("_us"):
        out[k_.replace("_us", "_GBps")] = 16 * n / (v * 1e-6) / 1e9
print(json.dumps(out))
