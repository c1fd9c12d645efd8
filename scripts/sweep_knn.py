"""kNN scan launch-shape sweep (measurement only): for each (waves/block, load pipeline depth,
ticket groups) check the C2 result bit-exactly against the C oracle, then time the ablation
modes (1 loads only, 7 no block tail, 8 block lists, 9 lists + separate final, 0 fused)
interleaved over rounds on a 4-window ring (no Infinity-Cache reuse)."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import cref  # noqa: E402  (checker only)
from spatialflink_amd import Context, _abi, synth  # noqa: E402

n = 10_000_000
W = 4
K = 50
shapes = [tuple(int(v) for v in s.split(",")) for s in sys.argv[1:]] or [
    (4, 1, 32, 1), (4, 1, 32, 0), (16, 1, 16, 1), (16, 1, 16, 0)]
ctx = Context(0)
bj = synth.BEIJING
q = synth.README_QUERY
x = torch.empty(W * n, dtype=torch.float64, device="cuda")
y = torch.empty(W * n, dtype=torch.float64, device="cuda")
for w in range(W):
    ctx.synth_uniform_async(x[w * n:(w + 1) * n], y[w * n:(w + 1) * n], 0, 2 + 7919 * w, bj)
torch.cuda.synchronize()
l = (bj[1] - bj[0]) / 100
grid = _abi.make_grid(bj[0], bj[2], l, 100)
want_i, want_d = cref.knn_pp(cref.grid(bj[0], bj[2], l, 100), x[:n].cpu().numpy(), y[:n].cpu().numpy(),
                             q[0], q[1], 0.5, K)
res = {}
for shape in shapes:
    _abi.debug_set_knn_config(*shape)
    ok = True
    for fused in (True, False):
        _abi.debug_set_knn_fused(fused)
        for rep in range(2):
            gi, gd = ctx.knn_pp(grid, x[:n], y[:n], q[0], q[1], 0.5, K)
            ok = ok and gi.cpu().numpy().astype(np.uint32).tolist() == want_i.tolist() and np.array_equal(
                gd.cpu().numpy().view(np.uint64), want_d.view(np.uint64))
    _abi.debug_set_knn_fused(True)
    modes = (1, 7, 8, 10, 11, 0, 9)
    t = {m: [] for m in modes}
    for rnd in range(5):
        for m in modes:
            t[m].append(ctx.debug_knn_scan_variant(m, grid, x, y, n, W, q[0], q[1], 0.5, K, reps=20) * 1e3)
    key = "_".join(str(v) for v in shape)
    res[key] = {"parity": ok, **{f"mode{m}_us": round(sorted(v)[len(v) // 2], 2) for m, v in t.items()}}
    res[key]["mode0_GBps"] = round(16 * n / (res[key]["mode0_us"] * 1e-6) / 1e9, 1)
    print(key, json.dumps(res[key]), flush=True)
_abi.debug_set_knn_config()
print(json.dumps(res))
