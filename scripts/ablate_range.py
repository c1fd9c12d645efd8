"""Fused range pass ablation (measurement only): full / counts only / loads only, C1 query shape
over 10M uniform points, 4 windows cycled, events around 50 launches per mode."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from spatialflink_amd import Context, _abi, synth  # noqa: E402

n, W = 10_000_000, 4
ctx = Context(0)
stream = torch.cuda.Stream()  # a real stream handle (the default stream's handle is 0)
torch.cuda.set_stream(stream)
ctx.set_stream(stream.cuda_stream)
bj, q = synth.BEIJING, synth.README_QUERY
xs = [torch.empty(n, dtype=torch.float64, device="cuda") for _ in range(W)]
ys = [torch.empty(n, dtype=torch.float64, device="cuda") for _ in range(W)]
for w in range(W):
    ctx.synth_uniform_async(xs[w], ys[w], 0, 1 + 7919 * w, bj)
g = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / 100, 100)
out = torch.empty(n, dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
for mode in (0, 1, 2, 3, 4, 0, 1, 2, 3, 4):
    _abi.debug_set_range_mode(mode)
    for s in range(5):
        ctx.range_pp_async(g, xs[s % W], ys[s % W], q[0], q[1], 0.5, False, out, n, cnt)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for s in range(50):
        ctx.range_pp_async(g, xs[s % W], ys[s % W], q[0], q[1], 0.5, False, out, n, cnt)
    e1.record()
    torch.cuda.synchronize()
    print(f"mode {mode}: {e0.elapsed_time(e1) / 50 * 1e3:.2f} us per launch (back to back)")
_abi.debug_set_range_mode(0)
