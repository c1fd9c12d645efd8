"""Measurement: C4 point-polygon range, exact vs approximate (bbox distance, no ring work) and
the join form, timed with the ctx's HIP events (the ppoly_eval + emit region)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

from spatialflink_amd import _abi, synth  # noqa: E402

ctx = _abi.Context(0)
bj = synth.BEIJING
g = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / 500, 500)
n = 50_000_000
x = torch.empty(n, dtype=torch.float64, device="cuda")
y = torch.empty(n, dtype=torch.float64, device="cuda")
ctx.synth_uniform_async(x, y, 0, 5, bj)
off, vx, vy = synth.star_polygons(1000, 6)
torch.cuda.synchronize()
for name, approx in (("exact", False), ("approx", True)):
    out = None
    for rep in range(2):
        res = ctx.range_ppoly(g, x, y, off, vx, vy, 0.005, approx)
    ctx.timing(reset=True)
    ctx.set_timing(True)
    for rep in range(5):
        res = ctx.range_ppoly(g, x, y, off, vx, vy, 0.005, approx)
    ctx.set_timing(False)
    ms, launches = ctx.timing(reset=True)
    print(f"{name}: {ms / launches * 1e3:.1f} us per call, {len(res)} pairs", flush=True)
