"""Measurement: a few C4 point-polygon range calls (exact) for rocprofv3 counter passes."""
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
for rep in range(3):
    res = ctx.range_ppoly(g, x, y, off, vx, vy, 0.005, False)
print(len(res))
