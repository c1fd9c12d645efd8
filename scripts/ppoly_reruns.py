"""How often the point-polygon stream re-runs a chunk whose per-wave LDS stage overflowed (the
direct-store path): the C4 window and windows packed around polygon edges, range and join.  Run
with GEOHIP_HOST_PROFILE=1 (GPU box); the library prints one line per call with the re-run count."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from spatialflink_amd import Context, _abi, synth  # noqa: E402

bj = synth.BEIJING
ctx = Context(0)
g = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / 500, 500)
off, vx, vy = synth.star_polygons(1000, 6)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


x = torch.empty(50_000_000, dtype=torch.float64, device="cuda")
y = torch.empty_like(x)
ctx.synth_uniform_async(x, y, 0, 5, bj)
print("C4 window, range", flush=True)
ctx.range_ppoly(g, x, y, off, vx, vy, 0.005)
print("C4 window, join", flush=True)
ctx.join_ppoly(g, g, x, y, off, vx, vy, 0.005)
rng = np.random.default_rng(1)
for sd, label in ((0.0005, "within 0.0005 of the vertices"), (0.002, "within 0.002 of the vertices")):
    k = 20
    ex = np.concatenate([vx + rng.normal(0, sd, len(vx)) for _ in range(k)])
    ey = np.concatenate([vy + rng.normal(0, sd, len(vy)) for _ in range(k)])
    print(f"edge-dense window ({len(ex)} points {label}), range", flush=True)
    ctx.range_ppoly(g, dev(ex), dev(ey), off, vx, vy, 0.005)
    print("  join", flush=True)
    ctx.join_ppoly(g, g, dev(ex), dev(ey), off, vx, vy, 0.005)
dense_off, dvx, dvy = synth.star_polygons(3000, 7, r_min=0.02, r_max=0.05)
print("3000 overlapping polygons (R 0.02-0.05) over the C4 window, range", flush=True)
ctx.range_ppoly(g, x, y, dense_off, dvx, dvy, 0.005)
