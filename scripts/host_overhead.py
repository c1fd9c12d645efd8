"""Host-side cost of one operator call (measurement only): tiny windows so the device work is
negligible; prints microseconds per call for ppoly (1 / 1000 polygons), join (10k queries), kNN."""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from spatialflink_amd import Context, _abi, synth  # noqa: E402

ctx = Context(0)
bj, q = synth.BEIJING, synth.README_QUERY
g5 = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / 500, 500)
x, y = synth.uniform(1000, 1)
tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
off, vx, vy = synth.star_polygons(1000, 6)
out = torch.empty((100000, 2), dtype=torch.int32, device="cuda")


def timeit(f, reps=20):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


print("ppoly 1000 polys  us", round(timeit(lambda: ctx.range_ppoly(g5, tx, ty, off, vx, vy, 0.005, out=out)), 1))
print("ppoly 1 poly      us", round(timeit(lambda: ctx.range_ppoly(g5, tx, ty, off[:2], vx[:51], vy[:51], 0.005, out=out)), 1))
qx, qy = synth.gaussian_clusters(10000, 4)
tqx, tqy = torch.from_numpy(qx).cuda(), torch.from_numpy(qy).cuda()
print("join 10k queries  us", round(timeit(lambda: ctx.join_pp(g5, g5, tx, ty, tqx, tqy, 0.05, out=out)), 1))
g1 = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / 100, 100)
oi = torch.empty(50, dtype=torch.int32, device="cuda")
od = torch.empty(50, dtype=torch.float64, device="cuda")
cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
print("knn async         us", round(timeit(lambda: ctx.knn_pp_async(g1, tx, ty, q[0], q[1], 0.5, 50, oi, od, cnt), 200), 1))
