"""The point-polygon stream on windows that overflow its per-wave LDS stages or its candidate
buffer: the C4 window, windows packed around polygon edges, and 3000 overlapping polygons over the
C4 window (range and join).  Run with GEOHIP_HOST_PROFILE=1 (GPU box); the library prints one line
per call (pairs, candidates, those past the buffer, early wave flushes, chunks decided by the
redo pass);
the dense window's device step time is printed for a first call (fresh ctx) and warm calls, and
its pair count / digest checked against the oracle (threaded C, slow: run once)."""
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
for label, join in (("range", False), ("join", True)):
    print(f"3000 overlapping polygons (R 0.02-0.05) over the C4 window, {label}", flush=True)
    c = Context(0)  # fresh: no candidate history, the first call sizes its buffer at n / 16
    cap = 340_000_000
    out = torch.empty((cap, 2), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    for rep in range(4):
        c.set_timing(True)
        cnt.zero_()
        if join:
            c.join_ppoly_async(g, g, x, y, dense_off, dvx, dvy, 0.005, False, out, cnt)
        else:
            c.range_ppoly_async(g, x, y, dense_off, dvx, dvy, 0.005, False, out, cnt)
        c.sync()
        sm, sn, km, kn = c.timing_kernels(reset=True)
        c.set_timing(False)
        print(f"  call {rep}: {int(cnt.item())} pairs, step {sm / max(sn, 1):.3f} ms, kernels {km / max(sn, 1):.3f} ms"
              + (" (first call: plan built, candidate buffer from n / 16)" if rep == 0 else ""), flush=True)
    m = int(cnt.item())
    if len(sys.argv) > 1 and sys.argv[1] == "--check":
        sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
        sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
        import cref
        from helpers import pair_digest
        cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / 500, 500)
        hx, hy = x.cpu().numpy(), y.cpu().numpy()
        want = (cref.join_ppoly_hash(cg, cg, hx, hy, dense_off, dvx, dvy, 0.005) if join
                else cref.range_ppoly_hash(cg, hx, hy, dense_off, dvx, dvy, 0.005))
        print(f"  oracle: {want[0]} pairs; digest match: {(m, pair_digest(out[:m])[1]) == want}", flush=True)
    del out
