"""C3 join: where the write pass's time goes (GPU box, measurement only).  Times, per window, the
whole async step (join_fused writing the pairs) against the count-only step (the same kernels with
join_fused's decisions but no emission), both through the ctx's kernel stamps, so the difference is
the emission's cost.  Run as: python scripts/join_phases.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from spatialflink_amd import Context, _abi, synth  # noqa: E402

bj = synth.BEIJING
ctx = Context(0)
g = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / 500, 500)
hx, hy = synth.gaussian_clusters(10_000_000, 3, sigma=0.1)
hqx, hqy = synth.gaussian_clusters(10_000, 4, sigma=0.1)
dx, dy, qx, qy = (torch.from_numpy(a).cuda() for a in (hx, hy, hqx, hqy))
m = ctx.join_pp_count(g, g, dx, dy, qx, qy, 0.05)
out = torch.empty((m + 8, 2), dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")


def timed(fn, reps=10):
    fn()
    ctx.sync()
    ctx.set_timing(True)
    for _ in range(reps):
        fn()
    ctx.sync()
    sm, sn, km, kn = ctx.timing_kernels(reset=True)
    ctx.set_timing(False)
    return sm / sn * 1e3, km / sn * 1e3


w_step, w_k = timed(lambda: ctx.join_pp_async(g, g, dx, dy, qx, qy, 0.05, False, out, cnt))
c_step, c_k = timed(lambda: ctx.join_pp_count(g, g, dx, dy, qx, qy, 0.05))
print(f"pairs {m}: write step {w_step:.1f} us (kernels {w_k:.1f}); count-only step {c_step:.1f} us (kernels {c_k:.1f}); "
      f"emission ~{w_k - c_k:.1f} us = {m * 8 / max(w_k - c_k, 1e-9) / 1e6:.2f} TB/s of pair bytes", flush=True)
