"""C3 join: per-block timeline of join_fused (measurement build with GEOHIP_JOIN_TRACE, which writes
each block's start, end, item count and last item start into the output's last 8192 slots).  Shows
how much of the pass is the tail after the first blocks run out of items.
    scripts/build_variant.sh jtrace cell_kernels.hip -DGEOHIP_JOIN_TRACE      (here)
    GEOHIP_LIB=spatialflink_amd/libgeohip_jtrace.so python scripts/join_tail.py   (GPU box)"""
import sys
from pathlib import Path

import numpy as np
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
out = torch.empty((m + 4 * 2048 + 64, 2), dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
for rep in range(4):
    cnt.zero_()
    ctx.join_pp_async(g, g, dx, dy, qx, qy, 0.05, False, out, cnt)
    ctx.sync()
    assert int(cnt.item()) == m
    tr = out[-4 * 2048:].contiguous().view(torch.int64).cpu().numpy()
    nb = 1280
    st, en, ni, la = tr[:nb], tr[2048:2048 + nb], tr[4096:4096 + nb], tr[6144:6144 + nb]
    t0 = st.min()
    to_us = lambda v: (v - t0) / 100.0  # s_memrealtime: 100 MHz
    e = np.sort(to_us(en))
    q = lambda a: " ".join(f"{np.quantile(a, p):7.1f}" for p in (0, 0.1, 0.5, 0.9, 0.99, 1))
    print(f"rep {rep}: pairs {m}; block start [{q(to_us(st))}] us")
    print(f"   block end   q0/10/50/90/99/100 [{q(e)}] us")
    print(f"   items/block [{q(ni.astype(float))}]; last item start [{q(to_us(la))}]")
    print(f"   longest last item: {np.max(to_us(en) - to_us(la)):.1f} us; mean active blocks after the 10% end: "
          f"{np.mean(e > np.quantile(e, 0.1)):.2f}", flush=True)
