"""Quick join smoke on the GPU box: a 2M-point Gaussian C3-shaped window vs the oracle."""
import sys, time
sys.path[:0] = ['.', 'oracle']
import numpy as np
import cref
from spatialflink_amd import Context, _abi, synth
ctx = Context(0)
BJ = synth.BEIJING
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000000
l = (BJ[1] - BJ[0]) / 500
ag = _abi.make_grid(BJ[0], BJ[2], l, 500)
cg = cref.grid(BJ[0], BJ[2], l, 500)
x, y = synth.gaussian_clusters(n, 3, sigma=0.1)
qx, qy = synth.gaussian_clusters(10000, 4, sigma=0.1)
print("start", flush=True)
t = time.time(); c = ctx.join_pp_count(ag, ag, x, y, qx, qy, 0.05); print("count", c, round(time.time() - t, 3), flush=True)
t = time.time(); p = ctx.join_pp(ag, ag, x, y, qx, qy, 0.05); print("pairs", len(p), round(time.time() - t, 3), flush=True)
w = cref.join_pp(cg, cg, x, y, qx, qy, 0.05)
a = np.sort(p.astype(np.int64)[:, 0] << 32 | p.astype(np.int64)[:, 1])
b = np.sort(w.astype(np.int64)[:, 0] << 32 | w.astype(np.int64)[:, 1])
print("match", c == len(w) and np.array_equal(a, b), flush=True)
