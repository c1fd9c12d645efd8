"""Three host-window C2 kNN calls (GEOHIP_MEM_HOST) for a rocprofv3 kernel + memory-copy trace:
the per-chunk knn_pass launches interleave with the H2D copies of later chunks."""
import sys

sys.path.insert(0, ".")
import numpy as np  # noqa: E402

from spatialflink_amd import Context, _abi, synth  # noqa: E402

bj, q = synth.BEIJING, synth.README_QUERY
g = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / 100, 100)
x, y = synth.uniform(10_000_000, 2)
ctx = Context(0)
for _ in range(3):
    i, d = ctx.knn_pp(g, x, y, q[0], q[1], 0.5, 50)
print("ok", len(i), flush=True)
