"""The tile-binned point-polygon path (csrc/cell_kernels.hip: bin_tiles, ppoly_words, ppoly_eval,
ppoly_emit, ppoly_outside) against the C oracle.

The streaming path (ppoly_stream + the candidate kernels) needs a cell table over the key space;
the tile-binned path runs instead whenever that table cannot be built:
  * grids of more than 2^24 cells (n > 4096 cells per side),
  * more than 16384 polygons (per-polygon candidate counters in LDS),
  * more than 2^28 polygon entries over the cells.
Each case below is reached the way a caller reaches it, plus the C4 shape with the streaming
path disabled (GEOHIP_PPOLY_TILES=1, read once per process: a child process).  Range, range
approximate and join (PointPolygonRangeQuery.java:76-124, PointPolygonJoinQuery.java:162-201),
with holes, polygons whose cells leave the grid, out-of-grid and NaN points, boundary points.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import cref
from helpers import edge_polygons, edge_window, pairs_sorted
from spatialflink_amd import _abi, synth

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING
ROOT = Path(__file__).resolve().parents[1]


def agrid(n):
    l = (BJ[1] - BJ[0]) / n
    return _abi.make_grid(BJ[0], BJ[2], l, n), cref.grid(BJ[0], BJ[2], l, n)


@pytest.mark.parametrize("r,approx", [(0.005, False), (0.005, True), (0.0012, False)])
def test_tiles_big_grid_range(ctx, r, approx):
    """5000 x 5000 cells (2.5e7 > 2^24): r = 0.005 has guaranteed cells (Lg = 7), r = 0.0012
    does not (Lg = -1, Lc = 3)."""
    off, vx, vy = edge_polygons(150, 301, 0.002, 0.006)
    x, y = edge_window(300_000, 302, off, vx, vy)
    ag, cg = agrid(5000)
    got = ctx.range_ppoly(ag, x, y, off, vx, vy, r, approx)
    want = cref.range_ppoly(cg, x, y, off, vx, vy, r, approx)
    assert len(want) > 1000
    assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()


def test_tiles_big_grid_join_and_holes(ctx):
    """The join form on the 5000 x 5000 grid, and polygons with holes on it."""
    off, vx, vy = edge_polygons(120, 311, 0.002, 0.006)
    x, y = edge_window(250_000, 312, off, vx, vy)
    ag, cg = agrid(5000)
    got = ctx.join_ppoly(ag, ag, x, y, off, vx, vy, 0.004)
    want = cref.join_ppoly(cg, cg, x, y, off, vx, vy, 0.004)
    assert len(want) > 1000
    assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
    pr, hoff, hvx, hvy, _ = synth.holed_polygons(60, 313, r_min=0.003, r_max=0.008)
    hx, hy = edge_window(200_000, 314, hoff, hvx, hvy)
    got = ctx.range_ppoly(ag, hx, hy, hoff, hvx, hvy, 0.002, poly_rings=pr)
    want = cref.range_ppoly(cg, hx, hy, hoff, hvx, hvy, 0.002, poly_rings=pr)
    assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()


def test_tiles_many_polygons(ctx):
    """17000 polygons (> 16384) on the 500 x 500 grid."""
    off, vx, vy = synth.star_polygons(17000, 321, n_vert=12, r_min=0.001, r_max=0.004)
    x, y = edge_window(400_000, 322, off, vx, vy)
    ag, cg = agrid(500)
    got = ctx.range_ppoly(ag, x, y, off, vx, vy, 0.003)
    want = cref.range_ppoly(cg, x, y, off, vx, vy, 0.003)
    assert len(want) > 10000
    assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
    got = ctx.join_ppoly(ag, ag, x, y, off, vx, vy, 0.003)
    want = cref.join_ppoly(cg, cg, x, y, off, vx, vy, 0.003)
    assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()


_CHILD = r"""
import json, sys
import numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[1] + '/tests']
from spatialflink_amd import Context, _abi, synth
from helpers import edge_polygons, edge_window
BJ = synth.BEIJING
ctx = Context(0)
l = (BJ[1] - BJ[0]) / 500
g = _abi.make_grid(BJ[0], BJ[2], l, 500)
off, vx, vy = edge_polygons(300, 331, 0.005, 0.02)
x, y = edge_window(500_000, 332, off, vx, vy)
for name, fn in (("range", lambda: ctx.range_ppoly(g, x, y, off, vx, vy, 0.005)),
                 ("approx", lambda: ctx.range_ppoly(g, x, y, off, vx, vy, 0.005, True)),
                 ("join", lambda: ctx.join_ppoly(g, g, x, y, off, vx, vy, 0.005))):
    np.save(sys.argv[2] + "/" + name + ".npy", np.asarray(fn(), dtype=np.int64))
print(json.dumps({"ok": True}))
"""


def test_tiles_forced_c4_shape(tmp_path):
    """The C4 shape (500 x 500, 50-vertex stars, r = 0.005) through the tile-binned path in a
    child process with GEOHIP_PPOLY_TILES=1, against the oracle."""
    env = dict(os.environ, GEOHIP_PPOLY_TILES="1")
    r = subprocess.run([sys.executable, "-c", _CHILD, str(ROOT), str(tmp_path)], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["ok"]
    off, vx, vy = edge_polygons(300, 331, 0.005, 0.02)
    x, y = edge_window(500_000, 332, off, vx, vy)
    _, cg = agrid(500)
    want = {"range": cref.range_ppoly(cg, x, y, off, vx, vy, 0.005),
            "approx": cref.range_ppoly(cg, x, y, off, vx, vy, 0.005, True),
            "join": cref.join_ppoly(cg, cg, x, y, off, vx, vy, 0.005)}
    for name, w in want.items():
        got = np.load(tmp_path / (name + ".npy"))
        assert len(w) > 1000
        assert pairs_sorted(got).tolist() == pairs_sorted(w).tolist(), name
