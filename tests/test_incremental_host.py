"""CPU: pane-reuse window assembly (spatialflink_amd.incremental) with the oracle standing in for
the device range call -- window results equal the oracle's full-window evaluation."""
import numpy as np
import pytest

import cref
from spatialflink_amd import _abi, synth
from spatialflink_amd.incremental import IncrementalRange, panes_per_window

BJ = synth.BEIJING
Q = synth.README_QUERY


class OracleCtx:
    """range_pp with the Context signature, evaluated by the C oracle (test double)."""

    def __init__(self, cg):
        self.cg = cg

    def range_pp(self, grid, x, y, qx, qy, r, approximate=False, point_base=0):
        hits = np.sort(cref.range_pp(self.cg, x, y, qx, qy, r, approximate)).astype(np.uint64)
        return ((hits + point_base) & 0xFFFFFFFF).astype(np.uint32)


def test_panes_per_window():
    assert panes_per_window(10, 5) == 2 and panes_per_window(15, 5) == 3 and panes_per_window(5, 5) == 1
    for bad in ((10, 3), (10, 0), (0, 5)):
        with pytest.raises(_abi.GeohipArgumentError):
            panes_per_window(*bad)


@pytest.mark.parametrize("p", [1, 2, 4])
def test_window_assembly_matches_full_evaluation(p):
    l = (BJ[1] - BJ[0]) / 100
    cg = cref.grid(BJ[0], BJ[2], l, 100)
    sizes = [3000, 0, 5000, 1234, 4000, 2500]
    panes, base = [], 0
    for s in sizes:
        panes.append(synth.uniform(s, 21, base=base))
        base += s
    inc = IncrementalRange(OracleCtx(cg), None, Q[0], Q[1], 0.5, False, p)
    for j, (x, y) in enumerate(panes):
        parts = inc.push(x, y)
        win = panes[max(0, j - p + 1):j + 1]
        wx = np.concatenate([w[0] for w in win])
        wy = np.concatenate([w[1] for w in win])
        want = np.sort(cref.range_pp(cg, wx, wy, Q[0], Q[1], 0.5))
        # pane results are stream positions: the window's first point is window_start
        got = np.concatenate([np.zeros(0, np.int64)] + [np.asarray(h, np.int64) for h in parts])
        assert (got - inc.window_start).tolist() == want.tolist()
        assert inc.window_local().tolist() == want.tolist()


def test_window_positions_wrap_mod_2_32():
    """Stream positions wrap at 2^32 (a window's local index is the difference mod 2^32)."""
    l = (BJ[1] - BJ[0]) / 100
    cg = cref.grid(BJ[0], BJ[2], l, 100)
    inc = IncrementalRange(OracleCtx(cg), None, Q[0], Q[1], 0.5, False, 2)
    inc.pos = (1 << 32) - 700
    a = synth.uniform(2000, 31)
    b = synth.uniform(2000, 31, base=2000)
    inc.push(*a)
    inc.push(*b)
    want = np.sort(cref.range_pp(cg, np.concatenate([a[0], b[0]]), np.concatenate([a[1], b[1]]), Q[0], Q[1], 0.5))
    assert inc.window_local().tolist() == want.tolist()
