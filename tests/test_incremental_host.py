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

    def range_pp(self, grid, x, y, qx, qy, r, approximate=False):
        return np.sort(cref.range_pp(self.cg, x, y, qx, qy, r, approximate)).astype(np.uint32)


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
        got = inc.push(x, y)
        win = panes[max(0, j - p + 1):j + 1]
        wx = np.concatenate([w[0] for w in win])
        wy = np.concatenate([w[1] for w in win])
        assert got.tolist() == np.sort(cref.range_pp(cg, wx, wy, Q[0], Q[1], 0.5)).tolist()
