"""GPU: the look-back waits end with an error instead of hanging when a block count never arrives.

range_fused and the kNN pass's fused range take block offsets from a decoupled look-back over
the earlier blocks' published counts (pp_kernels.hip, poll_block_counts).  A debug knob makes
those waits expect an epoch no block publishes, so every block past the first gives up after a
bounded number of polls; the call must then report GEOHIP_ERR_DEVICE (and a later call on the same
ctx, knob off, must be correct again: the ticket is re-armed, the fault word cleared).
"""
import numpy as np
import pytest

import cref
from spatialflink_amd import _abi, synth

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING
Q = synth.README_QUERY


def test_lookback_fault_returns_error(ctx):
    import torch
    n = 2_000_000  # several blocks, so blocks wait on earlier ones
    l = (BJ[1] - BJ[0]) / 100
    g = _abi.make_grid(BJ[0], BJ[2], l, 100)
    cg = cref.grid(BJ[0], BJ[2], l, 100)
    hx, hy = synth.uniform(n, 31)
    x = torch.from_numpy(hx).cuda()
    y = torch.from_numpy(hy).cuda()
    ctx.debug_lookback_inject(True)
    try:
        with pytest.raises(_abi.GeohipDeviceError, match="look-back"):
            ctx.range_pp(g, x, y, Q[0], Q[1], 0.5)
        with pytest.raises(_abi.GeohipDeviceError, match="look-back"):
            ctx.knn_range_pp(g, x, y, Q[0], Q[1], 0.5, 50)
        # the async form: the fault surfaces at the next ctx.sync()
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        ctx.range_pp_async(g, x, y, Q[0], Q[1], 0.5, False, out, n, cnt)
        with pytest.raises(_abi.GeohipDeviceError, match="look-back"):
            ctx.sync()
    finally:
        ctx.debug_lookback_inject(False)
    ctx.sync()  # nothing pending, no fault left over
    got = ctx.range_pp(g, x, y, Q[0], Q[1], 0.5)
    want = np.sort(cref.range_pp(cg, hx, hy, Q[0], Q[1], 0.5))
    assert np.array_equal(got.cpu().numpy().astype(np.int64), want.astype(np.int64))
    (ki, kd), ro = ctx.knn_range_pp(g, x, y, Q[0], Q[1], 0.5, 50)
    wi, wd = cref.knn_pp(cg, hx, hy, Q[0], Q[1], 0.5, 50)
    assert ki.cpu().numpy().astype(np.uint32).tolist() == wi.astype(np.uint32).tolist()
    assert np.array_equal(kd.cpu().numpy().view(np.uint64), wd.view(np.uint64))
    assert len(ro) == len(want)
