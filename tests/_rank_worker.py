"""One rank of tests/test_gpu_multirank.py: world-2 gloo group, both ranks on cuda:0, the default
libgeohip engines (no injected engine), collectives staged through host by distributed.py.
Writes this rank's results to <out>/rank<r>.npz.  Not a test module (no test_ prefix)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main(out_dir):
    import numpy as np
    import torch
    import torch.distributed as dist

    from spatialflink_amd import Context, _abi, synth
    from spatialflink_amd import distributed as D

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = Context(0)
    bj = synth.BEIJING
    q = synth.README_QUERY

    def grid(n):
        return _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / n, n)

    res = {}
    # C5-shaped kNN + range, arrival shards
    n_total = 2_000_003
    x, y = synth.uniform(n_total, 21)
    lo, hi = D.shard_bounds(n_total, world, rank)
    xl, yl = torch.from_numpy(x[lo:hi].copy()).cuda(), torch.from_numpy(y[lo:hi].copy()).cuda()
    g = grid(500)
    kr = D.knn_sharded(xl, yl, lo, q[0], q[1], 0.05, 100, grid=g, ctx=ctx)
    res["knn_i"], res["knn_d"] = kr.idx.cpu().numpy(), kr.dist.cpu().numpy()
    hits, off, total = D.range_sharded(xl, yl, lo, q[0], q[1], 0.05, grid=g, ctx=ctx)
    res["range"], res["range_off"], res["range_total"] = hits.cpu().numpy(), off, total
    # C3-shaped join: arrival and key-band ("cells") partitions
    dx, dy = synth.gaussian_clusters(400_001, 3, sigma=0.1)
    qx, qy = synth.gaussian_clusters(2000, 4, sigma=0.1)
    lo, hi = D.shard_bounds(len(dx), world, rank)
    dxl, dyl = torch.from_numpy(dx[lo:hi].copy()).cuda(), torch.from_numpy(dy[lo:hi].copy()).cuda()
    tqx, tqy = torch.from_numpy(qx).cuda(), torch.from_numpy(qy).cuda()
    for part in ("arrival", "cells"):
        pairs, off, total = D.join_sharded(dxl, dyl, lo, tqx, tqy, 0.02, grid_data=g, grid_query=g, ctx=ctx,
                                           partition=part)
        res[f"join_{part}"], res[f"join_{part}_off"], res[f"join_{part}_total"] = pairs.cpu().numpy(), off, total
    # the enqueue-only key-band join (bench's cells line): preallocated rows, device counts
    cout = torch.empty((16_000_000, 2), dtype=torch.int32, device="cuda")
    ccount = torch.zeros(1, dtype=torch.int64, device="cuda")
    ccounts = torch.zeros(world, dtype=torch.int64, device="cuda")
    step = D.join_cells_enqueue(dxl, dyl, lo, tqx, tqy, 0.02, grid_data=g, grid_query=g, ctx=ctx, out=cout,
                                count=ccount, counts=ccounts)
    pairs, off, total = step.result()
    res["join_enq"], res["join_enq_off"], res["join_enq_total"] = pairs.cpu().numpy(), off, total
    # the band pack kernel against its torch restatement on this shard
    bx, by, bi, bc = ctx.band_pack_async(g, 500, world, dxl, dyl, lo)
    tx, ty, ti, tc = D.torch_band_pack(g)(dxl, dyl, lo, 500, world)
    m = int(bc.sum().item())
    res["band_ok"] = int(bc.tolist() == tc.tolist() and torch.equal(bi[:m], ti) and torch.equal(bx[:m], tx)
                         and torch.equal(by[:m], ty))
    # point-polygon range / join / kNN with holed polygons, arrival shards
    pr, roff, vx, vy, _ = synth.holed_polygons(20, 22)
    x, y = synth.uniform(600_001, 23)
    lo, hi = D.shard_bounds(len(x), world, rank)
    pxl, pyl = torch.from_numpy(x[lo:hi].copy()).cuda(), torch.from_numpy(y[lo:hi].copy()).cuda()
    pairs, off, total = D.ppoly_sharded(pxl, pyl, lo, roff, vx, vy, 0.003, grid=g, ctx=ctx, poly_rings=pr)
    res["ppoly"], res["ppoly_total"] = pairs.cpu().numpy(), total
    pairs, off, total = D.join_ppoly_sharded(pxl, pyl, lo, roff, vx, vy, 0.003, grid_points=g, grid_query=g, ctx=ctx,
                                             poly_rings=pr)
    res["jppoly"], res["jppoly_total"] = pairs.cpu().numpy(), total
    a, b = pr[0], pr[1]
    kp = D.knn_ppoly_sharded(pxl, pyl, lo, vx[roff[a]:roff[b]], vy[roff[a]:roff[b]], 0.003, 50, grid=g, ctx=ctx,
                             ring_off=roff[a:b + 1] - roff[a])
    res["kppoly_i"], res["kppoly_d"] = kp.idx.cpu().numpy(), kp.dist.cpu().numpy()
    np.savez(Path(out_dir) / f"rank{rank}.npz", **{k: np.asarray(v) for k, v in res.items()})
    dist.barrier()
    dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main(sys.argv[1])
