"""CPU, world_size 2 (gloo): the sharded window path of spatialflink_amd.distributed.

The collective orchestration (arrival-order shards, global index offsets, all-gather of
per-rank top-k, merge, range offsets) is exercised with the gloo backend; the per-rank
engine is the C oracle (test infrastructure standing in for the device kernels, which
tests/test_gpu_parity.py::test_knn_async_and_merge covers on the GPU).  Results must equal
the unsharded oracle on the whole window.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sentinel_d(k):
    return torch.full((k,), -1, dtype=torch.int64).view(torch.float64)


def _worker(rank, world, port, out_path):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cref
    from spatialflink_amd import distributed as D
    from spatialflink_amd import synth

    bj = synth.BEIJING
    q = synth.README_QUERY
    cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / 100, 100)
    n_total = 200_003
    x, y = synth.uniform(n_total, 2)
    lo, hi = D.shard_bounds(n_total, world, rank)
    xl, yl = torch.from_numpy(x[lo:hi].copy()), torch.from_numpy(y[lo:hi].copy())

    def local_knn(xs, ys, qx, qy, r, k):
        oi, od = cref.knn_pp(cg, xs.numpy(), ys.numpy(), qx, qy, r, k)
        ti = torch.full((k,), -1, dtype=torch.int32)
        td = _sentinel_d(k)
        ti[:len(oi)] = torch.from_numpy(oi.astype(np.int64)).to(torch.int32)
        td[:len(od)] = torch.from_numpy(od)
        return ti, td

    def merge(all_d, all_i, k):
        d = all_d.reshape(-1).view(torch.int64).numpy().astype(np.uint64)
        i = all_i.reshape(-1).numpy().astype(np.int64) & 0xFFFFFFFF
        keep = i != 0xFFFFFFFF
        o = np.lexsort((i[keep], d[keep]))[:k]
        ti = torch.full((k,), -1, dtype=torch.int32)
        td = _sentinel_d(k)
        ti[:len(o)] = torch.from_numpy(i[keep][o].astype(np.int32))
        td[:len(o)] = torch.from_numpy(d[keep][o].view(np.float64))
        return ti, td

    res = D.knn_sharded(xl, yl, lo, q[0], q[1], 0.5, 50, local_knn=local_knn, merge=merge)

    def local_range(xs, ys, qx, qy, r, approximate):
        return torch.from_numpy(cref.range_pp(cg, xs.numpy(), ys.numpy(), qx, qy, r, approximate).astype(np.int64))

    hits, off, total = D.range_sharded(xl, yl, lo, q[0], q[1], 0.5, local_range=local_range)
    gathered = [None] * world
    dist.all_gather_object(gathered, (off, total, hits.numpy().tolist()))
    if rank == 0:
        np.savez(out_path, knn_i=res.idx.numpy(), knn_d=res.dist.numpy(),
                 range_hits=np.array(sum((g[2] for g in sorted(gathered)), []), dtype=np.int64),
                 offsets=np.array([g[0] for g in gathered]), totals=np.array([g[1] for g in gathered]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_knn_and_range_gloo(tmp_path, world):
    out = tmp_path / "res.npz"
    mp.spawn(_worker, args=(world, _free_port(), str(out)), nprocs=world, join=True)
    r = np.load(out)
    sys.path.insert(0, str(ROOT / "oracle"))
    import cref
    from spatialflink_amd import synth

    bj = synth.BEIJING
    q = synth.README_QUERY
    cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / 100, 100)
    x, y = synth.uniform(200_003, 2)
    wi, wd = cref.knn_pp(cg, x, y, q[0], q[1], 0.5, 50)
    assert r["knn_i"].astype(np.int64).tolist() == wi.astype(np.int64).tolist()
    assert np.array_equal(r["knn_d"].view(np.uint64), wd.view(np.uint64))
    want = cref.range_pp(cg, x, y, q[0], q[1], 0.5)
    assert r["range_hits"].tolist() == sorted(want.tolist())
    assert r["totals"].tolist() == [len(want)] * world
    assert r["offsets"][0] == 0


def _join_worker(rank, world, port, out_path):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cref
    from spatialflink_amd import distributed as D
    from spatialflink_amd import synth

    bj = synth.BEIJING
    out = {}
    for gn, r in ((100, 0.05), (37, 0.0), (500, 0.02)):
        cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / gn, gn)
        n_total = 40_001
        dx, dy = synth.gaussian_clusters(n_total, 3, sigma=0.1)
        dx[::997] = np.nan  # NaN data land in cell 0 (Java (int)NaN)
        qx, qy = synth.gaussian_clusters(257, 4, sigma=0.1)
        lo, hi = D.shard_bounds(n_total, world, rank)
        xl, yl = torch.from_numpy(dx[lo:hi].copy()), torch.from_numpy(dy[lo:hi].copy())
        tqx, tqy = torch.from_numpy(qx), torch.from_numpy(qy)

        def local_join(xs, ys, qxs, qys, rr, approximate):
            p = cref.join_pp(cg, cg, xs.numpy(), ys.numpy(), qxs.numpy(), qys.numpy(), rr, approximate)
            return torch.from_numpy(p.astype(np.int64)).reshape(-1, 2)

        for part in ("arrival", "cells"):
            pairs, off, total = D.join_sharded(xl, yl, lo, tqx, tqy, r, grid_data=cg, grid_query=cg,
                                               partition=part, local_join=local_join,
                                               band_pack=D.torch_band_pack(cg))
            got = [None] * world
            dist.all_gather_object(got, (rank, pairs.numpy().tolist(), off, total))
            out[f"{gn}_{r}_{part}"] = got
    # point-polygon range, polygons replicated
    cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / 200, 200)
    n_total = 60_001
    x, y = synth.uniform(n_total, 9)
    off_, vx, vy = synth.star_polygons(12, 10)
    lo, hi = D.shard_bounds(n_total, world, rank)

    def local_ppoly(xs, ys, ro, pvx, pvy, rr, approximate):
        p = cref.range_ppoly(cg, xs.numpy(), ys.numpy(), ro, pvx, pvy, rr, approximate)
        return torch.from_numpy(p.astype(np.int64)).reshape(-1, 2)

    pairs, off, total = D.ppoly_sharded(torch.from_numpy(x[lo:hi].copy()), torch.from_numpy(y[lo:hi].copy()), lo,
                                        off_, vx, vy, 0.01, local_ppoly=local_ppoly)
    got = [None] * world
    dist.all_gather_object(got, (rank, pairs.numpy().tolist(), off, total))
    out["ppoly"] = got
    if rank == 0:
        import json
        with open(out_path, "w") as f:
            json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


def _union(got):
    pairs = [tuple(p) for _, ps, _, _ in sorted(got) for p in ps]
    offs = [o for _, _, o, _ in sorted(got)]
    sizes = [len(ps) for _, ps, _, _ in sorted(got)]
    tot = {t for _, _, _, t in got}
    return pairs, offs, sizes, tot


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_join_and_ppoly_gloo(tmp_path, world):
    """join_sharded (arrival shards and key-band partition with an all-to-all and halo query
    replication) and ppoly_sharded: disjoint per-rank pair sets whose union equals the
    unsharded oracle, consistent offsets/totals."""
    import json

    out = tmp_path / "join.json"
    mp.spawn(_join_worker, args=(world, _free_port(), str(out)), nprocs=world, join=True)
    with open(out) as f:
        res = json.load(f)
    sys.path.insert(0, str(ROOT / "oracle"))
    import cref
    from spatialflink_amd import synth

    bj = synth.BEIJING
    for gn, r in ((100, 0.05), (37, 0.0), (500, 0.02)):
        cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / gn, gn)
        dx, dy = synth.gaussian_clusters(40_001, 3, sigma=0.1)
        dx[::997] = np.nan
        qx, qy = synth.gaussian_clusters(257, 4, sigma=0.1)
        want = sorted(map(tuple, cref.join_pp(cg, cg, dx, dy, qx, qy, r).astype(np.int64).tolist()))
        for part in ("arrival", "cells"):
            pairs, offs, sizes, tot = _union(res[f"{gn}_{r}_{part}"])
            assert len(pairs) == len(set(pairs)), (gn, r, part, "ranks overlap")
            assert sorted(pairs) == want, (gn, r, part)
            assert tot == {len(want)} and offs == [sum(sizes[:i]) for i in range(world)]
    cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / 200, 200)
    x, y = synth.uniform(60_001, 9)
    off_, vx, vy = synth.star_polygons(12, 10)
    want = sorted(map(tuple, cref.range_ppoly(cg, x, y, off_, vx, vy, 0.01).astype(np.int64).tolist()))
    pairs, offs, sizes, tot = _union(res["ppoly"])
    assert sorted(pairs) == want and tot == {len(want)}


def _ppx_worker(rank, world, port, out_path):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cref
    from spatialflink_amd import distributed as D
    from spatialflink_amd import synth

    bj = synth.BEIJING
    cu = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / 200, 200)
    cq = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / 500, 500)
    n_total = 80_001
    x, y = synth.uniform(n_total, 31)
    off_, vx, vy = synth.star_polygons(10, 32)
    lo, hi = D.shard_bounds(n_total, world, rank)
    xl, yl = torch.from_numpy(x[lo:hi].copy()), torch.from_numpy(y[lo:hi].copy())

    def local_join(xs, ys, ro, pvx, pvy, rr, approximate):
        p = cref.join_ppoly(cu, cq, xs.numpy(), ys.numpy(), ro, pvx, pvy, rr, approximate)
        return torch.from_numpy(p.astype(np.int64)).reshape(-1, 2)

    pairs, off, total = D.join_ppoly_sharded(xl, yl, lo, off_, vx, vy, 0.02, local_join=local_join)
    got = [None] * world
    dist.all_gather_object(got, (rank, pairs.numpy().tolist(), off, total))

    def local_knn(xs, ys, pvx, pvy, rr, k, approximate):
        oi, od = cref.knn_ppoly(cu, xs.numpy(), ys.numpy(), pvx, pvy, rr, k, approximate)
        ti = torch.full((k,), -1, dtype=torch.int32)
        td = _sentinel_d(k)
        ti[:len(oi)] = torch.from_numpy(oi.astype(np.int64)).to(torch.int32)
        td[:len(od)] = torch.from_numpy(od)
        return ti, td

    def merge(all_d, all_i, k):
        d = all_d.reshape(-1).view(torch.int64).numpy().astype(np.uint64)
        i = all_i.reshape(-1).numpy().astype(np.int64) & 0xFFFFFFFF
        keep = i != 0xFFFFFFFF
        o = np.lexsort((i[keep], d[keep]))[:k]
        ti = torch.full((k,), -1, dtype=torch.int32)
        td = _sentinel_d(k)
        ti[:len(o)] = torch.from_numpy(i[keep][o].astype(np.int32))
        td[:len(o)] = torch.from_numpy(d[keep][o].view(np.float64))
        return ti, td

    p0 = slice(off_[0], off_[1])
    res = D.knn_ppoly_sharded(xl, yl, lo, vx[p0], vy[p0], 0.05, 40, local_knn=local_knn, merge=merge)
    if rank == 0:
        import json
        with open(out_path, "w") as f:
            json.dump({"join": got, "knn_i": res.idx.numpy().tolist(),
                       "knn_d": res.dist.numpy().view(np.uint64).astype(str).tolist()}, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_ppoly_join_and_knn_gloo(tmp_path, world):
    """join_ppoly_sharded (two grids; pairs (point, polygon)) and knn_ppoly_sharded over arrival
    shards equal the unsharded oracle."""
    import json

    out = tmp_path / "ppx.json"
    mp.spawn(_ppx_worker, args=(world, _free_port(), str(out)), nprocs=world, join=True)
    with open(out) as f:
        res = json.load(f)
    sys.path.insert(0, str(ROOT / "oracle"))
    import cref
    from spatialflink_amd import synth

    bj = synth.BEIJING
    cu = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / 200, 200)
    cq = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / 500, 500)
    x, y = synth.uniform(80_001, 31)
    off_, vx, vy = synth.star_polygons(10, 32)
    want = sorted(map(tuple, cref.join_ppoly(cu, cq, x, y, off_, vx, vy, 0.02).astype(np.int64).tolist()))
    pairs, offs, sizes, tot = _union(res["join"])
    assert sorted(pairs) == want and len(pairs) == len(set(pairs)) and tot == {len(want)}
    assert offs == [sum(sizes[:i]) for i in range(world)]
    p0 = slice(off_[0], off_[1])
    wi, wd = cref.knn_ppoly(cu, x, y, vx[p0], vy[p0], 0.05, 40)
    assert res["knn_i"] == wi.astype(np.int64).tolist()
    assert [int(v) for v in res["knn_d"]] == wd.view(np.uint64).astype(np.int64).tolist() or \
        np.array_equal(np.array([int(v) for v in res["knn_d"]], dtype=np.uint64), wd.view(np.uint64))


def _cells_worker(rank, world, port, out_path):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cref
    from spatialflink_amd import _abi
    from spatialflink_amd import distributed as D
    from spatialflink_amd import synth

    bj = synth.BEIJING
    q = synth.README_QUERY
    out = {}
    for n_grid, r, k in ((100, 0.5, 50), (1000, 0.05, 100)):
        l = (bj[1] - bj[0]) / n_grid
        cg = cref.grid(bj[0], bj[2], l, n_grid)
        ag = _abi.make_grid(bj[0], bj[2], l, n_grid)
        n_total = 300_007
        x, y = synth.uniform(n_total, 5 + n_grid)
        x[:50] = q[0] + 1e-4 * np.arange(50)  # a dense clump at the query: one band owns it
        y[:50] = q[1]
        lo, hi = D.shard_bounds(n_total, world, rank)
        xl, yl = torch.from_numpy(x[lo:hi].copy()), torch.from_numpy(y[lo:hi].copy())

        def local(xs, ys, qx, qy, rr, kk, approximate):
            oi, od = cref.knn_pp(cg, xs.numpy(), ys.numpy(), qx, qy, rr, kk)
            ti = torch.full((kk,), -1, dtype=torch.int32)
            td = _sentinel_d(kk)
            ti[:len(oi)] = torch.from_numpy(oi.astype(np.int64)).to(torch.int32)
            td[:len(od)] = torch.from_numpy(od)
            hits = np.sort(cref.range_pp(cg, xs.numpy(), ys.numpy(), qx, qy, rr, approximate)).astype(np.int64)
            return ti, td, torch.from_numpy(hits)

        def merge(all_d, all_i, kk):
            d = all_d.reshape(-1).view(torch.int64).numpy().astype(np.uint64)
            i = all_i.reshape(-1).numpy().astype(np.int64) & 0xFFFFFFFF
            keep = i != 0xFFFFFFFF
            o = np.lexsort((i[keep], d[keep]))[:kk]
            ti = torch.full((kk,), -1, dtype=torch.int32)
            td = _sentinel_d(kk)
            ti[:len(o)] = torch.from_numpy(i[keep][o].astype(np.int32))
            td[:len(o)] = torch.from_numpy(d[keep][o].view(np.float64))
            return ti, td

        res, (hits, off, total), nrecv = D.knn_range_cells(
            xl, yl, lo, q[0], q[1], r, k, grid=ag, band_pack=D.torch_band_pack_query(ag, q[0], q[1], r),
            local=local, merge=merge)
        gathered = [None] * world
        dist.all_gather_object(gathered, (off, total, hits.numpy().tolist(), nrecv))
        out[f"knn_i_{n_grid}"] = res.idx.numpy()
        out[f"knn_d_{n_grid}"] = res.dist.numpy()
        out[f"hits_{n_grid}"] = np.array(sorted(sum((g[2] for g in gathered), [])), dtype=np.int64)
        out[f"totals_{n_grid}"] = np.array([g[1] for g in gathered])
        out[f"recv_{n_grid}"] = np.array([g[3] for g in gathered])
    if rank == 0:
        np.savez(out_path, **out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 4])
def test_knn_range_key_band_partition_gloo(tmp_path, world):
    """The north-star layout for point queries (filter to G u C, keyBy(gridID) as key bands,
    PointPointKNNQuery.java:137-151): the merged kNN and the union of the owners' range hits equal
    the unsharded oracle; every rank received only its band's candidates."""
    out = tmp_path / "cells.npz"
    mp.spawn(_cells_worker, args=(world, _free_port(), str(out)), nprocs=world, join=True)
    r = np.load(out)
    sys.path.insert(0, str(ROOT / "oracle"))
    import cref
    from spatialflink_amd import synth

    bj = synth.BEIJING
    q = synth.README_QUERY
    for n_grid, rad, k in ((100, 0.5, 50), (1000, 0.05, 100)):
        l = (bj[1] - bj[0]) / n_grid
        cg = cref.grid(bj[0], bj[2], l, n_grid)
        x, y = synth.uniform(300_007, 5 + n_grid)
        x[:50] = q[0] + 1e-4 * np.arange(50)
        y[:50] = q[1]
        wi, wd = cref.knn_pp(cg, x, y, q[0], q[1], rad, k)
        assert r[f"knn_i_{n_grid}"].astype(np.uint32).tolist() == wi.tolist()
        assert np.array_equal(r[f"knn_d_{n_grid}"].view(np.uint64), wd.view(np.uint64))
        want = np.sort(cref.range_pp(cg, x, y, q[0], q[1], rad)).astype(np.int64)
        assert r[f"hits_{n_grid}"].tolist() == want.tolist()
        assert (r[f"totals_{n_grid}"] == len(want)).all()
        # only G u C points moved; their total is the candidate count
        recv = r[f"recv_{n_grid}"]
        assert recv.sum() < len(x) * 0.3
        # block-cyclic columns spread the one query's G u C box over the ranks (contiguous bands
        # gave one rank all of it: skew = world); the 50-point clump sits in one column
        if world > 1:
            assert recv.max() / recv.mean() <= 1.5, recv.tolist()
