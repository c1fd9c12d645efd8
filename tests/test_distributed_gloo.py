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
