"""Multi-rank window evaluation with the real HIP engines: two processes
on the one GPU form a world-2 gloo group (collectives staged through host memory by
spatialflink_amd.distributed) and run knn_sharded / range_sharded / join_sharded (arrival and
key-band partitions; the owner pack is geohip_band_pack_async) / ppoly_sharded /
join_ppoly_sharded / knn_ppoly_sharded (polygons with holes) with the default libgeohip engines.
Each rank's result is checked against the unsharded C oracle on the whole window (test
infrastructure).  The ranks are child processes (subprocess, not exec)."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import cref
from spatialflink_amd import synth

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pairs(a):
    return sorted(map(tuple, np.asarray(a, dtype=np.int64).reshape(-1, 2).tolist()))


def test_world2_default_engines(tmp_path):
    world, port = 2, _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", str(ROOT / "tests" / "_rank_worker.py"), str(tmp_path)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    assert all(p.returncode == 0 for p in procs), "\n".join(o[-3000:] for o in outs)
    R = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    bj, q = synth.BEIJING, synth.README_QUERY
    cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / 500, 500)
    # kNN: every rank holds the merged result; range: rank-order concatenation
    x, y = synth.uniform(2_000_003, 21)
    wi, wd = cref.knn_pp(cg, x, y, q[0], q[1], 0.05, 100)
    for r in range(world):
        assert R[r]["knn_i"].astype(np.int64).tolist() == wi.astype(np.int64).tolist()
        assert np.array_equal(R[r]["knn_d"].view(np.uint64), wd.view(np.uint64))
    want = cref.range_pp(cg, x, y, q[0], q[1], 0.05).astype(np.int64).tolist()
    assert np.concatenate([R[r]["range"] for r in range(world)]).tolist() == want
    assert [int(R[r]["range_off"]) for r in range(world)] == [0, len(R[0]["range"])]
    # join: disjoint per-rank sets whose union is the window's join, both partitions
    dx, dy = synth.gaussian_clusters(400_001, 3, sigma=0.1)
    qx, qy = synth.gaussian_clusters(2000, 4, sigma=0.1)
    want = _pairs(cref.join_pp(cg, cg, dx, dy, qx, qy, 0.02))
    for part in ("arrival", "cells", "enq"):
        got = [p for r in range(world) for p in _pairs(R[r][f"join_{part}"])]
        assert len(got) == len(set(got)) and sorted(got) == want, part
        assert all(int(R[r][f"join_{part}_total"]) == len(want) for r in range(world))
    assert all(int(R[r]["band_ok"]) == 1 for r in range(world))
    # point-polygon with holes
    pr, roff, vx, vy, _ = synth.holed_polygons(20, 22)
    x, y = synth.uniform(600_001, 23)
    want = _pairs(cref.range_ppoly(cg, x, y, roff, vx, vy, 0.003, poly_rings=pr))
    got = [p for r in range(world) for p in _pairs(R[r]["ppoly"])]
    assert sorted(got) == want and len(want) > 100
    want = _pairs(cref.join_ppoly(cg, cg, x, y, roff, vx, vy, 0.003, poly_rings=pr))
    got = [p for r in range(world) for p in _pairs(R[r]["jppoly"])]
    assert sorted(got) == want
    a, b = pr[0], pr[1]
    wi, wd = cref.knn_ppoly(cg, x, y, vx[roff[a]:roff[b]], vy[roff[a]:roff[b]], 0.003, 50,
                            ring_off=roff[a:b + 1] - roff[a])
    for r in range(world):
        assert R[r]["kppoly_i"].astype(np.int64).tolist() == wi.astype(np.int64).tolist()
        assert np.array_equal(R[r]["kppoly_d"].view(np.uint64), wd.view(np.uint64))
