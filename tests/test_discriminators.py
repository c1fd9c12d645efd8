"""The parity-pinning kit (tests/golden/jts_discriminators.json) checked on
the CPU: the committed cases really discriminate (readings A and B differ on each), and the C
oracle (oracle/geohip_oracle.c, the checker of every GPU parity test) follows reading A on all of
them -- so a JVM run of jvm/ParityHarness.java that reports reading B for a question names exactly
the oracle and kernel code to change.  tests/test_gpu_discriminators.py asserts the same answers
for libgeohip on the GPU."""
import json
from pathlib import Path

import numpy as np

import cref

FIX = json.loads((Path(__file__).resolve().parent / "golden" / "jts_discriminators.json").read_text())


def f(h):
    return float.fromhex(h)


def _grid(g):
    return cref.grid(f(g["min_x"]), f(g["min_y"]), (f(g["max_x"]) - f(g["min_x"])) / g["n"], g["n"])


def test_q1_pairs_and_knn_follow_reading_a():
    q = [f(v) for v in FIX["Q1"]["pairs_from_query"]["query"]]
    for c in FIX["Q1"]["pairs_from_query"]["cases"]:
        assert c["A"] != c["B"]
        d = cref.hypot(q[0] - f(c["p"][0]), q[1] - f(c["p"][1]))
        assert d.hex() == c["A"]
    kn = FIX["Q1"]["knn"]
    assert kn["A"]["idx"] != kn["B"]["idx"]
    x = np.array([f(v) for v in kn["x"]])
    y = np.array([f(v) for v in kn["y"]])
    qq = [f(v) for v in kn["query"]]
    idx, dist = cref.knn_pp(_grid(kn["grid"]), x, y, qq[0], qq[1], f(kn["r"]), kn["k"])
    assert idx.tolist() == kn["A"]["idx"]
    assert [float(d).hex() for d in dist] == kn["A"]["dist"]


def test_q2_containment_follows_reading_a():
    ring = FIX["Q2"]["ring"]
    vx = np.array([f(a) for a, _ in ring])
    vy = np.array([f(b) for _, b in ring])
    for c in FIX["Q2"]["cases"]:
        assert c["A_inside"] != c["B_inside"]
        d = cref.point_polygon(f(c["p"][0]), f(c["p"][1]), vx, vy)
        assert (d == 0.0) == c["A_inside"] and d.hex() == c["A_dist"]


def test_q3_point_to_segment_follows_reading_a():
    ring = FIX["Q3"]["ring"]
    vx = np.array([f(a) for a, _ in ring])
    vy = np.array([f(b) for _, b in ring])
    for c in FIX["Q3"]["cases"]:
        assert c["A"] != c["B"]
        assert cref.point_polygon(f(c["p"][0]), f(c["p"][1]), vx, vy).hex() == c["A"]
