"""Shared helpers for the parity tests."""
import numpy as np


def fx(s):
    return float.fromhex(s)


def arr(lst):
    return np.array([float.fromhex(v) for v in lst], dtype=np.float64)


def grid_vals(gd):
    return fx(gd["min_x"]), fx(gd["min_y"]), fx(gd["cell_len"]), gd["n"]


def pairs_sorted(p):
    p = np.asarray(p, dtype=np.int64).reshape(-1, 2)
    if len(p) == 0:
        return p
    o = np.lexsort((p[:, 1], p[:, 0]))
    return p[o]
