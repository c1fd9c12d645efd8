"""GPU parity of the ingest codec (geohip_ingest_points) against the C oracle.

Batches go through the C ABI (device record split + per-lane parse on gfx950) and are compared
bit-for-bit with oracle/ingest_oracle.c on the same text: x/y bits, Long timestamps and
HelperClass.assignGridCellID cells; rejected batches must name the first record the oracle
rejects.  At full C2 size (10 M records) the check is the size-independent property of the
synthetic text: x == X / 10^13 exactly (one correctly rounded division of exact operands).
"""
from __future__ import annotations

import random
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import cref  # noqa: E402  (oracle: the checker)
from spatialflink_amd import _abi, synth  # noqa: E402

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING
L100 = (BJ[1] - BJ[0]) / 100


@pytest.fixture(scope="module")
def ctx():
    return _abi.Context(0)


def _grids(n=100):
    l = (BJ[1] - BJ[0]) / n
    return _abi.make_grid(BJ[0], BJ[2], l, n), cref.grid(BJ[0], BJ[2], l, n)


def _check(ctx, fmt, text: bytes, delim=",", fx=2, fy=3, fts=1, n=100, device=False):
    g, cg = _grids(n)
    want = cref.ingest(cref.ingest_spec(fmt, delim, fx, fy, fts), text, cg)
    src = text
    if device:
        import torch
        src = torch.frombuffer(bytearray(text) or bytearray(1), dtype=torch.uint8)[:len(text)].to("cuda:0")
    got = ctx.ingest_points(_abi.make_ingest_spec(fmt, delim, fx, fy, fts), src, g, with_ts=fts >= 0, with_cell=True)
    if device:
        got = {k: v.cpu().numpy() for k, v in got.items()}
    assert len(got["x"]) == len(want["x"])
    assert np.array_equal(got["x"].view(np.uint64), want["x"].view(np.uint64))
    assert np.array_equal(got["y"].view(np.uint64), want["y"].view(np.uint64))
    assert np.array_equal(got["cell"].view(np.uint32), want["cell"])
    if fts >= 0:
        assert np.array_equal(got["ts"], want["ts"])
    return len(want["x"])


def _ragged_csv(n, seed):
    rng = random.Random(seed)
    lines = []
    for i in range(n):
        x = rng.uniform(115.4, 117.7)
        y = rng.uniform(39.5, 41.2)
        style = rng.randrange(6)
        if style == 0:
            xs, ys = repr(x), repr(y)
        elif style == 1:
            xs, ys = f"{x:.6f}", f"{y:.3f}"
        elif style == 2:
            xs, ys = f"{x:.17e}", f"{y:.10E}"
        elif style == 3:
            xs, ys = f'"{x!r}"', f' {y!r} '
        elif style == 4:
            xs, ys = f"{x:.25f}", f"{y:.1f}"
        else:
            xs, ys = f"{int(x)}", f"{y!r}d"
        lines.append(f"{rng.randrange(10 ** rng.randrange(1, 9))} , {1611022449423 + i},{xs},{ys}")
    return "\n".join(lines).encode()


def _fast_forms_csv(n, seed):
    """Records the CSV fast paths take (no blanks or quotes): numbers of every length around the
    SWAR window (19 / 20 digits, 23-25 chars), leading zeros, signs, a bare integer, '-0.0',
    timestamps up to 18 digits (19 are outside the device grammar), object ids of 1 to 30
    characters; plus a few the fast paths hand on (exponent, trailing 'd')."""
    rng = random.Random(seed)
    lines = []
    for i in range(n):
        x = rng.uniform(115.4, 117.7)
        y = rng.uniform(39.5, 41.2)
        k = rng.randrange(14)
        if k == 0:
            xs, ys = repr(x), repr(-y)
        elif k == 1:
            nd = rng.randrange(0, 21)
            xs, ys = f"{x:.{nd}f}", f"{y:.{rng.randrange(0, 21)}f}"
        elif k == 2:
            xs, ys = "00" + f"{x:.10f}", "0.000" + str(rng.randrange(10 ** 12))
        elif k == 3:
            xs, ys = "-0.0", "0"
        elif k == 4:
            xs, ys = f"{x:.16f}", f"{y:.17f}"  # 19 and 19 digits
        elif k == 5:
            xs, ys = f"{x:.17f}", f"{y:.18f}"  # 20 digits: past the SWAR limit
        elif k == 6:
            xs, ys = "1" * rng.randrange(1, 20), "9" * rng.randrange(1, 20)
        elif k == 7:
            xs, ys = f"{x:.22f}", f"{y:.21f}"  # 25 / 23 characters
        elif k == 8:
            xs, ys = f"{x:e}", f"{y!r}"
        elif k == 9:
            xs, ys = f"{x!r}d", f"{y:E}"
        else:
            xs, ys = repr(x), repr(y)
        tsv = rng.choice([1611022449423 + i, -(10 ** 17) - i, 10 ** 17 + i, 10 ** 18 - 1 - i, 0])  # <= 18 digits
        oid = "".join(rng.choice("abcdef0123456789") for _ in range(rng.randrange(1, 31)))
        lines.append(f"{oid},{tsv},{xs},{ys}")
    return "\n".join(lines).encode()


def test_csv_fast_path_forms(ctx):
    text = _fast_forms_csv(60000, 5)
    g, cg = _grids()
    spec = cref.ingest_spec(cref.CSV, ",", 2, 3, 1)
    want = cref.ingest(spec, text, cg)
    got = ctx.ingest_points(_abi.make_ingest_spec(cref.CSV, ",", 2, 3, 1), text, g, with_ts=True, with_cell=True)
    assert np.array_equal(got["x"].view(np.uint64), want["x"].view(np.uint64))
    assert np.array_equal(got["y"].view(np.uint64), want["y"].view(np.uint64))
    assert np.array_equal(got["ts"], want["ts"])


def test_csv_ragged(ctx):
    assert _check(ctx, cref.CSV, _ragged_csv(50000, 1)) == 50000


def test_csv_trailing_newline_and_empty(ctx):
    assert _check(ctx, cref.CSV, _ragged_csv(3000, 2) + b"\n") == 3000
    assert _check(ctx, cref.CSV, b"") == 0
    assert _check(ctx, cref.CSV, b"a,1,116.5,39.75") == 1
    assert _check(ctx, cref.CSV, b"a,1,116.5,39.75\n") == 1


def test_tsv_and_no_timestamp(ctx):
    text = _ragged_csv(20000, 3).replace(b",", b"\t")
    assert _check(ctx, cref.CSV, text, delim="\t", fts=-1) == 20000


def test_wkt(ctx):
    rng = random.Random(4)
    lines = [f"{i},POINT ({rng.uniform(115, 118)!r} {rng.uniform(39, 42)!r}),{i}" for i in range(30000)]
    assert _check(ctx, cref.WKT, "\n".join(lines).encode(), fts=-1) == 30000


def test_geojson(ctx):
    rng = random.Random(5)
    lines = []
    for i in range(30000):
        x, y = rng.uniform(115, 118), rng.uniform(39, 42)
        lines.append('{"geometry":{"coordinates":[%r, %r],"type":"Point"},"properties":{"oID":"%d",'
                     '"timestamp":"2008-02-02 20:12:32"},"type":"Feature"}' % (x, y, i))
    assert _check(ctx, cref.GEOJSON, "\n".join(lines).encode(), fts=-1) == 30000


def test_tiny_records_dense_chunks(ctx):
    # 4-byte records: 2048 records per 8 KB chunk, every lane parses 8 records
    text = b"\n".join(b"%d,%d" % (i % 10, (i * 7) % 10) for i in range(200000))
    assert _check(ctx, cref.CSV, text, fx=0, fy=1, fts=-1) == 200000


def test_long_records_straddle_chunks(ctx):
    # records longer than the 4 KB LDS tail: the parser reads past the staged window from HBM
    rng = random.Random(6)
    lines = []
    for i in range(400):
        pad = "p" * rng.choice([10, 5000, 9000, 20000])
        lines.append(f"{pad},{i},{rng.uniform(115, 118)!r},{rng.uniform(39, 42)!r}")
    assert _check(ctx, cref.CSV, "\n".join(lines).encode()) == 400


def test_device_memory(ctx):
    assert _check(ctx, cref.CSV, _ragged_csv(10000, 7), device=True) == 10000


def test_rejection_names_first_bad_record(ctx):
    good = _ragged_csv(30000, 8).split(b"\n")
    for bad_at in (0, 12345, 29999):
        lines = list(good)
        lines[bad_at] = b"x,1,116.5,abc"
        text = b"\n".join(lines)
        with pytest.raises(cref.IngestRejected) as e:
            cref.ingest(cref.ingest_spec(cref.CSV, ",", 2, 3, 1), text)
        assert e.value.bad == bad_at
        with pytest.raises(_abi.GeohipUnsupportedError) as d:
            ctx.ingest_points(_abi.make_ingest_spec(cref.CSV, ",", 2, 3, 1), text)
        assert d.value.bad == bad_at


def test_rejection_in_overfull_chunk(ctx):
    """A run of blank lines (records the reference rejects) puts more record starts in one chunk
    than the hot kernel lists; the chunk goes whole to the general kernel, which must still name
    the first blank line and keep the good records around it."""
    good = _ragged_csv(20000, 12).split(b"\n")
    for at, run in ((0, 9000), (7000, 5000), (19999, 20000)):
        text = b"\n".join(good[:at] + [b""] * run + good[at:])
        with pytest.raises(cref.IngestRejected) as e:
            cref.ingest(cref.ingest_spec(cref.CSV, ",", 2, 3, 1), text)
        assert e.value.bad == at
        with pytest.raises(_abi.GeohipUnsupportedError) as d:
            ctx.ingest_points(_abi.make_ingest_spec(cref.CSV, ",", 2, 3, 1), text)
        assert d.value.bad == at


def test_capacity(ctx):
    text = _ragged_csv(1000, 9)
    with pytest.raises(_abi.GeohipCapacityError):
        ctx.ingest_points(_abi.make_ingest_spec(cref.CSV, ",", 2, 3, 1), text, cap=999)


def test_full_size_property(ctx):
    """C2 shape: 10 M records of synthetic CSV; every x/y equals X / 10^13 bit-for-bit and every
    cell equals the oracle's cell of that value; a 200 k prefix is also compared with the oracle."""
    import torch
    n = 10_000_000
    text, X, Y = synth.csv_text(n, 2)
    g, cg = _grids(100)
    dtext = torch.from_numpy(text).to("cuda:0")
    got = ctx.ingest_points(_abi.make_ingest_spec(cref.CSV, ",", 2, 3, 1), dtext, g, with_ts=True, with_cell=True)
    gx, gy = got["x"].cpu().numpy(), got["y"].cpu().numpy()
    assert len(gx) == n
    assert np.array_equal(gx.view(np.uint64), (X / 1e13).view(np.uint64))
    assert np.array_equal(gy.view(np.uint64), (Y / 1e13).view(np.uint64))
    assert np.array_equal(got["ts"].cpu().numpy(), 1611022449423 + np.arange(n, dtype=np.int64))
    cut = int(np.searchsorted(np.cumsum(text == 10), 200_000)) + 1
    want = cref.ingest(cref.ingest_spec(cref.CSV, ",", 2, 3, 1), text[:cut].tobytes(), cg)
    assert np.array_equal(got["cell"].cpu().numpy()[:200_000].view(np.uint32), want["cell"])


def test_csv_fast_path_shapes(ctx):
    """Records on and just off the device's CSV fast path (no blanks/quotes, '-'? digits
    ('.' digits)? numbers, <= 19 significant digits, <= 18 timestamp digits) against the oracle:
    both paths must agree bit-for-bit, and every rejected shape must still parse or reject as the
    general grammar does."""
    rng = random.Random(11)
    shapes = ["{x:.6f}", "-{x:.3f}", "00{x:.9f}", "{x:.16f}", "{x:.18f}", "{x:.20f}", "{i}", "-0", "0.000{i}",
              "{x:.6f}.", ".5", "1e3", "+{x:.6f}", "{x:.6f}d", "-", ""]
    lines = []
    for i in range(60000):
        x = rng.uniform(115.4, 117.7)
        y = rng.uniform(39.5, 41.2)
        sx = rng.choice(shapes[:9] if rng.random() < 0.9 else shapes).format(x=x, i=i)
        sy = rng.choice(shapes[:9]).format(x=y, i=i)
        ts = rng.choice([str(1611022449423 + i), "-" + str(i), "0" * 17 + "1", "+5"]) if rng.random() < 0.2 \
            else str(1611022449423 + i)
        oid = rng.choice([str(i), "id%d" % i, "a-b.c"])
        tail = rng.choice(["", ",extra", ",x y", ",\"q\""])
        lines.append(f"{oid},{ts},{sx},{sy}{tail}")
    text = "\n".join(lines).encode()
    spec = cref.ingest_spec(cref.CSV, ",", 2, 3, 1)
    try:
        cref.ingest(spec, text)
        rejected = None
    except cref.IngestRejected as e:
        rejected = e.bad
    if rejected is None:
        _check(ctx, cref.CSV, text)
    else:
        with pytest.raises(_abi.GeohipUnsupportedError) as d:
            ctx.ingest_points(_abi.make_ingest_spec(cref.CSV, ",", 2, 3, 1), text)
        assert d.value.bad == rejected
        good = b"\n".join(l for l in text.split(b"\n") if cref.ingest_record(spec, l) is not None)
        _check(ctx, cref.CSV, good)
