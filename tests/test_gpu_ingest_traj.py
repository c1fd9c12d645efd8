"""GPU: TrajectoryStream ingest (geohip_ingest_trajectory + geohip_ingest_oid_compact) against the
C oracle, and the round trip into the output codecs.

Every field of the Point the reference builds -- Point(objID, x, y, timeStampMillisec, uGrid),
spatialObjects/Point.java:91-100 -- for the three formats (CSVTSVToTSpatial Deserialization.java:
306-321, GeoJSONToTSpatial :149-208, WKTToTSpatial :258-284): x / y bits, timestamps, cells and
the objID bytes (null included) equal oracle/ingest_oracle.c's; rejected batches name the first
record the oracle rejects.  Round trip: device text -> device Points -> device objID strings ->
geohip_format_points (CSV and GeoJSON schemas, Serialization.java:28-50, 125-150) -> bytes equal
to oracle/jdk_double.py's restatement of the serializers applied to the oracle's Points.
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
import jdk_double as J  # noqa: E402  (oracle: the serializers restated)
from spatialflink_amd import _abi, synth  # noqa: E402

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING


def _grids(n=100):
    l = (BJ[1] - BJ[0]) / n
    return _abi.make_grid(BJ[0], BJ[2], l, n), cref.grid(BJ[0], BJ[2], l, n)


def _dev_text(text: bytes):
    import torch
    return torch.frombuffer(bytearray(text) or bytearray(1), dtype=torch.uint8)[:len(text)].to("cuda:0")


def _csv_records(n, seed, delim=","):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        k = rng.randrange(6)
        oid = (str(i) if k < 3 else f' "veh-{i}" ' if k == 3 else f"bus {i % 97}" if k == 4 else f"  lead{i}")
        x = rng.uniform(115.6, 117.5)
        y = rng.uniform(39.7, 41.0)
        xs = f"{x:.13f}" if rng.random() < 0.7 else repr(x)
        out.append(f"{oid}{delim}{1611022449423 + i}{delim}{xs}{delim}{y!r}")  # field 0 keeps leading blanks
    return "\n".join(out).encode()


def _geojson_records(n, seed):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        x, y = rng.uniform(115.6, 117.5), rng.uniform(39.7, 41.0)
        props = []
        if rng.random() < 0.9:
            props.append('"oID":' + rng.choice([f'"{i}"', str(i), f'"car {i % 50}"', "true"]))
        if rng.random() < 0.9:
            props.append(f'"timestamp":"{rng.randrange(2000, 2030)}-{rng.randrange(1, 13):02d}-'
                         f'{rng.randrange(1, 29):02d} {rng.randrange(24):02d}:{rng.randrange(60):02d}:'
                         f'{rng.randrange(60):02d}"')
        if rng.random() < 0.3:
            props.append(f'"speed":{rng.uniform(0, 30)!r}')
        rng.shuffle(props)
        mem = ['"type":"Feature"', f'"geometry":{{"type":"Point","coordinates":[{x!r},{y!r}]}}']
        if rng.random() < 0.95:
            mem.append('"properties":{' + ",".join(props) + "}")
        rng.shuffle(mem)
        out.append("{" + ",".join(mem) + "}")
    return "\n".join(out).encode()


def _check(ctx, spec_args, text: bytes, traj_args=None, n=100):
    g, cg = _grids(n)
    fmt = spec_args[0]
    want = cref.ingest_traj(cref.ingest_spec(*spec_args), cref.traj_spec(**traj_args) if traj_args is not None else None,
                            text, cg)
    spec = _abi.make_ingest_spec(*spec_args[:5], spec_args[5] if len(spec_args) > 5 else 0)
    traj = _abi.make_traj_spec(**traj_args) if traj_args is not None else None
    dtext = _dev_text(text)
    got = ctx.ingest_trajectory(spec, dtext, g, traj, with_ts=True, with_cell=True, with_oid=True)
    m = len(want["x"])
    assert len(got["x"]) == m
    assert np.array_equal(got["x"].cpu().numpy().view(np.uint64), want["x"].view(np.uint64))
    assert np.array_equal(got["y"].cpu().numpy().view(np.uint64), want["y"].view(np.uint64))
    assert np.array_equal(got["ts"].cpu().numpy(), want["ts"])
    assert np.array_equal(got["cell"].cpu().numpy().view(np.uint32), want["cell"])
    oid_text, oid_off = ctx.ingest_oid_compact(dtext, got["oid"])
    assert bytes(oid_text.cpu().numpy()) == want["oid_text"]
    assert np.array_equal(oid_off.cpu().numpy().view(np.uint64), want["oid_off"])
    return got, want, dtext, (oid_text, oid_off), fmt


def test_csv_trajectory_batch(ctx):
    got, want, *_ = _check(ctx, (0, ",", 2, 3, 1, 0), _csv_records(20000, 1))
    assert want["oid"][3] is not None


def test_tsv_and_objid_in_other_columns(ctx):
    rng = random.Random(5)
    lines = [f"{rng.uniform(115.6, 117.5)!r}\t{rng.uniform(39.7, 41)!r}\t{i}\tid {i}\t{rng.randrange(10**12)}"
             for i in range(5000)]
    _check(ctx, (0, "\t", 0, 1, 4, 3), "\n".join(lines).encode())


def test_geojson_trajectory_batch(ctx):
    got, want, *_ = _check(ctx, (1, ",", 0, 1, -1), _geojson_records(20000, 2), dict(utc_offset_min=480))
    assert any(o is None for o in want["oid"]) and any(o is not None for o in want["oid"])
    assert (want["ts"] != 0).any()


def test_wkt_trajectory_batch(ctx):
    text = "\n".join(f"{i}, POINT ({116 + i * 1e-4!r} {40 - i * 1e-4!r})" for i in range(3000)).encode()
    got, want, *_ = _check(ctx, (2, ",", 0, 1, -1), text)
    assert all(o is None for o in want["oid"]) and not want["ts"].any()


def test_rejection_names_first_bad_record(ctx):
    recs = _csv_records(4000, 9).split(b"\n")
    recs[1234] = b",5,116.5,39.9"        # "" objID: handed back to the host
    recs[3000] = b"x,5,116.5"            # IndexOutOfBounds in the reference
    text = b"\n".join(recs)
    with pytest.raises(cref.IngestRejected) as wo:
        cref.ingest_traj(cref.ingest_spec(0, ",", 2, 3, 1, 0), None, text)
    with pytest.raises(_abi.GeohipUnsupportedError) as wd:
        ctx.ingest_trajectory(_abi.make_ingest_spec(0, ",", 2, 3, 1, 0), _dev_text(text), _grids()[0])
    assert wo.value.bad == wd.value.bad == 1234
    gj = _geojson_records(3000, 4).split(b"\n")
    gj[777] = b'{"type":"Feature","geometry":{"type":"Point","coordinates":[1,2]},"properties":{"timestamp":7}}'
    text = b"\n".join(gj)
    with pytest.raises(_abi.GeohipUnsupportedError) as wd:
        ctx.ingest_trajectory(_abi.make_ingest_spec(1), _dev_text(text), _grids()[0], _abi.make_traj_spec())
    assert wd.value.bad == 777


def _decoded(want, i):
    o = want["oid"][i]
    return None if o is None else o.decode()


def test_round_trip_into_output_codecs(ctx):
    """Device ingest -> device objID strings -> geohip_format_points, byte-equal to the serializers
    restated (jdk_double.py) over the oracle's Points."""
    # CSV (PointToCSVTSVOutputSchema with the same [oid, ts, x, y] positions)
    got, want, dtext, (ot, oo), _ = _check(ctx, (0, ",", 2, 3, 1, 0), _csv_records(3000, 21))
    spec = _abi.make_csv_out_spec((0, 1, 2, 3), ",")
    text, _ = ctx.format_points_csv(spec, got["x"], got["y"], got["ts"], ot, oo)
    lines = bytes(text.cpu().numpy()).decode().split("\n")[:-1]
    assert len(lines) == len(want["x"])
    for i, line in enumerate(lines):
        assert line == J.format_point_csv(_decoded(want, i), int(want["ts"][i]), float(want["x"][i]),
                                          float(want["y"][i]), (0, 1, 2, 3), ","), i
    # GeoJSON (PointToGeoJSONOutputSchema: oID / timestamp properties, null objID omitted)
    got, want, dtext, (ot, oo), _ = _check(ctx, (1, ",", 0, 1, -1), _geojson_records(3000, 22),
                                           dict(utc_offset_min=480))
    gspec = _abi.make_text_out_spec(_abi.FMT_GEOJSON, date_format=1, utc_offset_min=480)
    text, _ = ctx.format_points(gspec, got["x"], got["y"], got["ts"], ot, oo)
    lines = bytes(text.cpu().numpy()).decode().split("\n")[:-1]
    for i, line in enumerate(lines):
        assert line == J.format_point_geojson(_decoded(want, i), int(want["ts"][i]), float(want["x"][i]),
                                              float(want["y"][i]), 480), i


def test_full_size_objids(ctx):
    """C2 window size: 10M CSVTSVToTSpatial records 'oid,ts,x,y' (oid = the record index) through
    the fast paths -- every objID span reads back as its record index."""
    import torch
    n = 10_000_000
    text, X, Y = synth.csv_text(n, 2)
    dtext = torch.from_numpy(text).to("cuda:0")
    got = ctx.ingest_trajectory(_abi.make_ingest_spec(0, ",", 2, 3, 1, 0), dtext, _grids()[0], None,
                                with_ts=True, with_cell=False, with_oid=True, cap=n)
    assert len(got["x"]) == n
    ot, oo = ctx.ingest_oid_compact(dtext, got["oid"])
    off = oo.cpu().numpy()
    digits = sum(d * max(0, min(n, 10 ** d) - (10 ** (d - 1) if d > 1 else 0)) for d in range(1, 9))
    assert int(off[n]) == digits
    sample = np.random.default_rng(0).integers(0, n, 2000)
    tb = bytes(ot.cpu().numpy())
    for i in sample.tolist():
        assert tb[int(off[i]):int(off[i + 1])] == str(i).encode()
    assert np.array_equal(got["ts"].cpu().numpy()[sample], 1611022449423 + sample)
