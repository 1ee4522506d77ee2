"""GKSTATE files (csrc/gk_format.h, gkarray_amd/stateio.py) on the host: round
trip of an oracle-produced state, checksum / version / truncation errors."""
import os

import numpy as np
import pytest

from gk_oracle_c import OracleSet
from gkarray_amd import stateio


def oracle_state(o):
    offs, v, g, d = o.tables()
    poffs, pv = o.pending()
    st = o.stats()
    return dict(eps=o.eps, offs=offs, v=v, g=g, d=d, poffs=poffs, pv=pv, n=st["n"], min=st["min"],
                max=st["max"], sum=st["sum"], avg=st["avg"])


def make_oracle(S=300, eps=0.01, seed=3):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 3000, S)
    lens[:3] = [0, 1, 101]
    offs = np.zeros(S + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    x = rng.lognormal(0, 1, int(offs[-1]))
    x[::17] = -0.0
    o = OracleSet(S, eps)
    o.ingest(x, offs)
    return o


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype.kind == "f":
        return a.shape == b.shape and np.array_equal(a.view(np.int64), np.asarray(b, np.float64).view(np.int64))
    return np.array_equal(a.astype(np.int64), np.asarray(b).astype(np.int64))


def test_roundtrip_oracle_state(tmp_path):
    o = make_oracle()
    st = oracle_state(o)
    p = str(tmp_path / "s.gks")
    stateio.write_state(p, st)
    back = stateio.read_state(p)
    assert back["eps"] == st["eps"]
    for k in ("offs", "v", "g", "d", "poffs", "pv", "n", "min", "max", "sum", "avg"):
        assert same(back[k], st[k]), k
    with open(p, "rb") as f:
        raw = f.read()
    assert raw[:8] == b"GKSTATE\0" and int.from_bytes(raw[8:12], "little") == 1
    assert len(raw) % 8 == 0


def test_empty_set(tmp_path):
    p = str(tmp_path / "e.gks")
    z = np.zeros(0)
    stateio.write_state(p, dict(eps=0.1, offs=[0], v=z, g=z, d=z, poffs=[0], pv=z, n=z, min=z, max=z,
                                sum=z, avg=z))
    b = stateio.read_state(p)
    assert b["offs"].tolist() == [0] and b["v"].size == 0


def test_corruption_is_detected(tmp_path):
    o = make_oracle(S=40)
    p = str(tmp_path / "c.gks")
    stateio.write_state(p, oracle_state(o))
    raw = bytearray(open(p, "rb").read())
    bad = bytearray(raw)
    bad[stateio.HEADER_BYTES + 200] ^= 0x01
    open(p, "wb").write(bytes(bad))
    with pytest.raises(stateio.StateFormatError, match="checksum"):
        stateio.read_state(p)
    bad = bytearray(raw)
    bad[8] = 2  # version
    open(p, "wb").write(bytes(bad))
    with pytest.raises(stateio.StateFormatError, match="version"):
        stateio.read_state(p)
    open(p, "wb").write(bytes(raw[:-8]))
    with pytest.raises(stateio.StateFormatError):
        stateio.read_state(p)
    open(p, "wb").write(b"not a state file at all" * 8)
    with pytest.raises(stateio.StateFormatError):
        stateio.read_state(p)
    assert os.path.exists(p)
