"""The drop-in's ``entries`` / ``incoming`` are mutable like the reference's
attributes (gkarray.py gk:23-24): edits -- Entry fields, list items, appends,
assignment -- are honoured by the next operation on the sketch.  Checked
against the oracle's lists given the same edits (the oracle mirrors the
reference's state as parallel lists)."""
import numpy as np
import pytest

from gk_oracle import OracleGK
from parity_util import same_q

QS = [0.01, 0.25, 0.5, 0.9, 0.99]


def same_state(sk, o):
    got = [(e.val, e.g, e.delta) for e in sk.entries]
    assert got == o.table()
    assert sk.incoming == o.pending


def scenario(device):
    from gkarray_amd import Entry, GKArray
    eps = 0.05
    rng = np.random.default_rng(4)
    xs = rng.lognormal(0, 1, 500)
    sk, o = GKArray(eps, device=device), OracleGK(eps)
    for x in xs[:230]:
        sk.add(x)
        o.add(x)
    same_state(sk, o)
    # edit Entry fields in place
    es = sk.entries
    es[3].g += 2
    o.g[3] += 2
    es[5].delta = 1
    o.d[5] = 1
    for x in xs[230:300]:  # the add flushes at n % 21 == 0 with the edited table
        sk.add(x)
        o.add(x)
    same_state(sk, o)
    # drop an entry and a pending value, append a pending value
    es = sk.entries
    del es[7]
    del o.v[7], o.g[7], o.d[7]
    inc = sk.incoming
    if inc:
        inc.pop(0)
        o.pending.pop(0)
    inc.append(1.25)
    o.pending.append(1.25)
    assert all(same_q(a, b, False) for a, b in zip(sk.quantiles(QS), o.quantiles(QS)))
    same_state(sk, o)
    # assignment
    sk.entries = [Entry(0.5, 1, 0), Entry(2.0, 3, 1)]
    o.v, o.g, o.d = [0.5, 2.0], [1, 3], [0, 1]
    o.pending = []
    sk.incoming = []
    for x in xs[300:]:
        sk.add(x)
        o.add(x)
    same_state(sk, o)
    got, exp = sk.quantiles(QS), o.quantiles(QS)
    assert all(same_q(a, b, False) for a, b in zip(got, exp))
    # a list obtained before an operation is detached after it
    es = sk.entries
    sk.size()
    es.clear()
    assert len(sk.entries) == len(o.table())


def test_mutable_entries_and_incoming_cpu_engine():
    scenario("cpu")


@pytest.mark.gpu
def test_mutable_entries_and_incoming_gpu(gpu_device):
    scenario(gpu_device)
