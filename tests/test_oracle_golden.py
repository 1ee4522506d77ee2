"""Pin the oracle: both CPU restatements (oracle/gk_oracle.py and the C
restatement oracle/gk_oracle.c) against the golden vectors that
tests/golden/make_golden.py produced from the unmodified reference gkarray.py.

Tolerance: exact (bitwise) everywhere, except one exactly named input class --
the sign of a zero returned by the small-n numpy.percentile branch (gk:171,
gk:202) when golden_io.zero_sign_unpinned holds (both interpolation positions
are zeros, gamma >= 0.5, and the table holds both +0.0 and -0.0): numpy's
partition places equal keys CPU-dependently ("parity unpinned" for the sign of
zero there only; the value 0 is pinned).  The restatements answer from the
stable table order there, as the GPU path does, so GPU-vs-oracle tests are
strict everywhere.
"""
import numpy as np
import pytest

import golden_io as G
from gk_oracle import OracleEpsMismatch, OracleGK, percentile_linear
from gk_oracle_c import OracleSet


def same_q(a, b, unpinned):
    """Bitwise; the sign of a zero is tolerated only for an answer in the
    unpinned class (golden_io.zero_sign_unpinned).  The rank walk (gk:173-185,
    209-230) returns a table value, _min or _max: exact, sign included."""
    if G.same_float(a, b):
        return True
    return bool(unpinned) and a == 0 and b == 0


def assert_qs(got, exp, what, unp):
    assert len(got) == len(exp), what
    for a, b, u in zip(got, exp, unp):
        assert same_q(a, b, u), "%s: %r vs %r" % (what, list(got), list(exp))


STREAMS = G.cases("stream")


@pytest.mark.parametrize("case", STREAMS, ids=lambda c: "c%d-e%s-%s-%d" % (c["id"], c["eps"], c["dist"], c["L"]))
def test_python_oracle_stream(case):
    cid, eps = case["id"], case["eps"]
    xs = G.get(cid, "x")
    o = OracleGK(eps)
    per = G.has(cid, "flush/sizes")
    tabs = []
    for x in xs:
        o.add(x)
        if per and not o.pending:
            tabs.append(o.table())
    if per:
        exp = G.tables(cid, "flush")
        assert len(exp) == len(tabs)
        for k, (a, b) in enumerate(zip(tabs, exp)):
            assert G.same_table(a, b), "flush %d" % k
        assert [int(n) for n in G.get(cid, "flush_n")] == [
            (k + 1) * (int(1.0 / eps) + 1) for k in range(len(tabs))]
    assert G.same_table(o.table(), G.tables(cid, "auto")[0])
    assert all(G.same_float(a, b) for a, b in zip(o.pending, G.get(cid, "pending")))
    before = [o.n, o.min, o.max, o.sum, o.avg]
    assert all(G.same_float(a, b) for a, b in zip(before, G.get(cid, "stats_before_query")))
    fin = G.tables(cid, "final")[0]
    um = lambda qs: G.unpinned_mask(fin, o.n, eps, qs)  # noqa: E731
    assert_qs([o.quantile(q) for q in G.index()["qs"]], G.get(cid, "q_single"), "quantile", um(G.index()["qs"]))
    assert G.same_table(o.table(), fin)
    assert_qs(o.quantiles(G.index()["qs"]), G.get(cid, "q_sorted"), "quantiles", um(G.index()["qs"]))
    assert_qs(o.quantiles(G.index()["qs_unsorted"]), G.get(cid, "q_unsorted"), "unsorted",
              um(G.index()["qs_unsorted"]))
    assert_qs(o.quantiles(G.index()["qs_oor"]), G.get(cid, "q_oor"), "out-of-range", um(G.index()["qs_oor"]))
    assert o.size() == int(G.get(cid, "size")[0])


def test_c_oracle_streams_batched():
    """All stream cases of one eps in ONE batched C-oracle set."""
    by_eps = {}
    for c in STREAMS:
        by_eps.setdefault(c["eps"], []).append(c)
    for eps, cs in by_eps.items():
        xs = [G.get(c["id"], "x") for c in cs]
        offs = np.zeros(len(cs) + 1, np.int64)
        offs[1:] = np.cumsum([len(x) for x in xs])
        o = OracleSet(len(cs), eps)
        o.ingest(np.concatenate(xs), offs)
        poffs, pv = o.pending()
        for k, c in enumerate(cs):
            assert G.same_table(o.table(k), G.tables(c["id"], "auto")[0]), c
            assert np.array_equal(pv[poffs[k]:poffs[k + 1]], G.get(c["id"], "pending")), c
        st = o.stats()
        for k, c in enumerate(cs):
            got = [st["n"][k], st["min"][k], st["max"][k], st["sum"][k], st["avg"][k]]
            assert all(G.same_float(a, b) for a, b in zip(got, G.get(c["id"], "stats_before_query")))
        um = lambda k, c, qs: G.unpinned_mask(G.tables(c["id"], "final")[0], st["n"][k], eps, qs)  # noqa: E731
        q = o.quantiles(G.index()["qs"], single=True)
        for k, c in enumerate(cs):
            assert_qs(q[k], G.get(c["id"], "q_single"), "c-quantile %r" % c, um(k, c, G.index()["qs"]))
            assert G.same_table(o.table(k), G.tables(c["id"], "final")[0]), c
        q = o.quantiles(G.index()["qs"])
        for k, c in enumerate(cs):
            assert_qs(q[k], G.get(c["id"], "q_sorted"), "c-quantiles %r" % c, um(k, c, G.index()["qs"]))
        q = o.quantiles(G.index()["qs_unsorted"])
        for k, c in enumerate(cs):
            assert_qs(q[k], G.get(c["id"], "q_unsorted"), "c-unsorted %r" % c, um(k, c, G.index()["qs_unsorted"]))


@pytest.mark.parametrize("case", G.cases("query_mid"), ids=lambda c: "c%d" % c["id"])
def test_oracles_query_mid(case):
    cid, eps = case["id"], case["eps"]
    xs = G.get(cid, "x")
    pts = [int(p) for p in G.get(cid, "query_points")]
    exp_q = G.get(cid, "mid_q")
    exp_t = G.tables(cid, "mid_tables")
    # python
    o = OracleGK(eps)
    k = 0
    for i, x in enumerate(xs):
        o.add(x)
        if i + 1 in pts:
            assert_qs(o.quantiles([0.1, 0.5, 0.9]), exp_q[k], "py mid %d" % k,
                      G.unpinned_mask(exp_t[k], o.n, eps, [0.1, 0.5, 0.9]))
            assert G.same_table(o.table(), exp_t[k])
            k += 1
    assert G.same_table(o.table(), exp_t[-1])
    # C, fed in chunks that end at the query points
    c = OracleSet(1, eps)
    prev = 0
    for k, pnt in enumerate(pts):
        c.ingest(xs[prev:pnt], [0, pnt - prev])
        assert_qs(c.quantiles([0.1, 0.5, 0.9])[0], exp_q[k], "c mid %d" % k,
                  G.unpinned_mask(exp_t[k], pnt, eps, [0.1, 0.5, 0.9]))
        assert G.same_table(c.table(0), exp_t[k])
        prev = pnt
    c.ingest(xs[prev:], [0, len(xs) - prev])
    assert G.same_table(c.table(0), exp_t[-1])


@pytest.mark.parametrize("case", G.cases("merge"), ids=lambda c: "c%d-k%d" % (c["id"], c["k"]))
def test_oracles_merge(case):
    cid, eps = case["id"], case["eps"]
    shards = G.shards(cid)
    steps = G.tables(cid, "merge_steps")
    others = G.tables(cid, "others_after")
    for impl in ("py", "c"):
        if impl == "py":
            sk = []
            for xs in shards:
                o = OracleGK(eps)
                o.add_many(xs)
                sk.append(o)
            acc = sk[0]
            for k, other in enumerate(sk[1:]):
                acc.merge(other)
                assert G.same_table(acc.table(), steps[k])
                assert G.same_table(other.table(), others[k])
            got = [acc.n, acc.min, acc.max, acc.sum, acc.avg]
            n_acc = acc.n
            q = acc.quantiles(G.index()["qs"])
        else:
            sk = []
            for xs in shards:
                o = OracleSet(1, eps)
                o.ingest(xs, [0, len(xs)])
                sk.append(o)
            acc = sk[0]
            for k, other in enumerate(sk[1:]):
                acc.merge(other)
                assert G.same_table(acc.table(0), steps[k])
                assert G.same_table(other.table(0), others[k])
            st = acc.stats()
            got = [st["n"][0], st["min"][0], st["max"][0], st["sum"][0], st["avg"][0]]
            n_acc = st["n"][0]
            q = acc.quantiles(G.index()["qs"])[0]
        assert all(G.same_float(a, b) for a, b in zip(got, G.get(cid, "merged_stats"))), impl
        # merge() raises eps to max(eps, other.eps) (gk:150): equal here
        assert_qs(q, G.get(cid, "merged_q"), impl, G.unpinned_mask(steps[-1] if steps else G.tables(cid, "merge_steps")[-1],
                                                                   n_acc, eps, G.index()["qs"]))


def check_merge_plan(case, build, table, stats_of, quantiles):
    """sk[0].merge(sk[p]) for p in the case's plan (p == 0: the sketch merged
    into itself, gk:111-154), every step's destination and source table, the
    final stats and quantiles against the reference's (make_golden.py 7)."""
    cid, eps = case["id"], case["eps"]
    sk = [build(xs) for xs in G.shards(cid)]
    steps, srcs = G.tables(cid, "merge_steps"), G.tables(cid, "others_after")
    for k, p in enumerate(int(p) for p in G.get(cid, "plan")):
        sk[0].merge(sk[p])
        assert G.same_table(table(sk[0]), steps[k]), (case, k)
        assert G.same_table(table(sk[p]), srcs[k]), (case, k)
    got = stats_of(sk[0])
    assert all(G.same_float(a, b) for a, b in zip(got, G.get(cid, "merged_stats"))), (case, got)
    assert_qs(quantiles(sk[0]), G.get(cid, "merged_q"), case,
              G.unpinned_mask(steps[-1], got[0], eps, G.index()["qs"]))
    assert G.same_table(table(sk[0]), G.tables(cid, "merged_final")[0]), case


MERGE_PLANS = G.cases("merge_plan")


@pytest.mark.parametrize("case", MERGE_PLANS, ids=lambda c: "c%d-e%s-L%d-%s" % (c["id"], c["eps"], c["L"], c["plan"]))
def test_oracles_merge_plan(case):
    eps = case["eps"]

    def py(xs):
        o = OracleGK(eps)
        o.add_many(xs)
        return o

    def c(xs):
        o = OracleSet(1, eps)
        o.ingest(xs, [0, len(xs)])
        return o

    check_merge_plan(case, py, lambda o: o.table(), lambda o: [o.n, o.min, o.max, o.sum, o.avg],
                     lambda o: o.quantiles(G.index()["qs"]))
    check_merge_plan(case, c, lambda o: o.table(0),
                     lambda o: [o.stats()[k][0] for k in ("n", "min", "max", "sum", "avg")],
                     lambda o: o.quantiles(G.index()["qs"])[0])


def test_merge_plans_cover_self_merge():
    plans = [c["plan"] for c in MERGE_PLANS]
    assert [0] in plans and [0, 0] in plans and [1, 0] in plans and [1, 1] in plans
    assert {c["L"] for c in MERGE_PLANS} >= {0, 1, 5}  # empty, small-n
    assert {c["eps"] for c in MERGE_PLANS} == {0.1, 0.01}


def test_eps_mismatch_raises():
    assert any(c["kind"] == "eps_mismatch" and c["raised"] for c in G.index()["cases"])
    a, b = OracleGK(0.01), OracleGK(0.02)
    a.add(1.0)
    b.add(2.0)
    with pytest.raises(OracleEpsMismatch):
        a.merge(b)


def test_known_answer_vectors():
    kat = G.index()["kat"]
    o = OracleGK(0.1)
    xs = [float((7 * i) % 23) for i in range(40)]
    o.add_many(xs[:33])
    assert o.table() == [tuple(r) for r in kat["kat1_table_after_33"]]
    assert len(o.pending) == kat["kat1_pending_after_33"] == 0  # flushed at n=33 (P=11)
    o.add_many(xs[33:])
    assert o.quantiles([0, .25, .5, .75, 1]) == kat["kat1_quantiles"] == [0, 5, 10, 19, 22]
    assert o.table() == [tuple(r) for r in kat["kat1_final_table"]]
    o = OracleGK(0.1)
    o.add_many([3.0, 1.0, 2.0])
    assert o.quantile(.5) == kat["kat2_q50"] == 2.0
    assert o.quantile(.25) == kat["kat2_q25"] == 1.5


def test_known_answer_1m_c_oracle():
    kat = G.index()["kat"]
    x = np.random.default_rng(0).random(1_000_000)
    o = OracleSet(1, 0.01)
    o.ingest(x, [0, x.size])
    q = o.quantiles([.5, .9, .99])[0].tolist()
    assert q == kat["kat3_quantiles"] == [0.49742269548761897, 0.9042186538756599, 0.9999998846722377]
    assert o.stats()["size"][0] == kat["kat3_size"] == 71
    assert o.table(0) == [tuple(r) for r in kat["kat3_table"]]


def test_percentile_restatement_matches_numpy():
    rng = np.random.default_rng(3)
    for _ in range(400):
        n = int(rng.integers(1, 60))
        a = np.sort(rng.normal(size=n) * 10.0 ** rng.integers(-3, 4))
        for q in np.concatenate([rng.random(5), [0.0, 1.0, 0.5, 0.25, 0.75]]):
            assert G.same_float(percentile_linear(list(a), q), np.percentile(a, q * 100))


def test_zero_sign_class_is_exact():
    """golden_io.zero_sign_unpinned names EXACTLY the inputs where numpy's
    percentile and the stable-order restatement may differ: fuzzed against
    numpy itself on tables of +0.0 / -0.0 / normals (stable-sorted, as a
    small-n table is), every mismatch lies in the class, and every answer
    outside it is bit-identical (the sign included)."""
    rng = np.random.default_rng(11)
    hits = 0
    for _ in range(20000):
        n = int(rng.integers(1, 40))
        nz = int(rng.integers(0, n + 1))
        vals = list(rng.normal(size=n - nz)) + [(-0.0 if rng.random() < 0.5 else 0.0) for _ in range(nz)]
        rng.shuffle(vals)
        tab = sorted(vals)  # stable: -0.0 / +0.0 keep their insertion order
        q = float(rng.choice([0.0, 0.1, 0.25, 0.5, 0.75, 0.9, 0.99, 1.0, rng.random()]))
        got = percentile_linear(tab, q)
        ref = np.percentile(tab, q * 100)
        unp = G.zero_sign_unpinned(tab, n, 1.0 / (n + 1), q)
        if not G.same_float(got, ref):
            assert unp and got == 0 and ref == 0, (tab, q, got, ref)
            hits += 1
    assert hits > 0  # the class is real on this numpy (AVX-512 partition network here)
