"""Parity of the HIP path (through the C ABI) with the reference.

* against the golden vectors produced by the reference itself
  (tests/golden/make_golden.py) -- every stream, mid-stream query and merge
  case, batched into StreamSets;
* against the C restatement of the oracle (pinned by test_oracle_golden.py) on
  seeded random batches, with random chunking of the ingest calls;
* size-independent properties at larger sizes.

Bar: bit-exact tables (v, g, delta), pending values, n/min/max/sum/avg and
quantiles.  Against the oracle: strict everywhere, the sign of zero included.
Against the reference's goldens, one exactly named tolerance: the sign of a
zero from the small-n numpy.percentile branch in golden_io.zero_sign_unpinned's
class (numpy's partition places +0.0 / -0.0 CPU-dependently there, see
test_oracle_golden.py); everything else bit for bit.
"""
import numpy as np
import pytest
import torch

import golden_io as G
from gk_oracle_c import OracleSet
from parity_util import (_ss, assert_same_quantiles, assert_same_state, assert_same_tables,
                         check_golden_merge_plans, csr, gen, ingest_np, golden_mask, small_of, tables_np)

pytestmark = pytest.mark.gpu


# ----------------------------------------------------------------------------
# golden vectors from the reference
# ----------------------------------------------------------------------------
def test_golden_streams(gpu_device):
    by_eps = {}
    for c in G.cases("stream"):
        by_eps.setdefault(c["eps"], []).append(c)
    for eps, cs in by_eps.items():
        ss = _ss(len(cs), eps, gpu_device)
        ingest_np(ss, [G.get(c["id"], "x") for c in cs])
        for k, c in enumerate(cs):
            assert G.same_table(ss.table(k), G.tables(c["id"], "auto")[0]), c
        poffs, pv = ss.pending()
        poffs, pv = poffs.cpu().numpy(), pv.cpu().numpy()
        st = {k: v.cpu().numpy() for k, v in ss.stats().items()}
        for k, c in enumerate(cs):
            assert np.array_equal(pv[poffs[k]:poffs[k + 1]].view(np.int64),
                                  G.get(c["id"], "pending").view(np.int64)), c
            got = [st["n"][k], st["min"][k], st["max"][k], st["sum"][k], st["avg"][k]]
            assert all(G.same_float(a, b) for a, b in zip(got, G.get(c["id"], "stats_before_query"))), c
        um = lambda k, c, qs: golden_mask(G.tables(c["id"], "final")[0], st["n"][k], eps, qs)  # noqa: E731
        q = ss.quantiles(G.index()["qs"], single=True).cpu().numpy()
        for k, c in enumerate(cs):
            assert_same_quantiles(q[k], G.get(c["id"], "q_single"), "quantile %r" % c, um(k, c, G.index()["qs"]))
            assert G.same_table(ss.table(k), G.tables(c["id"], "final")[0]), c
        q = ss.quantiles(G.index()["qs"]).cpu().numpy()
        q2 = ss.quantiles(G.index()["qs_unsorted"]).cpu().numpy()
        q3 = ss.quantiles(G.index()["qs_oor"]).cpu().numpy()
        for k, c in enumerate(cs):
            assert_same_quantiles(q[k], G.get(c["id"], "q_sorted"), "quantiles %r" % c, um(k, c, G.index()["qs"]))
            assert_same_quantiles(q2[k], G.get(c["id"], "q_unsorted"), "unsorted %r" % c, um(k, c, G.index()["qs_unsorted"]))
            assert_same_quantiles(q3[k], G.get(c["id"], "q_oor"), "oor %r" % c, um(k, c, G.index()["qs_oor"]))
        st = ss.stats()
        for k, c in enumerate(cs):
            assert int(st["size"][k]) == int(G.get(c["id"], "size")[0])


def test_golden_query_mid(gpu_device):
    for c in G.cases("query_mid"):
        cid, eps = c["id"], c["eps"]
        xs = G.get(cid, "x")
        pts = [int(p) for p in G.get(cid, "query_points")]
        exp_q = G.get(cid, "mid_q")
        exp_t = G.tables(cid, "mid_tables")
        ss = _ss(1, eps, gpu_device)
        prev = 0
        for k, p in enumerate(pts):
            ingest_np(ss, [xs[prev:p]])
            assert_same_quantiles(ss.quantiles([0.1, 0.5, 0.9]).cpu().numpy()[0], exp_q[k], "mid %r" % c,
                                  golden_mask(G.tables(cid, "mid_tables")[k], p, eps, [0.1, 0.5, 0.9]))
            assert G.same_table(ss.table(0), exp_t[k]), c
            prev = p
        ingest_np(ss, [xs[prev:]])
        assert G.same_table(ss.table(0), exp_t[-1]), c


def test_golden_merges(gpu_device):
    for c in G.cases("merge"):
        cid, eps = c["id"], c["eps"]
        shards = G.shards(cid)
        sets = []
        for xs in shards:
            ss = _ss(1, eps, gpu_device)
            ingest_np(ss, [xs])
            sets.append(ss)
        steps = G.tables(cid, "merge_steps")
        others = G.tables(cid, "others_after")
        acc = sets[0]
        for k, o in enumerate(sets[1:]):
            acc.merge_from([o])
            assert G.same_table(acc.table(0), steps[k]), (c, k)
            assert G.same_table(o.table(0), others[k]), (c, k)
        st = {k: v.cpu().numpy() for k, v in acc.stats().items()}
        got = [st["n"][0], st["min"][0], st["max"][0], st["sum"][0], st["avg"][0]]
        assert all(G.same_float(a, b) for a, b in zip(got, G.get(cid, "merged_stats"))), c
        assert_same_quantiles(acc.quantiles(G.index()["qs"]).cpu().numpy()[0], G.get(cid, "merged_q"), c,
                              golden_mask(steps[-1], st["n"][0], eps, G.index()["qs"]))


def test_golden_merge_plans(gpu_device):
    """a.merge(a) and repeated sources (gk:111-154) against the reference: the
    self-merge runs from a snapshot of the flushed set (gk_capi.cpp
    merge_self), bit-exact to every step of the reference's plan."""
    assert check_golden_merge_plans(gpu_device) == len(G.cases("merge_plan")) > 100


def test_dropin_self_merge(gpu_device):
    from gkarray_amd import GKArray
    from gk_oracle import OracleGK
    xs = np.random.default_rng(7).lognormal(0, 1, 1234)
    sk, o = GKArray(0.01), OracleGK(0.01)
    for x in xs:
        sk.add(x)
    o.add_many(xs)
    sk.merge(sk)
    o.merge(o)
    assert sk._n == o.n == 2468
    assert [(e.val, e.g, e.delta) for e in sk.entries] == o.table()
    assert sk.quantiles([.5, .9]) == o.quantiles([.5, .9])
    # StreamSet: the set itself inside a longer source list, at scale
    rng = np.random.default_rng(8)
    S, eps = 3000, 0.01
    seqs = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), rng.integers(0, 3000, S))]
    other = [gen(1, int(L), rng) for L in rng.integers(0, 3000, S)]
    a, b = _ss(S, eps, gpu_device), _ss(S, eps, gpu_device)
    oa, ob = OracleSet(S, eps), OracleSet(S, eps)
    ingest_np(a, seqs)
    ingest_np(b, other)
    oa.ingest(*csr(seqs))
    ob.ingest(*csr(other))
    a.merge_from([b, a, b, a])
    for src in (ob, oa, ob, oa):
        oa.merge(src)
    assert_same_state(a, oa, "self-merge fold")
    assert_same_state(b, ob, "repeated source")


def test_self_merge_promoted_streams_eps_0001(gpu_device):
    """a.merge(a) at eps = 0.001 (P = 1001: no small class) with streams
    promoted out of class 0 (descending streams: thousands of entries, the
    32768 class) beside short ones: the snapshot path of merge_self in the
    larger classes, twice in a row (its scratch set is made and released per
    merge), bit-exact vs the oracle."""
    rng = np.random.default_rng(31)
    eps = 0.001
    seqs = [np.arange(300000, 0, -1, dtype=np.float64), rng.random(50000), rng.lognormal(0, 1, 5000),
            np.zeros(0), np.arange(30000, 0, -1, dtype=np.float64) * 0.5, rng.pareto(1.5, 2999) + 1]
    a, oa = _ss(len(seqs), eps, gpu_device), OracleSet(len(seqs), eps)
    ingest_np(a, seqs)
    oa.ingest(*csr(seqs))
    assert a.num_promoted >= 1
    a.merge_from([a])
    oa.merge(oa)
    assert_same_state(a, oa, "self-merge eps=.001")
    more = [rng.random(int(L)) for L in rng.integers(0, 4000, len(seqs))]
    ingest_np(a, more)
    oa.ingest(*csr(more))
    a.merge_from([a, a])
    oa.merge(oa)
    oa.merge(oa)
    assert_same_state(a, oa, "self-merge twice eps=.001")


def test_eps_mismatch(gpu_device):
    from gkarray_amd import UnequalEpsilonException
    a = _ss(4, 0.01, gpu_device)
    b = _ss(4, 0.02, gpu_device)
    with pytest.raises(UnequalEpsilonException):
        a.merge_from([b])


def test_drop_in_gkarray_kat(gpu_device):
    from gkarray_amd import GKArray, UnequalEpsilonException
    kat = G.index()["kat"]
    sk = GKArray(0.1)
    xs = [float((7 * i) % 23) for i in range(40)]
    for x in xs[:33]:
        sk.add(x)
    assert [(e.val, e.g, e.delta) for e in sk.entries] == [tuple(r) for r in kat["kat1_table_after_33"]]
    for x in xs[33:]:
        sk.add(x)
    assert sk.quantiles([0, .25, .5, .75, 1]) == [0, 5, 10, 19, 22]
    assert [(e.val, e.g, e.delta) for e in sk.entries] == [tuple(r) for r in kat["kat1_final_table"]]
    sk = GKArray(0.1)
    for x in [3.0, 1.0, 2.0]:
        sk.add(x)
    assert sk.quantile(.5) == 2.0 and sk.quantile(.25) == 1.5
    assert sk.num_values() == 3 and sk.name == "GKArray"
    assert np.isnan(sk.quantile(1.5)) and np.isnan(sk.quantile(-0.1))
    e = GKArray(0.1)
    assert np.isnan(e.quantile(0.5)) and all(np.isnan(v) for v in e.quantiles([0.1, 0.2]))
    with pytest.raises(UnequalEpsilonException):
        sk.merge(GKArray(0.2))
    big = GKArray(0.01)
    big.add_many(np.random.default_rng(0).random(1_000_000))
    assert big.quantiles([.5, .9, .99]) == kat["kat3_quantiles"]
    assert big.size() == kat["kat3_size"]
    st = kat["kat3_stats"]
    assert [big._n, big._min, big._max, big._sum, big._avg] == st


# ----------------------------------------------------------------------------
# random batches against the C oracle
# ----------------------------------------------------------------------------
@pytest.mark.parametrize("eps", [0.2, 0.1, 0.05, 0.03, 0.015, 0.01, 0.001])
def test_random_batches_vs_oracle(gpu_device, eps):
    rng = np.random.default_rng(int(eps * 1e6) + 11)
    S = 600 if eps >= 0.01 else 120
    P = int(1.0 / eps) + 1
    lens = rng.integers(0, 12 * P, S)
    lens[:4] = [0, 1, P, P - 1]
    dists = rng.integers(0, 8, S)
    seqs = [gen(int(d), int(L), rng) for d, L in zip(dists, lens)]
    ss = _ss(S, eps, gpu_device)
    osx = OracleSet(S, eps)
    # ingest in 3 random chunks per stream (different split points per stream)
    cuts = [np.sort(rng.integers(0, max(len(x), 1) + 1, 2)) for x in seqs]
    for part in range(3):
        piece = []
        for x, c in zip(seqs, cuts):
            a = 0 if part == 0 else int(c[part - 1])
            b = int(c[part]) if part < 2 else len(x)
            piece.append(x[a:b])
        flat, offs = csr(piece)
        ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
        osx.ingest(flat, offs)
        assert_same_state(ss, osx, "eps=%g part %d" % (eps, part))
    for qs, single in (([0.5, 0.9, 0.99], False), ([0.99, 0.1, 0.5], False),
                       ([0.0, 0.25, 1.0, 1.2, -0.3], True)):
        got = ss.quantiles(qs, single=single).cpu().numpy()
        exp = osx.quantiles(qs, single=single)
        assert_same_quantiles(got, exp, "eps=%g qs=%r" % (eps, qs), small_of(osx, eps))
    assert_same_state(ss, osx, "after queries")


def test_overflow_promotion(gpu_device):
    """Descending streams outgrow the 256-entry fast class and are promoted."""
    rng = np.random.default_rng(5)
    S = 40
    seqs = [np.sort(rng.random(int(L)))[::-1].copy() for L in rng.integers(20000, 60000, S)]
    seqs[0] = rng.random(3000)
    ss = _ss(S, 0.01, gpu_device)
    osx = OracleSet(S, 0.01)
    flat, offs = csr(seqs)
    ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
    osx.ingest(flat, offs)
    assert ss.num_promoted > 0
    assert_same_state(ss, osx, "promoted")
    got = ss.quantiles([0.01, 0.5, 0.99]).cpu().numpy()
    assert_same_quantiles(got, osx.quantiles([0.01, 0.5, 0.99]), "promoted q", small_of(osx, 0.01))
    # keep ingesting after promotion
    seqs2 = [rng.random(int(L)) for L in rng.integers(0, 3000, S)]
    flat, offs = csr(seqs2)
    ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
    osx.ingest(flat, offs)
    assert_same_state(ss, osx, "after promotion")


@pytest.mark.parametrize("eps", [0.1, 0.01])
def test_merge_fold_vs_oracle(gpu_device, eps):
    rng = np.random.default_rng(17)
    S, K = 300, 8
    P = int(1.0 / eps) + 1
    gsets, osets = [], []
    for k in range(K):
        lens = rng.integers(0, 10 * P, S)
        if k == 0:
            lens[:10] = 0
        seqs = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), lens)]
        flat, offs = csr(seqs)
        g = _ss(S, eps, gpu_device)
        g.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
        o = OracleSet(S, eps)
        o.ingest(flat, offs)
        gsets.append(g)
        osets.append(o)
    gsets[0].merge_from(gsets[1:])
    for o in osets[1:]:
        osets[0].merge(o)
    assert_same_state(gsets[0], osets[0], "fold")
    for g, o in zip(gsets[1:], osets[1:]):
        assert_same_tables(g, o, what="mutated source")
    got = gsets[0].quantiles([0.5, 0.9, 0.99]).cpu().numpy()
    assert_same_quantiles(got, osets[0].quantiles([0.5, 0.9, 0.99]), "fold q", small_of(osets[0], eps))


def test_export_import_roundtrip(gpu_device):
    rng = np.random.default_rng(23)
    S = 500
    seqs = [rng.lognormal(0, 1, int(L)) for L in rng.integers(0, 3000, S)]
    a = _ss(S, 0.01, gpu_device)
    ingest_np(a, seqs)
    state = a.export_state()
    b = _ss(S, 0.01, gpu_device)
    b.import_state(state)
    more = [rng.random(int(L)) for L in rng.integers(0, 500, S)]
    ingest_np(a, more)
    ingest_np(b, more)
    qa = a.quantiles([0.1, 0.5, 0.9]).cpu().numpy()
    qb = b.quantiles([0.1, 0.5, 0.9]).cpu().numpy()
    assert np.array_equal(qa.view(np.int64), qb.view(np.int64))
    ta, tb = tables_np(a), tables_np(b)
    for x, y in zip(ta, tb):
        assert np.array_equal(x, y)


def test_large_batch_properties_and_sample(gpu_device):
    """cfg3-shaped batch (200k streams x 1000 Pareto values): size-independent
    properties on every stream, exact parity on a 2,000-stream sample."""
    S, L, eps = 200_000, 1000, 0.01
    g = torch.Generator(device=gpu_device)
    g.manual_seed(3)
    u = torch.rand(S * L, dtype=torch.float64, device=gpu_device, generator=g)
    x = (1.0 - u).pow(-1.0 / 1.5)  # Pareto(1.5) + 1
    offs = torch.arange(0, S * L + 1, L, dtype=torch.int64, device=gpu_device)
    ss = _ss(S, eps, gpu_device)
    ss.ingest(x, offs)
    st = ss.stats()
    assert bool((st["n"] == L).all())
    assert bool((st["pending"] == L % 101).all())
    offs_t, v, gg, dd = ss.tables()
    # sum of g == n - pending for add-only streams; table sorted by value
    seg = torch.repeat_interleave(torch.arange(S, device=gpu_device), (offs_t[1:] - offs_t[:-1]))
    gsum = torch.zeros(S, dtype=torch.int64, device=gpu_device).index_add_(0, seg, gg.to(torch.int64))
    assert bool((gsum == L - L % 101).all())
    same_seg = seg[1:] == seg[:-1]
    assert bool((v[1:][same_seg] >= v[:-1][same_seg]).all())
    q = ss.quantiles([0.5, 0.9, 0.99])
    assert bool((q[:, 0] <= q[:, 1]).all()) and bool((q[:, 1] <= q[:, 2]).all())
    # exact parity on a sample of streams
    idx = np.random.default_rng(1).choice(S, 2000, replace=False)
    xs = x.view(S, L)[torch.from_numpy(idx).to(gpu_device)].cpu().numpy()
    o = OracleSet(len(idx), eps)
    o.ingest(xs.reshape(-1), np.arange(0, len(idx) * L + 1, L))
    oq = o.quantiles([0.5, 0.9, 0.99])
    assert_same_quantiles(q.cpu().numpy()[idx], oq, "sample quantiles", small_of(o, eps))
    offs_t, v, gg, dd = ss.tables()  # after the query flush, like the oracle's
    go, gv, ggn, gdn = offs_t.cpu().numpy(), v.cpu().numpy(), gg.cpu().numpy(), dd.cpu().numpy()
    oo, ov, og, od = o.tables()
    for k, s in enumerate(idx[:500]):
        a, b = go[s], go[s + 1]
        assert np.array_equal(gv[a:b].view(np.int64), ov[oo[k]:oo[k + 1]].view(np.int64))
        assert np.array_equal(ggn[a:b].astype(np.int64), og[oo[k]:oo[k + 1]])
        assert np.array_equal(gdn[a:b].astype(np.int64), od[oo[k]:oo[k + 1]])


def test_fused_ingest_quantiles_vs_oracle(gpu_device):
    """gk_ingest_quantiles == gk_ingest then gk_quantiles (state and answers)."""
    rng = np.random.default_rng(31)
    for eps in (0.05, 0.01):
        S = 700
        P = int(1.0 / eps) + 1
        lens = rng.integers(0, 9 * P, S)
        lens[:3] = [0, 1, P]
        seqs = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), lens)]
        flat, offs = csr(seqs)
        ss = _ss(S, eps, gpu_device)
        osx = OracleSet(S, eps)
        for qs, single in (([0.5, 0.9, 0.99], False), ([0.99, 0.1], False), ([0.0, 1.0, 2.0], True)):
            got = ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs), quantiles=qs, single=single)
            osx.ingest(flat, offs)
            exp = osx.quantiles(qs, single=single)
            assert_same_quantiles(got.cpu().numpy(), exp, "fused eps=%g qs=%r" % (eps, qs), small_of(osx, eps))
            assert_same_state(ss, osx, "fused state eps=%g" % eps)


@pytest.mark.parametrize("fused", ["0", "1", "64"])
def test_stats_role_sizes_vs_oracle(gpu_device, monkeypatch, fused):
    """The gk:52-59 stats in every layout of the small-class launch: a
    separate k_stats launch (GK_FUSED_STATS=0), one stats wave (1/8 per CU:
    the stats finish last), every resident wave (64).  Mixed histories (n
    differs inside a 64-stream batch: per-lane reciprocals) and fresh batches
    (shared n: the reciprocal table), streams past GK_STATS_LONG (k_stats_long),
    and fused quantiles that are _min/_max (k_qfix markers)."""
    monkeypatch.setenv("GK_FUSED_STATS", fused)
    rng = np.random.default_rng(47)
    eps, S = 0.01, 900
    ss = _ss(S, eps, gpu_device)
    osx = OracleSet(S, eps)
    for part in range(3):
        lens = rng.integers(0, 2500, S) if part else np.full(S, 1000)
        if part == 2:
            lens[::97] = 20000
        seqs = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), lens)]
        flat, offs = csr(seqs)
        qs = [0.0, 0.5, 0.99, 1.0]
        got = ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs), quantiles=qs)
        osx.ingest(flat, offs)
        assert_same_quantiles(got.cpu().numpy(), osx.quantiles(qs), "stats role %s part %d" % (fused, part),
                              small_of(osx, eps))
        assert_same_state(ss, osx, "stats role %s part %d" % (fused, part))


def test_long_stream_stats(gpu_device):
    """Streams longer than GK_STATS_LONG (16384) take k_stats_long: _sum/_avg
    chain and first-occurrence _min/_max (signed zeros) across calls."""
    rng = np.random.default_rng(41)
    lens = [16385, 20000, 70001, 100, 0, 33333]
    dists = [6, 1, 6, 6, 0, 7]
    S = len(lens)
    for eps in (0.01, 0.001):
        ss = _ss(S, eps, gpu_device)
        osx = OracleSet(S, eps)
        for part in range(2):
            seqs = [gen(d, L // (part + 1), rng) for d, L in zip(dists, lens)]
            flat, offs = csr(seqs)
            ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
            osx.ingest(flat, offs)
            assert_same_state(ss, osx, "long eps=%g part %d" % (eps, part))
        got = ss.quantiles([0.5, 0.9, 0.99]).cpu().numpy()
        assert_same_quantiles(got, osx.quantiles([0.5, 0.9, 0.99]), "long q eps=%g" % eps, small_of(osx, eps))


def test_fused_query_long_streams_beside_stats(gpu_device):
    """Long streams (> GK_STATS_LONG values) walk their _sum/_avg chains on a
    second HIP stream beside the ingest launch, which takes them longest
    first; the fused query is re-answered for them once _min/_max are final
    (q = 1.0 returns _max, gk:229).  Lengths are distinct and unordered so the
    longest-first hand-out differs from stream order."""
    rng = np.random.default_rng(43)
    for eps in (0.01, 0.005, 0.001):
        S = 48
        lens = rng.integers(0, 3000, S)
        lens[rng.choice(S, 9, replace=False)] = [16385, 40000, 17000, 90001, 25000, 60000, 16384, 33000, 70000]
        dists = rng.integers(0, 8, S)
        ss = _ss(S, eps, gpu_device)
        osx = OracleSet(S, eps)
        for part, (qs, single) in enumerate((([0.0, 0.5, 0.99, 1.0], False), ([1.0, 0.25], False),
                                             ([0.5, 1.0], True))):
            seqs = [gen(int(d), int(L) // (part + 1), rng) for d, L in zip(dists, lens)]
            flat, offs = csr(seqs)
            got = ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs), quantiles=qs, single=single)
            osx.ingest(flat, offs)
            exp = osx.quantiles(qs, single=single)
            assert_same_quantiles(got.cpu().numpy(), exp, "long fused eps=%g part %d" % (eps, part),
                                  small_of(osx, eps))
            assert_same_state(ss, osx, "long fused state eps=%g part %d" % (eps, part))
        # plain ingest (no query) of long streams, then stats read right away
        seqs = [gen(int(d), int(L), rng) for d, L in zip(dists, lens)]
        flat, offs = csr(seqs)
        ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
        osx.ingest(flat, offs)
        assert_same_state(ss, osx, "long plain eps=%g" % eps)


def test_many_long_streams_grouped_stats(gpu_device):
    """More long streams than GK_SL_BCAST (1024): k_stats_long walks them 64
    per wave, one per lane (register ring of aligned 16-byte loads, one value
    peeled when a stream starts off 16-byte alignment).  Odd lengths make the
    starts alternate alignment; two calls carry n, min, max, sum, avg."""
    rng = np.random.default_rng(47)
    S = 1100
    for part in range(2):
        lens = rng.integers(16385, 19000, S) if part == 0 else rng.integers(16385, 17000, S)
        if part == 0:
            ss = _ss(S, 0.01, gpu_device)
            osx = OracleSet(S, 0.01)
        seqs = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), lens)]
        flat, offs = csr(seqs)
        got = ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs), quantiles=[0.5, 1.0])
        osx.ingest(flat, offs)
        assert_same_quantiles(got.cpu().numpy(), osx.quantiles([0.5, 1.0]), "grouped long q part %d" % part,
                              small_of(osx, 0.01))
        assert_same_state(ss, osx, "grouped long state part %d" % part)


def test_many_long_streams_uniform_n_stats(gpu_device):
    """Equal-length long streams (cfg4's rows): every lane of a k_stats_long
    group starts at the same n, so the gk:54 factors 1.0/n come from a
    64-entry LDS tile per 4 chunks instead of per-lane divisions.  1100
    streams (the last group 12 lanes), three calls (n carried), then a call
    whose lengths differ per stream (the per-lane path after the tile path)."""
    rng = np.random.default_rng(59)
    S = 1100
    ss = _ss(S, 0.01, gpu_device)
    osx = OracleSet(S, 0.01)
    for part, L in enumerate([16400, 16448, 20000, None]):
        lens = [L] * S if L else list(rng.integers(16385, 17000, S))
        seqs = [gen(int(d), int(n), rng) for d, n in zip(rng.integers(0, 8, S), lens)]
        flat, offs = csr(seqs)
        got = ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs), quantiles=[0.5, 1.0])
        osx.ingest(flat, offs)
        assert_same_quantiles(got.cpu().numpy(), osx.quantiles([0.5, 1.0]), "uniform long q part %d" % part,
                              small_of(osx, 0.01))
        assert_same_state(ss, osx, "uniform long state part %d" % part)


@pytest.mark.parametrize("eps", [0.05, 0.01, 0.001])
def test_merge_compress_records_vs_oracle(gpu_device, eps):
    """merge_compress(entries) with explicit (v, g, delta) records (gk:63-109):
    arbitrary g and delta exercise every rule of the wave-parallel walk
    (absorption by the running g, the removal carry, the tail chain), with
    pending values, ties between records and entries, and empty sides."""
    from gk_oracle import OracleGK
    rng = np.random.default_rng(53 + int(1 / eps))
    S = 240
    P = int(1.0 / eps) + 1
    lens = rng.integers(0, 4 * P, S)
    lens[:4] = [0, 1, P, P + 7]
    seqs = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), lens)]
    ss = _ss(S, eps, gpu_device)
    ingest_np(ss, seqs)
    ors = []
    for sq in seqs:
        o = OracleGK(eps)
        o.add_many(sq)
        ors.append(o)
    vals, gs, ds, offs = [], [], [], [0]
    recs_all = []
    for s in range(S):
        k = int(rng.integers(0, 60))
        if s % 7 == 0:
            k = 0
        base = seqs[s] if len(seqs[s]) else rng.random(4)
        v = np.sort(np.concatenate([rng.choice(base, size=k // 2), rng.lognormal(0, 1, k - k // 2)]))
        g = rng.integers(1, 3 + int(0.02 / eps), k)
        d = rng.integers(0, 2 + int(0.04 / eps), k)
        recs = list(zip(v.tolist(), g.tolist(), d.tolist()))
        recs_all.append(recs)
        vals += v.tolist(); gs += g.tolist(); ds += d.tolist(); offs.append(offs[-1] + k)
    ss.merge_compress(torch.tensor(vals, dtype=torch.float64), torch.tensor(gs, dtype=torch.int32),
                      torch.tensor(ds, dtype=torch.int32), torch.tensor(offs, dtype=torch.int64))
    to, tv, tg, td = (t.cpu() for t in ss.tables())
    for s in range(S):
        ors[s].flush(recs_all[s])
        a, b = int(to[s]), int(to[s + 1])
        got = list(zip(tv[a:b].tolist(), tg[a:b].tolist(), td[a:b].tolist()))
        assert got == ors[s].table(), "stream %d eps=%g" % (s, eps)
