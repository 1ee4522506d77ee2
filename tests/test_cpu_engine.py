"""The host engine (libgkarray_cpu.so, include/gk_cpu.h) -- SURVEY 8(f) rank 4:
the whole reference path (gk:19-232) on host threads, selected explicitly with
StreamSet(..., device="cpu").  Same bar as the GPU: bit-exact against the
goldens made by the reference and against the C oracle (which it does not
share code with), plus the cases the HIP engine bounds (tiny eps, huge tables).
These run without a GPU."""
import numpy as np
import pytest
import torch

import golden_io as G
from gk_oracle_c import OracleSet
from parity_util import (_ss, assert_same_quantiles, assert_same_state, assert_same_tables, check_golden_merge_plans, csr,
                         gen, ingest_np,
                         golden_mask, small_of)

CPU = "cpu"


def test_golden_streams_cpu():
    by_eps = {}
    for c in G.cases("stream"):
        by_eps.setdefault(c["eps"], []).append(c)
    for eps, cs in by_eps.items():
        ss = _ss(len(cs), eps, CPU)
        ingest_np(ss, [G.get(c["id"], "x") for c in cs])
        for k, c in enumerate(cs):
            assert G.same_table(ss.table(k), G.tables(c["id"], "auto")[0]), c
        poffs, pv = ss.pending()
        st = {k: v.numpy() for k, v in ss.stats().items()}
        for k, c in enumerate(cs):
            assert np.array_equal(pv[poffs[k]:poffs[k + 1]].numpy().view(np.int64),
                                  G.get(c["id"], "pending").view(np.int64)), c
            got = [st["n"][k], st["min"][k], st["max"][k], st["sum"][k], st["avg"][k]]
            assert all(G.same_float(a, b) for a, b in zip(got, G.get(c["id"], "stats_before_query"))), c
        um = lambda k, c, qs: golden_mask(G.tables(c["id"], "final")[0], st["n"][k], eps, qs)  # noqa: E731
        q = ss.quantiles(G.index()["qs"], single=True).numpy()
        for k, c in enumerate(cs):
            assert_same_quantiles(q[k], G.get(c["id"], "q_single"), "quantile %r" % c, um(k, c, G.index()["qs"]))
            assert G.same_table(ss.table(k), G.tables(c["id"], "final")[0]), c
        q = ss.quantiles(G.index()["qs"]).numpy()
        q2 = ss.quantiles(G.index()["qs_unsorted"]).numpy()
        q3 = ss.quantiles(G.index()["qs_oor"]).numpy()
        for k, c in enumerate(cs):
            assert_same_quantiles(q[k], G.get(c["id"], "q_sorted"), "quantiles %r" % c, um(k, c, G.index()["qs"]))
            assert_same_quantiles(q2[k], G.get(c["id"], "q_unsorted"), "unsorted %r" % c, um(k, c, G.index()["qs_unsorted"]))
            assert_same_quantiles(q3[k], G.get(c["id"], "q_oor"), "oor %r" % c, um(k, c, G.index()["qs_oor"]))


def test_per_flush_golden_snapshots_cpu():
    checked = 0
    for c in G.cases("stream"):
        if not G.has(c["id"], "flush/sizes"):
            continue
        eps = c["eps"]
        P = int(1.0 / eps) + 1
        xs = G.get(c["id"], "x")
        exp = G.tables(c["id"], "flush")
        ss = _ss(1, eps, CPU)
        for f, t in enumerate(exp):
            ingest_np(ss, [xs[f * P:(f + 1) * P]])
            assert G.same_table(ss.table(0), t), (c, f)
            checked += 1
    assert checked > 3000


def test_golden_merges_and_query_mid_cpu():
    for c in G.cases("merge"):
        cid, eps = c["id"], c["eps"]
        sets = []
        for xs in G.shards(cid):
            ss = _ss(1, eps, CPU)
            ingest_np(ss, [xs])
            sets.append(ss)
        steps = G.tables(cid, "merge_steps")
        others = G.tables(cid, "others_after")
        for k, o in enumerate(sets[1:]):
            sets[0].merge_from([o])
            assert G.same_table(sets[0].table(0), steps[k]), (c, k)
            assert G.same_table(o.table(0), others[k]), (c, k)
        st = {k: v.numpy() for k, v in sets[0].stats().items()}
        got = [st["n"][0], st["min"][0], st["max"][0], st["sum"][0], st["avg"][0]]
        assert all(G.same_float(a, b) for a, b in zip(got, G.get(cid, "merged_stats"))), c
        assert_same_quantiles(sets[0].quantiles(G.index()["qs"]).numpy()[0], G.get(cid, "merged_q"), c,
                              golden_mask(steps[-1], st["n"][0], eps, G.index()["qs"]))
    for c in G.cases("query_mid"):
        cid, eps = c["id"], c["eps"]
        xs = G.get(cid, "x")
        pts = [int(p) for p in G.get(cid, "query_points")]
        ss = _ss(1, eps, CPU)
        prev = 0
        for k, p in enumerate(pts):
            ingest_np(ss, [xs[prev:p]])
            assert_same_quantiles(ss.quantiles([0.1, 0.5, 0.9]).numpy()[0], G.get(cid, "mid_q")[k], c,
                                  golden_mask(G.tables(cid, "mid_tables")[k], p, eps, [0.1, 0.5, 0.9]))
            prev = p


def test_golden_merge_plans_cpu():
    """a.merge(a) and repeated sources (gk:111-154) against the reference."""
    assert check_golden_merge_plans(CPU) == len(G.cases("merge_plan")) > 100


def test_dropin_self_merge_cpu():
    from gkarray_amd import GKArray
    from gk_oracle import OracleGK
    rng = np.random.default_rng(7)
    xs = rng.lognormal(0, 1, 1234)
    sk, o = GKArray(0.01, device=CPU), OracleGK(0.01)
    for x in xs:
        sk.add(x)
    o.add_many(xs)
    sk.merge(sk)
    o.merge(o)
    assert sk._n == o.n == 2468
    assert [(e.val, e.g, e.delta) for e in sk.entries] == o.table()
    assert sk.quantiles([.5, .9]) == o.quantiles([.5, .9])


@pytest.mark.parametrize("eps", [0.2, 0.05, 0.03, 0.015, 0.01, 0.001, 0.0005, 0.0002])
def test_random_batches_vs_oracle_cpu(eps):
    """Three ingest chunks per stream (flush points straddle calls), sorted /
    unsorted / out-of-range queries; eps below 1/1023 too (no limit here)."""
    rng = np.random.default_rng(int(eps * 1e6) + 101)
    P = int(1.0 / eps) + 1
    S = 400 if eps >= 0.01 else 40
    lens = rng.integers(0, 8 * P, S)
    lens[:4] = [0, 1, P, P - 1]
    seqs = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), lens)]
    ss = _ss(S, eps, CPU)
    o = OracleSet(S, eps)
    cuts = [np.sort(rng.integers(0, max(len(x), 1) + 1, 2)) for x in seqs]
    for part in range(3):
        piece = [x[(0 if part == 0 else int(c[part - 1])):(int(c[part]) if part < 2 else len(x))]
                 for x, c in zip(seqs, cuts)]
        flat, offs = csr(piece)
        ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
        o.ingest(flat, offs)
        assert_same_state(ss, o, "cpu eps=%g part %d" % (eps, part))
    for qs, single in (([0.5, 0.9, 0.99], False), ([0.99, 0.1, 0.5], False), ([0.0, 0.25, 1.0, 1.2, -0.3], True)):
        assert_same_quantiles(ss.quantiles(qs, single=single).numpy(), o.quantiles(qs, single=single),
                              "cpu eps=%g qs=%r" % (eps, qs), small_of(o, eps))
    assert_same_state(ss, o, "after queries")


def test_huge_tables_and_fused_query_cpu():
    """Descending streams (tables far past the GPU's LDS classes) and the
    fused ingest + quantiles call."""
    rng = np.random.default_rng(7)
    S = 12
    seqs = [np.sort(rng.random(int(L)))[::-1].copy() for L in rng.integers(100000, 300000, S)]
    flat, offs = csr(seqs)
    ss = _ss(S, 0.001, CPU)
    o = OracleSet(S, 0.001)
    q = ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs), quantiles=[0.01, 0.5, 0.99])
    o.ingest(flat, offs)
    assert_same_quantiles(q.numpy(), o.quantiles([0.01, 0.5, 0.99]), "fused", small_of(o, 0.001))
    assert_same_state(ss, o, "huge")
    assert int(ss.stats()["size"].max()) > 2048


@pytest.mark.parametrize("eps", [0.1, 0.01])
def test_merge_fold_and_records_vs_oracle_cpu(eps):
    rng = np.random.default_rng(17)
    S, K = 200, 8
    P = int(1.0 / eps) + 1
    gs, os_ = [], []
    for k in range(K):
        lens = rng.integers(0, 10 * P, S)
        if k == 0:
            lens[:10] = 0
        seqs = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), lens)]
        flat, offs = csr(seqs)
        g = _ss(S, eps, CPU)
        g.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
        o = OracleSet(S, eps)
        o.ingest(flat, offs)
        gs.append(g)
        os_.append(o)
    gs[0].merge_from(gs[1:])
    for o in os_[1:]:
        os_[0].merge(o)
    assert_same_state(gs[0], os_[0], "cpu fold")
    for g, o in zip(gs[1:], os_[1:]):
        assert_same_tables(g, o, what="mutated source")


def test_threads_do_not_change_results():
    rng = np.random.default_rng(5)
    S = 3000
    seqs = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), rng.integers(0, 3000, S))]
    flat, offs = csr(seqs)
    a, b = _ss(S, 0.01, CPU), _ss(S, 0.01, CPU)
    a.set_threads(1)
    b.set_threads(8)
    qa = a.ingest(torch.from_numpy(flat), torch.from_numpy(offs), quantiles=[0.5, 0.99]).numpy()
    qb = b.ingest(torch.from_numpy(flat), torch.from_numpy(offs), quantiles=[0.5, 0.99]).numpy()
    assert np.array_equal(qa.view(np.int64), qb.view(np.int64))
    for x, y in zip(a.tables(), b.tables()):
        assert torch.equal(x, y)


def test_state_files_cpu(tmp_path):
    from gkarray_amd import StreamSet, stateio
    rng = np.random.default_rng(9)
    S = 300
    seqs = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), rng.integers(0, 2000, S))]
    ss = _ss(S, 0.01, CPU)
    ingest_np(ss, seqs)
    p = str(tmp_path / "cpu.gks")
    ss.save(p)
    r = stateio.read_state(p)
    st = ss.export_state()
    for k in ("offs", "v", "g", "d", "poffs", "pv", "n", "min", "max", "sum", "avg"):
        assert np.array_equal(np.asarray(r[k]).view(np.uint8), st[k].numpy().astype(r[k].dtype).view(np.uint8)), k
    b = StreamSet.load(p, device=CPU)
    more = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), rng.integers(0, 2000, S))]
    ingest_np(ss, more)
    ingest_np(b, more)
    for x, y in zip(ss.tables(), b.tables()):
        assert torch.equal(x, y)


def test_drop_in_gkarray_cpu():
    from gkarray_amd import GKArray, UnequalEpsilonException
    kat = G.index()["kat"]
    sk = GKArray(0.1, device=CPU)
    xs = [float((7 * i) % 23) for i in range(40)]
    for x in xs[:33]:
        sk.add(x)
    assert [(e.val, e.g, e.delta) for e in sk.entries] == [tuple(r) for r in kat["kat1_table_after_33"]]
    for x in xs[33:]:
        sk.add(x)
    assert sk.quantiles([0, .25, .5, .75, 1]) == [0, 5, 10, 19, 22]
    sk = GKArray(0.1, device=CPU)
    for x in [3.0, 1.0, 2.0]:
        sk.add(x)
    assert sk.quantile(.5) == 2.0 and sk.quantile(.25) == 1.5
    with pytest.raises(UnequalEpsilonException):
        sk.merge(GKArray(0.2, device=CPU))
    big = GKArray(0.01, device=CPU)
    big.add_many(np.random.default_rng(0).random(1_000_000))
    assert big.quantiles([.5, .9, .99]) == kat["kat3_quantiles"]
    assert big.size() == kat["kat3_size"]
    assert [big._n, big._min, big._max, big._sum, big._avg] == kat["kat3_stats"]
    tiny = GKArray(0.0005, device=CPU)  # flush period 2001
    tiny.add_many(np.arange(5000.0)[::-1])
    assert tiny.size() > 0 and tiny.num_values() == 5000


def test_cpu_symbols_match_headers():
    import ctypes
    import os
    import re
    from gkarray_amd import _lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    names = set()
    for h in ("gk_capi.h", "gk_cpu.h"):
        src = re.sub(r"/\*.*?\*/", "", open(os.path.join(root, "include", h)).read(), flags=re.S)
        names |= set(re.findall(r"\b(gk_[a-z_]+)\s*\(", src))
    assert sorted(_lib.CPU_SYMBOLS) == sorted(names)
    lib = ctypes.CDLL(_lib.CPU_LIB_PATH)
    assert all(hasattr(lib, n) for n in names)
    data = open(_lib.CPU_LIB_PATH, "rb").read()
    assert b"gko_" not in data  # independent of the oracle


def test_packed_state_round_trip_and_fold():
    """gk_pack / gk_fold_packed on the host engine: a packed state restores
    bit-exactly (fold of one buffer), a 3-way fold equals the oracle's left
    fold, and mismatched eps / stream counts are refused."""
    from gkarray_amd import StreamSet, UnequalEpsilonException
    from gkarray_amd._lib import GKBackendError
    rng = np.random.default_rng(17)
    eps, S = 0.01, 25
    sets, oracles = [], []
    for k in range(3):
        seqs = [gen(int(rng.integers(0, 8)), int(rng.integers(0, 900)), rng) for _ in range(S)]
        flat, offs = csr(seqs)
        ss = StreamSet(S, eps, device=CPU)
        ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
        o = OracleSet(S, eps)
        o.ingest(flat, offs)
        sets.append(ss)
        oracles.append(o)
    bufs = [s.pack() for s in sets]
    assert bufs[0].numel() == sets[0].pack_bytes()
    one = StreamSet(S, eps, device=CPU)
    one.fold_packed(bufs[:1])
    assert_same_state(one, oracles[0], "restored")
    big = torch.zeros(bufs[1].numel() + 4096, dtype=torch.uint8)  # padded slot
    sets[1].pack(big)
    dst = StreamSet(S, eps, device=CPU)
    dst.fold_packed([bufs[0], big, bufs[2]])
    oracles[0].merge(oracles[1])
    oracles[0].merge(oracles[2])
    assert_same_state(dst, oracles[0], "3-way fold")
    with pytest.raises(UnequalEpsilonException):
        StreamSet(S, 0.02, device=CPU).fold_packed(bufs[:1])
    with pytest.raises(GKBackendError):
        StreamSet(S + 1, eps, device=CPU).fold_packed(bufs[:1])
    with pytest.raises(GKBackendError):
        sets[0].pack(torch.zeros(16, dtype=torch.uint8))


def test_packed_state_corrupt_header_and_offsets_refused():
    """a packed buffer whose header sizes / byte count or
    offset arrays are inconsistent is refused before gk_import reads it."""
    from gkarray_amd import StreamSet
    from gkarray_amd._lib import GKBackendError
    rng = np.random.default_rng(18)
    eps, S = 0.01, 12
    seqs = [gen(int(rng.integers(0, 8)), int(rng.integers(1, 500)), rng) for _ in range(S)]
    flat, offs = csr(seqs)
    ss = StreamSet(S, eps, device=CPU)
    ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
    good = ss.pack()
    StreamSet(S, eps, device=CPU).fold_packed([good])  # sanity: the intact buffer folds
    hdr = good[:64].numpy().view(np.int64)  # magic, version|hbytes, eps, S, E, P, bytes, reserved
    for field, val in ((4, -1), (4, int(hdr[4]) + 1), (5, -3), (6, int(hdr[6]) - 256)):
        bad = good.clone()
        bad[:64].numpy().view(np.int64)[field] = val
        with pytest.raises(GKBackendError):
            StreamSet(S, eps, device=CPU).fold_packed([bad])
    # a non-monotone table offset array (section at 256-aligned offset after 5 header arrays)
    sec = lambda nbytes: (nbytes + 255) // 256 * 256
    eoffs_at = 256 + 5 * sec(8 * S)
    bad = good.clone()
    eo = bad[eoffs_at:eoffs_at + 8 * (S + 1)].numpy().view(np.int64)
    eo[3], eo[4] = eo[4] + 1, eo[3]
    with pytest.raises(GKBackendError, match="offsets"):
        StreamSet(S, eps, device=CPU).fold_packed([bad])


def test_import_rejects_unreachable_pending_cpu():
    """pending counts above n mod P are refused by the host
    engine's import too (and by the drop-in's incoming assignment)."""
    from gkarray_amd import GKArray, StreamSet
    from gkarray_amd._lib import GKBackendError
    eps, S = 0.01, 3
    P = int(1 / eps) + 1
    rng = np.random.default_rng(19)
    seqs = [rng.random(2 * P + 4) for _ in range(S)]
    flat, offs = csr(seqs)
    ss = StreamSet(S, eps, device=CPU)
    ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
    st = ss.export_state()
    bad = dict(st)
    bad["poffs"] = torch.tensor([0, 4, 14, 18], dtype=torch.int64)  # 10 pending at n mod P = 4
    bad["pv"] = torch.rand(18, dtype=torch.float64)
    with pytest.raises(GKBackendError, match="pending"):
        ss.import_state(bad)
    sk = GKArray(eps, device=CPU)
    for x in rng.random(P):  # n = P: just flushed, nothing can be pending
        sk.add(float(x))
    with pytest.raises(ValueError, match="pending"):
        sk.incoming = [0.5] * 28
        sk.size()
    sk2 = GKArray(eps, device=CPU)
    for x in rng.random(P + 30):
        sk2.add(float(x))
    sk2.incoming = [0.25] * 30  # n mod P = 30: allowed
    assert sk2.size() > 0
