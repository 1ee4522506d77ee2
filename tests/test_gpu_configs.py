"""Parity at the BASELINE.json workloads, by config name, plus the reference's
per-flush table snapshots.

* test_per_flush_golden_snapshots: every golden stream that carries the table
  after EACH automatic flush (tests/golden/make_golden.py, gk:60-61 -> gk:63-109)
  is ingested one flush period P at a time; after every call the HIP table must
  equal the reference's table after that flush.
* cfg2 / cfg3: the whole batch (10^9 values) against the C oracle (pinned by
  test_oracle_golden.py): every table, every stat and every quantile bit-exact,
  plus size-independent properties.  cfg3 also re-runs after reset().
* cfg4: 10k streams x 1M values cut into 8 row shards of 125k and folded with
  merge (gk:111-154) in shard order; the fold of 256 streams is checked against
  the oracle's fold (state, mutated sources, quantiles).
* cfg5: Zipf lengths (1..10^7) at eps = 0.001: the 10^7-value stream and 2,000
  sampled streams exact, size-independent properties on all 100k.

Tolerance: bit-exact (quantiles: the signed-zero allowance applies only to
n < 1/eps, parity_util.same_q).
"""
import time

import numpy as np
import pytest
import torch

import golden_io as G
from gk_oracle_c import OracleSet
from parity_util import _ss, assert_same_quantiles, small_of

pytestmark = pytest.mark.gpu

QS = [0.5, 0.9, 0.99]


def log(*a):
    print("[%s]" % time.strftime("%H:%M:%S"), *a, flush=True)


def gpu_pareto(S, L, seed, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    u = torch.rand(S * L, dtype=torch.float64, device=dev, generator=g)
    x = (1.0 - u).pow_(-1.0 / 1.5)  # numpy pareto(1.5) + 1 by inversion (bench.py)
    del u
    return x, torch.arange(0, S * L + 1, L, dtype=torch.int64, device=dev)


def gpu_lognormal(N, seed, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    return torch.randn(N, dtype=torch.float64, device=dev, generator=g).exp_()


def gpu_state(ss):
    offs, v, g, d = ss.tables()
    st = {k: t.cpu().numpy() for k, t in ss.stats().items()}
    return (offs.cpu().numpy(), v.cpu().numpy(), g.cpu().numpy().astype(np.int64),
            d.cpu().numpy().astype(np.int64)), st


def subset_csr(csr, idx):
    """Tables of streams idx (in that order) out of a CSR export."""
    o, v, g, d = csr
    idx = np.asarray(idx, np.int64)
    lens = o[idx + 1] - o[idx]
    sel = np.concatenate([np.arange(o[s], o[s + 1]) for s in idx]) if idx.size else np.zeros(0, np.int64)
    so = np.zeros(idx.size + 1, np.int64)
    so[1:] = np.cumsum(lens)
    return so, v[sel], g[sel], d[sel]


def assert_csr_equal(a, b, what):
    ao, av, ag, ad = a
    bo, bv, bg, bd = b
    if not np.array_equal(ao, bo):
        s = int(np.nonzero(np.diff(ao) != np.diff(bo))[0][0])
        raise AssertionError("%s: table size of stream %d: %d vs %d" % (what, s, ao[s + 1] - ao[s], bo[s + 1] - bo[s]))
    for name, x, y in (("v", av.view(np.int64), bv.view(np.int64)), ("g", ag, bg), ("d", ad, bd)):
        if not np.array_equal(x, y):
            i = int(np.nonzero(x != y)[0][0])
            s = int(np.searchsorted(ao, i, side="right") - 1)
            raise AssertionError("%s: %s differs at record %d (stream %d)" % (what, name, i, s))


def assert_stats_equal(st, ost, what, idx=None):
    for k in ("n", "size", "pending"):
        a = st[k] if idx is None else st[k][idx]
        assert np.array_equal(a.astype(np.int64), ost[k].astype(np.int64)), "%s %s" % (what, k)
    for k in ("min", "max", "sum", "avg"):
        a = st[k] if idx is None else st[k][idx]
        bad = np.nonzero(a.view(np.int64) != ost[k].view(np.int64))[0]
        assert bad.size == 0, "%s %s: %d streams differ, first %d: %r vs %r" % (
            what, k, bad.size, bad[0], a[bad[0]], ost[k][bad[0]])


def assert_properties(csr, st, lens, what, merged=False):
    """Size-independent properties of every stream: n, pending = n mod P for
    add-only streams, sum(g) = n - pending (not after a merge),
    values sorted, delta >= 0, g >= 1."""
    o, v, g, d = csr
    S = o.size - 1
    assert np.array_equal(st["n"].astype(np.int64), np.asarray(lens, np.int64)), what + " n"
    seg = np.repeat(np.arange(S), np.diff(o))
    if not merged:
        gs = np.bincount(seg, weights=g.astype(np.float64), minlength=S)
        assert np.array_equal(gs.astype(np.int64), st["n"] - st["pending"]), what + " sum(g) = n - pending"
    same = seg[1:] == seg[:-1]
    assert bool(np.all(v[1:][same] >= v[:-1][same])), what + " sorted"
    assert bool(np.all(g >= 1)) and bool(np.all(d >= 0)), what + " g >= 1, delta >= 0"


# ----------------------------------------------------------------------------
def test_per_flush_golden_snapshots(gpu_device):
    """Table after every automatic flush == the reference's (golden flush/*)."""
    by_eps = {}
    for c in G.cases("stream"):
        if G.has(c["id"], "flush/sizes"):
            by_eps.setdefault(c["eps"], []).append(c)
    checked = 0
    for eps, cs in sorted(by_eps.items()):
        P = int(1.0 / eps) + 1  # gk:60
        xs = [G.get(c["id"], "x") for c in cs]
        exp = [G.tables(c["id"], "flush") for c in cs]
        for k, c in enumerate(cs):
            assert [int(n) for n in G.get(c["id"], "flush_n")] == [(i + 1) * P for i in range(len(exp[k]))]
        ss = _ss(len(cs), eps, gpu_device)
        nflush = max(len(e) for e in exp)
        for f in range(nflush + 1):
            piece = [x[f * P:(f + 1) * P] for x in xs]
            offs = np.zeros(len(cs) + 1, np.int64)
            offs[1:] = np.cumsum([len(p) for p in piece])
            flat = np.concatenate(piece) if offs[-1] else np.zeros(0)
            ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
            if f == nflush:
                break
            to, tv, tg, td = (t.cpu().numpy() for t in ss.tables())
            for k in range(len(cs)):
                if f < len(exp[k]):
                    got = list(zip(tv[to[k]:to[k + 1]].tolist(), tg[to[k]:to[k + 1]].tolist(),
                                   td[to[k]:to[k + 1]].tolist()))
                    assert G.same_table(got, exp[k][f]), "case %d eps=%g flush %d" % (cs[k]["id"], eps, f)
                    checked += 1
        for k, c in enumerate(cs):
            assert G.same_table(ss.table(k), G.tables(c["id"], "auto")[0]), c
        log("eps=%g: %d streams, %d flushes" % (eps, len(cs), nflush))
    assert checked > 3000


def test_cfg3_full_batch_vs_oracle(gpu_device):
    """cfg3: 1,000,000 streams x 1,000 Pareto(1.5)+1 values, eps=0.01 -- the
    bench step (reset + fused ingest + quantiles) checked on EVERY stream."""
    S, L, eps = 1_000_000, 1000, 0.01
    x, offs = gpu_pareto(S, L, 3, gpu_device)
    ss = _ss(S, eps, gpu_device)
    q1 = ss.ingest(x, offs, quantiles=QS).cpu().numpy()
    ss.reset()
    q = ss.ingest(x, offs, quantiles=QS).cpu().numpy()
    assert np.array_equal(q1.view(np.int64), q.view(np.int64)), "reset + re-run differs"
    csr, st = gpu_state(ss)
    assert_properties(csr, st, np.full(S, L), "cfg3")
    log("gpu done")
    xh, oh = x.cpu().numpy(), offs.cpu().numpy()
    del x
    o = OracleSet(S, eps)
    o.ingest(xh, oh)
    oq = o.quantiles(QS)
    log("oracle done")
    assert_same_quantiles(q, oq, "cfg3 quantiles", small_of(o, eps))
    assert_stats_equal(st, o.stats(), "cfg3")
    assert_csr_equal(csr, o.tables(), "cfg3 tables")


def test_cfg2_full_batch_vs_oracle(gpu_device):
    """cfg2: 100,000 streams x 10,000 lognormal(0,1) values, eps=0.01, every
    stream exact (tables after the query flush, stats, quantiles)."""
    S, L, eps = 100_000, 10_000, 0.01
    x = gpu_lognormal(S * L, 2, gpu_device)
    offs = torch.arange(0, S * L + 1, L, dtype=torch.int64, device=gpu_device)
    ss = _ss(S, eps, gpu_device)
    ss.ingest(x, offs)
    csr0, st0 = gpu_state(ss)
    assert_properties(csr0, st0, np.full(S, L), "cfg2 after ingest")
    q = ss.quantiles(QS).cpu().numpy()
    csr, st = gpu_state(ss)
    log("gpu done")
    xh, oh = x.cpu().numpy(), offs.cpu().numpy()
    del x
    o = OracleSet(S, eps)
    o.ingest(xh, oh)
    assert_stats_equal(st0, o.stats(), "cfg2 before query")
    assert_csr_equal(csr0, o.tables(), "cfg2 tables before query")
    oq = o.quantiles(QS)
    log("oracle done")
    assert_same_quantiles(q, oq, "cfg2 quantiles", small_of(o, eps))
    assert_stats_equal(st, o.stats(), "cfg2")
    assert_csr_equal(csr, o.tables(), "cfg2 tables")


def test_stats_role_mixed_history_many_batches(gpu_device):
    """The stats role of the small-class launch reads each stream's pre-call n
    while ingest waves of the same launch rewrite n: far more 64-stream
    batches (3,125) than stats waves, histories that differ per stream, and
    the fewest stats waves (GK_FUSED_STATS=1) so that most streams are
    committed before their stats batch runs (_avg depends on n, gk:54)."""
    import os
    S, eps = 200_000, 0.01
    rng = np.random.default_rng(61)
    for fused in ("1", "7"):
        os.environ["GK_FUSED_STATS"] = fused
        try:
            ss = _ss(S, eps, gpu_device)
        finally:
            del os.environ["GK_FUSED_STATS"]
        o = OracleSet(S, eps)
        for part in range(2):
            lens = rng.integers(0, 1500, S) if part == 0 else np.full(S, 1000)
            offs = np.zeros(S + 1, np.int64)
            offs[1:] = np.cumsum(lens)
            flat = rng.lognormal(0, 1, int(offs[-1]))
            ss.ingest(torch.from_numpy(flat).to(gpu_device), torch.from_numpy(offs).to(gpu_device))
            o.ingest(flat, offs)
            csr, st = gpu_state(ss)
            assert_stats_equal(st, o.stats(), "fused=%s part %d" % (fused, part))
            assert_csr_equal(csr, o.tables(), "fused=%s part %d" % (fused, part))


def test_cfg4_row_shards_fold_vs_oracle(gpu_device):
    """cfg4: 10,000 streams x 1,000,000 lognormal values in 8 row shards of
    125,000 values per stream; every shard sketched on the GPU, then
    sk0.merge(sk1)...merge(sk7) (gk:111-154) for all streams; 256 streams
    checked against the oracle's fold, the rest by properties."""
    S, L, K, eps = 10_000, 1_000_000, 8, 0.01
    Lk = L // K
    idx = np.sort(np.random.default_rng(4).choice(S, 256, replace=False))
    idx_t = torch.from_numpy(idx).to(gpu_device)
    sets, osets = [], []
    offs = torch.arange(0, S * Lk + 1, Lk, dtype=torch.int64, device=gpu_device)
    o_sub = np.arange(0, idx.size * Lk + 1, Lk, dtype=np.int64)
    for k in range(K):
        x = gpu_lognormal(S * Lk, 40 + k, gpu_device)
        ss = _ss(S, eps, gpu_device)
        ss.ingest(x, offs)
        sets.append(ss)
        xs = x.view(S, Lk)[idx_t].cpu().numpy().reshape(-1)
        del x
        o = OracleSet(idx.size, eps)
        o.ingest(xs, o_sub)
        osets.append(o)
    log("shards sketched")
    sets[0].merge_from(sets[1:])
    for o in osets[1:]:
        osets[0].merge(o)
    log("folded")
    csr, st = gpu_state(sets[0])
    assert_properties(csr, st, np.full(S, L), "cfg4 fold", merged=True)
    assert_stats_equal(st, osets[0].stats(), "cfg4 fold", idx)
    assert_csr_equal(subset_csr(csr, idx), osets[0].tables(), "cfg4 fold tables")
    for k in range(1, K):  # merge flushes (mutates) each source, gk:126, 137
        c, _ = gpu_state(sets[k])
        assert_csr_equal(subset_csr(c, idx), osets[k].tables(), "cfg4 source %d" % k)
    q = sets[0].quantiles(QS).cpu().numpy()
    assert_same_quantiles(q[idx], osets[0].quantiles(QS), "cfg4 quantiles", small_of(osets[0], eps))
    for s in sets:
        s.close()


def test_cfg5_zipf_lengths_vs_oracle(gpu_device):
    """cfg5: 100,000 streams, lengths clip(zipf(1.5), 1, 10^7) with stream 0
    forced to 10^7, lognormal values, eps=0.001 (P=1001, ~1000-entry tables,
    the long-stream paths): stream 0 and 2,000 sampled streams exact, the
    size-independent properties on every stream."""
    S, eps, cap = 100_000, 0.001, 10_000_000
    lens = np.clip(np.random.default_rng(5).zipf(1.5, S), 1, cap).astype(np.int64)
    lens[0] = cap
    offs = np.zeros(S + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    x = gpu_lognormal(int(offs[-1]), 5, gpu_device)
    ss = _ss(S, eps, gpu_device)
    q = ss.ingest(x, torch.from_numpy(offs).to(gpu_device), quantiles=QS).cpu().numpy()
    csr, st = gpu_state(ss)
    log("gpu done: %d values, %d promoted" % (int(offs[-1]), ss.num_promoted))
    assert_properties(csr, st, lens, "cfg5")
    rest = np.random.default_rng(6).choice(np.arange(1, S), 2000, replace=False)
    idx = np.concatenate([[0], np.sort(rest)])
    xh = x.cpu().numpy()
    del x
    pieces = [xh[offs[s]:offs[s + 1]] for s in idx]
    so = np.zeros(idx.size + 1, np.int64)
    so[1:] = np.cumsum([p.size for p in pieces])
    o = OracleSet(idx.size, eps)
    o.ingest(np.concatenate(pieces), so)
    oq = o.quantiles(QS)
    log("oracle done")
    assert_same_quantiles(q[idx], oq, "cfg5 quantiles", small_of(o, eps))
    assert_stats_equal(st, o.stats(), "cfg5", idx)
    assert_csr_equal(subset_csr(csr, idx), o.tables(), "cfg5 tables")
