"""Shared helpers of the GPU parity tests (HIP path through the C ABI vs the
oracle / the golden vectors).  Test infrastructure only."""
import numpy as np
import torch

import golden_io as G
from gk_oracle_c import OracleSet  # noqa: F401  (re-exported for the tests)


def _ss(S, eps, dev, **kw):
    from gkarray_amd import StreamSet
    return StreamSet(S, eps, device=dev, **kw)


def same_q(a, b, unpinned):
    # signed-zero tolerance only in the exactly named class where the
    # reference's own answer depends on numpy's CPU dispatch
    # (golden_io.zero_sign_unpinned: comparisons with reference goldens only)
    return G.same_float(a, b) or (bool(unpinned) and a == 0 and b == 0)


def small_n(n, eps):
    """Per-stream flag of the small-n branch: n < 1/eps (gk:169 / gk:200)."""
    return np.asarray(n, dtype=np.float64) < 1.0 / eps


def small_of(osx, eps):
    """Tolerance mask for comparisons with the ORACLE: none.  The engines and
    the oracle answer the small-n branch from the same stable-ordered table
    with numpy's arithmetic, so they agree bit for bit, the sign of zero
    included (round 4; before, any zero of the small-n branch was tolerated)."""
    return None


def golden_mask(table, n, eps, qs):
    """Exact unpinned positions of a comparison with a reference golden."""
    return np.asarray(G.unpinned_mask(table, n, eps, qs), dtype=bool)


def csr(seqs):
    offs = np.zeros(len(seqs) + 1, np.int64)
    offs[1:] = np.cumsum([len(x) for x in seqs])
    flat = np.concatenate([np.asarray(x, np.float64) for x in seqs]) if len(seqs) else np.zeros(0)
    return flat, offs


def ingest_np(ss, seqs):
    flat, offs = csr(seqs)
    ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))


def tables_np(ss):
    offs, v, g, d = ss.tables()
    return offs.cpu().numpy(), v.cpu().numpy(), g.cpu().numpy(), d.cpu().numpy()


def assert_same_tables(ss, osx, ids=None, what=""):
    go, gv, gg, gd = tables_np(ss)
    oo, ov, og, od = osx.tables()
    S = ss.num_streams
    ids = range(S) if ids is None else ids
    for s in ids:
        a, b = go[s], go[s + 1]
        c, e = oo[s], oo[s + 1]
        assert b - a == e - c, "%s stream %d: size %d vs %d" % (what, s, b - a, e - c)
        assert np.array_equal(gv[a:b].view(np.int64), ov[c:e].view(np.int64)), "%s stream %d values" % (what, s)
        assert np.array_equal(gg[a:b].astype(np.int64), og[c:e]), "%s stream %d g" % (what, s)
        assert np.array_equal(gd[a:b].astype(np.int64), od[c:e]), "%s stream %d delta" % (what, s)


def assert_same_state(ss, osx, what=""):
    assert_same_tables(ss, osx, what=what)
    gp_o, gp_v = ss.pending()
    op_o, op_v = osx.pending()
    assert np.array_equal(gp_o.cpu().numpy(), op_o), what + " pending offsets"
    assert np.array_equal(gp_v.cpu().numpy().view(np.int64), op_v.view(np.int64)), what + " pending"
    st = {k: v.cpu().numpy() for k, v in ss.stats().items()}
    ost = osx.stats()
    for k in ("n", "size", "pending"):
        assert np.array_equal(st[k].astype(np.int64), ost[k].astype(np.int64)), what + " " + k
    for k in ("min", "max", "sum", "avg"):
        assert np.array_equal(st[k].view(np.int64), ost[k].view(np.int64)), what + " " + k


def assert_same_quantiles(got, exp, what, unpinned):
    """got/exp: [S, nq] or [nq].  unpinned: None (strict: every engine-vs-
    oracle comparison) or a boolean mask of got's shape (golden_mask) naming
    the answers whose zero sign the reference leaves to numpy's dispatch."""
    got = np.asarray(got)
    exp = np.asarray(exp)
    assert got.shape == exp.shape
    sm = (np.zeros(got.shape, dtype=bool) if unpinned is None
          else np.broadcast_to(np.asarray(unpinned, dtype=bool), got.shape))
    bad = [(i, got.flat[i], exp.flat[i]) for i in range(got.size)
           if not same_q(got.flat[i], exp.flat[i], sm.flat[i])]
    assert not bad, "%s: %d mismatches, first %r" % (what, len(bad), bad[:3])


def check_golden_merge_plans(dev):
    """The reference's merge plans (make_golden.py section 7): sk[0].merge(sk[p])
    for p in the plan, p == 0 merging a sketch into ITSELF (gk:111-154) and
    repeated sources.  The cases of one (eps, plan) run batched, one stream
    each, through StreamSet.merge_from([self]) / merge_from([src]); every
    step's destination and source tables, the final stats and quantiles are
    compared with the reference's.  Returns the number of cases checked."""
    groups = {}
    for c in G.cases("merge_plan"):
        groups.setdefault((c["eps"], tuple(c["plan"])), []).append(c)
    checked = 0
    for (eps, plan), cs in groups.items():
        nsh = max(plan) + 1
        sets = []
        for j in range(nsh):
            ss = _ss(len(cs), eps, dev)
            ingest_np(ss, [G.shards(c["id"])[j] for c in cs])
            sets.append(ss)
        for k, p in enumerate(plan):
            sets[0].merge_from([sets[p]])
            for i, c in enumerate(cs):
                assert G.same_table(sets[0].table(i), G.tables(c["id"], "merge_steps")[k]), (c, k)
                assert G.same_table(sets[p].table(i), G.tables(c["id"], "others_after")[k]), (c, k)
        st = {k: v.cpu().numpy() for k, v in sets[0].stats().items()}
        q = sets[0].quantiles(G.index()["qs"]).cpu().numpy()
        for i, c in enumerate(cs):
            got = [st["n"][i], st["min"][i], st["max"][i], st["sum"][i], st["avg"][i]]
            assert all(G.same_float(a, b) for a, b in zip(got, G.get(c["id"], "merged_stats"))), (c, got)
            assert_same_quantiles(q[i], G.get(c["id"], "merged_q"), c,
                                  golden_mask(G.tables(c["id"], "merge_steps")[-1], st["n"][i], eps,
                                              G.index()["qs"]))
            assert G.same_table(sets[0].table(i), G.tables(c["id"], "merged_final")[0]), c
            checked += 1
    return checked


def gen(dist, L, rng):
    if dist == 0:
        return rng.random(L)
    if dist == 1:
        return rng.lognormal(0, 1, L)
    if dist == 2:
        return rng.pareto(1.5, L) + 1
    if dist == 3:
        return np.sort(rng.random(L))[::-1].copy()
    if dist == 4:
        return np.sort(rng.random(L))
    if dist == 5:
        return rng.integers(0, 5, L).astype(np.float64)
    if dist == 6:
        return rng.choice(np.array([0.0, -0.0, 1.0, -1.0]), L)
    return np.round(rng.normal(0, 2, L), 1)
