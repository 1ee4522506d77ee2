"""Generate golden vectors from the UNMODIFIED reference gkarray.py.

Run only in the build container (the reference is not present on the GPU box):

    python tests/golden/make_golden.py

It loads ``/root/reference/gkarray/gkarray.py`` with ``importlib`` (never writing
bytecode into the read-only reference tree) through the harness shim described in
SURVEY.md section 8(c):

* ``np.NaN`` is aliased to ``np.nan`` (the reference uses ``np.NaN`` at gk:195,
  202, 217; numpy >= 2 removed it);
* every raw value is passed as ``V(x)``, a float subclass carrying ``g=1,
  delta=0`` and a ``.val`` property, which is the evident intent of gk:55 vs
  gk:72 (the reference as written raises AttributeError on plain floats at its
  first flush).

Outputs ``tests/golden/golden.npz`` (arrays only; load with
``allow_pickle=False``) and ``tests/golden/golden_index.json`` (case metadata).
Both files are data: inputs and the reference's outputs on them.
"""
import importlib.util
import json
import os
import sys

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

if not hasattr(np, "NaN"):
    np.NaN = np.nan

REF = "/root/reference/gkarray/gkarray.py"
HERE = os.path.dirname(os.path.abspath(__file__))


def load_reference():
    spec = importlib.util.spec_from_file_location("gkarray_reference", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class V(float):
    """Raw value == Entry(val, g=1, delta=0)."""
    __slots__ = ("g", "delta")

    def __new__(cls, x):
        o = float.__new__(cls, x)
        o.g = 1
        o.delta = 0
        return o

    @property
    def val(self):
        return float(self)


def snap(sk):
    return [(float(e.val), int(e.g), int(e.delta)) for e in sk.entries]


def gen_values(dist, L, rng):
    if dist == "uniform":
        return rng.random(L)
    if dist == "lognormal":
        return rng.lognormal(0.0, 1.0, L)
    if dist == "pareto":
        return rng.pareto(1.5, L) + 1.0
    if dist == "ascending":
        return np.sort(rng.random(L))
    if dist == "descending":
        return np.sort(rng.random(L))[::-1].copy()
    if dist == "fewdistinct":
        return rng.integers(0, 5, L).astype(np.float64)
    if dist == "zeros":
        # signed zeros mixed with a few small values: stability of ties matters
        x = rng.choice(np.array([0.0, -0.0, 1.0, -1.0, 0.5]), L,
                       p=[0.35, 0.35, 0.1, 0.1, 0.1])
        return x.astype(np.float64)
    if dist == "normal_dup":
        return np.round(rng.normal(0.0, 3.0, L), 1)
    raise ValueError(dist)


QS = [0.0, 0.01, 0.25, 0.5, 0.9, 0.99, 1.0]
QS_UNSORTED = [0.9, 0.1, 0.5, 1.0, 0.0]
QS_OOR = [-0.5, 0.0, 0.5, 1.0, 1.5]


class Store:
    def __init__(self):
        self.arrays = {}
        self.index = []

    def put(self, name, arr, dtype):
        self.arrays[name] = np.asarray(arr, dtype=dtype)

    def put_tables(self, prefix, tables):
        sizes = [len(t) for t in tables]
        flat = [r for t in tables for r in t]
        self.put(prefix + "/sizes", sizes, np.int64)
        self.put(prefix + "/v", [r[0] for r in flat], np.float64)
        self.put(prefix + "/g", [r[1] for r in flat], np.int64)
        self.put(prefix + "/d", [r[2] for r in flat], np.int64)


def stats(sk):
    return [float(sk._n), float(sk._min), float(sk._max), float(sk._sum), float(sk._avg)]


def run_stream_case(ref, st, cid, eps, xs, per_flush):
    """Add xs one by one; snapshot the table after every automatic flush."""
    sk = ref.GKArray(eps)
    tables, flush_n = [], []
    for x in xs:
        sk.add(V(x))
        if per_flush and len(sk.incoming) == 0:
            tables.append(snap(sk))
            flush_n.append(sk._n)
    pre = "case%d" % cid
    st.put(pre + "/x", xs, np.float64)
    if per_flush:
        st.put_tables(pre + "/flush", tables)
        st.put(pre + "/flush_n", flush_n, np.int64)
    st.put(pre + "/pending", [float(p) for p in sk.incoming], np.float64)
    st.put(pre + "/stats_before_query", stats(sk), np.float64)
    # table before any query-triggered flush (only the automatic flushes)
    st.put_tables(pre + "/auto", [snap(sk)])
    q1 = [float(sk.quantile(q)) for q in QS]             # flushes (mutation)
    st.put_tables(pre + "/final", [snap(sk)])
    q2 = [float(v) for v in sk.quantiles(QS)]
    q3 = [float(v) for v in sk.quantiles(QS_UNSORTED)]
    q4 = [float(v) for v in sk.quantiles(QS_OOR)]
    st.put(pre + "/q_single", q1, np.float64)
    st.put(pre + "/q_sorted", q2, np.float64)
    st.put(pre + "/q_unsorted", q3, np.float64)
    st.put(pre + "/q_oor", q4, np.float64)
    st.put(pre + "/stats", stats(sk), np.float64)
    st.put(pre + "/size", [sk.size()], np.int64)


def run_query_mid_case(ref, st, cid, eps, xs, query_points):
    """Queries in mid-stream flush pending values and change later decisions."""
    sk = ref.GKArray(eps)
    outs, tables = [], []
    qp = set(query_points)
    for k, x in enumerate(xs):
        sk.add(V(x))
        if (k + 1) in qp:
            outs.append([float(v) for v in sk.quantiles([0.1, 0.5, 0.9])])
            tables.append(snap(sk))
    tables.append(snap(sk))
    pre = "case%d" % cid
    st.put(pre + "/x", xs, np.float64)
    st.put(pre + "/query_points", query_points, np.int64)
    st.put(pre + "/mid_q", outs, np.float64)
    st.put_tables(pre + "/mid_tables", tables)
    st.put(pre + "/pending", [float(p) for p in sk.incoming], np.float64)
    st.put(pre + "/stats", stats(sk), np.float64)


def run_merge_case(ref, st, cid, eps, shards):
    """Left fold shards[0].merge(shards[1]).merge(shards[2]) ... (gk:111-154)."""
    sks = []
    for xs in shards:
        sk = ref.GKArray(eps)
        for x in xs:
            sk.add(V(x))
        sks.append(sk)
    pre = "case%d" % cid
    st.put(pre + "/shard_sizes", [len(s) for s in shards], np.int64)
    st.put(pre + "/x", np.concatenate([np.asarray(s, dtype=np.float64) for s in shards])
           if shards else [], np.float64)
    acc = sks[0]
    steps, others = [], []
    for other in sks[1:]:
        acc.merge(other)
        steps.append(snap(acc) + [])
        others.append(snap(other))
    pre_stats = stats(acc)
    st.put_tables(pre + "/merge_steps", steps)
    st.put_tables(pre + "/others_after", others)
    st.put(pre + "/merged_stats", pre_stats, np.float64)
    st.put(pre + "/merged_pending", [float(p) for p in acc.incoming], np.float64)
    q = [float(v) for v in acc.quantiles(QS)]
    st.put(pre + "/merged_q", q, np.float64)
    st.put_tables(pre + "/merged_final", [snap(acc)])


def run_merge_plan_case(ref, st, cid, eps, shards, plan):
    """sk[0].merge(sk[p]) for p in plan, in order; p == 0 merges the sketch
    into itself (the reference accepts it: gk:111-154)."""
    sks = []
    for xs in shards:
        sk = ref.GKArray(eps)
        for x in xs:
            sk.add(V(x))
        sks.append(sk)
    pre = "case%d" % cid
    st.put(pre + "/shard_sizes", [len(s) for s in shards], np.int64)
    st.put(pre + "/x", np.concatenate([np.asarray(s, dtype=np.float64) for s in shards]), np.float64)
    st.put(pre + "/plan", plan, np.int64)
    acc = sks[0]
    steps, srcs = [], []
    for p in plan:
        acc.merge(sks[p])
        steps.append(snap(acc))
        srcs.append(snap(sks[p]))
    st.put_tables(pre + "/merge_steps", steps)
    st.put_tables(pre + "/others_after", srcs)
    st.put(pre + "/merged_stats", stats(acc), np.float64)
    st.put(pre + "/merged_pending", [float(p) for p in acc.incoming], np.float64)
    st.put(pre + "/merged_q", [float(v) for v in acc.quantiles(QS)], np.float64)
    st.put_tables(pre + "/merged_final", [snap(acc)])


def main():
    ref = load_reference()
    st = Store()
    cid = 0
    rng = np.random.default_rng(20261015)
    dists = ["uniform", "lognormal", "pareto", "ascending", "descending",
             "fewdistinct", "zeros", "normal_dup"]
    eps_list = [0.2, 0.1, 0.05, 0.03, 0.015, 0.01]

    # -- 1. single streams, flush-by-flush tables ---------------------------
    for eps in eps_list:
        P = int(1.0 / eps) + 1
        lengths = sorted(set([1, 2, 7, P - 1, P, P + 1, 3 * P + 5, 1500]))
        for dist in dists:
            for L in lengths:
                xs = gen_values(dist, L, rng)
                run_stream_case(ref, st, cid, eps, xs, per_flush=True)
                st.index.append(dict(id=cid, kind="stream", eps=eps, dist=dist, L=int(L)))
                cid += 1
    # longer streams (fewer snapshots)
    for eps in [0.03, 0.01]:
        for dist in ["uniform", "descending", "fewdistinct", "pareto"]:
            xs = gen_values(dist, 12000, rng)
            run_stream_case(ref, st, cid, eps, xs, per_flush=False)
            st.index.append(dict(id=cid, kind="stream", eps=eps, dist=dist, L=12000))
            cid += 1
    for dist in ["lognormal", "ascending", "zeros"]:
        xs = gen_values(dist, 6000, rng)
        run_stream_case(ref, st, cid, 0.001, xs, per_flush=True)
        st.index.append(dict(id=cid, kind="stream", eps=0.001, dist=dist, L=6000))
        cid += 1

    # -- 2. query-triggered flushes in mid-stream ----------------------------
    for eps in [0.1, 0.03, 0.01]:
        P = int(1.0 / eps) + 1
        for dist in ["uniform", "pareto", "zeros"]:
            L = 6 * P + 17
            xs = gen_values(dist, L, rng)
            pts = sorted(set([3, P // 2, P, P + 1, 2 * P + 7, 4 * P - 1, 5 * P + 3]))
            run_query_mid_case(ref, st, cid, eps, xs, pts)
            st.index.append(dict(id=cid, kind="query_mid", eps=eps, dist=dist, L=int(L)))
            cid += 1

    # -- 3. merges (left folds, empty sides, Sigma g != n cases) --------------
    for eps in [0.1, 0.05, 0.01]:
        P = int(1.0 / eps) + 1
        for dist in ["uniform", "lognormal", "fewdistinct", "zeros", "descending"]:
            for k in [2, 3, 8]:
                lens = rng.integers(0, 8 * P, k)
                lens[0] = max(lens[0], 1)
                shards = [gen_values(dist, int(L), rng) for L in lens]
                run_merge_case(ref, st, cid, eps, shards)
                st.index.append(dict(id=cid, kind="merge", eps=eps, dist=dist, k=k))
                cid += 1
        # empty-side paths: other empty, self empty, both small
        for lens in ([0, 40], [40, 0], [0, 0, 5], [3, 2], [1, 1, 1, 1]):
            shards = [gen_values("uniform", int(L), rng) for L in lens]
            run_merge_case(ref, st, cid, eps, shards)
            st.index.append(dict(id=cid, kind="merge", eps=eps, dist="uniform-edge",
                                 k=len(lens)))
            cid += 1

    # -- 4. epsilon mismatch raises --------------------------------------------
    a, b = ref.GKArray(0.01), ref.GKArray(0.02)
    a.add(V(1.0)); b.add(V(2.0))
    try:
        a.merge(b)
        raised = False
    except ref.UnequalEpsilonException:
        raised = True
    assert raised
    st.index.append(dict(id=-1, kind="eps_mismatch", raised=True))

    # -- 5. known-answer vectors -------------------------
    kat = {}
    sk = ref.GKArray(0.1)
    xs = [float((7 * i) % 23) for i in range(40)]
    for x in xs[:33]:
        sk.add(V(x))
    kat["kat1_table_after_33"] = snap(sk)
    kat["kat1_pending_after_33"] = len(sk.incoming)
    for x in xs[33:]:
        sk.add(V(x))
    kat["kat1_quantiles"] = [float(v) for v in sk.quantiles([0, .25, .5, .75, 1])]
    kat["kat1_final_table"] = snap(sk)
    sk = ref.GKArray(0.1)
    for x in [3.0, 1.0, 2.0]:
        sk.add(V(x))
    kat["kat2_q50"] = float(sk.quantile(.5))
    kat["kat2_q25"] = float(sk.quantile(.25))
    sk = ref.GKArray(0.01)
    big = np.random.default_rng(0).random(1_000_000)
    for x in big:
        sk.add(V(x))
    kat["kat3_quantiles"] = [float(v) for v in sk.quantiles([.5, .9, .99])]
    kat["kat3_size"] = sk.size()
    kat["kat3_stats"] = stats(sk)
    kat["kat3_table"] = snap(sk)

    # -- 6. eps > 1 (gk:21 accepts any eps; gk:60 gives P = int(1/eps)+1 = 2
    #       at eps = 1 and 1 above it: every add flushes) -- appended last so
    #       that the cases above keep their ids and random draws
    rng6 = np.random.default_rng(20261017)
    for eps in [1.0, 1.5, 3.0]:
        for dist in ["uniform", "pareto", "descending", "fewdistinct", "zeros"]:
            for L in [1, 2, 3, 7, 60, 400]:
                xs = gen_values(dist, L, rng6)
                run_stream_case(ref, st, cid, eps, xs, per_flush=True)
                st.index.append(dict(id=cid, kind="stream", eps=eps, dist=dist, L=int(L)))
                cid += 1
        for dist in ["uniform", "zeros"]:
            L = 40
            xs = gen_values(dist, L, rng6)
            run_query_mid_case(ref, st, cid, eps, xs, [1, 2, 5, 17, 39])
            st.index.append(dict(id=cid, kind="query_mid", eps=eps, dist=dist, L=int(L)))
            cid += 1
        for k in [2, 3]:
            lens = rng6.integers(0, 120, k)
            lens[0] = max(lens[0], 1)
            shards = [gen_values("lognormal", int(L), rng6) for L in lens]
            run_merge_case(ref, st, cid, eps, shards)
            st.index.append(dict(id=cid, kind="merge", eps=eps, dist="lognormal", k=k))
            cid += 1

    # -- 7. merge plans: a.merge(a) (gk:111-154 with other IS self: the flush
    #       of gk:137 empties self's own incoming, gk:149 doubles _n) and
    #       repeated sources (a.merge(b); a.merge(b): b is flushed twice) --
    #       appended last so that the cases above keep their ids and draws
    rng7 = np.random.default_rng(20261018)
    for eps in [0.1, 0.01]:
        P = int(1.0 / eps) + 1
        for L in [0, 1, 5, 3 * P, 3 * P + 5, 9 * P + 40]:
            for dist in ["uniform", "zeros"]:
                for plan in ([0], [0, 0], [1, 0], [1, 1], [0, 1, 0]):
                    lens = [L] + ([int(rng7.integers(1, 4 * P))] if 1 in plan else [])
                    shards = [gen_values(dist, int(n), rng7) for n in lens]
                    run_merge_plan_case(ref, st, cid, eps, shards, plan)
                    st.index.append(dict(id=cid, kind="merge_plan", eps=eps, dist=dist, L=int(L),
                                         plan=list(plan)))
                    cid += 1

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **st.arrays)
    with open(os.path.join(HERE, "golden_index.json"), "w") as f:
        json.dump(dict(cases=st.index, kat=kat, qs=QS, qs_unsorted=QS_UNSORTED,
                       qs_oor=QS_OOR, generator="tests/golden/make_golden.py",
                       reference="gkarray.py (githomin/sketches-py) via SURVEY 8(c) shim",
                       numpy=np.__version__), f, indent=0)
    print("cases:", cid, "arrays:", len(st.arrays),
          "bytes:", os.path.getsize(os.path.join(HERE, "golden.npz")))


if __name__ == "__main__":
    main()
