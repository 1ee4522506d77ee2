"""Multi-rank paths of gkarray_amd.dist.

CPU (gloo, world_size 2, 127.0.0.1): the state exchange (sizes, padded
payloads, unpacking), the stream ranges and the rank-ordered fold, with the
per-stream merges done by the oracle on the gathered states and compared with
the single-process left fold of all shards (gk:111-154).
GPU: the same fold on one GPU over 8 virtual row shards (only the transport
differs from an 8-GPU run).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gk_oracle import OracleGK
from gk_oracle_c import OracleSet
from gkarray_amd import dist as gd


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def shard_data(rank, S, eps, seed=5):
    """Row shard `rank`: per stream, a rank-dependent number of values."""
    rng = np.random.default_rng(seed * 1000 + rank)
    P = int(1.0 / eps) + 1
    lens = rng.integers(0, 6 * P, S)
    lens[rank % S] = 0  # some empty sides
    vals = [rng.lognormal(0, 1, int(L)) for L in lens]
    offs = np.zeros(S + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    return np.concatenate(vals) if S else np.zeros(0), offs


def oracle_state(flat, offs, S, eps):
    o = OracleSet(S, eps)
    o.ingest(flat, offs)
    to, v, g, d = o.tables()
    po, pv = o.pending()
    st = o.stats()
    t = torch.from_numpy
    return {"eps": eps, "offs": t(to), "v": t(v), "g": t(g.astype(np.int32)), "d": t(d.astype(np.int32)),
            "poffs": t(po), "pv": t(pv), "n": t(st["n"].copy()), "min": t(st["min"].copy()),
            "max": t(st["max"].copy()), "sum": t(st["sum"].copy()), "avg": t(st["avg"].copy())}


def oracle_streams_from_state(state):
    out = []
    S = int(state["n"].numel())
    for s in range(S):
        o = OracleGK(state["eps"])
        a, b = int(state["offs"][s]), int(state["offs"][s + 1])
        o.v = state["v"][a:b].tolist()
        o.g = [int(x) for x in state["g"][a:b].tolist()]
        o.d = [int(x) for x in state["d"][a:b].tolist()]
        pa, pb = int(state["poffs"][s]), int(state["poffs"][s + 1])
        o.pending = state["pv"][pa:pb].tolist()
        o.n = int(state["n"][s])
        o.min, o.max = float(state["min"][s]), float(state["max"][s])
        o.sum, o.avg = float(state["sum"][s]), float(state["avg"][s])
        out.append(o)
    return out


def same_state(a, b):
    for k in ("offs", "poffs", "n", "g", "d"):
        if not torch.equal(a[k].to(torch.int64), b[k].to(torch.int64)):
            return False
    for k in ("v", "pv", "min", "max", "sum", "avg"):
        if not torch.equal(a[k].view(torch.int64), b[k].view(torch.int64)):
            return False
    return True


def _worker(rank, world, port, S, eps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = oracle_state(*shard_data(rank, S, eps), S, eps)
        states = gd.allgather_states(mine)
        ok_exchange = all(same_state(states[r], oracle_state(*shard_data(r, S, eps), S, eps))
                          for r in range(world))
        a, b = gd.stream_range(S, world, rank)
        # the all-to-all exchange hands this rank exactly its range of every shard
        a2a = gd.alltoall_states(mine)
        ok_exchange = ok_exchange and len(a2a) == world and all(
            same_state(a2a[r], gd.slice_state(states[r], a, b)) for r in range(world))
        parts = [oracle_streams_from_state(gd.slice_state(st, a, b)) for st in states]
        acc = parts[0]
        for other in parts[1:]:
            for x, y in zip(acc, other):
                x.merge(y)
        res = [(o.table(), o.n, o.min, o.max) for o in acc]
        q.put((rank, ok_exchange, (a, b), res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_row_shard_fold(world):
    S, eps = 40, 0.05
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, S, eps, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference: every shard ingested, then the rank-ordered fold
    shards = [oracle_streams_from_state(oracle_state(*shard_data(r, S, eps), S, eps)) for r in range(world)]
    ref = shards[0]
    for other in shards[1:]:
        for x, y in zip(ref, other):
            x.merge(y)
    covered = []
    for rank, ok_exchange, (a, b), res in sorted(results):
        assert ok_exchange, "rank %d received wrong states" % rank
        assert (a, b) == gd.stream_range(S, world, rank)
        for s, (tab, n, mn, mx) in zip(range(a, b), res):
            assert tab == ref[s].table() and n == ref[s].n
            assert mn == ref[s].min and mx == ref[s].max
        covered.extend(range(a, b))
    assert covered == list(range(S))


def test_stream_range_and_balance():
    for S in (0, 1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            rs = [gd.stream_range(S, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == S
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
    lens = np.random.default_rng(0).zipf(1.5, 1000).clip(1, 10 ** 7)
    parts = gd.balanced_assignment(lens, 8)
    assert sorted(torch.cat(parts).tolist()) == list(range(1000))
    loads = [int(lens[p.numpy()].sum()) for p in parts]
    assert max(loads) - min(loads) <= int(lens.max())


def test_pack_slice_concat_roundtrip():
    S, eps = 30, 0.1
    st = oracle_state(*shard_data(0, S, eps), S, eps)
    f, i, j, lens = gd.pack_state(st)
    back = gd.unpack_state(f, i, j, lens, eps)
    assert same_state(st, back)
    parts = [gd.slice_state(st, a, b) for a, b in ((0, 7), (7, 7), (7, 30))]
    assert same_state(gd.concat_states(parts), st)


@pytest.mark.gpu
def test_gpu_fold_of_virtual_row_shards(gpu_device):
    """8 virtual row shards folded on the GPU == the oracle's left fold."""
    S, eps, K = 300, 0.01, 8
    states = [oracle_state(*shard_data(r, S, eps, seed=9), S, eps) for r in range(K)]
    acc = gd.fold_states([{k: (v.to(gpu_device) if torch.is_tensor(v) else v) for k, v in st.items()}
                          for st in states], device=gpu_device)
    ref = OracleSet(S, eps)
    ref.ingest(*shard_data(0, S, eps, seed=9))
    for r in range(1, K):
        o = OracleSet(S, eps)
        o.ingest(*shard_data(r, S, eps, seed=9))
        ref.merge(o)
    offs, v, g, d = acc.tables()
    ro, rv, rg, rd = ref.tables()
    assert np.array_equal(offs.cpu().numpy(), ro)
    assert np.array_equal(v.cpu().numpy().view(np.int64), rv.view(np.int64))
    assert np.array_equal(g.cpu().numpy().astype(np.int64), rg)
    assert np.array_equal(d.cpu().numpy().astype(np.int64), rd)
    q = acc.quantiles([0.5, 0.9, 0.99]).cpu().numpy()
    rq = ref.quantiles([0.5, 0.9, 0.99])
    assert np.array_equal(q.view(np.int64), rq.view(np.int64))


def _merger_worker(rank, world, port, S, eps, exchange, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gkarray_amd import StreamSet
        flat, offs = shard_data(rank, S, eps)
        ss = StreamSet(S, eps, device="cpu")  # the host engine: same C ABI as the GPU path
        merger = gd.RowShardMerger(S, eps, "cpu", exchange=exchange)
        res = None
        for step in range(2):  # reused: same fold sets, fresh exchange each step
            ss.reset()
            ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
            m = merger(ss)
            to, v, g, d = (t.clone() for t in m.tables())
            st = {k: t.clone() for k, t in m.stats().items()}
            bits = lambda t: t.contiguous().view(torch.int64).tolist()  # float64 bit patterns (+0.0 != -0.0)
            res = (to.tolist(), bits(v), g.tolist(), d.tolist(), st["n"].tolist(), bits(st["min"]),
                   bits(st["max"]))
        q.put((rank, merger.range, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,exchange", [(2, "allgather"), (3, "allgather"), (2, "alltoall"), (3, "alltoall")])
def test_gloo_row_shard_merger(world, exchange):
    """RowShardMerger (preallocated fold sets, one host size sync, absolute-offset
    imports) over gloo with host-engine sets == the oracle's rank-ordered fold."""
    S, eps = 40, 0.05
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_merger_worker, args=(r, world, port, S, eps, exchange, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = OracleSet(S, eps)
    ref.ingest(*shard_data(0, S, eps))
    for r in range(1, world):
        o = OracleSet(S, eps)
        o.ingest(*shard_data(r, S, eps))
        ref.merge(o)
    ro, rv, rg, rd = ref.tables()
    rst = ref.stats()
    rvb = np.ascontiguousarray(rv).view(np.int64)
    rmn, rmx = rst["min"].view(np.int64), rst["max"].view(np.int64)
    covered = []
    for rank, (a, b), (to, v, g, d, n, mn, mx) in sorted(results):
        for k, s in enumerate(range(a, b)):
            exp = list(zip(rvb[ro[s]:ro[s + 1]].tolist(), rg[ro[s]:ro[s + 1]].tolist(), rd[ro[s]:ro[s + 1]].tolist()))
            got = list(zip(v[to[k]:to[k + 1]], g[to[k]:to[k + 1]], d[to[k]:to[k + 1]]))
            assert got == exp, (rank, s)
            assert n[k] == rst["n"][s] and mn[k] == rmn[s] and mx[k] == rmx[s]
        covered.extend(range(a, b))
    assert covered == list(range(S))


def _packed_worker(rank, world, port, S, eps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gkarray_amd import StreamSet
        flat, offs = shard_data(rank, S, eps)
        ss = StreamSet(S, eps, device="cpu")
        ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
        dst = StreamSet(S, eps, device="cpu")
        gd.fold_packed_allgather(ss, dst)
        to, v, g, d = dst.tables()
        st = dst.stats()
        po, pv = dst.pending()
        bits = lambda t: t.contiguous().view(torch.int64).tolist()  # float64 bit patterns (+0.0 != -0.0)
        q.put((rank, (to.tolist(), bits(v), g.tolist(), d.tolist(), st["n"].tolist(), bits(st["min"]),
                      bits(st["max"]), bits(st["sum"]), po.tolist(), bits(pv))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_fold_packed_allgather(world):
    """The C-ABI exchange (gk_pack -> all-gather of equal-sized padded buffers
    -> gk_fold_packed) over gloo with host-engine sets: every rank holds the
    oracle's rank-ordered fold of all shards, tables, header and pending."""
    S, eps = 30, 0.05
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_packed_worker, args=(r, world, port, S, eps, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = OracleSet(S, eps)
    ref.ingest(*shard_data(0, S, eps))
    for r in range(1, world):
        o = OracleSet(S, eps)
        o.ingest(*shard_data(r, S, eps))
        ref.merge(o)
    ro, rv, rg, rd = ref.tables()
    rst = ref.stats()
    rpo, rpv = ref.pending()
    b = lambda a: np.ascontiguousarray(a, dtype=np.float64).view(np.int64).tolist()
    for rank, (to, v, g, d, n, mn, mx, sm, po, pv) in results:
        assert to == ro.tolist() and v == b(rv) and g == rg.tolist() and d == rd.tolist(), rank
        assert n == rst["n"].tolist() and mn == b(rst["min"]) and mx == b(rst["max"]), rank
        assert sm == b(rst["sum"]), rank
        assert po == rpo.tolist() and pv == b(rpv), rank
