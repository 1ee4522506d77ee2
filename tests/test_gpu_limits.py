"""No eps / table-size limits on the GPU path (reference: any eps and
unbounded lists, gkarray.py gk:21-29, 60).  Flush periods beyond 1024 values
(eps < 1/1023) and tables beyond 32768 entries run in k_ingest_big, the
unbounded capacity classes; every case is bit-exact vs the C oracle (tables,
pending values, header, quantiles), through the C ABI."""
import numpy as np
import pytest
import torch

from gk_oracle_c import OracleSet
from parity_util import _ss, assert_same_quantiles, assert_same_state, assert_same_tables, csr, gen, small_of

pytestmark = pytest.mark.gpu

QS = [0.0, 0.001, 0.01, 0.25, 0.5, 0.75, 0.9, 0.99, 0.999, 1.0]


def desc(n):
    return np.arange(n, 0, -1, dtype=np.float64)


def check_q(ss, o, eps, what):
    sm = small_of(o, eps)
    assert_same_quantiles(ss.quantiles(QS).cpu().numpy(), o.quantiles(QS), what + " quantiles", sm)
    sq = [0.9, 0.1, 0.5]
    assert_same_quantiles(ss.quantiles(sq, single=True).cpu().numpy(), o.quantiles(sq, single=True),
                          what + " quantile()", sm)


def run_batches(ss, o, seq_batches, what):
    for b, seqs in enumerate(seq_batches):
        flat, offs = csr(seqs)
        ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
        o.ingest(flat, offs)
        assert_same_state(ss, o, "%s batch %d" % (what, b))


@pytest.mark.parametrize("eps", [0.0005, 0.0002, 0.0001])
def test_tiny_eps_mixed_streams_vs_oracle(gpu_device, eps):
    """P = 2001 / 5001 / 10001: every class is k_ingest_big; ragged lengths
    (0, 1, P-1, P, several P), all generators, three batches (pending values
    carried between calls), then quantiles (small-n and rank-walk branches)."""
    P = int(1.0 / eps) + 1
    rng = np.random.default_rng(int(1 / eps))
    S = 24
    batches = []
    for part in range(3):
        lens = rng.integers(0, 12 * P, S)
        lens[:5] = [0, 1, P - 1, P, 2 * P + 3]
        batches.append([gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), lens)])
    ss = _ss(S, eps, gpu_device)
    assert ss.flush_period == P
    o = OracleSet(S, eps)
    run_batches(ss, o, batches, "eps=%g" % eps)
    check_q(ss, o, eps, "eps=%g" % eps)
    assert_same_state(ss, o, "eps=%g after quantiles" % eps)


def test_gkarray_0005_descending_million(gpu_device):
    """The drop-in at eps = 0.0005: a descending 10^6-value stream (10670
    entries) and a small-n stream (< 1/eps values: numpy percentile branch)."""
    from gkarray_amd import GKArray
    eps = 0.0005
    a = GKArray(eps, device=gpu_device)
    x = desc(10 ** 6)
    a.add_many(x)
    o = OracleSet(1, eps)
    o.ingest(x, np.array([0, x.size]))
    assert a.num_values() == 10 ** 6
    o.flush(1)
    assert a.size() == int(o.stats()["size"][0])  # size() flushes (gk:44-47)
    ot = o.table(0)
    got = [(e.val, e.g, e.delta) for e in a.entries]
    assert len(got) == len(ot) > 10000
    assert all(np.float64(gv).view(np.int64) == np.float64(ov).view(np.int64) and gg == og and gd == od
               for (gv, gg, gd), (ov, og, od) in zip(got, ot))
    qs = [0.0, 0.01, 0.5, 0.99, 1.0]
    exp = o.quantiles(qs)[0]
    assert_same_quantiles(np.array(a.quantiles(qs)), exp, "GKArray(0.0005) quantiles", False)
    single = o.quantiles(qs, single=True)[0]
    assert_same_quantiles(np.array([a.quantile(q) for q in qs]), single, "GKArray(0.0005) quantile()", False)

    b = GKArray(eps, device=gpu_device)
    rng = np.random.default_rng(5)
    y = rng.lognormal(0, 1, 1500)
    for v in y:
        b.add(v)
    ob = OracleSet(1, eps)
    ob.ingest(y, np.array([0, y.size]))
    assert_same_quantiles(np.array(b.quantiles(qs)), ob.quantiles(qs)[0], "GKArray(0.0005) small n", True)


def test_descending_million_eps_001(gpu_device):
    """eps = 0.001: a descending 10^6 stream grows to 5888 entries (the
    32768 class); an ascending one and a duplicate-heavy one beside it."""
    eps = 0.001
    n = 10 ** 6
    rng = np.random.default_rng(9)
    seqs = [desc(n), np.arange(n, dtype=np.float64), rng.integers(0, 50, n).astype(np.float64)]
    ss = _ss(3, eps, gpu_device)
    o = OracleSet(3, eps)
    run_batches(ss, o, [seqs], "desc eps=.001")
    assert int(ss.stats()["size"][0]) > 2048
    check_q(ss, o, eps, "desc eps=.001")


@pytest.mark.parametrize("eps", [0.0002, 0.0001])
def test_tables_beyond_class0_promote_lazily(gpu_device, eps):
    """Descending 10^6 at eps = 0.0002 / 0.0001 (23427 / 41845 entries)
    outgrows class 0 (2P rounded up); the next unbounded class has no slots
    until first used: the stream is deferred, its arena allocated by the host,
    and the call re-run -- before the next call observes the set."""
    n = 10 ** 6
    ss = _ss(2, eps, gpu_device)
    o = OracleSet(2, eps)
    rng = np.random.default_rng(3)
    run_batches(ss, o, [[desc(n // 2), rng.random(1000)], [desc(n // 2) - n, rng.random(5000)]], "lazy eps=%g" % eps)
    assert int(ss.stats()["size"][0]) > ss.capacity(0)
    assert ss.num_promoted == 1
    check_q(ss, o, eps, "lazy eps=%g" % eps)


@pytest.mark.parametrize("caps", ["2048,4096,8192b", "2048,4096,65536"])
def test_unbounded_class_after_32768_ladder(gpu_device, monkeypatch, caps):
    """The default ladder puts k_ingest_big after the 32768 class; a short
    ladder (GK_CAPS) reaches it with eps = 0.001 tables (5888 entries):
    2048 (LDS) -> 4096 (global k_ingest) -> k_ingest_big (8192, or a lazily
    allocated 65536 class)."""
    monkeypatch.setenv("GK_CAPS", caps)
    eps = 0.001
    n = 10 ** 6
    ss = _ss(4, eps, gpu_device)
    assert ss.capacity(2) == int(caps.split(",")[2].rstrip("b"))
    o = OracleSet(4, eps)
    rng = np.random.default_rng(11)
    seqs = [desc(n), rng.random(20000), np.arange(3000, dtype=np.float64), rng.pareto(1.5, 50000) + 1]
    run_batches(ss, o, [seqs, [s[: len(s) // 3] for s in seqs]], "ladder " + caps)
    check_q(ss, o, eps, "ladder " + caps)


@pytest.mark.parametrize("caps", ["128,4096b", "128,2048,4096b"])
def test_small_class_partial_commit_then_promotion(gpu_device, monkeypatch, caps):
    """k_ingest_small commits the flushes of a call that fit its 128 entries
    and the promoted stream continues in the next class from value n - n0 of
    the call: a descending stream at eps = 0.01 flushes several
    times in class 0 before it outgrows it (462 entries after 20 000 values),
    in one call and over calls, into k_ingest<2048> or straight into
    k_ingest_big; beside it streams that stay small.  Bit-exact vs the
    oracle after every call."""
    monkeypatch.setenv("GK_CAPS", caps)
    eps = 0.01
    rng = np.random.default_rng(17)
    ss = _ss(5, eps, gpu_device)
    o = OracleSet(5, eps)
    d = desc(20000)
    b1 = [d[:6000], rng.random(3000), d[:250], rng.pareto(1.5, 999) + 1, np.zeros(0)]
    b2 = [d[6000:], rng.random(1234), d[250:20000] - 1e6, rng.pareto(1.5, 5000) + 1, d[:40]]
    run_batches(ss, o, [b1, b2], "partial commit " + caps)
    assert ss.num_promoted >= 2
    check_q(ss, o, eps, "partial commit " + caps)


@pytest.mark.parametrize("fuse,fork", [("1", False), ("0", False), ("1", True)])
def test_round6_call_paths_vs_oracle(gpu_device, monkeypatch, fuse, fork):
    """Round-6 call paths, bit-exact against the oracle after every call:
    promotion rounds fused into the class re-run launches (GK_PROMOTE_FUSE=1,
    the default) or as separate k_promote_dev launches (0), over a ladder
    of four classes (128 -> 256 -> 512 -> 4096: several rounds per call) and across calls
    (member-list launches, non-fresh rounds); streams longer than 16 384
    values in the small class (k_stats_long) with the fork decided by the
    last ingest's count (first call: behind the ingest on the call's stream)
    or always forked (GK_SL_FORK=1); a reset between calls (k_reset zeroes
    the per-call counters, the next call skips its memset)."""
    monkeypatch.setenv("GK_CAPS", "128,256,512,4096")
    monkeypatch.setenv("GK_PROMOTE_FUSE", fuse)
    if fork:
        monkeypatch.setenv("GK_SL_FORK", "1")
    else:
        monkeypatch.delenv("GK_SL_FORK", raising=False)
    eps = 0.01
    rng = np.random.default_rng(29)
    S = 40

    def batch(k):
        seqs = []
        for i in range(S):
            kind = (i + k) % 5
            if kind == 0:
                seqs.append(desc(int(rng.integers(20000, 60000))) - 1e6 * k)  # promoted, long
            elif kind == 1:
                seqs.append(rng.pareto(1.5, int(rng.integers(17000, 40000))) + 1)  # long stats chain
            elif kind == 2:
                seqs.append(rng.random(int(rng.integers(0, 3000))))
            elif kind == 3:
                seqs.append(np.zeros(int(rng.integers(0, 300))))
            else:
                seqs.append(rng.lognormal(0, 2, int(rng.integers(100, 9000))))
        return seqs

    ss = _ss(S, eps, gpu_device)
    o = OracleSet(S, eps)
    run_batches(ss, o, [batch(0), batch(1)], "round-6 paths fuse=%s fork=%s" % (fuse, fork))
    assert ss.num_promoted >= 8
    check_q(ss, o, eps, "round-6 paths")
    ss.reset()
    o = OracleSet(S, eps)
    run_batches(ss, o, [batch(2), batch(3)], "round-6 paths after reset")
    check_q(ss, o, eps, "round-6 paths after reset")


def test_small_class_fatal_stream_keeps_committed_prefix(gpu_device, monkeypatch):
    """A stream that outgrows every class (GK_CAPS=128,256: no unbounded
    class) is reported (sticky GK_E_OVERFLOW); what it keeps is the state
    after the last flush that fitted the small class -- exactly the oracle's
    state after that prefix of its values (a flush boundary: no pending
    value) -- and the other streams of the call are added in full."""
    monkeypatch.setenv("GK_CAPS", "128,256")
    eps = 0.01
    rng = np.random.default_rng(23)
    ss = _ss(3, eps, gpu_device)
    d = desc(20000)
    seqs = [rng.random(5000), d, rng.pareto(1.5, 777) + 1]
    flat, offs = csr(seqs)
    ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs), sync=False)
    with pytest.raises(Exception, match="outgrew"):
        ss.sync()
    st = {k: v.cpu().numpy() for k, v in ss.stats().items()}
    n1 = int(st["n"][1])
    P = int(1 / eps) + 1
    assert 0 < n1 < d.size and n1 % P == 0 and int(st["pending"][1]) == 0
    o = OracleSet(3, eps)
    o.ingest(*csr([seqs[0], d[:n1], seqs[2]]))
    assert_same_tables(ss, o, what="fatal prefix")
    ost = o.stats()
    for k in ("n", "size", "pending"):
        assert np.array_equal(st[k].astype(np.int64), ost[k].astype(np.int64)), "fatal prefix " + k
    # (min/max/sum/avg of the refused call's values are computed beside the
    # tables and include them -- DESIGN 4's documented deviation (3); the
    # other streams' are exact)
    for k in ("min", "max", "sum", "avg"):
        assert np.array_equal(st[k][[0, 2]].view(np.int64), ost[k][[0, 2]].view(np.int64)), "other streams " + k


def test_merge_tiny_eps_vs_oracle(gpu_device):
    """merge (gk:111-154) of P = 2001 sets, both with tables and pending values."""
    eps = 0.0005
    P = int(1 / eps) + 1
    rng = np.random.default_rng(21)
    S = 6
    mk = lambda: [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), rng.integers(0, 8 * P, S))]
    a, b = _ss(S, eps, gpu_device), _ss(S, eps, gpu_device)
    oa, ob = OracleSet(S, eps), OracleSet(S, eps)
    run_batches(a, oa, [mk()], "merge a")
    run_batches(b, ob, [mk()], "merge b")
    a.merge_from([b])
    oa.merge(ob)
    assert_same_state(a, oa, "merged")
    check_q(a, oa, eps, "merged")


def test_save_load_tiny_eps(gpu_device, tmp_path):
    from gkarray_amd import StreamSet
    eps = 0.0002
    ss = _ss(2, eps, gpu_device)
    o = OracleSet(2, eps)
    run_batches(ss, o, [[desc(400000), np.random.default_rng(1).random(12345)]], "save")
    p = str(tmp_path / "tiny.gks")
    ss.save(p)
    r = StreamSet.load(p, device=gpu_device)
    assert_same_state(r, o, "loaded")
    run_batches(r, o, [[desc(300000) - 1e6, np.random.default_rng(2).random(777)]], "loaded+")


def test_count_limit_is_an_error_not_a_clamp(gpu_device):
    """T = floor(2 eps (n-1)) must stay <= 2^30 (int32 tuples): a stream whose
    count would pass it is refused with GK_E_OVERFLOW, its state unchanged;
    the other streams of the call are added."""
    from gkarray_amd import StreamSet
    eps = 0.5  # P = 3, T = n - 1
    lim = (1 << 30) + 1  # largest n with T <= 2^30
    ss = _ss(2, eps, gpu_device)
    dev = gpu_device
    f64 = lambda a: torch.tensor(a, dtype=torch.float64, device=dev)
    i64 = lambda a: torch.tensor(a, dtype=torch.int64, device=dev)
    i32 = lambda a: torch.tensor(a, dtype=torch.int32, device=dev)
    n0 = lim - 2
    # stream 0: a plausible table at n0 (g sums to n0); stream 1 empty
    ss.import_arrays(i64([0, 2, 2]), f64([1.0, 2.0]), i32([n0 - 1, 1]), i32([0, 0]), i64([0, 0, 0]), f64([0.0]),
                     i64([n0, 0]), f64([1.0, np.inf]), f64([2.0, -np.inf]), f64([3.0, 0.0]), f64([1.5, 0.0]))
    ss.ingest(f64([5.0, 6.0, 7.0, 8.0]), i64([0, 3, 4]), sync=False)
    with pytest.raises(Exception, match="count limit|outgrew"):
        ss.sync()
    st = ss.stats()
    assert int(st["n"][0]) == n0  # refused (n and the table belong to the ingest kernels)
    assert int(st["size"][0]) == 2
    assert int(st["n"][1]) == 1 and int(st["pending"][1]) == 1
    # within the limit it is accepted
    ss2 = _ss(1, eps, dev)
    ss2.import_arrays(i64([0, 2]), f64([1.0, 2.0]), i32([n0 - 1, 1]), i32([0, 0]), i64([0, 0]), f64([0.0]),
                      i64([n0]), f64([1.0]), f64([2.0]), f64([3.0]), f64([1.5]))
    ss2.ingest(f64([5.0, 6.0]), i64([0, 2]))
    assert int(ss2.stats()["n"][0]) == lim
