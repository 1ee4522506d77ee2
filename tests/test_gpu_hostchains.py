"""Host-walked chains: the gk:52-59 `_sum`/`_avg`/`_min`/
`_max` chains of the longest streams of a batch run on host cores (the host
engine's step, cpu/gk_host_stats.h) while the GPU ingests; k_stats_long skips
them and k_hc_apply writes the host's results back.

The threshold is lowered (GK_HOST_CHAIN_MIN) so that a small batch exercises
the path: every stat must equal the C oracle's bit for bit and the run with
the path switched off (GK_HOST_CHAINS=0), across two calls (the second
starts from a non-trivial pre-call state), with signed zeros, infinities and
a NaN in the host-walked streams, and with a fused quantile query (answered
for the long streams after the host results are applied).

Round 4: the host walk is off by default (GK_HOST_CHAINS=1 or
GK_HOST_CHAIN_MIN turns it on): k_stats_long's speculative walk is faster.
When on, it is asynchronous (a worker thread of the set, joined on
the caller's stream by k_hc_wait): gk_ingest returns before the ingest kernel
completes; the number of streams the host took is asserted; a
failed host walk (GK_HC_FAIL=1 injects one) is walked on the device instead
(k_hc_fallback), with the same bits.
"""
import time

import numpy as np
import pytest
import torch

from gk_oracle_c import OracleSet
from parity_util import _ss, assert_same_quantiles, small_of

pytestmark = pytest.mark.gpu

QS = [0.0, 0.25, 0.5, 0.99, 1.0]
STATS = ("min", "max", "sum", "avg")


def batch(seed):
    """300 streams at eps = 0.001: 24 long ones (20k-150k values, past the
    16384-value long-stream limit), the rest short; special values in some
    long streams."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 3000, 300)
    lens[:24] = rng.integers(20_000, 150_000, 24)
    lens[5] = 0
    seqs = [rng.lognormal(0.0, 2.0, int(L)) for L in lens]
    seqs[1][[3, 1000, 5000]] = [-0.0, 0.0, -0.0]
    seqs[2][7] = np.inf
    seqs[3][100] = -np.inf
    seqs[4][[0, 12345]] = [np.nan, -1e300]
    seqs[6][:] = 0.0
    return seqs


def run(dev, monkeypatch, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ss = _ss(300, 0.001, dev)
    out = []
    for seed in (1, 2):
        seqs = batch(seed)
        offs = np.zeros(len(seqs) + 1, np.int64)
        offs[1:] = np.cumsum([len(x) for x in seqs])
        x = torch.from_numpy(np.concatenate(seqs)).to(dev)
        q = ss.ingest(x, torch.from_numpy(offs).to(dev), quantiles=QS).cpu().numpy()
        st = {k: t.cpu().numpy() for k, t in ss.stats().items()}
        st["taken"] = ss.host_chains_taken
        out.append((seqs, offs, q, st))
    return out


def bits(a):
    return np.asarray(a, np.float64).view(np.int64)


@pytest.mark.parametrize("threads", ["1", "4"])
def test_host_chains_match_oracle_and_device_path(gpu_device, monkeypatch, threads):
    host = run(gpu_device, monkeypatch, {"GK_HOST_CHAIN_MIN": "50000", "GK_HOST_CHAIN_THREADS": threads})
    dev = run(gpu_device, monkeypatch, {"GK_HOST_CHAINS": "0"})
    o = OracleSet(300, 0.001)
    for (seqs, offs, q, st), (_, _, qd, std) in zip(host, dev):
        assert st["taken"] > 0, "the host walked no chain"
        assert std["taken"] == 0
        o.ingest(np.concatenate(seqs), offs)
        ost = o.stats()
        for k in STATS:
            assert np.array_equal(bits(st[k]), bits(ost[k])), "host chains vs oracle: %s" % k
            assert np.array_equal(bits(st[k]), bits(std[k])), "host chains vs device chains: %s" % k
        assert np.array_equal(st["n"].astype(np.int64), ost["n"].astype(np.int64))
        keep = np.arange(300) != 4  # (stream 4 holds a NaN: stats only)
        assert_same_quantiles(q[keep], o.quantiles(QS)[keep], "fused quantiles", small_of(o, 0.001))
        assert np.array_equal(bits(q), bits(qd)), "quantiles: host chains vs device chains"


def test_host_chains_take_only_the_longest(gpu_device, monkeypatch):
    """With one host thread the per-call budget is 4 x the longest length:
    the rest of the long list stays on the device; the results do not depend
    on where the split falls."""
    host = run(gpu_device, monkeypatch, {"GK_HOST_CHAIN_MIN": "20000", "GK_HOST_CHAIN_THREADS": "1"})
    o = OracleSet(300, 0.001)
    for seqs, offs, q, st in host:
        assert 0 < st["taken"] < 24, st["taken"]  # 24 long streams, budget 4 x the longest
        o.ingest(np.concatenate(seqs), offs)
        ost = o.stats()
        for k in STATS:
            assert np.array_equal(bits(st[k]), bits(ost[k])), k


def test_failed_host_walk_is_walked_on_the_device(gpu_device, monkeypatch):
    """GK_HC_FAIL=1: the worker reports a failure after its walk; k_hc_wait
    sees status 2, k_hc_apply skips the records and k_hc_fallback walks the
    picked streams on the device -- same bits as the oracle and as the device
    path, and no error surfaces (the set is not broken)."""
    bad = run(gpu_device, monkeypatch, {"GK_HOST_CHAIN_MIN": "50000", "GK_HOST_CHAIN_THREADS": "2",
                                        "GK_HC_FAIL": "1"})
    monkeypatch.delenv("GK_HC_FAIL")
    dev = run(gpu_device, monkeypatch, {"GK_HOST_CHAINS": "0"})
    o = OracleSet(300, 0.001)
    for (seqs, offs, q, st), (_, _, qd, std) in zip(bad, dev):
        assert st["taken"] == 0
        o.ingest(np.concatenate(seqs), offs)
        ost = o.stats()
        for k in STATS:
            assert np.array_equal(bits(st[k]), bits(ost[k])), "fallback vs oracle: %s" % k
            assert np.array_equal(bits(st[k]), bits(std[k])), "fallback vs device chains: %s" % k
        assert np.array_equal(bits(q), bits(qd)), "quantiles: fallback vs device chains"


def test_ingest_with_host_chains_returns_before_the_kernel(gpu_device, monkeypatch):
    """with host chains on (GK_HOST_CHAINS=1; off by
    default since the device walk became speculative) and a stream past their
    threshold (2^20 values, the default) in the batch, gk_ingest_quantiles
    only enqueues -- it returns while the ingest is still running on the
    device -- and the joined results are exact."""
    monkeypatch.delenv("GK_HOST_CHAIN_MIN", raising=False)
    monkeypatch.setenv("GK_HOST_CHAINS", "1")
    rng = np.random.default_rng(77)
    lens = rng.integers(1, 2000, 64)
    lens[0] = 3 << 20
    seqs = [rng.lognormal(0.0, 1.0, int(L)) for L in lens]
    offs = np.zeros(65, np.int64)
    offs[1:] = np.cumsum(lens)
    x = torch.from_numpy(np.concatenate(seqs)).to(gpu_device)
    o_t = torch.from_numpy(offs).to(gpu_device)
    ss = _ss(64, 0.001, gpu_device)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    q = ss.ingest(x, o_t, quantiles=QS, sync=False)
    dt = time.perf_counter() - t0
    busy = not torch.cuda.current_stream(gpu_device).query()
    ss.sync()
    total = time.perf_counter() - t0
    assert busy, "the call returned after the device work had finished (%.1f ms, total %.1f ms)" % (
        dt * 1e3, total * 1e3)
    # taken == 1 only if the worker's walk was the one applied: a join that
    # timed out (20 s) and fell back to the device walk reports 0
    assert ss.host_chains_taken == 1
    assert total < 10.0, "the call's work took %.1f s (the host-chain join is bounded at 20 s)" % total
    o = OracleSet(64, 0.001)
    o.ingest(np.concatenate(seqs), offs)
    ost = o.stats()
    st = {k: t.cpu().numpy() for k, t in ss.stats().items()}
    for k in STATS:
        assert np.array_equal(bits(st[k]), bits(ost[k])), k
    assert_same_quantiles(q.cpu().numpy(), o.quantiles(QS), "fused quantiles", small_of(o, 0.001))
