"""The speculative walk of the long streams' gk:52-59 chains (k_stats_long,
DESIGN.md section 5, round 4): supersteps of 64 x GK_SPEC_W values whose
_sum/_avg chains run on all 64 lanes from estimated starts, are shifted onto
the true chain by a lane scan and checked step by step, bit for bit.

Parity bar: n/_sum/_avg/_min/_max bit-identical to the C oracle for streams
past the long-stream limit (16 384 values) with every value distribution the
parity suite uses plus the ones that make the speculation fail (signed
magnitudes over e^+-50: several rounds per superstep; infinities and a NaN:
the round limit hands the superstep, and after four in a row the rest of the
stream, to the one-at-a-time walk; an isolated burst superstep), over two calls
(the second starts from a non-trivial pre-call n/_sum/_avg), lengths around
the superstep size, and with the host walk off (every chain on the device)."""
import numpy as np
import pytest
import torch

from gk_oracle_c import OracleSet
from parity_util import _ss, assert_same_tables, gen

pytestmark = pytest.mark.gpu

EPS = 0.001


def batch(seed):
    rng = np.random.default_rng(seed)
    seqs = []
    lens = [16_385, 16_384 + 1024, 17_407, 20_000, 65_536, 100_003, 250_000]
    for i in range(40):
        L = lens[i % len(lens)] + (seed - 1) * 333
        d = i % 11
        if d < 8:
            x = gen(d, L, rng)
        elif d == 8:  # signed magnitudes over e^+-50
            x = rng.choice([-1.0, 1.0], L) * np.exp(rng.uniform(-50, 50, L))
        elif d == 9:  # heavy tail with zeros of both signs
            x = rng.pareto(0.8, L)
            x[rng.random(L) < 0.2] = 0.0
            x[rng.random(L) < 0.2] = -0.0
        else:  # mean near zero: the _avg update is dominated by (v - avg)
            x = rng.normal(0.0, 1.0, L) * 1e-3
        seqs.append(np.asarray(x, np.float64))
    seqs[3][5000] = np.inf
    seqs[14][16000] = -np.inf
    seqs[25][12] = np.nan
    seqs[36][:] = 1e308  # the _sum overflows to inf part-way
    seqs += [rng.random(int(L)) for L in rng.integers(0, 3000, 24)]  # short streams beside them
    # one superstep of +-1e20 bursts (each lane's chain absorbs its start
    # there: every lane fails once, past the round limit) amid lognormal
    # values: that superstep is walked one at a time, the speculation resumes
    # after it (round 5; before, the whole rest of the stream was walked)
    burst = rng.lognormal(0.0, 1.0, 20_000 + (seed - 1) * 333)
    blk = burst[2048:3072]
    blk[0::4] = 1e20
    blk[2::4] = -1e20
    seqs[-1] = burst
    return seqs


def test_spec_chain_matches_oracle(gpu_device, monkeypatch):
    monkeypatch.setenv("GK_HOST_CHAINS", "0")
    S = 64
    ss = _ss(S, EPS, gpu_device)
    o = OracleSet(S, EPS)
    for seed in (1, 2):
        seqs = batch(seed)
        assert len(seqs) == S
        offs = np.zeros(S + 1, np.int64)
        offs[1:] = np.cumsum([len(x) for x in seqs])
        flat = np.concatenate(seqs)
        ss.ingest(torch.from_numpy(flat).to(gpu_device), torch.from_numpy(offs).to(gpu_device))
        o.ingest(flat, offs)
        st = {k: v.cpu().numpy() for k, v in ss.stats().items()}
        ost = o.stats()
        for k in ("sum", "avg", "min", "max"):
            bad = np.nonzero(st[k].view(np.int64) != ost[k].view(np.int64))[0]
            assert bad.size == 0, "call %d %s: streams %s got %r want %r" % (
                seed, k, bad[:5].tolist(), st[k][bad[:3]].tolist(), ost[k][bad[:3]].tolist())
        assert np.array_equal(st["n"].astype(np.int64), ost["n"].astype(np.int64))
        # (stream 25 holds a NaN: stats only, NaN inputs to the flush are unsupported)
        assert_same_tables(ss, o, ids=[i for i in range(S) if i != 25], what="call %d" % seed)


def test_spec_chain_cfg5_like_lengths(gpu_device, monkeypatch):
    """A few streams of 10^6 - 3*10^6 lognormal values (cfg5's long tail) in
    one call with the host walk off: every stat bit-exact."""
    monkeypatch.setenv("GK_HOST_CHAINS", "0")
    rng = np.random.default_rng(11)
    lens = [3_000_000, 1_000_001, 2_222_222, 40_000] + list(rng.integers(0, 5000, 12))
    seqs = [rng.lognormal(0.0, 1.0, int(L)) for L in lens]
    S = len(seqs)
    offs = np.zeros(S + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    flat = np.concatenate(seqs)
    ss = _ss(S, EPS, gpu_device)
    ss.ingest(torch.from_numpy(flat).to(gpu_device), torch.from_numpy(offs).to(gpu_device))
    o = OracleSet(S, EPS)
    o.ingest(flat, offs)
    st = {k: v.cpu().numpy() for k, v in ss.stats().items()}
    ost = o.stats()
    for k in ("sum", "avg", "min", "max"):
        assert np.array_equal(st[k].view(np.int64), ost[k].view(np.int64)), k
