"""k_ingest_wg (round 4): the longest presorted streams of
a batch run one WORKGROUP per stream (the flush of gk:63-109 shared by 8
waves), beside the one-wave-per-stream class-0 launch, which skips them.

Parity bar: every stream's table, pending values, n/min/max/sum/avg and the
fused quantiles bit-identical to the C oracle and to the same calls with the
path switched off (GK_WG=0), over several calls, in the three presort
modes: the default (GK_WG_PRESORT=1, GK_WG_CONC=1: the register presort runs
BESIDE the workgroups, which rank batches unsorted until it has finished and
always rank a call's first batch -- the one holding pre-call pending values --
unsorted), the presort ahead of the workgroups (GK_WG_CONC=0) and no presort
(GK_WG_PRESORT=0: every batch ranked among its gaps' members); the presort
workspace is sized from the previous call's need, so presorted batches appear
from the second call on.  Pending values are carried
between calls, ties, signed zeros, and one adversarial (descending) long
stream whose table outgrows the 2048 class inside k_ingest_wg (promoted and
re-run in the next class).  GK_WG_TRACE=1 shows on stderr how many streams
the path took per call: it must be > 0."""
import re

import numpy as np
import pytest
import torch

from gk_oracle_c import OracleSet
from parity_util import _ss, assert_same_quantiles, assert_same_state, small_of

pytestmark = pytest.mark.gpu

EPS = 0.001
QS = [0.0, 0.01, 0.5, 0.9, 0.999, 1.0]


def batches(seed):
    """Three calls over 200 streams: 5 long ones (300-700 flushes of 1001
    values per call, >= GK_WG_MIN_FLUSHES = 256), one descending long stream,
    the rest short; lengths not multiples of P (pending values carry over)."""
    rng = np.random.default_rng(seed)
    out = []
    for call in range(3):
        lens = rng.integers(0, 4000, 200)
        lens[:5] = rng.integers(300_000, 700_000, 5)
        lens[7] = 400_000
        seqs = [rng.lognormal(0.0, 1.5, int(L)) for L in lens]
        seqs[1] = np.round(seqs[1], 1)  # ties
        seqs[2][::97] = 0.0
        seqs[2][::89] = -0.0  # signed zeros
        # heavy ties: crowded gaps (the per-gap records path of a sorted batch)
        # and a few values per gap (the entry-side emit)
        seqs[3] = rng.integers(0, 5, int(lens[3])).astype(np.float64)
        seqs[4] = rng.integers(0, 3000, int(lens[4])).astype(np.float64)
        if call > 0:  # descending from the second call (k_ingest_wg's first): outgrows 2048 inside it
            seqs[7] = np.linspace(1e6 - call * 1e5, 1.0 - call * 1e5, int(lens[7]))
        out.append(seqs)
    return out


def run(dev, monkeypatch, env, calls):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ss = _ss(200, EPS, dev)
    res = []
    for seqs in calls:
        offs = np.zeros(201, np.int64)
        offs[1:] = np.cumsum([len(x) for x in seqs])
        x = torch.from_numpy(np.concatenate(seqs)).to(dev)
        q = ss.ingest(x, torch.from_numpy(offs).to(dev), quantiles=QS).cpu().numpy()
        res.append((q, offs))
    return ss, res


@pytest.mark.parametrize("presort,conc,early", [("1", "1", "1"), ("1", "1", "0"), ("1", "0", "1"), ("0", "1", "1")])
def test_wg_streams_match_oracle_and_one_wave_path(gpu_device, monkeypatch, capfd, presort, conc, early):
    """presort 1, conc 1 (the default): presorted batches from the presort
    running beside the workgroups; conc 0: the presort ahead of them;
    presort 0: k_ingest_wg ranks every batch among its gaps' members (and
    sorts a batch with a crowded gap: the descending stream's batches all
    fall below the table).  early 1 (the default): the workgroups launched
    ahead of k_long_prep, spinning on its word; early 0: behind it."""
    calls = batches(5)
    ss, res = run(gpu_device, monkeypatch, {"GK_WG": "1", "GK_WG_TRACE": "1", "GK_WG_PRESORT": presort,
                                            "GK_WG_CONC": conc, "GK_WG_EARLY": early}, calls)
    err = capfd.readouterr().err
    took = [int(m) for m in re.findall(r"k_ingest_wg: (\d+) stream", err)]
    assert took and max(took) > 0, "k_ingest_wg took no stream: %r" % err[-2000:]
    ss_off, res_off = run(gpu_device, monkeypatch, {"GK_WG": "0", "GK_WG_PRESORT": "0", "GK_WG_CONC": "1"}, calls)
    o = OracleSet(200, EPS)
    for (q, offs), (q_off, _), seqs in zip(res, res_off, calls):
        o.ingest(np.concatenate(seqs), offs)
        assert np.array_equal(q.view(np.int64), q_off.view(np.int64)), "wg vs one-wave path quantiles"
        assert_same_quantiles(q, o.quantiles(QS), "wg quantiles vs oracle", small_of(o, EPS))
    assert_same_state(ss, o, "wg path")
    assert_same_state(ss_off, o, "one-wave path")
    assert ss.num_promoted >= 1  # the descending stream left the 2048 class


def test_wg_plain_ingest_then_query(gpu_device, monkeypatch, capfd):
    """Ingest without a fused query (pending values stay pending), then a
    separate quantiles() call flushes them: wg path vs oracle."""
    monkeypatch.setenv("GK_WG", "1")
    monkeypatch.setenv("GK_WG_TRACE", "1")
    rng = np.random.default_rng(9)
    ss = _ss(40, EPS, gpu_device)
    o = OracleSet(40, EPS)
    for call in range(3):
        lens = rng.integers(0, 3000, 40)
        lens[0] = 520_123 + call
        lens[3] = 333_333
        seqs = [rng.random(int(L)) for L in lens]
        offs = np.zeros(41, np.int64)
        offs[1:] = np.cumsum(lens)
        flat = np.concatenate(seqs)
        ss.ingest(torch.from_numpy(flat).to(gpu_device), torch.from_numpy(offs).to(gpu_device))
        o.ingest(flat, offs)
        assert_same_state(ss, o, "call %d" % call)
    took = [int(m) for m in re.findall(r"k_ingest_wg: (\d+) stream", capfd.readouterr().err)]
    assert took and max(took) > 0
    assert_same_quantiles(ss.quantiles(QS).cpu().numpy(), o.quantiles(QS), "final query", small_of(o, EPS))
    assert_same_state(ss, o, "after query")


SERIAL_SCRIPT = r'''
import sys, numpy as np, torch
sys.path[:0] = sys.argv[1].split(":")
from gk_oracle_c import OracleSet
from parity_util import _ss, assert_same_state
dev = torch.device("cuda", 0)
rng = np.random.default_rng(41)
lens = rng.integers(0, 3000, 40)
lens[:3] = [600_000, 450_123, 400_000]
ss = _ss(40, 0.001, dev)
o = OracleSet(40, 0.001)
for call in range(2):
    seqs = [rng.lognormal(0, 1, int(L)) for L in lens]
    offs = np.zeros(41, np.int64)
    offs[1:] = np.cumsum(lens)
    flat = np.concatenate(seqs)
    ss.ingest(torch.from_numpy(flat).to(dev), torch.from_numpy(offs).to(dev))
    o.ingest(flat, offs)
assert_same_state(ss, o, "serialised kernels")
print("OK")
'''


def test_wg_early_launch_survives_serialised_kernels(gpu_device, tmp_path):
    """the early k_ingest_wg grid spins on the device for
    k_long_prep's word.  With every kernel serialised (AMD_SERIALIZE_KERNEL=3,
    as under a profiler's counter passes) k_long_prep cannot run beside it:
    the spin is bounded (1 s), the workgroups leave without a stream, and the
    launch the call enqueues behind k_long_prep takes them -- no hang, the
    same bits as the oracle."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = ":".join([os.path.join(root, "sketches-py_amd"), os.path.join(root, "oracle"),
                      os.path.join(root, "tests")])
    env = dict(os.environ, AMD_SERIALIZE_KERNEL="3", GK_WG="1", GK_WG_EARLY="1", GK_WG_TRACE="1")
    r = subprocess.run([sys.executable, "-c", SERIAL_SCRIPT, paths], capture_output=True, text=True, timeout=240,
                       env=env)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
    took = [int(m) for m in re.findall(r"k_ingest_wg: (\d+) stream", r.stderr)]
    assert took and max(took) > 0, r.stderr[-2000:]
