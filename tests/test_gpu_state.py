"""Versioned state files on the GPU path (gk_save / gk_load through the C ABI):
checkpoint mid-stream, restore into a fresh set and continue -- bit-exact vs
an uninterrupted oracle run; import an oracle-produced state file and continue
on the GPU; GPU files read by the numpy reader; eps / stream-count mismatch."""
import numpy as np
import pytest
import torch

from gk_oracle_c import OracleSet
from gkarray_amd import stateio
from parity_util import _ss, assert_same_quantiles, assert_same_state, csr, gen, small_of

pytestmark = pytest.mark.gpu


def batches(S, eps, rng, parts=3):
    P = int(1.0 / eps) + 1
    out = []
    for part in range(parts):
        lens = rng.integers(0, 6 * P, S)
        lens[:4] = [0, 1, P - 1, P]
        seqs = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), lens)]
        out.append(csr(seqs))
    return out


@pytest.mark.parametrize("eps", [0.05, 0.01, 0.001])
def test_checkpoint_restore_continue(gpu_device, tmp_path, eps):
    from gkarray_amd import StreamSet
    rng = np.random.default_rng(71 + int(1 / eps))
    S = 400 if eps >= 0.01 else 80
    bs = batches(S, eps, rng)
    o = OracleSet(S, eps)  # uninterrupted
    a = _ss(S, eps, gpu_device)
    flat, offs = bs[0]
    a.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
    o.ingest(flat, offs)
    p = str(tmp_path / "ckpt.gks")
    a.save(p)
    a.close()
    b = StreamSet.load(p, device=gpu_device)  # fresh set from the file
    assert b.num_streams == S and b.eps == eps
    assert_same_state(b, o, "restored")
    for flat, offs in bs[1:]:
        b.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
        o.ingest(flat, offs)
        assert_same_state(b, o, "continued")
    q = b.quantiles([0.1, 0.5, 0.99]).cpu().numpy()
    assert_same_quantiles(q, o.quantiles([0.1, 0.5, 0.99]), "restored q", small_of(o, eps))


def test_import_oracle_state_file(gpu_device, tmp_path):
    from gkarray_amd import StreamSet
    eps, S = 0.01, 500
    rng = np.random.default_rng(73)
    bs = batches(S, eps, rng, parts=2)
    o = OracleSet(S, eps)
    flat, offs = bs[0]
    o.ingest(flat, offs)
    to, tv, tg, td = o.tables()
    po, pv = o.pending()
    st = o.stats()
    p = str(tmp_path / "oracle.gks")
    stateio.write_state(p, dict(eps=eps, offs=to, v=tv, g=tg, d=td, poffs=po, pv=pv, n=st["n"], min=st["min"],
                                max=st["max"], sum=st["sum"], avg=st["avg"]))
    g = StreamSet.load(p, device=gpu_device)
    assert_same_state(g, o, "imported")
    flat, offs = bs[1]
    q = g.ingest(torch.from_numpy(flat), torch.from_numpy(offs), quantiles=[0.5, 0.9, 0.99]).cpu().numpy()
    o.ingest(flat, offs)
    assert_same_quantiles(q, o.quantiles([0.5, 0.9, 0.99]), "imported q", small_of(o, eps))
    assert_same_state(g, o, "imported + continued")
    # and back: the GPU's file, read by the numpy reader, is the oracle's state
    p2 = str(tmp_path / "gpu.gks")
    g.save(p2)
    r = stateio.read_state(p2)
    to, tv, tg, td = o.tables()
    assert np.array_equal(r["offs"], to) and np.array_equal(r["v"].view(np.int64), tv.view(np.int64))
    assert np.array_equal(r["g"], tg) and np.array_equal(r["d"], td)
    assert np.array_equal(r["avg"].view(np.int64), o.stats()["avg"].view(np.int64))


def test_promoted_streams_roundtrip(gpu_device, tmp_path):
    """Tables beyond the small class (descending streams) survive the file."""
    from gkarray_amd import StreamSet
    rng = np.random.default_rng(79)
    S = 24
    seqs = [np.sort(rng.random(int(L)))[::-1].copy() for L in rng.integers(20000, 40000, S)]
    flat, offs = csr(seqs)
    a = _ss(S, 0.01, gpu_device)
    a.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
    o = OracleSet(S, 0.01)
    o.ingest(flat, offs)
    assert a.num_promoted > 0
    p = str(tmp_path / "big.gks")
    a.save(p)
    b = StreamSet.load(p, device=gpu_device)
    assert_same_state(b, o, "promoted restored")


def test_load_mismatch_errors(gpu_device, tmp_path):
    from gkarray_amd import GKBackendError, StreamSet, UnequalEpsilonException
    a = _ss(10, 0.01, gpu_device)
    a.ingest(torch.rand(1000, dtype=torch.float64), torch.arange(0, 1001, 100))
    p = str(tmp_path / "m.gks")
    a.save(p)
    with pytest.raises(UnequalEpsilonException):
        _ss(10, 0.02, gpu_device).load_state(p)
    with pytest.raises(GKBackendError):
        _ss(11, 0.01, gpu_device).load_state(p)
    raw = bytearray(open(p, "rb").read())
    raw[-3] ^= 0x40
    open(p, "wb").write(bytes(raw))
    with pytest.raises(GKBackendError, match="checksum"):
        StreamSet.load(p, device=gpu_device)


@pytest.mark.parametrize("asynchronous", [False, True])
def test_promotion_arena_exhaustion_defers_and_reruns(gpu_device, monkeypatch, asynchronous):
    """Capacity-class arenas with 2 slots (GK_POOL_SLOTS): most overflowing
    streams find no slot in their next class during the call, are deferred on
    the device and re-run from the call's own inputs before the set's next
    call (or in sync()).  State must equal the oracle's either way."""
    monkeypatch.setenv("GK_POOL_SLOTS", "2")
    rng = np.random.default_rng(83)
    S = 48
    ss = _ss(S, 0.01, gpu_device)
    o = OracleSet(S, 0.01)
    keep = []
    for part in range(3):
        seqs = [np.sort(rng.random(int(L)))[::-1].copy() if k % 3 else rng.random(int(L))
                for k, L in enumerate(rng.integers(5000, 30000, S))]
        flat, offs = csr(seqs)
        tf, to = torch.from_numpy(flat).to(gpu_device), torch.from_numpy(offs).to(gpu_device)
        keep.append((tf, to))  # inputs stay valid until the next call (async contract)
        ss.ingest(tf, to, sync=not asynchronous)
        o.ingest(flat, offs)
    ss.sync()
    assert ss.num_promoted > 2
    assert_same_state(ss, o, "deferred re-run")
    q = ss.quantiles([0.01, 0.5, 0.99]).cpu().numpy()
    assert_same_quantiles(q, o.quantiles([0.01, 0.5, 0.99]), "deferred q", small_of(o, 0.01))


@pytest.mark.parametrize("eps", [0.01, 0.0005])
def test_packed_states_fold_on_gpu(gpu_device, eps):
    """gk_pack / gk_fold_packed through the HIP library: a 3-way rank-ordered
    fold of device packed states == the oracle's left fold (eps = .0005: the
    unbounded class); a host-engine packed state (same bytes) folds on the GPU."""
    from gkarray_amd import StreamSet
    rng = np.random.default_rng(int(7 / eps))
    S = 60 if eps >= 0.01 else 8
    P = int(1 / eps) + 1
    sets, oracles, flats = [], [], []
    for k in range(3):
        seqs = [gen(int(d), int(L), rng) for d, L in zip(rng.integers(0, 8, S), rng.integers(0, 5 * P, S))]
        flat, offs = csr(seqs)
        ss = _ss(S, eps, gpu_device)
        ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
        o = OracleSet(S, eps)
        o.ingest(flat, offs)
        sets.append(ss)
        oracles.append(o)
        flats.append((flat, offs))
    bufs = [s.pack() for s in sets]
    assert bufs[0].device.type == "cuda"
    dst = _ss(S, eps, gpu_device)
    dst.fold_packed(bufs)
    oracles[0].merge(oracles[1])
    oracles[0].merge(oracles[2])
    assert_same_state(dst, oracles[0], "gpu 3-way fold")
    q = dst.quantiles([0.5, 0.99]).cpu().numpy()
    assert_same_quantiles(q, oracles[0].quantiles([0.5, 0.99]), "folded q", small_of(oracles[0], eps))
    # cross-engine: the host engine's packed bytes, moved to the device
    h = StreamSet(S, eps, device="cpu")
    h.ingest(torch.from_numpy(flats[1][0]), torch.from_numpy(flats[1][1]))
    hb = h.pack()
    g2 = _ss(S, eps, gpu_device)
    g2.fold_packed([hb.to(gpu_device)])
    o1 = OracleSet(S, eps)
    o1.ingest(*flats[1])
    assert_same_state(g2, o1, "host-packed on gpu")


def _deferring_batch(S, rng):
    """Streams that outgrow the small class (descending runs): with 2 arena
    slots (GK_POOL_SLOTS) most of them are deferred and re-run later."""
    seqs = [np.sort(rng.random(int(L)))[::-1].copy() if k % 3 else rng.random(int(L))
            for k, L in enumerate(rng.integers(5000, 30000, S))]
    return csr(seqs)


def test_deferred_query_keeps_its_own_qs(gpu_device, monkeypatch):
    """a fused ingest+quantiles call left in flight (sync=False)
    with deferred streams, then quantiles() with a longer q list (> 64: the
    device q buffer is reallocated).  The deferred streams of the first call
    are re-run with the FIRST call's q values into the first output; both
    outputs equal the oracle's."""
    monkeypatch.setenv("GK_POOL_SLOTS", "2")
    rng = np.random.default_rng(85)
    S = 48
    ss = _ss(S, 0.01, gpu_device)
    o = OracleSet(S, 0.01)
    flat, offs = _deferring_batch(S, rng)
    tf, to = torch.from_numpy(flat).to(gpu_device), torch.from_numpy(offs).to(gpu_device)
    q1 = [0.5, 0.9]
    out1 = ss.ingest(tf, to, quantiles=q1, sync=False)
    q2 = [float(x) for x in np.linspace(0.0, 1.0, 70)]
    out2 = ss.quantiles(q2)
    o.ingest(flat, offs)
    e1 = o.quantiles(q1)
    e2 = o.quantiles(q2)
    assert ss.num_promoted > 2
    assert_same_quantiles(out1.cpu().numpy(), e1, "first (deferred) query", small_of(o, 0.01))
    assert_same_quantiles(out2.cpu().numpy(), e2, "second query", small_of(o, 0.01))
    assert_same_state(ss, o, "after both queries")


def test_export_after_async_ingest_sees_deferred_streams(gpu_device, monkeypatch):
    """reads of the state (stats, sizes, tables, pending) right
    after ingest(sync=False) first re-run the call's deferred streams, so an
    export never mixes a deferred stream's old table with its new header."""
    monkeypatch.setenv("GK_POOL_SLOTS", "2")
    rng = np.random.default_rng(86)
    S = 48
    ss = _ss(S, 0.01, gpu_device)
    o = OracleSet(S, 0.01)
    flat, offs = _deferring_batch(S, rng)
    tf, to = torch.from_numpy(flat).to(gpu_device), torch.from_numpy(offs).to(gpu_device)
    ss.ingest(tf, to, sync=False)
    st = ss.export_state()  # no sync() in between
    o.ingest(flat, offs)
    o_off, o_v, o_g, o_d = o.tables()
    assert np.array_equal(st["offs"].cpu().numpy(), o_off)
    assert np.array_equal(st["v"].cpu().numpy().view(np.int64), np.asarray(o_v).view(np.int64))
    assert np.array_equal(st["g"].cpu().numpy(), o_g) and np.array_equal(st["d"].cpu().numpy(), o_d)
    ost = o.stats()
    assert np.array_equal(st["n"].cpu().numpy(), ost["n"])


def test_import_rejects_unreachable_pending(gpu_device):
    """a state whose pending count exceeds n mod P (no sequence
    of adds leaves it; its flush batch would exceed P values) is refused
    before anything is written; the set keeps its state."""
    from gkarray_amd import GKBackendError
    S, eps = 4, 0.01
    P = int(1 / eps) + 1
    rng = np.random.default_rng(87)
    seqs = [rng.random(3 * P + 5) for _ in range(S)]
    ss = _ss(S, eps, gpu_device)
    flat, offs = csr(seqs)
    ss.ingest(torch.from_numpy(flat), torch.from_numpy(offs))
    o = OracleSet(S, eps)
    o.ingest(flat, offs)
    st = ss.export_state()
    bad = dict(st)
    bad["poffs"] = torch.tensor([0, 5, 35, 40, 45], dtype=torch.int64)  # stream 1: 30 pending at n mod P = 5
    bad["pv"] = torch.rand(45, dtype=torch.float64)
    with pytest.raises(GKBackendError, match="pending"):
        ss.import_state(bad)
    assert_same_state(ss, o, "untouched after the refused import")


def test_reset_after_deferring_call_does_not_wait_or_replay(gpu_device, monkeypatch):
    """reset() right after an asynchronous call that deferred streams, then
    another deferring call: the first call's deferred re-run must not land
    after the reset, the last call's deferrals are re-run.  Three async calls
    with resets between them, 2 arena slots (most overflowing streams
    deferred): the state equals an oracle that saw only the last batch."""
    monkeypatch.setenv("GK_POOL_SLOTS", "2")
    rng = np.random.default_rng(87)
    S = 48
    ss = _ss(S, 0.01, gpu_device)
    keep = []
    for part in range(3):
        flat, offs = _deferring_batch(S, rng)
        tf, to = torch.from_numpy(flat).to(gpu_device), torch.from_numpy(offs).to(gpu_device)
        keep.append((tf, to))
        if part:
            ss.reset()
        q = ss.ingest(tf, to, quantiles=[0.25, 0.5, 0.99], sync=False)
    ss.sync()
    o = OracleSet(S, 0.01)
    o.ingest(flat, offs)
    # (the fused query flushes the pending values: the oracle's quantiles() too)
    assert_same_quantiles(q.cpu().numpy(), o.quantiles([0.25, 0.5, 0.99]), "fused q after reset",
                          small_of(o, 0.01))
    assert ss.num_promoted > 2
    assert_same_state(ss, o, "after reset + deferring call")
