"""StreamSet: S independent GKArray streams on one MI355X, batched.

Every stream behaves exactly like one reference ``GKArray`` (gkarray.py,
``gk:N``) fed the same values in the same order.  All work runs in the HIP
kernels of ``libgkarray_hip.so`` through the C ABI of ``include/gk_capi.h``;
PyTorch only allocates device tensors and supplies the current HIP stream.
"""
import contextlib
import ctypes
import os

import torch

from . import _lib as L

__all__ = ["StreamSet", "peek"]


def peek(path, cpu=False):
    """(eps, num_streams) from a GKSTATE file's header."""
    lib = L.load_cpu() if cpu else L.load()
    eps = ctypes.c_double()
    S = ctypes.c_int64()
    L.check(lib.gk_peek(os.fsencode(path), ctypes.byref(eps), ctypes.byref(S)), lib)
    return eps.value, S.value


def _stream_ptr(device):
    if device.type != "cuda":
        return None
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class StreamSet:
    """A batch of ``num_streams`` GKArray sketches sharing one ``eps``.

    ``ingest(values, offsets)`` is the batched ``add`` (gk:49-61): stream ``s``
    receives ``values[offsets[s]:offsets[s+1]]`` in order.
    """

    def __init__(self, num_streams, eps, device=None, cap_hint=0):
        """``device``: a cuda (HIP) device -- the MI355X engine, the default --
        or ``"cpu"`` for the host engine (libgkarray_cpu.so, same C ABI and
        results, multi-threaded over streams).  There is no implicit fallback
        from the GPU to the host engine."""
        if device is not None and torch.device(device).type == "cpu":
            self._lib = L.load_cpu()
            device = torch.device("cpu")
            dev_index = -1
        else:
            if not torch.cuda.is_available():
                raise L.GKBackendError(L.GK_E_HIP, "no GPU visible (the host engine is StreamSet(..., device='cpu'))")
            self._lib = L.load()
            if device is None:
                device = torch.device("cuda", torch.cuda.current_device())
            device = torch.device(device)
            if device.type != "cuda":
                raise ValueError("StreamSet needs a cuda (HIP) device or 'cpu', got %s" % device)
            if device.index is None:
                device = torch.device("cuda", torch.cuda.current_device())
            dev_index = device.index
        self.device = device
        self.num_streams = int(num_streams)
        self.eps = eps
        h = ctypes.c_void_p()
        with self._ctx():
            self._check(self._lib.gk_create(self.num_streams, float(eps), int(cap_hint), dev_index, ctypes.byref(h)))
        self._h = h

    @property
    def is_cpu(self):
        return self.device.type == "cpu"

    def _ctx(self):
        # (no device switch when the set's device is already current: the
        # context manager's get/set round trip is host time on every call)
        if self.device.type == "cpu" or torch.cuda.current_device() == self.device.index:
            return contextlib.nullcontext()
        return torch.cuda.device(self.device)

    def _check(self, rc):
        return L.check(rc, self._lib)

    def set_threads(self, threads):
        """Host threads of the CPU engine (0 = every CPU this process may use)."""
        if not self.is_cpu:
            raise ValueError("set_threads applies to the CPU engine only")
        self._check(self._lib.gk_cpu_set_threads(self._h, int(threads)))

    # ------------------------------------------------------------------ basics
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.gk_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @property
    def flush_period(self):
        return self._lib.gk_flush_period(self._h)

    def capacity(self, cls=0):
        return self._lib.gk_capacity(self._h, cls)

    @property
    def num_promoted(self):
        return self._lib.gk_num_promoted(self._h)

    @property
    def host_chains_taken(self):
        """Streams whose _sum/_avg chains the host walked in the last
        completed ingest (diagnostics; waits for the set's host worker)."""
        return self._lib.gk_host_chains_taken(self._h)

    def _sp(self):
        return _stream_ptr(self.device)

    def _dev(self, t, dtype):
        t = torch.as_tensor(t, dtype=dtype)
        if t.device != self.device:
            t = t.to(self.device)
        return t.contiguous()

    # ------------------------------------------------------------------ ingest
    def reset(self):
        """Every stream back to ``GKArray(eps)`` (gk:21-29)."""
        with self._ctx():
            self._check(self._lib.gk_reset(self._h, self._sp()))

    def sync(self):
        """Wait for this set's work on the current stream; raise an
        asynchronous error of an earlier call (a stream that outgrew every
        table capacity class keeps its previous state: GK_E_OVERFLOW)."""
        with self._ctx():
            try:
                self._check(self._lib.gk_sync(self._h, self._sp()))
            finally:
                self._inflight = None  # the last call's inputs are no longer read

    def ingest(self, values, offsets, quantiles=None, single=False, sync=True):
        """Batched ``GKArray.add`` (gk:49-61) over all streams.

        values: float64 [N] (device tensor preferred); offsets: int64 [S+1].
        With ``quantiles=qs`` the call continues with ``quantiles(qs)``
        (gk:187-232) for every stream in the same kernel pass (the leftover
        pending values are flushed, as the reference's quantiles() does) and
        returns the [S, len(qs)] float64 device tensor.
        ``sync=False`` only enqueues the work on the current HIP stream (the
        C ABI itself never blocks here); errors then surface at a later call
        or ``sync()``.
        """
        v = self._dev(values, torch.float64)
        o = self._dev(offsets, torch.int64)
        if o.numel() != self.num_streams + 1:
            raise ValueError("offsets must have num_streams+1 entries")
        if v.numel() == 0:
            v = torch.zeros(1, dtype=torch.float64, device=self.device)
        if quantiles is None:
            with self._ctx():
                self._check(self._lib.gk_ingest(self._h, _ptr(v), _ptr(o), self._sp()))
            # gk_capi.h: the inputs stay valid until the set's next call or
            # gk_sync (a deferred stream is re-run from them)
            self._inflight = (v, o)
            if sync:
                self.sync()
            return None
        qs = [float(q) for q in quantiles]
        nq = len(qs)
        out = torch.empty((self.num_streams, max(nq, 1)), dtype=torch.float64, device=self.device)
        arr = (ctypes.c_double * max(nq, 1))(*qs)
        mode = L.GK_Q_SINGLE if single else L.GK_Q_LIST
        with self._ctx():
            self._check(self._lib.gk_ingest_quantiles(self._h, _ptr(v), _ptr(o), arr, nq, _ptr(out), mode,
                                                  self._sp()))
        self._inflight = (v, o, out)
        if sync:
            self.sync()
        return out[:, :nq]

    def ingest_lists(self, seqs):
        """Convenience: ``seqs[s]`` is the list of values for stream s."""
        if len(seqs) != self.num_streams:
            raise ValueError("need one sequence per stream")
        lens = [len(x) for x in seqs]
        offs = [0]
        for n in lens:
            offs.append(offs[-1] + n)
        flat = [float(x) for s in seqs for x in s]
        self.ingest(torch.tensor(flat, dtype=torch.float64), torch.tensor(offs, dtype=torch.int64))

    def flush(self):
        """``merge_compress()`` where values are pending (gk:45-46, 166, 197)."""
        with self._ctx():
            self._check(self._lib.gk_flush(self._h, self._sp()))
        self.sync()

    # ------------------------------------------------------------------ query
    def quantiles(self, qs, single=False):
        """Batched ``GKArray.quantiles(qs)`` (gk:187-232); ``single=True``
        gives ``quantile(q)`` semantics for every q (gk:156-185).

        Returns a float64 device tensor [S, len(qs)].  Flushes pending values.
        """
        qs = [float(q) for q in qs]
        nq = len(qs)
        out = torch.empty((self.num_streams, max(nq, 1)), dtype=torch.float64, device=self.device)
        if nq == 0:
            return out[:, :0]
        arr = (ctypes.c_double * nq)(*qs)
        mode = L.GK_Q_SINGLE if single else L.GK_Q_LIST
        with self._ctx():
            self._check(self._lib.gk_quantiles(self._h, arr, nq, _ptr(out), mode, self._sp()))
        self.sync()
        return out

    def stats(self):
        """num_values/_min/_max/sum/avg (gk:25-42) and table / pending sizes,
        without flushing.  Dict of device tensors of length S."""
        S = max(self.num_streams, 1)
        d = dict(
            n=torch.empty(S, dtype=torch.int64, device=self.device),
            min=torch.empty(S, dtype=torch.float64, device=self.device),
            max=torch.empty(S, dtype=torch.float64, device=self.device),
            sum=torch.empty(S, dtype=torch.float64, device=self.device),
            avg=torch.empty(S, dtype=torch.float64, device=self.device),
            size=torch.empty(S, dtype=torch.int32, device=self.device),
            pending=torch.empty(S, dtype=torch.int32, device=self.device),
        )
        with self._ctx():
            self._check(self._lib.gk_stats(self._h, _ptr(d["n"]), _ptr(d["min"]), _ptr(d["max"]),
                                       _ptr(d["sum"]), _ptr(d["avg"]), _ptr(d["size"]),
                                       _ptr(d["pending"]), self._sp()))
        if self.num_streams == 0:
            d = {k: v[:0] for k, v in d.items()}
        return d

    # ------------------------------------------------------------------ export
    def tables(self):
        """All tables in CSR form: (offs int64[S+1], v f64, g i32, d i32)."""
        S = self.num_streams
        sizes = torch.empty(max(S, 1), dtype=torch.int32, device=self.device)
        with self._ctx():
            self._check(self._lib.gk_export_sizes(self._h, _ptr(sizes), self._sp()))
        sizes = sizes[:S]
        offs = torch.zeros(S + 1, dtype=torch.int64, device=self.device)
        if S:
            offs[1:] = torch.cumsum(sizes.to(torch.int64), 0)
        tot = int(offs[-1].item()) if S else 0
        v = torch.empty(max(tot, 1), dtype=torch.float64, device=self.device)
        g = torch.empty(max(tot, 1), dtype=torch.int32, device=self.device)
        d = torch.empty(max(tot, 1), dtype=torch.int32, device=self.device)
        with self._ctx():
            self._check(self._lib.gk_export(self._h, _ptr(offs), _ptr(v), _ptr(g), _ptr(d), self._sp()))
        return offs, v[:tot], g[:tot], d[:tot]

    def pending(self):
        """All pending (incoming) values in CSR form: (poffs int64[S+1], pv f64)."""
        S = self.num_streams
        sizes = torch.empty(max(S, 1), dtype=torch.int32, device=self.device)
        with self._ctx():
            self._check(self._lib.gk_export_pending_sizes(self._h, _ptr(sizes), self._sp()))
        sizes = sizes[:S]
        offs = torch.zeros(S + 1, dtype=torch.int64, device=self.device)
        if S:
            offs[1:] = torch.cumsum(sizes.to(torch.int64), 0)
        tot = int(offs[-1].item()) if S else 0
        pv = torch.empty(max(tot, 1), dtype=torch.float64, device=self.device)
        with self._ctx():
            self._check(self._lib.gk_export_pending(self._h, _ptr(offs), _ptr(pv), self._sp()))
        return offs, pv[:tot]

    def table(self, s):
        """Stream s's table as a list of (v, g, d) (the reference's entries)."""
        offs, v, g, d = self.tables()
        a, b = int(offs[s]), int(offs[s + 1])
        vv, gg, dd = v[a:b].cpu().tolist(), g[a:b].cpu().tolist(), d[a:b].cpu().tolist()
        return list(zip(vv, gg, dd))

    def export_state(self):
        """Full state (checkpoint / RCCL payload) as a dict of device tensors."""
        offs, v, g, d = self.tables()
        poffs, pv = self.pending()
        st = self.stats()
        return dict(eps=self.eps, offs=offs, v=v, g=g, d=d, poffs=poffs, pv=pv,
                    n=st["n"], min=st["min"], max=st["max"], sum=st["sum"], avg=st["avg"])

    def import_state(self, state):
        """Inverse of export_state (replaces every stream's state)."""
        if state["eps"] != self.eps:
            raise ValueError("eps mismatch on import")
        t = {k: self._dev(state[k], dt) for k, dt in (
            ("offs", torch.int64), ("v", torch.float64), ("g", torch.int32), ("d", torch.int32),
            ("poffs", torch.int64), ("pv", torch.float64), ("n", torch.int64),
            ("min", torch.float64), ("max", torch.float64), ("sum", torch.float64),
            ("avg", torch.float64))}
        for k in ("v", "g", "d", "pv"):
            if t[k].numel() == 0:
                t[k] = torch.zeros(1, dtype=t[k].dtype, device=self.device)
        with self._ctx():
            self._check(self._lib.gk_import(self._h, _ptr(t["offs"]), _ptr(t["v"]), _ptr(t["g"]),
                                        _ptr(t["d"]), _ptr(t["poffs"]), _ptr(t["pv"]),
                                        _ptr(t["n"]), _ptr(t["min"]), _ptr(t["max"]),
                                        _ptr(t["sum"]), _ptr(t["avg"]), self._sp()))

    # ------------------------------------------------------------------ files
    def save(self, path):
        """Write every stream's state (tables, pending values, n/min/max/sum/avg)
        to a versioned GKSTATE file (csrc/gk_format.h) without flushing."""
        with self._ctx():
            self._check(self._lib.gk_save(self._h, os.fsencode(path), self._sp()))

    def load_state(self, path):
        """Replace every stream's state with a GKSTATE file's (same stream
        count and eps as this set)."""
        with self._ctx():
            rc = self._lib.gk_load(self._h, os.fsencode(path), self._sp())
        if rc == L.GK_E_EPS_MISMATCH:
            from .gkarray import UnequalEpsilonException
            raise UnequalEpsilonException(L.last_error(self._lib))
        self._check(rc)

    @classmethod
    def load(cls, path, device=None):
        """A new StreamSet holding the state saved in ``path``."""
        eps, S = peek(path, cpu=device is not None and torch.device(device).type == "cpu")
        ss = cls(S, eps, device=device)
        ss.load_state(path)
        return ss

    def import_arrays(self, offs, v, g, d, poffs, pv, n, mn, mx, sm, av):
        """``gk_import`` on device tensors as they are (no copies): stream s's
        table is ``v/g/d[offs[s]:offs[s+1]]`` -- offsets may be absolute into
        a larger array (a slice of another set's export) -- and its pending
        values ``pv[poffs[s]:poffs[s+1]]``; header arrays have S entries."""
        with self._ctx():
            self._check(self._lib.gk_import(self._h, _ptr(offs), _ptr(v), _ptr(g), _ptr(d), _ptr(poffs), _ptr(pv),
                                            _ptr(n), _ptr(mn), _ptr(mx), _ptr(sm), _ptr(av), self._sp()))

    def export_sizes(self):
        """Device tensors (table sizes int32[S], pending counts int32[S]) -- no host sync."""
        S = max(self.num_streams, 1)
        e = torch.empty(S, dtype=torch.int32, device=self.device)
        p = torch.empty(S, dtype=torch.int32, device=self.device)
        with self._ctx():
            self._check(self._lib.gk_export_sizes(self._h, _ptr(e), self._sp()))
            self._check(self._lib.gk_export_pending_sizes(self._h, _ptr(p), self._sp()))
        return e[:self.num_streams], p[:self.num_streams]

    def export_into(self, offs, v, g, d, poffs, pv):
        """Tables / pending values into caller buffers at the given offsets (device, no host sync)."""
        with self._ctx():
            self._check(self._lib.gk_export(self._h, _ptr(offs), _ptr(v), _ptr(g), _ptr(d), self._sp()))
            self._check(self._lib.gk_export_pending(self._h, _ptr(poffs), _ptr(pv), self._sp()))

    # ------------------------------------------------------------------ merge
    def merge_from(self, others):
        """Left fold ``self.merge(others[0]); self.merge(others[1]); ...``
        stream by stream (gk:111-154).  Each source is flushed (mutated)."""
        if isinstance(others, StreamSet):
            others = [others]
        for o in others:
            if o.eps != self.eps:
                from .gkarray import UnequalEpsilonException
                raise UnequalEpsilonException("Cannot merge two GKArrays with different epsilon values")
        for o in others:
            if o.is_cpu != self.is_cpu:
                raise ValueError("cannot merge a CPU-engine set with a GPU-engine set (export / import the state)")
        arr = (ctypes.c_void_p * max(len(others), 1))(*[o._h for o in others])
        with self._ctx():
            rc = self._lib.gk_merge(self._h, arr, len(others), self._sp())
        if rc == L.GK_E_EPS_MISMATCH:
            from .gkarray import UnequalEpsilonException
            raise UnequalEpsilonException("Cannot merge two GKArrays with different epsilon values")
        self._check(rc)

    # ---- packed state (gk_pack_bytes / gk_pack / gk_fold_packed) -------------
    def pack_bytes(self):
        """Size of this set's packed state (one contiguous buffer: header
        words, tables, pending values; layout in csrc/gk_pack.h)."""
        b = ctypes.c_int64(0)
        with self._ctx():
            self._check(self._lib.gk_pack_bytes(self._h, ctypes.byref(b), self._sp()))
        return b.value

    def pack(self, buf=None):
        """The packed state as a uint8 tensor on the set's device (host for
        the CPU engine).  ``buf``: a uint8 tensor of at least pack_bytes()
        bytes to write into (e.g. an equal-sized all-gather slot)."""
        if buf is None:
            buf = torch.empty(self.pack_bytes(), dtype=torch.uint8, device=self.device)
        if buf.dtype != torch.uint8 or not buf.is_contiguous():
            raise ValueError("buf must be a contiguous uint8 tensor")
        with self._ctx():
            self._check(self._lib.gk_pack(self._h, _ptr(buf), buf.numel(), self._sp()))
        return buf

    def fold_packed(self, bufs):
        """self := bufs[0], then self.merge(bufs[r]) for r = 1.. (gk:111-154,
        every stream): the rank-ordered fold of packed states."""
        bufs = [b if b.device == torch.device(self.device) else b.to(self.device) for b in bufs]
        arr = (ctypes.c_void_p * max(len(bufs), 1))(*[b.data_ptr() for b in bufs])
        with self._ctx():
            rc = self._lib.gk_fold_packed(self._h, arr, len(bufs), self._sp())
        if rc == L.GK_E_EPS_MISMATCH:
            from .gkarray import UnequalEpsilonException
            raise UnequalEpsilonException("Cannot merge two GKArrays with different epsilon values")
        self._check(rc)

    def merge_compress(self, v=None, g=None, d=None, eoffs=None):
        """``merge_compress(entries)`` (gk:63-109) on every stream; stream s
        merges records [eoffs[s], eoffs[s+1]) (sorted by value).  With no
        records this is the unconditional ``merge_compress()``."""
        S = self.num_streams
        if eoffs is None:
            eoffs = torch.zeros(S + 1, dtype=torch.int64)
            v = torch.zeros(1, dtype=torch.float64)
            g = torch.zeros(1, dtype=torch.int32)
            d = torch.zeros(1, dtype=torch.int32)
        t_o = self._dev(eoffs, torch.int64)
        t_v = self._dev(v, torch.float64)
        t_g = self._dev(g, torch.int32)
        t_d = self._dev(d, torch.int32)
        if t_v.numel() == 0:
            t_v = torch.zeros(1, dtype=torch.float64, device=self.device)
            t_g = torch.zeros(1, dtype=torch.int32, device=self.device)
            t_d = torch.zeros(1, dtype=torch.int32, device=self.device)
        with self._ctx():
            self._check(self._lib.gk_merge_compress(self._h, _ptr(t_v), _ptr(t_g), _ptr(t_d),
                                                _ptr(t_o), self._sp()))

    # ------------------------------------------------------------------ timing
    def timing(self, on=True, stats=False):
        """HIP events around the ingest launch (and, stats=True, around the
        call's stats fork: two more event markers per call)."""
        self._check(self._lib.gk_timing_enable(self._h, (1 | (2 if stats else 0)) if on else 0))

    def read_timing(self):
        f = ctypes.c_double()
        s = ctypes.c_double()
        n = ctypes.c_int64()
        self._check(self._lib.gk_timing_read(self._h, ctypes.byref(f), ctypes.byref(s), ctypes.byref(n)))
        return f.value, s.value, n.value
