"""ctypes wrapper of oracle/gk_oracle.c -- TEST INFRASTRUCTURE ONLY.

Batched C restatement of the reference GKArray (see gk_oracle.c).  Used by the
parity tests, __graft_entry__.smoke() and the cpu_baseline leg of bench.py.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "libgkoracle.so")

_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            subprocess.run(["make", "-C", HERE], check=True, stdout=subprocess.DEVNULL)
        lib = ctypes.CDLL(SO)
        P = ctypes.c_void_p
        lib.gko_create.restype = P
        lib.gko_create.argtypes = [ctypes.c_int64, ctypes.c_double]
        lib.gko_destroy.argtypes = [P]
        lib.gko_ingest.argtypes = [P, P, P, ctypes.c_int]
        lib.gko_flush.argtypes = [P, ctypes.c_int, ctypes.c_int]
        lib.gko_quantiles.argtypes = [P, P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int]
        lib.gko_merge.argtypes = [P, P, ctypes.c_int]
        lib.gko_stats.argtypes = [P, P, P, P, P, P, P, P]
        lib.gko_export.argtypes = [P, P, P, P, P]
        lib.gko_export_pending.argtypes = [P, P, P]
        lib.gko_max_threads.restype = ctypes.c_int
        _lib = lib
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


class OracleSet:
    """S independent reference GKArray streams (C restatement)."""

    def __init__(self, S, eps, threads=0):
        self.lib = load()
        self.S = int(S)
        self.eps = eps
        self.threads = threads
        self.h = ctypes.c_void_p(self.lib.gko_create(self.S, float(eps)))

    def __del__(self):
        try:
            if self.h:
                self.lib.gko_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def ingest(self, values, offsets):
        v = np.ascontiguousarray(values, dtype=np.float64)
        o = np.ascontiguousarray(offsets, dtype=np.int64)
        assert o.size == self.S + 1
        if v.size == 0:
            v = np.zeros(1)
        self.lib.gko_ingest(self.h, _p(v), _p(o), self.threads)

    def flush(self, force=1):
        self.lib.gko_flush(self.h, force, self.threads)

    def quantiles(self, qs, single=False):
        """quantiles(qs) for every stream (flushes pending values first)."""
        q = np.ascontiguousarray(qs, dtype=np.float64)
        self.flush(1)
        mode = 1 if single else 0
        if not single and np.any(np.diff(q) < 0):
            mode = 1
        out = np.empty((self.S, max(q.size, 1)), dtype=np.float64)
        self.lib.gko_quantiles(self.h, _p(q), q.size, _p(out), mode, self.threads)
        return out[:, :q.size]

    def merge(self, other):
        rc = self.lib.gko_merge(self.h, other.h, self.threads)
        if rc == -2:
            raise ValueError("eps mismatch")
        if rc != 0:
            raise ValueError("stream count mismatch")

    def stats(self):
        S = max(self.S, 1)
        n = np.empty(S, np.int64)
        mn, mx, sm, av = (np.empty(S) for _ in range(4))
        E = np.empty(S, np.int32)
        p = np.empty(S, np.int32)
        self.lib.gko_stats(self.h, _p(n), _p(mn), _p(mx), _p(sm), _p(av), _p(E), _p(p))
        return dict(n=n[:self.S], min=mn[:self.S], max=mx[:self.S], sum=sm[:self.S],
                    avg=av[:self.S], size=E[:self.S], pending=p[:self.S])

    def tables(self):
        st = self.stats()
        offs = np.zeros(self.S + 1, np.int64)
        offs[1:] = np.cumsum(st["size"])
        tot = int(offs[-1])
        v = np.empty(max(tot, 1))
        g = np.empty(max(tot, 1), np.int64)
        d = np.empty(max(tot, 1), np.int64)
        self.lib.gko_export(self.h, _p(offs), _p(v), _p(g), _p(d))
        return offs, v[:tot], g[:tot], d[:tot]

    def pending(self):
        st = self.stats()
        offs = np.zeros(self.S + 1, np.int64)
        offs[1:] = np.cumsum(st["pending"])
        tot = int(offs[-1])
        v = np.empty(max(tot, 1))
        self.lib.gko_export_pending(self.h, _p(offs), _p(v))
        return offs, v[:tot]

    def table(self, s):
        offs, v, g, d = self.tables()
        a, b = offs[s], offs[s + 1]
        return list(zip(v[a:b].tolist(), g[a:b].tolist(), d[a:b].tolist()))
