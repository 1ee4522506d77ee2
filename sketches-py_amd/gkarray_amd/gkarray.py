"""Drop-in ``GKArray`` backed by the MI355X engine.

Mirrors ``gkarray/gkarray.py`` of githomin/sketches-py (``gk:N``): the same
class names (``Entry``, ``GKArray``, ``UnequalEpsilonException``), method
names, argument meaning, return values and errors.  Raw numbers may be passed
to ``add`` directly (the reference evidently intends ``Entry(val, 1, 0)`` for
them).

``add`` appends to a host-side buffer; the buffer is shipped to the GPU in one
``StreamSet.ingest`` call whenever state is observed (``_n``, ``entries``,
``quantile`` ...) or it reaches ``GKArray.SHIP_CHUNK`` values.  Because flush
points depend only on the running count ``n`` (gk:60), batching the adds does
not change any result.  One GKArray = a StreamSet of one stream: use
``StreamSet`` directly to sketch many streams at once.

``entries`` and ``incoming`` are lists materialised from the device, and like
the reference's attributes (gk:23-24) they may be mutated -- ``Entry`` fields,
list items, appends -- or assigned: the next operation on the sketch writes
the changed lists back to the device first (one ``gk_import``).  After that
operation a list obtained before it is detached (the reference detaches
``entries`` only at a flush, gk:108); read the attribute again.
"""
import math

import numpy as np
import torch

from .streamset import StreamSet

__all__ = ["Entry", "GKArray", "UnequalEpsilonException"]


class UnequalEpsilonException(Exception):
    """gk:4-5: raised by merge() when the two eps differ (gk:118-119)."""


class Entry:
    """gk:8-16 -- one (val, g, delta) record."""

    def __init__(self, val, g, delta):
        self.val = val
        self.g = g
        self.delta = delta

    def __repr__(self):
        return 'Entry(val={}, g={}, delta={})'.format(self.val, self.g, self.delta)


def _is_nan(q):
    try:
        return q != q
    except Exception:
        return False


class GKArray:
    SHIP_CHUNK = 1 << 20

    def __init__(self, eps, device=None):
        # gk:21-29
        self.eps = eps
        self._set = StreamSet(1, eps, device)
        self._buf = []
        self._offs = None
        self._views = None  # (entries list, incoming list, snapshot) handed out, not yet written back

    # ---------------------------------------------------------------- plumbing
    def _sync_views(self):
        """Write caller mutations of ``entries`` / ``incoming`` back to the
        device (gk:23-24 are plain attributes in the reference), then detach
        the lists."""
        if self._views is None:
            return
        ents, inc, snap = self._views
        self._views = None
        now = ([(e.val, e.g, e.delta) for e in ents], list(inc))
        if now != snap:
            self._push(now[0], now[1])

    def _push(self, recs, pending):
        """The stream's table := recs [(v, g, delta)], pending := values
        (header words kept): one gk_import."""
        P = self._set.flush_period
        dev = self._set.device
        st = self._set.stats()
        # add() leaves at most n mod P values pending (gk:60): the values added
        # since n last crossed a multiple of P; a longer list has no flush
        # schedule in this engine (one flush batch is at most P values)
        room = int(st["n"][0].item()) % P
        if len(pending) > room:
            raise ValueError("incoming holds %d values; at n=%d at most %d can be pending (n mod %d)"
                             % (len(pending), int(st["n"][0].item()), room, P))
        f64 = lambda a: torch.tensor(a if a else [0.0], dtype=torch.float64, device=dev)
        i32 = lambda a: torch.tensor(a if a else [0], dtype=torch.int32, device=dev)
        i64 = lambda a: torch.tensor(a, dtype=torch.int64, device=dev)
        self._set.import_arrays(i64([0, len(recs)]), f64([float(r[0]) for r in recs]), i32([int(r[1]) for r in recs]),
                                i32([int(r[2]) for r in recs]), i64([0, len(pending)]),
                                f64([float(x) for x in pending]), st["n"].to(torch.int64), st["min"], st["max"],
                                st["sum"], st["avg"])

    def _ship(self):
        self._sync_views()
        if self._buf:
            vals = torch.tensor(self._buf, dtype=torch.float64, device=self._set.device)
            offs = torch.tensor([0, len(self._buf)], dtype=torch.int64, device=self._set.device)
            self._buf = []
            self._set.ingest(vals, offs)

    def _stats(self):
        self._ship()
        st = self._set.stats()
        return {k: v[0].item() for k, v in st.items()}

    @property
    def name(self):
        return 'GKArray'  # gk:31-33

    # reference attributes, read-only views of the device state
    @property
    def _n(self):
        return int(self._stats()["n"])

    @property
    def _min(self):
        return float(self._stats()["min"])

    @property
    def _max(self):
        return float(self._stats()["max"])

    @property
    def _sum(self):
        return float(self._stats()["sum"])

    @property
    def _avg(self):
        return float(self._stats()["avg"])

    # convenience aliases named by the north star (eps is a plain attribute)
    @property
    def count(self):
        return self._n

    @property
    def min(self):
        return self._min

    @property
    def max(self):
        return self._max

    def _materialise(self):
        self._ship()
        ents = [Entry(v, g, d) for (v, g, d) in self._set.table(0)]
        offs, pv = self._set.pending()
        inc = pv.cpu().tolist()
        self._views = (ents, inc, ([(e.val, e.g, e.delta) for e in ents], list(inc)))
        return self._views

    @property
    def entries(self):
        """The table (gk:23) as a list of Entry; does not flush.  Mutations
        are written back by the next operation on the sketch."""
        return self._materialise()[0]

    @entries.setter
    def entries(self, value):
        self._ship()
        offs, pv = self._set.pending()
        self._push([(e.val, e.g, e.delta) for e in value], pv.cpu().tolist())

    @property
    def incoming(self):
        """Pending raw values (gk:24), insertion order; does not flush.
        Mutations are written back by the next operation on the sketch."""
        return self._materialise()[1]

    @incoming.setter
    def incoming(self, value):
        self._ship()
        self._push([(v, g, d) for (v, g, d) in self._set.table(0)], [float(x) for x in value])

    # ---------------------------------------------------------------- accessors
    def num_values(self):
        return self._n  # gk:35-36

    def avg(self):
        return self._avg  # gk:38-39

    def sum(self):
        return self._sum  # gk:41-42

    def size(self):
        # gk:44-47: flush pending values, then the table length
        self._ship()
        self._set.flush()
        return int(self._set.stats()["size"][0].item())

    # ---------------------------------------------------------------- ingest
    def add(self, val):
        """gk:49-61 (buffered; flush points are decided on the GPU)."""
        if self._views is not None:
            self._sync_views()  # caller edits of entries / incoming come first
        self._buf.append(float(val))
        if len(self._buf) >= self.SHIP_CHUNK:
            self._ship()

    def add_many(self, values):
        """Extension: ``for v in values: add(v)`` in one call."""
        self._ship()
        if not isinstance(values, torch.Tensor):
            values = np.ascontiguousarray(values, dtype=np.float64)  # any stride / sequence
        t = torch.as_tensor(values, dtype=torch.float64).reshape(-1)
        if t.numel():
            self._set.ingest(t.to(self._set.device),
                             torch.tensor([0, t.numel()], dtype=torch.int64, device=self._set.device))

    def merge_compress(self, entries=[]):
        """gk:63-109.  With entries, they are merged as records (v, g, delta)."""
        self._ship()
        if not entries:
            self._set.merge_compress()
            return
        recs = [(float(e.val), int(e.g), int(e.delta)) for e in entries]
        # sorted() in gk:72 is stable: records of equal value keep their order
        recs = sorted(recs, key=lambda r: r[0])
        v = torch.tensor([r[0] for r in recs], dtype=torch.float64)
        g = torch.tensor([r[1] for r in recs], dtype=torch.int32)
        d = torch.tensor([r[2] for r in recs], dtype=torch.int32)
        self._set.merge_compress(v, g, d, torch.tensor([0, len(recs)], dtype=torch.int64))

    # ---------------------------------------------------------------- merge
    def merge(self, other):
        """gk:111-154 (flushes `other`, like the reference)."""
        if self.eps != other.eps:
            raise UnequalEpsilonException("Cannot merge two GKArrays with different epsilon values")
        self._ship()
        other._ship()
        self._set.merge_from([other._set])
        self.eps = max(self.eps, other.eps)

    # ---------------------------------------------------------------- query
    def quantile(self, q):
        """gk:156-185."""
        if q < 0 or q > 1:
            return np.nan
        st = self._stats()
        if st["n"] == 0:
            return np.nan
        if _is_nan(q):
            self._set.flush()
            raise ValueError("cannot convert float NaN to integer")
        out = self._set.quantiles([q], single=True)
        return np.float64(out[0, 0].item())

    def quantiles(self, q_values):
        """gk:187-232."""
        st = self._stats()
        if st["n"] == 0:
            return [np.nan] * len(q_values)
        self._set.flush()
        small = st["n"] < 1.0 / self.eps
        qs = list(q_values)
        nan_pos = [k for k, q in enumerate(qs) if _is_nan(q)]
        if small:
            safe = [(-1.0 if _is_nan(q) else float(q)) for q in qs]
            out = self._set.quantiles(safe, single=True)[0].cpu().tolist() if qs else []
            return [np.nan if k in nan_pos else np.float64(v) for k, v in enumerate(out)]
        if isinstance(q_values, np.ndarray):
            # gk:205: `ndarray != list` is an elementwise array; numpy's truth
            # value of it raises unless it has exactly one element
            if q_values.size == 0:
                raise ValueError("The truth value of an empty array is ambiguous. "
                                 "Use `array.size > 0` to check that an array is not empty.")
            if q_values.size > 1:
                raise ValueError("The truth value of an array with more than one element is ambiguous. "
                                 "Use a.any() or a.all()")
            single = bool(nan_pos)  # [nan] != [nan]: per-q quantile(), which raises below
        else:
            # gk:205: a tuple never equals sorted(...) (a list) -> per-q quantile()
            single = (not isinstance(q_values, list)) or (qs != sorted(qs))
        if nan_pos:
            raise ValueError("cannot convert float NaN to integer")
        out = self._set.quantiles([float(q) for q in qs], single=single)[0].cpu().tolist()
        return [np.nan if math.isnan(v) else v for v in out]
