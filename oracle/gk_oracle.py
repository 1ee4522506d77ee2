"""CPU restatement of the reference GKArray algorithm -- TEST INFRASTRUCTURE ONLY.

This module is the parity *checker* for the MI355X engine.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may import
it.  The product path (``sketches-py_amd/gkarray_amd``) never imports, links or
executes anything under ``oracle/``.

It restates ``/root/reference/gkarray/gkarray.py`` (``gk:N`` = line N of that file)
with the semantics the reference evidently intends: every raw value added is the
record ``(val, g=1, delta=0)`` (the reference as written
crashes on plain floats at its first flush).  The state is kept structure-of-
arrays (three parallel lists) instead of ``Entry`` objects, and the four-rule
merge/compress walk of gk:76-106 is restated over those lists.

Pinning: the restatement is checked against golden vectors produced by the
unmodified reference (driven through the harness shim) in
``tests/golden/make_golden.py``; see ``tests/test_oracle_golden.py``.

The small-n branch (gk:169-171, gk:200-202) calls ``numpy.percentile`` with the
default linear method.  That is third-party arithmetic; it is restated here from
numpy 2.2.6 ``numpy/lib/_function_base_impl.py`` (q/100 at l.4257, virtual index
``(n-1)*q`` at l.107, index bounds l.4748-4750, gamma l.4632, ``_lerp``
l.4653-4657) so that the oracle does not depend on numpy at all.
"""
import math

__all__ = ["OracleGK", "OracleEpsMismatch", "percentile_linear", "flush_period",
           "removal_threshold"]


class OracleEpsMismatch(Exception):
    """Mirrors ``UnequalEpsilonException`` (gk:4-5)."""


def flush_period(eps):
    """Adds between automatic flushes: ``int(1.0/eps) + 1`` (gk:60)."""
    return int(1.0 / eps) + 1


def removal_threshold(eps, n):
    """``np.floor(2.0*eps*(n - 1))`` (gk:70), as an exact integer.

    Python evaluates ``2.0*eps`` first, then multiplies by the float of ``n-1``.
    """
    return math.floor((2.0 * eps) * float(n - 1))


def percentile_linear(sorted_vals, q):
    """``np.percentile(sorted_vals, q*100)`` (linear method) restated.

    numpy 2.2.6: qq = (q*100)/100; vi = (n-1)*qq; indexes at/above n-1 take the
    last element with previous index -1 (so gamma = vi + 1); otherwise
    previous = floor(vi), next = previous + 1; gamma = vi - previous;
    r = a + (b-a)*gamma, replaced by b - (b-a)*(1-gamma) when gamma >= 0.5.
    """
    n = len(sorted_vals)
    qq = (q * 100) / 100.0
    if qq != qq or qq < 0.0 or qq > 1.0:
        raise ValueError("Percentiles must be in the range [0, 100]")
    vi = float(n - 1) * qq
    if vi >= n - 1:
        prev_f = -1.0
        a = b = sorted_vals[-1]
    elif vi < 0:
        prev_f = 0.0
        a = b = sorted_vals[0]
    else:
        prev_f = math.floor(vi)
        a = sorted_vals[int(prev_f)]
        b = sorted_vals[int(prev_f) + 1]
    gamma = vi - prev_f
    diff = b - a
    if gamma >= 0.5:
        return b - diff * (1 - gamma)
    return a + diff * gamma


class OracleGK:
    """One GKArray stream (gk:19-232) as parallel lists ``v``, ``g``, ``d``."""

    def __init__(self, eps):
        # gk:21-29
        self.eps = eps
        self.v, self.g, self.d = [], [], []
        self.pending = []                 # raw values (g=1, delta=0), insertion order
        self.min = float("inf")
        self.max = float("-inf")
        self.n = 0
        self.sum = 0.0
        self.avg = 0.0

    # ------------------------------------------------------------------ state
    def table(self):
        return list(zip(self.v, self.g, self.d))

    def size(self):
        # gk:44-47 -- flushes pending values (state mutation)
        if self.pending:
            self.flush()
        return len(self.v)

    # ------------------------------------------------------------------ ingest
    def add(self, x):
        # gk:49-61
        x = float(x)
        self.n += 1
        self.sum += x
        self.avg += (x - self.avg) * (1.0 / self.n)
        self.pending.append(x)
        if x < self.min:
            self.min = x
        if x > self.max:
            self.max = x
        if self.n % flush_period(self.eps) == 0:
            self.flush()

    def add_many(self, xs):
        for x in xs:
            self.add(x)

    def flush(self, extra=()):
        """``merge_compress(entries)`` (gk:63-109).

        ``extra`` is a sequence of (val, g, delta) records that join the raw
        pending values (gk:71).  Both are stably sorted by value (gk:72), the
        raw values first on ties because they precede ``extra`` in the list.
        """
        T = removal_threshold(self.eps, self.n)
        inc = [[x, 1, 0] for x in self.pending] + [[a, b, c] for (a, b, c) in extra]
        inc.sort(key=lambda r: r[0])      # list.sort is stable, like sorted()
        ev, eg, ed = self.v, list(self.g), self.d
        out_v, out_g, out_d = [], [], []
        i = j = 0
        ni, ne = len(inc), len(ev)
        while i < ni or j < ne:
            if i < ni and (j == ne or inc[i][0] < ev[j]):
                rec = inc[i]
                if j == ne:
                    # gk:85-92: only incoming records are left
                    if i + 1 < ni and rec[1] + inc[i + 1][1] + inc[i + 1][2] <= T:
                        inc[i + 1][1] += rec[1]
                    else:
                        out_v.append(rec[0]); out_g.append(rec[1]); out_d.append(rec[2])
                else:
                    # gk:93-99: incoming record in front of entry j
                    if rec[1] + eg[j] + ed[j] <= T:
                        eg[j] += rec[1]
                    else:
                        out_v.append(rec[0]); out_g.append(rec[1])
                        out_d.append(eg[j] + ed[j] - rec[1])
                i += 1
            else:
                # gk:77-84 and gk:100-106: entry j (incoming exhausted, or
                # entry value <= incoming value)
                if j + 1 < ne and eg[j] + eg[j + 1] + ed[j + 1] <= T:
                    eg[j + 1] += eg[j]
                else:
                    out_v.append(ev[j]); out_g.append(eg[j]); out_d.append(ed[j])
                j += 1
        self.v, self.g, self.d = out_v, out_g, out_d
        self.pending = []

    # ------------------------------------------------------------------ merge
    def merge(self, other):
        """gk:111-154.  Mutates ``other`` (flushes it), like the reference."""
        if self.eps != other.eps:
            raise OracleEpsMismatch("Cannot merge two GKArrays with different epsilon values")
        if other.n == 0:
            self.flush()
            return
        if self.n == 0:
            other.flush()
            self.v, self.g, self.d = list(other.v), list(other.g), list(other.d)
            self.min, self.max = other.min, other.max
            self.n, self.sum, self.avg = other.n, other.sum, other.avg
            return
        spread = int(other.eps * (other.n - 1))     # before other's flush (gk:136)
        other.flush()
        L = len(other.v)
        conv = []
        first = other.g[0] + other.d[0] - spread - 1
        if first > 0:
            conv.append((other.min, first, 0))
        for k in range(L - 1):
            w = other.g[k + 1] + other.d[k + 1] - other.d[k]
            if w > 0:
                conv.append((other.v[k], w, 0))
        last = spread + 1 - other.d[L - 1]
        if last > 0:
            conv.append((other.v[L - 1], last, 0))
        self.n += other.n
        self.eps = max(self.eps, other.eps)
        # min()/max() return their first argument unless the second is strictly
        # smaller/larger (gk:151-152)
        if other.min < self.min:
            self.min = other.min
        if other.max > self.max:
            self.max = other.max
        self.flush(conv)

    # ------------------------------------------------------------------ query
    def _small(self):
        return self.n < 1.0 / self.eps

    def _walk(self, q, leftover_is_max):
        rank = int(q * (self.n - 1) + 1)
        spread = int(self.eps * (self.n - 1))
        acc = 0
        for i in range(len(self.v)):
            acc += self.g[i]
            if acc + self.d[i] - 1 > rank + spread:
                return self.min if i == 0 else self.v[i - 1]
        if leftover_is_max:
            return self.max
        return self.v[-1]

    def quantile(self, q):
        # gk:156-185
        if q < 0 or q > 1 or self.n == 0:
            return float("nan")
        if self.pending:
            self.flush()
        if self._small():
            return percentile_linear(self.v, q)
        if q != q:
            raise ValueError("cannot convert float NaN to integer")
        return self._walk(q, leftover_is_max=False)

    def quantiles(self, qs):
        # gk:187-232
        qs = list(qs)
        if self.n == 0:
            return [float("nan")] * len(qs)
        if self.pending:
            self.flush()
        if self._small():
            return [percentile_linear(self.v, q) if (q >= 0 and q <= 1) else float("nan")
                    for q in qs]
        if qs != sorted(qs):
            return [self.quantile(q) for q in qs]
        out = []
        for q in qs:
            if q < 0 or q > 1:
                out.append(float("nan"))
            else:
                if q != q:
                    raise ValueError("cannot convert float NaN to integer")
                out.append(self._walk(q, leftover_is_max=True))
        return out
