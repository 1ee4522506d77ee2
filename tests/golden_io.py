"""Loader for the committed golden vectors (tests/golden/*, made by make_golden.py)."""
import functools
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN_DIR = os.path.join(HERE, "golden")


@functools.lru_cache(maxsize=1)
def index():
    with open(os.path.join(GOLDEN_DIR, "golden_index.json")) as f:
        return json.load(f)


@functools.lru_cache(maxsize=1)
def arrays():
    with np.load(os.path.join(GOLDEN_DIR, "golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def get(cid, name):
    return arrays()["case%d/%s" % (cid, name)]


def has(cid, name):
    return ("case%d/%s" % (cid, name)) in arrays()


def tables(cid, prefix):
    """List of tables; each table is a list of (v, g, d) tuples."""
    a = arrays()
    sizes = a["case%d/%s/sizes" % (cid, prefix)]
    v = a["case%d/%s/v" % (cid, prefix)]
    g = a["case%d/%s/g" % (cid, prefix)]
    d = a["case%d/%s/d" % (cid, prefix)]
    out, o = [], 0
    for s in sizes:
        s = int(s)
        out.append([(float(v[o + k]), int(g[o + k]), int(d[o + k])) for k in range(s)])
        o += s
    return out


def cases(kind=None):
    return [c for c in index()["cases"] if kind is None or c["kind"] == kind]


def shards(cid):
    x = get(cid, "x")
    sizes = get(cid, "shard_sizes")
    out, o = [], 0
    for s in sizes:
        out.append(x[o:o + int(s)])
        o += int(s)
    return out


def same_float(a, b):
    """Bitwise equality that treats NaN == NaN and distinguishes -0.0 / +0.0."""
    a = np.float64(a)
    b = np.float64(b)
    if np.isnan(a) and np.isnan(b):
        return True
    return a.tobytes() == b.tobytes()


def zero_sign_unpinned(vals, n, eps, q):
    """True iff the reference's answer to q is a zero whose SIGN is not a
    function of the input: the small-n branch (n < 1/eps, gk:169-171 /
    gk:200-202) calls numpy.percentile on the table values, and numpy's
    partition (introselect, or x86-simd-sort's AVX-512 / AVX2 network on
    machines that have them -- CPU-dependent) may place -0.0 or +0.0 at the
    two interpolation positions.  numpy 2.2.6's _lerp returns -0.0 only in its
    gamma >= 0.5 branch with BOTH positions -0.0 (b - (b-a)(1-g) = -0 - +0);
    so the sign is open exactly when: gamma >= 0.5, prev < E-1, the stable-
    ordered values at prev and prev+1 are both zeros, and the table holds
    both +0.0 and -0.0.  Everywhere else the answer is pinned bit for bit
    (tests/test_oracle_golden.py::test_zero_sign_class_is_exact fuzzes the
    claim against numpy itself).  `vals`: the table values in table order."""
    if not (float(n) < 1.0 / eps) or not (0.0 <= q <= 1.0):
        return False
    E = len(vals)
    if E < 2:
        return False
    vi = float(E - 1) * ((q * 100) / 100.0)
    if vi >= E - 1 or vi < 0:
        return False
    prev = int(np.floor(vi))
    if vi - prev < 0.5 or vals[prev] != 0 or vals[prev + 1] != 0:
        return False
    zs = [bool(np.signbit(v)) for v in vals if v == 0]
    return any(zs) and not all(zs)


def unpinned_mask(table, n, eps, qs):
    """zero_sign_unpinned for each q of qs; `table`: list of (v, g, d)."""
    vals = [float(t[0]) for t in table]
    return [zero_sign_unpinned(vals, n, eps, float(q)) for q in qs]


def same_table(t1, t2):
    if len(t1) != len(t2):
        return False
    for (a, b, c), (x, y, z) in zip(t1, t2):
        if not same_float(a, x) or int(b) != int(y) or int(c) != int(z):
            return False
    return True
