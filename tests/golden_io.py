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


def same_table(t1, t2):
    if len(t1) != len(t2):
        return False
    for (a, b, c), (x, y, z) in zip(t1, t2):
        if not same_float(a, x) or int(b) != int(y) or int(c) != int(z):
            return False
    return True
