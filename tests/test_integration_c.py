"""INTEGRATION.md section 4 as a C program (tests/integration_fold.c): the
row-shard fold sequence -- gk_pack_bytes, a max all-reduce of the sizes,
gk_pack, an all-gather of the packed bytes, gk_fold_packed -- compiled with
gcc against the host engine (libgkarray_cpu.so, the same include/gk_capi.h),
the two collectives replaced by in-process stand-ins (a max over the ranks,
memcpy into one buffer).  Every rank's fold must be byte-identical (checked
inside the program) and rank 0's must equal the oracle's rank-ordered left fold
sk_0.merge(sk_1)...merge(sk_{N-1}) (gk:111-154): tables, pending values and
header, bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from gk_oracle_c import OracleSet

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "sketches-py_amd", "gkarray_amd")


@pytest.fixture(scope="module")
def prog(tmp_path_factory):
    if not os.path.exists(os.path.join(LIBDIR, "libgkarray_cpu.so")):
        pytest.skip("host engine not built")
    exe = str(tmp_path_factory.mktemp("cfold") / "integration_fold")
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "integration_fold.c"), "-L" + LIBDIR, "-lgkarray_cpu",
                    "-Wl,-rpath," + LIBDIR, "-o", exe], check=True)
    return exe


def shards(S, nranks, seed):
    rng = np.random.default_rng(seed)
    out = []
    for r in range(nranks):
        lens = rng.integers(0, 2500, S)
        offs = np.zeros(S + 1, np.int64)
        offs[1:] = np.cumsum(lens)
        v = rng.lognormal(0.0, 1.5, int(offs[-1]))
        if v.size > 10:
            v[rng.integers(0, v.size, 5)] = 0.0
            v[rng.integers(0, v.size, 5)] = -0.0
        out.append((offs, v))
    return out


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.int64)


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
def test_c_row_shard_fold_matches_oracle(prog, tmp_path, nranks):
    S, eps = 150, 0.01
    sh = shards(S, nranks, 11 + nranks)
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(inp, "wb") as f:
        f.write(np.int64(S).tobytes() + np.float64(eps).tobytes() + np.int32(nranks).tobytes())
        for offs, v in sh:
            f.write(offs.tobytes() + v.tobytes())
    r = subprocess.run([prog, str(inp), str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr

    acc = OracleSet(S, eps)
    acc.ingest(sh[0][1], sh[0][0])
    for offs, v in sh[1:]:
        o = OracleSet(S, eps)
        o.ingest(v, offs)
        acc.merge(o)  # gk:111-154, the rank-ordered left fold
    st = acc.stats()
    toffs, tv, tg, td = acc.tables()
    poffs, pv = acc.pending()

    b = open(out, "rb").read()
    pos = 0

    def take(dt, n):
        nonlocal pos
        a = np.frombuffer(b, dt, n, pos)
        pos += a.nbytes
        return a

    sizes, pend, n = take(np.int32, S), take(np.int32, S), take(np.int64, S)
    hdr = {k: take(np.float64, S) for k in ("min", "max", "sum", "avg")}
    E, Pn = int(sizes.sum()), int(pend.sum())
    v, g, d, p = take(np.float64, E), take(np.int32, E), take(np.int32, E), take(np.float64, Pn)
    assert pos == len(b)
    assert np.array_equal(sizes, st["size"]) and np.array_equal(pend, st["pending"])
    assert np.array_equal(n, st["n"])
    for k in hdr:
        assert np.array_equal(bits(hdr[k]), bits(st[k])), k
    assert np.array_equal(bits(v), bits(tv))
    assert np.array_equal(g.astype(np.int64), tg) and np.array_equal(d.astype(np.int64), td)
    assert np.array_equal(bits(p), bits(pv))
