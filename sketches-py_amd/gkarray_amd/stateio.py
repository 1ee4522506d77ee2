"""GKSTATE files in pure numpy: the versioned state format of csrc/gk_format.h.

``read_state(path)`` / ``write_state(path, state)`` use the same dict as
``StreamSet.export_state()`` (numpy arrays instead of device tensors):
``eps, offs, v, g, d, poffs, pv, n, min, max, sum, avg``.  They let host code
inspect, build or convert state files without the HIP library (for example a
state produced by another GKArray implementation, loaded into a StreamSet with
``StreamSet.load``).  The C ABI (gk_save / gk_load) reads and writes the same
bytes.
"""
import numpy as np

__all__ = ["MAGIC", "VERSION", "HEADER_BYTES", "read_state", "write_state", "StateFormatError"]

MAGIC = b"GKSTATE\0"
VERSION = 1
HEADER_BYTES = 80
_HDR = np.dtype([("magic", "S8"), ("version", "<u4"), ("header_bytes", "<u4"), ("eps", "<f8"),
                 ("S", "<i8"), ("E_total", "<i8"), ("P_total", "<i8"), ("sum_a", "<u8"),
                 ("sum_b", "<u8"), ("flags", "<u4"), ("reserved0", "<u4"), ("reserved1", "<u8")])
assert _HDR.itemsize == HEADER_BYTES


class StateFormatError(ValueError):
    pass


def _words(buf):
    b = np.frombuffer(buf, dtype=np.uint8)
    pad = (-b.size) % 8
    if pad:
        b = np.concatenate([b, np.zeros(pad, np.uint8)])
    return b.view("<u8")


def _checksum(payload):
    w = _words(payload)
    with np.errstate(over="ignore"):
        a = np.sum(w, dtype=np.uint64)
        b = np.sum(w * np.arange(1, w.size + 1, dtype=np.uint64), dtype=np.uint64)
    return int(a), int(b)


def _pad8(b):
    return b + b"\0" * ((-len(b)) % 8)


def write_state(path, state):
    """Write a state dict (export_state() layout, numpy or CPU arrays)."""
    offs = np.asarray(state["offs"], np.int64)
    poffs = np.asarray(state["poffs"], np.int64)
    S = offs.size - 1
    sizes = np.diff(offs).astype("<i4")
    psizes = np.diff(poffs).astype("<i4")
    parts = [np.concatenate([sizes, psizes]).tobytes()]
    parts.append(np.asarray(state["n"], "<i8").tobytes())
    for k in ("min", "max", "sum", "avg"):
        parts.append(np.asarray(state[k], "<f8").tobytes())
    parts.append(np.asarray(state["v"], "<f8").tobytes())
    parts.append(np.concatenate([np.asarray(state["g"], "<i4"), np.asarray(state["d"], "<i4")]).tobytes())
    parts.append(np.asarray(state["pv"], "<f8").tobytes())
    payload = b"".join(_pad8(p) for p in parts)
    a, b = _checksum(payload)
    hdr = np.zeros((), _HDR)
    hdr["magic"] = MAGIC
    hdr["version"] = VERSION
    hdr["header_bytes"] = HEADER_BYTES
    hdr["eps"] = float(state["eps"])
    hdr["S"] = S
    hdr["E_total"] = int(offs[-1] - offs[0]) if S >= 0 else 0
    hdr["P_total"] = int(poffs[-1] - poffs[0])
    hdr["sum_a"] = a
    hdr["sum_b"] = b
    with open(path, "wb") as f:
        f.write(hdr.tobytes())
        f.write(payload)


def read_state(path):
    """Read a GKSTATE file into a state dict of numpy arrays."""
    with open(path, "rb") as f:
        raw = f.read()
    if len(raw) < HEADER_BYTES:
        raise StateFormatError("%s: truncated header" % path)
    hdr = np.frombuffer(raw[:HEADER_BYTES], _HDR)[0]
    if bytes(hdr["magic"]).ljust(8, b"\0") != MAGIC:
        raise StateFormatError("%s: not a GKSTATE file" % path)
    if int(hdr["version"]) != VERSION:
        raise StateFormatError("%s: unsupported version %d" % (path, int(hdr["version"])))
    S, E, P = int(hdr["S"]), int(hdr["E_total"]), int(hdr["P_total"])
    payload = raw[HEADER_BYTES:]
    need = 8 * S + 8 * S * 5 + 8 * E + 8 * E + 8 * P
    if len(payload) != need:
        raise StateFormatError("%s: payload of %d bytes, expected %d" % (path, len(payload), need))
    if _checksum(payload) != (int(hdr["sum_a"]), int(hdr["sum_b"])):
        raise StateFormatError("%s: checksum mismatch" % path)
    o = 0

    def take(dt, count):
        nonlocal o
        a = np.frombuffer(payload, dt, count, o).copy()
        o += (a.nbytes + 7) // 8 * 8
        return a

    sp = take("<i4", 2 * S)
    sizes, psizes = sp[:S], sp[S:]
    st = {"eps": float(hdr["eps"])}
    st["n"] = take("<i8", S)
    for k in ("min", "max", "sum", "avg"):
        st[k] = take("<f8", S)
    st["v"] = take("<f8", E)
    gd = take("<i4", 2 * E)
    st["g"], st["d"] = gd[:E], gd[E:]
    st["pv"] = take("<f8", P)
    st["offs"] = np.concatenate([[0], np.cumsum(sizes, dtype=np.int64)])
    st["poffs"] = np.concatenate([[0], np.cumsum(psizes, dtype=np.int64)])
    if int(st["offs"][-1]) != E or int(st["poffs"][-1]) != P or (sizes < 0).any() or (psizes < 0).any():
        raise StateFormatError("%s: size arrays do not match the record totals" % path)
    return st
