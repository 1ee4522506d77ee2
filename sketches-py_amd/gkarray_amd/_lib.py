"""ctypes binding of the C ABI declared in ``include/gk_capi.h``.

The shared library ``libgkarray_hip.so`` (built in-tree by ``make -C
sketches-py_amd/csrc`` / ``__graft_entry__.build()``) holds every HIP kernel.
There is no CPU fallback: if the library or a GPU is missing, the product path
raises ``GKBackendError``.
"""
import ctypes
import os
import sys

__all__ = ["lib", "load", "load_cpu", "GKBackendError", "check", "LIB_PATH", "CPU_LIB_PATH", "SYMBOLS",
           "CPU_SYMBOLS",
           "GK_OK", "GK_E_ARG", "GK_E_EPS_MISMATCH", "GK_E_OVERFLOW", "GK_E_HIP",
           "GK_E_NOMEM", "GK_E_UNSUPPORTED", "GK_E_IO", "GK_E_FORMAT", "GK_Q_LIST", "GK_Q_SINGLE"]

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgkarray_hip.so")
# host engine (include/gk_cpu.h): same C ABI on host memory, selected explicitly
CPU_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgkarray_cpu.so")

GK_OK = 0
GK_E_ARG = -1
GK_E_EPS_MISMATCH = -2
GK_E_OVERFLOW = -3
GK_E_HIP = -4
GK_E_NOMEM = -5
GK_E_UNSUPPORTED = -6
GK_E_IO = -7
GK_E_FORMAT = -8
GK_Q_LIST = 0
GK_Q_SINGLE = 1


class GKBackendError(RuntimeError):
    """The HIP backend is missing or failed (no silent CPU fallback)."""

    def __init__(self, code, msg):
        super().__init__("gkarray_amd: %s (code %d)" % (msg, code))
        self.code = code


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_D = ctypes.c_double
_INT = ctypes.c_int

# name -> (restype, argtypes); must match include/gk_capi.h exactly
SYMBOLS = {
    "gk_version": (_INT, []),
    "gk_last_error": (ctypes.c_char_p, []),
    "gk_create": (_INT, [_I64, _D, _I64, _INT, ctypes.POINTER(_P)]),
    "gk_destroy": (_INT, [_P]),
    "gk_reset": (_INT, [_P, _P]),
    "gk_ingest": (_INT, [_P, _P, _P, _P]),
    "gk_flush": (_INT, [_P, _P]),
    "gk_sync": (_INT, [_P, _P]),
    "gk_quantiles": (_INT, [_P, ctypes.POINTER(_D), _INT, _P, _INT, _P]),
    "gk_ingest_quantiles": (_INT, [_P, _P, _P, ctypes.POINTER(_D), _INT, _P, _INT, _P]),
    "gk_stats": (_INT, [_P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "gk_merge": (_INT, [_P, ctypes.POINTER(_P), _INT, _P]),
    "gk_merge_compress": (_INT, [_P, _P, _P, _P, _P, _P]),
    "gk_export_sizes": (_INT, [_P, _P, _P]),
    "gk_export": (_INT, [_P, _P, _P, _P, _P, _P]),
    "gk_export_pending_sizes": (_INT, [_P, _P, _P]),
    "gk_export_pending": (_INT, [_P, _P, _P, _P]),
    "gk_import": (_INT, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "gk_save": (_INT, [_P, ctypes.c_char_p, _P]),
    "gk_pack_bytes": (_INT, [_P, ctypes.POINTER(_I64), _P]),
    "gk_pack": (_INT, [_P, _P, _I64, _P]),
    "gk_fold_packed": (_INT, [_P, ctypes.POINTER(_P), _INT, _P]),
    "gk_peek": (_INT, [ctypes.c_char_p, ctypes.POINTER(_D), ctypes.POINTER(_I64)]),
    "gk_load": (_INT, [_P, ctypes.c_char_p, _P]),
    "gk_num_streams": (_I64, [_P]),
    "gk_eps": (_D, [_P]),
    "gk_flush_period": (_INT, [_P]),
    "gk_capacity": (_INT, [_P, _INT]),
    "gk_num_promoted": (_I64, [_P]),
    "gk_host_chains_taken": (_I64, [_P]),
    "gk_timing_enable": (_INT, [_P, _INT]),
    "gk_timing_read": (_INT, [_P, ctypes.POINTER(_D), ctypes.POINTER(_D), ctypes.POINTER(_I64)]),
}

# the host engine exports every SYMBOLS entry plus these (include/gk_cpu.h)
CPU_SYMBOLS = dict(SYMBOLS)
CPU_SYMBOLS.update({
    "gk_cpu_set_threads": (_INT, [_P, _INT]),
    "gk_cpu_threads": (_INT, [_P]),
})

_lib = None
_cpu_lib = None


def load_cpu(path=None):
    """Load the host engine libgkarray_cpu.so (cached).  Only used when a
    caller asks for device="cpu"; never a fallback for the HIP library."""
    global _cpu_lib
    if _cpu_lib is not None and path is None:
        return _cpu_lib
    p = path or CPU_LIB_PATH
    if not os.path.exists(p):
        raise GKBackendError(GK_E_ARG, "CPU engine not built: %s (run __graft_entry__.build())" % p)
    handle = ctypes.CDLL(p)
    for name, (res, args) in CPU_SYMBOLS.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _cpu_lib = handle
    return handle


def load(path=None):
    """Load the HIP library (cached).  Raises GKBackendError if it is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # GK_LIB_PATH selects an alternative build (A/B experiments; reported by
    # library_identity() and announced on stderr); default in-tree
    p = path or os.environ.get("GK_LIB_PATH") or LIB_PATH
    if path is None and os.environ.get("GK_LIB_PATH"):
        sys.stderr.write("gkarray_amd: GK_LIB_PATH override: loading %s\n" % p)
    if not os.path.exists(p):
        raise GKBackendError(GK_E_HIP, "HIP library not built: %s (run __graft_entry__.build())" % p)
    try:
        handle = ctypes.CDLL(p)
    except OSError as e:  # pragma: no cover - depends on the ROCm install
        raise GKBackendError(GK_E_HIP, "cannot load %s: %s" % (p, e))
    override = path is None and bool(os.environ.get("GK_LIB_PATH"))
    for name, (res, args) in SYMBOLS.items():
        try:
            fn = getattr(handle, name)
        except AttributeError:
            if not override:
                raise
            # an older build under A/B (GK_LIB_PATH): entry points it predates stay unbound
            sys.stderr.write("gkarray_amd: %s lacks %s\n" % (p, name))
            continue
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = handle
    return handle


def lib():
    return load()


def library_identity():
    """The HIP library the process uses: path, sha256, and whether GK_LIB_PATH
    overrides the in-tree build."""
    import hashlib
    p = os.environ.get("GK_LIB_PATH") or LIB_PATH
    with open(p, "rb") as f:
        h = hashlib.sha256(f.read()).hexdigest()
    return {"path": os.path.relpath(p, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))),
            "sha256": h, "override": bool(os.environ.get("GK_LIB_PATH"))}


def last_error(handle=None):
    return (handle or load()).gk_last_error().decode("utf-8", "replace")


def check(rc, handle=None):
    if rc != GK_OK:
        raise GKBackendError(rc, last_error(handle))
    return rc
