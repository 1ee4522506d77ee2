"""gkarray_amd -- MI355X-native batched GKArray (githomin/sketches-py) engine.

Public API
  GKArray, Entry, UnequalEpsilonException   drop-in for gkarray/gkarray.py
  StreamSet                                 S independent streams, batched
  dist                                      multi-GPU helpers (torch.distributed)
The kernels live in libgkarray_hip.so (C ABI: include/gk_capi.h).
"""
from ._lib import GKBackendError, LIB_PATH  # noqa: F401
from .gkarray import Entry, GKArray, UnequalEpsilonException  # noqa: F401
from .streamset import StreamSet  # noqa: F401

__version__ = "0.1.0"
