"""One very long stream at eps = 0.01 (the 128-entry small class: no workgroup
path) beside short streams: its time per flush on the one-wave path.
Usage: long_small_eps.py [L] [S_short]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sketches-py_amd"))
from gkarray_amd import StreamSet  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
S_short = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(5)
lens = torch.full((S_short + 1,), 1000, dtype=torch.int64)
lens[0] = L
offs = torch.zeros(S_short + 2, dtype=torch.int64)
offs[1:] = torch.cumsum(lens, 0)
x = torch.exp(torch.randn(int(offs[-1]), device=dev, dtype=torch.float64, generator=g))
offs = offs.to(dev)
for eps in (0.01, 0.001):
    ss = StreamSet(S_short + 1, eps, device=dev)
    ss.ingest(x, offs)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        ss.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ss.ingest(x, offs, quantiles=[0.5, 0.9, 0.99])
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    P = int(1 / eps) + 1
    print("eps=%g: one stream of %d values + %d streams of 1000: %.1f ms per call, %.2f us per flush of the long stream"
          % (eps, L, S_short, best * 1e3, best * 1e6 / (L // P)))
