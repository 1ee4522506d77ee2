"""Host-side cost of enqueueing one bench step (reset + fused ingest +
quantiles, sync=False) against the GPU time of the step: if the host needs as
long to enqueue a step as the GPU to run it, the GPU idles between steps.
Usage: host_enqueue.py [S ...]   (cfg3 batches of S streams x 1000 values)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sketches-py_amd"))
from gkarray_amd import StreamSet  # noqa: E402

dev = torch.device("cuda", 0)
qs = [0.5, 0.9, 0.99]
for S in [int(a) for a in sys.argv[1:]] or [125_000, 1_000_000]:
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.rand(S * 1000, device=dev, dtype=torch.float64, generator=g).pow(-1.0 / 1.5)  # Pareto(1.5) + ...
    offs = torch.arange(S + 1, device=dev, dtype=torch.int64) * 1000
    ss = StreamSet(S, 0.01, device=dev)

    def step():
        ss.reset()
        return ss.ingest(x, offs, quantiles=qs, sync=False)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    K = 30
    host = []
    t0 = time.perf_counter()
    for _ in range(K):
        a = time.perf_counter()
        step()
        host.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host.sort()
    print("S=%d: wall %.1f us/step (enqueue loop %.1f us/step, drain %.1f us); host per step: median %.1f us, "
          "min %.1f, max %.1f" % (S, (t2 - t0) / K * 1e6, (t1 - t0) / K * 1e6, (t2 - t1) * 1e6,
                                  host[K // 2] * 1e6, host[0] * 1e6, host[-1] * 1e6))
