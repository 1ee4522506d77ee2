"""k_ingest_wg's time per flush with S long streams and nothing else in the
batch: S streams of L lognormal values at eps = 0.001 (every one a workgroup
stream), one reset + ingest per step.  Run under rocprofv3 --kernel-trace to
read the k_ingest_wg duration; prints the wall time per step and per flush.
Usage: wg_alone.py S [L] [steps]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sketches-py_amd"))
from gkarray_amd import StreamSet  # noqa: E402

S = int(sys.argv[1])
L = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(5)
x = torch.exp(torch.randn(S * L, device=dev, dtype=torch.float64, generator=g))
offs = torch.arange(S + 1, device=dev, dtype=torch.int64) * L
ss = StreamSet(S, 0.001, device=dev)
ss.ingest(x, offs)
torch.cuda.synchronize()
ts = []
for _ in range(steps):
    ss.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ss.ingest(x, offs)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
flushes = L // 1001
best = min(ts)
print("S=%d L=%d: step %.2f ms (best of %d), %.3f us per flush of the chain" % (S, L, best * 1e3, steps, best * 1e6 / flushes))
