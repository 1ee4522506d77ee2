"""Probe: per-flush latency of the ingest path and per-value latency of the
_sum/_avg chain for one long stream (eps=0.001), and the same with k copies
of it side by side.  Prints one line per case: kernel ms from the engine's own
HIP-event timing."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sketches-py_amd"))
import torch
from gkarray_amd import StreamSet

dev = torch.device("cuda", 0)
eps = float(os.environ.get("EPS", "0.001"))
for S, L in [(1, 1_000_000), (1, 4_000_000), (64, 1_000_000), (256, 1_000_000)]:
    g = torch.Generator(device=dev); g.manual_seed(1)
    x = torch.randn(S * L, dtype=torch.float64, device=dev, generator=g).exp_()
    offs = torch.arange(0, S * L + 1, L, dtype=torch.int64, device=dev)
    ss = StreamSet(S, eps, device=dev)
    ss.timing(True)
    for it in range(2):
        ss.reset()
        torch.cuda.synchronize(); t0 = time.perf_counter()
        ss.ingest(x, offs, quantiles=[0.5, 0.9, 0.99])
        torch.cuda.synchronize(); t1 = time.perf_counter()
    tm = ss.read_timing()
    P = int(1 / eps) + 1
    print("S=%d L=%d wall %.2f ms  timing %s  per-flush us %.2f" % (S, L, (t1 - t0) * 1e3, tm, (t1 - t0) * 1e6 / (L // P)), flush=True)
    ss.close()
