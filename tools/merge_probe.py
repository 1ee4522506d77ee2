"""Probe: GKArray.merge at scale -- K shard StreamSets of S streams (each
stream ingested with L values, eps=0.01), then set0.merge_from(set1..setK-1)
(the reference's left fold, gk:111-154), timed with HIP events on the caller's
stream.  Prints ms for the fold and the per-merge rate."""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sketches-py_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
from bench import make_input
from gkarray_amd import StreamSet

dev = torch.device("cuda", 0)
for S, L, K in [(100_000, 1000, 8), (1_000_000, 1000, 8), (10_000, 125_000, 8)]:
    sets = []
    inputs = [make_input(S, L, 11 + k, dev, "lognormal") for k in range(K)]
    for k in range(K):
        sets.append(StreamSet(S, 0.01, device=dev))
    for it in range(2):
        for (x, o), sk in zip(inputs, sets):
            sk.reset()
            sk.ingest(x, o)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sets[0].merge_from(sets[1:])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
    ms = (t1 - t0) * 1e3
    print("S=%d L=%d K=%d: fold %.2f ms, %.1f M stream-merges/s" % (S, L, K, ms, S * (K - 1) / (t1 - t0) / 1e6),
          flush=True)
    for sk in sets:
        sk.close()
    del inputs
    torch.cuda.empty_cache()
