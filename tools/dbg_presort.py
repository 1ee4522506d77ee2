"""Debug driver (round 3): the host-chain test's two calls, one phase at a
time with explicit device syncs and progress lines, under an env config
given on the command line (KEY=VAL ...).  Not part of the test suite."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sketches-py_amd"))
for kv in sys.argv[1:]:
    k, v = kv.split("=", 1)
    os.environ[k] = v
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gkarray_amd import StreamSet  # noqa: E402


def batch(seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 3000, 300)
    lens[:24] = rng.integers(20_000, 150_000, 24)
    lens[5] = 0
    seqs = [rng.lognormal(0.0, 2.0, int(L)) for L in lens]
    seqs[4][[0, 12345]] = [np.nan, -1e300]
    return seqs


t0 = time.time()
dev = torch.device("cuda:0")
ss = StreamSet(300, 0.001, device=dev)
for seed in (1, 2, 3):
    seqs = batch(seed)
    offs = np.zeros(len(seqs) + 1, np.int64)
    offs[1:] = np.cumsum([len(x) for x in seqs])
    x = torch.from_numpy(np.concatenate(seqs)).to(dev)
    print("%.1fs call %d: enqueue" % (time.time() - t0, seed), flush=True)
    q = ss.ingest(x, torch.from_numpy(offs).to(dev), quantiles=[0.5], sync=False)
    print("%.1fs call %d: enqueued" % (time.time() - t0, seed), flush=True)
    torch.cuda.synchronize()
    print("%.1fs call %d: device synced" % (time.time() - t0, seed), flush=True)
    ss.sync()
    print("%.1fs call %d: set synced" % (time.time() - t0, seed), flush=True)
print("DONE")
