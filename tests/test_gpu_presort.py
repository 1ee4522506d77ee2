"""Presorted flush batches of long streams (P > 128; DESIGN.md section 5, long
streams): k_long_prep plans the batches of the streams within a quarter of
the longest one's flush count, k_presort sorts them (value, then insertion
index: gk:71-72's stable sorted()) ahead of the ingest launch, and the flush
of a presorted batch places each value at its rank directly; the other long
streams flush unsorted.  Results never depend on which streams were planned.

The workspace is sized from the previous call's need, so call 0 flushes
unsorted and the later calls presort; pending values carried between calls
make every call's batch 0 start with them; every third stream holds rounded
values (ties: the stable order decides).  Every call's whole state (tables,
pending values, n/min/max/sum/avg) and the fused quantiles are compared bit
for bit with the oracle.
"""
import numpy as np
import pytest
import torch

from gk_oracle_c import OracleSet
from parity_util import _ss, assert_same_quantiles, assert_same_state, csr, small_of

pytestmark = pytest.mark.gpu

QS = [0.01, 0.5, 0.9, 0.99]


@pytest.mark.parametrize("seed", [0, 1])
def test_presorted_batches_across_calls(gpu_device, seed):
    S, eps = 48, 0.001  # P = 1001: class 0 is the 2048-entry LDS class
    rng = np.random.default_rng(1000 + seed)
    ss = _ss(S, eps, gpu_device)
    o = OracleSet(S, eps)
    for call in range(4):
        lens = rng.integers(0, 45_000, S)
        lens[0] = 180_000 + rng.integers(0, 2_000)  # the longest: presorted
        lens[1:4] = 60_000 + rng.integers(0, 5_000, 3)  # within a quarter of it: presorted
        lens[4] = 0  # an empty row
        seqs = []
        for s in range(S):
            v = rng.lognormal(0.0, 1.0, int(lens[s]))
            if s % 3 == 1:
                v = np.round(v, 1)  # ties: the stable order decides (insertion index)
            seqs.append(v)
        flat, offs = csr(seqs)
        if call == 3:
            q = ss.ingest(torch.from_numpy(flat).to(gpu_device), torch.from_numpy(offs).to(gpu_device),
                          quantiles=QS).cpu().numpy()
            o.ingest(flat, offs)
            assert_same_quantiles(q, o.quantiles(QS), "fused quantiles", small_of(o, eps))
        else:
            ss.ingest(torch.from_numpy(flat).to(gpu_device), torch.from_numpy(offs).to(gpu_device))
            o.ingest(flat, offs)
        assert_same_state(ss, o, "seed %d call %d" % (seed, call))
    ss.close()
