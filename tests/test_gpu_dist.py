"""The multi-rank row-shard path on DEVICE tensors:
RowShardMerger at world 1 on a GPU set vs the oracle, and world 2 on one GPU
over gloo (tests/rehearse_rowshard.py under torch.distributed.run: ranks
exchange device payloads -- staged through host memory by gloo -- import
them and fold in rank order), allgather and alltoall, bit-exact vs the
oracle's left fold."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from gk_oracle_c import OracleSet
from parity_util import assert_same_state

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_row_shard_merger_world1_device(gpu_device):
    from gkarray_amd import StreamSet
    from gkarray_amd import dist as gd
    rng = np.random.default_rng(91)
    S, eps = 400, 0.01
    lens = rng.integers(0, 2000, S)
    seqs = [rng.lognormal(0, 1, int(L)) for L in lens]
    offs = np.zeros(S + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    flat = np.concatenate(seqs)
    ss = StreamSet(S, eps, device=gpu_device)
    merger = gd.RowShardMerger(S, eps, gpu_device)
    o = OracleSet(S, eps)
    o.ingest(flat, offs)
    for _ in range(2):
        ss.reset()
        ss.ingest(torch.from_numpy(flat).to(gpu_device), torch.from_numpy(offs).to(gpu_device), sync=False)
        m = merger(ss)
        assert m.device.type == "cuda" and merger.range == (0, S)
        assert_same_state(m, o, "RowShardMerger world 1")


@pytest.mark.parametrize("exchange", ["allgather", "alltoall"])
def test_row_shard_world2_rehearsal_on_device(exchange):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=%d" % free_port(),
           os.path.join(HERE, "rehearse_rowshard.py"), "--exchange", exchange]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OMP_NUM_THREADS="4"))
    assert r.returncode == 0 and "REHEARSAL OK" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
