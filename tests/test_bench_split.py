"""bench.py's strong split: the metric's ONE batch cut
over N ranks by stream -- `stream_range` for cfg3's equal lengths,
`balanced_assignment` for cfg5's Zipf lengths -- gives every stream exactly
the quantiles the single-rank run gives it (bit patterns compared).

CPU: bench.py on the host engine (--device cpu) at world 1 and world 2 over
gloo.  GPU: the same at world 2 with both ranks on one card
(GK_BENCH_REHEARSE=1), against the single-rank GPU run."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_bench(args, world, dump, env_extra=None):
    env = dict(os.environ, OMP_NUM_THREADS="4", **(env_extra or {}))
    if world == 1:
        cmd = [sys.executable, BENCH]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % world,
               "--master-addr=127.0.0.1", "--master-port=%d" % free_port(), BENCH]
    cmd += args + ["--steps", "1", "--warmup", "0", "--no-cpu", "--dump", dump]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def gather(dump, world, S):
    parts = [np.load("%s.rank%d.npz" % (dump, r)) for r in range(world)]
    idx = np.concatenate([p["idx"] for p in parts])
    assert np.array_equal(np.sort(idx), np.arange(S)), "every stream on exactly one rank"
    q = np.zeros((S, parts[0]["q"].shape[1]))
    for p in parts:
        q[p["idx"]] = p["q"]
    return q, parts


def check_split(tmp_path, args, S, world, device_args, env_extra=None, min_ranks_len_ratio=None):
    one = run_bench(args + device_args, 1, str(tmp_path / "one"), env_extra)
    assert one["scaling"] == "weak" and one["config"]["split"] == "weak"
    line = run_bench(args + device_args, world, str(tmp_path / "split"), env_extra)
    assert line["scaling"] == "strong" and line["config"]["split"] == "strong" and line["n_gpus"] == world
    assert "weak" in line and line["weak"]["scaling"] == "weak"
    q1 = np.load(str(tmp_path / "one") + ".rank0.npz")["q"]
    qn, parts = gather(str(tmp_path / "split"), world, S)
    assert np.array_equal(q1.view(np.int64), qn.view(np.int64)), "strong split changed some stream's quantiles"
    return parts


@pytest.mark.parametrize("world", [2, 3])
def test_strong_split_cfg3_cpu(tmp_path, world):
    check_split(tmp_path, ["--workload", "cfg3", "--streams", "1500", "--values", "1000"], 1500, world,
                ["--device", "cpu"])


def test_strong_split_cfg5_balanced_cpu(tmp_path):
    S = 1200
    parts = check_split(tmp_path, ["--workload", "cfg5", "--streams", str(S), "--values", "30000"], S, 2,
                        ["--device", "cpu"])
    # the longest stream (id 0, forced to the cap) is alone against the rest
    # of the batch: balanced_assignment spreads the remaining length
    assert any(0 in p["idx"] for p in parts)
    assert all(len(p["idx"]) > 0 for p in parts)


@pytest.mark.gpu
def test_strong_split_cfg3_rehearsal_on_device(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    check_split(tmp_path, ["--workload", "cfg3", "--streams", "20000", "--values", "1000"], 20000, 2, [],
                env_extra={"GK_BENCH_REHEARSE": "1"})


@pytest.mark.gpu
def test_strong_split_cfg5_rehearsal_on_device(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    check_split(tmp_path, ["--workload", "cfg5", "--streams", "5000", "--values", "200000"], 5000, 2, [],
                env_extra={"GK_BENCH_REHEARSE": "1"})
