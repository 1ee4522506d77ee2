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


def run_bench(args, world, dump, env_extra=None, launcher="torchrun"):
    """launcher "torchrun": the driver's form (torch.distributed.run ... bench.py
    --gpus N); "self": plain `bench.py --gpus N`, which starts the N ranks."""
    env = dict(os.environ, OMP_NUM_THREADS="4", **(env_extra or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    if world == 1 or launcher == "self":
        cmd = [sys.executable, BENCH]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % world,
               "--master-addr=127.0.0.1", "--master-port=%d" % free_port(), BENCH]
    cmd += args + ["--gpus", str(world), "--steps", "1", "--warmup", "0", "--no-cpu", "--dump", dump]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0's line only
    return json.loads(lines[0])


def gather(dump, world, S):
    parts = [np.load("%s.rank%d.npz" % (dump, r)) for r in range(world)]
    idx = np.concatenate([p["idx"] for p in parts])
    assert np.array_equal(np.sort(idx), np.arange(S)), "every stream on exactly one rank"
    q = np.zeros((S, parts[0]["q"].shape[1]))
    for p in parts:
        q[p["idx"]] = p["q"]
    return q, parts


def check_split(tmp_path, args, S, world, device_args, env_extra=None, launcher="torchrun"):
    one = run_bench(args + device_args, 1, str(tmp_path / "one"), env_extra)
    assert one["scaling"] == "weak" and one["config"]["split"] == "weak" and one["n_gpus"] == 1
    line = run_bench(args + device_args, world, str(tmp_path / "split"), env_extra, launcher)
    assert line["scaling"] == "strong" and line["config"]["split"] == "strong" and line["n_gpus"] == world
    assert "weak" in line and line["weak"]["scaling"] == "weak"
    # N > 1: every rank's launch under roofline.per_rank,
    # the headline roofline = the slowest rank's launch on that rank's bytes
    rf = line["roofline"]
    pr = rf["per_rank"]
    assert [r["rank"] for r in pr] == list(range(world))
    assert sum(r["streams"] for r in pr) == S and sum(r["values"] for r in pr) > 0
    slow = max(pr, key=lambda r: r["launch_ms"])
    assert rf["rank"] == slow["rank"] and rf["launch_ms"] == slow["launch_ms"]
    assert rf["bytes_per_launch"] == slow["bytes_per_launch"]
    if slow["launch_ms"] > 0:
        assert abs(rf["frac"] - slow["frac"]) <= 1e-12 * max(1.0, abs(slow["frac"]))
    q1 = np.load(str(tmp_path / "one") + ".rank0.npz")["q"]
    qn, parts = gather(str(tmp_path / "split"), world, S)
    assert np.array_equal(q1.view(np.int64), qn.view(np.int64)), "strong split changed some stream's quantiles"
    return parts


@pytest.mark.parametrize("world", [2, 3])
def test_strong_split_cfg3_cpu(tmp_path, world):
    check_split(tmp_path, ["--workload", "cfg3", "--streams", "1500", "--values", "1000"], 1500, world,
                ["--device", "cpu"])


def test_gpus_flag_starts_the_ranks_cpu(tmp_path):
    """`bench.py --gpus 3` with no launcher around it runs 3 ranks (VERDICT r04
    item 2: --gpus used to be ignored), strong split bit-identical to 1 rank."""
    check_split(tmp_path, ["--workload", "cfg3", "--streams", "900", "--values", "500"], 900, 3,
                ["--device", "cpu"], launcher="self")


def test_gpus_flag_must_match_the_world(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=%d" % free_port(), BENCH, "--gpus", "3", "--device", "cpu",
           "--streams", "100", "--values", "100", "--steps", "1", "--warmup", "0", "--no-cpu"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and "launcher started 2 rank(s)" in r.stderr


def test_strong_split_cfg5_balanced_cpu(tmp_path):
    S = 1200
    parts = check_split(tmp_path, ["--workload", "cfg5", "--streams", str(S), "--values", "30000"], S, 2,
                        ["--device", "cpu"])
    # the longest stream (id 0, forced to the cap) is alone against the rest
    # of the batch: balanced_assignment spreads the remaining length
    assert any(0 in p["idx"] for p in parts)
    assert all(len(p["idx"]) > 0 for p in parts)


def test_proxy_ranks_cover_the_split_cpu(tmp_path):
    """`bench.py --proxy N --proxy-rank R` (one process: rank R's share of the
    N-way strong split, the single-GPU proxies of DESIGN 7) runs exactly the
    streams rank R of an N-rank run would, with the same quantiles."""
    S, N = 1000, 3
    args = ["--workload", "cfg5", "--streams", str(S), "--values", "20000", "--device", "cpu"]
    run_bench(args, 1, str(tmp_path / "one"))
    q1 = np.load(str(tmp_path / "one") + ".rank0.npz")["q"]
    seen = []
    for r in range(N):
        line = run_bench(args + ["--proxy", str(N), "--proxy-rank", str(r)], 1, str(tmp_path / ("p%d" % r)))
        assert line["n_gpus"] == 1 and "PROXY" in line["config"]["parallelism"]
        d = np.load(str(tmp_path / ("p%d" % r)) + ".rank0.npz")
        assert np.array_equal(d["q"].view(np.int64), q1[d["idx"]].view(np.int64))
        seen.append(d["idx"])
    assert np.array_equal(np.sort(np.concatenate(seen)), np.arange(S))


@pytest.mark.gpu
def test_strong_split_cfg3_rehearsal_on_device(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    check_split(tmp_path, ["--workload", "cfg3", "--streams", "20000", "--values", "1000"], 20000, 2, [],
                env_extra={"GK_BENCH_REHEARSE": "1"})


@pytest.mark.gpu
def test_gpus_flag_on_device(tmp_path):
    """`GK_BENCH_REHEARSE=1 bench.py --gpus 2` runs two ranks on one card and
    prints n_gpus 2; `bench.py --gpus K` beyond the node's GPUs fails loudly."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    check_split(tmp_path, ["--workload", "cfg3", "--streams", "20000", "--values", "1000"], 20000, 2, [],
                env_extra={"GK_BENCH_REHEARSE": "1"}, launcher="self")
    n = torch.cuda.device_count()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GK_BENCH_REHEARSE")}
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n + 1), "--steps", "1", "--warmup", "0", "--no-cpu"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and "GPU(s)" in r.stderr, r.stderr[-2000:]


@pytest.mark.gpu
def test_strong_split_cfg5_rehearsal_on_device(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    check_split(tmp_path, ["--workload", "cfg5", "--streams", "5000", "--values", "200000"], 5000, 2, [],
                env_extra={"GK_BENCH_REHEARSE": "1"})
