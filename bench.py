"""Benchmark of the batched GKArray ingest path on MI355X.

Metric (BASELINE.json): values ingested/sec (node) @1M streams eps=0.01, plus
the fraction of the HBM roofline reached by the dominant kernel (k_ingest).

Workload (BASELINE.json configs[2], the metric's configuration, which fits one
GPU): 1,000,000 streams x 1,000 Pareto(1.5)+1 float64 values per GPU, eps=0.01.
One step = reset every sketch, ingest the whole batch and answer
quantiles([0.5, 0.9, 0.99]) for every stream: k_stats (n/sum/avg/min/max
chain) then one k_ingest pass (9 automatic flushes per stream at the
reference's flush points, then the query flush of the 91 pending values,
gk:197, and the rank walk from the on-chip table).  Inputs are generated on the GPU (synthetic, seeded)
and are resident in HBM before the timed region.

Multi-GPU (one process per GPU, streams are independent: no collective on the
data path).  Default for N > 1 is the metric's configuration, STRONG split:
the one 1M-stream cfg3 batch (the same seeded batch a single GPU runs) is
split by ``dist.stream_range`` into N contiguous stream ranges, one per rank
(cfg5: ``dist.balanced_assignment`` by stream length, longest first); value =
the batch's values / max-over-ranks time.  The weak line (every rank its own
1M streams, seed + rank) is measured in the same run and reported beside it
under "weak" (``--split weak`` makes it the headline; ``--no-weak`` skips it).

    python bench.py [--gpus N --steps K --warmup W]   (N > 1: starts N ranks itself)
    torchrun --nproc-per-node N bench.py --gpus N ...  (--gpus must equal the world size)
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sketches-py_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, MI355X_MICROARCH.md "Chip-level parameters"
HEADER_BYTES = 60       # per stream: cls, slot, pend, E, n, offs pair, min, max read; n, E, pend written


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="cfg3", choices=["cfg3", "cfg2", "cfg4", "cfg5"],
                    help="cfg3 (default, the metric's config): 1M streams x 1k Pareto values per GPU; "
                         "cfg2: 100k x 10k lognormal; cfg4: 10k streams x 1M lognormal values "
                         "row-sharded over the GPUs, merged by all-gather + rank-ordered fold; "
                         "cfg5: 100k streams, lengths clip(zipf(1.5), 1, 1e7) (one forced to 1e7), "
                         "lognormal, eps=0.001")
    ap.add_argument("--streams", type=int, default=None, help="override: streams per GPU (cfg4: total)")
    ap.add_argument("--values", type=int, default=None, help="override: values per stream (cfg4: total)")
    ap.add_argument("--eps", type=float, default=None, help="default 0.01 (cfg5: 0.001)")
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--cpu-sample", type=int, default=1_000_000,
                    help="streams of the same workload timed on the host engine (rank 0, N=1); "
                         "default: the whole cfg3 batch")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = the CPUs this process may use (capped by OMP_NUM_THREADS if set)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-all-cores", action="store_true",
                    help="also time the host engine on every CPU of the affinity set (beyond this job's share)")
    ap.add_argument("--exchange", default="allgather", choices=["allgather", "alltoall"],
                    help="cfg4 row-shard exchange over RCCL before the merge fold")
    ap.add_argument("--split", default="auto", choices=["auto", "strong", "weak"],
                    help="N > 1, cfg2/3/5: strong = split the one batch over the ranks by stream "
                         "(the metric's configuration; the default), weak = every rank its own batch")
    ap.add_argument("--no-weak", action="store_true", help="N > 1 strong: skip the weak line beside it")
    ap.add_argument("--proxy", type=int, default=0, metavar="N",
                    help="one process, one GPU: run only rank --proxy-rank's share of the N-way strong split "
                         "(the single-GPU proxy of an N-GPU run; DESIGN 7)")
    ap.add_argument("--proxy-rank", type=int, default=0)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = the host engine (libgkarray_cpu.so): split / dump checks on CPU only")
    ap.add_argument("--dump", default=None,
                    help="write this rank's quantiles and global stream ids to DUMP.rank<r>.npz (tests)")
    ap.add_argument("--virtual-shards", type=int, default=1,
                    help="cfg4 on one process: sketch K row shards on this GPU and fold them with "
                         "GKArray.merge in shard order (the merge work of a K-GPU run, without the exchange)")
    return ap.parse_args()


def make_input(S, L, seed, device, dist_name="pareto"):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    if dist_name == "pareto":
        u = torch.rand(S * L, dtype=torch.float64, device=device, generator=g)
        x = (1.0 - u).pow_(-1.0 / 1.5)  # numpy pareto(1.5) + 1 by inversion
        del u
    else:  # lognormal(0, 1)
        x = torch.randn(S * L, dtype=torch.float64, device=device, generator=g).exp_()
    offs = torch.arange(0, S * L + 1, L, dtype=torch.int64, device=device)
    return x, offs


def make_zipf_input(S, seed, device, cap=10_000_000):
    """cfg5: stream lengths clip(zipf(1.5), 1, cap) with stream 0 forced to cap
    (numpy default_rng(seed)), lognormal(0,1) values on the GPU."""
    lens = np.clip(np.random.default_rng(seed).zipf(1.5, S), 1, cap).astype(np.int64)
    lens[0] = cap
    offs = np.zeros(S + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.randn(int(offs[-1]), dtype=torch.float64, device=device, generator=g).exp_()
    return x, torch.from_numpy(offs).to(device)


def pmc_traffic(workload):
    """(HBM bytes per k_ingest launch, provenance) from PMC counters of this
    workload (profiles/pmc_traffic.json, written by scripts/profile_cfg3.sh
    from a rocprofv3 --pmc run).  The entry is stamped with the sha256 of the
    library that ran; it is used only when the library loaded now has the same
    hash (else None: a stale measurement is never reported)."""
    from gkarray_amd import _lib
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            e = json.load(f)[workload]
    except (OSError, KeyError, ValueError):
        return None, "no PMC profile of this workload"
    h = _lib.library_identity()["sha256"]
    if e.get("lib_sha256") != h:
        return None, "PMC profile was taken on library %s, not this one (%s)" % (
            str(e.get("lib_sha256"))[:12], h[:12])
    return e["traffic_bytes"], "PMC (2*FETCH_SIZE + WRITE_SIZE) of this library (sha256 %s), %s" % (
        h[:12], e.get("source", ""))


def _library_identity():
    from gkarray_amd import _lib
    return _lib.library_identity()


def algorithmic_bytes(ss, S, N, nq):
    """Bytes one fused k_ingest launch must move on a fresh batch (SURVEY
    8(d)): 8 B per value + offsets + 16 B per table entry read and written +
    8 B per pending value read and written + the header words + 8 B per
    quantile answer.  Sizes are read after an untimed identical step."""
    st = ss.stats()
    e_out = int(st["size"].to(torch.int64).sum().item())
    p_out = int(st["pending"].to(torch.int64).sum().item())  # 0: the query flushed them
    e_in = p_in = 0  # every step starts from reset sketches
    return (8 * N + 8 * (S + 1) + 16 * (e_in + e_out) + 8 * (p_in + p_out) + HEADER_BYTES * S
            + 8 * nq * S)


def host_cores():
    """CPUs this process may run on (cgroup / affinity), the machine's count,
    and the threads the baseline uses: every CPU of the affinity set, capped
    by OMP_NUM_THREADS when the box sets it (the GPU box's per-GPU CPU share)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS")
    threads = min(aff, int(cap)) if cap and cap.isdigit() and int(cap) > 0 else aff
    return threads, aff, os.cpu_count() or aff


# gkarray.py itself (Entry objects), cfg3 shape, 1 process per core, measured in
# the build container (BASELINE.md / SURVEY 6); the reference never travels to
# the GPU box, so it is quoted, not re-timed here
REFERENCE_CFG3_RATE = {"1core": 529e3, "8cores": 3.59e6}


def cpu_baseline(x, offs, sample, threads, eps, gpu_q, py_streams=2000, all_cores=False):
    """The reference path on the host, timed on this box (rank 0, N=1):
    * the product's host engine (libgkarray_cpu.so, StreamSet(device="cpu"),
      threads over streams) on the first `sample` streams of the same batch, on
      the box's CPU share for this job (OMP_NUM_THREADS: 16 of the machine's
      CPUs) -- also a parity check of the GPU quantiles on that sample; with
      `all_cores` a second leg on every CPU of the affinity set (opt-in: the
      box asks jobs to keep to their share);
    * the reference algorithm restated over parallel lists (oracle/gk_oracle.py,
      test infrastructure: no Entry objects, so ~3x faster than gkarray.py) on
      ONE core on the first `py_streams` streams, beside gkarray.py's own rate
      measured in the build container (REFERENCE_CFG3_RATE)."""
    from gkarray_amd import StreamSet
    o_all = offs[: sample + 1].cpu().numpy()
    nv = int(o_all[-1] - o_all[0])
    xs = x[int(o_all[0]): int(o_all[-1])].cpu()
    o_loc = torch.from_numpy(o_all - o_all[0])
    hs = StreamSet(sample, eps, device="cpu")
    hs.set_threads(threads)
    t0 = time.perf_counter()
    q = hs.ingest(xs, o_loc, quantiles=[0.5, 0.9, 0.99]).numpy()
    dt = time.perf_counter() - t0
    same = np.array_equal(q.view(np.int64), gpu_q[:sample].view(np.int64))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from gk_oracle import OracleGK
    ps = min(py_streams, sample)
    xn = xs.numpy()
    t1 = time.perf_counter()
    for s in range(ps):
        g = OracleGK(eps)
        g.add_many(xn[o_all[s] - o_all[0]: o_all[s + 1] - o_all[0]].tolist())
        g.quantiles([0.5, 0.9, 0.99])
    dpy = time.perf_counter() - t1
    npy = int(o_all[ps] - o_all[0])
    _, aff, ncpu = host_cores()
    out = dict(value=nv / dt, unit="values/s", cores=threads, kind="port",
               sample="%d streams, %d values (the first streams of the GPU workload), ingest + "
                      "quantiles([.5,.9,.99]) in the host engine libgkarray_cpu.so on %d threads (this job's "
                      "CPU share), %.2f s" % (sample, nv, threads, dt),
               parity_on_sample=bool(same), host_cpus=ncpu, affinity_cpus=aff,
               per_thread=nv / dt / threads,
               python_1core=dict(value=npy / dpy, unit="values/s", cores=1,
                                 sample="%d streams, %d values, the reference algorithm restated over parallel "
                                        "lists in pure Python (oracle/gk_oracle.py: no Entry objects, ~3x "
                                        "gkarray.py's speed), %.2f s" % (ps, npy, dpy)),
               reference_gkarray_py=dict(value_1core=REFERENCE_CFG3_RATE["1core"],
                                         value_8cores=REFERENCE_CFG3_RATE["8cores"], unit="values/s",
                                         source="gkarray.py itself (Entry objects), cfg3 shape, 1 process per "
                                                "core, measured in the build container (BASELINE.md, SURVEY 6); "
                                                "quoted, the reference does not run on the GPU box"))
    if all_cores and aff > threads:
        hs.reset()
        hs.set_threads(aff)
        t2 = time.perf_counter()
        hs.ingest(xs, o_loc, quantiles=[0.5, 0.9, 0.99])
        d2 = time.perf_counter() - t2
        out["all_cores"] = dict(value=nv / d2, unit="values/s", cores=aff,
                                sample="same %d streams on every CPU of the affinity set, %.2f s" % (sample, d2))
    else:
        out["all_cores"] = dict(value=None, cores=aff, estimate=nv / dt / threads * aff,
                                note="not run by default (the box allots %d CPUs to this job); estimate = "
                                     "per-thread rate x %d CPUs, bench.py --cpu-all-cores measures it"
                                     % (threads, aff))
    return out


def sub_batch(x, offs, idx):
    """Streams `idx` (ascending global ids, int64 CPU tensor) of the CSR batch
    (x, offs) as a contiguous CSR batch of their own, values in the same
    order: a slice when the ids are one range (cfg3 strong split), else a
    gather (cfg5's balanced assignment)."""
    dev = x.device
    k = int(idx.numel())
    if k == 0:
        return torch.zeros(1, dtype=torch.float64, device=dev), torch.zeros(1, dtype=torch.int64, device=dev)
    lo, hi = int(idx[0]), int(idx[-1]) + 1
    if hi - lo == k:
        a, b = int(offs[lo].item()), int(offs[hi].item())
        return x[a:b].clone(), (offs[lo:hi + 1] - a).contiguous()
    i_d = idx.to(dev)
    starts = offs[i_d]
    lens = offs[i_d + 1] - starts
    o = torch.zeros(k + 1, dtype=torch.int64, device=dev)
    o[1:] = torch.cumsum(lens, 0)
    tot = int(o[-1].item())
    seg = torch.repeat_interleave(torch.arange(k, device=dev), lens)
    pos = starts[seg] + (torch.arange(tot, device=dev) - o[:-1][seg])
    return x[pos].contiguous(), o


def rank_streams(workload, offs, world, rank):
    """This rank's streams of the one batch (strong split): a contiguous
    `stream_range` (cfg2 / cfg3: equal lengths), or the longest-first
    `balanced_assignment` by stream length (cfg5's Zipf lengths)."""
    from gkarray_amd import dist as gd
    S = offs.numel() - 1
    if workload == "cfg5":
        lens = (offs[1:] - offs[:-1]).cpu()
        return gd.balanced_assignment(lens, world)[rank]
    a, b = gd.stream_range(S, world, rank)
    return torch.arange(a, b, dtype=torch.int64)


def free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` (N > 1) outside a torchrun environment: start the N
    ranks as ONE child launcher (torch.distributed.run, one process per GPU,
    rendezvous on 127.0.0.1) and return its exit code.  This process has made
    no GPU call (only torch.cuda.device_count(), which does not initialise the
    device) and is not replaced: the ranks are children; rank 0 prints the
    line."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr=127.0.0.1", "--master-port=%d" % free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    a = parse()
    on_gpu = a.device == "cuda"
    # GK_BENCH_REHEARSE=1: rehearse the N-rank path on fewer GPUs (ranks share
    # devices, gloo for the timing collectives; the numbers mean nothing)
    rehearse = os.environ.get("GK_BENCH_REHEARSE") == "1" or not on_gpu
    if a.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if on_gpu and not rehearse and a.gpus > torch.cuda.device_count():
        sys.exit("bench.py: --gpus %d but this node has %d GPU(s) (GK_BENCH_REHEARSE=1 shares them)"
                 % (a.gpus, torch.cuda.device_count()))
    if "WORLD_SIZE" not in os.environ:
        if a.gpus > 1:
            sys.exit(launch_ranks(a.gpus))
    elif int(os.environ["WORLD_SIZE"]) != a.gpus:
        sys.exit("bench.py: --gpus %d but the launcher started %s rank(s)" % (a.gpus, os.environ["WORLD_SIZE"]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if on_gpu:
        if rehearse:
            local %= max(torch.cuda.device_count(), 1)
            if world > max(torch.cuda.device_count(), 1):
                # ranks share a device: no rank's k_ingest_wg grid may spin on
                # CUs ahead of its k_long_prep (GK_WG_EARLY, gk_capi.cpp)
                os.environ.setdefault("GK_WG_EARLY", "0")
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if world > 1:
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    from gkarray_amd import StreamSet

    def gsync():
        if on_gpu:
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    def allreduce(v, op):
        if world == 1:
            return v
        import torch.distributed as dist
        t = torch.tensor([v], dtype=torch.float64, device="cpu" if rehearse else dev)
        dist.all_reduce(t, op=op)
        return float(t.item())

    defaults = {"cfg3": (1_000_000, 1000, "pareto"), "cfg2": (100_000, 10_000, "lognormal"),
                "cfg4": (10_000, 1_000_000, "lognormal"), "cfg5": (100_000, 0, "zipf-lengths lognormal")}
    S, L, dist_name = defaults[a.workload]
    S = a.streams or S
    L = a.values or L
    if a.eps is None:
        a.eps = 0.001 if a.workload == "cfg5" else 0.01
    qs = [0.5, 0.9, 0.99]
    split = a.split if a.split != "auto" else ("strong" if world > 1 or a.proxy > 1 else "weak")
    if a.proxy > 1 and (world > 1 or not 0 <= a.proxy_rank < a.proxy):
        sys.exit("bench.py: --proxy runs one rank's share in ONE process (0 <= --proxy-rank < --proxy)")
    if a.workload == "cfg4":
        split = "rows"

    def make_batch(seed):
        if a.workload == "cfg5":
            return make_zipf_input(S, seed, dev, cap=a.values or 10_000_000)
        return make_input(S, L, seed, dev, dist_name)

    # Untimed warm-up: the W steps asked for, then more until the warm-up has
    # lasted min_warm seconds.  The shader clock ramps over tens of ms of
    # load (measured 2.00 GHz after 4 cfg3 steps at 125k streams, 2.38 GHz
    # after 100; 1M streams: 2.00 GHz after 1 step, 2.38 after 40 --
    # profiles/r05/r05Z_clock_ramp.txt): without it a short run times the
    # ramp, not the engine.  The extra count is agreed over ranks (the same
    # number of steps everywhere: cfg4's steps hold collectives).
    min_warm = float(os.environ.get("GK_BENCH_MIN_WARM_S", "0.3" if on_gpu else "0"))
    warm_info = {"steps": 0, "seconds": 0.0}

    def timed(step, timed_sets):
        """W (+ extra, see min_warm) untimed steps, then K steps bracketed by barrier + device sync;
        (max-over-ranks seconds, launch ms summed over sets, stats ms, launches, last result)."""
        gsync()
        tw = time.perf_counter()
        nw = 0
        for _ in range(a.warmup):
            step()
            nw += 1
        if min_warm > 0:
            if nw == 0:
                step()
                nw = 1
            import torch.distributed as _dd
            for _ in range(4):  # (steps get faster as the clock ramps: re-estimate)
                gsync()
                el = time.perf_counter() - tw
                extra = 0 if el >= min_warm else min(5000, int(math.ceil((min_warm - el) / (el / nw))))
                extra = int(allreduce(float(extra), _dd.ReduceOp.MAX))
                if extra == 0:
                    break
                for _ in range(extra):
                    step()
                nw += extra
        gsync()
        warm_info["steps"], warm_info["seconds"] = nw, time.perf_counter() - tw
        for t_ss in timed_sets:
            t_ss.timing(True, stats=os.environ.get("GK_BENCH_STATS_TIMING") == "1")
            t_ss.read_timing()
        barrier()
        gsync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            q = step()
        gsync()
        barrier()
        dt = time.perf_counter() - t0
        f_ms = s_ms = 0.0
        n_l = 0
        for t_ss in timed_sets:  # every shard's ingest launches (cfg4 virtual shards)
            f, s_, n = t_ss.read_timing()
            t_ss.timing(False)
            f_ms, s_ms, n_l = f_ms + f, s_ms + s_, n_l + n
        import torch.distributed as _d
        return allreduce(dt, _d.ReduceOp.MAX) if world > 1 else dt, f_ms, s_ms, n_l, q

    K = 1
    idx = None
    if a.workload == "cfg4":
        # rows of every stream split over the ranks: this rank sketches its
        # L/world values of each of the S streams, then the shards are merged
        from gkarray_amd import dist as gd
        K = max(1, a.virtual_shards) if world == 1 else 1
        L = L // (world * K)
        N = S * L * K
        S_loc = S
        if K == 1:
            x, offs = make_input(S, L, a.seed + rank, dev, dist_name)
            ss = StreamSet(S, a.eps, device=dev)
            # fold sets allocated once; one host size sync per step (dist.RowShardMerger)
            merger = gd.RowShardMerger(S, a.eps, dev, exchange=a.exchange)

            def step():
                ss.reset()
                ss.ingest(x, offs, sync=False)
                return merger(ss).quantiles(qs)
        else:
            shards = [make_input(S, L, a.seed + k, dev, dist_name) for k in range(K)]
            sets = [StreamSet(S, a.eps, device=dev) for _ in range(K)]
            ss = sets[0]

            def step():
                for (xk, ok), sk in zip(shards, sets):
                    sk.reset()
                    sk.ingest(xk, ok, sync=False)
                sets[0].merge_from(sets[1:])  # sk0.merge(sk1)...merge(skK-1), gk:111-154
                return sets[0].quantiles(qs)
    else:
        if split == "strong":
            # the one batch every rank would run alone (same seed on every
            # rank), cut to this rank's streams
            x_full, offs_full = make_batch(5 if a.workload == "cfg5" else a.seed)
            if a.proxy > 1:
                idx = rank_streams(a.workload, offs_full, a.proxy, a.proxy_rank)
            else:
                idx = rank_streams(a.workload, offs_full, world, rank)
            x, offs = sub_batch(x_full, offs_full, idx)
            del x_full, offs_full
        else:
            x, offs = make_batch((5 if a.workload == "cfg5" else a.seed) + rank)
        S_loc = offs.numel() - 1
        N = int(offs[-1].item())
        ss = StreamSet(S_loc, a.eps, device=dev)

        def step():
            ss.reset()
            # add every value, then quantiles(qs) -- one fused pass (gk_ingest_quantiles),
            # enqueued without a host synchronisation (the timed region syncs at its end)
            return ss.ingest(x, offs, quantiles=qs, sync=False)

    # algorithmic bytes of one k_ingest_small launch (untimed identical step)
    timed_sets = [ss]
    if a.workload == "cfg4" and K > 1:
        # one shard's ingest launch (before the merges flush the sets)
        sets[0].reset()
        sets[0].ingest(shards[0][0], shards[0][1])
        bytes_per_launch = algorithmic_bytes(sets[0], S, S * L, 0)
        timed_sets = sets
        step()
    else:
        step()
        bytes_per_launch = algorithmic_bytes(ss, S_loc, N, len(qs) if a.workload != "cfg4" else 0)

    import torch.distributed as _d
    dt, flush_ms, stats_ms, launches, q = timed(step, timed_sets)
    if a.dump:
        np.savez("%s.rank%d.npz" % (a.dump, rank), q=q.cpu().numpy(),
                 idx=(idx if idx is not None else torch.arange(S_loc)).numpy())

    traffic, traffic_src = pmc_traffic(a.workload)
    if traffic is not None and (not on_gpu or S_loc != defaults[a.workload][0] or
                                (a.workload != "cfg5" and L != defaults[a.workload][1])):
        traffic, traffic_src = None, "the PMC profile is of the whole single-GPU workload, not this batch"
    total_values = allreduce(float(N), _d.ReduceOp.SUM) * a.steps if world > 1 else N * a.steps
    value = total_values / dt
    ms_step = dt / a.steps * 1e3
    k_ms = flush_ms / max(launches, 1)
    achieved = bytes_per_launch / (k_ms * 1e-3) / 1e9 if k_ms > 0 else None
    ratio = traffic / bytes_per_launch if traffic else None
    per_rank = None
    n_ranks = world
    if world > 1:
        # every rank's own launch time and algorithmic bytes; the headline
        # roofline is the SLOWEST rank's launch on that rank's bytes (the node
        # rate is bound by it), the others are listed beside it
        import torch.distributed as dist
        n_ranks = dist.get_world_size()  # the ranks that joined the process group
        mine = {"rank": rank, "device": str(dev), "streams": S_loc, "values": N, "launch_ms": k_ms,
                "bytes_per_launch": bytes_per_launch,
                "frac": (bytes_per_launch / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if k_ms > 0 else None}
        per_rank = [None] * n_ranks
        dist.all_gather_object(per_rank, mine)
        slow = max(per_rank, key=lambda r: r["launch_ms"])
        k_ms, bytes_per_launch = slow["launch_ms"], slow["bytes_per_launch"]
        achieved = bytes_per_launch / (k_ms * 1e-3) / 1e9 if k_ms > 0 else None
        ratio = traffic / bytes_per_launch if traffic else None
    if a.workload == "cfg4":
        parallelism = ("row-sharded x%d, RCCL %s + merge" % (world, a.exchange) if K == 1 else
                       "row-sharded: %d virtual shards on 1 GPU, merge fold (no exchange)" % K)
        workload = ("cfg4: %d streams x %d values, row-sharded %d values per stream per shard "
                    "(%d GPU x %d shard), eps=%g, ingest + %s + rank-ordered merge + quantiles"
                    % (S, L * world * K, L, world, K, a.eps, a.exchange))
    else:
        lens_txt = ("%d" % L) if a.workload != "cfg5" else "clip(zipf(1.5),1,1e7)"
        if split == "strong":
            if a.proxy > 1:
                parallelism = ("PROXY of a %d-GPU strong split on 1 GPU: rank %d's share only, by %s (the node "
                               "rate of an N-rank run is the batch's values / the slowest share's time)"
                               % (a.proxy, a.proxy_rank, "balanced_assignment (longest first)"
                                  if a.workload == "cfg5" else "stream_range"))
            else:
                parallelism = ("stream-sharded, strong: the one %d-stream batch split over %d rank(s) by %s "
                               "(no collective)" % (S, world, "balanced_assignment (longest first)"
                                                    if a.workload == "cfg5" else "stream_range"))
            workload = ("%s: %d streams x %s values (one batch, node), %d on this rank, eps=%g, %s, "
                        "ingest + quantiles(.5,.9,.99)" % (a.workload, S, lens_txt, S_loc, a.eps, dist_name))
        else:
            parallelism = "stream-sharded x%d, weak: every rank its own batch (no collective)" % world
            workload = ("%s: %d streams x %s values per GPU, eps=%g, %s, ingest + quantiles(.5,.9,.99)"
                        % (a.workload, S, lens_txt, a.eps, dist_name))
    line = {
        "metric": "values ingested/sec (node) @1M streams eps=0.01; % of HBM roofline",
        "value": value,
        "unit": "values/s",
        "n_gpus": n_ranks,
        "steps": a.steps,
        "warmup": a.warmup,
        "warmup_run": {"steps": warm_info["steps"], "seconds": round(warm_info["seconds"], 4),
                       "min_seconds": min_warm, "why": "untimed; the GPU clock ramps over tens of ms of load "
                       "(profiles/r05/r05Z_clock_ramp.txt)"},
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak" if split == "weak" else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: %s float64 generated on %s (seed %d%s)" % (
            "Pareto(1.5)+1" if dist_name == "pareto" else "lognormal(0,1)", "GPU" if on_gpu else "CPU",
            5 if a.workload == "cfg5" else a.seed, " + rank" if split in ("weak", "rows") else ", one batch"),
        "config": {"workload": workload, "split": split,
                   "streams_per_gpu": S_loc, "values_per_stream": L if a.workload != "cfg5" else N / max(S_loc, 1),
                   "eps": a.eps,
                   "parallelism": parallelism},
        "roofline": {"bound": "hbm", "kernel": "k_ingest_small" if a.workload != "cfg5" else
                     "k_ingest<2048> beside k_ingest_wg (the span of both)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
                     "traffic_ratio": ratio, "traffic_source": traffic_src,
                     "bytes_per_launch": bytes_per_launch, "launch_ms": k_ms,
                     "launch_ms_source": ("HIP events recorded by the small-class launch itself (hipExtLaunchKernel "
                                          "start/stop), mean over the timed steps" if a.workload != "cfg5" else
                                          "HIP event markers around the class-0 launch and k_ingest_wg beside it, "
                                          "mean over the timed steps"),
                     "stats_kernel_ms": (stats_ms / max(launches, 1)
                                         if os.environ.get("GK_BENCH_STATS_TIMING") == "1" else None)},
        "library": _library_identity(),
    }
    if per_rank is not None:
        line["roofline"]["rank"] = slow["rank"]
        line["roofline"]["per_rank"] = per_rank
        line["roofline"]["note"] = ("N > 1: achieved / frac / launch_ms / bytes_per_launch of the slowest rank's "
                                    "launch on that rank's own bytes; every rank under per_rank")
    if not on_gpu:
        line["device"] = "cpu (host engine libgkarray_cpu.so): a split check, not a GPU number"
    if world > 1 and split == "strong" and not a.no_weak:
        # the weak line beside it: every rank its own whole batch (seed + rank)
        del ss, x, offs, q
        xw, ow = make_batch((5 if a.workload == "cfg5" else a.seed) + rank)
        nw = int(ow[-1].item())
        sw = StreamSet(ow.numel() - 1, a.eps, device=dev)

        def step_w():
            sw.reset()
            return sw.ingest(xw, ow, quantiles=qs, sync=False)

        step_w()
        dtw, fw, _, lw, _ = timed(step_w, [sw])
        tot_w = allreduce(float(nw), _d.ReduceOp.SUM) * a.steps
        line["weak"] = {"value": tot_w / dtw, "ms_per_step": dtw / a.steps * 1e3, "scaling": "weak",
                        "streams_per_gpu": S, "launch_ms": fw / max(lw, 1),
                        "note": "every rank its own %d-stream batch (seed + rank), same K/W" % S}
    if rank == 0 and world == 1 and on_gpu and not a.no_cpu and a.workload != "cfg4":
        threads = a.cpu_threads or host_cores()[0]
        sample = min(a.cpu_sample, S)
        if a.workload == "cfg5":  # the long streams dominate: a bounded prefix of streams
            sample = min(sample, 20000)
        line["cpu_baseline"] = cpu_baseline(x, offs, sample, threads, a.eps, q.cpu().numpy(),
                                            all_cores=a.cpu_all_cores)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
