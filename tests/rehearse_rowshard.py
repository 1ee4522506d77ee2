"""Rehearsal of the row-shard exchange on DEVICE tensors (SURVEY 8(e),
gk:111-154): N ranks share one GPU over gloo (dist.py stages the device
payloads through host memory for gloo; RCCL moves them directly), each rank
sketches its row shard of the same S streams in a StreamSet on cuda:0, then

  * dist.RowShardMerger (exchange "allgather" or "alltoall"), called twice
    (fold sets reused): every rank ends with the rank-ordered left fold
    sk_0.merge(sk_1)...merge(sk_{N-1}) of its stream range, imported from the
    device payloads received from the other ranks;
  * dist.fold_packed_allgather: the C-ABI packed states (gk_pack ->
    all-gather -> gk_fold_packed), every rank holds the whole fold.

Rank 0 compares every stream (tables, pending values, n/min/max/sum/avg, bit
patterns) with the oracle's left fold of the same shards and prints
"REHEARSAL OK".  Test infrastructure (it imports the oracle); run by
tests/test_gpu_dist.py as

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port P tests/rehearse_rowshard.py --exchange allgather
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "sketches-py_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def shard(rank, S, eps, seed=11):
    rng = np.random.default_rng(seed * 1000 + rank)
    P = int(1.0 / eps) + 1
    lens = rng.integers(0, 6 * P, S)
    lens[rank % S] = 0  # an empty side
    vals = [rng.lognormal(0, 1, int(L)) for L in lens]
    offs = np.zeros(S + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    return (np.concatenate(vals) if S else np.zeros(0)), offs


def state_of(ss):
    """Every stream's state as host numpy arrays (floats as int64 bit patterns)."""
    to, v, g, d = ss.tables()
    po, pv = ss.pending()
    st = ss.stats()
    b = lambda t: t.cpu().contiguous().view(torch.int64).numpy().copy()
    return dict(offs=to.cpu().numpy().copy(), v=b(v), g=g.cpu().numpy().astype(np.int64),
                d=d.cpu().numpy().astype(np.int64), poffs=po.cpu().numpy().copy(), pv=b(pv),
                n=st["n"].cpu().numpy().copy(), min=b(st["min"]), max=b(st["max"]), sum=b(st["sum"]),
                avg=b(st["avg"]))


def oracle_fold(world, S, eps):
    from gk_oracle_c import OracleSet
    ref = OracleSet(S, eps)
    ref.ingest(*shard(0, S, eps))
    for r in range(1, world):
        o = OracleSet(S, eps)
        o.ingest(*shard(r, S, eps))
        ref.merge(o)
    to, v, g, d = ref.tables()
    po, pv = ref.pending()
    st = ref.stats()
    b = lambda a: np.ascontiguousarray(a, dtype=np.float64).view(np.int64)
    return dict(offs=to, v=b(v), g=np.asarray(g, np.int64), d=np.asarray(d, np.int64), poffs=po, pv=b(pv),
                n=st["n"], min=b(st["min"]), max=b(st["max"]), sum=b(st["sum"]), avg=b(st["avg"]))


def compare(got, ref, a, b, what):
    """got: state of streams [a, b); ref: state of all streams."""
    for k in ("n", "min", "max", "sum", "avg"):
        if not np.array_equal(got[k], ref[k][a:b]):
            return "%s: %s differs" % (what, k)
    for s in range(a, b):
        i = s - a
        for k, o in (("v", "offs"), ("g", "offs"), ("d", "offs"), ("pv", "poffs")):
            x = got[k][got[o][i]:got[o][i + 1]]
            y = ref[k][ref[o][s]:ref[o][s + 1]]
            if not np.array_equal(x, y):
                return "%s: stream %d %s differs" % (what, s, k)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--exchange", default="allgather", choices=["allgather", "alltoall"])
    ap.add_argument("--streams", type=int, default=300)
    ap.add_argument("--eps", type=float, default=0.01)
    ap.add_argument("--device", default="cuda:0", help="cuda:0, or cpu (the host engine: CPU dry run)")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    from gkarray_amd import StreamSet
    from gkarray_amd import dist as gd
    S, eps = a.streams, a.eps
    flat, offs = shard(rank, S, eps)
    x, o = torch.from_numpy(flat).to(dev), torch.from_numpy(offs).to(dev)
    ss = StreamSet(S, eps, device=dev)
    merger = gd.RowShardMerger(S, eps, dev, exchange=a.exchange)
    res = None
    for step in range(2):  # the merger is reused: same fold sets, fresh exchange
        ss.reset()
        ss.ingest(x, o, sync=False)
        m = merger(ss)
        assert m.device.type == dev.type
        res = state_of(m)
    ss.reset()
    ss.ingest(x, o)
    dst = StreamSet(S, eps, device=dev)
    gd.fold_packed_allgather(ss, dst)
    packed = state_of(dst) if rank == 0 else None
    gathered = [None] * world
    dist.all_gather_object(gathered, (rank, merger.range, res))
    ok = True
    if rank == 0:
        ref = oracle_fold(world, S, eps)
        covered = []
        for r, (lo, hi), st in sorted(gathered, key=lambda t: t[0]):
            err = compare(st, ref, lo, hi, "RowShardMerger(%s) rank %d" % (a.exchange, r))
            if err:
                print("MISMATCH", err, flush=True)
                ok = False
            covered.extend(range(lo, hi))
        if covered != list(range(S)):
            print("MISMATCH: ranges do not cover the streams", flush=True)
            ok = False
        err = compare(packed, ref, 0, S, "fold_packed_allgather")
        if err:
            print("MISMATCH", err, flush=True)
            ok = False
        if ok:
            print("REHEARSAL OK: world %d, %s, %d streams, RowShardMerger x2 + packed fold == oracle fold"
                  % (world, a.exchange, S), flush=True)
    flag = torch.tensor([0 if ok else 1], dtype=torch.int64)
    dist.all_reduce(flag)
    dist.destroy_process_group()
    sys.exit(int(flag.item() != 0))


if __name__ == "__main__":
    main()
