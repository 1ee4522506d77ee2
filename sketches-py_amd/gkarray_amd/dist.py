"""Multi-GPU helpers: one process per GPU, torch.distributed (RCCL over xGMI
with backend "nccl"; gloo on CPU for tests).

Two ways streams meet several GPUs:

* **stream-sharded** -- every stream lives on exactly one rank
  (``stream_range``, or ``balanced_assignment`` by length); ranks never talk
  on the data path.  bench.py splits the metric's ONE batch this way (strong
  scaling: the node's work is fixed as N grows).
* **row-sharded** -- every rank sketched a slice of the rows of the SAME
  streams; the sketches are combined with the reference's left fold
  ``sk_0.merge(sk_1) ... .merge(sk_{N-1})`` (gk:111-154).  ``merge_row_shards``
  hands every rank the N shard states of the streams of its own range and the
  rank folds them in rank order -- the merge work is split N ways and the
  result is stream-sharded.  The default exchange is the all-gather the
  north star names (every rank's whole state to every rank);
  ``exchange="alltoall"`` (``alltoall_states``: rank r sends each peer only
  that peer's stream range, so every table crosses xGMI once) moves 1/(N-1)
  of the bytes -- SURVEY 8(f)'s next step, same fold, same results.

The exchange helpers (``pack_state`` / ``unpack_state`` / ``all_gather_varlen``
/ ``allgather_states`` / ``alltoall_states`` / ``slice_state``) work on tensors of any device, so the
same code runs over gloo on CPU tensors.

``fold_packed_allgather`` is the same row-shard combine through the C ABI's
packed states (gk_pack / gk_fold_packed): one contiguous buffer per rank,
padded to the largest, one all-gather, the rank-ordered fold in the library
-- the call sequence a non-Python host (cgo / JNI over RCCL or MPI) uses,
INTEGRATION.md.
"""
import torch
import torch.distributed as dist

__all__ = ["stream_range", "balanced_assignment", "pack_state", "unpack_state", "all_gather_varlen",
           "allgather_states", "alltoall_states", "slice_state", "concat_states", "fold_states",
           "merge_row_shards", "RowShardMerger", "allgather_packed", "fold_packed_allgather"]

_F64 = ("v", "pv", "min", "max", "sum", "avg")
_I64 = ("offs", "poffs", "n")
_I32 = ("g", "d")


def _host_staged(t, group=None):
    """True when the group's backend cannot move tensors of t's device: gloo
    with device tensors (a rehearsal of the N-rank path on one GPU, or CPU
    tests).  RCCL ("nccl") moves device tensors directly."""
    return t.device.type != "cpu" and dist.get_backend(group) == "gloo"


def _all_gather(out, t, group=None):
    """dist.all_gather into `out` (a list of tensors shaped like t); over gloo
    device tensors are staged through host memory."""
    if not _host_staged(t, group):
        dist.all_gather(out, t, group=group)
        return
    tc = t.cpu()
    oc = [torch.empty_like(tc) for _ in out]
    dist.all_gather(oc, tc, group=group)
    for o, c in zip(out, oc):
        o.copy_(c)


def _all_to_all_single(out, inp, out_splits=None, in_splits=None, group=None):
    if not _host_staged(inp, group):
        dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits, group=group)
        return
    oc = torch.empty(out.shape, dtype=out.dtype)
    dist.all_to_all_single(oc, inp.cpu(), output_split_sizes=out_splits, input_split_sizes=in_splits, group=group)
    out.copy_(oc)


def _all_reduce(t, op, group=None):
    if not _host_staged(t, group):
        dist.all_reduce(t, op=op, group=group)
        return
    c = t.cpu()
    dist.all_reduce(c, op=op, group=group)
    t.copy_(c)


def stream_range(S, world, rank):
    """Contiguous, balanced stream range [a, b) of `rank` out of `world`."""
    q, r = divmod(S, world)
    a = rank * q + min(rank, r)
    return a, a + q + (1 if rank < r else 0)


def balanced_assignment(lengths, world):
    """Longest-first greedy assignment of streams to ranks by total length
    (skewed / Zipf stream lengths).  Returns a list of index tensors."""
    lengths = torch.as_tensor(lengths, dtype=torch.int64).cpu()
    order = torch.argsort(lengths, descending=True).tolist()
    load = [0] * world
    parts = [[] for _ in range(world)]
    for s in order:
        k = min(range(world), key=lambda i: load[i])
        parts[k].append(s)
        load[k] += int(lengths[s])
    return [torch.tensor(sorted(p), dtype=torch.int64) for p in parts]


def pack_state(state):
    """State dict (StreamSet.export_state) -> three flat tensors + lengths."""
    lens = [int(state[k].numel()) for k in _F64 + _I64 + _I32]
    f = torch.cat([state[k].reshape(-1).to(torch.float64) for k in _F64])
    i = torch.cat([state[k].reshape(-1).to(torch.int64) for k in _I64])
    j = torch.cat([state[k].reshape(-1).to(torch.int32) for k in _I32])
    return f, i, j, lens


def unpack_state(f, i, j, lens, eps):
    names = _F64 + _I64 + _I32
    out = {"eps": eps}
    o = {"f": 0, "i": 0, "j": 0}
    for name, n in zip(names, lens):
        src, key = (f, "f") if name in _F64 else ((i, "i") if name in _I64 else (j, "j"))
        out[name] = src[o[key]:o[key] + n]
        o[key] += n
    return out


def all_gather_varlen(t, group=None):
    """all_gather of 1-D tensors whose length differs by rank (sizes first,
    then payloads padded to the longest)."""
    world = dist.get_world_size(group)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    _all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes) if sizes else 0
    pad = torch.zeros(m, dtype=t.dtype, device=t.device)
    pad[:t.numel()] = t
    bufs = [torch.empty(m, dtype=t.dtype, device=t.device) for _ in range(world)]
    _all_gather(bufs, pad, group=group)
    return [b[:s] for b, s in zip(bufs, sizes)]


def allgather_states(state, group=None):
    """Every rank's state (list indexed by rank), on this rank's device."""
    f, i, j, lens = pack_state(state)
    fs = all_gather_varlen(f, group)
    is_ = all_gather_varlen(i, group)
    js = all_gather_varlen(j, group)
    lt = all_gather_varlen(torch.tensor(lens, dtype=torch.int64, device=f.device), group)
    return [unpack_state(a, b, c, [int(x) for x in l.tolist()], state["eps"])
            for a, b, c, l in zip(fs, is_, js, lt)]


def alltoall_states(state, group=None):
    """Row-shard exchange by all-to-all: this rank's state is cut into the
    ``stream_range`` of every rank and part r goes to rank r only.  Returns
    the list (indexed by source rank) of the states of THIS rank's stream
    range.  One all-to-all of counts (fixed size), then one variable-size
    ``all_to_all_single`` per payload dtype."""
    world = dist.get_world_size(group)
    S = int(state["n"].numel())
    dev = state["n"].device
    parts = [pack_state(slice_state(state, *stream_range(S, world, r))) for r in range(world)]
    nlen = len(_F64 + _I64 + _I32)
    # per destination: payload lengths (f, i, j) and the component lengths
    meta = torch.tensor([[p[0].numel(), p[1].numel(), p[2].numel()] + p[3] for p in parts],
                        dtype=torch.int64, device=dev)
    flat_in = meta.reshape(-1).contiguous()
    flat_out = torch.empty_like(flat_in)
    _all_to_all_single(flat_out, flat_in, group=group)
    rmeta = flat_out.reshape(world, 3 + nlen).cpu()
    out = []
    for k in range(3):
        src = torch.cat([p[k] for p in parts])
        recv = torch.empty(int(rmeta[:, k].sum()), dtype=src.dtype, device=dev)
        _all_to_all_single(recv, src, rmeta[:, k].tolist(), [int(p[k].numel()) for p in parts], group=group)
        out.append(list(torch.split(recv, rmeta[:, k].tolist())))
    return [unpack_state(out[0][r], out[1][r], out[2][r], [int(x) for x in rmeta[r, 3:].tolist()], state["eps"])
            for r in range(world)]


def slice_state(state, a, b):
    """The state of streams [a, b) of a CSR state dict."""
    offs, poffs = state["offs"], state["poffs"]
    t0, t1 = int(offs[a]), int(offs[b])
    p0, p1 = int(poffs[a]), int(poffs[b])
    return {"eps": state["eps"],
            "offs": offs[a:b + 1] - offs[a], "v": state["v"][t0:t1], "g": state["g"][t0:t1],
            "d": state["d"][t0:t1], "poffs": poffs[a:b + 1] - poffs[a], "pv": state["pv"][p0:p1],
            "n": state["n"][a:b], "min": state["min"][a:b], "max": state["max"][a:b],
            "sum": state["sum"][a:b], "avg": state["avg"][a:b]}


def concat_states(states):
    """Streams of several states, in order, as one state."""
    out = {"eps": states[0]["eps"]}
    for k in ("v", "g", "d", "pv", "n", "min", "max", "sum", "avg"):
        out[k] = torch.cat([s[k] for s in states])
    for k in ("offs", "poffs"):
        parts, base = [], 0
        for s in states:
            parts.append(s[k][:-1] + base)
            base += int(s[k][-1])
        parts.append(torch.tensor([base], dtype=torch.int64, device=states[0][k].device))
        out[k] = torch.cat(parts)
    return out


def fold_states(states, device=None):
    """Left fold states[0].merge(states[1])...merge(states[-1]) on the GPU,
    stream by stream (gk:111-154).  Returns the resulting StreamSet."""
    from .streamset import StreamSet
    S = int(states[0]["n"].numel())
    eps = states[0]["eps"]
    acc = StreamSet(S, eps, device=device)
    acc.import_state(states[0])
    others = []
    for st in states[1:]:
        o = StreamSet(S, eps, device=device)
        o.import_state(st)
        others.append(o)
    if others:
        acc.merge_from(others)
    return acc


def merge_row_shards(ss, group=None, exchange="allgather"):
    """Row-sharded sketches -> merged sketches of this rank's stream range.

    `ss` is this rank's StreamSet over all S streams (built from its slice of
    the rows).  Returns (StreamSet over streams [a, b), (a, b)); the fold is in
    rank order, identical to the reference's sk0.merge(sk1)...merge(skN-1).
    `exchange`: "allgather" (north star) or "alltoall" (each table crosses once).
    One-off form (state dicts, fresh fold sets); repeated exchanges should
    keep a ``RowShardMerger``, which allocates once and syncs the host once.
    """
    if exchange not in ("alltoall", "allgather"):
        raise ValueError("exchange must be 'alltoall' or 'allgather'")
    if not (dist.is_available() and dist.is_initialized()):
        states, world, rank = [ss.export_state()], 1, 0
        a, b = stream_range(ss.num_streams, world, rank)
        mine = [slice_state(st, a, b) for st in states]
    else:
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        a, b = stream_range(ss.num_streams, world, rank)
        if exchange == "alltoall":
            mine = alltoall_states(ss.export_state(), group)
        else:
            mine = [slice_state(st, a, b) for st in allgather_states(ss.export_state(), group)]
    return fold_states(mine, device=ss.device), (a, b)


class RowShardMerger:
    """Row-shard exchange + rank-ordered fold, built once and reused every step.

    ``merger(ss)``: ``ss`` is this rank's StreamSet over all S streams (its
    slice of the rows); returns the StreamSet of this rank's stream range
    [a, b) holding ``sk_0.merge(sk_1)...merge(sk_{N-1})`` (gk:111-154) of every
    stream in it.  Per call:

    * ONE host synchronisation: each rank's record totals (table entries,
      pending values) are all-gathered on the device and read back together;
    * tables are exported on the device straight into buffers padded to the
      largest rank's totals (the caching allocator reuses them), packed into
      three flat payloads (f64 / i64 / i32) and all-gathered over RCCL with no
      further size exchange ("allgather", the north star's exchange); with
      ``exchange="alltoall"`` every rank receives only its own stream range of
      each peer (one extra all-gather of range-boundary offsets, same sync);
    * the N fold sets were allocated at construction: each is filled by
      ``gk_import`` with offsets that point into the received payload as it is
      (no slicing on the host), then folded by ``gk_merge`` in rank order.
    """

    def __init__(self, num_streams, eps, device, group=None, exchange="allgather"):
        from .streamset import StreamSet
        if exchange not in ("alltoall", "allgather"):
            raise ValueError("exchange must be 'alltoall' or 'allgather'")
        self.S = int(num_streams)
        self.eps = eps
        self.device = torch.device(device)
        self.group = group
        self.exchange = exchange
        on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        self.range = stream_range(self.S, self.world, self.rank)
        self.bounds = torch.tensor([stream_range(self.S, self.world, r)[0] for r in range(self.world)] + [self.S],
                                   dtype=torch.int64, device=self.device)
        n = self.range[1] - self.range[0]
        self.sets = [StreamSet(n, eps, device=self.device) for _ in range(self.world)]

    def _gather(self, t):
        if self.world == 1:
            return [t]
        out = [torch.empty_like(t) for _ in range(self.world)]
        _all_gather(out, t, group=self.group)
        return out

    def __call__(self, ss):
        S, world, dev = self.S, self.world, self.device
        a, b = self.range
        e, p = ss.export_sizes()
        offs = torch.zeros(S + 1, dtype=torch.int64, device=dev)
        poffs = torch.zeros(S + 1, dtype=torch.int64, device=dev)
        torch.cumsum(e.to(torch.int64), 0, out=offs[1:])
        torch.cumsum(p.to(torch.int64), 0, out=poffs[1:])
        # record offsets at every rank's range boundary (alltoall splits) -- the
        # totals are the last ones; one all-gather, one readback
        eb, pb = offs[self.bounds], poffs[self.bounds]
        meta = torch.stack(self._gather(torch.cat([eb, pb])))  # [world, 2 (world+1)]
        meta_h = meta.cpu()  # the one host synchronisation of the exchange
        W1 = world + 1
        if self.exchange == "allgather":
            Emax = int(meta_h[:, W1 - 1].max())
            Pmax = int(meta_h[:, 2 * W1 - 1].max())
        else:
            Emax = Pmax = 0
        E_loc, P_loc = int(meta_h[self.rank, W1 - 1]), int(meta_h[self.rank, 2 * W1 - 1])
        v = torch.empty(max(E_loc, Emax, 1), dtype=torch.float64, device=dev)
        gd = torch.empty(2 * max(E_loc, Emax, 1), dtype=torch.int32, device=dev)
        pv = torch.empty(max(P_loc, Pmax, 1), dtype=torch.float64, device=dev)
        nE = v.numel()
        ss.export_into(offs, v, gd[:nE], gd[nE:], poffs, pv)
        st = ss.stats()
        hdr_f = torch.cat([st["min"], st["max"], st["sum"], st["avg"]])
        hdr_i = torch.cat([offs, poffs, st["n"]])
        if self.exchange == "allgather":
            fs = self._gather(torch.cat([v, pv, hdr_f]))
            is_ = self._gather(hdr_i)
            js = self._gather(gd)
            nP = pv.numel()
            views = []
            for k in range(world):
                f, i, j = fs[k], is_[k], js[k]
                views.append(dict(v=f[:nE], pv=f[nE:nE + nP], hf=f[nE + nP:].view(4, S),
                                  offs=i[:S + 1], poffs=i[S + 1:2 * S + 2], n=i[2 * S + 2:],
                                  g=j[:nE], d=j[nE:], lo=a, hi=b))
        else:
            views = self._alltoall(meta_h, v[:E_loc], gd[:nE][:E_loc], gd[nE:][:E_loc], pv[:P_loc], hdr_f,
                                   offs, poffs, st["n"])
        for k, w in enumerate(views):
            lo, hi = w["lo"], w["hi"]
            self.sets[k].import_arrays(w["offs"][lo:hi + 1], w["v"], w["g"], w["d"], w["poffs"][lo:hi + 1],
                                       w["pv"], w["n"][lo:hi], w["hf"][0, lo:hi], w["hf"][1, lo:hi],
                                       w["hf"][2, lo:hi], w["hf"][3, lo:hi])
        if world > 1:
            self.sets[0].merge_from(self.sets[1:])
        return self.sets[0]

    def _alltoall(self, meta_h, v, g, d, pv, hdr_f, offs, poffs, n):
        """Each peer receives exactly its stream range of this rank's state."""
        S, world, dev, W1 = self.S, self.world, self.device, self.world + 1
        bnd = [int(x) for x in self.bounds.tolist()]  # static (construction-time) boundaries

        def splits(row, base):  # per destination: records of its range in source `row`
            return [int(meta_h[row, base + r + 1] - meta_h[row, base + r]) for r in range(world)]
        e_in, p_in = splits(self.rank, 0), splits(self.rank, W1)
        e_out = [splits(k, 0)[self.rank] for k in range(world)]
        p_out = [splits(k, W1)[self.rank] for k in range(world)]
        hf = hdr_f.view(4, S)
        n_rng = [bnd[r + 1] - bnd[r] for r in range(world)]
        a, b = self.range
        # per destination r: its range's offsets rebased to the records sent to it
        offs_parts = [offs[bnd[r]:bnd[r + 1] + 1] - offs[bnd[r]] for r in range(world)]
        poffs_parts = [poffs[bnd[r]:bnd[r + 1] + 1] - poffs[bnd[r]] for r in range(world)]
        i_send = torch.cat([torch.cat([o, po, n[bnd[r]:bnd[r + 1]]]) for r, (o, po) in
                            enumerate(zip(offs_parts, poffs_parts))])
        # f payload per destination: its tables' values, its pending values, its 4 header rows
        v_parts = list(torch.split(v, e_in))
        pv_parts = list(torch.split(pv, p_in))
        f_send = torch.cat([torch.cat([v_parts[r], pv_parts[r], hf[:, bnd[r]:bnd[r + 1]].reshape(-1)])
                            for r in range(world)])
        f_in_sizes = [e_in[r] + p_in[r] + 4 * n_rng[r] for r in range(world)]
        f_out_sizes = [e_out[k] + p_out[k] + 4 * (b - a) for k in range(world)]
        j_send = torch.cat([torch.cat([gp, dp]) for gp, dp in zip(torch.split(g, e_in), torch.split(d, e_in))])
        j_in_sizes = [2 * e_in[r] for r in range(world)]
        j_out_sizes = [2 * e_out[k] for k in range(world)]
        i_in_sizes = [2 * (n_rng[r] + 1) + n_rng[r] for r in range(world)]
        i_out_sizes = [2 * (b - a + 1) + (b - a) for _ in range(world)]
        f_recv = torch.empty(sum(f_out_sizes), dtype=torch.float64, device=dev)
        i_recv = torch.empty(sum(i_out_sizes), dtype=torch.int64, device=dev)
        j_recv = torch.empty(max(sum(j_out_sizes), 1), dtype=torch.int32, device=dev)
        _all_to_all_single(f_recv, f_send, f_out_sizes, f_in_sizes, group=self.group)
        _all_to_all_single(i_recv, i_send, i_out_sizes, i_in_sizes, group=self.group)
        _all_to_all_single(j_recv[:sum(j_out_sizes)], j_send, j_out_sizes, j_in_sizes, group=self.group)
        views = []
        fo = io = jo = 0
        m = b - a
        for k in range(world):
            f = f_recv[fo:fo + f_out_sizes[k]]
            i = i_recv[io:io + i_out_sizes[k]]
            j = j_recv[jo:jo + j_out_sizes[k]]
            fo, io, jo = fo + f_out_sizes[k], io + i_out_sizes[k], jo + j_out_sizes[k]
            ek, pk = e_out[k], p_out[k]
            views.append(dict(v=f[:ek] if ek else f[:1], pv=f[ek:ek + pk] if pk else f[:1],
                              hf=f[ek + pk:].view(4, m), offs=i[:m + 1], poffs=i[m + 1:2 * m + 2],
                              n=i[2 * m + 2:], g=j[:ek] if ek else torch.zeros(1, dtype=torch.int32, device=dev),
                              d=j[ek:2 * ek] if ek else torch.zeros(1, dtype=torch.int32, device=dev), lo=0, hi=m))
        return views


def allgather_packed(ss, group=None):
    """Every rank's packed state (StreamSet.pack), in rank order: the sizes
    agree by one all-reduce (max), each rank packs into a zero-padded buffer
    of that size, one all-gather moves them."""
    dev = ss.device
    n = torch.tensor([ss.pack_bytes()], dtype=torch.int64, device=dev)
    _all_reduce(n, dist.ReduceOp.MAX, group=group)
    buf = torch.zeros(int(n.item()), dtype=torch.uint8, device=dev)
    ss.pack(buf)
    out = [torch.empty_like(buf) for _ in range(dist.get_world_size(group))]
    _all_gather(out, buf, group=group)
    return out


def fold_packed_allgather(ss, dst, group=None):
    """dst := rank 0's state, then dst.merge(rank r's state) for r = 1 ..
    N-1 (gk:111-154) -- every rank gets the whole fold (row shards of the same
    streams)."""
    dst.fold_packed(allgather_packed(ss, group))
    return dst
