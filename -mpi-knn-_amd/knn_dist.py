"""Multi-process decomposition of the KNN classify path (one process per GPU).

Replaces the reference's MPI decomposition (knn_mpi.cpp cpp:136-138 batch
sizes, cpp:224-227 Bcast/Scatter, cpp:340/383 Gather) with torch.distributed
collectives (backend "nccl" = RCCL over xGMI on the GPU box; "gloo" in the
CPU tests).  The per-rank compute is passed in, so the same decomposition
drives the HIP library on GPUs and the CPU oracle in tests.

  query-sharded (north_star mode a): train rows broadcast from rank 0, each
    rank classifies its contiguous query shard; no data-path collective.
  train-sharded (mode b): each rank holds rows [n*r/W, n*(r+1)/W), returns
    its exact local top-w per query (global indices + labels); the lists are
    all-gathered ([W][m][w]) and rank r merges/votes queries
    [m*r/W, m*(r+1)/W).
"""
import time

import torch
import torch.distributed as dist


def shard_range(n, world, rank):
    """Contiguous, ragged-allowed shard [lo, hi) (the reference requires
    n % world == 0, cpp:127-129; here any n works)."""
    return n * rank // world, n * (rank + 1) // world


def world_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def broadcast_train(X, labels, src=0):
    """≙ MPI_Bcast(Data_train) + MPI_Bcast(Train_label), cpp:224-225."""
    world, _ = world_info()
    if world > 1:
        dist.broadcast(X, src)
        dist.broadcast(labels, src)


def timed(step, steps, warmup, sync, device=None):
    """W untimed steps, then exactly `steps` steps bracketed by barrier+sync;
    returns the MAX elapsed seconds over ranks (every rank gets it)."""
    world, _ = world_info()
    for _ in range(warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return float(el.item())


def gather_slices(local, total_rows, device=None):
    """Concatenate every rank's contiguous slice (≙ MPI_Gather, cpp:340/383);
    slices may be ragged.  Returns the full tensor on every rank."""
    world, rank = world_info()
    if world == 1:
        return local
    lo, hi = shard_range(total_rows, world, rank)
    assert local.shape[0] == hi - lo
    maxrows = total_rows - total_rows * (world - 1) // world  # largest shard
    pad = torch.zeros((maxrows,) + tuple(local.shape[1:]), dtype=local.dtype, device=device)
    pad[: hi - lo] = local
    out = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(out, pad)
    parts = []
    for r in range(world):
        a, b = shard_range(total_rows, world, r)
        parts.append(out[r][: b - a])
    return torch.cat(parts, 0)


def _all_gather_stack(t):
    world, _ = world_info()
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return torch.stack(out, 0)


def _all_gather_packed(d, i, l):
    """The three partial-list tensors of this rank as one byte buffer
    [dist | idx | label] and a single all-gather (one collective per step,
    like knn_group_classify's ncclAllGather); unpacked into [W][m][w] each."""
    parts = [t.contiguous().reshape(-1).view(torch.uint8) for t in (d, i, l)]
    sizes = [p.numel() for p in parts]
    packed = torch.cat(parts)
    out = _all_gather_stack(packed)
    res, o = [], 0
    for t, nb in zip((d, i, l), sizes):
        res.append(out[:, o:o + nb].contiguous().view(t.dtype).reshape((-1,) + tuple(t.shape)))
        o += nb
    return tuple(res)


def normalize_sharded(local_sets, minmax, apply, d, device=None):
    """Transductive min-max normalisation with the reference's decomposition
    (cpp:229-306): minmax(set, mx, mn, init) folds this rank's rows of each
    set into per-dim bounds (init: start from -1 / 999999, cpp:239-243), the
    bounds are all-reduced MAX / MIN (≙ MPI_Allreduce cpp:276-277), then
    apply(set, mx, mn) rewrites the local rows in place.  Returns (mx, mn)."""
    world, _ = world_info()
    mx = torch.full((d,), -1.0, dtype=torch.float64, device=device)
    mn = torch.full((d,), 999999.0, dtype=torch.float64, device=device)
    for i, s in enumerate(local_sets):
        minmax(s, mx, mn, i == 0)
    if world > 1:
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    for s in local_sets:
        apply(s, mx, mn)
    return mx, mn


def train_sharded(search_partial, merge_vote, Q, m, w, k, device=None, ties=None):
    """Mode b.  search_partial(Q) -> (dist f64[m,w], idx i64[m,w], lab i32[m,w])
    for this rank's train shard (global indices); merge_vote(d, i, l, parts,
    q0, q1) -> labels i32[q1-q0] for the query slice of the [parts][m][w]
    lists.  ties (optional, see resolve_ties) restores the reference's order
    among equal distances across shards for the queries the merge flagged.
    Returns this rank's label slice and its [q0, q1)."""
    world, rank = world_info()
    d, i, l = search_partial(Q)
    if world > 1:  # one all-gather of the packed partial lists -> [W][m][w] each
        gd, gi, gl = _all_gather_packed(d, i, l)
    else:
        gd, gi, gl = d[None], i[None], l[None]
    q0, q1 = shard_range(m, world, rank)
    out = merge_vote(gd, gi, gl, world, q0, q1)
    if ties is not None:
        resolve_ties(ties, m, device)
    return out, (q0, q1)


def resolve_ties(ties, m, device=None, budget_bytes=1 << 30):
    """The reference sorts all N_train records of a query with std::sort
    (cpp:366): among EXACTLY equal distances its order depends on every
    row, so a merged query whose label that order decides (the merge's
    KNN_FLAG_TIE_PENDING) needs every shard's exact distances.  `ties`:
      pending()           -> int64[T_r] this rank's flagged rows of its slice
      shard_distances(s)  -> f64[len(s), n_rank] exact distances of this
                             rank's rows to the global query rows s (int32)
      resolve(D, rows, o) -> rewrite slice rows o (int32) from D = the
                             blocks [T][rows[g]] of every rank in row order
      n_total             -> train rows over all ranks
    Per batch: all-gather of the flagged ids, each rank's distances, one
    all-to-all (≙ the owner receiving every shard's block), resolve on the
    owner.  Returns the number of queries resolved over all ranks."""
    world, rank = world_info()
    n = ties.n_total
    rows = [shard_range(n, world, r)[1] - shard_range(n, world, r)[0] for r in range(world)]
    pend = ties.pending().to(torch.int64)
    q0 = shard_range(m, world, rank)[0]
    cnt = torch.tensor([pend.numel()], dtype=torch.int64, device=device)
    if world > 1:
        counts = [int(c.item()) for c in _all_gather_stack(cnt)]
    else:
        counts = [int(cnt.item())]
    total = sum(counts)
    if total == 0:
        return 0
    if hasattr(ties, "prepare"):  # collective set-up every rank runs (e.g. the global labels)
        ties.prepare()
    pad = torch.full((max(counts),), -1, dtype=torch.int64, device=device)
    pad[:pend.numel()] = pend + q0
    ids = _all_gather_stack(pad) if world > 1 else pad[None]
    owned = [ids[r, :counts[r]] for r in range(world)]  # global query rows, owner order
    B = max(1, min(4096, budget_bytes // (8 * n)))
    pos = [0] * world
    while True:
        take, left = [], B
        for r in range(world):
            t = min(left, counts[r] - pos[r])
            take.append(t)
            left -= t
        if sum(take) == 0:
            break
        sel = torch.cat([owned[r][pos[r]:pos[r] + take[r]] for r in range(world)]).to(torch.int32)
        mine = owned[rank][pos[rank]:pos[rank] + take[rank]]
        for r in range(world):
            pos[r] += take[r]
        D = ties.shard_distances(sel).reshape(-1)
        if world > 1:
            recv = torch.empty(take[rank] * n, dtype=torch.float64, device=device)
            dist.all_to_all_single(recv, D, [take[rank] * rows[g] for g in range(world)],
                                   [take[r] * rows[rank] for r in range(world)])
        else:
            recv = D
        if take[rank]:
            ties.resolve(recv, rows, (mine - q0).to(torch.int32))
    return total


class HipTies:
    """The `ties` of resolve_ties on the HIP library (knn_amd.Classifier of
    this rank's shard): the merge's KNN_FLAG_TIE_PENDING rows of the slice
    outputs, knn_shard_distances_device, knn_tie_resolve_device into the same
    outputs.  Every train label is all-gathered the first time any rank has
    a flagged query (4 B per row).  stream: the HIP stream of the library
    calls; default torch's current stream on `device`, the stream the torch
    tensors (D, the flags read by pending(), the all-to-all) are ordered on."""
    FLAG_TIE_PENDING = 64

    def __init__(self, ctx, Q, lab_shard, n_total, k, outs, mq, metric=0, stream=None,
                 device=None):
        if stream is None:
            stream = torch.cuda.current_stream(device).cuda_stream
        self.ctx, self.Q, self.lab_shard, self.n_total, self.k = ctx, Q, lab_shard, n_total, k
        self.o_lab, self.o_idx, self.o_dist, self.o_flags = outs
        self.mq, self.metric, self.stream, self.device = mq, metric, stream, device
        self.lab_all = None
        self.resolved = 0

    def pending(self):
        return torch.nonzero(self.o_flags[:self.mq] & self.FLAG_TIE_PENDING).flatten()

    def prepare(self):
        if self.lab_all is None:
            self.lab_all = gather_slices(self.lab_shard, self.n_total, self.device).contiguous()

    def shard_distances(self, sel):
        sel = sel.contiguous()
        D = torch.empty((sel.numel(), self.lab_shard.shape[0]), dtype=torch.float64,
                        device=self.device)
        self.ctx.shard_distances_device(self.Q.data_ptr(), sel.data_ptr(), sel.numel(),
                                        self.metric, D.data_ptr(), self.stream)
        return D

    def resolve(self, D, rows, orow):
        orow = orow.contiguous()
        self.ctx.tie_resolve_device(D.data_ptr(), rows, orow.numel(), self.lab_all.data_ptr(),
                                    orow.data_ptr(), self.k, self.o_lab.data_ptr(),
                                    None if self.o_idx is None else self.o_idx.data_ptr(),
                                    None if self.o_dist is None else self.o_dist.data_ptr(),
                                    self.o_flags.data_ptr(), self.stream)
        self.resolved += orow.numel()
