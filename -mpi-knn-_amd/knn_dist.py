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


def train_sharded(search_partial, merge_vote, Q, m, w, k, device=None):
    """Mode b.  search_partial(Q) -> (dist f64[m,w], idx i64[m,w], lab i32[m,w])
    for this rank's train shard (global indices); merge_vote(d, i, l, parts,
    q0, q1) -> labels i32[q1-q0] for the query slice of the [parts][m][w]
    lists.  Returns this rank's label slice and its [q0, q1)."""
    world, rank = world_info()
    d, i, l = search_partial(Q)
    if world > 1:  # one all-gather of the packed partial lists -> [W][m][w] each
        gd, gi, gl = _all_gather_packed(d, i, l)
    else:
        gd, gi, gl = d[None], i[None], l[None]
    q0, q1 = shard_range(m, world, rank)
    return merge_vote(gd, gi, gl, world, q0, q1), (q0, q1)
