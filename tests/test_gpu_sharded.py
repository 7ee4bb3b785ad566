"""GPU parity of the train-sharded mode (north_star mode b) on the reference's
kind of data, and the group's collective paths on a one-GPU box.

* Reference tie order across shards: the reference sorts all N_train records
  of a query with std::sort (cpp:323/366), so among EXACTLY equal distances
  its order -- and, where it decides the vote, its label -- depends on every
  shard's rows.  The merge flags those queries (KNN_FLAG_TIE_PENDING), every
  shard computes their exact distances (knn_shard_distances_device), the
  owner re-sorts them as the reference does (knn_tie_resolve_device).
  Checked through knn_group mode 1 (which does the exchange itself) and
  through the ABI building blocks the torch ranks use (3-shard
  search_partial + merge_vote + shard distances + resolve).
* Collectives on one GPU: KNN_GROUP_RCCL runs every RCCL call of the path
  (ncclCommInitAll, ncclBroadcast, ncclAllGather, ncclAllReduce) through a
  one-rank communicator; repeated devices run the whole G-rank decomposition
  (ragged shards, packed all-gather offsets, G-way merges, the tie exchange)
  over loopback copies.  Only the xGMI transport itself is left to a
  multi-GPU node.
"""
import numpy as np
import pytest

import oracle
from test_gpu_parity import TIE_VOTES, _mix, assert_neighbors_match

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def knn():
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location(
        "knn_amd", os.path.join(root, "-mpi-knn-_amd", "knn_amd.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    if mod.lib().knn_device_count() < 1:
        pytest.fail("no HIP device visible: the KNN path has no CPU fallback")
    return mod


def _tie_set(metric, n=5000, m=300, d=6, seed=171):
    """Integer codes 0..9 in 6 dims with labels independent of position:
    nearly every query has exactly equal distances with different labels in
    its top k (the oracle finds 299 of 300 at k = 10), and a tie across the
    k-th place in most -- the label then depends on the reference's
    std::sort order."""
    rng = np.random.default_rng(seed + metric)
    X = rng.integers(0, 10, (n + m, d)).astype(np.float64)
    lab = rng.integers(0, 5, n + m).astype(np.int32)
    return X[:n].copy(), lab[:n].copy(), X[n:].copy()


def _count(knn, got, want, flags):
    """Tie votes into the suite's TIE_VOTES record; returns (tie votes, differing)."""
    tv = (flags & knn.FLAG_TIE_VOTE) != 0
    differs = int((got[tv] != want[tv]).sum())
    TIE_VOTES["tie_vote"] += int(tv.sum())
    TIE_VOTES["tie_vote_label_differs"] += differs
    TIE_VOTES["queries"] += int(len(got))
    TIE_VOTES["cases"] += 1
    TIE_VOTES["sharded_tie_vote"] = TIE_VOTES.get("sharded_tie_vote", 0) + int(tv.sum())
    return int(tv.sum()), differs


GROUPS = [  # (devices, rccl): transport none / one-rank RCCL / 3 and 2 ranks over loopback
    ([0], False), ([0], True), ([0, 0, 0], False), ([0, 0], False)]


@pytest.mark.parametrize("devs,rccl", GROUPS)
@pytest.mark.parametrize("metric", [0, 1])
def test_group_train_sharded_reference_tie_order(knn, devs, rccl, metric):
    """knn_group mode 1 on integer data full of exact ties: labels equal the
    reference's for every query (tie votes > 50, none differing); the
    queries re-ordered by the exchange carry KNN_FLAG_TIE_REF and the
    reference's neighbour order index for index; with "ties" = 2 every tied
    query is re-ordered and all indices equal the oracle's."""
    tr, lab, te = _tie_set(metric)
    g = knn.Group(devs, 1, rccl=rccl)
    g.set_train(tr, lab, 5)
    tie_votes = 0
    for k in (10, 37):
        want, widx, wdist = oracle.knn(tr, lab, te, k, metric == 0, 5, n_out=k)
        got, idx, dist, flags = g.classify(te, k, metric, return_neighbors=True)
        tv, differs = _count(knn, got, want, flags)
        tie_votes += tv
        assert differs == 0, "%d exact-tie votes differ from the reference order" % differs
        np.testing.assert_array_equal(got, want)
        assert not (flags & knn.FLAG_TIE_PENDING).any()
        ref = (flags & knn.FLAG_TIE_REF) != 0
        assert ref.sum() == g.last_tie_count()
        np.testing.assert_array_equal(idx[ref], widx[ref])
        assert_neighbors_match(idx, dist, widx, wdist, flags)
    assert tie_votes > 50, "expected many exact-tie votes"
    # without the exchange ("ties" = 0: index order inside ties) some labels
    # differ from the reference's -- the set exercises label-deciding ties
    want, _, _ = oracle.knn(tr, lab, te, 10, metric == 0, 5)
    g.set_tuning("ties", 0)
    got0 = g.classify(te, 10, metric)
    assert (got0 != want).sum() > 0
    g.set_tuning("ties", 2)
    want, widx, wdist = oracle.knn(tr, lab, te, 10, metric == 0, 5, n_out=10)
    got, idx, dist, flags = g.classify(te, 10, metric, return_neighbors=True)
    tied = (flags & 14) != 0
    assert tied.sum() > 50 and ((flags & knn.FLAG_TIE_REF) != 0).sum() == tied.sum()
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(idx, widx)
    assert (dist.view(np.int64) == wdist.view(np.int64)).all()
    g.close()


def _sharded_blocks(knn, tr, lab, Q, shards, w, metric, dev):
    """Per shard a context on device 0 with its rows (global offsets) and its
    exact top-w lists [parts][m][w]."""
    import torch
    m = Q.shape[0]
    parts = len(shards)
    gd = torch.empty((parts, m, w), dtype=torch.float64, device=dev)
    gi = torch.empty((parts, m, w), dtype=torch.int64, device=dev)
    gl = torch.empty((parts, m, w), dtype=torch.int32, device=dev)
    ctxs = []
    for p, (r0, r1) in enumerate(shards):
        c = knn.Classifier(0)
        Xs = torch.from_numpy(tr[r0:r1].copy()).to(dev)
        Ls = torch.from_numpy(lab[r0:r1].copy()).to(dev)
        c.set_train_device(Xs.data_ptr(), Ls.data_ptr(), r1 - r0, tr.shape[1], 5, idx_offset=r0,
                           keep=(Xs, Ls))
        c.search_partial_device(Q.data_ptr(), m, w, metric, gd[p].data_ptr(), gi[p].data_ptr(),
                                gl[p].data_ptr())
        c.sync()
        ctxs.append(c)
    return ctxs, gd, gi, gl


def _resolve_pending(knn, ctxs, shards, Q, lab_all, k, metric, out, dev, q0=0):
    """The exchange of knn_dist.resolve_ties on one GPU: the flagged rows of
    the merged slice [q0, ...), every shard's distance block, the owner's
    resolve.  Returns the number of queries resolved."""
    import torch
    ol, oi, od, of = out
    pend = torch.nonzero(of & knn.FLAG_TIE_PENDING).flatten().to(torch.int32)
    T = pend.numel()
    if T == 0:
        return 0
    sel = (pend + q0).to(torch.int32)
    rows = [r1 - r0 for r0, r1 in shards]
    blocks = []
    for c, nr in zip(ctxs, rows):
        D = torch.empty((T, nr), dtype=torch.float64, device=dev)
        c.shard_distances_device(Q.data_ptr(), sel.data_ptr(), T, metric, D.data_ptr())
        c.sync()
        blocks.append(D.reshape(-1))
    Dall = torch.cat(blocks)
    ctxs[0].tie_resolve_device(Dall.data_ptr(), rows, T, lab_all.data_ptr(), pend.data_ptr(), k,
                               ol.data_ptr(), oi.data_ptr(), od.data_ptr(), of.data_ptr())
    ctxs[0].sync()
    return T


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("ties", [1, 2])
def test_partial_merge_reference_tie_order(knn, metric, ties):
    """The ABI building blocks of the torch ranks' mode b (knn_dist.py) on
    3 ragged shards: merge_vote flags the queries whose label (ties = 1) or
    neighbour order (ties = 2) the reference's tie order decides; shard
    distances + tie_resolve give the oracle's labels for every query (and
    its indices for every query at ties = 2), also for a query slice."""
    import torch
    dev = torch.device("cuda", 0)
    tr, lab, te = _tie_set(metric, n=4001, m=250)
    n, m, k = tr.shape[0], te.shape[0], 10
    w = k + 1
    shards = [(0, 1300), (1300, 2701), (2701, n)]
    Q = torch.from_numpy(te).to(dev)
    lab_all = torch.from_numpy(lab).to(dev)
    ctxs, gd, gi, gl = _sharded_blocks(knn, tr, lab, Q, shards, w, metric, dev)
    want, widx, wdist = oracle.knn(tr, lab, te, k, metric == 0, 5, n_out=k)
    ctxs[0].set_tuning("ties", ties)
    total = 0
    for q0, q1 in ((0, m), (0, 101), (101, m)):
        mq = q1 - q0
        out = (torch.empty(mq, dtype=torch.int32, device=dev),
               torch.empty((mq, k), dtype=torch.int64, device=dev),
               torch.empty((mq, k), dtype=torch.float64, device=dev),
               torch.empty(mq, dtype=torch.int32, device=dev))
        ctxs[0].merge_vote_device(gd.data_ptr(), gi.data_ptr(), gl.data_ptr(), 3, m, w, k,
                                  out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                                  out[3].data_ptr(), q0=q0, mq=mq)
        ctxs[0].sync()
        flags0 = out[3].cpu().numpy()
        if ties == 2:
            assert ((flags0 & knn.FLAG_TIE_PENDING) != 0).sum() == ((flags0 & 14) != 0).sum()
        total += _resolve_pending(knn, ctxs, shards, Q, lab_all, k, metric, out, dev, q0)
        got, idx, dist, flags = (t.cpu().numpy() for t in out)
        tv, differs = _count(knn, got, want[q0:q1], flags)
        assert differs == 0
        np.testing.assert_array_equal(got, want[q0:q1])
        assert not (flags & knn.FLAG_TIE_PENDING).any()
        ref = (flags & knn.FLAG_TIE_REF) != 0
        np.testing.assert_array_equal(idx[ref], widx[q0:q1][ref])
        if ties == 2:
            np.testing.assert_array_equal(idx, widx[q0:q1])
        assert_neighbors_match(idx, dist, widx[q0:q1], wdist[q0:q1], flags)
    assert total > 20
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("metric", [0, 1])
def test_hip_ties_default_stream(knn, metric):
    """knn_dist.resolve_ties through knn_dist.HipTies as bench.py's mode b
    drives it, here at world 1 and with HipTies' default stream (torch's
    current one: the flags, the distance blocks and the library calls on one
    stream): 3 shard contexts' lists merged in one context, every flagged
    query resolved, labels = the oracle's, none left pending."""
    import importlib.util
    import os
    import torch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location(
        "knn_dist", os.path.join(root, "-mpi-knn-_amd", "knn_dist.py"))
    kd = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(kd)
    dev = torch.device("cuda", 0)
    tr, lab, te = _tie_set(metric, n=4001, m=250)
    n, m, k = tr.shape[0], te.shape[0], 10
    w = k + 1
    shards = [(0, 1300), (1300, 2701), (2701, n)]
    Q = torch.from_numpy(te).to(dev)
    ctxs, gd, gi, gl = _sharded_blocks(knn, tr, lab, Q, shards, w, metric, dev)
    for c in ctxs[1:]:
        c.close()
    # one context over every row (world 1): its shard distances cover all rows
    c = ctxs[0]
    Xa = torch.from_numpy(tr).to(dev)
    La = torch.from_numpy(lab).to(dev)
    c.set_train_device(Xa.data_ptr(), La.data_ptr(), n, tr.shape[1], 5, keep=(Xa, La))
    outs = (torch.empty(m, dtype=torch.int32, device=dev),
            torch.empty((m, k), dtype=torch.int64, device=dev),
            torch.empty((m, k), dtype=torch.float64, device=dev),
            torch.empty(m, dtype=torch.int32, device=dev))
    stream = torch.cuda.current_stream(dev).cuda_stream
    c.merge_vote_device(gd.data_ptr(), gi.data_ptr(), gl.data_ptr(), 3, m, w, k,
                        outs[0].data_ptr(), outs[1].data_ptr(), outs[2].data_ptr(),
                        outs[3].data_ptr(), stream=stream)
    ties = kd.HipTies(c, Q, La, n, k, outs, m, metric=metric, device=dev)
    resolved = kd.resolve_ties(ties, m, dev)
    torch.cuda.synchronize()
    got, idx, dist, flags = (t.cpu().numpy() for t in outs)
    want, widx, wdist = oracle.knn(tr, lab, te, k, metric == 0, 5, n_out=k)
    assert resolved > 20 and ties.resolved == resolved
    assert not (flags & knn.FLAG_TIE_PENDING).any()
    np.testing.assert_array_equal(got, want)
    ref = (flags & knn.FLAG_TIE_REF) != 0
    np.testing.assert_array_equal(idx[ref], widx[ref])
    assert_neighbors_match(idx, dist, widx, wdist, flags)
    c.close()


@pytest.mark.parametrize("k", [7, 1500])
def test_merge_nonfinite_query(knn, k):
    """A query with a NaN / inf coordinate through both merge kernels (the LDS
    merge at 2 x 8 entries; the rank merge at 3 x 1501 entries, beyond the
    LDS image's 4096): label -1, KNN_FLAG_NONFINITE, idx -1, dist NaN -- the
    same sentinels as the single-context path; every other query exact."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    tr, lab, te = _mix(rng, 6000, 40, 16, 5)
    te[3, 2] = np.nan
    te[11, 0] = np.inf
    n, m = tr.shape[0], te.shape[0]
    parts = 3 if k > 1000 else 2
    shards = [(n * p // parts, n * (p + 1) // parts) for p in range(parts)]
    w = k + 1
    Q = torch.from_numpy(te).to(dev)
    ctxs, gd, gi, gl = _sharded_blocks(knn, tr, lab, Q, shards, w, 0, dev)
    ol = torch.empty(m, dtype=torch.int32, device=dev)
    oi = torch.empty((m, k), dtype=torch.int64, device=dev)
    od = torch.empty((m, k), dtype=torch.float64, device=dev)
    of = torch.empty(m, dtype=torch.int32, device=dev)
    ctxs[0].merge_vote_device(gd.data_ptr(), gi.data_ptr(), gl.data_ptr(), parts, m, w, k,
                              ol.data_ptr(), oi.data_ptr(), od.data_ptr(), of.data_ptr())
    ctxs[0].sync()
    _resolve_pending(knn, ctxs, shards, Q, torch.from_numpy(lab).to(dev), k, 0,
                     (ol, oi, od, of), dev)
    got, idx, dist, flags = ol.cpu().numpy(), oi.cpu().numpy(), od.cpu().numpy(), of.cpu().numpy()
    bad = np.array([3, 11])
    assert (got[bad] == -1).all() and (flags[bad] == knn.FLAG_NONFINITE).all()
    assert (idx[bad] == -1).all() and np.isnan(dist[bad]).all()
    ok = np.setdiff1d(np.arange(m), bad)
    want, widx, wdist = oracle.knn(tr, lab, te[ok], k, True, 5, n_out=k)
    np.testing.assert_array_equal(got[ok], want)
    assert_neighbors_match(idx[ok], dist[ok], widx, wdist, flags[ok])
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("order", [0, 3])
@pytest.mark.parametrize("devs,rccl", GROUPS)
def test_group_modes_transports(knn, devs, rccl, order):
    """Both group modes and the sharded normalisation on every transport a
    one-GPU box offers, ragged shards, against the oracle; with every shard's
    images in train order and in region order (3 regions per shard: list
    positions mapped back to shard rows, then to global rows)."""
    rng = np.random.default_rng(37)
    tr, lab, te = _mix(rng, 5001, 333, 48, 6, grid=None)
    va = te[::2].copy()
    t_n, e_n, v_n = tr.copy(), te.copy(), va.copy()
    oracle.normalize(t_n, e_n, v_n)
    g = knn.Group(devs, 0, rccl=rccl)
    assert g.transport() == (2 if len(devs) > 1 else 1 if rccl else 0)
    g.normalize(tr, te, va)
    for a, b in ((tr, t_n), (te, e_n), (va, v_n)):
        assert a.tobytes() == b.tobytes()
    want, widx, wdist = oracle.knn(tr, lab, te, 7, True, 6, n_out=7)
    g.set_tuning("order", order)
    g.set_train(tr, lab, 6)
    got, idx, dist, flags = g.classify(te, 7, knn.L2, return_neighbors=True)
    np.testing.assert_array_equal(got, want)
    assert_neighbors_match(idx, dist, widx, wdist, flags)
    g.close()
    g = knn.Group(devs, 1, rccl=rccl)
    g.set_tuning("order", order)
    g.set_train(tr, lab, 6)
    got, idx, dist, flags = g.classify(te, 7, knn.L2, return_neighbors=True)
    np.testing.assert_array_equal(got, want)
    assert_neighbors_match(idx, dist, widx, wdist, flags)
    # k beyond the LDS merge (G x (k+1) > 4096 entries): the rank merge
    k = 2100
    want2, widx2, wdist2 = oracle.knn(tr, lab, te[:20], k, True, 6, n_out=k)
    got2, idx2, dist2, flags2 = g.classify(te[:20], k, knn.L2, return_neighbors=True)
    np.testing.assert_array_equal(got2, want2)
    assert_neighbors_match(idx2, dist2, widx2, wdist2, flags2)
    g.close()
