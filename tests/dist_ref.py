"""Test-side reference for the train-sharded merge (numpy): per query, the
union of the per-shard sorted lists ordered by (dist, global idx), first k,
then the reference vote (first label whose running count strictly exceeds the
running max, cpp:324-337).  TEST INFRASTRUCTURE ONLY."""
import numpy as np


def vote(labels):
    cnt = {}
    best, best_lab = 0, -1
    for lab in labels:
        cnt[lab] = cnt.get(lab, 0) + 1
        if cnt[lab] > best:
            best, best_lab = cnt[lab], lab
    return best_lab


def merge_vote(gd, gi, gl, k, q0, q1, pending=None):
    """gd/gi/gl: [parts][m][w] arrays; returns labels, idx[k], dist[k] for q0..q1.
    pending (a list) receives the slice rows with any exact tie in the top k
    or across the k-th place (the merge's KNN_FLAG_TIE_PENDING at ties = 2)."""
    parts = gd.shape[0]
    labs, idxs, dists = [], [], []
    for q in range(q0, q1):
        ent = []
        for p in range(parts):
            for c in range(gd.shape[2]):
                if gi[p, q, c] >= 0:
                    ent.append((gd[p, q, c], gi[p, q, c], gl[p, q, c]))
        ent.sort(key=lambda e: (e[0], e[1]))
        top = ent[:k]
        labs.append(vote([e[2] for e in top]))
        idxs.append([e[1] for e in top])
        dists.append([e[0] for e in top])
        dv = [e[0] for e in ent[:k + 1]]
        if pending is not None and any(a == b for a, b in zip(dv, dv[1:])):
            pending.append(q - q0)
    return np.array(labs, np.int32), np.array(idxs, np.int64), np.array(dists, np.float64)


def sorted_partial(tr_shard, r0, lab_shard, Q, w, euclidean=True):
    """A shard's exact top-w per query ordered by (dist, global idx), from
    the oracle's reference-arithmetic distances (knn_search_partial's
    semantics): (dist[m][w], idx[m][w], label[m][w])."""
    import oracle
    m = Q.shape[0]
    dd = np.empty((m, w), np.float64)
    ii = np.empty((m, w), np.int64)
    for q in range(m):
        D = oracle.row_distances(Q[q], tr_shard, euclidean)
        o = np.lexsort((np.arange(D.shape[0]), D))[:w]
        dd[q], ii[q] = D[o], o + r0
    return dd, ii, lab_shard[ii - r0].astype(np.int32)


def minmax_fold(X, mx, mn, init):
    """Per-rank statistics of cpp:245-274 on a torch CPU shard (the caller
    starts mx/mn at -1/999999): strict compares, NaN never wins."""
    if X.shape[0] == 0:
        return
    a = X.numpy()
    colmax = np.where(np.isnan(a), -np.inf, a).max(0)
    colmin = np.where(np.isnan(a), np.inf, a).min(0)
    m, n = mx.numpy(), mn.numpy()
    np.copyto(m, np.where(colmax > m, colmax, m))
    np.copyto(n, np.where(colmin < n, colmin, n))


def minmax_apply(X, mx, mn):
    """cpp:279-305: (x - min)/(max - min) where max - min != 0."""
    a, m, n = X.numpy(), mx.numpy(), mn.numpy()
    r = m - n
    keep = r != 0
    a[:, keep] = (a[:, keep] - n[keep]) / r[keep]
