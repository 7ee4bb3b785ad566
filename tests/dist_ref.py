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


def merge_vote(gd, gi, gl, k, q0, q1):
    """gd/gi/gl: [parts][m][w] arrays; returns labels, idx[k], dist[k] for q0..q1."""
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
    return np.array(labs, np.int32), np.array(idxs, np.int64), np.array(dists, np.float64)


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
