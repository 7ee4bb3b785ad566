"""ctypes wrapper of oracle/liboracle.so (CPU restatement of the reference).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        i64, i32, f64 = ctypes.c_int64, ctypes.c_int, ctypes.c_double
        L.oracle_normalize.argtypes = [P, i64, P, i64, P, i64, i32]
        L.oracle_normalize.restype = None
        L.oracle_minmax.argtypes = [P, i64, i32, P, P, i32]
        L.oracle_minmax.restype = None
        L.oracle_knn.argtypes = [P, P, i64, i32, P, i64, i32, i32, i32, P, P, P, i32, i32]
        L.oracle_knn.restype = i32
        L.oracle_distance.argtypes = [P, P, i32, i32]
        L.oracle_distance.restype = f64
        L.oracle_acc.argtypes = [P, P, i64]
        L.oracle_acc.restype = f64
        L.oracle_read_csv.argtypes = [ctypes.c_char_p, i32, i32, i64, P, P]
        L.oracle_read_csv.restype = i64
        L.oracle_row_distances.argtypes = [P, P, i64, i32, i32, P]
        L.oracle_row_distances.restype = None
        L.oracle_sort_vote.argtypes = [P, P, i64, i32, i32, P, i32]
        L.oracle_sort_vote.restype = i32
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def normalize(train, test, val=None):
    """In place, cpp:229-306."""
    for a in (train, test, val):
        assert a is None or (a.dtype == np.float64 and a.flags.c_contiguous)
    dim = train.shape[1]
    lib().oracle_normalize(_p(train), train.shape[0], _p(test), test.shape[0], _p(val),
                           0 if val is None else val.shape[0], dim)


def knn(train, train_label, queries, K, euclidean=True, class_cnt=None, n_out=0,
        nthreads=None):
    """cpp:308-381.  Returns (labels, idx[n_q,n_out], dist[n_q,n_out])."""
    train = np.ascontiguousarray(train, dtype=np.float64)
    queries = np.ascontiguousarray(queries, dtype=np.float64)
    train_label = np.ascontiguousarray(train_label, dtype=np.int32)
    if class_cnt is None:
        class_cnt = int(train_label.max()) + 1
    n_q, dim = queries.shape
    labels = np.empty(n_q, np.int32)
    idx = np.empty((n_q, n_out), np.int64) if n_out else None
    dist = np.empty((n_q, n_out), np.float64) if n_out else None
    if nthreads is None:
        nthreads = os.cpu_count() or 1
    rc = lib().oracle_knn(_p(train), _p(train_label), train.shape[0], dim, _p(queries), n_q,
                          K, int(bool(euclidean)), class_cnt, _p(labels), _p(idx), _p(dist),
                          n_out, nthreads)
    if rc:
        raise ValueError("oracle_knn rejected inputs (rc=%d)" % rc)
    return labels, idx, dist


def distance(q, x, euclidean=True):
    q = np.ascontiguousarray(q, np.float64)
    x = np.ascontiguousarray(x, np.float64)
    return lib().oracle_distance(_p(q), _p(x), q.shape[0], int(bool(euclidean)))


def row_distances(q, X, euclidean=True):
    """dist(q, X[j]) for every row j (cpp:33-67 arithmetic)."""
    q = np.ascontiguousarray(q, np.float64)
    X = np.ascontiguousarray(X, np.float64)
    out = np.empty(X.shape[0], np.float64)
    lib().oracle_row_distances(_p(q), _p(X), X.shape[0], X.shape[1], int(bool(euclidean)),
                               _p(out))
    return out


def sort_vote(D, labels, K, class_cnt, n_out=0):
    """The reference's std::sort of records (labels[j], D[j]) in fill order j,
    then its vote over the first K: (label, first n_out record indices)."""
    D = np.ascontiguousarray(D, np.float64)
    labels = np.ascontiguousarray(labels, np.int32)
    idx = np.empty(max(n_out, 1), np.int64)
    lab = lib().oracle_sort_vote(_p(D), _p(labels), D.shape[0], int(K), int(class_cnt), _p(idx),
                                 int(n_out))
    return int(lab), idx[:n_out]


def acc(real, pred):
    real = np.ascontiguousarray(real, np.int32)
    pred = np.ascontiguousarray(pred, np.int32)
    return lib().oracle_acc(_p(real), _p(pred), real.shape[0])


def read_csv(path, dim, with_label, max_rows):
    data = np.zeros((max_rows, dim), np.float64)
    labels = np.zeros(max_rows, np.int32)
    n = lib().oracle_read_csv(path.encode(), dim, int(with_label), max_rows, _p(data),
                              _p(labels))
    if n < 0:
        raise FileNotFoundError(path)
    return data, (labels if with_label else None), n
