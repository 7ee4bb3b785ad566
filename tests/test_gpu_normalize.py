"""GPU min-max normalisation (knn_normalize.hip, cpp:229-306) against the
oracle: bit-exact fp64 on every value, bounds included.

Edge cases the reference's code implies: constant dimensions (max == min,
left untouched), dimensions entirely below -1 / above 999999 (the quirky
initial values win), +-inf (range inf / nan), NaN values (never win a
compare), empty query sets, Validation=false (two sets), and sizes past
one grid sweep.  At 1M x 128 the check is the same formula restated in
vectorised numpy (identical IEEE operations)."""
import numpy as np
import pytest
import torch

import oracle

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


@pytest.fixture(scope="module")
def clf(knn):
    c = knn.Classifier(0)
    yield c
    c.close()


def _sets(n, m, v, d, seed, special=True):
    rng = np.random.default_rng(seed)
    X = rng.normal(0, 3, (n + m + v, d))
    if special and d >= 8:
        X[:, 0] = 2.5                                # constant dim
        X[:, 1] = rng.uniform(-9, -2, n + m + v)     # all below -1: max stays -1
        X[:, 2] = rng.uniform(1.5e6, 2e6, n + m + v)  # all above 999999: min stays 999999
        X[:, 3] = np.round(X[:, 3])                  # integer-valued, ties
        N = n + m + v                                # tiny sets: wrap the special rows
        X[5 % N, 4] = np.inf                         # range inf -> values nan / 0
        X[7 % N, 5] = -np.inf
        X[11 % N, 6] = np.nan                        # NaN never wins a compare
        X[:, 7] = 0.0                                # zero-range zeros
    return X[:n].copy(), X[n:n + m].copy(), X[n + m:].copy()


def _same_bits(a, b):
    """Bit-identical, except that any NaN matches any NaN: inf/inf yields the
    host's default NaN (sign bit set on x86) and the GPU's (sign clear)."""
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return False
    same = a.view(np.int64) == b.view(np.int64)
    return bool((same | (np.isnan(a) & np.isnan(b))).all())


@pytest.mark.parametrize("n,m,v,d", [(1000, 200, 100, 16), (5000, 777, 0, 33), (3, 1, 2, 8),
                                     (20000, 300, 300, 128), (700, 0, 0, 784)])
def test_normalize_matches_oracle(clf, n, m, v, d):
    tr, te, va = _sets(n, m, v, d, seed=n + d)
    wtr, wte, wva = tr.copy(), te.copy(), va.copy()
    oracle.normalize(wtr, wte, wva if v else None)
    mx, mn = clf.normalize(tr, te, va) if v else clf.normalize(tr, te)
    assert _same_bits(tr, wtr) and _same_bits(te, wte) and _same_bits(va, wva)
    # bounds: the reference's scan of the raw values (NaN never wins)
    raw = np.concatenate(_sets(n, m, v, d, seed=n + d))
    np.testing.assert_array_equal(mx, np.nanmax(np.concatenate([raw, np.full((1, d), -1.0)]), 0))
    np.testing.assert_array_equal(mn, np.nanmin(np.concatenate([raw, np.full((1, d), 999999.0)]),
                                                0))


@pytest.mark.parametrize("devs,rccl", [([0], False), ([0], True), ([0, 0, 0], False)])
def test_group_normalize_matches_oracle(knn, devs, rccl):
    """The group's sharded normalisation: one GPU; one GPU with the MAX / MIN
    all-reduce through a one-rank RCCL communicator; three ranks on one GPU
    (loopback transport: ragged shards, the all-reduce over three partials)."""
    tr, te, va = _sets(4099, 501, 250, 96, seed=3)
    wtr, wte, wva = tr.copy(), te.copy(), va.copy()
    oracle.normalize(wtr, wte, wva)
    g = knn.Group(devs, mode=0, rccl=rccl)
    try:
        assert g.transport() == (2 if len(devs) > 1 else 1 if rccl else 0)
        g.normalize(tr, te, va)
    finally:
        g.close()
    assert _same_bits(tr, wtr) and _same_bits(te, wte) and _same_bits(va, wva)


def test_device_api_and_sharded_decomposition(knn, clf):
    """The device entry points under knn_dist.normalize_sharded (world 1),
    i.e. the per-rank half of the multi-process path."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location(
        "knn_dist", os.path.join(root, "-mpi-knn-_amd", "knn_dist.py"))
    kd = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(kd)
    tr, te, va = _sets(3000, 400, 0, 40, seed=9)
    wtr, wte = tr.copy(), te.copy()
    oracle.normalize(wtr, wte, None)
    dev = torch.device("cuda", 0)
    ttr, tte = torch.from_numpy(tr).to(dev), torch.from_numpy(te).to(dev)
    torch.cuda.synchronize()

    def fold(X, mx, mn, init):
        clf.minmax_device(X.data_ptr(), X.shape[0], X.shape[1], mx.data_ptr(), mn.data_ptr(),
                          init=init)

    def apply(X, mx, mn):
        clf.normalize_device(X.data_ptr(), X.shape[0], X.shape[1], mx.data_ptr(), mn.data_ptr())

    kd.normalize_sharded([ttr, tte], fold, apply, 40, device=dev)
    clf.sync()
    assert _same_bits(ttr.cpu().numpy(), wtr) and _same_bits(tte.cpu().numpy(), wte)


def test_normalize_full_size(clf):
    """cfg2 shape (1M train + 10k + 10k, d=128): vectorised restatement."""
    rng = np.random.default_rng(5)
    tr = rng.normal(0.3, 2.0, (1_000_000, 128))
    te = rng.normal(0.3, 2.0, (10_000, 128))
    va = rng.normal(0.3, 2.0, (10_000, 128))
    mx = np.maximum(np.maximum(tr.max(0), te.max(0)), np.maximum(va.max(0), -1.0))
    mn = np.minimum(np.minimum(tr.min(0), te.min(0)), np.minimum(va.min(0), 999999.0))
    r = mx - mn
    want = [(a - mn) / r for a in (tr, te, va)]
    gmx, gmn = clf.normalize(tr, te, va)
    assert _same_bits(gmx, mx) and _same_bits(gmn, mn)
    for a, w in zip((tr, te, va), want):
        assert _same_bits(a, w)
    assert tr.min() >= 0.0 and tr.max() <= 1.0
