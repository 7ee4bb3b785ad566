"""Region order of the train images (knn_order.hip): the candidate pass
streams each query tile's own region first.  The order changes no result:
the same labels, neighbour indices and fp64 distances, bit for bit, with
the region order off, automatic and at 64 regions, on the int8 kernels
(16x16x64 at d = 128, 32x32x32 at d = 96) and the fp16 kernel; a slice of
the queries also against the CPU oracle.  Sizes put the automatic choice
above its threshold on the int8 paths (12 regions at n = 200000; the fp16 case
forces 64)."""
import numpy as np
import pytest

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


def _data(path, n, m, seed):
    rng = np.random.default_rng(seed)
    d = 96 if path == "i8w" else 128
    classes = 10
    cen = rng.uniform(40, 215, (classes, d))
    lab = rng.integers(0, classes, n + m).astype(np.int32)
    X = cen[lab] + 25 * rng.standard_normal((n + m, d))
    if path in ("i8", "i8w"):
        X = np.clip(np.rint(X), 0, 255) / 256.0   # byte grid: the int8 pass
    else:
        X = X / 256.0                             # continuous: fp16
    return X[:n].copy(), lab[:n].copy(), X[n:].copy(), classes


@pytest.mark.parametrize("path", ["i8", "i8w", "fp16"])
def test_region_order_changes_no_result(knn, path):
    n, m, k = 200000, 4500, 10
    tr, lab, te, classes = _data(path, n, m, 4242)
    outs = {}
    for order in (0, -1, 64):
        c = knn.Classifier(0)
        c.set_tuning("order", order)
        # (64 regions: streams start at each tile's own region, not at one of
        # the default 8 phases)
        c.set_tuning("ophase", 0 if order == 64 else -1)
        if path == "fp16":
            c.set_precision(knn.PRECISION_FP16)
        if path == "i8":  # the 16x16x64 kernel (AUTO takes 32x32x32 at d = 128)
            c.set_tuning("i8w", 0)
        c.set_train(tr, lab, classes)
        got, idx, dist, flags = c.classify(te, k, 0, return_neighbors=True)
        assert c.last_candidate_path() == {"i8": 5, "i8w": 6, "fp16": 4}[path]
        outs[order] = (got, idx, dist, c.last_rescan_count())
        c.close()
    base = outs[0]
    for order in (-1, 64):
        got, idx, dist, _ = outs[order]
        np.testing.assert_array_equal(got, base[0])
        np.testing.assert_array_equal(idx, base[1])
        np.testing.assert_array_equal(dist.view(np.int64), base[2].view(np.int64))
    # a slice against the oracle (the full set takes the C oracle minutes)
    sl = slice(0, 200)
    want, widx, wdist = oracle.knn(tr, lab, te[sl], k, True, classes, n_out=k)
    np.testing.assert_array_equal(base[0][sl], want)
    np.testing.assert_array_equal(base[2][sl].view(np.int64), wdist.view(np.int64))


def test_region_order_small_batches_and_retrain(knn):
    """Batches below one query tile, ragged batches, a second train set
    through the same context (the layout is rebuilt), and a context switched
    to order 0 after a region-ordered train set (queries in call order, lists
    still mapped to train rows): all exact against the oracle."""
    tr, lab, te, classes = _data("i8", 40000, 700, 77)
    c = knn.Classifier(0)
    c.set_tuning("order", 5)
    c.set_tuning("i8", 1)
    c.set_tuning("ties", 2)  # every tie in the reference's order: indices comparable
    for X, L in ((tr, lab), (tr[::-1].copy(), lab[::-1].copy())):
        c.set_train(X, L, classes)
        for q in (te[:1], te[:37], te[:700]):
            got, idx, dist, _ = c.classify(q, 7, 0, return_neighbors=True)
            want, widx, wdist = oracle.knn(X, L, q, 7, True, classes, n_out=7)
            np.testing.assert_array_equal(got, want)
            np.testing.assert_array_equal(dist.view(np.int64), wdist.view(np.int64))
            np.testing.assert_array_equal(idx, widx)
    c.set_tuning("order", 0)
    got, idx, dist, _ = c.classify(te, 7, 0, return_neighbors=True)
    want, widx, wdist = oracle.knn(tr[::-1].copy(), lab[::-1].copy(), te, 7, True, classes, n_out=7)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(idx, widx)
    c.close()


def test_region_order_large_query_batch(knn):
    """More than 64 sort blocks of queries (m > 65536): the query sort's scan
    kernel runs between the fused histogram and the scatter.  Same results
    as train order, bit for bit."""
    tr, lab, te, classes = _data("i8", 200000, 70000, 99)
    outs = []
    for order in (0, -1):
        c = knn.Classifier(0)
        c.set_tuning("order", order)
        c.set_tuning("i8w", 0)  # the 16x16x64 kernel (AUTO takes 32x32x32 at d = 128)
        c.set_train(tr, lab, classes)
        got, idx, dist, _ = c.classify(te, 10, 0, return_neighbors=True)
        assert c.last_candidate_path() == 5
        outs.append((got, idx, dist))
        c.close()
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    np.testing.assert_array_equal(outs[0][2].view(np.int64), outs[1][2].view(np.int64))
    want, _, wdist = oracle.knn(tr, lab, te[:100], 10, True, classes, n_out=10)
    np.testing.assert_array_equal(outs[1][0][:100], want)
    np.testing.assert_array_equal(outs[1][2][:100].view(np.int64), wdist.view(np.int64))
