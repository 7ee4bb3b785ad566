"""GPU parity: the HIP path (through the C ABI) against the reference.

Two anchors:
  * golden fixtures produced by the reference binary itself (tests/golden);
  * the CPU oracle (oracle/knn_oracle.cpp, itself pinned to those fixtures)
    on seeded inputs at sizes the oracle finishes in seconds, including the
    edge cases the reference's structure implies (ragged sizes, k=1, k=n,
    tiny n, duplicated rows / exact ties, adversarial row order, L1).
Bar: labels identical; neighbour indices and fp64 distances bit-identical,
except that among EXACTLY equal distances the reference's std::sort order
is unspecified -- there we require the same distance multiset and accept
any order (such queries carry KNN_FLAG_TIE_* in out_flags).
"""
import numpy as np
import pytest

import golden_io
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


@pytest.fixture(scope="module",
                params=["auto", "fp32", "m16", "fp16", "fp16w", "i8", "i8w", "ord", "ordh", "nb", "nbw"])
def clf(knn, request):
    """Every parity test runs with the default candidate path (AUTO: int8 for
    integer-coded data and fp16 otherwise for batches of >= 4096 queries at
    d <= 256, else bf16x3 on 32x32x16 for L2), with the fp32 path forced,
    with bf16x3 on the 16x16x32 MFMA layout forced, with the fp16 path forced
    (every batch size), with the fp16 path's alternative forms (fp16w: the S3
    kernel on 32x32x16 above 256 dims, the resident kernel publishing list
    thresholds, gk = 0), and with the int8 path forced wherever the data are
    integer-coded, on its AUTO kernel (i8) and on v_mfma_i32_32x32x32_i8 at
    every width (i8w); other data take the AUTO path.  ord / ordh: the train
    images in region order (tuning "order" = 4 regions, knn_order.hip) with
    the AUTO path and with fp16 forced: queries sorted by region, streams
    starting at each query tile's region, lists mapped back to train rows.
    nb / nbw: the int8 path forced (16x16x64 / 32x32x32) on norm-blocked
    images (tuning "nblk" = 1, knn_order.hip: every 16K-row window sorted by
    code norm; nbw on top of the region order), where the int8 kernels'
    sub-tile seed bound is tight."""
    c = knn.Classifier(0)
    c.set_precision({"auto": knn.PRECISION_AUTO, "fp32": knn.PRECISION_FP32,
                     "m16": knn.PRECISION_BF16X3, "fp16": knn.PRECISION_FP16,
                     "fp16w": knn.PRECISION_FP16, "i8": knn.PRECISION_AUTO,
                     "i8w": knn.PRECISION_AUTO, "ord": knn.PRECISION_AUTO,
                     "ordh": knn.PRECISION_FP16, "nb": knn.PRECISION_AUTO,
                     "nbw": knn.PRECISION_AUTO}[request.param])
    c.set_tuning("mfma16", 1 if request.param == "m16" else -1)
    if request.param in ("i8", "i8w", "nb", "nbw"):
        c.set_tuning("i8", 1)
    if request.param in ("i8w", "nbw"):
        c.set_tuning("i8w", 1)
    c.set_tuning("nblk", 1 if request.param in ("nb", "nbw") else -1)
    if request.param == "fp16w":
        c.set_tuning("s3q", 0)
        c.set_tuning("gk", 0)
    # (the train layout is decided at set_train: every case's own)
    c.set_tuning("order", 4 if request.param in ("ord", "ordh", "nbw") else 0)
    yield c
    c.close()


def assert_neighbors_match(idx, dist, widx, wdist, flags=None, labels_msg=""):
    """Bit-exact distances; indices exact except inside groups of equal distance."""
    assert idx.shape == widx.shape
    dbits, wbits = dist.view(np.int64), wdist.view(np.int64)
    bad = np.nonzero((dbits != wbits).any(1))[0]
    assert bad.size == 0, "distance mismatch at queries %s" % bad[:10]
    diff = np.nonzero((idx != widx).any(1))[0]
    k = idx.shape[1]
    for q in diff:
        # differing indices are only allowed inside runs of equal distances
        d = dist[q]
        boundary = flags is None or bool(flags[q] & 2)  # dist[k-1] == dist[k]
        for t in np.nonzero(idx[q] != widx[q])[0]:
            run = np.nonzero(d == d[t])[0]
            at_edge = run[-1] == k - 1 and boundary
            assert len(run) > 1 or at_edge, "query %d pos %d: index differs without a tie" % (q, t)
            # the same set of indices over the tie run is required unless the run
            # reaches the k-th position and ties past it (membership ambiguous)
            if not at_edge:
                assert set(idx[q][run]) == set(widx[q][run]), "query %d tie group differs" % q
        if flags is not None:
            assert flags[q] & 14, "query %d differs but is not flagged as a tie" % q


# Exact-tie votes over the whole parity suite: queries whose top k holds equal
# distances with different labels (KNN_FLAG_TIE_VOTE), and how many of those
# got a label other than the reference's std::sort order gives (the vote
# then depends on an order the reference leaves unspecified; ours is by train
# index).  Reported at the end of the run (conftest.py) and written to
# gpurun_out/tie_votes.json.
TIE_VOTES = {"cases": 0, "queries": 0, "tie_vote": 0, "tie_vote_label_differs": 0, "where": []}


def run_case(clf, knn, train, lab, queries, k, metric, classes):
    clf.set_train(train, lab, classes)
    got, idx, dist, flags = clf.classify(queries, k, metric, return_neighbors=True)
    want, widx, wdist = oracle.knn(train, lab, queries, k, metric == 0, classes, n_out=k)
    tie_vote = (flags & knn.FLAG_TIE_VOTE) != 0
    assert (got[~tie_vote] == want[~tie_vote]).all(), "labels differ on untied queries"
    differs = int((got[tie_vote] != want[tie_vote]).sum())
    # queries re-ordered as the reference's std::sort (the tied queries whose
    # label that order could change): the same neighbour order as the
    # oracle, index for index; every other tie leaves the label unchanged
    ref = (flags & knn.FLAG_TIE_REF) != 0
    assert not (ref & ((flags & 14) == 0)).any(), "untied query re-ordered"
    np.testing.assert_array_equal(idx[ref], widx[ref])
    TIE_VOTES["reordered"] = TIE_VOTES.get("reordered", 0) + int(ref.sum())
    TIE_VOTES["cases"] += 1
    TIE_VOTES["queries"] += int(len(got))
    TIE_VOTES["tie_vote"] += int(tie_vote.sum())
    TIE_VOTES["tie_vote_label_differs"] += differs
    if differs:
        TIE_VOTES["where"].append(dict(n=int(train.shape[0]), m=int(len(got)), d=int(train.shape[1]),
                                       k=int(k), metric=int(metric), differs=differs))
    assert_neighbors_match(idx, dist, widx, wdist, flags)
    assert differs == 0, "%d exact-tie votes differ from the reference order" % differs
    return got, want, flags


@pytest.mark.parametrize("name", golden_io.names())
def test_golden_fixture(name, clf, knn, fmt_cout):
    fx = golden_io.Fixture(name)
    s = fx.spec
    tr, trl, te, tel, va, val_ = fx.normalized()
    metric = 0 if s["Euclidean_distance"] else 1
    K = s["K"]
    clf.set_train(tr, trl, s["class_cnt"])
    got, idx, dist, flags = clf.classify(te, K, metric, return_neighbors=True)
    np.testing.assert_array_equal(got, fx.test_labels)
    nq = fx.test_nbr_idx.shape[0]
    assert_neighbors_match(idx[:nq], dist[:nq], fx.test_nbr_idx[:nq, :K],
                           fx.test_nbr_dist[:nq, :K], flags[:nq])
    if s["Validation"]:
        vl, vidx, vdist, vflags = clf.classify(va, K, metric, return_neighbors=True)
        acc = float((vl == val_).sum()) / len(val_)  # acc_calc, cpp:69-84
        assert "accuracy = " + fmt_cout(acc) == str(fx.accuracy_line)
        nv = fx.val_nbr_idx.shape[0]
        assert_neighbors_match(vidx[:nv], vdist[:nv], fx.val_nbr_idx[:nv, :K],
                               fx.val_nbr_dist[:nv, :K], vflags[:nv])


def _mix(rng, n, m, d, classes, spread=2.0, grid=1024.0):
    centres = rng.uniform(-spread, spread, (classes, d))
    lab = rng.integers(0, classes, n + m).astype(np.int32)
    X = centres[lab] + rng.standard_normal((n + m, d))
    if grid:
        X = np.round(X * grid) / grid
    tr, te = X[:n].copy(), X[n:].copy()
    oracle.normalize(tr, te, None)
    return tr, lab[:n].copy(), te


CASES = [
    # n, m, d, k, metric, classes
    (5000, 300, 128, 10, 0, 10),
    (4099, 257, 96, 10, 0, 7),      # ragged n (not /32), ragged m (not /128)
    (3000, 130, 13, 5, 0, 3),       # odd dim -> zero padding
    (2000, 64, 1, 3, 0, 2),         # d = 1
    (1000, 100, 64, 1, 0, 4),       # k = 1
    (20, 50, 16, 20, 0, 3),         # k = n, n < one tile
    (31, 40, 8, 30, 1, 3),          # L1, n just under a tile, k = n-1
    (6000, 200, 40, 7, 1, 5),       # L1
    (3000, 150, 256, 50, 0, 10),    # largest register-resident dim, K=50
    (4000, 100, 64, 100, 0, 10),    # K=100 (cfg5's k)
    (8000, 128, 24, 16, 0, 6),
    # large d: bf16x3 S3 stream kernel (auto) / fp32 stream kernel (fp32)
    (3000, 300, 300, 10, 0, 10),    # d not a multiple of 16 -> zero padding, ragged m
    (2500, 257, 784, 50, 0, 10),    # the reference's MNIST dimension, K=50
    (4000, 200, 960, 100, 0, 10),   # cfg5 shape (d=960, k=100), scaled down
    (700, 40, 520, 5, 1, 4),        # L1 at large d (fp32 stream kernel in both modes)
]


@pytest.mark.parametrize("n,m,d,k,metric,classes", CASES)
def test_vs_oracle(n, m, d, k, metric, classes, clf, knn):
    rng = np.random.default_rng(n * 7 + m * 3 + d + k)
    tr, lab, te = _mix(rng, n, m, d, classes)
    run_case(clf, knn, tr, lab, te, k, metric, classes)


def test_duplicates_force_rescan(clf, knn):
    """Many exact duplicates of the nearest rows: the candidate set cannot be
    certified from the fp32 pass, so the exact fp64 rescan must run."""
    rng = np.random.default_rng(7)
    tr, lab, te = _mix(rng, 3000, 64, 32, 4)
    tr[1000:1400] = tr[5]           # 400 identical rows
    lab[1000:1400] = rng.integers(0, 4, 400)
    te[:32] = tr[5]                  # queries sitting exactly on them
    got, want, flags = run_case(clf, knn, tr, lab, te, 9, 0, 4)
    assert clf.last_rescan_count() > 0
    assert (flags[:32] & knn.FLAG_EXACT_RESCAN).all()


def test_scale_extremes(clf, knn):
    """Operand scaling edge cases of the reduced-precision candidate passes:
    queries far outside the train range (fp16 overflow -> rescan), a train
    set of tiny magnitude, and one of huge magnitude; exact results in every
    mode."""
    rng = np.random.default_rng(19)
    tr, lab, te = _mix(rng, 3000, 96, 64, 4)
    te[:8] *= 1e4                    # ~1e4 x the train spread
    te[8:12] = 1e12
    run_case(clf, knn, tr, lab, te, 7, 0, 4)
    run_case(clf, knn, tr * 1e-30, lab, te * 1e-30, 7, 0, 4)
    run_case(clf, knn, tr * 1e25, lab, te * 1e25, 7, 0, 4)
    run_case(clf, knn, tr * 1e-30, lab, te * 1e-30, 7, 1, 4)
    run_case(clf, knn, tr * 1e25, lab, te * 1e25, 7, 1, 4)


def test_integer_ties(clf, knn):
    """SIFT-like integer data: many exact distance ties."""
    rng = np.random.default_rng(11)
    centres = rng.integers(0, 256, (5, 16))
    lab = rng.integers(0, 5, 4200).astype(np.int32)
    X = np.clip(centres[lab] + rng.integers(-6, 7, (4200, 16)), 0, 255).astype(np.float64)
    tr, te = X[:4000].copy(), X[4000:].copy()
    run_case(clf, knn, tr, lab[:4000].copy(), te, 10, 0, 5)
    run_case(clf, knn, tr, lab[:4000].copy(), te, 10, 1, 5)


@pytest.mark.parametrize("metric", [0, 1])
def test_reference_tie_order_everywhere(knn, metric):
    """Tuning "ties" = 2: every query with equal distances in its top k is
    re-ordered as the reference's std::sort orders it (libstdc++ introsort
    emulated over all n exact distances): labels, neighbour indices and
    their order equal the oracle's for EVERY query of an integer data set
    full of exact ties; "ties" = 0 keeps index order inside ties (labels may
    then differ only on flagged queries)."""
    rng = np.random.default_rng(71 + metric)
    centres = rng.integers(0, 256, (5, 12))
    lab = rng.integers(0, 5, 5300).astype(np.int32)
    X = np.clip(centres[lab] + rng.integers(-5, 6, (5300, 12)), 0, 255).astype(np.float64)
    tr, te, lab = X[:5000].copy(), X[5000:].copy(), lab[:5000].copy()
    for k in (10, 37):
        want, widx, wdist = oracle.knn(tr, lab, te, k, metric == 0, 5, n_out=k)
        c = knn.Classifier(0)
        c.set_tuning("ties", 2)
        c.set_train(tr, lab, 5)
        c.tie_totals(reset=True)
        got, idx, dist, flags = c.classify(te, k, metric, return_neighbors=True)
        tied = (flags & 14) != 0
        assert tied.sum() > 50, "expected many tied queries"
        assert ((flags & knn.FLAG_TIE_REF) != 0).sum() == tied.sum()
        assert c.tie_totals() == tied.sum()
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(idx, widx)
        assert (dist.view(np.int64) == wdist.view(np.int64)).all()
        c.set_tuning("ties", 0)
        got0, idx0, dist0, flags0 = c.classify(te, k, metric, return_neighbors=True)
        assert not (flags0 & knn.FLAG_TIE_REF).any()
        np.testing.assert_array_equal(got0[(flags0 & 6) == 0], want[(flags0 & 6) == 0])
        c.close()


def test_sorted_train_rows(clf, knn):
    """Train rows sorted by class (all near neighbours in one contiguous run)."""
    rng = np.random.default_rng(5)
    tr, lab, te = _mix(rng, 12000, 256, 32, 3, spread=3.0)
    order = np.argsort(lab, kind="stable")
    run_case(clf, knn, np.ascontiguousarray(tr[order]), lab[order].copy(), te, 20, 0, 3)


def _grid_codes(rng, n, m, d, classes, lo=0, hi=255, scale=256.0):
    """SIFT-like byte features on the grid (code) / scale, codes in [lo, hi]."""
    centres = rng.uniform(lo + 40, hi - 40, (classes, d))
    lab = rng.integers(0, classes, n + m).astype(np.int32)
    X = np.clip(np.rint(centres[lab] + 25 * rng.standard_normal((n + m, d))), lo, hi) / scale
    return X[:n].copy(), lab[:n].copy(), X[n:].copy()


def _i8_kernel(d, i8w):
    """(kernel metric, padded dim) the int8 pass runs at: 32x32x32 (metric 6,
    K granularity 32) where it pads less than 16x16x64 (metric 5, K 64) and
    at DP = 128, or as forced by the "i8w" tuning key."""
    w = min(p for p in (32, 64, 96, 128, 160, 192, 256) if p >= d)
    q = (d + 63) // 64 * 64
    if i8w == 1 or (i8w < 0 and (w < q or w == 128)):
        return 6, w
    return 5, q


@pytest.mark.parametrize("d", [32, 64, 96, 128, 200, 256])
@pytest.mark.parametrize("i8w", [-1, 0, 1])
def test_int8_codes(knn, d, i8w):
    """The int8 pass (exact integer dot products of the data's codes) against
    the oracle on 8-bit grid data -- the full byte range (codes 0..255, centre
    128) -- forced and in AUTO at 4096+ queries, on both kernels:
    v_mfma_i32_16x16x64_i8 (metric 5, dims padded to 64) and
    v_mfma_i32_32x32x32_i8 (metric 6, dims padded to 32: AUTO's choice at
    d = 32 and 96); every padded width (d = 200 pads to 256)."""
    rng = np.random.default_rng(80 + d)
    tr, lab, te = _grid_codes(rng, 9000, 4200, d, 7)
    assert tr.min() == 0.0 and tr.max() == 255 / 256.0
    km, dp = _i8_kernel(d, i8w)
    for mode in ("forced", "auto"):
        c = knn.Classifier(0)
        c.set_tuning("i8w", i8w)
        if mode == "forced":
            c.set_tuning("i8", 1)
        run_case(c, knn, tr, lab, te, 10, 0, 7)
        assert c.last_candidate_path() == km, mode
        # (metric 6: two 4-entry lists per lane by default, knn_api.cpp)
        assert c.last_kernel_name().startswith("cand_kernel<%d,4,%d,8>" % (dp, km))
        assert c.last_rescan_count() * 16 <= te.shape[0]
        c.close()


def test_int8_off_grid_queries(knn):
    """Queries the int8 codes cannot hold exactly -- off the train grid,
    beyond the code range -- are coded rounded / saturated and their measured
    coding error widens the bound (far-out ones fail certification and take
    the exact rescan); integer data at scale 1 with negative values; k = 50.
    Exact answers."""
    rng = np.random.default_rng(91)
    tr, lab, te = _grid_codes(rng, 6000, 300, 48, 5, lo=-100, hi=120, scale=1.0)
    te[:5, 3] += 0.5          # off the integer grid
    te[5:9, 7] = 121.0 + 200  # beyond the codes the centre leaves room for
    c = knn.Classifier(0)
    c.set_tuning("i8", 1)
    got, want, flags = run_case(c, knn, tr, lab, te, 50, 0, 5)
    assert c.last_candidate_path() == 5
    assert (flags[5:9] & knn.FLAG_EXACT_RESCAN).all()
    # a train set off any 8-bit grid: the int8 pass is not available, the
    # forced request falls back to the other paths (still exact)
    tr2 = tr.copy()
    tr2[17, 2] += 1e-3
    run_case(c, knn, tr2, lab, te, 10, 0, 5)
    assert c.last_candidate_path() != 5
    c.close()


@pytest.mark.parametrize("order", [0, 4])
@pytest.mark.parametrize("path", ["i8", "i8w", "fp16", "s3"])
def test_targeted_rescan(knn, path, order):
    """Per-split certification: with few splits (tuning S = 2, 3) a lane list
    often holds R of a query's top W, so its bound fails; the merge then
    flags only the splits whose own bound fails, hands the re-ranked rows of
    the others to the rescan, and the rescan scans just the flagged splits'
    rows (knn_select.hip).  Exact answers against the oracle on the int8
    (grid data), fp16 (continuous data) and fp16 S3 (d = 300) paths, with the
    train images in train order and in region order (order = 4: a split's
    rows are then image positions, mapped back to train rows)."""
    rng = np.random.default_rng(123)
    if path in ("i8", "i8w"):
        tr, lab, te = _grid_codes(rng, 20000, 600, 64 if path == "i8" else 96, 6)
        k = 10
    else:
        d = 300 if path == "s3" else 64
        k = 40 if path == "s3" else 10
        cen = rng.uniform(-1, 1, (6, d))
        lab_all = rng.integers(0, 6, 20600).astype(np.int32)
        X = cen[lab_all] + 0.35 * rng.standard_normal((20600, d))
        tr, te, lab = X[:20000].copy(), X[20000:].copy(), lab_all[:20000].copy()
    rescans = 0
    # metric 6 (i8w): the failed queries' rescan filters the int8 image on the
    # codes (i8resc auto) and, as a check of both filters, the fp32 image
    for S, i8resc in ((2, -1), (3, -1)) + (((2, 0),) if path == "i8w" else ()):
        c = knn.Classifier(0)
        if path in ("i8", "i8w"):
            c.set_tuning("i8", 1)
        else:
            c.set_precision(knn.PRECISION_FP16)
        c.set_tuning("S", S)
        c.set_tuning("order", order)
        c.set_tuning("i8resc", i8resc)
        run_case(c, knn, tr, lab, te, k, 0, 6)
        assert c.last_candidate_path() == {"i8": 5, "i8w": 6}.get(path, 4)
        assert c.last_geometry()["splits"] == S
        rescans += c.last_rescan_count()
        c.close()
    assert rescans > 0, "expected certification failures with 2-3 splits"


@pytest.mark.parametrize("path", ["i8", "fp16"])
def test_seeded_thresholds(knn, path):
    """Seeded global thresholds (knn_api.cpp seed_rows / ensure_sample; an
    experiment option, off by default): a pre-pass of the same candidate
    kernel over a strided sample of the train rows seeds every query's slots
    with the need-th smallest of its sample lists; exact answers with and
    without it, and after a new train set (the sample image is rebuilt)."""
    rng = np.random.default_rng(321)
    if path == "i8":
        tr, lab, te = _grid_codes(rng, 40000, 4500, 64, 6)
    else:
        cen = rng.uniform(-1, 1, (6, 64))
        lab_all = rng.integers(0, 6, 44500).astype(np.int32)
        X = cen[lab_all] + 0.35 * rng.standard_normal((44500, 64))
        tr, te, lab = X[:40000].copy(), X[40000:].copy(), lab_all[:40000].copy()
    for seed in (0, 8192, 32768):
        c = knn.Classifier(0)
        if path == "fp16":
            c.set_precision(knn.PRECISION_FP16)
        c.set_tuning("seed", seed)
        run_case(c, knn, tr, lab, te, 10, 0, 6)
        assert c.last_candidate_path() == (5 if path == "i8" else 4)
        # a second train set through the same context: the sample is rebuilt
        run_case(c, knn, tr[::-1].copy(), lab[::-1].copy(), te, 10, 0, 6)
        assert c.last_candidate_path() == (5 if path == "i8" else 4)
        c.close()


def test_k_zero_and_errors(clf, knn):
    rng = np.random.default_rng(3)
    tr, lab, te = _mix(rng, 500, 10, 8, 2)
    clf.set_train(tr, lab, 2)
    assert (clf.classify(te, 0) == -1).all()   # cpp:324: max_label = -1
    with pytest.raises(knn.KnnError):
        clf.classify(te, 501)                  # k > n_train (reference UB)
    with pytest.raises(knn.KnnError):
        clf.set_train(tr, np.full(500, 2, np.int32), 2)  # label out of range


@pytest.mark.parametrize("n,m,d,k,metric,grid", [
    (3000, 40, 20, 1500, 0, 1024.0),   # k > 1000: the exact large-k path (L2)
    (2600, 33, 7, 1200, 1, 1024.0),    # L1
    (1500, 20, 4, 1499, 0, 16.0),      # k = n - 1 on a coarse grid: long exact-tie runs
])
def test_large_k(n, m, d, k, metric, grid, clf, knn):
    """k beyond the candidate lists' capacity (the reference accepts any
    K <= N_train, cpp:328): the exact large-k path -- labels, neighbour
    distances and indices against the oracle, and a partial (w > 1001) list."""
    rng = np.random.default_rng(n + k)
    tr, lab, te = _mix(rng, n, m, d, 5, grid=grid)
    run_case(clf, knn, tr, lab, te, k, metric, 5)
    # a NaN / inf query coordinate on the large-k path: label -1 and
    # KNN_FLAG_NONFINITE (its test is a bit test; the TU ignores NaNs)
    te2 = te.copy()
    te2[1, 0] = np.nan
    te2[2, d - 1] = -np.inf
    got2, idx2, dist2, flags2 = clf.classify(te2, k, metric, return_neighbors=True)
    assert (got2[[1, 2]] == -1).all() and (flags2[[1, 2]] & knn.FLAG_NONFINITE).all()
    assert (idx2[[1, 2]] == -1).all() and np.isnan(dist2[[1, 2]]).all()
    ok = np.setdiff1d(np.arange(m), [1, 2])
    got1 = clf.classify(te, k, metric)
    np.testing.assert_array_equal(got2[ok], got1[ok])
    import torch
    dev = torch.device("cuda", 0)
    X = torch.from_numpy(tr).to(dev)
    L = torch.from_numpy(lab).to(dev)
    Q = torch.from_numpy(te).to(dev)
    clf.set_train_device(X.data_ptr(), L.data_ptr(), n, d, 5, keep=(X, L))
    w = k + 1
    pd = torch.empty((m, w), dtype=torch.float64, device=dev)
    pi = torch.empty((m, w), dtype=torch.int64, device=dev)
    pl = torch.empty((m, w), dtype=torch.int32, device=dev)
    clf.search_partial_device(Q.data_ptr(), m, w, metric, pd.data_ptr(), pi.data_ptr(),
                              pl.data_ptr())
    clf.sync()
    _, widx, wdist = oracle.knn(tr, lab, te, k, metric == 0, 5, n_out=w)
    assert_neighbors_match(pi.cpu().numpy(), pd.cpu().numpy(), widx, wdist)
    np.testing.assert_array_equal(pl.cpu().numpy(), lab[pi.cpu().numpy()])


def test_device_api_and_partial_merge(clf, knn):
    """knn_classify_device + search_partial/merge_vote (train-sharded building
    blocks) on one GPU: shard the train set in two contexts, merge, compare."""
    import torch
    rng = np.random.default_rng(9)
    tr, lab, te = _mix(rng, 6000, 300, 48, 5)
    k = 10
    want, widx, wdist = oracle.knn(tr, lab, te, k, True, 5, n_out=k)
    dev = torch.device("cuda", 0)
    parts, half = 2, 3000
    w = k + 1
    c2 = knn.Classifier(0)
    Xs = [torch.from_numpy(tr[:half]).to(dev), torch.from_numpy(tr[half:]).to(dev)]
    Ls = [torch.from_numpy(lab[:half]).to(dev), torch.from_numpy(lab[half:]).to(dev)]
    Q = torch.from_numpy(te).to(dev)
    m = te.shape[0]
    gd = torch.empty((parts, m, w), dtype=torch.float64, device=dev)
    gi = torch.empty((parts, m, w), dtype=torch.int64, device=dev)
    gl = torch.empty((parts, m, w), dtype=torch.int32, device=dev)
    for p, c in enumerate((clf, c2)):
        c.set_train_device(Xs[p].data_ptr(), Ls[p].data_ptr(), half, 48, 5, idx_offset=p * half,
                           keep=(Xs[p], Ls[p]))
        c.search_partial_device(Q.data_ptr(), m, w, knn.L2, gd[p].data_ptr(), gi[p].data_ptr(),
                                gl[p].data_ptr())
        c.sync()
    ol = torch.empty(m, dtype=torch.int32, device=dev)
    oi = torch.empty((m, k), dtype=torch.int64, device=dev)
    od = torch.empty((m, k), dtype=torch.float64, device=dev)
    of = torch.empty(m, dtype=torch.int32, device=dev)
    clf.merge_vote_device(gd.data_ptr(), gi.data_ptr(), gl.data_ptr(), parts, m, w, k,
                          ol.data_ptr(), oi.data_ptr(), od.data_ptr(), of.data_ptr())
    clf.sync()
    np.testing.assert_array_equal(ol.cpu().numpy(), want)
    assert_neighbors_match(oi.cpu().numpy(), od.cpu().numpy(), widx, wdist, of.cpu().numpy())
    # device classify on the full set
    Xf = torch.from_numpy(tr).to(dev)
    Lf = torch.from_numpy(lab).to(dev)
    clf.set_train_device(Xf.data_ptr(), Lf.data_ptr(), 6000, 48, 5, keep=(Xf, Lf))
    clf.classify_device(Q.data_ptr(), m, k, knn.L2, ol.data_ptr(), oi.data_ptr(), od.data_ptr(),
                        of.data_ptr())
    clf.sync()
    np.testing.assert_array_equal(ol.cpu().numpy(), want)
    c2.close()


@pytest.mark.parametrize("metric", [0, 1])
def test_partial_merge_large_k(knn, metric):
    """Train-sharded merge of unions beyond the LDS merge (4 shards x 1201 =
    4804 entries at k = 1200; the reference accepts any K <= N_train,
    cpp:328): each shard's exact top-1201 (large-k path), then the rank merge
    + vote -- labels, neighbour distances and indices against the oracle."""
    import torch
    rng = np.random.default_rng(60 + metric)
    n, m, d, k, parts = 8000, 40, 16, 1200, 4
    tr, lab, te = _mix(rng, n, m, d, 5)
    want, widx, wdist = oracle.knn(tr, lab, te, k, metric == 0, 5, n_out=k)
    dev = torch.device("cuda", 0)
    w = k + 1
    Q = torch.from_numpy(te).to(dev)
    gd = torch.empty((parts, m, w), dtype=torch.float64, device=dev)
    gi = torch.empty((parts, m, w), dtype=torch.int64, device=dev)
    gl = torch.empty((parts, m, w), dtype=torch.int32, device=dev)
    keep = []
    for p in range(parts):
        r0, r1 = n * p // parts, n * (p + 1) // parts
        c = knn.Classifier(0)
        Xs = torch.from_numpy(tr[r0:r1].copy()).to(dev)
        Ls = torch.from_numpy(lab[r0:r1].copy()).to(dev)
        c.set_train_device(Xs.data_ptr(), Ls.data_ptr(), r1 - r0, d, 5, idx_offset=r0,
                           keep=(Xs, Ls))
        c.search_partial_device(Q.data_ptr(), m, w, metric, gd[p].data_ptr(), gi[p].data_ptr(),
                                gl[p].data_ptr())
        c.sync()
        keep.append(c)
    lab_all = torch.from_numpy(lab).to(dev)
    rows = [n * (p + 1) // parts - n * p // parts for p in range(parts)]
    # the whole slice, then two ragged query slices (q0 > 0)
    for q0, q1 in ((0, m), (0, 17), (17, m)):
        mq = q1 - q0
        ol = torch.empty(mq, dtype=torch.int32, device=dev)
        oi = torch.empty((mq, k), dtype=torch.int64, device=dev)
        od = torch.empty((mq, k), dtype=torch.float64, device=dev)
        of = torch.empty(mq, dtype=torch.int32, device=dev)
        keep[0].merge_vote_device(gd.data_ptr(), gi.data_ptr(), gl.data_ptr(), parts, m, w, k,
                                  ol.data_ptr(), oi.data_ptr(), od.data_ptr(), of.data_ptr(),
                                  q0=q0, mq=mq)
        keep[0].sync()
        # flagged queries: the reference's order over the whole train set
        # (every shard's distances, then the owner's resolve)
        pend = torch.nonzero(of & knn.FLAG_TIE_PENDING).flatten().to(torch.int32)
        if pend.numel():
            sel = pend + q0
            blocks = []
            for c, nr in zip(keep, rows):
                D = torch.empty((pend.numel(), nr), dtype=torch.float64, device=dev)
                c.shard_distances_device(Q.data_ptr(), sel.data_ptr(), pend.numel(), metric,
                                         D.data_ptr())
                c.sync()
                blocks.append(D.reshape(-1))
            Dall = torch.cat(blocks)
            keep[0].tie_resolve_device(Dall.data_ptr(), rows, pend.numel(), lab_all.data_ptr(),
                                       pend.data_ptr(), k, ol.data_ptr(), oi.data_ptr(),
                                       od.data_ptr(), of.data_ptr())
            keep[0].sync()
        got = ol.cpu().numpy()
        flags = of.cpu().numpy()
        tv = (flags & knn.FLAG_TIE_VOTE) != 0
        TIE_VOTES["tie_vote"] += int(tv.sum())
        TIE_VOTES["tie_vote_label_differs"] += int((got[tv] != want[q0:q1][tv]).sum())
        np.testing.assert_array_equal(got, want[q0:q1])
        assert_neighbors_match(oi.cpu().numpy(), od.cpu().numpy(), widx[q0:q1], wdist[q0:q1],
                               flags)
    for c in keep:
        c.close()


def test_group_train_sharded_k_beyond_lds(knn):
    """knn_group mode 1 with k + 1 > 4096 (one GPU): the rank merge serves
    what the LDS merge cannot (formerly refused: ngpus * (k+1) <= 4096)."""
    rng = np.random.default_rng(62)
    tr, lab, te = _mix(rng, 6000, 24, 8, 5)
    k = 4500
    want, widx, wdist = oracle.knn(tr, lab, te, k, True, 5, n_out=k)
    g = knn.Group([0], 1)
    g.set_train(tr, lab, 5)
    got, idx, dist, flags = g.classify(te, k, knn.L2, return_neighbors=True)
    tv = (flags & knn.FLAG_TIE_VOTE) != 0
    TIE_VOTES["tie_vote"] += int(tv.sum())
    TIE_VOTES["tie_vote_label_differs"] += int((got[tv] != want[tv]).sum())
    np.testing.assert_array_equal(got, want)
    assert_neighbors_match(idx, dist, widx, wdist, flags)
    g.close()


def test_group_single_gpu_modes(knn):
    rng = np.random.default_rng(21)
    tr, lab, te = _mix(rng, 5000, 333, 32, 6)
    want, widx, wdist = oracle.knn(tr, lab, te, 7, True, 6, n_out=7)
    for mode in (0, 1):
        g = knn.Group([0], mode)
        g.set_train(tr, lab, 6)
        got, idx, dist, flags = g.classify(te, 7, knn.L2, return_neighbors=True)
        np.testing.assert_array_equal(got, want)
        assert_neighbors_match(idx, dist, widx, wdist, flags)
        g.close()


def test_driver_matches_reference_outputs(tmp_path, knn):
    """The native drop-in driver on the reference's CSV files reproduces
    Test_label.csv and the accuracy line of the reference run."""
    for name in ("f1_cfg1", "f3_l1", "f5_csv_crlf", "f7_nonorm_noval"):
        fx = golden_io.Fixture(name)
        s = fx.spec
        d = tmp_path / name
        d.mkdir()
        cfg = knn.KnnConfig(dim=s["dim"], K=s["K"], N_train=s["N_train"], N_test=s["N_test"],
                            N_val=s["N_val"], class_cnt=s["class_cnt"],
                            Euclidean_distance=s["Euclidean_distance"], Normalize=s["Normalize"],
                            Validation=s["Validation"])
        fx.write_inputs(str(d), names=(cfg.train_file_name, cfg.validation_file_name,
                                       cfg.test_file_name))
        out = knn.run_driver(cfg, str(d))
        labels = np.loadtxt(d / "Test_label.csv", dtype=np.int64, ndmin=1)
        np.testing.assert_array_equal(labels, fx.test_labels)
        if s["Validation"]:
            assert str(fx.accuracy_line) in out
        assert "Running time is " in out


@pytest.mark.parametrize("nw", [4, 8, 16])
def test_fp16_workgroup_sizes(knn, nw):
    """The fp16 kernel at 4, 8 and 16 waves per workgroup (16: 512 queries
    share each staged tile), and the "nw" override on the other paths
    (16 is clamped to 8 there): every launch matches the oracle."""
    rng = np.random.default_rng(nw)
    tr, lab, te = _mix(rng, 6000, 700, 128, 6)
    for prec in (knn.PRECISION_FP16, knn.PRECISION_BF16X3, knn.PRECISION_FP32):
        c = knn.Classifier(0)
        c.set_precision(prec)
        c.set_tuning("nw", nw)
        run_case(c, knn, tr, lab, te, 10, 0, 6)
        c.close()


@pytest.mark.parametrize("gk", [0, 1, 2, 3, 4])
def test_global_threshold_ranks(knn, gk):
    """The resident fp16 kernel with every global-threshold publish rule (gk:
    0 = the lists' R-th entries in 4 groups, K = 1..4 = the K-th smallest of
    the union of a workgroup's lists in 8 groups).  K = 1 guarantees fewer
    rows below the threshold than k+1 (certification then fails more and
    the rescan finishes those queries): the answer is exact either way."""
    rng = np.random.default_rng(40 + gk)
    tr, lab, te = _mix(rng, 20000, 600, 128, 6)
    c = knn.Classifier(0)
    c.set_precision(knn.PRECISION_FP16)
    c.set_tuning("gk", gk)
    run_case(c, knn, tr, lab, te, 10, 0, 6)
    c.close()


@pytest.mark.parametrize("qres", [1, 0])
@pytest.mark.parametrize("gk", [0, 1, 6, 16])
def test_s3_global_threshold_ranks(knn, gk, qres):
    """The fp16 d > 256 kernels with quad lists -- the query-resident kernel
    (qres 1) and S3 on 16x16x32 (qres 0) -- with the global
    threshold off (gk 0) and published at ranks 1, 6 and 16 of each
    workgroup's quad union."""
    rng = np.random.default_rng(50 + gk)
    tr, lab, te = _mix(rng, 6000, 300, 300, 5)
    c = knn.Classifier(0)
    c.set_precision(knn.PRECISION_FP16)
    c.set_tuning("gk", gk)
    c.set_tuning("qres", qres)
    run_case(c, knn, tr, lab, te, 40, 0, 5)
    assert c.last_kernel_name() == ("cand_qres_kernel<10>" if qres else "cand_s3_kernel<8,true,true>")
    c.close()


@pytest.mark.parametrize("d", [260, 300, 500, 784, 960])
def test_query_resident_dims(knn, d):
    """The query-resident fp16 kernel (knn_cand_qres.hip) at padded widths 288,
    320, 512, 800 and 960 (9, 10, 16, 25 and 30 chunks: its chunkings of 3, 2
    and 5 k-steps) on ragged n and m, against the oracle; the S3 kernel gives
    the same answer."""
    rng = np.random.default_rng(900 + d)
    tr, lab, te = _mix(rng, 3001, 301, d, 6)
    c = knn.Classifier(0)
    c.set_precision(knn.PRECISION_FP16)
    c.set_tuning("qres", 1)
    run_case(c, knn, tr, lab, te, 12, 0, 6)
    assert c.last_kernel_name() == "cand_qres_kernel<%d>" % ((d + 31) // 32)
    c.set_tuning("qres", 0)
    run_case(c, knn, tr, lab, te, 12, 0, 6)
    assert c.last_kernel_name() == "cand_s3_kernel<8,true,true>"
    c.close()


def test_nonfinite_inputs(knn):
    """NaN / inf: a train set holding one is refused (host and device entry
    points; the reference's distances would be undefined for every query);
    a query holding one gets label -1 and KNN_FLAG_NONFINITE with no
    neighbours, and every other query of the batch is unaffected."""
    import torch
    rng = np.random.default_rng(23)
    tr, lab, te = _mix(rng, 3000, 80, 32, 4)
    c = knn.Classifier(0)
    for bad in (np.nan, np.inf, -np.inf):
        t2 = tr.copy()
        t2[1234, 7] = bad
        with pytest.raises(knn.KnnError, match="non-finite"):
            c.set_train(t2, lab, 4)
        dev = torch.device("cuda", 0)
        Xd, Ld = torch.from_numpy(t2).to(dev), torch.from_numpy(lab).to(dev)
        with pytest.raises(knn.KnnError, match="non-finite"):
            c.set_train_device(Xd.data_ptr(), Ld.data_ptr(), 3000, 32, 4, keep=(Xd, Ld))
    dev = torch.device("cuda", 0)
    Xd, Ld = torch.from_numpy(tr).to(dev), torch.from_numpy(lab).to(dev)
    Ld[17] = 4  # label out of range, checked on the device
    with pytest.raises(knn.KnnError, match="labels outside"):
        c.set_train_device(Xd.data_ptr(), Ld.data_ptr(), 3000, 32, 4, keep=(Xd, Ld))
    te2 = te.copy()
    te2[3, 0] = np.nan
    te2[40, 31] = np.inf
    for prec in (knn.PRECISION_AUTO, knn.PRECISION_FP32, knn.PRECISION_FP16):
        c.set_precision(prec)
        c.set_train(tr, lab, 4)
        got, idx, dist, flags = c.classify(te2, 5, knn.L2, return_neighbors=True)
        bad = np.array([3, 40])
        assert (got[bad] == -1).all() and (flags[bad] & knn.FLAG_NONFINITE).all()
        assert (idx[bad] == -1).all() and np.isnan(dist[bad]).all()
        ok = np.setdiff1d(np.arange(te2.shape[0]), bad)
        want, widx, wdist = oracle.knn(tr, lab, te2[ok], 5, True, 4, n_out=5)
        np.testing.assert_array_equal(got[ok], want)
        assert_neighbors_match(idx[ok], dist[ok], widx, wdist, flags[ok])
    c.close()


def test_rescan_paths_large_d(clf, knn):
    """d > 256: uncertified queries go through the device-driven fast rescan
    (fp32 filter reading the rows in place) and, with 400 duplicates of the
    nearest row (more rows within reach than the fast path keeps), the full
    exact scan; exact results either way."""
    rng = np.random.default_rng(29)
    tr, lab, te = _mix(rng, 3000, 64, 300, 4)
    tr[1000:1400] = tr[5]
    lab[1000:1400] = rng.integers(0, 4, 400)
    te[:16] = tr[5]
    got, want, flags = run_case(clf, knn, tr, lab, te, 9, 0, 4)
    assert clf.last_rescan_count() >= 16
    assert (flags[:16] & knn.FLAG_EXACT_RESCAN).all()
    # heavy near-ties without exact duplicates: fast rescan finishes them
    tr2 = tr.copy()
    tr2[1000:1400] = tr[5] + rng.standard_normal((400, 300)) * 1e-9
    run_case(clf, knn, tr2, lab, te, 9, 0, 4)


def test_rescan_totals_and_async(knn):
    """knn_classify_device returns without waiting for the device; the rescan
    counts and phase times of a batch of calls are read back afterwards, and
    the last call's outputs equal the host API's and the oracle's."""
    import torch
    rng = np.random.default_rng(31)
    tr, lab, te = _mix(rng, 4000, 256, 64, 5)
    tr[100:300] = tr[7]
    te[:8] = tr[7]
    dev = torch.device("cuda", 0)
    c = knn.Classifier(0)
    c.set_timing(True)
    c.set_train(tr, lab, 5)
    Q = torch.from_numpy(te).to(dev)
    out = torch.empty(256, dtype=torch.int32, device=dev)
    fl = torch.empty(256, dtype=torch.int32, device=dev)
    c.rescan_totals(reset=True)
    c.timing_totals(reset=True)
    for _ in range(5):
        c.classify_device(Q.data_ptr(), 256, 10, knn.L2, out.data_ptr(), d_flags=fl.data_ptr())
    failed, full = c.rescan_totals(reset=True)
    ms, calls = c.timing_totals(reset=True)
    assert calls == 5 and all(v >= 0 for v in ms) and ms[1] > 0
    assert failed >= 5 * 8 and 0 <= full <= failed
    assert c.last_kernel_name().startswith("cand_")
    got, idx, dist, flags = c.classify(te, 10, knn.L2, return_neighbors=True)
    np.testing.assert_array_equal(out.cpu().numpy(), got)
    np.testing.assert_array_equal(fl.cpu().numpy(), flags)
    want, widx, wdist = oracle.knn(tr, lab, te, 10, True, 5, n_out=10)
    tv = (flags & knn.FLAG_TIE_VOTE) != 0
    TIE_VOTES["tie_vote"] += int(tv.sum())
    TIE_VOTES["tie_vote_label_differs"] += int((got[tv] != want[tv]).sum())
    np.testing.assert_array_equal(got, want)
    assert_neighbors_match(idx, dist, widx, wdist, flags)
    c.close()


def test_group_two_gpus(knn):
    """knn_group with 2 GPUs (RCCL broadcast / all-gather / all-reduce over
    xGMI): both modes and the sharded normalisation against the oracle, with
    ragged shards.  Skipped on a one-GPU box."""
    if knn.lib().knn_device_count() < 2:
        pytest.skip("needs 2 GPUs")
    rng = np.random.default_rng(37)
    tr, lab, te = _mix(rng, 5001, 333, 48, 6, grid=None)
    va = te[::2].copy()
    t_n, e_n, v_n = tr.copy(), te.copy(), va.copy()
    oracle.normalize(t_n, e_n, v_n)
    g = knn.Group([0, 1], 0)
    g.normalize(tr, te, va)
    for a, b in ((tr, t_n), (te, e_n), (va, v_n)):
        assert a.tobytes() == b.tobytes()
    want, widx, wdist = oracle.knn(tr, lab, te, 7, True, 6, n_out=7)
    g.set_train(tr, lab, 6)
    got, idx, dist, flags = g.classify(te, 7, knn.L2, return_neighbors=True)
    np.testing.assert_array_equal(got, want)
    assert_neighbors_match(idx, dist, widx, wdist, flags)
    g.close()
    g = knn.Group([0, 1], 1)
    g.set_train(tr, lab, 6)
    got, idx, dist, flags = g.classify(te, 7, knn.L2, return_neighbors=True)
    np.testing.assert_array_equal(got, want)
    assert_neighbors_match(idx, dist, widx, wdist, flags)
    g.close()
