"""Parity gate of the A/B tooling (tools/gpu_round.sh runs it on every
library variant before timing it; with no KNN_GATE it checks the default
build's AUTO path as part of the GPU suite).

KNN_GATE: tune.py variant strings separated by ';' (e.g. "auto:0:0;auto:0:0,i8w=0"),
KNN_GATE_N / KNN_GATE_M / KNN_GATE_D / KNN_GATE_K / KNN_GATE_DATA: the workload
(default cfg2: 1M x 10k, d = 128, k = 10, bench.synth's 8-bit grid data;
"continuous" for its min-max normalised form, the fp16 path).  Per variant:
  * the oracle (oracle/knn_oracle.cpp, pinned to the reference's own
    outputs) bit for bit on 8 queries -- labels, fp64 distances, indices
    except inside exact ties;
  * optimality on 256 queries against the independent fp64 brute force;
  * labels of the whole batch equal to the first variant's."""
import os
import sys

import numpy as np
import pytest
import torch

import bench
from test_gpu_fullsize import check_optimal, check_oracle

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_variant_parity_gate():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from tune import apply_variant
    knn = bench.load_knn()
    if knn.lib().knn_device_count() < 1:
        pytest.fail("no HIP device visible: the KNN path has no CPU fallback")
    variants = [v for v in os.environ.get("KNN_GATE", "auto:0:0").split(";") if v]
    n = int(os.environ.get("KNN_GATE_N", 1_000_000))
    m = int(os.environ.get("KNN_GATE_M", 10_000))
    d = int(os.environ.get("KNN_GATE_D", 128))
    k = int(os.environ.get("KNN_GATE_K", 10))
    data = os.environ.get("KNN_GATE_DATA", "grid")
    X, lab, Q, _ = bench.synth(n, m, d, 10, 1234, 5678, DEV, data=data)
    torch.cuda.synchronize()
    clf = knn.Classifier(0)
    clf.set_tuning("order", int(os.environ.get("KNN_GATE_ORDER", -1)))  # the train layout
    clf.set_train_device(X.data_ptr(), lab.data_ptr(), n, d, 10, keep=(X, lab))
    lab_all = lab.cpu().numpy()
    first = None
    for v in variants:
        abl = apply_variant(knn, clf, v)
        assert not (abl & 27), "timing-only ablations give invalid results: not gateable (%s)" % v
        out = torch.empty(m, dtype=torch.int32, device=DEV)
        idx = torch.empty((m, k), dtype=torch.int64, device=DEV)
        dist = torch.empty((m, k), dtype=torch.float64, device=DEV)
        clf.classify_device(Q.data_ptr(), m, k, knn.L2, out.data_ptr(), idx.data_ptr(), dist.data_ptr())
        clf.sync()
        got, gi, gd = out.cpu().numpy(), idx.cpu().numpy(), dist.cpu().numpy()
        check_optimal(X, Q, k, gd, np.unique(np.linspace(0, m - 1, 256).astype(np.int64)))
        check_oracle(X, lab_all, Q, k, got, gi, gd, np.arange(0, m, m // 8)[:8])
        if first is None:
            first = got
        np.testing.assert_array_equal(got, first, err_msg="labels of %s differ from %s" % (v, variants[0]))
        print("gate %s (%s data): 256 queries optimal, 8 = oracle, %s" % (v, data, clf.last_kernel_name()))
    clf.close()
