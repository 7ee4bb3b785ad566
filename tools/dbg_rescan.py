#!/usr/bin/env python3
"""Which bench query fails certification on the int8 path, and why: its exact
fp64 neighbour distances around the W-th place (GPU brute force)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

dev = torch.device("cuda", 0)
knn = bench.load_knn()
n, m, d, k, C = 1_000_000, 10_000, 128, 10, 10
X, lab, Q, _ = bench.synth(n, m, d, C, 1234, 5678, dev)
clf = knn.Classifier(0)
clf.set_train_device(X.data_ptr(), lab.data_ptr(), n, d, C, keep=(X, lab))
out = torch.empty(m, dtype=torch.int32, device=dev)
flg = torch.empty(m, dtype=torch.int32, device=dev)
for i8 in (-1, 0):
    clf.set_tuning("i8", i8)
    clf.classify_device(Q.data_ptr(), m, k, knn.L2, out.data_ptr(), None, None, flg.data_ptr())
    clf.sync()
    bad = torch.nonzero(flg & 1).flatten().tolist()
    print("i8=%d path %d rescanned %s" % (i8, clf.last_candidate_path(), bad))
    for q in bad[:4]:
        d2 = ((X - Q[q]) ** 2).sum(1)
        v, i = torch.topk(d2, 40, largest=False)
        print(" q %d: exact d^2 (x 65536) of the 40 nearest:" % q,
              [round(float(x) * 65536, 3) for x in v], "idx", i[:14].tolist())
        print("   rows tied with the 11th:", int((d2 == v[10]).sum()), "with the 10th:",
              int((d2 == v[9]).sum()))
        print("   query min/max", float(Q[q].min()), float(Q[q].max()))
