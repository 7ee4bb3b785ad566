#!/usr/bin/env python3
"""Probe: how much does the ORDER in which a split streams the train rows
change the int8 candidate pass?  Queries all from one cluster of the cfg2
mixture; train rows (a) in generation order, (b) that cluster's rows first
(every split's stream starts on them: tight thresholds from the start),
(c) that cluster's rows last.  Same rows, same exact answers (checked);
only the candidate-pass time differs.  Usage: python tools/order_probe.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    knn = bench.load_knn()
    n, m, d, k, C = 1_000_000, 10_000, 128, 10, 10
    X, lab, Q, qlab = bench.synth(n, 12 * m, d, C, 1234, 5678, dev)
    Q = Q[qlab == 0][:m].contiguous()
    assert Q.shape[0] == m
    first = torch.argsort((lab != 0).to(torch.int32), stable=True)   # cluster 0 first
    last = torch.argsort((lab == 0).to(torch.int32), stable=True)    # cluster 0 last
    orders = {"generated": None, "cluster_first": first, "cluster_last": last}
    out = torch.empty(m, dtype=torch.int32, device=dev)
    res = {}
    ref = None
    for name, perm in orders.items():
        Xp = X if perm is None else X[perm].contiguous()
        Lp = lab if perm is None else lab[perm].contiguous()
        clf = knn.Classifier(0)
        clf.set_train_device(Xp.data_ptr(), Lp.data_ptr(), n, d, C, keep=(Xp, Lp))
        clf.set_timing(True)
        ts = []
        for r in range(6):
            clf.classify_device(Q.data_ptr(), m, k, knn.L2, out.data_ptr())
            clf.sync()
            if r:
                ts.append(clf.last_phase_ms(knn.PHASE_CANDIDATE))
        if ref is None:
            ref = out.clone()
        res[name] = (np.median(ts), bool(torch.equal(ref, out)), clf.last_rescan_count())
        clf.close()
        del Xp, Lp
    for name, (ms, same, resc) in res.items():
        print("%-14s cand %.3f ms  labels_equal=%s rescans=%d" % (name, ms, same, resc))


if __name__ == "__main__":
    main()
