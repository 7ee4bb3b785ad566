#!/usr/bin/env python3
"""In-process A/B timing of candidate-kernel variants on cfg2-shaped data
(interleaved rounds, medians; cdna_hip_programming.md §5.4 rule 24).
Usage: python tools/tune.py [--rounds 5] [--n 1000000 --m 10000 --d 128 --k 10]
Variants: "prec:R:S[:ablate[:nw]]" e.g. auto:0:0 fp32:8:0 auto:8:0:1:8
(prec: auto | fp32 | bf16x3 | m16 = bf16x3 on the 16x16x32 MFMA layout | fp16
 = fp16 on the 16x16x32 MFMA)
(ablate bits: 1 = no staging loads, 2 = no selection epilogue; timing only;
nw = waves per candidate workgroup, 0 auto / 4 / 8)
Extra tuning keys after a comma, e.g. "fp16:0:0,mfma16=1" (keys listed in
`defaults` and not named by a variant are reset to automatic).

Parity gate (before any time is logged): the first call of every variant
returns its neighbour distances, and --gate queries (default 256, spread over
the batch) must hold the k smallest distances over ALL train rows (the
independent fp64 brute force of tests/test_gpu_fullsize.py) and every label
must equal the first variant's; a variant that fails exits non-zero with no
timing line.  (The oracle half of the gate -- 8 queries bit for bit -- is
tests/test_gpu_gate.py, which tools/gpu_round.sh runs on every library
variant before its A/B.)  Round 5's r5ai variant, which skipped query loads,
would have stopped here instead of being logged as a gain."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from test_gpu_fullsize import brute_force_kdist  # noqa: E402  (torch fp64 GEMM, not the oracle)

DEFAULTS = {"gk": -1, "s3q": -1, "xhswz": 1, "i8": -1, "i8w": -1, "seed": 0, "ophase": -1, "s3gq": 0,
            "gg": -1, "qblk": 0, "i8resc": -1, "qres": -1}


def apply_variant(knn, clf, v):
    """Set a variant string's precision and tuning keys on clf; returns its
    ablation bits."""
    prec = {"auto": knn.PRECISION_AUTO, "fp32": knn.PRECISION_FP32, "bf16x3": knn.PRECISION_BF16X3,
            "m16": knn.PRECISION_BF16X3, "fp16": knn.PRECISION_FP16}
    base, *extra = v.split(",")
    kv = dict(DEFAULTS)
    for e in extra:
        key, val = e.split("=")
        kv[key] = int(val)
    for key, val in kv.items():
        clf.set_tuning(key, val)
    parts = base.split(":")
    p, R, S = parts[:3]
    abl = int(parts[3]) if len(parts) > 3 else 0
    nw = int(parts[4]) if len(parts) > 4 else 0
    clf.set_tuning("nw", nw)
    clf.set_precision(prec[p])
    clf.set_tuning("mfma16", 1 if p == "m16" else (0 if p == "bf16x3" else -1))
    clf.set_tuning("R", int(R))
    clf.set_tuning("S", int(S))
    clf.set_tuning("ablate", abl)
    return abl


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--m", type=int, default=10_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--data", default="grid", choices=("grid", "continuous"))
    ap.add_argument("--order", type=int, default=-1,
                    help="region order of the train layout (tuning key 'order', set before set_train)")
    ap.add_argument("--nblk", type=int, default=-1,
                    help="norm blocks of the train layout (tuning key 'nblk', set before set_train)")
    ap.add_argument("--gate", type=int, default=256,
                    help="queries checked for optimality per variant before timing (0: off)")
    ap.add_argument("variants", nargs="*", default=["auto:0:0", "auto:4:0", "auto:8:0", "fp32:0:0"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    knn = bench.load_knn()
    X, lab, Q, _ = bench.synth(a.n, a.m, a.d, 10, 1234, 5678, dev, data=a.data)
    clf = knn.Classifier(0)
    clf.set_tuning("order", a.order)
    clf.set_tuning("nblk", a.nblk)
    clf.set_train_device(X.data_ptr(), lab.data_ptr(), a.n, a.d, 10, keep=(X, lab))
    clf.set_timing(True)
    out = torch.empty(a.m, dtype=torch.int32, device=dev)
    ref = None
    res = {v: [] for v in a.variants}
    tot = {}
    ph = {}
    info = {}
    # int8 selection counts of a KNN_COUNT_SEL build (knn_cand_res.hip), per variant
    try:
        cnt_fn = getattr(knn.lib(), "_ZN4knnk16res_sel_countersEPyi")
    except AttributeError:
        cnt_fn = None
    selc = {}
    cbuf = (ctypes.c_ulonglong * 8)()
    gq = np.unique(np.linspace(0, a.m - 1, min(a.gate, a.m)).astype(np.int64)) if a.gate > 0 else None
    idx = torch.empty((a.m, a.k), dtype=torch.int64, device=dev)
    dist = torch.empty((a.m, a.k), dtype=torch.float64, device=dev)
    bf = None
    for r in range(a.rounds + 1):
        for v in a.variants:
            abl = apply_variant(knn, clf, v)
            if cnt_fn is not None:
                cnt_fn(cbuf, 1)
            if r == 0 and gq is not None:
                clf.classify_device(Q.data_ptr(), a.m, a.k, knn.L2, out.data_ptr(), idx.data_ptr(),
                                    dist.data_ptr())
            else:
                clf.classify_device(Q.data_ptr(), a.m, a.k, knn.L2, out.data_ptr())
            clf.sync()
            if r == 0 and gq is not None and not (abl & 27):
                # parity gate (timing-only ablations, bits 1/2/8/16, give invalid results)
                if bf is None:
                    bf = brute_force_kdist(X, Q[gq], a.k)
                got = dist.cpu().numpy()[gq]
                bad = np.nonzero(~np.isclose(got, bf, rtol=1e-10, atol=0).all(1))[0]
                if bad.size or (ref is not None and not torch.equal(ref, out)):
                    print("PARITY GATE FAILED for %s: %d of %d gate queries miss a true neighbour "
                          "(e.g. query %s), labels equal to the first variant: %s" %
                          (v, bad.size, gq.size, gq[bad[:4]], ref is None or bool(torch.equal(ref, out))))
                    sys.exit(3)
                print("parity gate %s: %d queries optimal, labels %s" %
                      (v, gq.size, "reference" if ref is None else "= first variant"))
            if cnt_fn is not None and r > 0:
                cnt_fn(cbuf, 1)
                if any(cbuf):
                    selc[v] = list(cbuf)
            if r == 0:
                if ref is None and not (abl & 27):
                    ref = out.clone()
                info[v] = (clf.last_geometry(), clf.last_rescan_count(),
                           ref is not None and bool(torch.equal(ref, out)))
                continue
            res[v].append(clf.last_phase_ms(knn.PHASE_CANDIDATE))
            tot.setdefault(v, []).append(sum(clf.last_phase_ms(p) for p in range(4)))
            ph.setdefault(v, []).append([clf.last_phase_ms(p) for p in range(4)])
    flops = 2.0 * a.n * a.d * a.m
    for v in a.variants:
        if v in selc:
            c = selc[v]
            print("%-14s int8 selection per launch: calls %d, lane passes %.4f, wave passes %.4f, "
                  "inserts per lane-call %.4f" % (v, c[0], c[1] / max(1, c[0]), c[2] * 64 / max(1, c[0]),
                                                 c[3] / max(1, c[0])))
            if c[4]:
                print("%-14s seed-free bound: sub-tile tests %d (wave), passing %.4f; exact wave passes "
                      "per test %.4f" % (v, c[4], c[5] / c[4], c[2] / c[4]))
            if c[6]:
                print("%-14s   first two staged tiles: %d tests (%.3f of all), passing %.4f -> %.3f of "
                      "all passing tests" % (v, c[6], c[6] / c[4], c[7] / c[6], c[7] / max(1, c[5])))
        ms = np.median(res[v])
        print("%-14s cand %8.3f ms (min %8.3f)  %7.1f TF/s  all phases %8.3f ms  %s rescans=%d "
              "same_labels=%s" % (v, ms, np.min(res[v]), flops / ms / 1e9, np.median(tot[v]),
                                  info[v][0], info[v][1], info[v][2]))
        print("%-14s phases ms: prep %.3f cand %.3f rerank %.3f rescan %.3f" %
              ((v,) + tuple(np.median(np.array(ph[v]), axis=0))))


if __name__ == "__main__":
    main()
