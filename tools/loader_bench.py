#!/usr/bin/env python3
"""End-to-end timing of the drop-in driver (bin/knn_mpi_amd) on cfg2-sized
CSV files -- 1M x 128 train rows + 10k test rows, the reference's formats
(cpp:154-222) -- against the reference program (oracle/_ref, compiled from
/root/reference/knn_mpi.cpp by oracle/build_ref.py) on the same files.

Prints one JSON line: the driver's per-phase seconds (--timings: csv parse,
normalisation, set_train, test pass, output) and "Running time", the
reference's "Running time" and test-loop seconds (its CSV parse + MPI_Bcast
= the difference), both runs' Test_label.csv identical or not.
Usage: python tools/loader_bench.py [--n 1000000] [--m 10000] [--ref-queries 512]"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import build_ref  # noqa: E402
import ref_runner  # noqa: E402

DRIVER = os.path.join(ROOT, "-mpi-knn-_amd", "bin", "knn_mpi_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--m", type=int, default=10_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--ref-queries", type=int, default=512,
                    help="test rows the reference classifies (its loop is ~8 ms/query/rank)")
    a = ap.parse_args()
    rng = np.random.default_rng(1)
    centres = rng.integers(40, 216, (a.classes, a.d))
    lab = rng.integers(0, a.classes, a.n).astype(np.int32)
    codes = np.clip(centres[lab] + rng.normal(0, 24, (a.n, a.d)), 0, 255).astype(np.uint8)
    qlab = rng.integers(0, a.classes, a.m)
    qcodes = np.clip(centres[qlab] + rng.normal(0, 24, (a.m, a.d)), 0, 255).astype(np.uint8)
    wd = tempfile.mkdtemp(prefix="knn_loader_", dir=os.environ.get("TMPDIR", "/tmp"))
    out = {"workload": "%d train x %d test rows, d=%d, k=%d (8-bit grid values, 10-byte tokens)"
                       % (a.n, a.m, a.d, a.k)}
    try:
        t0 = time.perf_counter()
        ref_runner.write_grid_csv(os.path.join(wd, "mnist_train.csv"), codes, lab)
        ref_runner.write_grid_csv(os.path.join(wd, "mnist_test.csv"), qcodes)
        out["csv_write_s"] = time.perf_counter() - t0
        out["train_csv_bytes"] = os.path.getsize(os.path.join(wd, "mnist_train.csv"))
        # the driver, the reference's constants as flags (Normalize and
        # Validation off, like the bench's reference leg)
        args = [DRIVER, "--dim", str(a.d), "--K", str(a.k), "--N_train", str(a.n), "--N_test",
                str(a.m), "--N_val", "0", "--class_cnt", str(a.classes), "--Normalize", "false",
                "--Validation", "false", "--timings"]
        r = subprocess.run(args, cwd=wd, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise RuntimeError(r.stderr[-2000:])
        out["driver_phases_s"] = {m.group(1): float(m.group(2)) for m in
                                  re.finditer(r"\[knn_mpi_amd\] (\w+)\s+([0-9.]+) s", r.stderr)}
        out["driver_running_time_s"] = float(re.search(r"Running time is ([0-9.eE+-]+)",
                                                       r.stdout).group(1))
        drv = np.loadtxt(os.path.join(wd, "Test_label.csv"), dtype=np.int64)
        # the reference on the first ref-queries test rows (same train file)
        if build_ref.ref_available() or os.path.isdir(os.path.join(ROOT, "oracle", "_ref")):
            P = 16
            cfg = dict(dim=a.d, K=a.k, N_train=a.n, N_test=a.ref_queries, N_val=a.ref_queries,
                       class_cnt=a.classes, Validation=False, Normalize=False,
                       Euclidean_distance=True)
            exe = build_ref.build_ref(cfg, instrument=False, timing=True)
            sub = os.path.join(wd, "ref")
            os.makedirs(sub)
            os.link(os.path.join(wd, "mnist_train.csv"), os.path.join(sub, "mnist_train.csv"))
            ref_runner.write_grid_csv(os.path.join(sub, "mnist_test.csv"), qcodes[:a.ref_queries])
            labels, loop_s, run_s = ref_runner.run_reference(exe, sub, P)
            out["reference"] = {"ranks": P, "running_time_s": run_s, "test_loop_s": loop_s,
                                "csv_parse_and_bcast_s": run_s - loop_s,
                                "queries": a.ref_queries}
            out["labels_equal_on_reference_queries"] = bool(
                (labels == drv[:a.ref_queries]).all())
    finally:
        shutil.rmtree(wd, ignore_errors=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
