"""Runs the REFERENCE program (oracle/_ref, built by build_ref.py from
/root/reference/knn_mpi.cpp) under mpirun on host cores: the CPU baseline
leg of bench.py and a test helper.  TEST INFRASTRUCTURE ONLY -- nothing in
the product imports this.

Inputs are written in the reference's CSV formats (cpp:154-222: train/val
rows "label,x1,..,xd", test rows "x1,..,xd").  The values are 8-bit grid
values k/256 (SIFT-like features scaled into [0,1)), printed with their exact
8-digit decimal expansion, so the reference's atof reads back the identical
fp64 values the GPU path classified."""
import os
import re
import subprocess
import time

import numpy as np

MPIRUN = "/opt/conda/bin/mpirun"
_TABLE = np.array([("0.%08d" % (k * 390625)).encode() for k in range(256)], dtype="S10")


def grid_values(codes):
    """fp64 values of 8-bit grid codes (exact)."""
    return codes.astype(np.float64) / 256.0


def write_grid_csv(path, codes, labels=None, chunk=1 << 16):
    """codes: uint8 [rows][dim] -> CSV of k/256 values (10 bytes each)."""
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    rows, dim = codes.shape
    tb = np.frombuffer(_TABLE.tobytes(), dtype=np.uint8).reshape(256, 10)
    with open(path, "wb") as f:
        for r0 in range(0, rows, chunk):
            c = codes[r0:r0 + chunk]
            n = c.shape[0]
            body = np.empty((n, dim, 11), dtype=np.uint8)
            body[:, :, :10] = tb[c]
            body[:, :, 10] = ord(",")
            body[:, -1, 10] = ord("\n")
            if labels is None:
                f.write(body.tobytes())
            else:
                lab = np.char.add(labels[r0:r0 + n].astype(str), ",").astype("S")
                width = max(len(x) for x in lab)
                pre = np.full((n, width), ord(" "), dtype=np.uint8)
                lb = np.frombuffer(lab.astype("S%d" % width).tobytes(), dtype=np.uint8)
                pre[:] = lb.reshape(n, width)
                pre[pre == 0] = ord(" ")  # shorter labels: left-aligned, blank padded
                # atoi skips leading blanks only; keep the label first and pad after the comma
                line = np.concatenate([pre, body.reshape(n, dim * 11)], axis=1)
                f.write(line.tobytes())


def run_reference(exe, workdir, nprocs, timeout=600):
    """Runs the reference binary in workdir (which holds its input CSVs) and
    returns (test labels, test-loop seconds or None, running time seconds)."""
    t0 = time.perf_counter()
    out = subprocess.run([MPIRUN, "-np", str(nprocs), exe], cwd=workdir, capture_output=True,
                         text=True, timeout=timeout)
    wall = time.perf_counter() - t0
    if out.returncode != 0:
        raise RuntimeError("reference failed (%d): %s" % (out.returncode, out.stderr[-2000:]))
    m = re.search(r"KNN_TEST_LOOP_SECONDS ([0-9.eE+-]+)", out.stdout)
    r = re.search(r"Running time is ([0-9.eE+-]+) second", out.stdout)
    labels = np.loadtxt(os.path.join(workdir, "Test_label.csv"), dtype=np.int64, ndmin=1)
    return (labels, float(m.group(1)) if m else None, float(r.group(1)) if r else wall)
