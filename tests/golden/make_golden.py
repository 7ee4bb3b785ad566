#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE itself.

Runs only in the build container (needs /root/reference and MPICH); the GPU
box and the test suite only read the committed .npz files.

For every fixture spec below:
  1. write the three CSV inputs with tests/datagen.py (deterministic; the
     sha256 of the bytes is stored so tests can prove they regenerated the
     same inputs),
  2. build /root/reference/knn_mpi.cpp with that spec's constants via
     oracle/build_ref.py (instrumented to dump the first K+2 sorted records
     per query -- see oracle/ref_dump.h),
  3. run it with /opt/conda/bin/mpirun -np P in a scratch directory,
  4. store: Test_label.csv (as int32), the `accuracy = ` line, and the dumped
     neighbour idx/dis for test and validation queries.
A fixture is data: inputs are stored as their generator spec + hash, outputs
as arrays.  No reference source text is stored.
"""
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import datagen  # noqa: E402
from build_ref import build_ref  # noqa: E402

MPIRUN = "/opt/conda/bin/mpirun"
REF_NAMES = ("mnist_train.csv", "mnist_validation.csv", "mnist_test.csv")  # cpp:117-119

# name -> spec.  Keys match the reference's constant names (cpp:108-116).
SPECS = {
    "f1_cfg1": dict(kind="gauss", seed=11, dim=16, K=5, N_train=10000, N_test=1000,
                    N_val=1000, class_cnt=3, np=4),
    "f2_vote_ties": dict(kind="noisy", seed=12, dim=8, K=4, N_train=2000, N_test=400,
                         N_val=400, class_cnt=4, np=4),
    "f3_l1": dict(kind="gauss", seed=13, dim=12, K=7, N_train=4000, N_test=400, N_val=400,
                  class_cnt=5, Euclidean_distance=False, np=4),
    "f4_normedge": dict(kind="normedge", seed=14, dim=10, K=5, N_train=2000, N_test=200,
                        N_val=200, class_cnt=3, np=4),
    "f5_csv_crlf": dict(kind="gauss", seed=15, dim=6, K=3, N_train=1000, N_test=100,
                        N_val=100, class_cnt=2, np=4, crlf=True, trailing_newline=False),
    "f6_int_ties": dict(kind="int", seed=16, dim=16, K=10, N_train=4000, N_test=400,
                        N_val=400, class_cnt=5, np=4),
    "f7_nonorm_noval": dict(kind="gauss", seed=17, dim=20, K=9, N_train=3000, N_test=300,
                            N_val=300, class_cnt=6, Normalize=False, Validation=False, np=2),
    "f8_sorted_train": dict(kind="sorted", seed=19, dim=32, K=20, N_train=8000, N_test=500,
                            N_val=500, class_cnt=4, np=4),
    "f9_k100": dict(kind="gauss", seed=20, dim=64, K=100, N_train=5000, N_test=300,
                    N_val=300, class_cnt=10, np=4),
    "f10_l1_int": dict(kind="int", seed=21, dim=24, K=6, N_train=3000, N_test=300,
                       N_val=300, class_cnt=4, Euclidean_distance=False, np=4),
    # The reference's own default configuration (cpp:108-116: MNIST shape).
    "f11_mnist_shape": dict(kind="gauss", seed=18, dim=784, K=50, N_train=60000,
                            N_test=10000, N_val=10000, class_cnt=10, np=8,
                            max_dump_queries=400),
}

REF_KEYS = ("dim", "K", "N_train", "N_test", "N_val", "class_cnt", "Euclidean_distance",
            "Normalize", "Validation")


def full_spec(spec):
    s = dict(Euclidean_distance=True, Normalize=True, Validation=True, crlf=False,
             trailing_newline=True, max_dump_queries=None)
    s.update(spec)
    return s


def parse_dumps(workdir, tag, nq, ndump, max_q):
    nq_keep = nq if max_q is None else min(nq, max_q)
    idx = np.full((nq_keep, ndump), -1, np.int64)
    dis = np.full((nq_keep, ndump), np.inf, np.float64)
    seen = np.zeros(nq_keep, bool)
    for fn in sorted(os.listdir(workdir)):
        if not fn.startswith("dump_%s_" % tag):
            continue
        with open(os.path.join(workdir, fn)) as f:
            for line in f:
                parts = line.split()
                q = int(parts[0])
                if q >= nq_keep:
                    continue
                for t, p in enumerate(parts[1:]):
                    a, b = p.split(":")
                    idx[q, t] = int(a)
                    dis[q, t] = float(b)
                seen[q] = True
    assert seen.all(), "missing dumped queries for " + tag
    return idx, dis


def make(name, spec, force=False):
    out = os.path.join(HERE, name + ".npz")
    if os.path.exists(out) and not force:
        print("exists", out)
        return out
    s = full_spec(spec)
    cfg = {k: s[k] for k in REF_KEYS}
    exe = build_ref(cfg, instrument=True)
    ndump = min(s["K"] + 2, s["N_train"])
    with tempfile.TemporaryDirectory() as wd:
        _, sha = datagen.write_csvs(wd, s, names=REF_NAMES, crlf=s["crlf"],
                                    trailing_newline=s["trailing_newline"])
        env = dict(os.environ, KNN_DUMP_N=str(ndump))
        r = subprocess.run([MPIRUN, "-np", str(s["np"]), exe], cwd=wd, env=env,
                           capture_output=True, text=True, check=True)
        acc_line = ""
        m = re.search(r"^accuracy = (.*)$", r.stdout, re.M)
        if m:
            acc_line = m.group(0)
        test_labels = np.loadtxt(os.path.join(wd, "Test_label.csv"), dtype=np.int64,
                                 ndmin=1).astype(np.int32)
        t_idx, t_dis = parse_dumps(wd, "test", s["N_test"], ndump, s["max_dump_queries"])
        arrays = dict(spec=np.array(json.dumps(s)), csv_sha256=np.array(sha),
                      test_labels=test_labels, accuracy_line=np.array(acc_line),
                      test_nbr_idx=t_idx, test_nbr_dist=t_dis)
        if s["Validation"]:
            v_idx, v_dis = parse_dumps(wd, "val", s["N_val"], ndump, s["max_dump_queries"])
            arrays.update(val_nbr_idx=v_idx, val_nbr_dist=v_dis)
    np.savez_compressed(out, **arrays)
    print("wrote", out, acc_line, r.stdout.strip().splitlines()[-1])
    return out


if __name__ == "__main__":
    names = sys.argv[1:] or list(SPECS)
    force = os.environ.get("FORCE") == "1"
    for n in names:
        make(n, SPECS[n], force=force)
