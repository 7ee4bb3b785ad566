#!/usr/bin/env python3
"""Build the REFERENCE program (/root/reference/knn_mpi.cpp) into oracle/_ref/.

TEST INFRASTRUCTURE ONLY -- the product never loads anything built here.

The reference has no flags: its configuration is the constant block at
cpp:108-119 (dim, K, N_train, N_test, N_val, class_cnt, Euclidean_distance,
Normalize, Validation).  This recipe streams the source from where it lies
under /root/reference through `sed` (substituting those constants, and
optionally adding the neighbour-dump instrumentation described in
oracle/ref_dump.h) straight into the image's MPICH compiler wrapper
(/opt/conda/bin/mpicxx, MPICH 3.3.2, with MPICH_CXX=g++ 11.4, -O2).  No copy
of the reference source is written anywhere; only the binary lands in
oracle/_ref/ (git-ignored).

Usage (python):  build_ref(cfg, instrument=True, timing=False) -> path to binary
(timing=True adds a timer around the test-query loop, see sed_script)
CLI:             python oracle/build_ref.py dim=16 K=5 N_train=10000 ...
"""
import hashlib
import os
import subprocess
import sys

REF = "/root/reference/knn_mpi.cpp"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_ref")
MPICXX = "/opt/conda/bin/mpicxx"

DEFAULTS = dict(dim=784, K=50, N_train=60000, N_test=10000, N_val=10000,
                class_cnt=10, Euclidean_distance=True, Normalize=True,
                Validation=True)


def _c(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(int(v))


def sed_script(cfg, instrument, timing=False):
    s = []
    # cpp:108-116 -- the constant block (each line is "\t<name> = <value>; //...").
    for name, default in DEFAULTS.items():
        s += ["-e", r"s/^\(\s*%s\) = %s;/\1 = %s;/" % (name, _c(default), _c(cfg[name]))]
    if instrument:
        s += ["-e", r"s/^\(\s*\)int label;/\1int label; int idx;/",            # cpp:20
              "-e", r"s/d1\[j\]\.label = Train_label\[j\];/&  d1[j].idx = j;/",  # cpp:319
              "-e", r"s/d2\[j\]\.label = Train_label\[j\];/&  d2[j].idx = j;/",  # cpp:362
              "-e", r's/sort(d1, d1 + N_train, Comp);/& KNN_DUMP(d1, "val", myid * batch_val + i);/',
              "-e", r's/sort(d2, d2 + N_train, Comp);/& KNN_DUMP(d2, "test", myid * batch_test + i);/']
    if timing:
        # wall time of the test-query loop alone (cpp:352-382), max over ranks
        # via barriers, printed by rank 0: the compute-only rate of the
        # reference, without its CSV parse and MPI_Bcast of the train set
        s += ["-e", r"s/^\(\s*\)train_data_dis\* d2;/\1MPI_Barrier(MPI_COMM_WORLD); "
                    r"double knn_tq0 = MPI_Wtime(); train_data_dis* d2;/",
              "-e", r"s/^\(\s*\)MPI_Gather(Test_label_buffer/\1MPI_Barrier(MPI_COMM_WORLD); "
                    r"if (!myid) printf(\"KNN_TEST_LOOP_SECONDS %.6f\\n\", MPI_Wtime() - knn_tq0); "
                    r"MPI_Gather(Test_label_buffer/"]
    return s


def ref_available():
    return os.path.exists(REF) and os.path.exists(MPICXX)


def build_ref(cfg=None, instrument=True, force=False, timing=False):
    full = dict(DEFAULTS)
    full.update(cfg or {})
    flags = bytes([instrument]) + (b"t" if timing else b"")
    tag = hashlib.sha1(repr(sorted(full.items())).encode() + flags).hexdigest()[:12]
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "knn_ref_" + tag)
    if os.path.exists(exe) and not force:
        return exe
    if not ref_available():
        raise FileNotFoundError("reference source or MPICH wrapper missing")
    sed = subprocess.run(["sed"] + sed_script(full, instrument, timing) + [REF],
                         check=True, capture_output=True)
    src = sed.stdout
    # every substitution must have hit exactly once
    for name in DEFAULTS:
        needle = ("%s = %s;" % (name, _c(full[name]))).encode()
        if src.count(needle) < 1:
            raise RuntimeError("constant substitution failed for " + name)
    if instrument and src.count(b"KNN_DUMP(") != 2:
        raise RuntimeError("instrumentation substitution failed")
    if timing and src.count(b"KNN_TEST_LOOP_SECONDS") != 1:
        raise RuntimeError("timing substitution failed")
    env = dict(os.environ, MPICH_CXX="g++")
    cmd = [MPICXX, "-O2", "-w", "-x", "c++"]
    if instrument:
        cmd += ["-include", os.path.join(HERE, "ref_dump.h")]
    cmd += ["-", "-o", exe]
    subprocess.run(cmd, input=src, check=True, env=env)
    return exe


if __name__ == "__main__":
    cfg = {}
    for a in sys.argv[1:]:
        k, v = a.split("=")
        cfg[k] = (v.lower() == "true") if v.lower() in ("true", "false") else int(v)
    print(build_ref(cfg))
