"""Python mirror of the MI355X KNN classifier (ctypes over lib/libknn_amd.so).

The reference (Jason-Woo/-MPI-KNN-, knn_mpi.cpp) has no library API: its
interface is the constant block (cpp:108-119), the CSV formats and the
outputs.  `KnnConfig` carries those constants under the same names;
`Classifier` is the per-GPU hot path (set_train / classify); `run_driver`
reproduces the reference's main() end to end through the native drop-in
driver (bin/knn_mpi_amd) -- the product, not the reference program.

There is no CPU compute path: every call goes through the HIP library and
fails loudly (KnnError) when the library or the GPU is missing.
"""
import ctypes
import dataclasses
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libknn_amd.so")
# experiment builds (tools/build_variant.sh) are selected by file name under lib/
if os.environ.get("KNN_AMD_VARIANT"):
    LIB_PATH = os.path.join(HERE, "lib", "libknn_amd_%s.so" % os.environ["KNN_AMD_VARIANT"])
DRIVER_PATH = os.path.join(HERE, "bin", "knn_mpi_amd")

L2, L1 = 0, 1
FLAG_EXACT_RESCAN, FLAG_TIE_BOUNDARY, FLAG_TIE_VOTE, FLAG_TIE_ORDER = 1, 2, 4, 8
FLAG_NONFINITE, FLAG_TIE_REF, FLAG_TIE_PENDING = 16, 32, 64
EXPORTED = (
    "knn_version", "knn_last_error", "knn_device_count", "knn_create", "knn_destroy",
    "knn_set_train", "knn_set_train_device", "knn_classify", "knn_classify_device",
    "knn_search_partial_device", "knn_merge_vote_device", "knn_sync", "knn_last_rescan_count",
    "knn_group_create", "knn_group_destroy", "knn_group_set_train", "knn_group_classify",
    "knn_group_last_compute_seconds", "knn_set_timing", "knn_last_phase_ms",
    "knn_last_geometry", "knn_set_precision", "knn_last_candidate_path", "knn_set_tuning",
    "knn_minmax_device", "knn_normalize_device", "knn_normalize", "knn_group_normalize",
    "knn_timing_totals", "knn_rescan_totals", "knn_last_kernel_name", "knn_tie_totals",
    "knn_shard_distances_device", "knn_tie_resolve_device", "knn_group_transport",
    "knn_group_last_tie_count", "knn_group_set_precision", "knn_group_set_tuning",
)
GROUP_RCCL = 0x100  # knn_group_create mode flag: RCCL collectives also at one GPU
TRANSPORT_NONE, TRANSPORT_RCCL, TRANSPORT_LOOPBACK = 0, 1, 2
PRECISION_AUTO, PRECISION_FP32, PRECISION_BF16X3, PRECISION_FP16 = 0, 1, 2, 3
PHASE_PREP, PHASE_CANDIDATE, PHASE_RERANK, PHASE_RESCAN = 0, 1, 2, 3


class KnnError(RuntimeError):
    pass


@dataclasses.dataclass
class KnnConfig:
    """The reference's configuration constants (cpp:108-119), same defaults."""
    dim: int = 784
    K: int = 50
    N_train: int = 60000
    N_test: int = 10000
    N_val: int = 10000
    class_cnt: int = 10
    Euclidean_distance: bool = True
    Normalize: bool = True
    Validation: bool = True
    train_file_name: str = "mnist_train.csv"
    validation_file_name: str = "mnist_validation.csv"
    test_file_name: str = "mnist_test.csv"


def build(jobs=8):
    subprocess.run(["make", "-s", "-j%d" % jobs, "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise KnnError("HIP library not built: %s (run build())" % LIB_PATH)
    # PyTorch-ROCm bundles its own HIP/HSA runtime with the same sonames as
    # /opt/rocm's.  If torch is in the process, let it bring up its runtime
    # first so this library binds to the already-loaded one (two runtimes in
    # one process leave torch without devices).
    if "torch" in sys.modules:
        try:
            sys.modules["torch"].cuda.init()
        except Exception:
            pass
    L = ctypes.CDLL(LIB_PATH)
    P, i32, i64, f64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
    sig = {
        "knn_version": ([], ctypes.c_char_p),
        "knn_last_error": ([], ctypes.c_char_p),
        "knn_device_count": ([], ctypes.c_int),
        "knn_create": ([ctypes.POINTER(P), ctypes.c_int], ctypes.c_int),
        "knn_destroy": ([P], ctypes.c_int),
        "knn_set_train": ([P, P, P, i64, i32, i32], ctypes.c_int),
        "knn_set_train_device": ([P, P, P, i64, i32, i32, i64], ctypes.c_int),
        "knn_classify": ([P, P, i64, i32, i32, P, P, P, P], ctypes.c_int),
        "knn_classify_device": ([P, P, i64, i32, i32, P, P, P, P, P], ctypes.c_int),
        "knn_search_partial_device": ([P, P, i64, i32, i32, P, P, P, P], ctypes.c_int),
        "knn_merge_vote_device": ([P, P, P, P, i32, i64, i32, i32, i64, i64, P, P, P, P, P],
                                  ctypes.c_int),
        "knn_sync": ([P], ctypes.c_int),
        "knn_last_rescan_count": ([P], i64),
        "knn_group_create": ([ctypes.POINTER(P), ctypes.c_int, P, ctypes.c_int], ctypes.c_int),
        "knn_group_destroy": ([P], ctypes.c_int),
        "knn_group_set_train": ([P, P, P, i64, i32, i32], ctypes.c_int),
        "knn_group_classify": ([P, P, i64, i32, i32, P, P, P, P], ctypes.c_int),
        "knn_group_last_compute_seconds": ([P], f64),
        "knn_set_timing": ([P, ctypes.c_int], ctypes.c_int),
        "knn_last_phase_ms": ([P, ctypes.c_int], f64),
        "knn_last_geometry": ([P, ctypes.POINTER(i64)], ctypes.c_int),
        "knn_set_precision": ([P, ctypes.c_int], ctypes.c_int),
        "knn_last_candidate_path": ([P], ctypes.c_int),
        "knn_set_tuning": ([P, ctypes.c_char_p, i64], ctypes.c_int),
        "knn_minmax_device": ([P, P, i64, i32, P, P, i32, P], ctypes.c_int),
        "knn_normalize_device": ([P, P, i64, i32, P, P, P], ctypes.c_int),
        "knn_normalize": ([P, P, P, i32, i32, P, P], ctypes.c_int),
        "knn_group_normalize": ([P, P, P, i32, i32], ctypes.c_int),
        "knn_timing_totals": ([P, ctypes.POINTER(f64), ctypes.POINTER(i64), ctypes.c_int],
                              ctypes.c_int),
        "knn_rescan_totals": ([P, ctypes.POINTER(i64), ctypes.c_int], ctypes.c_int),
        "knn_last_kernel_name": ([P], ctypes.c_char_p),
        "knn_tie_totals": ([P, ctypes.POINTER(i64), ctypes.c_int], ctypes.c_int),
        "knn_shard_distances_device": ([P, P, P, i32, i32, P, P], ctypes.c_int),
        "knn_tie_resolve_device": ([P, P, i32, ctypes.POINTER(i64), i32, P, P, i32, P, P, P, P,
                                    P], ctypes.c_int),
        "knn_group_transport": ([P], ctypes.c_int),
        "knn_group_last_tie_count": ([P], i64),
        "knn_group_set_precision": ([P, ctypes.c_int], ctypes.c_int),
        "knn_group_set_tuning": ([P, ctypes.c_char_p, i64], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        raise KnnError("knn error %d: %s" % (rc, lib().knn_last_error().decode()))


def _ptr(a):
    return None if a is None else a.ctypes.data


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _set_arrays(sets):
    """Host sets (C-contiguous float64 [rows, d], normalised in place) ->
    (pointer array, rows array, nsets, d)."""
    sets = [s for s in sets if s is not None]
    if not sets:
        raise ValueError("no sets")
    d = sets[0].shape[1]
    for s in sets:
        if s.dtype != np.float64 or not s.flags["C_CONTIGUOUS"] or s.ndim != 2 or s.shape[1] != d:
            raise ValueError("sets must be C-contiguous float64 [rows, %d] arrays" % d)
    ptrs = (ctypes.c_void_p * len(sets))(*[s.ctypes.data for s in sets])
    rows = (ctypes.c_int64 * len(sets))(*[s.shape[0] for s in sets])
    return ptrs, rows, len(sets), d


class Classifier:
    """One GPU (≙ one MPI rank).  set_train ≙ MPI_Bcast of Data_train
    (cpp:224-225); classify ≙ the query loop cpp:358-381."""

    def __init__(self, device=0):
        self._h = ctypes.c_void_p()
        _check(lib().knn_create(ctypes.byref(self._h), device))
        self.device = device
        self.n_train = 0
        self.dim = 0

    def close(self):
        if self._h:
            lib().knn_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_train(self, X, labels, class_cnt):
        X = _f64(X)
        labels = np.ascontiguousarray(labels, dtype=np.int32)
        n, d = X.shape
        _check(lib().knn_set_train(self._h, _ptr(X), _ptr(labels), n, d, int(class_cnt)))
        self.n_train, self.dim = n, d
        self._keep = None

    def set_train_device(self, dX_ptr, dlab_ptr, n, d, class_cnt, idx_offset=0, keep=None):
        """Device pointers (e.g. torch tensors' data_ptr()); `keep` holds the
        owning objects alive for the library (the pointers are borrowed)."""
        _check(lib().knn_set_train_device(self._h, dX_ptr, dlab_ptr, n, d, int(class_cnt),
                                          int(idx_offset)))
        self.n_train, self.dim = n, d
        self._keep = keep

    def classify(self, Q, k, metric=L2, return_neighbors=False):
        """Returns labels (int32[m]) and, if requested, (idx[m,k], dist[m,k], flags[m])."""
        Q = _f64(Q)
        m = Q.shape[0]
        labels = np.empty(m, np.int32)
        flags = np.empty(m, np.int32)
        idx = np.empty((m, max(k, 1)), np.int64) if return_neighbors else None
        dist = np.empty((m, max(k, 1)), np.float64) if return_neighbors else None
        _check(lib().knn_classify(self._h, _ptr(Q), m, int(k), int(metric), _ptr(labels),
                                  _ptr(idx), _ptr(dist), _ptr(flags)))
        if return_neighbors:
            return labels, idx[:, :k], dist[:, :k], flags
        return labels

    def classify_device(self, dQ_ptr, m, k, metric, d_labels, d_idx=None, d_dist=None,
                        d_flags=None, stream=None):
        _check(lib().knn_classify_device(self._h, dQ_ptr, m, int(k), int(metric), d_labels, d_idx,
                                         d_dist, d_flags, stream))

    def search_partial_device(self, dQ_ptr, m, w, metric, d_dist, d_idx, d_lab, stream=None):
        _check(lib().knn_search_partial_device(self._h, dQ_ptr, m, int(w), int(metric), d_dist,
                                               d_idx, d_lab, stream))

    def merge_vote_device(self, d_dist, d_idx, d_lab, parts, m, w, k, d_labels, d_out_idx=None,
                          d_out_dist=None, d_flags=None, stream=None, q0=0, mq=None):
        """k-way merge of [parts][m][w] lists + vote for queries [q0, q0+mq)."""
        mq = m - q0 if mq is None else mq
        _check(lib().knn_merge_vote_device(self._h, d_dist, d_idx, d_lab, int(parts), m, int(w),
                                           int(k), int(q0), int(mq), d_labels, d_out_idx,
                                           d_out_dist, d_flags, stream))

    def shard_distances_device(self, dQ_ptr, d_qsel, nsel, metric, d_out, stream=None):
        """Exact fp64 distances of this context's shard rows to nsel queries
        (dQ rows d_qsel[i], or i when d_qsel is None): d_out [nsel][n_shard]."""
        _check(lib().knn_shard_distances_device(self._h, dQ_ptr, d_qsel, int(nsel), int(metric),
                                                d_out, stream))

    def tie_resolve_device(self, d_D, rows, nsel, d_lab_all, d_orow, k, d_labels, d_idx=None,
                           d_dist=None, d_flags=None, stream=None):
        """Reference order (std::sort over the whole train set) for nsel
        queries whose distances to every row are in d_D as len(rows) blocks
        [nsel][rows[p]] in global row order; rewrites output rows d_orow."""
        arr = (ctypes.c_int64 * len(rows))(*[int(r) for r in rows])
        _check(lib().knn_tie_resolve_device(self._h, d_D, len(rows), arr, int(nsel), d_lab_all,
                                            d_orow, int(k), d_labels, d_idx, d_dist, d_flags,
                                            stream))

    def sync(self):
        _check(lib().knn_sync(self._h))

    def last_rescan_count(self):
        """Queries of the last call that failed certification (waits for it)."""
        return int(lib().knn_last_rescan_count(self._h))

    def rescan_totals(self, reset=False):
        """(failed certification, finished by the full exact scan) summed over
        the calls since the last reset (waits for them)."""
        out = (ctypes.c_int64 * 2)()
        _check(lib().knn_rescan_totals(self._h, out, int(bool(reset))))
        return int(out[0]), int(out[1])

    def tie_totals(self, reset=False):
        """Queries re-ordered as the reference's std::sort orders them
        (KNN_FLAG_TIE_REF), summed over calls since the last reset."""
        out = ctypes.c_int64()
        _check(lib().knn_tie_totals(self._h, ctypes.byref(out), int(bool(reset))))
        return int(out.value)

    def timing_totals(self, reset=False):
        """(per-phase ms summed over timed calls since the last reset, calls)."""
        ms = (ctypes.c_double * 4)()
        calls = ctypes.c_int64()
        _check(lib().knn_timing_totals(self._h, ms, ctypes.byref(calls), int(bool(reset))))
        return [float(v) for v in ms], int(calls.value)

    def last_kernel_name(self):
        """Candidate kernel of the last call, rocprofv3-style ("cand_kernel<128,4,4,8>")."""
        return lib().knn_last_kernel_name(self._h).decode()

    def set_precision(self, mode):
        """PRECISION_AUTO (int8 on integer-coded data, else fp16 / bf16x3 by
        shape, knn_amd.h), PRECISION_FP32, PRECISION_BF16X3, PRECISION_FP16.
        Results are the exact fp64 top-k in every mode."""
        _check(lib().knn_set_precision(self._h, int(mode)))

    def set_tuning(self, key, value):
        """Experiment overrides (knn_amd.h, knn_set_tuning): "R", "S", "nw",
        "ablate", "fp16", "mfma16", "i8", "i8w", "gk", "s3q", "qres", "s3gq", "xhswz",
        "ties", "seed", "order", "ophase", "nblk"; 0 (or -1 where stated) =
        automatic.  "order" and "nblk" shape the train layout and are read by
        set_train: "order" -1 = region order only for integer-coded sets whose
        int8 image is <= 192 MB (n / 16384 regions, up to 64, at least 8),
        1 = n / 16384 regions (off below n = 32768); "nblk" -1 = norm blocks
        for integer-coded sets of more than 16384 rows (d <= 256), 1 on, 2 on
        as plain sorted windows, 3 without spreading the sub-tiles over the
        window's tiles."""
        _check(lib().knn_set_tuning(self._h, key.encode(), int(value)))

    def last_candidate_path(self):
        return int(lib().knn_last_candidate_path(self._h))

    def set_timing(self, enable=True, kernel_only=False):
        """HIP-event phase timing (knn_set_timing): every phase, or with
        kernel_only the candidate kernel alone (2 events per call instead of
        5; each event record holds the stream a few microseconds)."""
        _check(lib().knn_set_timing(self._h, 0 if not enable else (2 if kernel_only else 1)))

    def last_phase_ms(self, phase):
        return float(lib().knn_last_phase_ms(self._h, int(phase)))

    def last_geometry(self):
        out = (ctypes.c_int64 * 4)()
        _check(lib().knn_last_geometry(self._h, out))
        return dict(workgroups=out[0], splits=out[1], lists=out[2], rerank=out[3])

    def normalize(self, *sets):
        """Min-max normalisation of host sets in place (cpp:229-306): e.g.
        normalize(train, test, val).  Returns (max, min) per dimension."""
        ptrs, rows, ns, d = _set_arrays(sets)
        mx, mn = np.empty(d), np.empty(d)
        _check(lib().knn_normalize(self._h, ptrs, rows, ns, d, _ptr(mx), _ptr(mn)))
        return mx, mn

    def minmax_device(self, dX_ptr, rows, d, d_max, d_min, init=True, stream=None):
        """Fold a device set into per-dim bounds (init: start at -1/999999)."""
        _check(lib().knn_minmax_device(self._h, dX_ptr, int(rows), int(d), d_max, d_min,
                                       int(bool(init)), stream))

    def normalize_device(self, dX_ptr, rows, d, d_max, d_min, stream=None):
        _check(lib().knn_normalize_device(self._h, dX_ptr, int(rows), int(d), d_max, d_min,
                                          stream))


class Group:
    """Single-process multi-GPU classifier over RCCL (mode 0 query-sharded,
    1 train-sharded); see include/knn_amd.h.  rccl=True runs every
    collective through RCCL even on one GPU; repeated devices (e.g. [0, 0])
    run several ranks on one GPU over loopback copies."""

    def __init__(self, devices, mode=0, rccl=False):
        self._h = ctypes.c_void_p()
        arr = (ctypes.c_int * len(devices))(*devices)
        flags = GROUP_RCCL if rccl else 0
        _check(lib().knn_group_create(ctypes.byref(self._h), len(devices), arr, int(mode) | flags))

    def transport(self):
        return int(lib().knn_group_transport(self._h))

    def set_precision(self, mode):
        _check(lib().knn_group_set_precision(self._h, int(mode)))

    def set_tuning(self, key, value):
        _check(lib().knn_group_set_tuning(self._h, key.encode(), int(value)))

    def last_tie_count(self):
        return int(lib().knn_group_last_tie_count(self._h))

    def close(self):
        if self._h:
            lib().knn_group_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_train(self, X, labels, class_cnt):
        X = _f64(X)
        labels = np.ascontiguousarray(labels, dtype=np.int32)
        n, d = X.shape
        _check(lib().knn_group_set_train(self._h, _ptr(X), _ptr(labels), n, d, int(class_cnt)))

    def classify(self, Q, k, metric=L2, return_neighbors=False):
        Q = _f64(Q)
        m = Q.shape[0]
        labels = np.empty(m, np.int32)
        flags = np.empty(m, np.int32)
        idx = np.empty((m, max(k, 1)), np.int64) if return_neighbors else None
        dist = np.empty((m, max(k, 1)), np.float64) if return_neighbors else None
        _check(lib().knn_group_classify(self._h, _ptr(Q), m, int(k), int(metric), _ptr(labels),
                                        _ptr(idx), _ptr(dist), _ptr(flags)))
        if return_neighbors:
            return labels, idx[:, :k], dist[:, :k], flags
        return labels

    def last_compute_seconds(self):
        return float(lib().knn_group_last_compute_seconds(self._h))

    def normalize(self, *sets):
        """Sharded normalisation of host sets in place with an RCCL MAX/MIN
        all-reduce of the bounds (cpp:229-306)."""
        ptrs, rows, ns, d = _set_arrays(sets)
        _check(lib().knn_group_normalize(self._h, ptrs, rows, ns, d))


def run_driver(cfg: KnnConfig, workdir, gpus=1, mode="query", extra=()):
    """Runs the native drop-in driver (bin/knn_mpi_amd) the way `mpiexec
    knn_mpi` runs the reference, in `workdir`; returns its stdout."""
    if not os.path.exists(DRIVER_PATH):
        raise KnnError("driver not built: " + DRIVER_PATH)
    args = [DRIVER_PATH]
    for f in ("dim", "K", "N_train", "N_test", "N_val", "class_cnt"):
        args += ["--" + f, str(getattr(cfg, f))]
    for f in ("Euclidean_distance", "Normalize", "Validation"):
        args += ["--" + f, "true" if getattr(cfg, f) else "false"]
    args += ["--train_file", cfg.train_file_name, "--validation_file", cfg.validation_file_name,
             "--test_file", cfg.test_file_name, "--gpus", str(gpus), "--mode", mode]
    args += list(extra)
    r = subprocess.run(args, cwd=workdir, capture_output=True, text=True)
    if r.returncode != 0:
        raise KnnError("driver failed (%d): %s" % (r.returncode, r.stderr.strip()))
    return r.stdout
