"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every
function include/knn_amd.h declares (and the Python mirror binds the same
set), and -- with no GPU in the process -- refuses to run instead of falling
back to any CPU path.  No compute calls are made."""
import ctypes
import os
import re
import subprocess

import pytest
import torch

import importlib.util

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "-mpi-knn-_amd")
HEADER = os.path.join(ROOT, "include", "knn_amd.h")


def _load_mirror():
    spec = importlib.util.spec_from_file_location("knn_amd", os.path.join(PKG, "knn_amd.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(knn_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def libpath():
    knn = _load_mirror()
    if not os.path.exists(knn.LIB_PATH):
        knn.build()
    return knn.LIB_PATH


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("knn_create", "knn_destroy", "knn_set_train", "knn_classify",
                 "knn_search_partial_device", "knn_merge_vote_device", "knn_last_error",
                 "knn_normalize", "knn_group_normalize", "knn_group_classify"):
        assert must in names


def test_library_exports_every_declared_symbol(libpath):
    L = ctypes.CDLL(libpath)
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", libpath], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (knn_\w+)", out))
    assert set(declared_functions()) <= exported
    # no C++-mangled knn entry points leak as the interface
    assert all(not n.startswith("_Z") for n in exported)


def test_python_mirror_binds_exactly_the_header():
    knn = _load_mirror()
    assert sorted(knn.EXPORTED) == declared_functions()


def test_version_string(libpath):
    L = ctypes.CDLL(libpath)
    L.knn_version.restype = ctypes.c_char_p
    assert b"gfx950" in L.knn_version()


class _CandLaunch(ctypes.Structure):
    """knnk::CandLaunch (csrc/knn_kernels.h), field for field."""
    _fields_ = [("metric", ctypes.c_int), ("DP", ctypes.c_int), ("R", ctypes.c_int),
                ("S", ctypes.c_int), ("n_qt", ctypes.c_int), ("n_pad", ctypes.c_int64),
                ("X32", ctypes.c_void_p), ("xinit", ctypes.c_void_p), ("Q32", ctypes.c_void_p),
                ("out_v", ctypes.c_void_p), ("out_i", ctypes.c_void_p), ("ablate", ctypes.c_int),
                ("nw", ctypes.c_int), ("qpb", ctypes.c_int), ("gthr", ctypes.c_void_p),
                ("xsw", ctypes.c_int), ("gk", ctypes.c_int)]


def test_resident_kernel_refuses_mismatched_query_tile(libpath):
    """The resident candidate kernels index nw x (queries per wave) queries per
    workgroup; a launch whose host query tile differs (the round-3 fault:
    group objects of two builds) is refused before anything reaches the
    device: launch_cand returns false (knn_run_search -> KNN_ERR_ARG).
    Only the refusal is exercised here -- no kernel is launched."""
    L = ctypes.CDLL(libpath)
    sym = "_ZN4knnk11launch_candERKNS_10CandLaunchEP12ihipStream_t"
    fn = getattr(L, sym)
    fn.argtypes = [ctypes.POINTER(_CandLaunch), ctypes.c_void_p]
    fn.restype = ctypes.c_bool
    for metric, DP, nw, qpb in ((5, 128, 8, 257), (5, 128, 8, 512), (4, 128, 8, 128),
                                (0, 64, 4, 64), (5, 96, 8, 0)):
        c = _CandLaunch(metric=metric, DP=DP, R=4 if metric >= 3 else 8, S=1, n_qt=1,
                        n_pad=256, nw=nw, qpb=qpb)
        assert fn(ctypes.byref(c), None) is False, (metric, DP, nw, qpb)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_no_gpu_fails_loudly(libpath):
    knn = _load_mirror()
    with pytest.raises(knn.KnnError, match="no CPU fallback"):
        knn.Classifier(0)
    with pytest.raises(knn.KnnError):
        knn.Group([0], mode=0)
