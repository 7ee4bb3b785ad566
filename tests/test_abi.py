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


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_no_gpu_fails_loudly(libpath):
    knn = _load_mirror()
    with pytest.raises(knn.KnnError, match="no CPU fallback"):
        knn.Classifier(0)
    with pytest.raises(knn.KnnError):
        knn.Group([0], mode=0)
