"""CPU check of the drop-in driver's CSV reader (-mpi-knn-_amd/host/csv.cpp:
parallel pread + std::from_chars fast path with an atof fallback) against
the oracle's restatement of the reference's reader (cpp:154-222: getline /
stringstream split on ',' / atof / atoi), bit for bit, on tokens that
exercise every fallback: blanks, '+', CRLF, hex, inf/nan spellings, trailing
garbage, empty tokens, subnormals, overflow.  The reader is compiled here
into a small test library (the driver itself needs a GPU to run)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "-mpi-knn-_amd", "host")

WRAP = r'''
#include "csv.h"
extern "C" long long csv_read(const char* path, int dim, int with_label, long long rows,
                              double* data, int* labels, int threads) {
  knnhost::CsvResult r = knnhost::read_csv(path, dim, with_label != 0, rows, data, labels, threads);
  return r.ok ? (long long)r.tokens : -1;
}
'''


@pytest.fixture(scope="module")
def reader(tmp_path_factory):
    d = tmp_path_factory.mktemp("csvlib")
    src = d / "wrap.cpp"
    src.write_text(WRAP)
    lib = d / "libcsvtest.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread", "-I", HOST,
                    str(src), os.path.join(HOST, "csv.cpp"), "-o", str(lib)], check=True)
    L = ctypes.CDLL(str(lib))
    L.csv_read.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_longlong,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.csv_read.restype = ctypes.c_longlong
    return L


def _read_both(reader, path, dim, with_label, rows, threads):
    got = np.zeros((rows, dim), np.float64)
    glab = np.zeros(rows, np.int32)
    n = reader.csv_read(str(path).encode(), dim, int(with_label), rows, got.ctypes.data,
                        glab.ctypes.data, threads)
    want, wlab, wn = oracle.read_csv(str(path), dim, with_label, rows)
    return n, got, glab, wn, want, wlab


TRICKY = ["0.1", "-0.0", "1e-310", "  5.5", "+3", "0x1p-3", "inf", "-INF", "nan", "1.5abc", "",
          ".5", "5.", "1e400", "4.9e-324", "-7", "0.30000000000000004", "123456789012345678901",
          "  -2.5e+3", "1E5", "abc", "0000.25"]


@pytest.mark.parametrize("threads", [1, 4])
def test_tricky_tokens_match_reference_reader(reader, tmp_path, threads):
    rng = np.random.default_rng(5)
    dim, rows = 7, 4000
    lines = []
    for r in range(rows):
        toks = [TRICKY[i] for i in rng.integers(0, len(TRICKY), dim)]
        if r % 5 == 0:
            toks = ["%.17g" % v for v in rng.standard_normal(dim)]
        line = "%d," % (r % 10) + ",".join(toks)
        lines.append(line + ("\r\n" if r % 3 == 0 else "\n"))
    text = "".join(lines)
    p = tmp_path / "train.csv"
    p.write_text(text[:-1])  # the last line without its newline
    # a file over 1 MiB so the parallel path (threads > 1) is taken
    big = tmp_path / "big.csv"
    big.write_text(text * 8)
    for path, nrows in ((p, rows), (big, rows * 8)):
        n, got, glab, wn, want, wlab = _read_both(reader, path, dim, True, nrows, threads)
        assert n == wn
        assert got.tobytes() == want.tobytes()
        np.testing.assert_array_equal(glab, wlab)


def test_test_file_format_and_bounds(reader, tmp_path):
    """Test rows carry no label (cpp:186-195); rows beyond N are counted but
    not stored (the reference overflows its buffer there, cpp:140)."""
    rng = np.random.default_rng(9)
    X = rng.standard_normal((300, 5))
    p = tmp_path / "test.csv"
    p.write_text("".join(",".join("%.17g" % v for v in row) + "\n" for row in X))
    n, got, _, wn, want, _ = _read_both(reader, p, 5, False, 250, 4)
    assert n == wn == 300 * 5
    assert got.tobytes() == want.tobytes()
    assert got.tobytes() == X[:250].tobytes()


def test_bench_grid_csv_roundtrip(reader, tmp_path):
    """bench.py's drop-in inputs (8-bit grid values k/256 in the reference's
    train / test CSV formats) read back exactly by the driver's reader."""
    import bench
    rng = np.random.default_rng(8)
    codes = rng.integers(0, 256, (1000, 24)).astype(np.uint8)
    lab = rng.integers(0, 10, 1000).astype(np.int32)
    for labels in (lab, None):
        p = tmp_path / ("tr.csv" if labels is not None else "te.csv")
        bench.write_grid_csv(str(p), codes, labels, chunk=300)
        data = np.empty((1000, 24))
        got_l = np.empty(1000, np.int32)
        n = reader.csv_read(str(p).encode(), 24, int(labels is not None), 1000, data.ctypes.data,
                            got_l.ctypes.data if labels is not None else None, 4)
        assert n == 1000 * (24 + (labels is not None))
        assert data.tobytes() == (codes.astype(np.float64) / 256.0).tobytes()
        if labels is not None:
            np.testing.assert_array_equal(got_l, lab)
