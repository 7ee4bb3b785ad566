"""Deterministic synthetic inputs in the reference's CSV formats.

The reference reads three CSV files (cpp:154-222, pdf p.11):
  train / validation: ``label,f1,...,f_dim`` per row (integer label first)
  test:               ``f1,...,f_dim`` per row (no label)
There is no network here for MNIST, so fixtures and benches use seeded
synthetic data of the same shape.  Every generator is a pure function of
(kind, seed, shape): the golden fixtures store only the spec plus a sha256 of
the CSV bytes, and tests regenerate the files and check the hash.

kinds
  gauss   -- Gaussian mixture, class = cluster id, values on a 1/1024 grid
             (exact binary fractions, printed %.17g, so CSV text -> atof
             reproduces the generator's doubles bit for bit)
  int     -- SIFT-like integers 0..255 around integer centres (many exact ties)
  noisy   -- heavily overlapping clusters (vote ties at small K)
  normedge-- gauss plus dims that hit the normalisation quirks of cpp:239-243:
             a constant dim, a dim entirely < -1, a dim entirely > 999999
  sorted  -- gauss with train rows sorted by class (adversarial split load)
"""
import hashlib
import io
import os

import numpy as np


def _rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def make_sets(kind, seed, n_train, n_test, n_val, dim, class_cnt):
    """Returns (train, train_lab, test, test_lab, val, val_lab) as float64/int32."""
    rng = _rng(seed)
    n_all = n_train + n_test + n_val
    if kind in ("gauss", "normedge", "sorted", "noisy"):
        spread = 1.0 if kind == "noisy" else 2.0
        centres = rng.uniform(-spread, spread, size=(class_cnt, dim))
        lab = rng.integers(0, class_cnt, size=n_all).astype(np.int32)
        x = centres[lab] + rng.standard_normal((n_all, dim))
        x = np.round(x * 1024.0) / 1024.0
        if kind == "normedge" and dim >= 4:
            x[:, 0] = 3.25                      # constant dim: max==min -> untouched
            x[:, 1] = -5.0 - np.abs(x[:, 1])    # all < -1: max stays at the -1 init
            x[:, 2] = 1.0e6 + np.abs(x[:, 2])   # all > 999999: min stays at 999999
            x[:, 3] = np.round(x[:, 3] * 1000.0 * 1024.0) / 1024.0
    elif kind == "int":
        centres = rng.integers(0, 256, size=(class_cnt, dim))
        lab = rng.integers(0, class_cnt, size=n_all).astype(np.int32)
        x = centres[lab] + rng.integers(-24, 25, size=(n_all, dim))
        x = np.clip(x, 0, 255).astype(np.float64)
    else:
        raise ValueError(kind)
    tr, te, va = x[:n_train], x[n_train:n_train + n_test], x[n_train + n_test:]
    trl, tel, val_ = lab[:n_train], lab[n_train:n_train + n_test], lab[n_train + n_test:]
    if kind == "sorted":
        order = np.argsort(trl, kind="stable")
        tr, trl = tr[order], trl[order]
    return (np.ascontiguousarray(tr), trl.copy(), np.ascontiguousarray(te), tel.copy(),
            np.ascontiguousarray(va), val_.copy())


def _fmt_rows(x, labels=None, kind="gauss"):
    """CSV text; %.17g (exact for grid values), %d for integer kinds."""
    buf = io.StringIO()
    fmt = "%d" if kind == "int" else "%.17g"
    if labels is not None:
        np.savetxt(buf, np.column_stack([labels.astype(np.float64), x]),
                   fmt=["%d"] + [fmt] * x.shape[1], delimiter=",")
    else:
        np.savetxt(buf, x, fmt=fmt, delimiter=",")
    return buf.getvalue()


def write_csvs(dirpath, spec, names=("train.csv", "validation.csv", "test.csv"),
               crlf=False, trailing_newline=True):
    """Writes the three files; returns (arrays, sha256-of-concatenated-bytes)."""
    sets = make_sets(spec["kind"], spec["seed"], spec["N_train"], spec["N_test"],
                     spec["N_val"], spec["dim"], spec["class_cnt"])
    tr, trl, te, tel, va, val_ = sets
    kind = spec["kind"]
    texts = [_fmt_rows(tr, trl, kind), _fmt_rows(va, val_, kind), _fmt_rows(te, None, kind)]
    h = hashlib.sha256()
    for name, t in zip(names, texts):
        if crlf:
            t = t.replace("\n", "\r\n")
        if not trailing_newline:
            t = t.rstrip("\r\n")
        b = t.encode()
        h.update(b)
        with open(os.path.join(dirpath, name), "wb") as f:
            f.write(b)
    return sets, h.hexdigest()
