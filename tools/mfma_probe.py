#!/usr/bin/env python3
"""Numerics probe of v_mfma_f32_32x32x16_bf16 (and, as a control,
v_mfma_f32_32x32x2_f32) on the GPU: which rounding model reproduces every
output bit for bit?  The candidate pass's certification bound
(knn_api.cpp err_factor) depends on how many roundings an MFMA performs.

Models, each computed exactly (Fractions) and rounded to fp32:
  fused_rn   D = RN(C + sum_k a_k b_k)            one rounding per MFMA
  fused_rz   D = RZ(C + sum_k a_k b_k)
  seq_rn     D = RN(...RN(RN(C + p_0) + p_1)...)   k-ordered fma chain
  seq_rn_rev the same chain from k = K-1 down to 0
  halves_rn  RN(RN(C + sum_{k<K/2}) + sum_{k>=K/2})  (two fused halves)
Run on a GPU box: python tools/mfma_probe.py  (builds nothing; needs
tools/libmfma_probe.so, made by `make -C tools`)."""
import ctypes
import os
import sys
from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def rn_f32(x: Fraction, mode="rn"):
    """Exact rounding of a rational to fp32 (round-to-nearest-even or toward zero)."""
    if x == 0:
        return 0.0
    s = -1.0 if x < 0 else 1.0
    a = -x if x < 0 else x
    e = a.numerator.bit_length() - a.denominator.bit_length()
    if Fraction(2) ** e > a:
        e -= 1
    ulp_e = max(e - 23, -149)
    q = a / (Fraction(2) ** ulp_e)
    n = q.numerator // q.denominator
    r = q - n
    if mode == "rn":
        if r > Fraction(1, 2) or (r == Fraction(1, 2) and n % 2 == 1):
            n += 1
    return s * float(Fraction(n) * Fraction(2) ** ulp_e)


def bf16_bits(x):
    """RN-even float32 -> bf16 bit patterns, and the bf16 values as float64."""
    f = np.asarray(x, dtype=np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    vals = (r.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    return r, vals


def models(c, prods):
    K = len(prods)
    C = Fraction(float(c))
    P = [Fraction(float(p)) for p in prods]
    out = {}
    out["fused_rn"] = rn_f32(C + sum(P))
    out["fused_rz"] = rn_f32(C + sum(P), "rz")
    acc = float(c)
    for p in P:
        acc = rn_f32(Fraction(acc) + p)
    out["seq_rn"] = acc
    acc = float(c)
    for p in reversed(P):
        acc = rn_f32(Fraction(acc) + p)
    out["seq_rn_rev"] = acc
    h = rn_f32(C + sum(P[:K // 2]))
    out["halves_rn"] = rn_f32(Fraction(h) + sum(P[K // 2:]))
    return out


def families(rng, K):
    """(name, A[32][K], B[K][32], C[32][32]) float64 values (bf16/fp32-representable later)."""
    def rnd(shape, lo=-20, hi=20):
        return rng.choice([-1.0, 1.0], shape) * (1 + rng.random(shape)) * 2.0 ** rng.integers(lo, hi, shape)
    fam = []
    fam.append(("typical", rng.standard_normal((32, K)), rng.standard_normal((K, 32)),
                rng.standard_normal((32, 32))))
    fam.append(("tiny_addends", np.full((32, K), 2.0 ** -13), np.full((K, 32), 2.0 ** -12),
                np.ones((32, 32))))
    A = np.zeros((32, K)); A[:, 0] = 3 * 2.0 ** -13
    fam.append(("three_quarter_ulp", A, np.full((K, 32), 2.0 ** -12), np.ones((32, 32))))
    fam.append(("half_ulp_ties", np.full((32, K), 2.0 ** -12), np.full((K, 32), 2.0 ** -12),
                np.ones((32, 32)) + 2.0 ** -23 * rng.integers(0, 4, (32, 32))))
    fam.append(("wide_exponents", rnd((32, K)), rnd((K, 32)), rnd((32, 32), -30, 30)))
    A = rng.standard_normal((32, K)); B = rng.standard_normal((K, 32))
    if K >= 2:
        A[:, 1] = -A[:, 0]; B[1] = B[0]    # exact cancellation of the first pair
    fam.append(("cancellation", A, B, rng.standard_normal((32, 32)) * 2.0 ** -10))
    fam.append(("positive_knn_like", rng.random((32, K)), rng.random((K, 32)) * -2,
                rng.random((32, 32)) * K / 3))
    fam.append(("c_zero", rng.standard_normal((32, K)), rng.standard_normal((K, 32)),
                np.zeros((32, 32))))
    return fam


def main():
    import torch
    torch.cuda.init()
    lib = ctypes.CDLL(os.path.join(HERE, "libmfma_probe.so"))
    rng = np.random.default_rng(1)
    dev = torch.device("cuda", 0)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for kind, K in (("bf16", 16), ("f32", 2)):
        tally = {}
        worst = {}
        for rep in range(reps):
            for name, A, B, C in families(rng, K):
                C32 = C.astype(np.float32)
                if kind == "bf16":
                    Ab, Av = bf16_bits(A)
                    Bb, Bv = bf16_bits(B)
                    ta = torch.from_numpy(Ab.view(np.int16).copy()).to(dev)
                    tb = torch.from_numpy(Bb.view(np.int16).copy()).to(dev)
                else:
                    Av = A.astype(np.float32).astype(np.float64)
                    Bv = B.astype(np.float32).astype(np.float64)
                    ta = torch.from_numpy(A.astype(np.float32)).to(dev)
                    tb = torch.from_numpy(B.astype(np.float32)).to(dev)
                tc = torch.from_numpy(C32).to(dev)
                td = torch.empty_like(tc)
                fn = lib.probe_bf16 if kind == "bf16" else lib.probe_f32
                assert fn(ctypes.c_void_p(ta.data_ptr()), ctypes.c_void_p(tb.data_ptr()),
                          ctypes.c_void_p(tc.data_ptr()), ctypes.c_void_p(td.data_ptr()), 1) == 0
                D = td.cpu().numpy()
                t = tally.setdefault(name, {})
                for r in range(32):
                    for c in range(0, 32, 3 if name == "typical" else 5):
                        prods = Av[r, :] * Bv[:, c]  # exact in fp64 (<= 48-bit products)
                        ms = models(C32[r, c], prods)
                        got = float(D[r, c])
                        for mname, v in ms.items():
                            t.setdefault(mname, [0, 0])
                            t[mname][0] += (np.float32(v).view(np.uint32) == np.float32(got).view(np.uint32))
                            t[mname][1] += 1
                        # error of the hardware vs exact, in units of u * (|C| + sum|p|)
                        ex = Fraction(float(C32[r, c])) + sum(Fraction(float(p)) for p in prods)
                        mag = abs(float(C32[r, c])) + float(np.abs(prods).sum())
                        if mag > 0:
                            err = abs(float(Fraction(got) - ex)) / (mag * 2.0 ** -24)
                            worst[name] = max(worst.get(name, 0.0), err)
        print("== %s MFMA (K=%d): bit-exact match rate per model" % (kind, K))
        for name, t in tally.items():
            print("  %-18s " % name + "  ".join("%s %d/%d" % (m, v[0], v[1]) for m, v in t.items())
                  + "   max|err|/(u*(|C|+sum|p|)) = %.3f" % worst.get(name, 0.0))


if __name__ == "__main__":
    main()
