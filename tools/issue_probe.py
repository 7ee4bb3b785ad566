#!/usr/bin/env python3
"""MFMA rate beside a VALU load: 16x16x32 vs 32x32x16 fp16, 16x16x64 vs 32x32x32 int8
(tools/issue_probe.hip).
Run on a GPU box: python tools/issue_probe.py (needs tools/libissue_probe.so)."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libissue_probe.so"))
lib.issue_probe.restype = ctypes.c_float
lib.issue_probe.argtypes = [ctypes.c_int] * 4
BLOCKS, ITERS = 1024, 4000
flops = BLOCKS * 4 * ITERS * 32768.0
print("VALU per unit | 2 x 16x16x32 f16 | 1 x 32x32x16 f16 (TF/s, unit 32768 flops) | "
      "2 x 16x16x64 i8 | 1 x 32x32x32 i8 (TOPS, unit 65536 ops)")
for nv in (0, 2, 4, 6, 8, 12, 16):
    r = []
    for shape in (0, 1, 2, 3):
        ms = min(lib.issue_probe(shape, nv, BLOCKS, ITERS) for _ in range(3))
        f = flops * (2 if shape >= 2 else 1)
        r.append(f / (ms * 1e-3) / 1e12 if ms > 0 else float("nan"))
    print("%3d | %7.1f | %7.1f | %7.1f | %7.1f" % (nv, r[0], r[1], r[2], r[3]), flush=True)
