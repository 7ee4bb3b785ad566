"""CPU check of the built gfx950 code objects: no candidate, merge or rescan
kernel uses scratch (a register spill turns the fp16 S3 kernel ~10x slower
-- it happened once this round when a filter change pushed its epilogue into
private memory), and the register-resident candidate kernels stay within the
VGPR budget their occupancy assumes (<= 128 for 4 waves per SIMD).  Reads the
AMDGPU metadata notes of the device code objects bundled in libknn_amd.so
(llvm-objdump --offloading into a temporary directory, llvm-readelf
--notes); no GPU needed."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "-mpi-knn-_amd", "lib", "libknn_amd.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def kernel_metadata(tmp):
    if not os.path.exists(LIB):
        pytest.skip("libknn_amd.so not built")
    if not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("llvm-objdump not available")
    lib = os.path.join(tmp, "lib.so")
    shutil.copy(LIB, lib)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", lib], cwd=tmp,
                   check=True, capture_output=True)
    meta = {}
    for f in sorted(os.listdir(tmp)):
        if "amdgcn" not in f:
            continue
        out = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", os.path.join(tmp, f)],
                             check=True, capture_output=True, text=True).stdout
        # one YAML map per kernel under .kernels: an entry starts at "  - .key"
        # (its first key, e.g. .agpr_count, precedes .name)
        entry = {}

        def flush():
            if "name" in entry:
                meta.setdefault(entry["name"], {}).update(
                    {k: v for k, v in entry.items() if k != "name"})

        for line in out.splitlines():
            if re.match(r"\s+- \.", line):
                flush()
                entry = {}
            m = re.match(r"\s+(?:- )?\.name:\s+(\S+)", line)
            if m:
                entry["name"] = m.group(1)
                continue
            m = re.match(r"\s+(?:- )?\.(private_segment_fixed_size|vgpr_count|agpr_count):\s+(\d+)",
                         line)
            if m:
                entry[m.group(1)] = int(m.group(2))
        flush()
    return meta


def test_hot_kernels_use_no_scratch(tmp_path):
    """The default paths' kernels -- the fp16 resident kernels (metric 4),
    every S3 kernel, the merge and the rescan kernels -- use no scratch."""
    meta = kernel_metadata(str(tmp_path))
    hot = {k: v for k, v in meta.items()
           if re.search(r"cand_kernelILi\d+ELi\d+ELi[456]E", k)
           or any(s in k for s in ("cand_s3_kernel", "merge_rerank", "rescan"))}
    assert len(hot) > 15, "expected the candidate / merge / rescan kernels in the code objects"
    spilled = sorted(k for k, v in hot.items() if v.get("private_segment_fixed_size", 0) != 0)
    assert not spilled, "kernels using scratch: %s" % spilled[:5]


def test_no_kernel_spills_more_than_a_few_registers(tmp_path):
    """Elsewhere at most a few registers' worth of scratch (today: the
    bf16x3 16x16x32 and 32x32 R = 8 kernels at DP = 128, the L1 kernel at
    DP = 8 and the large-k kernel, 12-28 B each, outside the default paths)."""
    meta = kernel_metadata(str(tmp_path))
    big = sorted((k, v["private_segment_fixed_size"]) for k, v in meta.items()
                 if v.get("private_segment_fixed_size", 0) > 32)
    assert not big, big[:5]


def test_fp16_resident_kernels_fit_4_waves(tmp_path):
    # cand_kernel<DP, 4, 4 | 5 | 6, NW> and <DP, 8, 6, NW> (the fp16 / int8
    # default paths): <= 128 registers per lane (VGPR + AGPR) so two 8-wave
    # workgroups share a CU
    meta = kernel_metadata(str(tmp_path))
    fp16 = {k: v for k, v in meta.items()
            if re.search(r"cand_kernelILi\d+ELi4ELi[456]ELi8E|cand_kernelILi\d+ELi8ELi6ELi8E", k)}
    assert fp16, "no fp16 resident kernels found"
    for k, v in fp16.items():
        dp = int(re.search(r"cand_kernelILi(\d+)E", k).group(1))
        if dp > 128:
            continue  # DP 160 .. 256 run at lower occupancy (AGPRs in use) by design
        assert v.get("vgpr_count", 0) + v.get("agpr_count", 0) <= 128, (k, v)
