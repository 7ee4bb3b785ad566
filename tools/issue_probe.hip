// issue_probe.hip -- MFMA throughput beside a given VALU load (test tooling,
// not part of the library).  Question for the fp16 candidate kernel: at the
// chip's held clock, does v_mfma_f32_32x32x16_f16 (32 cycles, vector issue
// held 8) leave more room for the selection's VALU than two
// v_mfma_f32_16x16x32_f16 (16 cycles each, issue held 8 each) doing the same
// flops?  Each wave runs `iters` units of 32768 flops (one 32x32x16 or two
// 16x16x32 MFMAs on independent accumulators) and `nv` independent v_add_f32
// per unit; 4 waves per SIMD (16 per CU), every CU busy.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/issue_probe.hip -o tools/libissue_probe.so
#include <hip/hip_runtime.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

template <int NV>
__device__ __forceinline__ void valu(float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < NV; ++i) asm volatile("v_add_f32 %0, 1.0, %0" : "+v"(v[i & 7]));
}

template <int SHAPE, int NV>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4)))
probe_kernel(float* out, int iters, float seed) {
  const int l = threadIdx.x & 63;
  f16x8 a, b;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    a[u] = (_Float16)(seed * (l + u));
    b[u] = (_Float16)(seed * (l - u));
  }
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = seed * i;
  float r = 0.f;
  if constexpr (SHAPE == 0) {
    f32x4 c[8] = {};
    for (int it = 0; it < iters; it += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        c[2 * u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c[2 * u], 0, 0, 0);
        c[2 * u + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c[2 * u + 1], 0, 0, 0);
        valu<NV>(v);
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) r += c[u][0] + c[u][3];
  } else if constexpr (SHAPE == 2) {
    // int8: 2 x v_mfma_i32_16x16x64_i8 per unit (65536 ops)
    const i32x4 ai = __builtin_bit_cast(i32x4, a), bi = __builtin_bit_cast(i32x4, b);
    i32x4 c[8] = {};
    for (int it = 0; it < iters; it += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        c[2 * u] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ai, bi, c[2 * u], 0, 0, 0);
        c[2 * u + 1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ai, bi, c[2 * u + 1], 0, 0, 0);
        valu<NV>(v);
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) r += (float)(c[u][0] + c[u][3]);
  } else if constexpr (SHAPE == 3) {
    // int8: 1 x v_mfma_i32_32x32x32_i8 per unit (65536 ops)
    const i32x4 ai = __builtin_bit_cast(i32x4, a), bi = __builtin_bit_cast(i32x4, b);
    i32x16 c[4] = {};
    for (int it = 0; it < iters; it += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        c[u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(ai, bi, c[u], 0, 0, 0);
        valu<NV>(v);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) r += (float)(c[u][0] + c[u][15]);
  } else {
    f32x16 c[4] = {};
    for (int it = 0; it < iters; it += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        c[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c[u], 0, 0, 0);
        valu<NV>(v);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) r += c[u][0] + c[u][15];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) r += v[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int SHAPE, int NV>
static float run_one(float* out, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((probe_kernel<SHAPE, NV>), dim3(blocks), dim3(256), 0, 0, out, iters, 1e-3f);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL((probe_kernel<SHAPE, NV>), dim3(blocks), dim3(256), 0, 0, out, iters, 1e-3f);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms;
}

// ms of one launch of `blocks` 4-wave workgroups, `iters` units each
// (shape 0: 2 x 16x16x32 f16, 1: 1 x 32x32x16 f16, 2: 2 x 16x16x64 i8, 3: 1 x 32x32x32 i8;
// nv in {0, 2, 4, 6, 8, 12, 16}); -1 on error
extern "C" float issue_probe(int shape, int nv, int blocks, int iters) {
  float* out = nullptr;
  if (hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)) != hipSuccess) return -1.f;
  float ms = -1.f;
#define KNN_P(NV)                                                                         \
  if (nv == NV) ms = shape == 0 ? run_one<0, NV>(out, blocks, iters)                       \
                   : shape == 1 ? run_one<1, NV>(out, blocks, iters)                       \
                   : shape == 2 ? run_one<2, NV>(out, blocks, iters) : run_one<3, NV>(out, blocks, iters);
  KNN_P(0) KNN_P(2) KNN_P(4) KNN_P(6) KNN_P(8) KNN_P(12) KNN_P(16)
#undef KNN_P
  hipFree(out);
  return ms;
}
