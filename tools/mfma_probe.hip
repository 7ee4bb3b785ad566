// mfma_probe.hip -- numerics probe for the candidate pass's MFMA instructions
// (test tooling, not part of the library).  One wave per case computes
// D = C + A.B with a single v_mfma_f32_32x32x16_bf16 (A 32x16, B 16x32 bf16,
// C/D 32x32 fp32, all row-major in memory) or a single
// v_mfma_f32_32x32x2_f32 (A 32x2, B 2x32 fp32); tools/mfma_probe.py compares
// the results with candidate rounding models computed exactly on the host.
// Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC tools/mfma_probe.hip -o tools/libmfma_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__global__ void __launch_bounds__(64) probe_bf16_kernel(const uint16_t* A, const uint16_t* B,
                                                        const float* C, float* D) {
  const int cs = blockIdx.x, l = threadIdx.x, j = l & 31, h = l >> 5;
  const uint16_t* a = A + (size_t)cs * 32 * 16;
  const uint16_t* b = B + (size_t)cs * 16 * 32;
  const float* c = C + (size_t)cs * 1024;
  float* d = D + (size_t)cs * 1024;
  uint16_t av[8], bv[8];
  for (int u = 0; u < 8; ++u) {
    av[u] = a[j * 16 + 8 * h + u];  // A row j, k = 8h + u
    bv[u] = b[(8 * h + u) * 32 + j];  // B col j, k = 8h + u
  }
  bf16x8 af, bf;
  for (int u = 0; u < 8; ++u) {
    af[u] = __builtin_bit_cast(__bf16, av[u]);
    bf[u] = __builtin_bit_cast(__bf16, bv[u]);
  }
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = c[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + j];
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc, 0, 0, 0);
  for (int i = 0; i < 16; ++i) d[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + j] = acc[i];
}

__global__ void __launch_bounds__(64) probe_f32_kernel(const float* A, const float* B,
                                                       const float* C, float* D) {
  const int cs = blockIdx.x, l = threadIdx.x, j = l & 31, h = l >> 5;
  const float* a = A + (size_t)cs * 32 * 2;
  const float* b = B + (size_t)cs * 2 * 32;
  const float* c = C + (size_t)cs * 1024;
  float* d = D + (size_t)cs * 1024;
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = c[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + j];
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j * 2 + h], b[h * 32 + j], acc, 0, 0, 0);
  for (int i = 0; i < 16; ++i) d[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + j] = acc[i];
}

extern "C" int probe_bf16(const void* A, const void* B, const void* C, void* D, int ncases) {
  hipLaunchKernelGGL(probe_bf16_kernel, dim3(ncases), dim3(64), 0, 0, (const uint16_t*)A,
                     (const uint16_t*)B, (const float*)C, (float*)D);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

extern "C" int probe_f32(const void* A, const void* B, const void* C, void* D, int ncases) {
  hipLaunchKernelGGL(probe_f32_kernel, dim3(ncases), dim3(64), 0, 0, (const float*)A,
                     (const float*)B, (const float*)C, (float*)D);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
