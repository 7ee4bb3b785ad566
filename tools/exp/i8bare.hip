// Experiment (not part of the library): the bare loop of the int8 32x32x32
// candidate pass at cfg2's shape (1M rows x 10,240 queries, d = 128, 144-B
// image rows, 256-row tiles through LDS by LDS-DMA, one barrier per tile),
// to compare workgroup shapes before building one:
//   QH query halves per wave (1: 32 queries, as cand_kernel<128,4,6,8>; 2: 64
//   queries, each A fragment read from LDS feeds two MFMAs), NW waves per
//   workgroup, WPE waves per SIMD the registers are sized for.
// SEL 1 adds the fast path of the selection (a v_max3 tree over the previous
// sub-tile's 16 accumulators and a wave-uniform branch that never passes);
// SEL 2 the same over 8 of them; SEL 3 the 16-value tree without the branch; SEL 0 none (the sub-tiles' MFMAs chain into
// one accumulator, so none is dead code);
// NOSTAGE re-reads the split's first tile (no row stream).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/exp/i8bare.hip -o tools/exp/i8bare
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

#ifndef STG
#define STG 0
#endif
#ifndef NODMA
#define NODMA 0
#endif
#ifndef NOLDS
#define NOLDS 0
#endif
#ifndef NOBAR
#define NOBAR 0
#endif
#ifndef PF
#define PF 0
#endif
#ifndef NOSTAGE
#define NOSTAGE 0
#endif
constexpr int DP = 128, RSF = DP / 4 + 4;  // floats per row (144 B)
constexpr int TPB = 8, TR = 32 * TPB, TBY = TR * RSF * 4, NG = (TBY + 1023) / 1024, BUFF = NG * 256, NB = 2;

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
      : "memory");
}

__device__ __forceinline__ void wait_barrier0() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ int max16(const i32x16& a) {
  auto m3 = [](int x, int y, int z) { return max(max(x, y), z); };
  return max(m3(m3(a[0], a[1], a[2]), m3(a[3], a[4], a[5]), m3(a[6], a[7], a[8])),
             m3(m3(a[9], a[10], a[11]), m3(a[12], a[13], a[14]), a[15]));
}

__device__ __forceinline__ int max8(const i32x16& a) {
  auto m3 = [](int x, int y, int z) { return max(max(x, y), z); };
  return m3(m3(a[0], a[1], a[2]), m3(a[3], a[4], a[5]), max(a[6], a[7]));
}

template <int QH, int NW, int WPE, int SEL>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
bare(const char* __restrict__ X, const char* Q, int n_tiles, int S, int n_qt, int* out, int thr) {
  __shared__ __attribute__((aligned(16))) float lds[NB * BUFF];
  // XCD-aware: consecutive logical ids on one XCD (grid % 8 == 0)
  const int g = gridDim.x, b = blockIdx.x;
  const int bid = (b & 7) * (g >> 3) + (b >> 3);
  const int split = bid / n_qt, qt = bid - split * n_qt;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, h = lane >> 5;
  constexpr int QW = 32 * QH;
  i32x4 qf[QH][DP / 32];
#pragma unroll
  for (int qh = 0; qh < QH; ++qh) {
    const char* qp = Q + ((long)qt * (NW * QW) + wv * QW + qh * 32 + j) * DP + 16 * h;
#pragma unroll
    for (int ks = 0; ks < DP / 32; ++ks) {
      i32x4 v;
      asm volatile("global_load_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(qp + 32 * ks) : "memory");
      qf[qh][ks] = v;
    }
  }
  // (NOLDS 3: 8 fragments of random rows in registers stand in for the rows:
  // every MFMA gets an A operand unlike its neighbours' and unlike B)
  i32x4 rf[NOLDS == 3 ? 8 : 1];
  if constexpr (NOLDS == 3) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      i32x4 v;
      asm volatile("global_load_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)"
                   : "=&v"(v) : "v"(X + ((long)(bid * 8 + u) * 37 + j) * RSF * 4 + 16 * h) : "memory");
      rf[u] = v;
    }
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds;
  auto issue = [&](int t, int bsel) {
    const char* gp = X + (long)t * TBY + lane * 16;
    const uint32_t l = lds_base + (uint32_t)(bsel * BUFF * 4);
    for (int i = wv; i < NG; i += NW) glds16(gp + i * 1024, l + (uint32_t)(i * 1024));
  };
  const int my_nt = split < n_tiles ? (n_tiles - split + S - 1) / S : 0;
  auto tile_of = [&](int i) { return NOSTAGE ? split : split + i * S; };
  if (my_nt > 0) issue(tile_of(0), 0);
  int hits = 0, mx_all = -0x7fffffff;
  i32x16 accp[QH];
#pragma unroll
  for (int qh = 0; qh < QH; ++qh) accp[qh] = i32x16{};
  int cur = 0;
  for (int it = 0; it < my_nt; ++it) {
    if (NOBAR) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else wait_barrier0();
    __builtin_amdgcn_sched_barrier(0);
    // STG: the next tile by plain loads into registers, written to LDS by
    // ds_write_b128 at mid-tile (instead of LDS-DMA pieces)
    constexpr int NPW = (NG + NW - 1) / NW;
    i32x4 stg[STG ? NPW : 1];
    if (STG && it + 1 < my_nt) {
      const char* gp = X + (long)tile_of(it + 1) * TBY + lane * 16;
#pragma unroll
      for (int k = 0; k < NPW; ++k) {
        const int i = wv + k * NW;
        if (i < NG) stg[k] = *(const i32x4*)(gp + i * 1024);
      }
    } else if (!STG && it + 1 < my_nt && !NODMA) {
      issue(tile_of(it + 1), cur ^ 1);  // (NODMA: only the first tile)
    }
    i32x4 afn[DP / 32];
#pragma unroll
    for (int sub = 0; sub < TPB; ++sub) {
      if (STG && sub == TPB / 2 && it + 1 < my_nt) {
#pragma unroll
        for (int k = 0; k < NPW; ++k) {
          const int i = wv + k * NW;
          if (i < NG) *(i32x4*)((char*)(lds + (cur ^ 1) * BUFF) + i * 1024 + lane * 16) = stg[k];
        }
      }
      const float* base = lds + cur * BUFF + sub * 32 * RSF;
      i32x4 af[DP / 32];
      if (NOLDS) {
        // (NOLDS: the query fragments stand in for the rows -- no LDS read;
        // NOLDS 2: the rows are still read, into a sink the MFMAs do not use)
#pragma unroll
        for (int ks = 0; ks < DP / 32; ++ks) af[ks] = NOLDS == 3 ? rf[(ks + sub) & 7] : qf[0][(ks + sub) & 3];
        if (NOLDS == 2) {
#pragma unroll
          for (int ks = 0; ks < DP / 32; ++ks) {
            const i32x4 x = __builtin_bit_cast(i32x4, *(const float4*)(base + j * RSF + 8 * ks + 4 * h));
            hits ^= x[ks];
          }
        }
      } else if (!PF || sub == 0) {
#pragma unroll
        for (int ks = 0; ks < DP / 32; ++ks)
          af[ks] = __builtin_bit_cast(i32x4, *(const float4*)(base + j * RSF + 8 * ks + 4 * h));
      } else {
#pragma unroll
        for (int ks = 0; ks < DP / 32; ++ks) af[ks] = afn[ks];
      }
      if (PF && sub + 1 < TPB) {
        // (PF) the next sub-tile's A fragments in flight behind this one's MFMAs
#pragma unroll
        for (int ks = 0; ks < DP / 32; ++ks)
          afn[ks] = __builtin_bit_cast(i32x4, *(const float4*)(base + 32 * RSF + j * RSF + 8 * ks + 4 * h));
      }
      __builtin_amdgcn_sched_barrier(0);  // (PF: the next sub-tile's reads stay ahead of these MFMAs)
      i32x16 acc[QH];
#pragma unroll
      for (int ks = 0; ks < DP / 32; ++ks)
#pragma unroll
        for (int qh = 0; qh < QH; ++qh)
          acc[qh] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[ks], qf[qh][ks],
                                                          ks == 0 ? (SEL == 0 ? accp[qh] : i32x16{}) : acc[qh], 0, 0, 0);
      if constexpr (SEL) {
#pragma unroll
        for (int qh = 0; qh < QH; ++qh) {
          const int mx = SEL == 2 ? max8(accp[qh]) : max16(accp[qh]);
          if constexpr (SEL == 3) {
            hits += mx > thr;  // (SEL 3: the same tree, no ballot and no branch)
          } else if (__builtin_amdgcn_ballot_w64(mx > thr)) {
            ++hits;
            mx_all = max(mx_all, mx);
          }
        }
      }
#pragma unroll
      for (int qh = 0; qh < QH; ++qh) accp[qh] = acc[qh];
    }
    cur ^= 1;
  }
  int m = mx_all + hits;
#pragma unroll
  for (int qh = 0; qh < QH; ++qh) m = max(m, max16(accp[qh]));
  out[(long)bid * NW * 64 + tid] = m;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <int QH, int NW, int WPE, int SEL>
void run(const char* X, const char* Q, int n, int m, int S, int* out) {
  const int QPWG = NW * 32 * QH;
  const int n_qt = m / QPWG, n_tiles = n / TR;
  const int grid = n_qt * S;
  if (grid % 8) {
    printf("grid %d not a multiple of 8\n", grid);
    return;
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f, sum = 0;
  const int reps = 5;
  for (int r = 0; r < reps + 1; ++r) {
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((bare<QH, NW, WPE, SEL>), dim3(grid), dim3(NW * 64), 0, 0, X, Q, n_tiles, S, n_qt, out,
                       0x7fffffff);
    CK(hipGetLastError());
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r) {
      best = ms < best ? ms : best;
      sum += ms;
    }
  }
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, bare<QH, NW, WPE, SEL>, NW * 64, 0));
  const double ops = 2.0 * n * (double)(n_qt * QPWG) * DP;
  printf("STG=%d NODMA=%d NOLDS=%d NOBAR=%d PF=%d QH=%d NW=%d WPE=%d SEL=%d nostage=%d S=%d grid=%d wg/CU=%d: mean %.3f ms best %.3f ms  %.0f TOPS = %.3f of 5 POPS\n",
         STG, NODMA, NOLDS, NOBAR, PF, QH, NW, WPE, SEL, NOSTAGE, S, grid, occ, sum / reps, best, ops / (best * 1e-3) / 1e12,
         ops / (best * 1e-3) / 5e15);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int n = 3907 * TR, m = 10240;  // 1,000,192 rows (256-row tiles), 10,240 queries
  std::vector<signed char> hx((size_t)n * RSF * 4 + 4096), hq((size_t)m * DP);
  srand(1);
  for (auto& v : hx) v = (signed char)((rand() & 127) - 64);
  for (auto& v : hq) v = (signed char)((rand() & 127) - 64);
  char *X, *Q;
  int* out;
  CK(hipMalloc(&X, hx.size()));
  CK(hipMemcpy(X, hx.data(), hx.size(), hipMemcpyHostToDevice));
  CK(hipMalloc(&Q, hq.size()));
  CK(hipMemcpy(Q, hq.data(), hq.size(), hipMemcpyHostToDevice));
  CK(hipMalloc(&out, (size_t)64 << 20));
  const int S = argc > 1 ? atoi(argv[1]) : 40;
  for (int pass = 0; pass < 2; ++pass) {
    run<1, 8, 4, 1>(X, Q, n, m, S, out);
    run<1, 8, 4, 3>(X, Q, n, m, S, out);
    run<2, 4, 2, 1>(X, Q, n, m, S, out);
    run<2, 4, 2, 3>(X, Q, n, m, S, out);
  }
  return 0;
}
