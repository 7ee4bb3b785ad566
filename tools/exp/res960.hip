// Experiment (not part of the library): the bare MFMA + LDS loop of a
// query-resident fp16 candidate pass at d = 960 (cfg5), to measure whether
// that structure can beat the S3 kernel's 18.8 ms (0.41 of the fp16 peak)
// before building its selection.  Each wave keeps its queries' fp16 codes in
// registers for the whole kernel (QB = 2: 32 queries x 960 dims = 240 VGPRs,
// one wave per SIMD; QB = 1: 16 queries, two waves per SIMD); 32-row train
// tiles (1936 B rows) stream through two LDS buffers by LDS-DMA, one barrier
// per tile; no selection (a min over the accumulators keeps them live).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/exp/res960.hip -o tools/exp/res960
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef RPAD
#define RPAD 8
#endif
// floats per row: 488 (RPAD 8) makes the 16x16 fragment reads conflict-free
// (484, the odd 16-B stride of the 32x32 layouts, is 2-way here: measured
// SQ_LDS_BANK_CONFLICT = 4 cycles per ds_read_b128)
constexpr int DP = 960, DPF = DP / 2, RSF = DPF + RPAD;
#ifndef TRT
#define TRT 32
#endif
#ifndef NBUF
#define NBUF 2
#endif
#ifndef NOSTAGE
#define NOSTAGE 0
#endif
#ifndef NOBAR
#define NOBAR 0
#endif
// TRT rows per staged tile (16 or 32), NBUF LDS buffers (prefetch distance
// NBUF - 1 tiles); NOSTAGE: every tile re-reads the split's first tile (L2
// resident: the loop without the row stream); NOBAR: no workgroup barrier
// (timing only)
constexpr int TR = TRT, TBY = TR * RSF * 4, NG = (TBY + 1023) / 1024, BUFF = NG * 256, NB = NBUF, PD = NB - 1;
constexpr int RB = TR / 16;

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
      : "memory");
}

// query fragments loaded straight into AGPRs (MFMA srcB may be an AGPR on
// gfx950), leaving the VGPRs for the A fragments in flight
#ifndef QAGPR
#define QAGPR 1
#endif
#ifndef KCH
#define KCH 5
#endif
#if QAGPR
#define QAG "=&a"
#else
#define QAG "=&v"
#endif

template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <int QB, int NW, int WPE>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
bare(const float* __restrict__ X, const float* Q, int n_tiles, int S, int n_qt, float* out) {
  __shared__ __attribute__((aligned(16))) float lds[NB * BUFF];
  const int bid = blockIdx.x;
  const int split = bid / n_qt, qt = bid - split * n_qt;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, g16 = lane >> 4;
  constexpr int QW = 16 * QB, NQF = QB * DP / 32;
  const long qb0 = (long)qt * (NW * QW) + wv * QW + c16;
  float4 qf[NQF];
#pragma unroll
  for (int c0 = 0; c0 < NQF; c0 += 4) {
    const float* p[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + u < NQF ? c0 + u : c0;
      const int ks = c % (DP / 32), qb = c / (DP / 32);
      p[u] = Q + (qb0 + 16 * qb) * DPF + 16 * ks + 4 * g16;
    }
    float4 v0, v1, v2, v3;
    asm volatile(
        "global_load_dwordx4 %0, %4, off\n\t"
        "global_load_dwordx4 %1, %5, off\n\t"
        "global_load_dwordx4 %2, %6, off\n\t"
        "global_load_dwordx4 %3, %7, off\n\t"
        "s_waitcnt vmcnt(0)"
        : QAG(v0), QAG(v1), QAG(v2), QAG(v3)
        : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3])
        : "memory");
    qf[c0] = v0;
    if (c0 + 1 < NQF) qf[c0 + 1] = v1;
    if (c0 + 2 < NQF) qf[c0 + 2] = v2;
    if (c0 + 3 < NQF) qf[c0 + 3] = v3;
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds;
  auto issue = [&](int t, int b) {
    const char* g = (const char*)X + (long)t * TBY + lane * 16;
    const uint32_t l = lds_base + (uint32_t)(b * BUFF * 4);
    for (int i = wv; i < NG; i += NW) glds16(g + i * 1024, l + (uint32_t)(i * 1024));
  };
  const int my_nt = split < n_tiles ? (n_tiles - split + S - 1) / S : 0;
  auto tile_of = [&](int i) { return NOSTAGE ? split : split + i * S; };
#pragma unroll
  for (int p = 0; p < PD; ++p)
    if (p < my_nt) issue(tile_of(p), p);
  constexpr int G_HI = (NG + NW - 1) / NW, G_LO = NG / NW;
  const bool g_hi = wv < NG % NW || NG % NW == 0;
  float m = 3.0e38f;
  int cur = 0, nxt = PD;
  for (int it = 0; it < my_nt; ++it) {
    const int ahead = min(PD - 1, my_nt - 1 - it);
    if (NOBAR) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (ahead == PD - 1 && PD > 1) {
      if (g_hi) wait_barrier<(PD - 1) * G_HI>(); else wait_barrier<(PD - 1) * G_LO>();
    } else {
      wait_barrier<0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    if (it + PD < my_nt) issue(tile_of(it + PD), nxt);
    const float* base = lds + cur * BUFF;
    f32x4 acc[RB][QB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) acc[rb][qb] = f32x4{0, 0, 0, 0};
    // A fragments software-pipelined in chunks of KC k-steps: chunk c+1's
    // reads are issued before chunk c's MFMAs (one wave per SIMD: no other
    // wave hides the LDS latency)
    constexpr int KC = KCH, NC = (DP / 32) / KC;
    static_assert(NC * KC == DP / 32, "chunking");
    float4 af[2][KC][RB];
    auto rd = [&](int c, int bsel) {
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          af[bsel][k][rb] = *(const float4*)(base + (rb * 16 + c16) * RSF + 16 * (c * KC + k) + 4 * g16);
    };
    rd(0, 0);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (c + 1 < NC) rd(c + 1, (c + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const int ks = c * KC + k;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          const f16x8 a = __builtin_bit_cast(f16x8, af[c & 1][k][rb]);
#pragma unroll
          for (int qb = 0; qb < QB; ++qb)
            acc[rb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, __builtin_bit_cast(f16x8, qf[qb * (DP / 32) + ks]),
                                                                acc[rb][qb], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int qb = 0; qb < QB; ++qb)
        m = __builtin_fminf(m, __builtin_fminf(__builtin_fminf(acc[rb][qb][0], acc[rb][qb][1]),
                                               __builtin_fminf(acc[rb][qb][2], acc[rb][qb][3])));
    cur = cur + 1 == NB ? 0 : cur + 1;
    nxt = nxt + 1 == NB ? 0 : nxt + 1;
  }
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

template <int QB, int NW, int WPE>
void run(const float* X, const float* Q, int n, int m, int S, float* out) {
  const int QPWG = NW * 16 * QB;
  const int n_qt = m / QPWG, n_tiles = n / TR;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f, sum = 0;
  const int reps = 5;
  for (int r = 0; r < reps + 1; ++r) {
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((bare<QB, NW, WPE>), dim3(n_qt * S), dim3(NW * 64), 0, 0, X, Q, n_tiles, S, n_qt, out);
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
  const double fl = 2.0 * n * (double)(n_qt * QPWG) * DP;
  printf("TR=%d NB=%d KC=%d nostage=%d nobar=%d QB=%d NW=%d WPE=%d S=%d: mean %.3f ms best %.3f ms  %.1f TF/s = %.3f of 2.5 PF\n", TR, NB, KCH, NOSTAGE, NOBAR, QB, NW, WPE, S,
         sum / reps, best, fl / (best * 1e-3) / 1e12, fl / (best * 1e-3) / 2.5e15);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int n = 1000448, m = 10240;  // 1M rows (multiple of 32 * 64), 10k queries (multiple of 128)
  std::vector<float> h((size_t)n * RSF + 1024);
  for (size_t i = 0; i < h.size(); ++i) {
    const _Float16 x = (_Float16)((rand() & 1023) / 1024.0f), y = (_Float16)((rand() & 1023) / 1024.0f);
    uint32_t u = (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
    h[i] = __builtin_bit_cast(float, u);
  }
  float *X, *Q, *out;
  CK(hipMalloc(&X, h.size() * 4));
  CK(hipMemcpy(X, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&Q, (size_t)m * DPF * 4));
  CK(hipMemcpy(Q, h.data(), (size_t)m * DPF * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&out, (size_t)16 << 22));
  const int S = argc > 1 ? atoi(argv[1]) : 64;
  run<2, 4, 1>(X, Q, n, m, S, out);
  return 0;
}
