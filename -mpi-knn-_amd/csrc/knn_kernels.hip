// knn_kernels.hip -- MI355X (gfx950, CDNA4) kernels of the KNN classify path.
//
// Pipeline per classify call (reference loop: cpp:308-381):
//   1. prep_queries      fp64 queries -> fp32 (x -2 for L2) MFMA operands
//   2. cand_kernel       fused distance + per-lane top-R selection.
//        L2: -2 q.x^T on v_mfma_f32_32x32x2_f32 with the accumulator seeded by
//            ||x||^2, so the chain ends at ||x||^2 - 2 q.x (the rank-equivalent
//            of ||q - x||^2 for a fixed query; cpp:33-50).
//        L1: sum |q - x| on the VALU (cpp:51-67; no GEMM identity exists).
//        The distance matrix is never materialised: each lane keeps a sorted
//        register list of its R best rows and a threshold filter.
//   3. merge_rerank      per query: union of all lists -> best C by the fp32
//        proxy -> exact fp64 reference distances for those C (sequential sum,
//        no FMA, correctly rounded sqrt) -> sort by (dist, idx) -> certify
//        that no excluded row can enter the top-w (rigorous fp32 error
//        bound) -> first-to-max vote (cpp:324-337) or partial list output.
//   4. rescan (rare)     queries that fail certification get an exact fp64
//        scan over every row (chunked sort + tree reduce).
// The result is the reference's fp64 top-k with ties ordered by train index.
#include "knn_kernels.h"

#include <float.h>
#include <limits.h>

#include <type_traits>

#pragma clang fp contract(off)

namespace knnk {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define KNN_INF_F __builtin_inff()
#define KNN_INF_D __builtin_inf()


// ---------------------------------------------------------------- helpers
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // Blocks are dispatched round-robin over the 8 XCDs; give each XCD a
  // contiguous range of logical ids so workgroups that stream the same train
  // split share an L2 (bijective for any nwg).
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_or_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Reference distance, bit-exact with cpp:33-50 (L2: returns the squared sum
// before sqrt) and cpp:51-67 (L1): fp64, dims in order, multiply then add.
template <int METRIC>
__device__ __forceinline__ double exact_dist_raw(const double* __restrict__ q,
                                                 const double* __restrict__ x, int d) {
  double r = 0.0;
#pragma unroll 8
  for (int i = 0; i < d; ++i) {
    const double t = q[i] - x[i];
    if (METRIC == 0) r = r + t * t;
    else r = r + __builtin_fabs(t);
  }
  return r;
}
template <int METRIC>
__device__ __forceinline__ double exact_dist(const double* __restrict__ q,
                                             const double* __restrict__ x, int d) {
  const double r = exact_dist_raw<METRIC>(q, x, d);
  return METRIC == 0 ? __builtin_sqrt(r) : r;  // llvm.sqrt.f64: correctly rounded
}

template <typename K, typename I>
__device__ __forceinline__ bool pair_less(K ka, I ia, K kb, I ib) {
  return ka < kb || (ka == kb && ia < ib);
}

// Bitonic sort of n (power of two) (key, id) pairs in LDS, ascending by
// (key, id).  All threads of the block participate.
template <typename K, typename I>
__device__ void bitonic_sort_lds(K* key, I* id, int n, int tid, int nthr) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int t = tid; t < (n >> 1); t += nthr) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const K ka = key[lo], kb = key[hi];
        const I ia = id[lo], ib = id[hi];
        const bool sw = up ? pair_less(kb, ib, ka, ia) : pair_less(ka, ia, kb, ib);
        if (sw) {
          key[lo] = kb; key[hi] = ka;
          id[lo] = ib; id[hi] = ia;
        }
      }
    }
  }
  __syncthreads();
}

__device__ __forceinline__ int pow2_ceil(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// ------------------------------------------------------------------ prep
// One wave per train row: fp64 -> fp32 (zero padded to DP), fl32(||x32||^2)
// seeds for the L2 accumulator, 0 seeds for L1, +inf on pad rows; running
// max of ||x||_2^2 and ||x||_1 (fp64, non-negative -> ordered as u64 bits).
__global__ void __launch_bounds__(256)
prep_train_kernel(const double* __restrict__ X64, int64_t n, int d, int DP, int64_t n_pad,
                  float* __restrict__ X32, float* __restrict__ xl2, float* __restrict__ xl1,
                  unsigned long long* __restrict__ stats) {
  const int RSF = DP + 4;  // padded row: [x32 (DP) | ||x32||^2, l1 seed, 0, 0]
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  double m2 = 0.0, m1 = 0.0;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n_pad; row += wstride) {
    double s32 = 0.0, s64 = 0.0, a64 = 0.0;
    for (int c = lane; c < DP; c += 64) {
      float v = 0.0f;
      if (row < n && c < d) {
        const double x = X64[row * d + c];
        v = (float)x;
        s64 += x * x;
        a64 += __builtin_fabs(x);
      }
      X32[row * RSF + c] = v;
      s32 += (double)v * (double)v;
    }
    s32 = wave_sum_d(s32);
    s64 = wave_sum_d(s64);
    a64 = wave_sum_d(a64);
    if (lane < 4) {
      const float s2 = row < n ? (float)s32 : KNN_INF_F;
      const float s1 = row < n ? 0.0f : KNN_INF_F;
      X32[row * RSF + DP + lane] = lane == 0 ? s2 : (lane == 1 ? s1 : 0.0f);
      if (lane == 0) {
        xl2[row] = s2;
        xl1[row] = s1;
      }
    }
    m2 = fmax(m2, s64);
    m1 = fmax(m1, a64);
  }
  if (lane == 0) {
    // small relative slack covers the order of the fp64 sums above
    atomicMax(&stats[0], (unsigned long long)__double_as_longlong(m2 * (1.0 + 1e-12)));
    atomicMax(&stats[1], (unsigned long long)__double_as_longlong(m1 * (1.0 + 1e-12)));
  }
}

void launch_prep_train(const double* X64, int64_t n, int d, int DP, int64_t n_pad, float* X32,
                       float* xl2, float* xl1, unsigned long long* stats, hipStream_t s) {
  int64_t blocks = (n_pad + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(prep_train_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X64, n, d, DP,
                     n_pad, X32, xl2, xl1, stats);
}

__global__ void __launch_bounds__(256)
prep_queries_kernel(const double* __restrict__ Q64, int64_t m, int d, int DP, int64_t m_pad,
                    float scale, float* __restrict__ Q32) {
  const int64_t total = m_pad * DP;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int64_t row = e / DP;
    const int c = (int)(e - row * DP);
    float v = 0.0f;
    if (row < m && c < d) v = scale * (float)Q64[row * d + c];  // x(-2) is exact
    Q32[e] = v;
  }
}

void launch_prep_queries(const double* Q64, int64_t m, int d, int DP, int64_t m_pad,
                         float scale, float* Q32, hipStream_t s) {
  int64_t blocks = (m_pad * DP + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(prep_queries_kernel, dim3((unsigned)blocks), dim3(256), 0, s, Q64, m, d,
                     DP, m_pad, scale, Q32);
}

// bf16 hi/lo split of fp64 rows: row r of the output is [hi(DP) | lo(DP)]
// with hi = bf16(x), lo = bf16(x - hi) (x - hi exact in fp64), scaled by
// `scale` (exact power of two), zero padding beyond d and on pad rows.
__device__ __forceinline__ void split_bf16(double x, unsigned short& hi, unsigned short& lo) {
  const __bf16 h = (__bf16)(float)x;
  const double r = x - (double)(float)h;
  const __bf16 l = (__bf16)(float)r;
  hi = __builtin_bit_cast(unsigned short, h);
  lo = __builtin_bit_cast(unsigned short, l);
}

__global__ void __launch_bounds__(256)
prep_split_kernel(const double* __restrict__ X64, int64_t n, int d, int DP, int64_t n_pad,
                  double scale, unsigned short* __restrict__ out, int row_shorts,
                  const float* __restrict__ xl2, const float* __restrict__ xl1) {
  // row r of `out` (row_shorts 16-bit words) = [hi(DP) | lo(DP) | seeds...]
  const int64_t total = n_pad * DP;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int64_t row = e / DP;
    const int c = (int)(e - row * DP);
    unsigned short hi = 0, lo = 0;
    if (row < n && c < d) split_bf16(scale * X64[row * d + c], hi, lo);
    out[row * row_shorts + c] = hi;
    out[row * row_shorts + DP + c] = lo;
    if (xl2 && c < 4) {  // train rows: the padded row's seed floats
      float* seed = (float*)(out + row * row_shorts + 2 * DP);
      seed[c] = c == 0 ? xl2[row] : (c == 1 ? xl1[row] : 0.0f);
    }
  }
}

void launch_prep_split(const double* X64, int64_t n, int d, int DP, int64_t n_pad, double scale,
                       unsigned short* out, int row_shorts, const float* xl2, const float* xl1,
                       hipStream_t s) {
  int64_t blocks = (n_pad * DP + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(prep_split_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X64, n, d, DP,
                     n_pad, scale, out, row_shorts, xl2, xl1);
}

__global__ void fill_i32_kernel(int32_t* p, int64_t n, int32_t v) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
    p[e] = v;
}
void launch_fill_i32(int32_t* p, int64_t n, int32_t v, hipStream_t s) {
  if (n <= 0) return;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(fill_i32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, n, v);
}

// ------------------------------------------------------- candidate kernel
// Sorted insertion of v (< L[R-1]) into the ascending register list (L, I);
// the previous last entry drops out.  Fully unrolled: no dynamic register
// indexing (which would go to scratch).
template <int R>
__device__ __forceinline__ void list_insert(float (&L)[R], int (&I)[R], float v, int id) {
  // L'[t] = max(L[t-1], min(v, L[t])) shifts the tail and drops L[R-1];
  // the index follows with two selects.  Branch-free: v_min/v_max/v_cndmask
  // (the TU is built with -fno-honor-nans so fminf/fmaxf need no quieting).
  bool cc = true;  // v < L[R-1] by precondition
#pragma unroll
  for (int t = R - 1; t > 0; --t) {
    const bool cp = v < L[t - 1];
    L[t] = __builtin_fmaxf(L[t - 1], __builtin_fminf(v, L[t]));
    I[t] = cp ? I[t - 1] : (cc ? id : I[t]);
    cc = cp;
  }
  I[0] = cc ? id : I[0];
  L[0] = __builtin_fminf(v, L[0]);
}

// One 16-B-per-lane LDS-DMA piece (global_load_lds_dwordx4): 64 lanes x 16 B
// from per-lane global addresses to LDS [lds_addr, lds_addr + 1 KiB).  Issued
// from inline asm so hipcc neither counts it nor inserts its own
// s_waitcnt vmcnt(0) before later LDS reads (it would drain the pipeline);
// the kernel waits with explicit counted vmcnt + s_barrier instead.  M0 is
// compiler-reserved, so it is saved and restored inside the statement.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
      : "memory");
}

// Fused top-R selection over one 32x32 accumulator block: lane (j, h) holds
// the values of query j against rows row0 + rho(i, h), i = 0..15.  Once the
// list is warm this is a 16-way min (v_min3) and one compare per block; a
// value is inserted only under a branch that no lane of the wave skips.
template <int R>
__device__ __forceinline__ void select_block(const f32x16& acc, int row0, int h, float (&L)[R],
                                             int (&I)[R], float& thr) {
  // Lanes l and l^32 hold the same query: filtering with the smaller of the
  // two list thresholds is safe -- anything dropped is >= some list's final
  // R-th entry, which the merge's lower bound (min over lists) accounts for.
  float te = __builtin_fminf(thr, __shfl_xor(thr, 32, 64));
  float mn = __builtin_fminf(acc[0], acc[1]);
#pragma unroll
  for (int i = 2; i < 16; ++i) mn = __builtin_fminf(mn, acc[i]);
  if (mn < te) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float v = acc[i];
      if (v < te) {
        list_insert<R>(L, I, v, row0 + (i & 3) + 8 * (i >> 2) + 4 * h);
        thr = L[R - 1];
        te = __builtin_fminf(te, thr);
      }
    }
  }
}

// Lists are stored [query][split][half][R] so a query's 2S lists are contiguous.
template <int R>
__device__ __forceinline__ void write_lists(float* __restrict__ out_v, int* __restrict__ out_i,
                                            int64_t qg, int S, int split, int h,
                                            const float (&L)[R], const int (&I)[R]) {
  const int64_t o = ((qg * (2 * S)) + split * 2 + h) * R;
#pragma unroll
  for (int t = 0; t < R; t += 4) {
    *(float4*)(out_v + o + t) = make_float4(L[t], L[t + 1], L[t + 2], L[t + 3]);
    *(int4*)(out_i + o + t) = make_int4(I[t], I[t + 1], I[t + 2], I[t + 3]);
  }
}

// Train rows in HBM (X32 for fp32/L1, XB for bf16x3) share one padded row
// format of RSF = DP + 4 floats: [payload (DP floats) | ||x32||^2, l1 seed,
// 0, 0], where payload is DP fp32 values or [hi(DP) | lo(DP)] bf16.  A tile
// is 32 consecutive rows = one contiguous block, copied linearly into LDS;
// the odd 16-B row stride (DP/4 + 1 chunks) makes the A-fragment reads
// (ds_read_b128, 16-lane groups on distinct rows) bank-conflict free, and the
// accumulator seeds come from the same rows.  Pad rows carry +inf seeds.
//
// Workgroup = 4 waves = 128 queries; it streams the 32-row train tiles
// split, split+S, split+2S, ... (round-robin so a run of similar rows is
// spread over all splits).  Lane (j = lane&31, h = lane>>5) of wave w owns
// query j of the wave and the train rows rho(i,h) = (i&3) + 8(i>>2) + 4h of
// every tile (the 32x32 MFMA C/D layout with train rows on A, queries on B).
//
// METRIC 0, per tile and wave: DP/2 MFMAs 32x32x2 f32; lane (r, h) reads
// float4 X[r][8c+4h ..] for the four k-steps of group c.  METRIC 2: 3*DP/16
// MFMAs 32x32x16 bf16 (see below).  The B operand (queries, -2 q) stays in
// VGPRs for the whole kernel.  Accumulators start at ||x_row||^2, so
// acc = ||x||^2 - 2 q.x.
//
// NW waves (32 queries each) share every staged tile: NW = 8 halves the
// staging instructions and L2 traffic per MFMA relative to NW = 4.
//
// Staging: global_load_lds (LDS-DMA, no VGPRs), 3 LDS buffers: tile it+2 is
// issued right after the barrier that opens tile it, and each wave waits
// with a counted vmcnt for its own pieces of tile it before that barrier --
// two tiles of latency hidden, one barrier per tile.  (A register-staged
// variant measured the same or slower; removed.)
template <int DP, int R, int METRIC, int NW>
__global__ void __launch_bounds__(NW * 64)
cand_kernel(const float* __restrict__ Xr, const float* Q32, int n_tiles, int S,
            int n_qt, float* __restrict__ out_v, int* __restrict__ out_i, int abl) {
  // Q32 is deliberately not __restrict__: with it hipcc treats the query
  // fragments as invariant and re-loads them inside the tile loop instead of
  // keeping them in VGPRs (its waits would then also drain the LDS-DMA queue).
  // abl: timing-only ablations (results invalid): bit0 = no staging loads
  // after the first tiles, bit1 = no selection epilogue.  0 in production.
  constexpr int RSF = DP + 4;               // row stride (floats), HBM and LDS
  constexpr int TBY = kTR * RSF * 4;        // tile bytes
  constexpr int NG = (TBY + 1023) / 1024;   // 1-KiB LDS-DMA pieces per tile
  constexpr int NB = 3;                     // LDS buffers (prefetch distance 2)
  constexpr int BUFF = NG * 256;            // floats per buffer
  constexpr int SEED = METRIC == 1 ? DP + 1 : DP;  // seed float within a row
  __shared__ __attribute__((aligned(16))) float lds[NB * BUFF];

  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / n_qt;
  const int qt = bid - split * n_qt;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, h = lane >> 5;
  const int64_t qg = (int64_t)qt * (NW * 32) + wv * 32 + j;
  const float* qrow = Q32 + qg * DP;

  // B operand resident in VGPRs for the whole kernel.  METRIC 0: fp32 -2q,
  // float4 c holds dims 8c+4h..8c+4h+3 (four 32x32x2 k-steps).  METRIC 2:
  // the row is [qh | ql] in bf16 (-2q split hi/lo); float4 t (t < DP/16) is
  // qh dims 16t+8h..16t+8h+7, float4 DP/16+t the same dims of ql.
  float4 qf[METRIC != 1 ? DP / 8 : 1];
  if constexpr (METRIC != 1) {
    // Loaded with inline asm (loads + their vmcnt(0) in one statement): with
    // ordinary loads hipcc places the vmcnt waits for these registers at
    // their first MFMA use INSIDE the tile loop, where each executes every
    // tile and -- counting all vector-memory ops -- drains the in-flight
    // LDS-DMA pieces of the staging pipeline.
#pragma unroll
    for (int c0 = 0; c0 < DP / 8; c0 += 4) {
      const float* p[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = c0 + u < DP / 8 ? c0 + u : c0;
        const int off = METRIC == 0 ? 8 * c : (c < DP / 16 ? 8 * c : DP / 2 + 8 * (c - DP / 16));
        p[u] = qrow + off + 4 * h;
      }
      float4 v0, v1, v2, v3;
      asm volatile(
          "global_load_dwordx4 %0, %4, off\n\t"
          "global_load_dwordx4 %1, %5, off\n\t"
          "global_load_dwordx4 %2, %6, off\n\t"
          "global_load_dwordx4 %3, %7, off\n\t"
          "s_waitcnt vmcnt(0)"
          : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
          : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3])
          : "memory");
      qf[c0] = v0;
      if (c0 + 1 < DP / 8) qf[c0 + 1] = v1;
      if (c0 + 2 < DP / 8) qf[c0 + 2] = v2;
      if (c0 + 3 < DP / 8) qf[c0 + 3] = v3;
    }
  }

  float L[R];
  int I[R];
#pragma unroll
  for (int t = 0; t < R; ++t) { L[t] = KNN_INF_F; I[t] = -1; }
  float thr = KNN_INF_F;

  const int my_nt = split < n_tiles ? (n_tiles - split + S - 1) / S : 0;

  // ---- staging: this wave's LDS-DMA pieces i = wv, wv+NW, ... of tile t ->
  // buffer b.  The last piece may read past the tile (and past the last row:
  // the HBM allocation carries 1 KiB of slack); it lands in the buffer tail.
  constexpr int G_HI = (NG + NW - 1) / NW, G_LO = NG / NW;
  static_assert(G_HI <= 15, "vmcnt immediate range");
  // LDS byte address of the staging array (wave-uniform)
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds;
#define KNN_ISSUE(t_, b_)                                                              \
  do {                                                                                 \
    const char* g_ = (const char*)Xr + (int64_t)(t_) * TBY + lane * 16;                \
    const uint32_t l_ = lds_base + (uint32_t)((b_) * BUFF * 4);                        \
    for (int i_ = wv; i_ < NG; i_ += NW) glds16(g_ + i_ * 1024, l_ + (uint32_t)(i_ * 1024)); \
  } while (0)

  if (my_nt > 0) KNN_ISSUE(split, 0);
  if (my_nt > 1) KNN_ISSUE(split + S, 1);

  for (int it = 0; it < my_nt; ++it) {
    const int t = split + it * S;
    int cur;
    {
      // this wave's pieces of tile `it` have landed once at most the pieces
      // of tile it+1 remain outstanding; the barrier then publishes all
      // waves' pieces and retires every read of buffer (it-1)%3 before it is
      // refilled with tile it+2.
      // wait + barrier in ONE asm statement with a memory clobber, so no LDS
      // read can be hoisted above the barrier (a bare s_barrier builtin does
      // not order memory) and no vmcnt(0) drains the in-flight tiles.
      if (it + 1 < my_nt) {
        if (wv < NG % NW || NG % NW == 0)
          asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "n"(G_HI) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "n"(G_LO) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      if (it + 2 < my_nt && !(abl & 1)) KNN_ISSUE(t + 2 * S, (it + 2) % 3);
      cur = it % 3;
    }
    const float* base = lds + cur * BUFF;

    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = base[((i & 3) + 8 * (i >> 2) + 4 * h) * RSF + SEED];
    if constexpr (METRIC == 0) {
      const float* arow = base + j * RSF + 4 * h;
#pragma unroll
      for (int c = 0; c < DP / 8; ++c) {
        const float4 a = *(const float4*)(arow + 8 * c);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, qf[c].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, qf[c].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, qf[c].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, qf[c].w, acc, 0, 0, 0);
      }
    } else if constexpr (METRIC == 2) {
      // bf16x3 split product on v_mfma_f32_32x32x16_bf16:
      //   q.x ~= qh.xh + ql.xh + qh.xl   (train row payload = [xh | xl])
      // i.e. one bf16 GEMM with K = 3*DP; ~2^-16 relative product error,
      // 16x the f32 MFMA rate per instruction -> 5.3x per fp32-equivalent flop.
      const float* arow = base + j * RSF + 4 * h;
#pragma unroll
      for (int tt = 0; tt < DP / 16; ++tt) {
        const bf16x8 ah = __builtin_bit_cast(bf16x8, *(const float4*)(arow + 8 * tt));
        const bf16x8 al = __builtin_bit_cast(bf16x8, *(const float4*)(arow + DP / 2 + 8 * tt));
        const bf16x8 bh = __builtin_bit_cast(bf16x8, qf[tt]);
        const bf16x8 bl = __builtin_bit_cast(bf16x8, qf[DP / 16 + tt]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
      }
    } else {
      // L1 on the VALU: lane's query against its 16 rows, dims in chunks of 4.
#pragma unroll 2
      for (int c = 0; c < DP / 4; ++c) {
        const float4 qv = *(const float4*)(qrow + 4 * c);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int r = (i & 3) + 8 * (i >> 2) + 4 * h;
          const float4 xv = *(const float4*)(base + r * RSF + 4 * c);
          float a = acc[i];
          a = a + __builtin_fabsf(qv.x - xv.x);
          a = a + __builtin_fabsf(qv.y - xv.y);
          a = a + __builtin_fabsf(qv.z - xv.z);
          a = a + __builtin_fabsf(qv.w - xv.w);
          acc[i] = a;
        }
      }
    }

    if (!(abl & 2)) select_block<R>(acc, t * kTR, h, L, I, thr);
    else if (acc[0] == 1234.5f && acc[15] == 1234.5f) thr = acc[7];  // keep acc live

  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  write_lists<R>(out_v, out_i, qg, S, split, h, L, I);
#undef KNN_ISSUE
}

// Large-dimension variant (DP > 256, e.g. the reference's MNIST default
// d=784): the query tile no longer fits in VGPRs, so both operands are staged
// through LDS in chunks of DC dims.  Workgroup tile = 128 queries x 128 train
// rows (4 waves x (32 queries x 4 row blocks)); per chunk each wave issues
// 4 x DC/2 MFMAs reading its B fragment once per 8 dims and reusing it over
// the 4 row blocks.  LDS: 2 buffers x (A 128xDC + B 128xDC), rows padded by
// 16 B (DC/4 + 1 odd -> conflict-free ds_read_b128).  Same selection epilogue
// after the last chunk of a tile.
template <int DC, int R, int METRIC>
__global__ void __launch_bounds__(256)
cand_stream_kernel(const float* __restrict__ X32, const float* __restrict__ xinit,
                   const float* __restrict__ Q32, int DP, int n_tiles, int S, int n_qt,
                   float* __restrict__ out_v, int* __restrict__ out_i) {
  constexpr int TRS = 128;          // train rows per tile
  constexpr int LS = DC + 4;        // LDS row stride (floats)
  constexpr int OP = TRS * LS;      // floats per operand image
  constexpr int CPR = DC / 4;       // float4 per row chunk
  constexpr int NCH = TRS * CPR;    // float4 per operand chunk
  constexpr int CPT = NCH / 256;    // per thread
  static_assert(CPT == 4, "staging below is written for 4 float4 per operand");
  __shared__ __attribute__((aligned(16))) float lds[2 * 2 * OP + 2 * TRS];
  float* ldsn = lds + 4 * OP;

  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / n_qt;
  const int qt = bid - split * n_qt;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t qg = (int64_t)qt * kQPB + wv * 32 + j;
  const int nch = DP / DC;

  float L[R];
  int I[R];
#pragma unroll
  for (int t = 0; t < R; ++t) { L[t] = KNN_INF_F; I[t] = -1; }
  float thr = KNN_INF_F;

  const int my_nt = split < n_tiles ? (n_tiles - split + S - 1) / S : 0;
  const int total = my_nt * nch;

  float4 a0, a1, a2, a3, b0, b1, b2, b3;
  float4 stn = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* qbase = Q32 + (int64_t)qt * kQPB * DP;
#define KNN_SLOAD(st_)                                                                  \
  do {                                                                                  \
    const int it_ = (st_) / nch, c_ = (st_) - it_ * nch;                                \
    const int t_ = split + it_ * S;                                                     \
    const float* xs_ = X32 + (int64_t)t_ * TRS * (DP + 4) + c_ * DC;                    \
    const float* qs_ = qbase + c_ * DC;                                                 \
    int e_ = tid;                                                                       \
    a0 = *(const float4*)(xs_ + (e_ / CPR) * (DP + 4) + (e_ % CPR) * 4);                \
    b0 = *(const float4*)(qs_ + (e_ / CPR) * DP + (e_ % CPR) * 4);                      \
    e_ += 256;                                                                          \
    a1 = *(const float4*)(xs_ + (e_ / CPR) * (DP + 4) + (e_ % CPR) * 4);                \
    b1 = *(const float4*)(qs_ + (e_ / CPR) * DP + (e_ % CPR) * 4);                      \
    e_ += 256;                                                                          \
    a2 = *(const float4*)(xs_ + (e_ / CPR) * (DP + 4) + (e_ % CPR) * 4);                \
    b2 = *(const float4*)(qs_ + (e_ / CPR) * DP + (e_ % CPR) * 4);                      \
    e_ += 256;                                                                          \
    a3 = *(const float4*)(xs_ + (e_ / CPR) * (DP + 4) + (e_ % CPR) * 4);                \
    b3 = *(const float4*)(qs_ + (e_ / CPR) * DP + (e_ % CPR) * 4);                      \
    if (c_ == 0 && tid < TRS / 4) stn = ((const float4*)(xinit + (int64_t)t_ * TRS))[tid]; \
  } while (0)
#define KNN_SSTORE(st_, buf_)                                                           \
  do {                                                                                  \
    float* A_ = lds + (buf_) * 2 * OP;                                                  \
    float* B_ = A_ + OP;                                                                \
    int e_ = tid;                                                                       \
    *(float4*)(A_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = a0;                             \
    *(float4*)(B_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = b0;                             \
    e_ += 256;                                                                          \
    *(float4*)(A_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = a1;                             \
    *(float4*)(B_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = b1;                             \
    e_ += 256;                                                                          \
    *(float4*)(A_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = a2;                             \
    *(float4*)(B_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = b2;                             \
    e_ += 256;                                                                          \
    *(float4*)(A_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = a3;                             \
    *(float4*)(B_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = b3;                             \
    const int c_ = (st_) % nch;                                                         \
    if (c_ == 0 && tid < TRS / 4) *(float4*)(ldsn + (buf_) * TRS + 4 * tid) = stn;      \
  } while (0)

  if (total > 0) {
    KNN_SLOAD(0);
    KNN_SSTORE(0, 0);
  }
  __syncthreads();

  f32x16 acc0, acc1, acc2, acc3;
  for (int st = 0; st < total; ++st) {
    const int it = st / nch, c = st - it * nch;
    const int t = split + it * S;
    const bool more = st + 1 < total;
    if (more) KNN_SLOAD(st + 1);
    const float* A = lds + (st & 1) * 2 * OP;
    const float* B = A + OP;
    if (c == 0) {
      // the norms were staged with chunk 0 of this tile into buffer (st & 1)
      const float* nb = ldsn + (st & 1) * TRS;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 n0 = *(const float4*)(nb + 0 * 32 + 8 * g + 4 * h);
        const float4 n1 = *(const float4*)(nb + 1 * 32 + 8 * g + 4 * h);
        const float4 n2 = *(const float4*)(nb + 2 * 32 + 8 * g + 4 * h);
        const float4 n3 = *(const float4*)(nb + 3 * 32 + 8 * g + 4 * h);
        acc0[4 * g] = n0.x; acc0[4 * g + 1] = n0.y; acc0[4 * g + 2] = n0.z; acc0[4 * g + 3] = n0.w;
        acc1[4 * g] = n1.x; acc1[4 * g + 1] = n1.y; acc1[4 * g + 2] = n1.z; acc1[4 * g + 3] = n1.w;
        acc2[4 * g] = n2.x; acc2[4 * g + 1] = n2.y; acc2[4 * g + 2] = n2.z; acc2[4 * g + 3] = n2.w;
        acc3[4 * g] = n3.x; acc3[4 * g + 1] = n3.y; acc3[4 * g + 2] = n3.z; acc3[4 * g + 3] = n3.w;
      }
    }
    if constexpr (METRIC == 0) {
      const float* brow = B + (wv * 32 + j) * LS + 4 * h;
      const float* arow = A + j * LS + 4 * h;
#pragma unroll
      for (int g = 0; g < DC / 8; ++g) {
        const float4 b = *(const float4*)(brow + 8 * g);
        const float4 x0 = *(const float4*)(arow + 0 * 32 * LS + 8 * g);
        const float4 x1 = *(const float4*)(arow + 1 * 32 * LS + 8 * g);
        const float4 x2 = *(const float4*)(arow + 2 * 32 * LS + 8 * g);
        const float4 x3 = *(const float4*)(arow + 3 * 32 * LS + 8 * g);
#define KNN_MF4(acc_, x_)                                                               \
  acc_ = __builtin_amdgcn_mfma_f32_32x32x2f32(x_.x, b.x, acc_, 0, 0, 0);                \
  acc_ = __builtin_amdgcn_mfma_f32_32x32x2f32(x_.y, b.y, acc_, 0, 0, 0);                \
  acc_ = __builtin_amdgcn_mfma_f32_32x32x2f32(x_.z, b.z, acc_, 0, 0, 0);                \
  acc_ = __builtin_amdgcn_mfma_f32_32x32x2f32(x_.w, b.w, acc_, 0, 0, 0);
        KNN_MF4(acc0, x0) KNN_MF4(acc1, x1) KNN_MF4(acc2, x2) KNN_MF4(acc3, x3)
#undef KNN_MF4
      }
    } else {
      const float* brow = B + (wv * 32 + j) * LS;
#pragma unroll 2
      for (int g = 0; g < DC / 4; ++g) {
        const float4 qv = *(const float4*)(brow + 4 * g);
#define KNN_L1B(acc_, blk_)                                                             \
  _Pragma("unroll") for (int i = 0; i < 16; ++i) {                                      \
    const int r = (blk_) * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;                         \
    const float4 xv = *(const float4*)(A + r * LS + 4 * g);                             \
    float a = acc_[i];                                                                  \
    a = a + __builtin_fabsf(qv.x - xv.x);                                               \
    a = a + __builtin_fabsf(qv.y - xv.y);                                               \
    a = a + __builtin_fabsf(qv.z - xv.z);                                               \
    a = a + __builtin_fabsf(qv.w - xv.w);                                               \
    acc_[i] = a;                                                                        \
  }
        KNN_L1B(acc0, 0) KNN_L1B(acc1, 1) KNN_L1B(acc2, 2) KNN_L1B(acc3, 3)
#undef KNN_L1B
      }
    }
    if (c == nch - 1) {
      select_block<R>(acc0, t * TRS + 0, h, L, I, thr);
      select_block<R>(acc1, t * TRS + 32, h, L, I, thr);
      select_block<R>(acc2, t * TRS + 64, h, L, I, thr);
      select_block<R>(acc3, t * TRS + 96, h, L, I, thr);
    }
    if (more) KNN_SSTORE(st + 1, (st + 1) & 1);
    __syncthreads();
  }
  write_lists<R>(out_v, out_i, qg, S, split, h, L, I);
#undef KNN_SLOAD
#undef KNN_SSTORE
}

#define KNN_DP_LIST(X) X(8) X(16) X(24) X(32) X(48) X(64) X(96) X(128) X(160) X(192) X(256)

int pad_dim(int d) {
#define KNN_CASE(v) if (d <= v) return v;
  KNN_DP_LIST(KNN_CASE)
#undef KNN_CASE
  return (d + kStreamDC - 1) / kStreamDC * kStreamDC;  // streamed kernel
}

bool cand_supported(int DP) { return DP > 0 && pad_dim(DP) == DP; }

// bf16x3 path: resident kernel only (DP multiple of 16, <= 256).
int pad_dim_bf16x3(int d) {
  const int DP = pad_dim((d + 15) / 16 * 16);
  return (DP <= 256 && DP % 16 == 0) ? DP : -1;
}

template <class KernelT>
static int occupancy_of(KernelT k, int threads) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, threads, 0) != hipSuccess) return 1;
  return nb > 0 ? nb : 1;
}

template <int DP, int R, int METRIC, int NW>
static void launch_res(const CandLaunch& c, hipStream_t s) {
  hipLaunchKernelGGL((cand_kernel<DP, R, METRIC, NW>), dim3((unsigned)(c.n_qt * c.S)),
                     dim3(NW * 64), 0, s, c.X32, c.Q32, (int)(c.n_pad / kTR), c.S, c.n_qt,
                     c.out_v, c.out_i, c.ablate);
}
template <int R, int METRIC>
static void launch_str(const CandLaunch& c, hipStream_t s) {
  hipLaunchKernelGGL((cand_stream_kernel<kStreamDC, R, METRIC>), dim3((unsigned)(c.n_qt * c.S)),
                     dim3(256), 0, s, c.X32, c.xinit, c.Q32, c.DP, (int)(c.n_pad / 128), c.S,
                     c.n_qt, c.out_v, c.out_i);
}

// Compile-time dispatch over (R, METRIC): R in {4, 8, 16}; METRIC 0/1/2
// (2 = bf16x3, resident kernel with DP % 16 == 0 only).
template <class F>
static void with_R(int R, F f) {
  if (R == 8) f(std::integral_constant<int, 8>{});
  else f(std::integral_constant<int, 16>{});
}
template <class F>
static void with_M(int M, F f) {
  if (M == 0) f(std::integral_constant<int, 0>{});
  else if (M == 1) f(std::integral_constant<int, 1>{});
  else f(std::integral_constant<int, 2>{});
}

// Instantiated variants: R in {8, 16}; METRIC 0/2 with NW in {4, 8};
// METRIC 1 (L1, not perf-graded) with NW = 4; METRIC 2 needs DP % 16 == 0.
template <int DP, int R, int M, int NW>
constexpr bool res_variant() {
  return (M != 2 || DP % 16 == 0) && (M != 1 || NW == 4);
}

template <int DP>
static int blocks_per_cu_res(int R, int metric, int nw) {
  int out = 1;
  with_R(R, [&](auto Rc) {
    with_M(metric, [&](auto Mc) {
      if (nw == 8) {
        if constexpr (res_variant<DP, Rc.value, Mc.value, 8>())
          out = occupancy_of(cand_kernel<DP, Rc.value, Mc.value, 8>, 512);
      } else {
        if constexpr (res_variant<DP, Rc.value, Mc.value, 4>())
          out = occupancy_of(cand_kernel<DP, Rc.value, Mc.value, 4>, 256);
      }
    });
  });
  return out;
}

int cand_blocks_per_cu(int metric, int DP, int R, int nw) {
#define KNN_CASE(v) if (DP == v) return blocks_per_cu_res<v>(R, metric, nw);
  KNN_DP_LIST(KNN_CASE)
#undef KNN_CASE
  int out = 1;
  with_R(R, [&](auto Rc) {
    if (metric == 1) out = occupancy_of(cand_stream_kernel<kStreamDC, Rc.value, 1>, 256);
    else out = occupancy_of(cand_stream_kernel<kStreamDC, Rc.value, 0>, 256);
  });
  return out;
}

int cand_tile_rows(int DP) { return DP <= 256 ? kTR : 128; }

template <int DP>
static void launch_res_dp(const CandLaunch& c, hipStream_t s) {
  with_R(c.R, [&](auto Rc) {
    with_M(c.metric, [&](auto Mc) {
      if (c.nw == 8) {
        if constexpr (res_variant<DP, Rc.value, Mc.value, 8>())
          launch_res<DP, Rc.value, Mc.value, 8>(c, s);
      } else {
        if constexpr (res_variant<DP, Rc.value, Mc.value, 4>())
          launch_res<DP, Rc.value, Mc.value, 4>(c, s);
      }
    });
  });
}

void launch_cand(const CandLaunch& c, hipStream_t s) {
#define KNN_CASE(v)                \
  if (c.DP == v) {                 \
    launch_res_dp<v>(c, s);        \
    return;                        \
  }
  KNN_DP_LIST(KNN_CASE)
#undef KNN_CASE
  with_R(c.R, [&](auto Rc) {
    if (c.metric == 1) launch_str<Rc.value, 1>(c, s);
    else launch_str<Rc.value, 0>(c, s);
  });
}

// ------------------------------------------------ finish: vote / outputs
// Sorted exact neighbours (dk ascending, di local train index) are in LDS;
// ls[t] already holds the label of entry t for t < needed.  One wave.
//
// Vote (cpp:324-337): scanning t = 0..k-1, label l_t's running count
// c_t = #{s <= t : l_s == l_t}; the reference keeps the label whose count
// first strictly exceeds the running max, i.e. l at the first t reaching
// max_t c_t.  max_label = -1 when k == 0.
__device__ void finish_single(int64_t q, const double* dk, const int* di, const int* ls, int cnt,
                              int k, int64_t idx_off, int flag0, const Sink& sink) {
  const int lane = threadIdx.x & 63;
  int bc = 0, bt = INT_MAX;
  for (int t = lane; t < k; t += 64) {
    const int lt = ls[t];
    int c = 0;
    for (int s2 = 0; s2 <= t; ++s2) c += (ls[s2] == lt);
    if (c > bc) { bc = c; bt = t; }
  }
  const int M = wave_max_i(bc);
  const int tmin = wave_min_i(bc == M ? bt : INT_MAX);
  int tie = 0;
  for (int t = lane; t + 1 < k; t += 64)
    if (dk[t] == dk[t + 1]) tie |= ls[t] != ls[t + 1] ? 4 : 8;  // TIE_VOTE / TIE_ORDER
  tie = wave_or_i(tie);
  if (lane == 0) {
    sink.labels[q] = k > 0 ? ls[tmin] : -1;
    if (sink.flags) {
      int f = flag0 | tie;
      if (k > 0 && k < cnt && dk[k - 1] == dk[k]) f |= 2;  // KNN_FLAG_TIE_BOUNDARY
      sink.flags[q] = f;
    }
  }
  for (int t = lane; t < k; t += 64) {
    if (sink.idx) sink.idx[q * k + t] = (int64_t)di[t] + idx_off;
    if (sink.dist) sink.dist[q * k + t] = dk[t];
  }
}

__device__ void finish_partial(int64_t q, const double* dk, const int* di, const int* ls,
                               int cnt, int w, int64_t idx_off, const Sink& sink) {
  const int lane = threadIdx.x & 63;
  for (int t = lane; t < w; t += 64) {
    const bool ok = t < cnt;
    sink.dist[q * w + t] = ok ? dk[t] : KNN_INF_D;
    sink.idx[q * w + t] = ok ? (int64_t)di[t] + idx_off : -1;
    sink.plab[q * w + t] = ok ? ls[t] : -1;
  }
}

// --------------------------------------------- merge + exact re-rank
// One wave per query.  Dynamic LDS: dk[C2] f64 | di[C2] | ls[C2] | uk[U2] f32 | ui[U2].
template <int METRIC>
__global__ void __launch_bounds__(64)
merge_rerank_kernel(const float* __restrict__ cv, const int* __restrict__ ci, int U, int U2,
                    int R, TrainDev t, const double* __restrict__ Q64, int W, int C, int C2,
                    double f_err, Sink sink, int* __restrict__ rescan_q,
                    int* __restrict__ rescan_cnt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* dk = (double*)smem;
  int* di = (int*)(dk + C2);
  int* ls = di + C2;
  float* uk = (float*)(ls + C2);
  int* ui = (int*)(uk + U2);
  const int64_t q = blockIdx.x;
  const int lane = threadIdx.x;
  const int d = t.d;

  // 1. union of the 2S lists; min over lists of their worst kept entry
  const float* lv = cv + q * U;
  const int* li = ci + q * U;
  float mlr = KNN_INF_F;
  for (int e = lane; e < U2; e += 64) {
    float v = KNN_INF_F;
    int id = INT_MAX;
    if (e < U) {
      v = lv[e];
      if (v < KNN_INF_F) id = li[e];
      if ((e % R) == R - 1) mlr = fminf(mlr, v);
    }
    uk[e] = v;
    ui[e] = id;
  }
  mlr = wave_min(mlr);
  bitonic_sort_lds(uk, ui, U2, lane, 64);
  int nv = 0;
  for (int e = lane; e < U2; e += 64) nv += (uk[e] < KNN_INF_F);
  nv = wave_sum_i(nv);

  // 2. best C by the fp32 proxy; lower bound of every row not re-ranked
  const int Cn = min(C, nv);
  const float T = Cn < nv ? uk[Cn] : KNN_INF_F;
  const float LBa = fminf(T, mlr);

  // 3. exact fp64 distances for the C best, sorted by (dist, idx)
  const double* qrow = Q64 + q * d;
  for (int c = lane; c < C2; c += 64) {
    double v = KNN_INF_D;
    int id = INT_MAX;
    if (c < Cn) {
      id = ui[c];
      v = exact_dist<METRIC>(qrow, t.X64 + (int64_t)id * d, d);
    }
    dk[c] = v;
    di[c] = id;
  }
  bitonic_sort_lds(dk, di, C2, lane, 64);

  // 4. certification: every excluded row has proxy >= LBa, so its exact
  //    distance is >= the bound below (rigorous fp32 error bound f_err).
  bool cert;
  if (!(LBa < KNN_INF_F)) {
    cert = true;  // every row was re-ranked exactly
  } else if (Cn < W) {
    cert = false;
  } else {
    double qa = 0.0;
    for (int c = lane; c < d; c += 64) {
      const double x = qrow[c];
      qa += METRIC == 0 ? x * x : __builtin_fabs(x);
    }
    qa = wave_sum_d(qa) * (1.0 + 1e-12);
    const double dw = dk[W - 1];
    if (METRIC == 0) {
      const double E = f_err * (t.x2max + 2.1 * __builtin_sqrt(qa) * __builtin_sqrt(t.x2max)) + 1e-30;
      const double bound = ((double)LBa + qa * (1.0 - 2e-12) - E) * (1.0 - 1e-12);
      cert = bound > dw * dw * (1.0 + 1e-12);
    } else {
      const double E = f_err * (qa + t.x1max) + 1e-30;
      const double bound = ((double)LBa - E) * (1.0 - 1e-12);
      cert = bound > dw * (1.0 + 1e-12);
    }
  }
  if (!cert) {
    if (lane == 0) {
      const int s = atomicAdd(rescan_cnt, 1);
      rescan_q[s] = (int)q;
    }
    return;
  }

  // 5. outputs
  const int need = sink.mode == MODE_SINGLE ? sink.k : sink.w;
  for (int c = lane; c < need && c < Cn; c += 64) ls[c] = t.lab[di[c]];
  __syncthreads();
  if (sink.mode == MODE_SINGLE)
    finish_single(q, dk, di, ls, Cn, sink.k, sink.idx_off, 0, sink);
  else
    finish_partial(q, dk, di, ls, Cn, sink.w, sink.idx_off, sink);
}

void launch_merge_rerank(int metric, const float* cv, const int* ci, int NL, int R,
                         const TrainDev& t, const double* Q64, int64_t m, int W, int C,
                         double f_err, const Sink& sink, int* rescan_q, int* rescan_cnt,
                         hipStream_t s) {
  const int U = NL * R;
  int U2 = 1;
  while (U2 < U) U2 <<= 1;
  int C2 = 1;
  while (C2 < C) C2 <<= 1;
  const size_t lds = (size_t)C2 * (8 + 4 + 4) + (size_t)U2 * 8;
  if (metric == 0)
    hipLaunchKernelGGL((merge_rerank_kernel<0>), dim3((unsigned)m), dim3(64), lds, s, cv, ci, U,
                       U2, R, t, Q64, W, C, C2, f_err, sink, rescan_q, rescan_cnt);
  else
    hipLaunchKernelGGL((merge_rerank_kernel<1>), dim3((unsigned)m), dim3(64), lds, s, cv, ci, U,
                       U2, R, t, Q64, W, C, C2, f_err, sink, rescan_q, rescan_cnt);
}

// ------------------------------------------------------ exact rescan path
// Queries whose candidate set is not certified (near-duplicate clusters,
// large exact-tie groups, adversarial row orders) are re-done exactly:
// every row's fp64 reference distance, kSortN rows per block sorted in LDS,
// the best W per block kept, then lists reduced by the same sort until one
// remains.  Rare by construction; correctness path, not the fast path.
template <int METRIC>
__global__ void __launch_bounds__(256)
rescan_chunk_kernel(TrainDev t, const double* __restrict__ Q64, const int* __restrict__ rescan_q,
                    int f0, int W, int n_chunks, double* __restrict__ pk, int* __restrict__ pi) {
  __shared__ double sk[kSortN];
  __shared__ int si[kSortN];
  const int chunk = blockIdx.x;
  const int64_t q = rescan_q[f0 + blockIdx.y];
  const double* qrow = Q64 + q * t.d;
  for (int e = threadIdx.x; e < kSortN; e += 256) {
    const int64_t row = (int64_t)chunk * kSortN + e;
    double v = KNN_INF_D;
    int id = INT_MAX;
    if (row < t.n) {
      v = exact_dist<METRIC>(qrow, t.X64 + row * t.d, t.d);
      id = (int)row;
    }
    sk[e] = v;
    si[e] = id;
  }
  bitonic_sort_lds(sk, si, kSortN, threadIdx.x, 256);
  const int64_t o = ((int64_t)blockIdx.y * n_chunks + chunk) * W;
  for (int e = threadIdx.x; e < W; e += 256) {
    pk[o + e] = sk[e];
    pi[o + e] = si[e];
  }
}

__global__ void __launch_bounds__(256)
rescan_reduce_kernel(const double* __restrict__ ik, const int* __restrict__ ii, int P, int W,
                     int G, double* __restrict__ ok, int* __restrict__ oi, int P2) {
  __shared__ double sk[kSortN];
  __shared__ int si[kSortN];
  const int b = blockIdx.x, f = blockIdx.y;
  const int l0 = b * G, l1 = min(P, l0 + G);
  const int ne = (l1 - l0) * W;
  const int64_t src = ((int64_t)f * P + l0) * W;
  for (int e = threadIdx.x; e < kSortN; e += 256) {
    sk[e] = e < ne ? ik[src + e] : KNN_INF_D;
    si[e] = e < ne ? ii[src + e] : INT_MAX;
  }
  bitonic_sort_lds(sk, si, kSortN, threadIdx.x, 256);
  const int64_t o = ((int64_t)f * P2 + b) * W;
  for (int e = threadIdx.x; e < W; e += 256) {
    ok[o + e] = sk[e];
    oi[o + e] = si[e];
  }
}

__global__ void __launch_bounds__(64)
rescan_finish_kernel(TrainDev t, const double* __restrict__ pk, const int* __restrict__ pi,
                     const int* __restrict__ rescan_q, int f0, int W, Sink sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* dk = (double*)smem;
  int* di = (int*)(dk + W);
  int* ls = di + W;
  const int f = blockIdx.x;
  const int64_t q = rescan_q[f0 + f];
  const int lane = threadIdx.x;
  const int cnt = (int)(t.n < W ? t.n : W);
  for (int e = lane; e < W; e += 64) {
    dk[e] = pk[(int64_t)f * W + e];
    di[e] = pi[(int64_t)f * W + e];
    ls[e] = e < cnt ? t.lab[di[e]] : -1;
  }
  __syncthreads();
  if (sink.mode == MODE_SINGLE)
    finish_single(q, dk, di, ls, cnt, sink.k, sink.idx_off, 1 /*KNN_FLAG_EXACT_RESCAN*/, sink);
  else
    finish_partial(q, dk, di, ls, cnt, sink.w, sink.idx_off, sink);
}

size_t rescan_scratch_entries(int64_t n, int W) {
  const int64_t n_chunks = (n + kSortN - 1) / kSortN;
  return (size_t)n_chunks * W;
}

void launch_rescan(int metric, const TrainDev& t, const double* Q64, const int* rescan_q,
                   int f0, int nf, int W, double* pa_k, int* pa_i, double* pb_k, int* pb_i,
                   const Sink& sink, hipStream_t s) {
  const int n_chunks = (int)((t.n + kSortN - 1) / kSortN);
  if (metric == 0)
    hipLaunchKernelGGL((rescan_chunk_kernel<0>), dim3(n_chunks, nf), dim3(256), 0, s, t, Q64,
                       rescan_q, f0, W, n_chunks, pa_k, pa_i);
  else
    hipLaunchKernelGGL((rescan_chunk_kernel<1>), dim3(n_chunks, nf), dim3(256), 0, s, t, Q64,
                       rescan_q, f0, W, n_chunks, pa_k, pa_i);
  int P = n_chunks;
  double* ik = pa_k; int* ii = pa_i;
  double* ok = pb_k; int* oi = pb_i;
  const int G = kSortN / W;  // W <= kMaxK + 1 <= kSortN / 2
  while (P > 1) {
    const int P2 = (P + G - 1) / G;
    hipLaunchKernelGGL(rescan_reduce_kernel, dim3(P2, nf), dim3(256), 0, s, ik, ii, P, W, G, ok,
                       oi, P2);
    double* tk = ik; ik = ok; ok = tk;
    int* ti = ii; ii = oi; oi = ti;
    P = P2;
  }
  const size_t lds = (size_t)W * 16;
  hipLaunchKernelGGL(rescan_finish_kernel, dim3(nf), dim3(64), lds, s, t, ik, ii, rescan_q, f0,
                     W, sink);
}

// ------------------------------------------ train-sharded k-way merge + vote
// lists [parts][m][w] sorted by (dist, global idx); one wave per query merges
// them (bitonic in LDS) and runs the reference vote on the first k.
__global__ void __launch_bounds__(64)
merge_vote_partials_kernel(const double* __restrict__ dist, const int64_t* __restrict__ idx,
                           const int32_t* __restrict__ lab, int parts, int64_t m, int w, int k,
                           int P2, int64_t q0, Sink sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* dk = (double*)smem;
  int64_t* gi = (int64_t*)(dk + P2);
  int* ls = (int*)(gi + P2);
  const int64_t q = q0 + blockIdx.x;  // query in the [parts][m][w] lists
  const int64_t qo = blockIdx.x;      // row in the outputs
  const int lane = threadIdx.x;
  const int ne = parts * w;
  for (int e = lane; e < P2; e += 64) {
    double v = KNN_INF_D;
    int64_t id = LLONG_MAX;
    if (e < ne) {
      const int p = e / w, c = e - p * w;
      const int64_t src = ((int64_t)p * m + q) * w + c;
      if (idx[src] >= 0) { v = dist[src]; id = idx[src]; }
    }
    dk[e] = v;
    gi[e] = id;
  }
  bitonic_sort_lds(dk, gi, P2, lane, 64);
  // labels travel with the lists: place each one at its entry's sorted slot
  for (int e = lane; e < ne; e += 64) {
    const int p = e / w, c = e - p * w;
    const int64_t src = ((int64_t)p * m + q) * w + c;
    if (idx[src] < 0) continue;
    // position of (dist, idx) in the sorted array: binary search
    const double v = dist[src];
    const int64_t id = idx[src];
    int lo = 0, hi = P2;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (pair_less(dk[mid], gi[mid], v, id)) lo = mid + 1; else hi = mid;
    }
    if (lo < k + 1) ls[lo] = lab[src];
  }
  __syncthreads();
  int cnt = 0;
  for (int e = lane; e < P2; e += 64) cnt += (gi[e] != LLONG_MAX);
  cnt = wave_sum_i(cnt);
  int bc = 0, bt = INT_MAX;
  for (int t = lane; t < k; t += 64) {
    const int lt = ls[t];
    int c = 0;
    for (int s2 = 0; s2 <= t; ++s2) c += (ls[s2] == lt);
    if (c > bc) { bc = c; bt = t; }
  }
  const int M = wave_max_i(bc);
  const int tmin = wave_min_i(bc == M ? bt : INT_MAX);
  int tie = 0;
  for (int t = lane; t + 1 < k; t += 64)
    if (dk[t] == dk[t + 1]) tie |= ls[t] != ls[t + 1] ? 4 : 8;
  tie = wave_or_i(tie);
  if (lane == 0) {
    sink.labels[qo] = k > 0 ? ls[tmin] : -1;
    if (sink.flags) {
      int f = tie;
      if (k > 0 && k < cnt && dk[k - 1] == dk[k]) f |= 2;
      sink.flags[qo] = f;
    }
  }
  for (int t = lane; t < k; t += 64) {
    if (sink.idx) sink.idx[qo * k + t] = gi[t];
    if (sink.dist) sink.dist[qo * k + t] = dk[t];
  }
}

void launch_merge_vote_partials(const double* dist, const int64_t* idx, const int32_t* lab,
                                int parts, int64_t m, int w, int k, int32_t* out_lab,
                                int64_t* out_idx, double* out_dist, int32_t* out_flags,
                                hipStream_t s, int64_t q0, int64_t mq) {
  if (mq < 0) mq = m - q0;
  if (mq <= 0) return;
  int P2 = 1;
  while (P2 < parts * w) P2 <<= 1;
  Sink sink{};
  sink.mode = MODE_SINGLE;
  sink.k = k;
  sink.labels = out_lab;
  sink.idx = out_idx;
  sink.dist = out_dist;
  sink.flags = out_flags;
  const size_t lds = (size_t)P2 * (8 + 8 + 4);
  hipLaunchKernelGGL(merge_vote_partials_kernel, dim3((unsigned)mq), dim3(64), lds, s, dist, idx,
                     lab, parts, m, w, k, P2, q0, sink);
}

}  // namespace knnk
