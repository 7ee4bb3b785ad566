// knn_device.h -- device helpers shared by the gfx950 kernel translation
// units (knn_prep.hip, knn_cand*.hip, knn_select.hip).  Internal.
#pragma once
#include "knn_kernels.h"

#include <float.h>
#include <limits.h>

#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

#pragma clang fp contract(off)

namespace knnk {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

#define KNN_INF_F __builtin_inff()
// Timing-only kernel ablations (tuning key "ablate", bits 0/1/3/4) are
// compiled in only with -DKNN_ABLATIONS=1 (tools/build_variant.sh): in the
// production build the candidate kernels carry no per-tile checks for them.
#ifndef KNN_ABLATIONS
#define KNN_ABLATIONS 0
#endif
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
__device__ __forceinline__ uint32_t wave_min_u(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_max_u(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
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

// NaN / inf test on the exponent bits, usable in every TU.  The bits pass
// through an empty asm first: LLVM rewrites the plain mask test into an
// fp-class test (is-inf-or-nan), and under -fno-honor-nans it then drops the
// NaN half -- measured on the large-k path: a NaN query went through as
// finite while -inf was caught.
// train row of candidate-image row (position) p (region order)
__device__ __forceinline__ int train_row(const TrainDev& t, int p) { return t.perm ? t.perm[p] : p; }

// Source row of image row `row` under an optional permutation (region order,
// knn_order.hip): perm[row] for real rows, the row itself otherwise.
__device__ __forceinline__ int64_t src_row(const int* perm, int64_t row, int64_t n) {
  return perm && row < n ? (int64_t)perm[row] : row;
}

__device__ __forceinline__ bool nonfinite_bits(double x) {
  long long b = __double_as_longlong(x);
  asm volatile("" : "+v"(b));
  return (b & 0x7FF0000000000000ll) == 0x7FF0000000000000ll;
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

// The fp16 candidate operand of an fp64 value: one rounding of v * 2^jx.
// Shared by every fp16 image builder and by the merge, which rebuilds a
// query's operands to measure their representation error.
__device__ __forceinline__ _Float16 f16_operand(double v, int jx) {
  return (_Float16)__builtin_ldexp(v, jx);
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

// fp16 kernel (KNN_M4_FAST): the fp16 resident kernel's no-candidate test as
// a v_min3 tree + wave-uniform branch and med3 list shifts
// (continuous cfg2: candidate kernel 2.43-2.44 -> 2.33-2.35 ms in 3
// interleaved process pairs, profiles/ab_log.md r6f)
#ifndef KNN_M4_FAST
#define KNN_M4_FAST 1
#endif
// the S3 kernel's quad selection (select_quad_f) in the same form
#ifndef KNN_S3_FAST
#define KNN_S3_FAST 0
#endif
// list_insert with each tail shift one v_med3_f32: for L[t-1] <= L[t] the
// median of (v, L[t], L[t-1]) is max(L[t-1], min(v, L[t])) (no NaNs: the
// candidate values are finite or +inf)
template <int R>
__device__ __forceinline__ void list_insert_med3(float (&L)[R], int (&I)[R], float v, int id) {
  bool cc = true;  // v < L[R-1] by precondition
#pragma unroll
  for (int t = R - 1; t > 0; --t) {
    const bool cp = v < L[t - 1];
    float r;
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(v), "v"(L[t]), "v"(L[t - 1]));
    L[t] = r;
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

// Order-preserving float <-> uint32 keys (unsigned compares order like the
// floats; +inf -> 0xFF800000).
__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return u ^ ((u >> 31) ? 0xFFFFFFFFu : 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k >> 31) ? (k ^ 0x80000000u) : ~k);
}
constexpr uint32_t kKeyInf = 0xFF800000u;  // f2key(+inf)

// Fused top-R selection over one 32x32 accumulator block: lane (j, h) holds
// the values of query j against rows row0 + rho(i, h), i = 0..15.  Once the
// list is warm this is a 16-way min (v_min3) and one compare per block; a
// value is inserted only under a branch that no lane of the wave skips.
// tq: an extra filter bound valid for the whole query (the global per-query
// threshold of cand_kernel, +inf elsewhere).
template <int R>
__device__ __forceinline__ void select_block(const f32x16& acc, int row0, int h, float (&L)[R],
                                             int (&I)[R], float& thr, float tq) {
  // Lanes l and l^32 hold the same query: filtering with the smaller of the
  // two list thresholds is safe -- anything dropped is >= some list's final
  // R-th entry, which the merge's lower bound (min over lists) accounts for.
  // v_permlane32_swap of thr with itself: r[0] = lower half, r[1] = upper
  // half of every lane pair, so min(r[0], r[1]) = min over lanes l, l^32
  // (one VALU op instead of an LDS ds_bpermute round trip).
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(thr), __float_as_uint(thr),
                                                   false, false);
  float te = __builtin_fminf(__builtin_fminf(__uint_as_float(sw[0]), __uint_as_float(sw[1])), tq);
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

// min over the 4 lanes l&15 + 16r (r = 0..3) that hold the same query in the
// 16x16 MFMA layout
__device__ __forceinline__ float quad_min(float x) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                   false);
  x = __builtin_fminf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
  // v_permlane16_swap: r[0], r[1] = the values of lanes l and l^16 (in some
  // order) -- a VALU op, no LDS round trip as a ds_swizzle would take
  const auto s2 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                   false);
  return __builtin_fminf(__uint_as_float(s2[0]), __uint_as_float(s2[1]));
}

// Top-R selection for the 16x16 layout: 8 values of one query (rows row0 + i
// of block a, row0 + 16 + i of block b), threshold shared by the query's 4
// lanes (each keeps its own list; the merge's bound is the min over lists).
template <int R>
__device__ __forceinline__ void select_quad(const f32x4& a, const f32x4& b, int row0,
                                            float (&L)[R], int (&I)[R], float& thr, float tq) {
  float te = __builtin_fminf(quad_min(thr), tq);
  const float mn = __builtin_fminf(__builtin_fminf(__builtin_fminf(a[0], a[1]),
                                                   __builtin_fminf(a[2], a[3])),
                                   __builtin_fminf(__builtin_fminf(b[0], b[1]),
                                                   __builtin_fminf(b[2], b[3])));
  if (mn < te) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float v = i < 4 ? a[i] : b[i - 4];
      if (v < te) {
        list_insert<R>(L, I, v, row0 + (i < 4 ? i : 16 + i - 4));
        thr = L[R - 1];
        te = __builtin_fminf(te, thr);
      }
    }
  }
}

// select_quad with a filter tf fixed by the caller for a whole tile (the
// quad's shared threshold at the tile's start) and this lane's own R-th entry:
// no cross-lane operation per call.
template <int R>
__device__ __forceinline__ void select_quad_f(const f32x4& a, const f32x4& b, int row0,
                                              float (&L)[R], int (&I)[R], float tf) {
  float te = __builtin_fminf(tf, L[R - 1]);
#if KNN_S3_FAST
  // (as select_quad_te with KNN_M4_FAST: v_min3 tree, wave-uniform branch,
  // med3 list shifts)
  const float m1 = __builtin_fminf(__builtin_fminf(a[0], a[1]), a[2]);
  const float m2 = __builtin_fminf(__builtin_fminf(a[3], b[0]), b[1]);
  const float m3 = __builtin_fminf(__builtin_fminf(b[2], b[3]), m1);
  if (__builtin_amdgcn_ballot_w64(__builtin_fminf(m2, m3) < te)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float v = i < 4 ? a[i] : b[i - 4];
      if (v < te) {
        list_insert_med3<R>(L, I, v, row0 + (i < 4 ? i : 16 + i - 4));
        te = __builtin_fminf(te, L[R - 1]);
      }
    }
  }
#else
  const float mn = __builtin_fminf(__builtin_fminf(__builtin_fminf(a[0], a[1]),
                                                   __builtin_fminf(a[2], a[3])),
                                   __builtin_fminf(__builtin_fminf(b[0], b[1]),
                                                   __builtin_fminf(b[2], b[3])));
  if (mn < te) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float v = i < 4 ? a[i] : b[i - 4];
      if (v < te) {
        list_insert<R>(L, I, v, row0 + (i < 4 ? i : 16 + i - 4));
        te = __builtin_fminf(te, L[R - 1]);
      }
    }
  }
#endif
}

// select_quad with the quad's filter te kept by the caller (refreshed from
// the 4 lanes' thresholds once per staged tile); an insertion lowers it to
// this lane's new R-th entry.  thr is then L[R-1] and needs no copy.
// row + c computed where it is used: a plain add is hoisted out of the
// insertion branch by the compiler and then costs one VALU op per value on
// every tile, inserting or not
#ifndef KNN_ROW_AT
#define KNN_ROW_AT 1
#endif
__device__ __forceinline__ int row_at(int row0, int c) {
#if KNN_ROW_AT
  int r;
  asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(row0), "i"(c));
  return r;
#else
  return row0 + c;
#endif
}

// The 4 smallest of the union of two ascending 4-lists, ascending: the
// elementwise min of a and reversed b is bitonic and holds them; two
// compare-exchange stages sort it.
__device__ __forceinline__ void merge_top4(float (&a)[4], const float (&b)[4]) {
  float m0 = __builtin_fminf(a[0], b[3]), m1 = __builtin_fminf(a[1], b[2]);
  float m2 = __builtin_fminf(a[2], b[1]), m3 = __builtin_fminf(a[3], b[0]);
  const float n0 = __builtin_fminf(m0, m2), n2 = __builtin_fmaxf(m0, m2);
  const float n1 = __builtin_fminf(m1, m3), n3 = __builtin_fmaxf(m1, m3);
  a[0] = __builtin_fminf(n0, n1);
  a[1] = __builtin_fmaxf(n0, n1);
  a[2] = __builtin_fminf(n2, n3);
  a[3] = __builtin_fmaxf(n2, n3);
}

// K-th smallest (K in 1..4, wave-uniform) of the union of the ascending
// lists t[0..3] held by lanes l and l^32 (LANES = 2) or by the four lanes
// l&15 + 16r (LANES = 4, the 16x16 MFMA layout's quad).  The lanes hold
// disjoint row sets, so the result has >= K distinct rows at or below it.
template <int LANES>
__device__ __forceinline__ float union_kth(const float (&t)[4], int K) {
  float lo[4], hi[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    // r[0] = the value of lane l&31, r[1] = that of lane (l&31)+32
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(t[e]), __float_as_uint(t[e]),
                                                    false, false);
    lo[e] = __uint_as_float(r[0]);
    hi[e] = __uint_as_float(r[1]);
  }
  merge_top4(lo, hi);
  if constexpr (LANES == 4) {
    float a[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      // the lists of lanes l and l^16 (order irrelevant: the merge is symmetric)
      const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo[e]),
                                                      __float_as_uint(lo[e]), false, false);
      a[e] = __uint_as_float(r[0]);
      hi[e] = __uint_as_float(r[1]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) lo[e] = a[e];
    merge_top4(lo, hi);
  }
  return K <= 1 ? lo[0] : K == 2 ? lo[1] : K == 3 ? lo[2] : lo[3];
}

// Ascending sort of a bitonic sequence of N (power of two) in registers.
template <int N>
__device__ __forceinline__ void bitonic_sort_reg(float (&x)[N]) {
#pragma unroll
  for (int st = N / 2; st > 0; st >>= 1) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if ((i & st) == 0) {
        const float lo = __builtin_fminf(x[i], x[i + st]), hi = __builtin_fmaxf(x[i], x[i + st]);
        x[i] = lo;
        x[i + st] = hi;
      }
    }
  }
}

// K-th smallest (K in 1..16, wave-uniform) of the union of the ascending
// 8-lists t held by the four lanes l&15 + 16r (the 16x16 layout's quad):
// both 8-lists of lanes l, l^32 merged into a sorted 16, then the 16
// smallest of that and lane l^16's 16.  Rows of different lanes are
// distinct, so >= K distinct rows lie at or below the result.
__device__ __forceinline__ float quad_union_kth16(const float (&t)[8], int K) {
  float a[16], b[16];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(t[e]), __float_as_uint(t[e]),
                                                    false, false);
    a[e] = __uint_as_float(r[0]);       // ascending
    a[15 - e] = __uint_as_float(r[1]);  // descending: a is bitonic
  }
  bitonic_sort_reg<16>(a);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[e]), __float_as_uint(a[e]),
                                                    false, false);
    a[e] = __uint_as_float(r[0]);
    b[e] = __uint_as_float(r[1]);
  }
  // the 16 smallest of two ascending 16-lists, as a bitonic sequence
#pragma unroll
  for (int e = 0; e < 16; ++e) a[e] = __builtin_fminf(a[e], b[15 - e]);
  bitonic_sort_reg<16>(a);
  float v = a[0];
#pragma unroll
  for (int e = 1; e < 16; ++e) v = K == e + 1 ? a[e] : v;
  return v;
}

template <int R>
__device__ __forceinline__ void select_quad_te(const f32x4& a, const f32x4& b, int row0,
                                               float (&L)[R], int (&I)[R], float& te) {
#if KNN_M4_FAST
  // 4 v_min3-shaped ops for 8 values and a wave-uniform branch (v_cmp into
  // an SGPR pair + s_cbranch_vccz: no exec save / restore), as the int8
  // kernels; insertions as v_med3_f32 shifts
  const float m1 = __builtin_fminf(__builtin_fminf(a[0], a[1]), a[2]);
  const float m2 = __builtin_fminf(__builtin_fminf(a[3], b[0]), b[1]);
  const float m3 = __builtin_fminf(__builtin_fminf(b[2], b[3]), m1);
  const float mn = __builtin_fminf(m2, m3);
  if (__builtin_amdgcn_ballot_w64(mn < te)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float v = i < 4 ? a[i] : b[i - 4];
      if (v < te) {
        list_insert_med3<R>(L, I, v, row_at(row0, i < 4 ? i : 16 + i - 4));
        te = __builtin_fminf(te, L[R - 1]);
      }
    }
  }
#else
  const float mn = __builtin_fminf(__builtin_fminf(__builtin_fminf(a[0], a[1]),
                                                   __builtin_fminf(a[2], a[3])),
                                   __builtin_fminf(__builtin_fminf(b[0], b[1]),
                                                   __builtin_fminf(b[2], b[3])));
  if (mn < te) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float v = i < 4 ? a[i] : b[i - 4];
      if (v < te) {
        list_insert<R>(L, I, v, row_at(row0, i < 4 ? i : 16 + i - 4));
        te = __builtin_fminf(te, L[R - 1]);
      }
    }
  }
#endif
}

// int8 kernel (metric 5): the accumulators hold acc = q.k - ceil(||k||^2 / 2)
// (exact int32), the proxy is -2 acc = ||k||^2 - 2 q.k (+1 for an odd
// ||k||^2): a row beats the quad filter te (an even integer or +inf) iff
// acc > -te / 2, so the filter runs on the accumulators as they stand (a
// max-tree, no per-value conversion); only an insertion forms the proxy.
typedef int i32x4 __attribute__((ext_vector_type(4)));
// Below every real accumulator: codes and query codes lie in [-128, 127] and
// d <= 256, so q.k >= -2^22 and the seed >= -2^21, i.e. acc > -2^23.  Pad
// rows carry it as their seed (acc = kI8Floor exactly, the codes being 0),
// empty list entries and the empty filter hold it, and the strict test
// acc > tn never selects a pad row.  Keys acc * 8 + position fit in int32.
constexpr int kI8Floor = -(1 << 23);
__device__ __forceinline__ int i8_neg_half(float te) {
  // -te/2 as an int (te: even integers, +inf -> kI8Floor: every real row passes)
  return te > 3.0e38f ? kI8Floor : (int)(-0.5f * te);
}
// tn = i8_neg_half(te), kept by the caller (refreshed with te per tile):
// the no-insertion case is 4 v_max3 + 1 compare per call.
// KNN_I8_UBR: the no-candidate test as a wave-uniform branch (v_cmp into an
// SGPR pair + s_cbranch_vccz) instead of an exec-masked region (cfg2
// candidate pass -1.3 %, profiles/ab_log.md: r3d_ab_*)
#ifndef KNN_I8_UBR
#define KNN_I8_UBR 1
#endif
// KNN_COUNT_SEL (experiment builds only): per-lane counts of the int8
// selection -- calls whose lane passes the filter, calls where some lane of
// the wave does (the slow path runs), values inserted -- summed into
// knn_sel_cnt at the end of cand_kernel (knn_cand_res.hip)
// Candidate kernels: fetch the per-query global thresholds once before the
// first tile (what workgroups of earlier grid rounds published for these
// queries), so the first tile's selection already filters with them instead
// of inserting everything until the first exchange lands
#ifndef KNN_X_START
#define KNN_X_START 1
#endif
#ifndef KNN_COUNT_SEL
#define KNN_COUNT_SEL 0
#endif
struct SelCount {
  unsigned calls = 0, lane_pass = 0, wave_pass = 0, inserts = 0;
  unsigned bcalls = 0, bpass = 0;  // seed-free int8: sub-tile bound tests / waves passing them
  unsigned bcold = 0, bpcold = 0;  // the same in a workgroup's first two staged tiles
};
template <int R>
__device__ __forceinline__ void select_quad_i8(const i32x4& a, const i32x4& b, int row0,
                                               float (&L)[R], int (&I)[R], float& te, int& tn,
                                               SelCount& sc) {
  const int m1 = max(max(a[0], a[1]), a[2]);
  const int m2 = max(max(a[3], b[0]), b[1]);
  const int m3 = max(max(b[2], b[3]), m1);
  const int mx = max(m2, m3);
#if KNN_COUNT_SEL
  sc.calls++;
  sc.lane_pass += mx > tn;
  sc.wave_pass += __builtin_amdgcn_ballot_w64(mx > tn) != 0;
#endif
#if KNN_I8_UBR
  if (__builtin_amdgcn_ballot_w64(mx > tn)) {
#else
  if (mx > tn) {
#endif
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int v = i < 4 ? a[i] : b[i - 4];
      if (v > tn) {
#if KNN_COUNT_SEL
        sc.inserts++;
#endif
        list_insert<R>(L, I, (float)(-2 * v), row_at(row0, i < 4 ? i : 16 + i - 4));
        te = __builtin_fminf(te, L[R - 1]);
        tn = i8_neg_half(te);
      }
    }
  }
}

// int8 kernel lists in the accumulator domain (KNN_I8_ILIST): entries are the
// int32 accumulators themselves, best (largest) first, kI8Floor = empty; the
// proxy -2 acc (a float, exact below 2^24) is formed only where a float is
// needed -- the per-tile exchange and the final write.  An insertion is then
// integer min/max selects and the filter update one v_max (no conversions).
#ifndef KNN_I8_ILIST
#define KNN_I8_ILIST 1
#endif
__device__ __forceinline__ float i8_proxy(int acc) {
  return acc <= kI8Floor ? KNN_INF_F : (float)(-2 * acc);
}
// a list entry as the proxy the merge reads (float lists: itself)
__device__ __forceinline__ float lval(float v) { return v; }
__device__ __forceinline__ float lval(int acc) { return i8_proxy(acc); }
// L[t] = min(L[t-1], max(v, L[t])) in one v_med3_i32 (L[t-1] >= L[t]: the
// median of the three is that clamp); the compiler only forms med3 from
// constant bounds and otherwise emits a v_max + v_min pair per position
#ifndef KNN_MED3
#define KNN_MED3 1
#endif
__device__ __forceinline__ int clamp_desc(int v, int lo, int hi) {
#if KNN_MED3
  int r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(v), "v"(lo), "v"(hi));
  return r;
#else
  return min(hi, max(v, lo));
#endif
}
template <int R>
__device__ __forceinline__ void list_insert_desc(int (&L)[R], int (&I)[R], int v, int id) {
  bool cc = true;  // v > L[R-1] by precondition
#pragma unroll
  for (int t = R - 1; t > 0; --t) {
    const bool cp = v > L[t - 1];
    L[t] = clamp_desc(v, L[t], L[t - 1]);
    I[t] = cp ? I[t - 1] : (cc ? id : I[t]);
    cc = cp;
  }
  I[0] = cc ? id : I[0];
  L[0] = max(v, L[0]);
}
// tn: the quad's filter (i8_neg_half of the tile's te) raised by this lane's
// own insertions; tn >= L[R-1] always, so v > tn meets the insert precondition
template <int R>
__device__ __forceinline__ void select_quad_i8i(const i32x4& a, const i32x4& b, int row0,
                                                int (&L)[R], int (&I)[R], int& tn, SelCount& sc) {
  const int m1 = max(max(a[0], a[1]), a[2]);
  const int m2 = max(max(a[3], b[0]), b[1]);
  const int m3 = max(max(b[2], b[3]), m1);
  const int mx = max(m2, m3);
#if KNN_COUNT_SEL
  sc.calls++;
  sc.lane_pass += mx > tn;
  sc.wave_pass += __builtin_amdgcn_ballot_w64(mx > tn) != 0;
#endif
  if (__builtin_amdgcn_ballot_w64(mx > tn)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int v = i < 4 ? a[i] : b[i - 4];
      if (v > tn) {
#if KNN_COUNT_SEL
        sc.inserts++;
#endif
        list_insert_desc<R>(L, I, v, row_at(row0, i < 4 ? i : 16 + i - 4));
        tn = max(tn, L[R - 1]);
      }
    }
  }
}

// METRIC 6 (v_mfma_i32_32x32x32_i8, the 32x32 layout): lane (j, h) holds
// query j against rows row0 + (i&3) + 8(i>>2), i = 0..15 (row0 includes 4h),
// one list per lane; lanes l and l^32 share the query (pair_min of their
// thresholds is the per-tile filter).  The no-candidate test is a max over
// 16 values; a slow call loops over the half (8 values) that has a pass.
typedef int i32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ float pair_min(float x) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                   false);
  return __builtin_fminf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
}
template <int R>
__device__ __forceinline__ void select_block_i8(const i32x16& a, int row0, int (&L)[R], int (&I)[R],
                                                int& tn, SelCount& sc) {
  const int h0 = max(max(max(a[0], a[1]), max(a[2], a[3])), max(max(a[4], a[5]), max(a[6], a[7])));
  const int h1 = max(max(max(a[8], a[9]), max(a[10], a[11])),
                     max(max(a[12], a[13]), max(a[14], a[15])));
#if KNN_COUNT_SEL
  sc.calls++;
  sc.lane_pass += max(h0, h1) > tn;
  sc.wave_pass += __builtin_amdgcn_ballot_w64(max(h0, h1) > tn) != 0;
#endif
  if (__builtin_amdgcn_ballot_w64(max(h0, h1) > tn)) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (__builtin_amdgcn_ballot_w64((half ? h1 : h0) > tn)) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = 8 * half + e;
          const int v = a[i];
          if (v > tn) {
#if KNN_COUNT_SEL
            sc.inserts++;
#endif
            list_insert_desc<R>(L, I, v, row_at(row0, (i & 3) + 8 * (i >> 2)));
            tn = max(tn, L[R - 1]);
          }
        }
      }
    }
  }
}

// select_block_i8 with two lists per lane (metric 6, KNN_I8W_Q4): values i <
// 8 go to (L, I), i >= 8 to (L2, I2); tn >= both lists' R-th entries
template <int R>
__device__ __forceinline__ void select_block_i8w4(const i32x16& a, int row0, int (&L)[R], int (&I)[R],
                                                  int (&L2)[R], int (&I2)[R], int& tn, SelCount& sc) {
  const int h0 = max(max(max(a[0], a[1]), max(a[2], a[3])), max(max(a[4], a[5]), max(a[6], a[7])));
  const int h1 = max(max(max(a[8], a[9]), max(a[10], a[11])),
                     max(max(a[12], a[13]), max(a[14], a[15])));
#if KNN_COUNT_SEL
  sc.calls++;
  sc.lane_pass += max(h0, h1) > tn;
  sc.wave_pass += __builtin_amdgcn_ballot_w64(max(h0, h1) > tn) != 0;
#endif
  if (__builtin_amdgcn_ballot_w64(h0 > tn)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int v = a[i];
      if (v > tn) {
#if KNN_COUNT_SEL
        sc.inserts++;
#endif
        list_insert_desc<R>(L, I, v, row_at(row0, (i & 3) + 8 * (i >> 2)));
        tn = max(tn, L[R - 1]);
      }
    }
  }
  if (__builtin_amdgcn_ballot_w64(h1 > tn)) {
#pragma unroll
    for (int i = 8; i < 16; ++i) {
      const int v = a[i];
      if (v > tn) {
#if KNN_COUNT_SEL
        sc.inserts++;
#endif
        list_insert_desc<R>(L2, I2, v, row_at(row0, (i & 3) + 8 * (i >> 2)));
        tn = max(tn, L2[R - 1]);
      }
    }
  }
}

// KNN_I8_SLOW = 2: the slow path inserts each lane's best passing value
// first, found with its position by a max over keys acc * 8 + position
// (exact and order-preserving: acc >= kI8Floor = -2^23), and tests the lane's second
// best before the per-value loop: the common slow call (each passing lane
// has one passing value) is one insertion for all its lanes instead of one
// per distinct position, and no per-value exec-mask branches
#ifndef KNN_I8_SLOW
#define KNN_I8_SLOW 1
#endif
template <int R>
__device__ __forceinline__ void select_quad_i8t(const i32x4& a, const i32x4& b, int row0,
                                                int (&L)[R], int (&I)[R], int& tn, SelCount& sc) {
  const int m1 = max(max(a[0], a[1]), a[2]);
  const int m2 = max(max(a[3], b[0]), b[1]);
  const int m3 = max(max(b[2], b[3]), m1);
  const int mx = max(m2, m3);
#if KNN_COUNT_SEL
  sc.calls++;
  sc.lane_pass += mx > tn;
  sc.wave_pass += __builtin_amdgcn_ballot_w64(mx > tn) != 0;
#endif
  if (__builtin_amdgcn_ballot_w64(mx > tn)) {
    int k[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) k[i] = (i < 4 ? a[i] : b[i - 4]) * 8 + i;
    // top two keys of the eight
    int hi[4], lo[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      hi[p] = max(k[2 * p], k[2 * p + 1]);
      lo[p] = min(k[2 * p], k[2 * p + 1]);
    }
    const int hA = max(hi[0], hi[1]), lA = max(min(hi[0], hi[1]), max(lo[0], lo[1]));
    const int hB = max(hi[2], hi[3]), lB = max(min(hi[2], hi[3]), max(lo[2], lo[3]));
    const int k1 = max(hA, hB), k2 = max(min(hA, hB), max(lA, lB));
    int tk = tn * 8 + 7;  // acc > tn  <=>  key > tk (acc, tn >= kI8Floor: no overflow)
    if (k1 > tk) {
#if KNN_COUNT_SEL
      sc.inserts++;
#endif
      const int p = k1 & 7;
      list_insert_desc<R>(L, I, k1 >> 3, row0 + p + 12 * (p >> 2));
      tn = max(tn, L[R - 1]);
      tk = tn * 8 + 7;
    }
    if (__builtin_amdgcn_ballot_w64(k2 > tk)) {  // a lane with more passing values
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (k[i] > tk && k[i] != k1) {
#if KNN_COUNT_SEL
          sc.inserts++;
#endif
          list_insert_desc<R>(L, I, k[i] >> 3, row_at(row0, i < 4 ? i : 16 + i - 4));
          tn = max(tn, L[R - 1]);
          tk = tn * 8 + 7;
        }
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

// fp16 resident-kernel image (XH): 16-B chunk ch of row r's payload is
// stored at chunk ch ^ xh_swz(r).  With the odd row stride of DP/8 + 1 chunks
// the 16x16x32 A-fragment reads (lane l: row l & 15, chunk 4ks + (l >> 4))
// then hit 16 distinct 16-B bank groups in every 16-lane group of a
// ds_read_b128 for every DP the kernel serves; unswizzled, each group had a
// 2-way conflict at DP = 128 (4 extra LDS cycles per read) and more at
// other DPs (exhaustive check over DP = 32 .. 256).
__device__ __forceinline__ int xh_swz(int r) { return ((r >> 2) ^ (r >> 3)) & 1; }

// S3 (bf16x3, DP > 256) image geometry; see knn_cand.hip
constexpr int kS3Q = 256;   // queries per workgroup
constexpr int kS3R = 256;   // train rows per tile
constexpr int kS3DC = 16;   // dims per staged chunk

__device__ __forceinline__ int s3_slot(int r, int s) { return s ^ ((r >> 2) & 3); }
// fp16 S3 images: slot s of row r at s ^ g((r >> 2) & 3), g = (0, 2, 3, 1).
// Conflict-free for both read patterns of a 16-B-per-lane ds_read_b128:
// the 32x32x16 one (lanes on rows 0-31, one slot per half-wave) and the
// 16x16x32 one (lanes on rows l & 15, slot l >> 4): every 16-lane group of the
// instruction lands on 16 distinct 16-B bank groups.
__device__ __forceinline__ int s3h_swz(int q) { return (0x78 >> (2 * (q & 3))) & 3; }
__device__ __forceinline__ int s3h_slot(int r, int s) { return s ^ s3h_swz(r >> 2); }

// Resident workgroups per CU of a kernel variant: a property of the code
// object (registers, LDS), asked of the runtime once per (kernel, block
// size) and cached -- choose_geometry runs on every classify call, which
// must stay enqueue-only with no runtime queries in the timed loop.
template <class KernelT>
static int occupancy_of(KernelT k, int threads) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> cache;
  const auto key = std::make_pair((const void*)k, threads);
  std::lock_guard<std::mutex> lock(mu);
  const auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, threads, 0) != hipSuccess) return 1;
  return cache[key] = nb > 0 ? nb : 1;
}

#define KNN_DP_LIST(X) X(8) X(16) X(24) X(32) X(48) X(64) X(96) X(128) X(160) X(192) X(256)

}  // namespace knnk
