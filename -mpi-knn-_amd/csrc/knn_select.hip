// knn_select.hip -- merge / exact fp64 re-rank / certification / vote,
// the exact rescan path and the train-sharded k-way merge (gfx950).
#include "knn_device.h"

#include <algorithm>

// Timing-only experiment builds (tools: a variant library): the merge kernel
// returns after stage N (1 loads + error bound, 2 + selection, 3 + exact
// re-rank); 0 in production.  KNN_DEBUG_CERT: print each certification
// failure's bounds (diagnostic build).
#ifndef KNN_MERGE_STOP
#define KNN_MERGE_STOP 0
#endif
#ifndef KNN_DEBUG_CERT
#define KNN_DEBUG_CERT 0
#endif

namespace knnk {

// ------------------------------------------------ finish: vote / outputs
// Could the reference's order among EXACTLY equal distances (what its
// std::sort over all rows leaves, cpp:323/366) give this query another
// label than the (dist, idx) order?  mode 1: the runner-up count m2 (classes
// other than the winner) and gin, the top-k entries of a tie across the k-th
// place -- the order among equal distances only decides between classes
// sharing the top count, and the membership of that tie group moves at most
// gin entries from one class to another; mode 2: any tie in the top k.
// lab(t) / dist(t): entry t of the (dist, idx)-sorted top k; M the winner's
// count; tie the TIE_VOTE / TIE_ORDER bits; bnd: dist[k-1] == dist[k];
// m2_known >= 0 supplies the runner-up count.  One wave, wave-uniform result.
template <class LabAt, class DistAt>
__device__ bool tie_order_matters(LabAt lab, DistAt dist, int k, int winner, int M, int tie,
                                  bool bnd, int mode, int m2_known = -1) {
  if (mode == 2) return bnd || tie != 0;
  if (mode != 1 || !(bnd || (tie & 4))) return false;
  const int lane = threadIdx.x & 63;
  int m2 = 0, gin = 0;
  const double dlast = dist(k - 1);
  for (int t = lane; t < k; t += 64) {
    const int lt = lab(t);
    if (m2_known < 0 && lt != winner) {
      int c = 0;
      for (int s2 = 0; s2 < k; ++s2) c += (lab(s2) == lt);
      m2 = max(m2, c);
    }
    gin += bnd && dist(t) == dlast;
  }
  m2 = m2_known >= 0 ? m2_known : wave_max_i(m2);
  gin = wave_sum_i(gin);
  return (bnd && M - m2 <= 2 * gin) || ((tie & 4) && m2 == M);
}

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
  const int winner = k > 0 ? ls[tmin] : -1;
  int tie = 0;
  for (int t = lane; t + 1 < k; t += 64)
    if (dk[t] == dk[t + 1]) tie |= ls[t] != ls[t + 1] ? 4 : 8;  // TIE_VOTE / TIE_ORDER
  tie = wave_or_i(tie);
  const bool bnd = k > 0 && k < cnt && dk[k - 1] == dk[k];  // KNN_FLAG_TIE_BOUNDARY
  const bool queue = tie_order_matters([&](int t) { return ls[t]; }, [&](int t) { return dk[t]; },
                                       k, winner, M, tie, bnd, sink.tie_mode);
  if (lane == 0) {
    sink.labels[q] = winner;
    const int f = flag0 | tie | (bnd ? 2 : 0);
    if (sink.flags) sink.flags[q] = f;
    // the order among exactly equal distances is the reference's std::sort's:
    // queue the query for the reference-order pass (tie_order_kernel)
    if (queue) sink.tie_q[atomicAdd(sink.tie_cnt, 1)] = (int)q;
  }
  for (int t = lane; t < k; t += 64) {
    if (sink.idx) sink.idx[q * k + t] = (int64_t)di[t] + idx_off;
    if (sink.dist) sink.dist[q * k + t] = dk[t];
  }
}

// A query with a non-finite coordinate: label -1, KNN_FLAG_NONFINITE, no
// neighbours (idx -1, dist NaN); partial lists empty.  One wave.
__device__ void finish_nonfinite(int64_t q, const Sink& sink) {
  const int lane = threadIdx.x & 63;
  if (sink.mode == MODE_SINGLE) {
    if (lane == 0) {
      sink.labels[q] = -1;
      if (sink.flags) sink.flags[q] = 16;  // KNN_FLAG_NONFINITE
    }
    for (int t = lane; t < sink.k; t += 64) {
      if (sink.idx) sink.idx[q * sink.k + t] = -1;
      if (sink.dist) sink.dist[q * sink.k + t] = __longlong_as_double(0x7FF8000000000000ll);  // quiet NaN
    }
  } else {
    for (int t = lane; t < sink.w; t += 64) {
      sink.dist[q * sink.w + t] = KNN_INF_D;
      sink.idx[q * sink.w + t] = -1;
      sink.plab[q * sink.w + t] = -1;
    }
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

// The fast rescan's setup of one failed query (one wave; the merge runs it
// for the queries it fails): the centred fp32 query row qf (x -2 for L2, the
// candidate pass's operand) and the proxy threshold *thr every row with
// exact distance <= tau passes (fp32 fmaf-chain error bound f_err of t.DP).
template <int METRIC>
__device__ void rescan_prep_query(const RescanPrep& t, int d, const double* __restrict__ qr,
                                  double tq, float* __restrict__ qf, float* __restrict__ thr) {
  const int lane = threadIdx.x & 63, DP = t.DP;
  const double f_err = t.f_err;
  double qa = 0.0, q1 = 0.0;
  for (int i = lane; i < DP; i += 64) {
    float v = 0.0f;
    if (i < d) {
      const double x = qr[i] - t.mu[i];
      qa += METRIC == 0 ? x * x : __builtin_fabs(x);
      q1 += __builtin_fabs(x);
      v = (float)__builtin_ldexp(x * (METRIC == 0 ? -2.0 : 1.0), t.jx);  // X32's scale
    }
    qf[i] = v;
  }
  qa = wave_sum_d(qa) * (1.0 + 1e-12);
  q1 = wave_sum_d(q1) * (1.0 + 1e-12);
  if (lane == 0) {
    const double sinv = __builtin_ldexp(1.0, -t.jx);
    double T;
    // unscaled threshold (+ the fp32 absolute terms of the merge), then
    // scaled to the proxies' units
    if (METRIC == 0) {
      const double E = f_err * (t.x2max + 2.1 * __builtin_sqrt(qa) * __builtin_sqrt(t.x2max)) +
                       0x1p-125 * 1.001 * (2.0 * q1 + t.x1max) * sinv +
                       DP * 0x1p-124 * sinv * sinv + 1e-300;
      T = __builtin_ldexp(tq * tq * (1.0 + 1e-12) - qa * (1.0 - 2e-12) + E, 2 * t.jx);
    } else {
      const double E = f_err * (qa + t.x1max) + 2.0 * 0x1p-125 * 1.001 * DP * sinv + 1e-300;
      T = __builtin_ldexp(tq * (1.0 + 1e-12) + E, t.jx);
    }
    // round T up to a float (the order-preserving key's successor is the next float up)
    float tf = (float)T;
    if ((double)tf < T && tf < KNN_INF_F) tf = key2f(f2key(tf) + 1u);
    *thr = tq < KNN_INF_D ? tf : -KNN_INF_F;  // unknown tau: nothing passes, full scan
  }
}

// --------------------------------------------- merge + exact re-rank
// One block per query (NT = 64 or 256 threads).
//  1. wave 0 holds the union of the 2S lists in registers (EPL per lane),
//     finds the W-th smallest proxy v_W by a 32-step radix select on the
//     order-preserving key bits (ballot counts, no sort), and selects every
//     row with proxy <= v_W + 2E: only those can beat the W-th exact
//     distance (|proxy + ||q'||^2 - d^2| <= E for every row), so the re-rank
//     set adapts to the certified error instead of a fixed 2W.
//     LB = min(first unselected proxy, min over lists of the R-th entry,
//     the query's final global threshold) is a lower bound on the proxy of
//     every row not re-ranked.
//  2. exact fp64 reference distances of the selected rows: rows are read
//     coalesced (16 lanes per 128-B row piece) into an LDS tile of squared
//     differences, then each thread adds its candidate's terms in dimension
//     order -- bit-exact with cpp:33-50 / cpp:51-67 (sequential, no FMA).
//  3. sort (dist, idx), certify LB + ||q'||^2 - E > d_W^2, vote / output.
// Dynamic LDS: qv[d] f64 (d <= kMergeLdsDim) | dk[C2] f64 | tb[NT][17] f64 |
// di[C2] | ls[C2].
constexpr int kMergeLdsDim = 4096;
__device__ __forceinline__ int lanes_below(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// Exact fp64 distances of rows di[0..cn) to the query row qv, in the
// reference's operation order: rows are read coalesced into an LDS tile of
// squared (L1: absolute) differences, then thread c adds its candidate's
// terms in dimension order -- bit-exact with cpp:33-50 / cpp:51-67
// (sequential, no FMA; sqrt correctly rounded).
// (The squared difference is formed from the same fp64 operands in the
// same operation as before the prefetch: the result bits are unchanged.)
// Pads [cn, C2) with (+inf, INT_MAX) and sorts (dist, idx) ascending.
// All NT threads; rows go in batches of RB = NT * EPT / 16, each batch in
// chunks of DC dims: as many as the EPT values per thread and the tile tb
// (tbcap doubles, >= RB * 17) hold -- a small candidate set is read in one
// or two rounds of loads instead of d / 16 dependent ones (the rescan's
// exact finish: ~15 rows, all 128 dims at once; the merge at cfg2: 11-16
// rows, 32 dims per round).  EPT = 8 halves the prefetch registers where
// the candidate set is at most NT / 2 rows.
template <int METRIC, int NT, int EPT = 16>
__device__ void exact_sorted(const TrainDev& t, const double* qv, int* di, double* dk, double* tb,
                             int cn, int C2, int tid, int tbcap) {
  const int d = t.d;
  constexpr int RB = NT * EPT / 16;
  for (int b0 = 0; b0 < cn; b0 += RB) {
    const int nb = min(RB, cn - b0);
    // chunk width DC = 2^lg: the largest power of two the registers and the
    // tile hold, >= 16 (nb <= RB and tbcap >= 17 RB), <= d rounded up
    const int cap = min(NT * EPT, tbcap - nb) / nb;
    int lg = 4;
    while (lg < 12 && (2 << lg) <= cap && (1 << lg) < d) ++lg;
    const int DC = 1 << lg;
    const int ne = nb * DC, ts = DC + 1;  // elements per chunk, tb row stride
    // element e of a chunk: row c = e >> lg (-1 past the chunk), dim e & (DC - 1)
    auto row_of = [&](int e) { return e < ne ? e >> lg : -1; };
    // the raw fp64 values of a chunk, EPT per thread; two register sets in
    // flight: chunk c+2's loads overlap chunk c's sums and barriers
    auto fetch = [&](int c0, double (&o)[EPT]) {
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const int e = tid + k * NT, c = row_of(e), j = e & (DC - 1);
        o[k] = (c >= 0 && c0 + j < d) ? t.X64[(int64_t)di[b0 + c] * d + c0 + j] : 0.0;
      }
    };
    double r = 0.0;
    // stage chunk c0 (values in x) into tb, refill x with chunk c0 + 2 DC, add
    auto step = [&](int c0, double (&x)[EPT]) {
      const int nd = min(DC, d - c0);
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const int e = tid + k * NT, c = row_of(e), j = e & (DC - 1);
        if (c >= 0) {
          double val = 0.0;
          if (j < nd) {
            const double tq = qv[c0 + j] - x[k];
            val = METRIC == 0 ? tq * tq : __builtin_fabs(tq);
          }
          tb[c * ts + j] = val;
        }
      }
      __syncthreads();
      if (c0 + 2 * DC < d) fetch(c0 + 2 * DC, x);
      if (tid < nb) {
        const double* row = tb + tid * ts;
        if (nd == 16) {
#pragma unroll
          for (int j = 0; j < 16; ++j) r = r + row[j];
        } else {
          for (int j = 0; j < nd; ++j) r = r + row[j];
        }
      }
      __syncthreads();
    };
    double xa[EPT], xb[EPT];
    fetch(0, xa);
    if (DC < d) fetch(DC, xb);
    for (int c0 = 0; c0 < d; c0 += 2 * DC) {
      step(c0, xa);
      if (c0 + DC < d) step(c0 + DC, xb);
    }
    if (tid < nb) dk[b0 + tid] = METRIC == 0 ? __builtin_sqrt(r) : r;  // correctly rounded
  }
  for (int c = tid; c < C2; c += NT) {
    if (c >= cn) {
      dk[c] = KNN_INF_D;
      di[c] = INT_MAX;
    }
  }
  bitonic_sort_lds(dk, di, C2, tid, NT);
}

// The exact re-rank of a query on the int8 pass's train grid (every
// coordinate q_i = (cent_i + kq_i) / 2^s, as every train value is): each
// term (q_i - x_i)^2 = (kq_i - kx_i)^2 / 4^s of the reference's sequential
// fp64 sum (cpp:33-50) is exact, and so is every partial sum (multiples of
// 4^-s below d 255^2 / 4^s < 2^53 4^-s), i.e. the reference's r is exactly
// (||kq||^2 + ||kx||^2 - 2 kq.kx) / 4^s -- integer arithmetic on the codes,
// v_dot4_i32_i8 over 16-B chunks of the int8 image rows (a row's 144 B
// instead of its 1 KiB of fp64 values: the merge at cfg2 reads ~13 rows per
// query) -- and sqrt(r) is the reference's distance bit for bit.  di holds
// image positions on entry and train rows on exit; then as exact_sorted
// (pads, (dist, idx) sort).  8 lanes per row, NT / 8 rows per pass.
template <int NT>
__device__ void exact_sorted_i8(const TrainDev& t, const ProxyScale& ps, const signed char* qc,
                                int qq, int* di, double* dk, int cn, int C2, int tid) {
  // 32 rows per pass (one wave: 2 lanes per row), so cfg2's ~13-27 selected
  // rows take one dependent load round instead of 2-4; each row's train row
  // (region order) is loaded with its codes, not in a second round
  constexpr int G = NT / 32 < 1 ? 1 : NT / 32, RP = NT / G;
  const int g = tid & (G - 1);
  const int nch = ps.i8dp / 16;
  const double sc = __builtin_ldexp(1.0, -2 * t.jx);  // (t.jx = s: the pass's scale)
  for (int r0 = 0; r0 < cn; r0 += RP) {
    const int c = r0 + tid / G;
    int dot = 0, xx = 0, tr = 0;
    if (c < cn) {
      const int p = di[c];
      tr = t.perm && g == 0 ? t.perm[p] : p;
      const signed char* row = ps.i8x + (int64_t)p * ps.i8rb;
      const int sw = ps.i8swz ? xh_swz(p & 15) : 0;
      for (int ch = g; ch < nch; ch += G) {
        const int4 xv = *(const int4*)(row + ((ch ^ sw) << 4));
        const int4 qv = *(const int4*)(qc + (ch << 4));
        dot = __builtin_amdgcn_sdot4(xv.x, qv.x, dot, false);
        dot = __builtin_amdgcn_sdot4(xv.y, qv.y, dot, false);
        dot = __builtin_amdgcn_sdot4(xv.z, qv.z, dot, false);
        dot = __builtin_amdgcn_sdot4(xv.w, qv.w, dot, false);
        xx = __builtin_amdgcn_sdot4(xv.x, xv.x, xx, false);
        xx = __builtin_amdgcn_sdot4(xv.y, xv.y, xx, false);
        xx = __builtin_amdgcn_sdot4(xv.z, xv.z, xx, false);
        xx = __builtin_amdgcn_sdot4(xv.w, xv.w, xx, false);
      }
    }
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
      dot += __shfl_xor(dot, o, 64);
      xx += __shfl_xor(xx, o, 64);
    }
    if (c < cn && g == 0) {
      dk[c] = __builtin_sqrt((double)(qq + xx - 2 * dot) * sc);
      di[c] = tr;  // image position -> train row (its group has read di[c] already)
    }
  }
  __syncthreads();
  for (int c = tid; c < C2; c += NT) {
    if (c >= cn) {
      dk[c] = KNN_INF_D;
      di[c] = INT_MAX;
    }
  }
  bitonic_sort_lds(dk, di, C2, tid, NT);
}

// The certification test: every row whose proxy is >= LB (unscaled) has an
// exact distance beyond dw, the W-th exact distance re-ranked (rigorous error
// bound E; +inf LB: no such row can be closer)
template <int METRIC>
__device__ __forceinline__ bool bound_ok(double LB, double dw, double qa, double E) {
  if (METRIC == 0) return (LB + qa * (1.0 - 2e-12) - E) * (1.0 - 1e-12) > dw * dw * (1.0 + 1e-12);
  return (LB - E) * (1.0 - 1e-12) > dw * (1.0 + 1e-12);
}

// (EPT 8, the small candidate sets of cfg2: 6 waves per SIMD at 80 VGPRs,
// -6 us per cfg2 step against 5 at 83, profiles/ab_log.md r4mg)
template <int METRIC, int NT, int EPL, int EPT = 16>
__global__ void __launch_bounds__(NT)
__attribute__((amdgpu_waves_per_eu(EPT == 8 ? 6 : 1)))
merge_rerank_kernel(const float* __restrict__ cv, const int* __restrict__ ci, int U, int R,
                    TrainDev t, const double* __restrict__ Q64, int W, int Cmax, int C2,
                    double f_err, ProxyScale ps, const uint32_t* __restrict__ gthr, Sink sink,
                    int* __restrict__ rescan_q, double* __restrict__ rescan_tau,
                    int* __restrict__ rescan_cnt, SplitMap sm, RescanPrep rp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int s_cn, s_cert, s_f;
  __shared__ double s_lb, s_lbr, s_qa, s_e, s_pinv;
  // the int8 pass: the query's codes and their squared norm, and whether it
  // is on the train grid (exact_sorted_i8)
  __shared__ __attribute__((aligned(16))) signed char s_qc[256];
  __shared__ int s_qq, s_i8x;
  __shared__ uint32_t s_bs[64];  // per split: min over its full lists' R-th entries (keys)
  const int d = t.d;
  // the query row is staged in LDS up to kMergeLdsDim dims, else read in place
  const bool q_in_lds = d <= kMergeLdsDim;
  double* dk = (double*)smem + (q_in_lds ? d : 0);
  double* tb = dk + C2;
  // (exact_sorted stages at most min(NT, C2) rows per batch: cn <= C2)
  int* di = (int*)(tb + min(NT, C2) * 17);
  int* ls = di + C2;
  const int64_t q = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;

  const double* qrow = Q64 + q * d;
  const double* qv = q_in_lds ? (const double*)smem : qrow;
  if (q_in_lds)
    for (int c = tid; c < d; c += NT) ((double*)smem)[c] = qrow[c];
  if (tid < 64) s_bs[tid] = kKeyInf;
  __syncthreads();

  bool i8x = false;  // (wave 0) exact re-rank on the int8 codes
  if (tid < 64) {
    // error bound of this query's proxies (the candidate operands are centred)
    double qa = 0.0, q1 = 0.0;
    for (int c = lane; c < d; c += 64) {
      const double x = qv[c] - t.mu[c];
      qa += METRIC == 0 ? x * x : __builtin_fabs(x);
      q1 += __builtin_fabs(x);
    }
    qa = wave_sum_d(qa) * (1.0 + 1e-12);
    double E =
        (METRIC == 0 ? f_err * (t.x2max + 2.1 * __builtin_sqrt(qa) * __builtin_sqrt(t.x2max))
                     : f_err * (qa + t.x1max)) + 1e-300;
    if (METRIC == 0 && ps.f16) {
      // fp16 operands: f_err covers the accumulation only; add the measured
      // representation error (q' = q - mu, x' = x - mu, dq / dx the operand
      // errors in unscaled units):  2 |q'.dx + dq.x' + dq.dx| <=
      // 2 (|q'| dxmax + |dq| (xmax + dxmax)), plus the fl32 seed's own
      // rounding (3u ||x'||^2, u = 2^-24).  The query's operand is rebuilt
      // here exactly as knn_prep.hip rounds it (one fp64 -> fp16 rounding
      // of -2 * 2^jx (q - mu)), so its error is measured, not assumed.
      const double qs = -__builtin_ldexp(0.5, -t.jx);  // operand = -2 * 2^jx q'
      double dq2 = 0.0;
      for (int c = lane; c < d; c += 64) {
        const double x = qv[c] - t.mu[c];
        const _Float16 h = f16_operand(-2.0 * x, t.jx);
        const double e = (double)h * qs - x;
        dq2 += e * e;
      }
      const double qn = __builtin_sqrt(qa), xm = __builtin_sqrt(t.x2max);
      const double dq = __builtin_sqrt(wave_sum_d(dq2) * (1.0 + 1e-12)) * (1.0 + 1e-12) +
                        0x1p-50 * qn;
      E = f_err * (t.x2max + 2.0 * (qn + dq) * (xm + t.dxmax) * 1.001) + 3.01 * 0x1p-24 * t.x2max +
          2.0 * (qn * t.dxmax + dq * (xm + t.dxmax)) * 1.001 + 1e-300;
    }
    if (METRIC == 0 && ps.i8c) {
      // int8 codes: the query's code k_q = clamp(rint(Q), -128, 127) of
      // Q = q 2^s - cent (rebuilt here exactly as prep_i8_queries_kernel
      // does); with delta = Q - k_q, |qa + proxy - d^2| gains
      // 2 |delta . k_x| 4^-s <= 2 ||delta|| 2^-s sqrt(x2max) (value units)
      double dq2 = 0.0;
      int qq = 0;
      for (int c = lane; c < d; c += 64) {
        const double y = __builtin_ldexp(qv[c], t.jx) - ps.i8c[c];
        const double r = __builtin_fmin(__builtin_fmax(__builtin_rint(y), -128.0), 127.0);
        dq2 += (y - r) * (y - r);
        if (ps.i8x && c < 256) {
          s_qc[c] = (signed char)(int)r;
          qq += (int)r * (int)r;
        }
      }
      if (ps.i8x)
        for (int c = d + lane; c < ps.i8dp && c < 256; c += 64) s_qc[c] = 0;
      dq2 = wave_sum_d(dq2);
      qq = wave_sum_i(qq);
      const double dq = __builtin_sqrt(dq2 * (1.0 + 1e-12)) * (1.0 + 1e-12);
      E += 2.0 * __builtin_ldexp(dq, -t.jx) * __builtin_sqrt(t.x2max) * 1.001;
      // on the grid (no coding error): the exact re-rank runs on the codes
      i8x = ps.i8x && dq2 == 0.0 && ps.i8dp <= 256;
      if (lane == 0) s_qq = qq;
    }
    // proxies are in scaled units (operands 2^jx (x - mu), knn_prep.hip):
    // unscale exactly; operand values outside the format's normal range add
    // absolute error terms (ue per element, up per product, scaled units)
    const double pinv = __builtin_ldexp(1.0, METRIC == 0 ? -2 * t.jx : -t.jx);
    const double sinv = __builtin_ldexp(1.0, -t.jx);
    q1 = wave_sum_d(q1) * (1.0 + 1e-12);
    if (METRIC == 0) E += ps.ue * 1.001 * (2.0 * q1 + t.x1max) * sinv + t.DP * ps.up * pinv;
    else E += 2.0 * ps.ue * 1.001 * t.DP * sinv;
    // valid: 1 usable, 0 operands out of the format's range (exact rescan),
    // -1 a non-finite input value (no neighbours are reported)
    const float vq = ps.valid ? ps.valid[q] : 1.0f;
    const bool void_q = !(vq > 0.0f);
    const bool nonfinite = vq < 0.0f;
    // union in registers; min over full lists of their R-th (worst kept) entry
    // (queries in region order: the query's lists sit at its position)
    const int64_t qp = ps.qpos ? ps.qpos[q] : q;
    const float* lv = cv + qp * U;
    const int* li = ci + qp * U;
    // the query's final global-threshold slots (cand_kernel), loaded with the
    // lists: the kernel also filtered with them, so rows it dropped have
    // proxy >= max over the slots (lane s < kGthrSlots holds slot s)
    const uint32_t gsl = gthr && lane < kGthrSlots ? gthr[qp * kGthrSlots + lane] : 0u;
    float v[EPL];
    int id[EPL];
    float mlr = KNN_INF_F;
    int nv = 0;
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int x = lane + 64 * e;
      v[e] = KNN_INF_F;
      id[e] = -1;
      if (x < U) {
        v[e] = lv[x];
        id[e] = li[x];
        if (x % R == R - 1) {
          mlr = fminf(mlr, v[e]);
          if (sm.S && v[e] < KNN_INF_F) atomicMin(&s_bs[x / (sm.lps * R)], f2key(v[e]));
        }
      }
      nv += __popcll(__ballot(v[e] < KNN_INF_F));
    }
    mlr = wave_min(mlr);
#if KNN_MERGE_STOP == 1
    if (nv >= 0) return;  // (timing-only experiment build: the loads and the error bound)
#endif
    double tsel = KNN_INF_D;  // select proxies <= tsel
    if (nv > W) {
      // radix select of the key of the W-th smallest proxy (finite: nv > W),
      // from the highest bit in which the finite keys differ (the common
      // prefix of their min and max is its prefix), and done as soon as
      // exactly W keys lie at or below the probe: it is then their largest
      // (cfg2: ~10 probes instead of 32)
      uint32_t ky[EPL];
      uint32_t kmn = kKeyInf, kmx = 0;
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        ky[e] = f2key(v[e]);
        kmn = min(kmn, ky[e]);
        if (v[e] < KNN_INF_F) kmx = max(kmx, ky[e]);
      }
      kmn = wave_min_u(kmn);
      kmx = wave_max_u(kmx);
      const uint32_t dif = kmn ^ kmx;
      const int hb = dif ? 31 - __builtin_clz(dif) : -1;
      uint32_t pre = hb < 0 ? kmn : hb == 31 ? 0u : kmn & ~((2u << hb) - 1u);
      for (int b = hb; b >= 0; --b) {
        const uint32_t T = pre | ((1u << b) - 1u);
        int cnt = 0;
#pragma unroll
        for (int e = 0; e < EPL; ++e) cnt += __popcll(__ballot(ky[e] <= T));
        if (cnt < W) {
          pre |= 1u << b;
        } else if (cnt == W) {
          uint32_t mx = 0;
#pragma unroll
          for (int e = 0; e < EPL; ++e) mx = ky[e] <= T ? max(mx, ky[e]) : mx;
          pre = wave_max_u(mx);
          break;
        }
      }
      const double vw = (double)key2f(pre) * pinv;
      tsel = vw + 2.0 * E + 1e-9 * (__builtin_fabs(vw) + qa + E) + 1e-300;
    }
    float lbx = KNN_INF_F;
    int cn = 0;
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const bool valid = v[e] < KNN_INF_F;
      const bool sel = valid && (double)v[e] * pinv <= tsel;
      if (valid && !sel) lbx = fminf(lbx, v[e]);
      const unsigned long long mk = __ballot(sel);
      if (sel) {
        const int pos = cn + lanes_below(mk);
        if (pos < Cmax) di[pos] = id[e];
      }
      cn += __popcll(mk);
    }
    lbx = wave_min(lbx);
    if (cn > Cmax) {
      // more rows inside the selection window than this launch re-ranks:
      // re-rank the Cmax smallest proxies instead (ties at the cut filled in
      // lane order).  Rows left out have proxy >= the cut, so the bound
      // below may still certify; if not, the W-th exact distance of these
      // rows still bounds the fast rescan.
      uint32_t pre = 0;  // key of the Cmax-th smallest proxy
      for (int b = 31; b >= 0; --b) {
        const uint32_t T = pre | ((1u << b) - 1u);
        int cnt = 0;
#pragma unroll
        for (int e = 0; e < EPL; ++e) cnt += __popcll(__ballot(v[e] < KNN_INF_F && f2key(v[e]) <= T));
        if (cnt < Cmax) pre |= 1u << b;
      }
      cn = 0;
      for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const uint32_t ky = f2key(v[e]);
          const bool sel = v[e] < KNN_INF_F && (pass == 0 ? ky < pre : ky == pre);
          const unsigned long long mk = __ballot(sel);
          if (sel) {
            const int pos = cn + lanes_below(mk);
            if (pos < Cmax) di[pos] = id[e];
          }
          cn += __popcll(mk);
        }
      }
      cn = min(cn, Cmax);
      lbx = key2f(pre);
    }
    if (t.perm && !i8x) {
      // image positions -> train rows (region order), one batch of
      // independent loads (the wave's own LDS writes above complete first;
      // exact_sorted_i8 reads the image rows first and maps after)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const int nsel = min(cn, Cmax);
      for (int i = lane; i < nsel; i += 64) di[i] = t.perm[di[i]];
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    const float tq = gthr ? key2f(wave_max_u(gsl)) : KNN_INF_F;
    if (lane == 0) {
      // void proxies: exact rescan below; non-finite query: no neighbours
      s_cn = nonfinite ? -1 : (void_q ? Cmax + 1 : cn);
      s_lb = (double)fminf(fminf(lbx, mlr), tq) * pinv;
      s_lbr = (double)fminf(lbx, tq) * pinv;  // the bound without the lists' R-th entries
      s_pinv = pinv;
      s_qa = qa;
      s_e = E;
      s_i8x = i8x;
    }
  }
  __syncthreads();
  const int cn = s_cn;
  if (cn < 0) {  // a NaN / inf coordinate: the reference's distances are undefined
    if (tid < 64) finish_nonfinite(q, sink);
    return;
  }
  if (cn > Cmax) {  // void proxies (the window overflow is handled above): exact rescan
    if (tid == 0) {
      const int f = atomicAdd(rescan_cnt, 1);
      rescan_q[f] = (int)q;
      rescan_tau[f] = KNN_INF_D;
      if (sm.mask) {
        sm.mask[f] = ~0ull;
        if (f < sm.cap) sm.nkeep[f] = 0;
      }
      s_f = f;
    }
    __syncthreads();
    // the fast rescan's setup: tau unknown, nothing passes its filter (the
    // full scan takes the query)
    if (tid < 64 && s_f < rp.cap) {
      rescan_prep_query<METRIC>(rp, d, qv, KNN_INF_D, rp.qf + (int64_t)s_f * rp.DP, rp.thr + s_f);
      if (tid == 0) {
        rp.fcnt[s_f] = 0;
        if (rp.t8) rp.t8[s_f] = -1;  // (tau unknown: the full scan takes it)
      }
    }
    return;
  }

#if KNN_MERGE_STOP == 2
  if (cn >= 0) return;  // (timing-only experiment build: + selection)
#endif
  if (METRIC == 0 && s_i8x)
    exact_sorted_i8<NT>(t, ps, s_qc, s_qq, di, dk, cn, C2, tid);
  else
    exact_sorted<METRIC, NT, EPT>(t, qv, di, dk, tb, cn, C2, tid, min(NT, C2) * 17);
#if KNN_MERGE_STOP == 3
  if (cn >= 0) return;  // (timing-only experiment build: + exact re-rank and sort)
#endif

  // certification: every row not re-ranked has proxy >= LB, hence exact
  // distance >= the bound below (rigorous error bound E)
  if (tid == 0) {
    const double LB = s_lb;
    bool cert;
    if (cn < W) {
      cert = false;  // fewer rows than the top W re-ranked (e.g. non-finite proxies)
    } else if (!(LB < KNN_INF_D)) {
      // no bound on the rows left out (lists that never filled and no filter
      // threshold): not certified, the rescan decides
      cert = false;
    } else {
      cert = bound_ok<METRIC>(LB, dk[W - 1], s_qa, s_e);
    }
    s_cert = cert;
    if (!cert) {
      // the W-th exact distance among the re-ranked rows bounds the true
      // W-th from above: the fast rescan keeps every row that can reach it
      const int f = atomicAdd(rescan_cnt, 1);
      s_f = f;
      rescan_q[f] = (int)q;
      rescan_tau[f] = cn >= W ? dk[W - 1] : KNN_INF_D;
#if KNN_DEBUG_CERT
      // (diagnostic build only: which bound failed)
      printf("cert fail q %d cn %d W %d LB %.6f LBr %.6f qa %.6f E %.3g dW2 %.6f dW1 %.6f dlast %.6f\n",
             (int)q, cn, W, LB, s_lbr, s_qa, s_e, cn >= W ? dk[W - 1] * dk[W - 1] : -1.0,
             cn >= W + 1 ? dk[W] * dk[W] : -1.0, dk[cn - 1] * dk[cn - 1]);
#endif
      if (sm.mask) {
        // Per split: rows a split dropped have proxy >= min(its lists' final
        // R-th entries, the final global threshold) -- its quad filter and
        // the lists only tighten.  When the bound holds without the lists'
        // R-th entries, only the splits whose own bound fails can hold a row
        // of the top W outside the re-ranked set: the rescan scans those
        // splits' rows, and the re-ranked rows of the other splits within
        // tau go along (every other row of theirs is beyond tau).
        unsigned long long mk = ~0ull;
        if (sm.S && cn >= W && bound_ok<METRIC>(s_lbr, dk[W - 1], s_qa, s_e)) {
          mk = 0;
          for (int sp = 0; sp < sm.S; ++sp) {
            const double b = (double)key2f(s_bs[sp]) * s_pinv;
            if (!bound_ok<METRIC>(b, dk[W - 1], s_qa, s_e)) mk |= 1ull << sp;
          }
          if (mk == 0) mk = ~0ull;
        }
        sm.mask[f] = mk;
        if (f < sm.cap) {
          int nk = 0;
          if (mk != ~0ull) {
            const double tau = dk[W - 1];
            for (int i = 0; i < cn; ++i) {
              const int r = di[i];  // (a train row; its split by its image position)
              const int sp = (int)(((int64_t)(t.ipos ? t.ipos[r] : r) / sm.trows) % sm.S);
              if (dk[i] <= tau && !((mk >> sp) & 1)) sm.keep[(int64_t)f * kRescanCap + nk++] = r;
            }
          }
          sm.nkeep[f] = nk;
          if (f < rp.cap) rp.fcnt[f] = nk;  // (cap = sm.cap)
        }
      } else if (f < rp.cap) {
        rp.fcnt[f] = 0;
      }
    }
  }
  __syncthreads();
  if (!s_cert) {
    // the fast rescan's setup of this query (tau: its W-th exact distance)
    if (tid < 64 && s_f < rp.cap) {
      rescan_prep_query<METRIC>(rp, d, qv, cn >= W ? dk[W - 1] : KNN_INF_D,
                                rp.qf + (int64_t)s_f * rp.DP, rp.thr + s_f);
      if (METRIC == 0 && rp.t8) {
        // on the train grid: the rescan filters on the codes, exactly.  The
        // reference's r = (qq + xx - 2 q.x) 4^-s is exact there (DESIGN.md
        // section 2), so a row reaches tau only if its integer r_int <=
        // tau^2 4^s (+ a relative 1e-12 and 2 for the rounding of tau^2)
        const bool ok = s_i8x && cn >= W;
        if (ok)
          for (int c = lane; c < 256; c += 64) rp.qc8[(int64_t)s_f * 256 + c] = s_qc[c];
        if (lane == 0) {
          long long T = -1;
          if (ok) {
            const double tt = __builtin_ldexp(dk[W - 1] * dk[W - 1], 2 * t.jx) * (1.0 + 1e-12);
            T = tt < 0x1p62 ? (long long)tt + 2 : (1ll << 62);  // (the filter forms qq + xx - 2 q.x)
          }
          rp.t8[s_f] = T;
        }
      }
    }
    return;
  }

  const int need = sink.mode == MODE_SINGLE ? sink.k : sink.w;
  for (int c = tid; c < need && c < cn; c += NT) ls[c] = t.lab[di[c]];
  __syncthreads();
  if (tid < 64) {
    if (sink.mode == MODE_SINGLE)
      finish_single(q, dk, di, ls, cn, sink.k, sink.idx_off, 0, sink);
    else
      finish_partial(q, dk, di, ls, cn, sink.w, sink.idx_off, sink);
  }
}

template <int METRIC, int NT, int EPL, int EPT = 16>
static void launch_mr(const float* cv, const int* ci, int U, int R, const TrainDev& t,
                      const double* Q64, int64_t m, int W, int Cmax, int C2, double f_err,
                      ProxyScale ps, const uint32_t* gthr, const Sink& sink, int* rescan_q,
                      double* rescan_tau, int* rescan_cnt, const SplitMap& sm,
                      const RescanPrep& rp, hipStream_t s) {
  // (the staging tile only as large as the candidate set: a smaller
  // footprint keeps more of these latency-bound workgroups per CU)
  const size_t lds = (size_t)(t.d <= kMergeLdsDim ? t.d : 0) * 8 + (size_t)C2 * 8 +
                     (size_t)std::min(NT, C2) * 17 * 8 + (size_t)C2 * 8;
  hipLaunchKernelGGL((merge_rerank_kernel<METRIC, NT, EPL, EPT>), dim3((unsigned)m), dim3(NT), lds, s,
                     cv, ci, U, R, t, Q64, W, Cmax, C2, f_err, ps, gthr, sink, rescan_q, rescan_tau,
                     rescan_cnt, sm, rp);
}

void launch_merge_rerank(int metric, const float* cv, const int* ci, int NL, int R,
                         const TrainDev& t, const double* Q64, int64_t m, int W, int C,
                         double f_err, ProxyScale ps, const uint32_t* gthr, const Sink& sink,
                         int* rescan_q, double* rescan_tau, int* rescan_cnt, const SplitMap& sm_in,
                         const RescanPrep& rp, hipStream_t s) {
  if (m <= 0) return;
  SplitMap sm = sm_in;
  if (sm.S > 64 || sm.trows <= 0) sm.S = 0;  // per-split bounds need S <= 64 mask bits
  const int U = NL * R;  // <= 2 * 64 * 16 (choose_geometry bounds S and R)
  int C2 = 1;
  while (C2 < C) C2 <<= 1;
  const bool big = C2 > 64, wide = U > 1024;
#define KNN_MR(M_, NT_, EPL_) KNN_MRE(M_, NT_, EPL_, 16)
#define KNN_MRE(M_, NT_, EPL_, EPT_) \
  launch_mr<M_, NT_, EPL_, EPT_>(cv, ci, U, R, t, Q64, m, W, C, C2, f_err, ps, gthr, sink,  \
                                 rescan_q, rescan_tau, rescan_cnt, sm, rp, s)
  // fewer entries per lane when the union is small (cfg2: 152 lists x 4 =
  // 608 entries -> 10 per lane): every radix-select step and the selection
  // loops run over EPL unrolled entries
  const bool narrow = U <= 640;
  if (metric == 0) {
    if (big) { if (wide) KNN_MR(0, 256, 32); else KNN_MR(0, 256, 16); }
    // (candidate sets of <= 32 rows, cfg2's 27: half the prefetch registers,
    // 4 waves per SIMD for this latency-bound kernel)
    else { if (wide) KNN_MR(0, 64, 32); else if (narrow && C2 <= 32) KNN_MRE(0, 64, 10, 8);
           else if (narrow) KNN_MR(0, 64, 10); else KNN_MR(0, 64, 16); }
  } else {
    if (big) { if (wide) KNN_MR(1, 256, 32); else KNN_MR(1, 256, 16); }
    else { if (wide) KNN_MR(1, 64, 32); else KNN_MR(1, 64, 16); }
  }
#undef KNN_MR
#undef KNN_MRE
}

// ------------------------------------------------- rescan (device-driven)
#ifndef KNN_DEBUG_RESCAN
#define KNN_DEBUG_RESCAN 0  // (diagnostic builds: the filters' query modes)
#endif
// Queries whose candidate set was not certified (a list overflowed near the
// top, heavy ties, operands out of the candidate format's range).  The
// whole path is enqueued on every call and sized on the device: the merge
// counts the failed queries in cnt[0] (their ids in rescan_q, their bound in
// rescan_tau); every kernel below reads the counts itself and exits at once
// when there is nothing to do, so a classify call never waits for the host.
//
//  1. fast path, for the first `cap` failed queries: tau = the W-th exact
//     distance among the query's re-ranked rows (>= the true W-th).
//     rescan_filter streams the fp32 train copy (lane = train row; queries
//     broadcast from LDS) and appends every row whose centred fp32 proxy --
//     an fmaf chain with the candidate pass's certified error bound -- is
//     within reach of tau; the appended set therefore holds every row with
//     exact distance <= tau, i.e. the exact top-W with all its ties.
//     rescan_finish_fast re-ranks it exactly.
//  2. full scan, for the queries the fast path cannot finish (tau unknown,
//     more than kRescanCap rows within reach, or failed queries beyond
//     `cap`): one 1024-thread workgroup per query computes every row's exact
//     distance and keeps the top W by (dist, idx) with a threshold-filtered
//     LDS buffer.

// Appends image row `row` (as its train row) to query s's list if its proxy
// passes (pad rows never do: +inf seeds).
__device__ __forceinline__ void rescan_append(float acc, float th, int s, int64_t row,
                                              const TrainDev& t, int* __restrict__ fcnt,
                                              int* __restrict__ buf) {
  if (acc <= th) {
    const int pos = atomicAdd(&fcnt[s], 1);
    if (pos < kRescanCap) buf[(int64_t)s * kRescanCap + pos] = train_row(t, (int)row);
  }
}

// DP <= 256: block = NWB waves, wave w owns the 64 consecutive train rows
// starting at blockIdx.x*64*NWB + 64w (lane = row), copied once into LDS by
// LDS-DMA (the padded X32 layout, odd 16-B stride -> conflict-free
// ds_read_b128) and reused for every group of FQ failed queries.
template <int METRIC, int FQ>
__global__ void __launch_bounds__(256)
rescan_filter_kernel(TrainDev t, const float* __restrict__ qf, const float* __restrict__ thr,
                     const int* __restrict__ cnt, int cap, int* __restrict__ fcnt,
                     int* __restrict__ buf, const unsigned long long* __restrict__ mask, int S,
                     int64_t trows, const long long* __restrict__ t8) {
  const int nf = min(cnt[0], cap);
  if (nf == 0) return;
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  const int DP = t.DP, RSF = DP + 4;
  const int NWB = blockDim.x >> 6;
  float* qs = fsm;                          // [FQ][DP] centred queries (x -2 for L2)
  float* thr_s = qs + FQ * DP;              // [FQ] proxy thresholds
  float* rows = thr_s + FQ;                 // [NWB][64][RSF]
  __shared__ unsigned long long mask_s[FQ];  // splits each query of the group scans
  __shared__ unsigned long long s_u;         // union of the failed queries' splits
  __shared__ int s_sp[64], s_ns;             // its splits, in order, and their count
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid == 0) {
    unsigned long long u = ~0ull;
    if (mask && nf <= 64) {
      u = 0;
      for (int f = 0; f < nf; ++f)
        if (!(t8 && t8[f] >= 0)) u |= mask[f];  // (int8-filtered queries: not here)
    }
    s_u = u;
    int ns = 0;
    if (u != ~0ull)
      for (int b = 0; b < 64; ++b)
        if ((u >> b) & 1) s_sp[ns++] = b;
    s_ns = ns;
  }
  __syncthreads();
#if KNN_DEBUG_RESCAN
  if (blockIdx.x == 0 && tid == 0)
    printf("fp32 filter: nf %d u %llx ns %d t8 %p mask %p\n", nf, s_u, s_ns, (const void*)t8,
           (const void*)mask);
#endif
  const unsigned long long need = s_u;
  // Units of 64 rows, one per wave; a workgroup's NWB waves take NWB
  // consecutive units per step (grid-stride).  A targeted rescan (every
  // failed query flags some splits) walks only those splits' tiles -- tile
  // sp + k S holds trows / 64 units (64 | trows) -- so a workgroup loads
  // only rows it scans and no step is spent skipping (cfg2: one failed
  // query, one split's 103 tiles, at most one tile per workgroup); else
  // every row, unit u = rows 64 u ...
  const bool tgt = mask && need != ~0ull;
  const int gpt = tgt ? (int)(trows / 64) : 1;
  const int64_t ntile = tgt ? (t.n_pad + trows - 1) / trows : 0;
  const int64_t units = tgt ? (int64_t)s_ns * ((ntile + S - 1) / S) * gpt : (t.n_pad + 63) / 64;
  for (int64_t u0 = (int64_t)blockIdx.x * NWB; u0 < units; u0 += (int64_t)gridDim.x * NWB) {
  const int64_t u = u0 + wv;
  int64_t row0 = -1;
  int wsp = 0;  // split of this wave's 64 rows
  if (u < units) {
    if (tgt) {
      const int64_t r = u / gpt, k = r / s_ns;
      const int sp = s_sp[r - k * s_ns];
      const int64_t tile = sp + k * S;
      if (tile < ntile) {
        row0 = tile * trows + (u - r * gpt) * 64;
        wsp = sp;
      }
    } else {
      row0 = u * 64;
      wsp = mask ? (int)((row0 / trows) % S) : 0;
    }
  }
  const bool active = row0 >= 0 && row0 < t.n_pad;
  __syncthreads();  // every wave is done with the previous step's group loop

  float* my_rows = rows + (size_t)wv * 64 * RSF;
  if (active) {  // X32 carries 1 KiB of slack past the last row
    const int bytes = 64 * RSF * 4;
    const char* src = (const char*)(t.X32 + row0 * RSF) + lane * 16;
    const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)my_rows;
    for (int p = 0; p * 1024 < bytes; ++p) glds16(src + p * 1024, dst + p * 1024);
  }
  const float* xr = my_rows + lane * RSF;
  for (int g0 = 0; g0 < nf; g0 += FQ) {
    const int nfg = min(FQ, nf - g0);
    __syncthreads();  // the previous group's reads of qs are done
    for (int e = tid; e < FQ * DP; e += blockDim.x) {
      const int qi = e / DP;
      qs[e] = qi < nfg ? qf[(int64_t)g0 * DP + e] : 0.0f;
    }
    if (tid < FQ) {
      // absent, or filtered on the int8 codes (rescan_filter_i8_kernel): no row passes
      thr_s[tid] = tid < nfg && !(t8 && t8[g0 + tid] >= 0) ? thr[g0 + tid] : -KNN_INF_F;
      mask_s[tid] = tid < nfg && mask ? mask[g0 + tid] : ~0ull;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (active) {
      const float seed = xr[METRIC == 0 ? DP : DP + 1];  // +inf on pad rows: never passes
      float acc[FQ];
#pragma unroll
      for (int qi = 0; qi < FQ; ++qi) acc[qi] = seed;
      for (int c = 0; c < DP / 4; ++c) {
        const float4 x4 = *(const float4*)(xr + 4 * c);
#pragma unroll
        for (int qi = 0; qi < FQ; ++qi) {
          if (qi >= nfg) break;  // group-uniform: no LDS reads for empty query slots
          const float4 q4 = *(const float4*)(qs + qi * DP + 4 * c);
          float a = acc[qi];
          if (METRIC == 0) {  // the candidate pass's fp32 model: an fmaf chain
            a = __builtin_fmaf(q4.x, x4.x, a);
            a = __builtin_fmaf(q4.y, x4.y, a);
            a = __builtin_fmaf(q4.z, x4.z, a);
            a = __builtin_fmaf(q4.w, x4.w, a);
          } else {
            a = a + __builtin_fabsf(q4.x - x4.x);
            a = a + __builtin_fabsf(q4.y - x4.y);
            a = a + __builtin_fabsf(q4.z - x4.z);
            a = a + __builtin_fabsf(q4.w - x4.w);
          }
          acc[qi] = a;
        }
      }
#pragma unroll
      for (int qi = 0; qi < FQ; ++qi)
        if (qi < nfg && ((mask_s[qi] >> wsp) & 1))
          rescan_append(acc[qi], thr_s[qi], g0 + qi, row0 + lane, t, fcnt, buf);
    }
  }
  }  // units
}

// The fast rescan's filter on the int8 codes (kernel metric 6 images: plain
// rows of i8rb bytes, codes of i8dp dims), for the failed queries on the
// train grid (t8[f] >= 0; the others go through rescan_filter_kernel): lane =
// image row, its codes read in place (i8dp / 16 x 16 B), the exact integer
// squared distance qq + xx - 2 q.x (code units, v_dot4) against t8 -- 144 B
// per row instead of the fp32 filter's 528 (cfg2), and no error bound: every
// row within tau (and its ties) is appended exactly.  Same unit walk as the
// fp32 filter: only the flagged splits' tiles of a targeted rescan.
constexpr int kI8RescanRB = 272;  // LDS bytes per staged row of the int8 filter (>= the largest rb)
template <int FQ>
__global__ void __launch_bounds__(256)
rescan_filter_i8_kernel(TrainDev t, const signed char* __restrict__ img, int rb, int dp,
                        const signed char* __restrict__ qc8, const long long* __restrict__ t8,
                        const int* __restrict__ cnt, int cap, int* __restrict__ fcnt,
                        int* __restrict__ buf, const unsigned long long* __restrict__ mask, int S,
                        int64_t trows) {
  const int nf = min(cnt[0], cap);
  if (nf == 0) return;
  __shared__ __attribute__((aligned(16))) signed char qs[FQ][256];
  __shared__ long long ts[FQ];
  __shared__ int qqs[FQ];
  __shared__ unsigned long long mask_s[FQ];
  __shared__ unsigned long long s_u;
  __shared__ int s_sp[64], s_ns, s_any;
  // each wave's 64 staged rows (+ 1 KiB: the last piece may run past them)
  __shared__ __attribute__((aligned(16))) signed char rows_s[4 * 64 * kI8RescanRB + 1024];
  const int tid = threadIdx.x, lane = tid & 63;
  const int NWB = blockDim.x >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nch = dp / 16;
  if (tid == 0) {
    // the splits the int8-mode queries flag (every row if any flags all, or
    // more than 64 failed queries)
    unsigned long long u = mask && nf <= 64 ? 0ull : ~0ull;
    int any = 0;
    for (int f = 0; f < nf; ++f)
      if (t8[f] >= 0) {
        any = 1;
        if (mask && nf <= 64) u |= mask[f];
      }
    s_any = any;
    s_u = u;
    int ns = 0;
    if (u != ~0ull)
      for (int b = 0; b < 64; ++b)
        if ((u >> b) & 1) s_sp[ns++] = b;
    s_ns = ns;
  }
  __syncthreads();
#if KNN_DEBUG_RESCAN
  if (blockIdx.x == 0 && tid == 0)
    for (int f = 0; f < nf; ++f)
      printf("i8 filter: nf %d f %d t8 %lld mask %llx any %d u %llx ns %d\n", nf, f, t8[f],
             mask ? mask[f] : 0ull, s_any, s_u, s_ns);
#endif
  if (!s_any) return;
  const unsigned long long need = s_u;
  const bool tgt = mask && need != ~0ull;
  const int gpt = tgt ? (int)(trows / 64) : 1;
  const int64_t ntile = tgt ? (t.n_pad + trows - 1) / trows : 0;
  const int64_t units = tgt ? (int64_t)s_ns * ((ntile + S - 1) / S) * gpt : (t.n_pad + 63) / 64;
  // every failed query in groups of FQ (fp32-mode ones get ts = -1: no row
  // passes, r >= 0), the rows of each group's units re-read from L2
  for (int g0 = 0; g0 < nf; g0 += FQ) {
    const int nfg = min(FQ, nf - g0);
    __syncthreads();  // the previous group's reads of qs are done
    for (int e = tid; e < FQ * 256; e += blockDim.x) {
      const int a = e >> 8;
      qs[a][e & 255] = a < nfg && t8[g0 + a] >= 0 ? qc8[(int64_t)(g0 + a) * 256 + (e & 255)] : 0;
    }
    if (tid < FQ) {
      ts[tid] = tid < nfg ? t8[g0 + tid] : -1;
      mask_s[tid] = tid < nfg && mask ? mask[g0 + tid] : ~0ull;
    }
    __syncthreads();
    if (tid < FQ) {
      int qq = 0;
      for (int c = 0; c < dp; ++c) qq += (int)qs[tid][c] * (int)qs[tid][c];
      qqs[tid] = qq;
    }
    __syncthreads();
    bool grp = false;  // (block-uniform) any int8-mode query in this group
#pragma unroll
    for (int a = 0; a < FQ; ++a) grp |= ts[a] >= 0;
    if (!grp) continue;
    for (int64_t u = (int64_t)blockIdx.x * NWB + wv; u < units; u += (int64_t)gridDim.x * NWB) {
      int64_t row0 = -1;
      int wsp = 0;
      if (tgt) {
        const int64_t r = u / gpt, k = r / s_ns;
        const int sp = s_sp[r - k * s_ns];
        const int64_t tile = sp + k * S;
        if (tile < ntile) {
          row0 = tile * trows + (u - r * gpt) * 64;
          wsp = sp;
        }
      } else {
        row0 = u * 64;
        wsp = mask ? (int)((row0 / trows) % S) : 0;
      }
      if (row0 < 0) continue;  // (wave-uniform)
      const int64_t row = row0 + lane;
      // the wave's 64 rows are contiguous in the image: coalesced 1-KiB
      // LDS-DMA pieces into its own LDS tile (at the image's row stride rb,
      // an odd number of 16-B chunks: conflict-free ds_read_b128), then lane
      // = row reads its row there
      {
        const char* src = (const char*)(img + row0 * rb) + lane * 16;
        const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) signed char*)&rows_s[wv * 64 * kI8RescanRB];
        for (int p = 0; p * 1024 < 64 * rb; ++p) glds16(src + p * 1024, dst + p * 1024);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (row >= t.n) continue;  // (image rows >= n are padding)
      const signed char* xr = &rows_s[wv * 64 * kI8RescanRB + lane * rb];  // (copied at the image's stride)
      int xx = 0;
      int dot[FQ];
#pragma unroll
      for (int a = 0; a < FQ; ++a) dot[a] = 0;
      for (int ch = 0; ch < nch; ++ch) {
        const int4 xv = *(const int4*)(xr + 16 * ch);
        xx = __builtin_amdgcn_sdot4(xv.x, xv.x, xx, false);
        xx = __builtin_amdgcn_sdot4(xv.y, xv.y, xx, false);
        xx = __builtin_amdgcn_sdot4(xv.z, xv.z, xx, false);
        xx = __builtin_amdgcn_sdot4(xv.w, xv.w, xx, false);
#pragma unroll
        for (int a = 0; a < FQ; ++a) {
          const int4 qv = *(const int4*)(&qs[a][16 * ch]);
          int dd = dot[a];
          dd = __builtin_amdgcn_sdot4(xv.x, qv.x, dd, false);
          dd = __builtin_amdgcn_sdot4(xv.y, qv.y, dd, false);
          dd = __builtin_amdgcn_sdot4(xv.z, qv.z, dd, false);
          dd = __builtin_amdgcn_sdot4(xv.w, qv.w, dd, false);
          dot[a] = dd;
        }
      }
#pragma unroll
      for (int a = 0; a < FQ; ++a) {
        const long long r = (long long)qqs[a] + xx - 2ll * dot[a];
        if (((mask_s[a] >> wsp) & 1) && r <= ts[a]) {
          const int f = g0 + a;
          const int pos = atomicAdd(&fcnt[f], 1);
          if (pos < kRescanCap) buf[(int64_t)f * kRescanCap + pos] = train_row(t, (int)row);
        }
      }
    }
  }
}

// DP > 256 (rows too long to stage 64 per wave): 4 lanes per train row, 16
// rows per wave step; lane part p of row r reads float4 p, p+4, p+8, ... of
// the row (a wave-instruction covers 64 contiguous bytes of each of its 16
// rows, read in place from X32) against the queries in LDS, and the 4
// partial sums of each query are added by two xor-shuffles.  The fp32 error
// bound of the fmaf chain holds for any summation order (Higham 3.1).
template <int METRIC, int FQ>
__global__ void __launch_bounds__(256)
rescan_filter_wide_kernel(TrainDev t, const float* __restrict__ qf, const float* __restrict__ thr,
                          const int* __restrict__ cnt, int cap, int* __restrict__ fcnt,
                          int* __restrict__ buf, const unsigned long long* __restrict__ mask,
                          int S, int64_t trows) {
  const int nf = min(cnt[0], cap);
  if (nf == 0) return;
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  const int DP = t.DP, RSF = DP + 4;
  float* qs = fsm;             // [FQ][DP]
  float* thr_s = qs + FQ * DP; // [FQ]
  __shared__ unsigned long long mask_s[FQ];
  __shared__ unsigned long long s_u;
  const int tid = threadIdx.x, lane = tid & 63, part = lane & 3;
  if (tid == 0) {
    unsigned long long u = ~0ull;
    if (mask && nf <= 64) {
      u = 0;
      for (int f = 0; f < nf; ++f) u |= mask[f];
    }
    s_u = u;
  }
  __syncthreads();
  const unsigned long long need = s_u;
  const int64_t nrb = (t.n_pad + 63) / 64;
  for (int64_t rbk = blockIdx.x; rbk < nrb; rbk += gridDim.x) {
  const int64_t row = (rbk * 4 + (tid >> 6)) * 16 + (lane >> 2);
  const bool active = row < t.n_pad;
  // the block's 64 rows lie in one tile (64 | trows): its split
  const int bsp = mask ? (int)(((rbk * 64) / trows) % S) : 0;
  if (mask && !((need >> bsp) & 1)) continue;  // (block-uniform)
  const float* xr = t.X32 + (active ? row : 0) * RSF;
  for (int g0 = 0; g0 < nf; g0 += FQ) {
    const int nfg = min(FQ, nf - g0);
    __syncthreads();
    for (int e = tid; e < FQ * DP; e += blockDim.x) {
      const int qi = e / DP;
      qs[e] = qi < nfg ? qf[(int64_t)g0 * DP + e] : 0.0f;
    }
    if (tid < FQ) {
      thr_s[tid] = tid < nfg ? thr[g0 + tid] : -KNN_INF_F;
      mask_s[tid] = tid < nfg && mask ? mask[g0 + tid] : ~0ull;
    }
    __syncthreads();
    float acc[FQ];
#pragma unroll
    for (int qi = 0; qi < FQ; ++qi) acc[qi] = 0.0f;
#pragma unroll 4
    for (int c = 4 * part; c < DP; c += 16) {
      const float4 x4 = *(const float4*)(xr + c);
#pragma unroll
      for (int qi = 0; qi < FQ; ++qi) {
        if (qi >= nfg) break;  // group-uniform: no LDS reads for empty query slots
        const float4 q4 = *(const float4*)(qs + qi * DP + c);
        float a = acc[qi];
        if (METRIC == 0) {
          a = __builtin_fmaf(q4.x, x4.x, a);
          a = __builtin_fmaf(q4.y, x4.y, a);
          a = __builtin_fmaf(q4.z, x4.z, a);
          a = __builtin_fmaf(q4.w, x4.w, a);
        } else {
          a = a + __builtin_fabsf(q4.x - x4.x);
          a = a + __builtin_fabsf(q4.y - x4.y);
          a = a + __builtin_fabsf(q4.z - x4.z);
          a = a + __builtin_fabsf(q4.w - x4.w);
        }
        acc[qi] = a;
      }
    }
    const float seed = xr[METRIC == 0 ? DP : DP + 1];  // +inf on pad rows: never passes
#pragma unroll
    for (int qi = 0; qi < FQ; ++qi) {
      float a = acc[qi];
      a += __shfl_xor(a, 1, 64);
      a += __shfl_xor(a, 2, 64);
      acc[qi] = a + seed;
    }
    if (active && part == 0) {
#pragma unroll
      for (int qi = 0; qi < FQ; ++qi)
        if (qi < nfg && ((mask_s[qi] >> bsp) & 1))
          rescan_append(acc[qi], thr_s[qi], g0 + qi, row, t, fcnt, buf);
    }
  }
  }  // row blocks
}

// Exact re-rank of each fast-rescanned query's appended rows (a loop over
// the failed queries; the block's LDS is reused).  Queries it cannot finish
// are appended to slow_q (count cnt[1]) for the full scan.
// Dynamic LDS: qv[d] | dk[kRescanCap] | tb[NT][17] | di[kRescanCap] | ls[kRescanCap].
template <int METRIC, int NT>
__global__ void __launch_bounds__(NT)
rescan_finish_fast_kernel(TrainDev t, const double* __restrict__ Q64,
                          const int* __restrict__ rescan_q, const double* __restrict__ tau,
                          int* __restrict__ cnt, int cap, int W, const int* __restrict__ fcnt,
                          const int* __restrict__ buf, Sink sink, int* __restrict__ slow_q) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int nf = min(cnt[0], cap);
  const int d = t.d;
  const bool q_in_lds = d <= 1024;  // keeps the block's LDS under 64 KiB
  double* dk = (double*)smem + (q_in_lds ? d : 0);
  double* tb = dk + kRescanCap;
  int* di = (int*)(tb + NT * 17);
  int* ls = di + kRescanCap;
  const int tid = threadIdx.x;
  const int need_rows = (int)min((int64_t)W, t.n);
  for (int s = blockIdx.x; s < nf; s += gridDim.x) {
    __syncthreads();  // the previous query's LDS reads are done
    const int64_t q = rescan_q[s];
    const int c = fcnt[s];
    if (!(tau[s] < KNN_INF_D) || c > kRescanCap || c < need_rows) {
      if (tid == 0) slow_q[atomicAdd(&cnt[1], 1)] = (int)q;
      continue;
    }
    const double* qrow = Q64 + q * d;
    const double* qv = q_in_lds ? (const double*)smem : qrow;
    if (q_in_lds)
      for (int i = tid; i < d; i += NT) ((double*)smem)[i] = qrow[i];
    for (int i = tid; i < c; i += NT) di[i] = buf[(int64_t)s * kRescanCap + i];
    __syncthreads();
    int C2 = 1;
    while (C2 < c) C2 <<= 1;
    exact_sorted<METRIC, NT>(t, qv, di, dk, tb, c, C2, tid, NT * 17);
    const int need = sink.mode == MODE_SINGLE ? sink.k : sink.w;
    for (int i = tid; i < need && i < c; i += NT) ls[i] = t.lab[di[i]];
    __syncthreads();
    if (tid < 64) {
      if (sink.mode == MODE_SINGLE)
        finish_single(q, dk, di, ls, c, sink.k, sink.idx_off, 1 /*KNN_FLAG_EXACT_RESCAN*/, sink);
      else
        finish_partial(q, dk, di, ls, c, sink.w, sink.idx_off, sink);
    }
  }
}

// Full exact scan: one 1024-thread workgroup per query (a loop over the
// queries the fast path passed on, then the failed queries beyond `cap`).
// Each wave takes 64 rows per step: coalesced 64-B row pieces (8 lanes per
// row) go into the wave's own LDS tile as squared (L1: absolute)
// differences, and lane r adds its row's terms in dimension order -- the
// reference's operation order -- with no workgroup barrier inside the
// row's dimensions.  Rows with distance <= tau (the current W-th) are
// appended to an LDS buffer that holds the running top W in its first W
// slots; when it cannot take another step it is sorted by (dist, idx) and
// cut back to W.
// counts (host-mapped, nullable): {failed queries, full scans} of this call;
// totals (device): running sums of the same.
constexpr int kFullN = 4096;    // LDS candidate buffer (entries)
constexpr int kFullDC = 8;      // dims per staged row piece (64 B)
constexpr int kFullThreads = 1024;
template <int METRIC>
__global__ void __launch_bounds__(kFullThreads)
rescan_full_kernel(TrainDev t, const double* __restrict__ Q64, const int* __restrict__ rescan_q,
                   const int* __restrict__ cnt, int cap, const int* __restrict__ slow_q, int W,
                   Sink sink, int* __restrict__ counts, unsigned long long* __restrict__ totals) {
  __shared__ double sk[kFullN];
  __shared__ int si[kFullN];
  __shared__ double tiles[kFullThreads / 64][64 * (kFullDC + 1)];
  __shared__ int ls[kMaxK + 1];
  __shared__ int s_nb;
  __shared__ double s_tau;
  const int nslow = cnt[1];
  const int nover = max(0, cnt[0] - cap);
  const int total = nslow + nover;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (blockIdx.x == 0 && tid == 0) {
    if (counts) {
      counts[0] = cnt[0];
      counts[1] = total;
    }
    if (totals) {
      atomicAdd(&totals[0], (unsigned long long)cnt[0]);
      atomicAdd(&totals[1], (unsigned long long)total);
    }
  }
  const int d = t.d;
  const int64_t n = t.n;
  double* tb = tiles[wv];
  for (int f = blockIdx.x; f < total; f += gridDim.x) {
    const int64_t q = f < nslow ? slow_q[f] : rescan_q[cap + f - nslow];
    const double* qrow = Q64 + q * d;
    __syncthreads();  // the previous query's LDS reads are done
    for (int e = tid; e < W; e += kFullThreads) {
      sk[e] = KNN_INF_D;
      si[e] = INT_MAX;
    }
    if (tid == 0) {
      s_nb = W;
      s_tau = KNN_INF_D;
    }
    __syncthreads();
    for (int64_t s0 = 0; s0 < n; s0 += kFullThreads) {
      const int64_t r0 = s0 + wv * 64;  // this wave's 64 rows
      const int nr = (int)max((int64_t)0, min((int64_t)64, n - r0));
      double r = 0.0;
      for (int c0 = 0; c0 < d && nr > 0; c0 += kFullDC) {
        const int nd = min(kFullDC, d - c0);
#pragma unroll
        for (int i = 0; i < kFullDC; ++i) {
          const int e = lane + 64 * i, rr = e / kFullDC, j = e % kFullDC;
          double val = 0.0;
          if (rr < nr && j < nd) {
            const double tq = qrow[c0 + j] - t.X64[(r0 + rr) * d + c0 + j];
            val = METRIC == 0 ? tq * tq : __builtin_fabs(tq);
          }
          tb[rr * (kFullDC + 1) + j] = val;
        }
        // the wave's own tile: LDS operations of one wave complete in order
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (lane < nr) {
          const double* row = tb + lane * (kFullDC + 1);
          for (int j = 0; j < nd; ++j) r = r + row[j];
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      if (lane < nr) {
        const double dd = METRIC == 0 ? __builtin_sqrt(r) : r;
        if (dd <= s_tau) {
          const int pos = atomicAdd(&s_nb, 1);
          sk[pos] = dd;  // pos < kFullN: at most kFullThreads appends per step and
          si[pos] = (int)(r0 + lane);  // the buffer is cut back below kFullN - kFullThreads
        }
      }
      __syncthreads();
      const int nb = s_nb;
      if (nb > kFullN - kFullThreads || s0 + kFullThreads >= n) {
        for (int e = nb + tid; e < kFullN; e += kFullThreads) {
          sk[e] = KNN_INF_D;
          si[e] = INT_MAX;
        }
        bitonic_sort_lds(sk, si, kFullN, tid, kFullThreads);
        if (tid == 0) {
          s_nb = W;
          s_tau = sk[W - 1];
        }
        __syncthreads();
      }
    }
    const int cntq = (int)min((int64_t)W, n);
    const int need = sink.mode == MODE_SINGLE ? sink.k : sink.w;
    for (int i = tid; i < need && i < cntq; i += kFullThreads) ls[i] = t.lab[si[i]];
    __syncthreads();
    if (tid < 64) {
      if (sink.mode == MODE_SINGLE)
        finish_single(q, sk, si, ls, cntq, sink.k, sink.idx_off, 1 /*KNN_FLAG_EXACT_RESCAN*/, sink);
      else
        finish_partial(q, sk, si, ls, cntq, sink.w, sink.idx_off, sink);
    }
  }
}

void launch_rescan(int metric, const TrainDev& t, const double* Q64, const RescanBufs& rb, int cap,
                   int W, double f_err, const Sink& sink, int full_blocks, hipStream_t s) {
  if (cap > 0) {
    // per-split masks (targeted rescans) need the launch's split geometry
    const unsigned long long* mk = rb.S > 0 && rb.S <= 64 && rb.trows > 0 ? rb.mask : nullptr;
    const int mS = mk ? rb.S : 1;
    const int64_t mT = mk ? rb.trows : 64;
    constexpr int FQ = 16;
    const size_t qbytes = (size_t)FQ * (t.DP + 1) * 4;
    if (t.DP <= kRescanStageMaxDP) {
      // waves per block: as many 64-row tiles as fit beside the queries in ~150 KiB
      const size_t tile = (size_t)64 * (t.DP + 4) * 4;
      const int nwb = (int)std::max<size_t>(1, std::min<size_t>(4, (150 * 1024 - qbytes) / tile));
      const int64_t rpb = 64 * nwb;
      // (grid-stride over 64-row units, a targeted rescan's only over the
      // flagged splits' tiles; one block per CU -- its ~150 KiB of LDS admits
      // no second one)
      const dim3 fg((unsigned)std::min<int64_t>((t.n_pad + rpb - 1) / rpb, std::max(1, rb.cus)));
      const size_t flds = qbytes + nwb * tile;
      // the int8 filter first (its queries never pass the fp32 one): both
      // exit at once when they have no query
      const bool i8f = metric == 0 && rb.t8 && rb.qc8 && rb.i8img && rb.i8dp % 16 == 0 &&
                       rb.i8dp <= 256;
      if (i8f)
        hipLaunchKernelGGL((rescan_filter_i8_kernel<4>), dim3(std::max(1, rb.cus)), dim3(256), 0, s,
                           t, rb.i8img, rb.i8rb, rb.i8dp, rb.qc8, rb.t8, rb.cnt, cap, rb.fcnt,
                           rb.buf, mk, mS, mT);
      if (metric == 0)
        hipLaunchKernelGGL((rescan_filter_kernel<0, FQ>), fg, dim3(64 * nwb), flds, s, t, rb.qf,
                           rb.thr, rb.cnt, cap, rb.fcnt, rb.buf, mk, mS, mT, i8f ? rb.t8 : nullptr);
      else
        hipLaunchKernelGGL((rescan_filter_kernel<1, FQ>), fg, dim3(64 * nwb), flds, s, t, rb.qf,
                           rb.thr, rb.cnt, cap, rb.fcnt, rb.buf, mk, mS, mT, nullptr);
    } else {
      // 64 rows per 4-wave block; 8 queries per pass (a failed query is rare
      // at d > 256: the LDS of 8 query rows leaves room for 5 blocks per CU,
      // i.e. more row loads in flight than 2 blocks with 16 queries)
      constexpr int FQW = 8;
      const size_t qbw = (size_t)FQW * (t.DP + 1) * 4;
      const dim3 fg((unsigned)std::min<int64_t>((t.n_pad + 63) / 64, 4096));
      if (metric == 0)
        hipLaunchKernelGGL((rescan_filter_wide_kernel<0, FQW>), fg, dim3(256), qbw, s, t, rb.qf,
                           rb.thr, rb.cnt, cap, rb.fcnt, rb.buf, mk, mS, mT);
      else
        hipLaunchKernelGGL((rescan_filter_wide_kernel<1, FQW>), fg, dim3(256), qbw, s, t, rb.qf,
                           rb.thr, rb.cnt, cap, rb.fcnt, rb.buf, mk, mS, mT);
    }
    const size_t lds = (size_t)(t.d <= 1024 ? t.d : 0) * 8 + (size_t)kRescanCap * 8 +
                       (size_t)256 * 17 * 8 + (size_t)kRescanCap * 8;
    const int gf = std::min(cap, 512);
    if (metric == 0)
      hipLaunchKernelGGL((rescan_finish_fast_kernel<0, 256>), dim3(gf), dim3(256), lds, s, t, Q64,
                         rb.q, rb.tau, rb.cnt, cap, W, rb.fcnt, rb.buf, sink, rb.slow_q);
    else
      hipLaunchKernelGGL((rescan_finish_fast_kernel<1, 256>), dim3(gf), dim3(256), lds, s, t, Q64,
                         rb.q, rb.tau, rb.cnt, cap, W, rb.fcnt, rb.buf, sink, rb.slow_q);
  }
  if (full_blocks <= 0) return;  // (timing-only ablations)
  const int gs = full_blocks;
  if (metric == 0)
    hipLaunchKernelGGL(rescan_full_kernel<0>, dim3(gs), dim3(kFullThreads), 0, s, t, Q64, rb.q,
                       rb.cnt, cap, rb.slow_q, W, sink, rb.counts, rb.totals);
  else
    hipLaunchKernelGGL(rescan_full_kernel<1>, dim3(gs), dim3(kFullThreads), 0, s, t, Q64, rb.q,
                       rb.cnt, cap, rb.slow_q, W, sink, rb.counts, rb.totals);
}

// ------------------------------------------------ reference tie order
// The reference sorts all N_train records {label, dis} of a query with
// std::sort (cpp:323/366): libstdc++'s introsort, which is not stable -- the
// order it leaves among EXACTLY equal distances follows from its pivots and
// swaps over the whole array.  The vote (cpp:324-337) reads the labels in that
// order, so a query whose top k holds equal distances with different labels
// (or a tie across the k-th place) can get a different label under any other
// tie order.  For such queries this pass recomputes every row's exact
// distance in the reference's fill order (d[j] for j = 0..n-1, cpp:360-365)
// and runs the libstdc++ (GCC 11, bits/stl_algo.h / stl_heap.h) algorithm
// itself, restricted to the sub-ranges that can reach the first k positions:
//   __introsort_loop: while a range holds > 16 records: depth limit 0 ->
//     heap sort (__partial_sort of the whole range); else median-of-3 of
//     (first+1, mid, last-1) swapped to first, Hoare-style
//     __unguarded_partition of [first+1, last) around *first, recurse on the
//     right part, loop on the left;
//   __final_insertion_sort: insertion sort (strict <) over the whole array.
// Every partition leaves left <= pivot <= right, so a record never leaves the
// range it was partitioned into: ranges starting at or beyond k cannot reach
// positions < k and are skipped, and the insertion sort over [0, E) -- E the
// end of the last range that starts below k -- gives positions < k exactly.
// The partition itself runs in parallel: its left scan stops at the records
// >= pivot (ascending), its right scan at the records <= pivot (descending);
// the t-th swap exchanges the t-th of each until they cross (T), and the
// cut is min(L[T], R[T-1]) (after a swap the left scan also stops at the
// swapped-in record).  Pairs t < T never share a position, so the swaps are
// independent.
constexpr int kTieThreads = 1024;
constexpr int kTieStack = 64;  // > 2 log2(2^31): one pending left range per depth level

struct RefSortShared {
  int sc[2 * (kTieThreads / 64) + 2];  // block scan
  int st_f[kTieStack], st_l[kTieStack], st_d[kTieStack];
  int sp, cut, T, done, emax;
  double pv;
};

// Exclusive prefix of a and inclusive prefix of b over the threads (in
// thread order), and their totals.  All threads; sh is reused on return.
__device__ void block_scan2(int a, int b, int& a_ex, int& b_in, int& a_tot, int& b_tot, int* sh) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int ai = a, bi = b;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int x = __shfl_up(ai, o, 64), y = __shfl_up(bi, o, 64);
    if (lane >= o) { ai += x; bi += y; }
  }
  if (lane == 63) { sh[wv] = ai; sh[nw + wv] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int sa = 0, sb = 0;
    for (int w = 0; w < nw; ++w) {
      const int ta = sh[w], tb = sh[nw + w];
      sh[w] = sa; sh[nw + w] = sb;
      sa += ta; sb += tb;
    }
    sh[2 * nw] = sa; sh[2 * nw + 1] = sb;
  }
  __syncthreads();
  a_ex = sh[wv] + ai - a;
  b_in = sh[nw + wv] + bi;
  a_tot = sh[2 * nw];
  b_tot = sh[2 * nw + 1];
  __syncthreads();
}

__device__ __forceinline__ void rec_swap(double* D, int* P, int a, int b) {
  const double t = D[a]; D[a] = D[b]; D[b] = t;
  const int p = P[a]; P[a] = P[b]; P[b] = p;
}

// std::__unguarded_partition_pivot on [f, l) (l - f > 16); returns the cut.
__device__ int ref_partition(double* D, int* P, int* Lb, int* Rb, int f, int l, RefSortShared& s) {
  const int tid = threadIdx.x, nt = blockDim.x;
  if (tid == 0) {  // __move_median_to_first(first, first + 1, mid, last - 1)
    const int a = f + 1, b = f + (l - f) / 2, c = l - 1;
    const double da = D[a], db = D[b], dc = D[c];
    int m;
    if (da < db) m = db < dc ? b : (da < dc ? c : a);
    else m = da < dc ? a : (db < dc ? c : b);
    rec_swap(D, P, f, m);
    s.pv = D[f];
  }
  __syncthreads();
  const double pv = s.pv;
  const int seg = (l - f + nt - 1) / nt;
  const int a0 = min(l, f + tid * seg), a1 = min(l, a0 + seg);
  int cg = 0, ce = 0;
  for (int i = a0; i < a1; ++i) {
    const double v = D[i];
    cg += i > f && !(v < pv);  // left scan stops: !(*first < pivot)
    ce += !(pv < v);           // right scan stops: !(pivot < *last)
  }
  int g_ex, e_in, g_tot, e_tot;
  block_scan2(cg, ce, g_ex, e_in, g_tot, e_tot, s.sc);
  for (int i = a0, r = g_ex; i < a1; ++i)
    if (i > f && !(D[i] < pv)) Lb[r++] = i;
  for (int i = a1 - 1, r = e_tot - e_in; i >= a0; --i)  // right stops in descending order
    if (!(pv < D[i])) Rb[r++] = i;
  __syncthreads();
  if (tid == 0) {
    int lo = 0, hi = min(g_tot, e_tot);  // first t with L[t] >= R[t] (monotone)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (Lb[mid] >= Rb[mid]) hi = mid; else lo = mid + 1;
    }
    const int LT = lo < g_tot ? Lb[lo] : l;
    s.T = lo;
    s.cut = lo == 0 ? LT : min(LT, Rb[lo - 1]);
  }
  __syncthreads();
  const int T = s.T;
  for (int t = tid; t < T; t += nt) rec_swap(D, P, Lb[t], Rb[t]);
  __syncthreads();
  return s.cut;
}

// std::__adjust_heap / __push_heap over records [f, f + len) (one thread)
__device__ void ref_adjust_heap(double* D, int* P, int f, int hole, int len, double v, int pv) {
  const int top = hole;
  int sc = hole;
  while (sc < (len - 1) / 2) {
    sc = 2 * (sc + 1);
    if (D[f + sc] < D[f + sc - 1]) sc--;
    D[f + hole] = D[f + sc]; P[f + hole] = P[f + sc];
    hole = sc;
  }
  if ((len & 1) == 0 && sc == (len - 2) / 2) {
    sc = 2 * (sc + 1);
    D[f + hole] = D[f + sc - 1]; P[f + hole] = P[f + sc - 1];
    hole = sc - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && D[f + parent] < v) {
    D[f + hole] = D[f + parent]; P[f + hole] = P[f + parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  D[f + hole] = v; P[f + hole] = pv;
}

// std::__partial_sort(first, last, last): __make_heap + __sort_heap (one thread)
__device__ void ref_heap_sort(double* D, int* P, int f, int l) {
  const int len = l - f;
  if (len >= 2)
    for (int parent = (len - 2) / 2;; --parent) {
      ref_adjust_heap(D, P, f, parent, len, D[f + parent], P[f + parent]);
      if (parent == 0) break;
    }
  for (int last = len; last > 1;) {  // __pop_heap(first, last, last)
    --last;
    const double v = D[f + last];
    const int pv = P[f + last];
    D[f + last] = D[f]; P[f + last] = P[f];
    ref_adjust_heap(D, P, f, 0, last, v, pv);
  }
}

// std::sort of records (D[j], P[j]), j < n, by D, as libstdc++ leaves
// positions [0, k) (above).  All threads of the block.
__device__ void ref_sort_prefix(double* D, int* P, int* Lb, int* Rb, int n, int k,
                                RefSortShared& s) {
  const int tid = threadIdx.x;
  if (tid == 0) {
    s.sp = 0;
    s.emax = 0;
  }
  int f = 0, l = n, dl = n > 1 ? 2 * (31 - __clz(n)) : 0;  // std::__lg(n) * 2
  __syncthreads();
  while (true) {
    if (l - f > 16 && f < k) {
      if (dl == 0) {
        if (tid == 0) {
          ref_heap_sort(D, P, f, l);
          s.emax = max(s.emax, l);
        }
        __syncthreads();
      } else {
        --dl;
        const int cut = ref_partition(D, P, Lb, Rb, f, l, s);
        // recurse on the right part first (as __introsort_loop), keep the left
        if (tid == 0) {
          s.st_f[s.sp] = f; s.st_l[s.sp] = cut; s.st_d[s.sp] = dl;
          ++s.sp;
        }
        f = cut;
        continue;
      }
    } else if (f < k && tid == 0) {
      s.emax = max(s.emax, l);  // a range left to the final insertion sort
    }
    __syncthreads();
    if (tid == 0) {
      s.done = s.sp == 0;
      if (!s.done) --s.sp;
    }
    __syncthreads();
    if (s.done) break;
    f = s.st_f[s.sp]; l = s.st_l[s.sp]; dl = s.st_d[s.sp];
    __syncthreads();
  }
  if (tid == 0) {  // __final_insertion_sort, positions [0, emax)
    const int e = min(n, s.emax);
    for (int i = 1; i < e; ++i) {
      const double v = D[i];
      const int p = P[i];
      int j = i;
      for (; j > 0 && v < D[j - 1]; --j) { D[j] = D[j - 1]; P[j] = P[j - 1]; }
      D[j] = v; P[j] = p;
    }
  }
  __syncthreads();
}

// Exact distances of rows [r_begin, r_end) to qrow (reference operation
// order, as rescan_full) into D[j] (absolute row index j): per-wave staged
// 64-B row pieces.  All threads.
template <int METRIC>
__device__ void exact_rows_dist(const TrainDev& t, const double* qrow, int64_t r_begin,
                                int64_t r_end, double* D, double* tb) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nt = blockDim.x;
  const int d = t.d;
  const int64_t n = r_end;
  for (int64_t s0 = r_begin; s0 < n; s0 += nt) {
    const int64_t r0 = s0 + wv * 64;
    const int nr = (int)max((int64_t)0, min((int64_t)64, n - r0));
    double r = 0.0;
    for (int c0 = 0; c0 < d && nr > 0; c0 += kFullDC) {
      const int nd = min(kFullDC, d - c0);
#pragma unroll
      for (int i = 0; i < kFullDC; ++i) {
        const int e = lane + 64 * i, rr = e / kFullDC, j = e % kFullDC;
        double val = 0.0;
        if (rr < nr && j < nd) {
          const double tq = qrow[c0 + j] - t.X64[(r0 + rr) * d + c0 + j];
          val = METRIC == 0 ? tq * tq : __builtin_fabs(tq);
        }
        tb[rr * (kFullDC + 1) + j] = val;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (lane < nr) {
        const double* row = tb + lane * (kFullDC + 1);
        for (int j = 0; j < nd; ++j) r = r + row[j];
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    if (lane < nr) D[r0 + lane] = METRIC == 0 ? __builtin_sqrt(r) : r;
  }
}

template <int METRIC>
__device__ void exact_all_dist(const TrainDev& t, const double* qrow, double* D, double* tb) {
  exact_rows_dist<METRIC>(t, qrow, 0, t.n, D, tb);
}

// Outputs of a query whose first k records are in reference order: the
// vote exactly as cpp:324-337 (sequential, per-class counts in `cnt`; lab
// indexed by the records' row numbers P), idx = P + idx_base, dist, flags
// |= KNN_FLAG_TIE_REF (and KNN_FLAG_TIE_PENDING cleared).  All threads.
__device__ void ref_finish(int64_t q, const double* D, const int* P, int k, const int32_t* lab,
                           int64_t idx_base, int class_cnt, int* cnt, const Sink& sink) {
  const int tid = threadIdx.x;
  for (int c = tid; c < class_cnt; c += blockDim.x) cnt[c] = 0;
  __syncthreads();
  if (tid == 0) {
    int best = 0, winner = -1;
    for (int i = 0; i < k; ++i) {
      const int lb = lab[P[i]];
      if ((unsigned)lb >= (unsigned)class_cnt) continue;  // (labels are range-checked at set_train)
      const int c = ++cnt[lb];
      if (c > best) { best = c; winner = lb; }
    }
    sink.labels[q] = winner;
    if (sink.flags) sink.flags[q] = (sink.flags[q] & ~kFlagTiePending) | kFlagTieRef;
  }
  for (int i = tid; i < k; i += blockDim.x) {
    if (sink.idx) sink.idx[q * k + i] = (int64_t)P[i] + idx_base;
    if (sink.dist) sink.dist[q * k + i] = D[i];
  }
  __syncthreads();
}

// per workgroup: D[n] f64 | P[n] | Lb[n] | Rb[n] | class counts
int64_t tie_scratch_bytes(int64_t n, int class_cnt) {
  return (n * 20 + (int64_t)class_cnt * 4 + 255) / 256 * 256;
}

template <int METRIC>
__global__ void __launch_bounds__(kTieThreads)
tie_order_kernel(TrainDev t, const double* __restrict__ Q64, const int* __restrict__ tie_q,
                 const int* __restrict__ tie_cnt, int class_cnt, unsigned char* __restrict__ scratch,
                 int64_t per_wg, Sink sink, unsigned long long* totals) {
  __shared__ double tiles[kTieThreads / 64][64 * (kFullDC + 1)];
  __shared__ RefSortShared s;
  const int count = *tie_cnt;
  if (blockIdx.x == 0 && threadIdx.x == 0 && totals && count)
    atomicAdd(totals, (unsigned long long)count);  // running count of re-ordered queries
  const int64_t n = t.n;
  unsigned char* base = scratch + (int64_t)blockIdx.x * per_wg;
  double* D = (double*)base;
  int* P = (int*)(D + n);
  int* Lb = P + n;
  int* Rb = Lb + n;
  int* cnt = Rb + n;
  for (int i = blockIdx.x; i < count; i += gridDim.x) {
    const int64_t q = tie_q[i];
    exact_all_dist<METRIC>(t, Q64 + q * t.d, D, tiles[threadIdx.x >> 6]);
    for (int64_t j = threadIdx.x; j < n; j += kTieThreads) P[j] = (int)j;
    __syncthreads();
    ref_sort_prefix(D, P, Lb, Rb, (int)n, sink.k, s);
    ref_finish(q, D, P, sink.k, t.lab, sink.idx_off, class_cnt, cnt, sink);
  }
}

// ---- the same for the train-sharded mode (north_star mode b).  The
// reference's std::sort runs over all N_train records of the WHOLE train set
// in global row order (cpp:360-366), so its order among equal distances
// depends on every shard's distances.  After the k-way merge flags a query
// KNN_FLAG_TIE_PENDING, every shard computes that query's exact distances to
// all of its rows (shard_dist_kernel), the blocks travel to the query's owner
// (an all-to-all: RCCL send/recv in knn_group, torch.distributed in
// knn_dist.py), which assembles them in global row order and runs the same
// introsort emulation and vote (tie_resolve_kernel).

// out[i][j] = exact distance of shard row j to query qsel[i] (qsel null: i).
// Grid (ceil(n / kTieThreads), nsel): one 1024-row chunk of one query.
template <int METRIC>
__global__ void __launch_bounds__(kTieThreads)
shard_dist_kernel(TrainDev t, const double* __restrict__ Q64, const int* __restrict__ qsel,
                  double* __restrict__ out) {
  __shared__ double tiles[kTieThreads / 64][64 * (kFullDC + 1)];
  const int64_t i = blockIdx.y;
  const int64_t q = qsel ? qsel[i] : i;
  const int64_t r0 = (int64_t)blockIdx.x * kTieThreads;
  exact_rows_dist<METRIC>(t, Q64 + q * t.d, r0, min(t.n, r0 + kTieThreads), out + i * t.n,
                          tiles[threadIdx.x >> 6]);
}

void launch_shard_dist(int metric, const TrainDev& t, const double* Q64, const int* qsel, int nsel,
                       double* out, hipStream_t s) {
  const unsigned nx = (unsigned)((t.n + kTieThreads - 1) / kTieThreads);
  for (int i0 = 0; i0 < nsel; i0 += 65535) {  // grid y limit
    const int ny = min(65535, nsel - i0);
    const int* qs = qsel ? qsel + i0 : nullptr;
    double* o = out + (int64_t)i0 * t.n;
    const double* Qb = qsel ? Q64 : Q64 + (int64_t)i0 * t.d;
    if (metric == 0)
      hipLaunchKernelGGL(shard_dist_kernel<0>, dim3(nx, ny), dim3(kTieThreads), 0, s, t, Qb, qs, o);
    else
      hipLaunchKernelGGL(shard_dist_kernel<1>, dim3(nx, ny), dim3(kTieThreads), 0, s, t, Qb, qs, o);
  }
}

// D: the nsel queries' distances to every row as parts blocks, block p =
// [nsel][rows_p] at offset nsel * off[p] (global rows off[p] .. off[p+1]).
// Output row orow[i] of the sink (labels / idx / dist / flags).
__global__ void __launch_bounds__(kTieThreads)
tie_resolve_kernel(const double* __restrict__ Din, PartRows pr, int nsel,
                   const int32_t* __restrict__ lab_all, const int* __restrict__ orow, int class_cnt,
                   unsigned char* __restrict__ scratch, int64_t per_wg, Sink sink,
                   unsigned long long* totals) {
  __shared__ RefSortShared s;
  const int64_t n = pr.off[pr.parts];
  if (blockIdx.x == 0 && threadIdx.x == 0 && totals) atomicAdd(totals, (unsigned long long)nsel);
  unsigned char* base = scratch + (int64_t)blockIdx.x * per_wg;
  double* D = (double*)base;
  int* P = (int*)(D + n);
  int* Lb = P + n;
  int* Rb = Lb + n;
  int* cnt = Rb + n;
  for (int i = blockIdx.x; i < nsel; i += gridDim.x) {
    for (int p = 0; p < pr.parts; ++p) {  // global row order = the reference's fill order
      const int64_t o = pr.off[p], rows = pr.off[p + 1] - o;
      const double* src = Din + (int64_t)nsel * o + (int64_t)i * rows;
      for (int64_t j = threadIdx.x; j < rows; j += kTieThreads) {
        D[o + j] = src[j];
        P[o + j] = (int)(o + j);
      }
    }
    __syncthreads();
    ref_sort_prefix(D, P, Lb, Rb, (int)n, sink.k, s);
    ref_finish(orow[i], D, P, sink.k, lab_all, 0, class_cnt, cnt, sink);
  }
}

void launch_tie_resolve(const double* D, const PartRows& pr, int nsel, const int32_t* lab_all,
                        const int* orow, int class_cnt, unsigned char* scratch, int64_t per_wg,
                        int nwg, const Sink& sink, unsigned long long* totals, hipStream_t s) {
  if (nwg <= 0 || nsel <= 0) return;
  hipLaunchKernelGGL(tie_resolve_kernel, dim3(nwg), dim3(kTieThreads), 0, s, D, pr, nsel, lab_all,
                     orow, class_cnt, scratch, per_wg, sink, totals);
}

void launch_tie_order(int metric, const TrainDev& t, const double* Q64, const int* tie_q,
                      const int* tie_cnt, int class_cnt, unsigned char* scratch, int64_t per_wg,
                      int nwg, const Sink& sink, unsigned long long* totals, hipStream_t s) {
  if (nwg <= 0) return;
  if (metric == 0)
    hipLaunchKernelGGL(tie_order_kernel<0>, dim3(nwg), dim3(kTieThreads), 0, s, t, Q64, tie_q,
                       tie_cnt, class_cnt, scratch, per_wg, sink, totals);
  else
    hipLaunchKernelGGL(tie_order_kernel<1>, dim3(nwg), dim3(kTieThreads), 0, s, t, Q64, tie_q,
                       tie_cnt, class_cnt, scratch, per_wg, sink, totals);
}

// ------------------------------------------------ large k (k > kMaxK)
// The candidate lists hold at most kMaxUnion entries, so a k beyond kMaxK
// (the reference accepts any K <= N_train, cpp:328) runs this exact path
// instead: one 1024-thread workgroup per query (a loop over the queries),
// with its own global scratch.
//  1. every row's exact fp64 distance in the reference's operation order
//     (per-wave staged 64-B row pieces as in rescan_full) -> D[n];
//  2. the key (bit pattern; distances are >= 0) of the W-th smallest by a
//     radix select, 11 bits per pass, LDS histograms;
//  3. rows below the pivot plus the lowest-index rows equal to it (an
//     index-ordered scan) -> W entries, sorted by (dist, idx) (bitonic in the
//     scratch);
//  4. the reference vote, sequentially as in cpp:324-337 (per-class counts
//     in the scratch), flags, outputs.
constexpr int kLkThreads = 1024;
constexpr int kLkBits = 11;
__device__ __forceinline__ uint64_t lk_key(double v) { return (uint64_t)__double_as_longlong(v); }

template <int METRIC>
__global__ void __launch_bounds__(kLkThreads)
large_k_kernel(TrainDev t, const double* __restrict__ Q64, int64_t m, int W, int class_cnt,
               unsigned char* __restrict__ scratch, int64_t scratch_per_wg, Sink sink) {
  __shared__ double tiles[kLkThreads / 64][64 * (kFullDC + 1)];
  __shared__ unsigned hist[1 << kLkBits];
  __shared__ uint64_t s_prefix;
  __shared__ int s_rank, s_nlt, s_neq, s_bad;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int d = t.d;
  const int64_t n = t.n;
  int W2 = 1;
  while (W2 < W) W2 <<= 1;
  unsigned char* base = scratch + (int64_t)blockIdx.x * scratch_per_wg;
  double* D = (double*)base;                       // [n]
  double* od = D + n;                              // [W2]
  int* oi = (int*)(od + W2);                       // [W2]
  int* ol = oi + W2;                               // [W2] labels in sorted order
  int* cnt = ol + W2;                              // [class_cnt] vote counts
  __shared__ int s_flags;
  double* tb = tiles[wv];
  for (int64_t q = blockIdx.x; q < m; q += gridDim.x) {
    const double* qrow = Q64 + q * d;
    __syncthreads();
    if (tid == 0) s_bad = 0;
    __syncthreads();
    for (int c = tid; c < d; c += kLkThreads)
      if (nonfinite_bits(qrow[c])) s_bad = 1;  // (this TU: -fno-honor-nans)
    __syncthreads();
    if (s_bad) {  // a NaN / inf coordinate: no neighbours (as the merge reports it)
      if (tid < 64) finish_nonfinite(q, sink);
      continue;
    }
    // 1. exact distances
    exact_all_dist<METRIC>(t, qrow, D, tb);
    // 2. radix select of the W-th smallest key (digits from the top)
    if (tid == 0) {
      s_prefix = 0;
      s_rank = W;  // rank still to find among keys matching the prefix
    }
    for (int shift = 64 - kLkBits; shift > -kLkBits; shift -= kLkBits) {
      const int sh = max(shift, 0);
      const int nbits = shift >= 0 ? kLkBits : kLkBits + shift;  // last digit: the low bits
      const uint64_t hi_mask = (sh + nbits >= 64) ? 0 : (~0ull << (sh + nbits));
      __syncthreads();  // the previous pass's digit choice has read hist
      for (int b = tid; b < (1 << kLkBits); b += kLkThreads) hist[b] = 0;
      __syncthreads();  // (also publishes D and the previous pass's prefix)
      const uint64_t pre = s_prefix;
      for (int64_t r = tid; r < n; r += kLkThreads) {
        const uint64_t k = lk_key(D[r]);
        if ((k & hi_mask) == pre) atomicAdd(&hist[(k >> sh) & ((1u << nbits) - 1)], 1u);
      }
      __syncthreads();
      if (tid == 0) {
        int rank = s_rank;
        unsigned b = 0;
        for (; b < (1u << nbits); ++b) {
          if ((int)hist[b] >= rank) break;
          rank -= hist[b];
        }
        s_prefix = pre | ((uint64_t)b << sh);
        s_rank = rank;
      }
    }
    __syncthreads();
    const uint64_t pivot = s_prefix;  // key of the W-th smallest distance
    // 3. the W smallest by (dist, idx): all keys below the pivot (unordered),
    //    then the lowest-index rows equal to it (ordered scan)
    if (tid == 0) { s_nlt = 0; s_neq = 0; }
    __syncthreads();
    for (int64_t r = tid; r < n; r += kLkThreads)
      if (lk_key(D[r]) < pivot) {
        const int p = atomicAdd(&s_nlt, 1);
        od[p] = D[r];
        oi[p] = (int)r;
      }
    __syncthreads();
    const int nlt = s_nlt;  // < W
    for (int64_t s0 = 0; s0 < n; s0 += kLkThreads) {
      const int64_t r = s0 + tid;
      const bool eq = r < n && lk_key(D[r]) == pivot;
      // index-ordered positions: wave prefix, then the waves in order
      const unsigned long long mk = __ballot(eq);
      const int before_w = __popcll(mk & ((1ull << lane) - 1));
      if (lane == 0) hist[wv] = __popcll(mk);
      __syncthreads();
      int off = s_neq;
      for (int x = 0; x < wv; ++x) off += hist[x];
      const int p = nlt + off + before_w;
      if (eq && p < W) {
        od[p] = D[r];
        oi[p] = (int)r;
      }
      __syncthreads();
      if (tid == 0) {
        int tot = 0;
        for (int x = 0; x < kLkThreads / 64; ++x) tot += hist[x];
        s_neq += tot;
      }
      __syncthreads();
      if (nlt + s_neq >= W) break;
    }
    for (int c = W + tid; c < W2; c += kLkThreads) {
      od[c] = KNN_INF_D;
      oi[c] = INT_MAX;
    }
    bitonic_sort_lds(od, oi, W2, tid, kLkThreads);  // (global scratch; same code path)
    // 4. labels, vote, outputs
    const int need = sink.mode == MODE_SINGLE ? sink.k : sink.w;
    for (int c = tid; c < need && c < W; c += kLkThreads) ol[c] = t.lab[oi[c]];
    for (int c = tid; c < class_cnt; c += kLkThreads) cnt[c] = 0;
    __syncthreads();
    if (sink.mode == MODE_SINGLE) {
      const int k = sink.k;
      if (tid == 0) {  // cpp:324-337, sequentially: the first label to strictly exceed
        int best = 0, lab = -1;
        for (int i = 0; i < k; ++i) {
          const int c = ++cnt[ol[i]];
          if (c > best) { best = c; lab = ol[i]; }
        }
        sink.labels[q] = lab;
        int m2 = 0;  // runner-up count (see finish_single)
        for (int c = 0; c < class_cnt; ++c)
          if (c != lab) m2 = max(m2, cnt[c]);
        s_rank = best - m2;  // (s_rank is free here)
      }
      int tie = 0;
      for (int i = tid; i + 1 < k; i += kLkThreads)
        if (od[i] == od[i + 1]) tie |= ol[i] != ol[i + 1] ? 4 : 8;
      if (tie) atomicOr(&s_bad, tie);  // s_bad is 0 here: reused for the flags
      __syncthreads();
      if (tid == 0) {
        int f = s_bad;
        const bool bnd = k < W && od[k - 1] == od[k];
        if (bnd) f |= 2;  // KNN_FLAG_TIE_BOUNDARY
        if (sink.flags) sink.flags[q] = f;
        int gin = 0;
        for (int i = k - 1; bnd && i >= 0 && od[i] == od[k - 1]; --i) ++gin;
        // queue for the reference-order pass: the rule of finish_single
        s_flags = sink.tie_mode == 2 ? (f & 14) != 0
                : sink.tie_mode == 1 ? (bnd && s_rank <= 2 * gin) || ((f & 4) && s_rank == 0)
                                     : 0;
      }
      for (int i = tid; i < k; i += kLkThreads) {
        if (sink.idx) sink.idx[q * k + i] = (int64_t)oi[i] + sink.idx_off;
        if (sink.dist) sink.dist[q * k + i] = od[i];
      }
      // exact ties: queued for the reference-order pass (tie_order_kernel)
      if (tid == 0 && s_flags) sink.tie_q[atomicAdd(sink.tie_cnt, 1)] = (int)q;
    } else {
      for (int i = tid; i < sink.w; i += kLkThreads) {
        const bool ok = i < W;
        sink.dist[q * sink.w + i] = ok ? od[i] : KNN_INF_D;
        sink.idx[q * sink.w + i] = ok ? (int64_t)oi[i] + sink.idx_off : -1;
        sink.plab[q * sink.w + i] = ok ? ol[i] : -1;
      }
    }
  }
}

int64_t large_k_scratch_bytes(int64_t n, int W, int class_cnt) {
  int64_t W2 = 1;
  while (W2 < W) W2 <<= 1;
  return ((n * 8 + W2 * 16 + (int64_t)class_cnt * 4) + 255) / 256 * 256;
}

void launch_large_k(int metric, const TrainDev& t, const double* Q64, int64_t m, int W,
                    int class_cnt, unsigned char* scratch, int64_t per_wg, int nwg,
                    const Sink& sink, hipStream_t s) {
  if (m <= 0) return;
  const dim3 g((unsigned)std::min<int64_t>(m, nwg));
  if (metric == 0)
    hipLaunchKernelGGL(large_k_kernel<0>, g, dim3(kLkThreads), 0, s, t, Q64, m, W, class_cnt,
                       scratch, per_wg, sink);
  else
    hipLaunchKernelGGL(large_k_kernel<1>, g, dim3(kLkThreads), 0, s, t, Q64, m, W, class_cnt,
                       scratch, per_wg, sink);
}

// ------------------------------------------ train-sharded k-way merge + vote
// lists [parts][m][w] sorted by (dist, global idx); one wave per query merges
// them (bitonic in LDS) and runs the reference vote on the first k.
__global__ void __launch_bounds__(64)
merge_vote_partials_kernel(const double* __restrict__ dist, const int64_t* __restrict__ idx,
                           const int32_t* __restrict__ lab, int parts, int64_t m, int w, int k,
                           int P2, int64_t q0, int64_t pstride, Sink sink) {
  // pstride = 0: three arrays [parts][m][w]; pstride > 0: one packed buffer
  // per part at byte offset p * pstride from dist, holding that part's
  // [m][w] dists | [m][w] idx | [m][w] labels (knn_group's single all-gather)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* dk = (double*)smem;
  int64_t* gi = (int64_t*)(dk + P2);
  int* ls = (int*)(gi + P2);
  const int64_t q = q0 + blockIdx.x;  // query in the [parts][m][w] lists
  const int64_t qo = blockIdx.x;      // row in the outputs
  const int lane = threadIdx.x;
  const int ne = parts * w;
  auto entry = [&](int e, double& v, int64_t& id, int32_t& lb) {
    const int p = e / w, c = e - p * w;
    if (pstride > 0) {
      const unsigned char* pb = (const unsigned char*)dist + p * pstride;
      const int64_t o = q * w + c, mw = m * w;
      v = ((const double*)pb)[o];
      id = ((const int64_t*)(pb + 8 * mw))[o];
      lb = ((const int32_t*)(pb + 16 * mw))[o];
    } else {
      const int64_t src = ((int64_t)p * m + q) * w + c;
      v = dist[src];
      id = idx[src];
      lb = lab[src];
    }
  };
  for (int e = lane; e < P2; e += 64) {
    double v = KNN_INF_D;
    int64_t id = LLONG_MAX;
    if (e < ne) {
      double ev;
      int64_t eid;
      int32_t elb;
      entry(e, ev, eid, elb);
      if (eid >= 0) { v = ev; id = eid; }
    }
    dk[e] = v;
    gi[e] = id;
    ls[e] = -1;  // fewer than k entries (tiny shards, non-finite queries): label -1
  }
  bitonic_sort_lds(dk, gi, P2, lane, 64);
  // labels travel with the lists: place each one at its entry's sorted slot
  for (int e = lane; e < ne; e += 64) {
    double v;
    int64_t id;
    int32_t lb;
    entry(e, v, id, lb);
    if (id < 0) continue;
    // position of (dist, idx) in the sorted array: binary search
    int lo = 0, hi = P2;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (pair_less(dk[mid], gi[mid], v, id)) lo = mid + 1; else hi = mid;
    }
    if (lo < k + 1) ls[lo] = lb;
  }
  __syncthreads();
  int cnt = 0;
  for (int e = lane; e < P2; e += 64) cnt += (gi[e] != LLONG_MAX);
  cnt = wave_sum_i(cnt);
  if (cnt == 0 && k > 0) {  // no shard listed a neighbour: a non-finite query
    finish_nonfinite(qo, sink);
    return;
  }
  int bc = 0, bt = INT_MAX;
  for (int t = lane; t < k; t += 64) {
    const int lt = ls[t];
    int c = 0;
    for (int s2 = 0; s2 <= t; ++s2) c += (ls[s2] == lt);
    if (c > bc) { bc = c; bt = t; }
  }
  const int M = wave_max_i(bc);
  const int tmin = wave_min_i(bc == M ? bt : INT_MAX);
  const int winner = k > 0 ? ls[tmin] : -1;
  const int kk = min(k, cnt);  // slots [kk, k) are empty (fewer rows than k)
  int tie = 0;
  for (int t = lane; t + 1 < kk; t += 64)
    if (dk[t] == dk[t + 1]) tie |= ls[t] != ls[t + 1] ? 4 : 8;
  tie = wave_or_i(tie);
  const bool bnd = k > 0 && k < cnt && dk[k - 1] == dk[k];
  // the order among equal distances across shards is the reference's
  // std::sort's over the whole train set: flagged for the exchange of
  // knn_group / knn_dist.py and tie_resolve_kernel
  const bool pend = kk == k &&
                    tie_order_matters([&](int t) { return ls[t]; }, [&](int t) { return dk[t]; },
                                      k, winner, M, tie, bnd, sink.tie_mode);
  if (lane == 0) {
    sink.labels[qo] = winner;
    if (sink.flags) sink.flags[qo] = tie | (bnd ? 2 : 0) | (pend ? kFlagTiePending : 0);
    if (pend && sink.tie_q) sink.tie_q[atomicAdd(sink.tie_cnt, 1)] = (int)qo;
  }
  for (int t = lane; t < k; t += 64) {
    if (sink.idx) sink.idx[qo * k + t] = t < kk ? gi[t] : -1;
    if (sink.dist) sink.dist[qo * k + t] = t < kk ? dk[t] : KNN_INF_D;
  }
}

// ---- the same merge for unions beyond the LDS image (parts * w > 4096:
// e.g. 8 GPUs at k >= 512; the reference accepts any K <= N_train, cpp:328).
// No sort at all: the lists are already sorted by (dist, global idx), keys
// distinct, so entry c of list p lands at merged position
//   c + sum over the other lists p' of #{entries of p' before it}
// (one binary search per other list).  Pass 1 scatters the entries that land
// below k+1 into a per-query scratch row; pass 2 (a kernel boundary later:
// the row is complete and visible) votes over the first k in order.
constexpr int kMergeLdsEntries = 4096;  // union size the LDS kernel holds (80 KiB)
constexpr int kMergeRankThreads = 256;
constexpr int kVoteLdsClasses = 8192;  // sequential vote with per-class counts in LDS

struct PartLists {
  const double* dist;
  const int64_t* idx;
  const int32_t* lab;
  int64_t m, pstride;  // pstride > 0: packed parts (see merge_vote_partials_kernel)
  int w;
  __device__ __forceinline__ void at(int p, int64_t q, int c, double& v, int64_t& id,
                                     int32_t& lb) const {
    if (pstride > 0) {
      const unsigned char* pb = (const unsigned char*)dist + p * pstride;
      const int64_t o = q * w + c, mw = m * w;
      v = ((const double*)pb)[o];
      id = ((const int64_t*)(pb + 8 * mw))[o];
      lb = ((const int32_t*)(pb + 16 * mw))[o];
    } else {
      const int64_t src = ((int64_t)p * m + q) * w + c;
      v = dist[src];
      id = idx[src];
      lb = lab[src];
    }
  }
};

// scratch row of one query: K1 = k + 1 slots {dist f64 | idx i64 | label i32}
__host__ __device__ inline int64_t merge_row_bytes(int k) {
  return ((int64_t)(k + 1) * 20 + 15) / 16 * 16;
}

__global__ void __launch_bounds__(kMergeRankThreads)
merge_rank_scatter_kernel(PartLists L, int parts, int k, int64_t q0, int nch,
                          unsigned char* __restrict__ scratch) {
  const int64_t qo = blockIdx.x / nch;
  const int ch = blockIdx.x - (int)(qo * nch);
  const int64_t q = q0 + qo;
  const int e = ch * kMergeRankThreads + threadIdx.x;
  const int w = L.w;
  if (e >= parts * w) return;
  const int p = e / w, c = e - p * w;
  double v;
  int64_t id;
  int32_t lb;
  L.at(p, q, c, v, id, lb);
  if (id < 0) return;  // padding (short shard, non-finite query): not a neighbour
  int64_t rank = c;
  if (rank > k) return;
  for (int p2 = 0; p2 < parts; ++p2) {
    if (p2 == p) continue;
    int lo = 0, hi = w;  // first entry of list p2 not before (v, id)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      double v2;
      int64_t id2;
      int32_t lb2;
      L.at(p2, q, mid, v2, id2, lb2);
      // padding (+inf, -1) sorts after every neighbour
      if (id2 >= 0 && pair_less(v2, id2, v, id)) lo = mid + 1; else hi = mid;
    }
    rank += lo;
    if (rank > k) return;
  }
  unsigned char* row = scratch + qo * merge_row_bytes(k);
  const int K1 = k + 1;
  ((double*)row)[rank] = v;
  ((int64_t*)(row + 8 * K1))[rank] = id;
  ((int32_t*)(row + 16 * K1))[rank] = lb;
}

__global__ void __launch_bounds__(64)
merge_rank_vote_kernel(PartLists L, int parts, int k, int64_t q0,
                       const unsigned char* __restrict__ scratch, Sink sink) {
  __shared__ int counts[kVoteLdsClasses];
  const int64_t qo = blockIdx.x, q = q0 + qo;
  const int lane = threadIdx.x, w = L.w, K1 = k + 1;
  // valid entries: a prefix of every list
  int64_t cnt = 0;
  for (int p = lane; p < parts; p += 64) {
    int lo = 0, hi = w;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      double v;
      int64_t id;
      int32_t lb;
      L.at(p, q, mid, v, id, lb);
      if (id >= 0) lo = mid + 1; else hi = mid;
    }
    cnt += lo;
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if (cnt == 0 && k > 0) {  // no shard listed a neighbour: a non-finite query
    finish_nonfinite(qo, sink);
    return;
  }
  const int kk = (int)min<int64_t>(k, cnt);  // slots [kk, k) are empty: label -1
  const unsigned char* row = scratch + qo * merge_row_bytes(k);
  const double* rd = (const double*)row;
  const int64_t* ri = (const int64_t*)(row + 8 * K1);
  const int32_t* rl = (const int32_t*)(row + 16 * K1);
  auto slot_lab = [&](int t) { return t < kk ? rl[t] : -1; };
  int maxlab = -1;
  for (int t = lane; t < kk; t += 64) maxlab = max(maxlab, rl[t]);
  maxlab = wave_max_i(maxlab);
  int winner = -1, M = 0, m2 = -1;
  if (maxlab + 2 <= kVoteLdsClasses) {
    // cpp:324-337 as written: counts per class (slot 0: the empty label -1),
    // the first label whose count strictly exceeds the running max wins
    for (int c = lane; c < maxlab + 2; c += 64) counts[c] = 0;
    __syncthreads();
    if (lane == 0) {
      int best = 0;
      for (int t = 0; t < k; ++t) {
        const int lb = slot_lab(t);
        const int c = ++counts[lb + 1];
        if (c > best) { best = c; winner = lb; }
      }
      M = best;
    }
    __syncthreads();
    winner = __shfl(winner, 0, 64);
    M = __shfl(M, 0, 64);
    int r2 = 0;  // the runner-up count, for the tie rule
    for (int c = lane; c < maxlab + 2; c += 64)
      if (c != winner + 1) r2 = max(r2, counts[c]);
    m2 = wave_max_i(r2);
  } else {
    // (labels beyond the LDS table) the same rule in parallel: the winner is
    // the label of the first slot whose running count reaches the final max
    int bc = 0, bt = INT_MAX;
    for (int t = lane; t < k; t += 64) {
      const int lt = slot_lab(t);
      int c = 0;
      for (int s2 = 0; s2 <= t; ++s2) c += (slot_lab(s2) == lt);
      if (c > bc) { bc = c; bt = t; }
    }
    M = wave_max_i(bc);
    const int tmin = wave_min_i(bc == M ? bt : INT_MAX);
    winner = k > 0 ? slot_lab(tmin) : -1;
  }
  int tie = 0;
  for (int t = lane; t + 1 < kk; t += 64)
    if (rd[t] == rd[t + 1]) tie |= rl[t] != rl[t + 1] ? 4 : 8;
  tie = wave_or_i(tie);
  const bool bnd = k > 0 && k < cnt && rd[k - 1] == rd[k];
  const bool pend = kk == k && tie_order_matters(slot_lab, [&](int t) { return rd[t]; }, k, winner,
                                                 M, tie, bnd, sink.tie_mode, m2);
  if (lane == 0) {
    sink.labels[qo] = winner;
    if (sink.flags) sink.flags[qo] = tie | (bnd ? 2 : 0) | (pend ? kFlagTiePending : 0);
    if (pend && sink.tie_q) sink.tie_q[atomicAdd(sink.tie_cnt, 1)] = (int)qo;
  }
  for (int t = lane; t < k; t += 64) {
    if (sink.idx) sink.idx[qo * k + t] = t < kk ? ri[t] : -1;
    if (sink.dist) sink.dist[qo * k + t] = t < kk ? rd[t] : KNN_INF_D;
  }
}

int64_t merge_scratch_bytes(int parts, int w, int k, int64_t mq) {
  if ((int64_t)parts * w <= kMergeLdsEntries) return 0;  // the LDS kernel needs none
  return mq * merge_row_bytes(k);
}

void launch_merge_vote_partials(const double* dist, const int64_t* idx, const int32_t* lab,
                                int parts, int64_t m, int w, int k, int32_t* out_lab,
                                int64_t* out_idx, double* out_dist, int32_t* out_flags,
                                hipStream_t s, int64_t q0, int64_t mq, int64_t pstride,
                                void* scratch, const MergeTies& mt) {
  if (mq < 0) mq = m - q0;
  if (mq <= 0) return;
  Sink sink{};
  sink.mode = MODE_SINGLE;
  sink.k = k;
  sink.labels = out_lab;
  sink.idx = out_idx;
  sink.dist = out_dist;
  sink.flags = out_flags;
  sink.tie_mode = mt.mode;
  sink.tie_q = mt.q;
  sink.tie_cnt = mt.cnt;
  if ((int64_t)parts * w > kMergeLdsEntries) {
    const PartLists L{dist, idx, lab, m, pstride, w};
    const int nch = (parts * w + kMergeRankThreads - 1) / kMergeRankThreads;
    hipLaunchKernelGGL(merge_rank_scatter_kernel, dim3((unsigned)(mq * nch)),
                       dim3(kMergeRankThreads), 0, s, L, parts, k, q0, nch,
                       (unsigned char*)scratch);
    hipLaunchKernelGGL(merge_rank_vote_kernel, dim3((unsigned)mq), dim3(64), 0, s, L, parts, k,
                       q0, (const unsigned char*)scratch, sink);
    return;
  }
  int P2 = 1;
  while (P2 < parts * w) P2 <<= 1;
  const size_t lds = (size_t)P2 * (8 + 8 + 4);
  hipLaunchKernelGGL(merge_vote_partials_kernel, dim3((unsigned)mq), dim3(64), lds, s, dist, idx,
                     lab, parts, m, w, k, P2, q0, pstride, sink);
}

}  // namespace knnk
