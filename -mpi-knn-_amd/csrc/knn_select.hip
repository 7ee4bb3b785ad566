// knn_select.hip -- merge / exact fp64 re-rank / certification / vote,
// the exact rescan path and the train-sharded k-way merge (gfx950).
#include "knn_device.h"

#include <algorithm>

namespace knnk {

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
// reference's operation order: rows are read coalesced (16 lanes per 128-B
// row piece) into an LDS tile of squared (L1: absolute) differences, then
// thread c adds its candidate's terms in dimension order -- bit-exact with
// cpp:33-50 / cpp:51-67 (sequential, no FMA; sqrt correctly rounded).
// Pads [cn, C2) with (+inf, INT_MAX) and sorts (dist, idx) ascending.
// All NT threads; tb holds NT x 17 doubles.
template <int METRIC, int NT>
__device__ void exact_sorted(const TrainDev& t, const double* qv, int* di, double* dk, double* tb,
                             int cn, int C2, int tid) {
  const int d = t.d;
  for (int b0 = 0; b0 < cn; b0 += NT) {
    const int nb = min(NT, cn - b0);
    double r = 0.0;
    for (int c0 = 0; c0 < d; c0 += 16) {
      const int nd = min(16, d - c0);
      for (int e = tid; e < nb * 16; e += NT) {
        const int c = e >> 4, j = e & 15;
        double val = 0.0;
        if (j < nd) {
          const double x = t.X64[(int64_t)di[b0 + c] * d + c0 + j];
          const double tq = qv[c0 + j] - x;
          val = METRIC == 0 ? tq * tq : __builtin_fabs(tq);
        }
        tb[c * 17 + j] = val;
      }
      __syncthreads();
      if (tid < nb) {
        const double* row = tb + tid * 17;
        if (nd == 16) {
#pragma unroll
          for (int j = 0; j < 16; ++j) r = r + row[j];
        } else {
          for (int j = 0; j < nd; ++j) r = r + row[j];
        }
      }
      __syncthreads();
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

template <int METRIC, int NT, int EPL>
__global__ void __launch_bounds__(NT)
merge_rerank_kernel(const float* __restrict__ cv, const int* __restrict__ ci, int U, int R,
                    TrainDev t, const double* __restrict__ Q64, int W, int Cmax, int C2,
                    double f_err, ProxyScale ps, const uint32_t* __restrict__ gthr, Sink sink,
                    int* __restrict__ rescan_q, double* __restrict__ rescan_tau,
                    int* __restrict__ rescan_cnt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int s_cn, s_cert;
  __shared__ double s_lb, s_qa, s_e;
  const int d = t.d;
  // the query row is staged in LDS up to kMergeLdsDim dims, else read in place
  const bool q_in_lds = d <= kMergeLdsDim;
  double* dk = (double*)smem + (q_in_lds ? d : 0);
  double* tb = dk + C2;
  int* di = (int*)(tb + NT * 17);
  int* ls = di + C2;
  const int64_t q = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;

  const double* qrow = Q64 + q * d;
  const double* qv = q_in_lds ? (const double*)smem : qrow;
  if (q_in_lds)
    for (int c = tid; c < d; c += NT) ((double*)smem)[c] = qrow[c];
  __syncthreads();

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
    if (METRIC == 0 && ps.qh) {
      // fp16 operands: f_err covers the accumulation only; add the measured
      // representation error (q' = q - mu, x' = x - mu, dq / dx the operand
      // errors in unscaled units):  2 |q'.dx + dq.x' + dq.dx| <=
      // 2 (|q'| dxmax + |dq| (xmax + dxmax)), plus the fl32 seed's own
      // rounding (3u ||x'||^2, u = 2^-24)
      const unsigned short* qh = ps.qh + q * (int64_t)ps.qh_stride;
      const double qs = -__builtin_ldexp(0.5, -t.jx);  // operand = -2 * 2^jx q'
      double dq2 = 0.0;
      for (int c = lane; c < d; c += 64) {
        const double e = (double)__builtin_bit_cast(_Float16, qh[c]) * qs - (qv[c] - t.mu[c]);
        dq2 += e * e;
      }
      const double qn = __builtin_sqrt(qa), xm = __builtin_sqrt(t.x2max);
      const double dq = __builtin_sqrt(wave_sum_d(dq2) * (1.0 + 1e-12)) * (1.0 + 1e-12) +
                        0x1p-50 * qn;
      E = f_err * (t.x2max + 2.0 * (qn + dq) * (xm + t.dxmax) * 1.001) + 3.01 * 0x1p-24 * t.x2max +
          2.0 * (qn * t.dxmax + dq * (xm + t.dxmax)) * 1.001 + 1e-300;
    }
    // proxies are in scaled units (operands 2^jx (x - mu), knn_prep.hip):
    // unscale exactly; operand values outside the format's normal range add
    // absolute error terms (ue per element, up per product, scaled units)
    const double pinv = __builtin_ldexp(1.0, METRIC == 0 ? -2 * t.jx : -t.jx);
    const double sinv = __builtin_ldexp(1.0, -t.jx);
    q1 = wave_sum_d(q1) * (1.0 + 1e-12);
    if (METRIC == 0) E += ps.ue * 1.001 * (2.0 * q1 + t.x1max) * sinv + t.DP * ps.up * pinv;
    else E += 2.0 * ps.ue * 1.001 * t.DP * sinv;
    const bool void_q = ps.valid && !(ps.valid[q] > 0.0f);
    // union in registers; min over full lists of their R-th (worst kept) entry
    const float* lv = cv + q * U;
    const int* li = ci + q * U;
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
        if (x % R == R - 1) mlr = fminf(mlr, v[e]);
      }
      nv += __popcll(__ballot(v[e] < KNN_INF_F));
    }
    mlr = wave_min(mlr);
    double tsel = KNN_INF_D;  // select proxies <= tsel
    if (nv > W) {
      uint32_t pre = 0;  // radix select: key of the W-th smallest proxy
      for (int b = 31; b >= 0; --b) {
        const uint32_t T = pre | ((1u << b) - 1u);
        int cnt = 0;
#pragma unroll
        for (int e = 0; e < EPL; ++e) cnt += __popcll(__ballot(f2key(v[e]) <= T));
        if (cnt < W) pre |= 1u << b;
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
    // the candidate kernel also filtered with the query's global threshold
    // (cand_kernel): rows it dropped have proxy >= its final value
    float tq = KNN_INF_F;
    if (gthr) {
      const uint32_t* g = gthr + q * 4;
      tq = key2f(max(max(g[0], g[1]), max(g[2], g[3])));
    }
    if (lane == 0) {
      s_cn = void_q ? Cmax + 1 : cn;  // void proxies: exact rescan below
      s_lb = (double)fminf(fminf(lbx, mlr), tq) * pinv;
      s_qa = qa;
      s_e = E;
    }
  }
  __syncthreads();
  const int cn = s_cn;
  if (cn > Cmax) {  // void proxies (the window overflow is handled above): exact rescan
    if (tid == 0) {
      const int f = atomicAdd(rescan_cnt, 1);
      rescan_q[f] = (int)q;
      rescan_tau[f] = KNN_INF_D;
    }
    return;
  }

  exact_sorted<METRIC, NT>(t, qv, di, dk, tb, cn, C2, tid);

  // certification: every row not re-ranked has proxy >= LB, hence exact
  // distance >= the bound below (rigorous error bound E)
  if (tid == 0) {
    const double LB = s_lb;
    bool cert;
    if (!(LB < KNN_INF_D)) {
      cert = true;  // nothing was left out: every row was re-ranked exactly
    } else if (cn < W) {
      cert = false;
    } else {
      const double dw = dk[W - 1], qa = s_qa, E = s_e;
      if (METRIC == 0) {
        const double bound = (LB + qa * (1.0 - 2e-12) - E) * (1.0 - 1e-12);
        cert = bound > dw * dw * (1.0 + 1e-12);
      } else {
        const double bound = (LB - E) * (1.0 - 1e-12);
        cert = bound > dw * (1.0 + 1e-12);
      }
    }
    s_cert = cert;
    if (!cert) {
      // the W-th exact distance among the re-ranked rows bounds the true
      // W-th from above: the fast rescan keeps every row that can reach it
      const int f = atomicAdd(rescan_cnt, 1);
      rescan_q[f] = (int)q;
      rescan_tau[f] = cn >= W ? dk[W - 1] : KNN_INF_D;
    }
  }
  __syncthreads();
  if (!s_cert) return;

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

template <int METRIC, int NT, int EPL>
static void launch_mr(const float* cv, const int* ci, int U, int R, const TrainDev& t,
                      const double* Q64, int64_t m, int W, int Cmax, int C2, double f_err,
                      ProxyScale ps, const uint32_t* gthr, const Sink& sink, int* rescan_q,
                      double* rescan_tau, int* rescan_cnt, hipStream_t s) {
  const size_t lds = (size_t)(t.d <= kMergeLdsDim ? t.d : 0) * 8 + (size_t)C2 * 8 +
                     (size_t)NT * 17 * 8 + (size_t)C2 * 8;
  hipLaunchKernelGGL((merge_rerank_kernel<METRIC, NT, EPL>), dim3((unsigned)m), dim3(NT), lds, s,
                     cv, ci, U, R, t, Q64, W, Cmax, C2, f_err, ps, gthr, sink, rescan_q, rescan_tau,
                     rescan_cnt);
}

void launch_merge_rerank(int metric, const float* cv, const int* ci, int NL, int R,
                         const TrainDev& t, const double* Q64, int64_t m, int W, int C,
                         double f_err, ProxyScale ps, const uint32_t* gthr, const Sink& sink,
                         int* rescan_q, double* rescan_tau, int* rescan_cnt, hipStream_t s) {
  if (m <= 0) return;
  const int U = NL * R;  // <= 2 * 64 * 16 (choose_geometry bounds S and R)
  int C2 = 1;
  while (C2 < C) C2 <<= 1;
  const bool big = C2 > 64, wide = U > 1024;
#define KNN_MR(M_, NT_, EPL_) \
  launch_mr<M_, NT_, EPL_>(cv, ci, U, R, t, Q64, m, W, C, C2, f_err, ps, gthr, sink, rescan_q, \
                           rescan_tau, rescan_cnt, s)
  if (metric == 0) {
    if (big) { if (wide) KNN_MR(0, 256, 32); else KNN_MR(0, 256, 16); }
    else { if (wide) KNN_MR(0, 64, 32); else KNN_MR(0, 64, 16); }
  } else {
    if (big) { if (wide) KNN_MR(1, 256, 32); else KNN_MR(1, 256, 16); }
    else { if (wide) KNN_MR(1, 64, 32); else KNN_MR(1, 64, 16); }
  }
#undef KNN_MR
}

// ------------------------------------------------- fast rescan (filtered)
// Queries whose candidate set was not certified (a list overflowed near the
// top, heavy ties).  tau = the W-th exact distance among the query's
// re-ranked rows, >= the true W-th.  rescan_filter streams the fp32 train
// copy once per 4 or 16 such queries (lane = train row, queries broadcast
// from LDS) and appends every row whose centred fp32 proxy --
// an fmaf chain with the candidate pass's certified error bound -- is within
// reach of tau; the appended set therefore holds every row with exact
// distance <= tau, i.e. the exact top-W with all its ties.  rescan_finish
// re-ranks it exactly.  Unknown tau or more than kRescanCap rows: the full
// exact scan below.

// Block = NWB waves, wave w owns the 64 consecutive train rows starting at
// blockIdx.x*64*NWB + 64w (lane = row).  The wave copies its rows (the
// padded fp32 X32 layout, odd 16-B stride -> conflict-free ds_read_b128) into
// LDS by LDS-DMA, then runs kFiltQ accumulators per lane against the block's
// queries, read as LDS broadcasts.
// One wave per failed query: the centred fp32 query row (x -2 for L2, the
// candidate pass's operand) and the proxy threshold every row with exact
// distance <= tau passes (fp32 fmaf-chain error bound f_err of t.DP).
template <int METRIC>
__global__ void __launch_bounds__(64)
rescan_prep_kernel(TrainDev t, const double* __restrict__ Q64, const int* __restrict__ rescan_q,
                   const double* __restrict__ tau, int f0, double f_err, float* __restrict__ qf,
                   float* __restrict__ thr) {
  const int s = blockIdx.x, lane = threadIdx.x, d = t.d, DP = t.DP;
  const double* qr = Q64 + (int64_t)rescan_q[f0 + s] * d;
  double qa = 0.0, q1 = 0.0;
  for (int i = lane; i < DP; i += 64) {
    float v = 0.0f;
    if (i < d) {
      const double x = qr[i] - t.mu[i];
      qa += METRIC == 0 ? x * x : __builtin_fabs(x);
      q1 += __builtin_fabs(x);
      v = (float)__builtin_ldexp(x * (METRIC == 0 ? -2.0 : 1.0), t.jx);  // X32's scale
    }
    qf[(int64_t)s * DP + i] = v;
  }
  qa = wave_sum_d(qa) * (1.0 + 1e-12);
  q1 = wave_sum_d(q1) * (1.0 + 1e-12);
  if (lane == 0) {
    const double tq = tau[f0 + s];
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
    thr[s] = tq < KNN_INF_D ? tf : -KNN_INF_F;  // unknown tau: nothing passes, full scan
  }
}

template <int METRIC, int kFiltQ>  // kFiltQ: failed queries per block (LDS broadcasts)
__global__ void __launch_bounds__(256)
rescan_filter_kernel(TrainDev t, const float* __restrict__ qf, const float* __restrict__ thr,
                     int nf, int* __restrict__ cnt, int* __restrict__ buf) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  const int DP = t.DP, RSF = DP + 4;
  const int NWB = blockDim.x >> 6;
  float* qs = fsm;                          // [kFiltQ][DP] centred queries (x -2 for L2)
  float* thr_s = qs + kFiltQ * DP;          // [kFiltQ] proxy thresholds
  float* rows = thr_s + kFiltQ;             // [NWB][64][RSF]
  __shared__ int s_dummy;
  (void)s_dummy;
  const int g0 = blockIdx.y * kFiltQ;
  const int nfg = min(kFiltQ, nf - g0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t row0 = ((int64_t)blockIdx.x * NWB + wv) * 64;
  const bool active = row0 < t.n_pad;

  // this wave's 64 rows -> LDS (X32 carries 1 KiB of slack past the last row)
  float* my_rows = rows + (size_t)wv * 64 * RSF;
  if (active) {
    const int bytes = 64 * RSF * 4;
    const char* src = (const char*)(t.X32 + row0 * RSF) + lane * 16;
    const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)my_rows;
    for (int p = 0; p * 1024 < bytes; ++p) glds16(src + p * 1024, dst + p * 1024);
  }
  for (int e = tid; e < kFiltQ * DP; e += blockDim.x) {
    const int qi = e / DP;
    qs[e] = qi < nfg ? qf[(int64_t)g0 * DP + e] : 0.0f;
  }
  if (tid < kFiltQ) thr_s[tid] = tid < nfg ? thr[g0 + tid] : -KNN_INF_F;  // absent: no row passes
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (!active) return;

  const float* xr = my_rows + lane * RSF;
  const float seed = xr[METRIC == 0 ? DP : DP + 1];  // +inf on pad rows: never passes
  float acc[kFiltQ];
#pragma unroll
  for (int qi = 0; qi < kFiltQ; ++qi) acc[qi] = seed;
  for (int c = 0; c < DP / 4; ++c) {
    const float4 x4 = *(const float4*)(xr + 4 * c);
#pragma unroll
    for (int qi = 0; qi < kFiltQ; ++qi) {
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
  for (int qi = 0; qi < kFiltQ; ++qi) {
    if (acc[qi] <= thr_s[qi]) {
      const int pos = atomicAdd(&cnt[g0 + qi], 1);
      if (pos < kRescanCap) buf[(int64_t)(g0 + qi) * kRescanCap + pos] = (int)(row0 + lane);
    }
  }
}

// One block per fast-rescanned query: exact re-rank of its appended rows.
// Dynamic LDS: qv[d] | dk[kRescanCap] | tb[NT][17] | di[kRescanCap] | ls[kRescanCap].
template <int METRIC, int NT>
__global__ void __launch_bounds__(NT)
rescan_finish_fast_kernel(TrainDev t, const double* __restrict__ Q64,
                          const int* __restrict__ rescan_q, const double* __restrict__ tau, int f0,
                          int W, const int* __restrict__ cnt, const int* __restrict__ buf,
                          Sink sink, int* __restrict__ slow_q, int* __restrict__ slow_cnt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int d = t.d;
  const bool q_in_lds = d <= 1024;  // keeps the block's LDS under 64 KiB
  double* dk = (double*)smem + (q_in_lds ? d : 0);
  double* tb = dk + kRescanCap;
  int* di = (int*)(tb + NT * 17);
  int* ls = di + kRescanCap;
  const int s = blockIdx.x, tid = threadIdx.x;
  const int64_t q = rescan_q[f0 + s];
  const int c = cnt[s];
  const int need_rows = (int)min((int64_t)W, t.n);
  if (!(tau[f0 + s] < KNN_INF_D) || c > kRescanCap || c < need_rows) {
    if (tid == 0) slow_q[atomicAdd(slow_cnt, 1)] = (int)q;
    return;
  }
  const double* qrow = Q64 + q * d;
  const double* qv = q_in_lds ? (const double*)smem : qrow;
  if (q_in_lds)
    for (int i = tid; i < d; i += NT) ((double*)smem)[i] = qrow[i];
  for (int i = tid; i < c; i += NT) di[i] = buf[(int64_t)s * kRescanCap + i];
  __syncthreads();
  int C2 = 1;
  while (C2 < c) C2 <<= 1;
  exact_sorted<METRIC, NT>(t, qv, di, dk, tb, c, C2, tid);
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

void launch_rescan_fast(int metric, const TrainDev& t, const double* Q64, const int* rescan_q,
                        const double* tau, int f0, int nf, int W, double f_err, float* qf,
                        float* thr, int* cnt, int* buf, const Sink& sink, int* slow_q,
                        int* slow_cnt, hipStream_t s) {
  if (nf <= 0) return;
  if (metric == 0)
    hipLaunchKernelGGL(rescan_prep_kernel<0>, dim3((unsigned)nf), dim3(64), 0, s, t, Q64,
                       rescan_q, tau, f0, f_err, qf, thr);
  else
    hipLaunchKernelGGL(rescan_prep_kernel<1>, dim3((unsigned)nf), dim3(64), 0, s, t, Q64,
                       rescan_q, tau, f0, f_err, qf, thr);
  // queries per block: 4 for a handful of failed queries (list overflows),
  // else 16; waves per block: as many 64-row tiles as fit in ~150 KiB
  const int fq = nf <= 4 ? 4 : 16;
  const size_t tile = (size_t)64 * (t.DP + 4) * 4, qbytes = (size_t)fq * (t.DP + 1) * 4;
  const int nwb = (int)std::max<size_t>(1, std::min<size_t>(4, (150 * 1024 - qbytes) / tile));
  const int64_t rpb = 64 * nwb;
  const dim3 fg((unsigned)((t.n_pad + rpb - 1) / rpb), (unsigned)((nf + fq - 1) / fq));
  const size_t flds = qbytes + nwb * tile;
#define KNN_FILT(M_, Q_)                                                                      \
  hipLaunchKernelGGL((rescan_filter_kernel<M_, Q_>), fg, dim3(64 * nwb), flds, s, t, qf, thr, nf, \
                     cnt, buf)
  if (metric == 0) {
    if (fq == 4) KNN_FILT(0, 4); else KNN_FILT(0, 16);
  } else {
    if (fq == 4) KNN_FILT(1, 4); else KNN_FILT(1, 16);
  }
#undef KNN_FILT
  const size_t lds = (size_t)(t.d <= 1024 ? t.d : 0) * 8 + (size_t)kRescanCap * 8 +
                     (size_t)256 * 17 * 8 + (size_t)kRescanCap * 8;
  if (metric == 0)
    hipLaunchKernelGGL((rescan_finish_fast_kernel<0, 256>), dim3((unsigned)nf), dim3(256), lds, s,
                       t, Q64, rescan_q, tau, f0, W, cnt, buf, sink, slow_q, slow_cnt);
  else
    hipLaunchKernelGGL((rescan_finish_fast_kernel<1, 256>), dim3((unsigned)nf), dim3(256), lds, s,
                       t, Q64, rescan_q, tau, f0, W, cnt, buf, sink, slow_q, slow_cnt);
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
