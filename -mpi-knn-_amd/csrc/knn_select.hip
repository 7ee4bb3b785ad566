// knn_select.hip -- merge / exact fp64 re-rank / certification / vote,
// the exact rescan path and the train-sharded k-way merge (gfx950).
#include "knn_device.h"

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
      const double x = qrow[c] - t.mu[c];  // centred like the candidate operands
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
