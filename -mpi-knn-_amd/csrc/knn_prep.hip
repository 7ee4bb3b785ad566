// knn_prep.hip -- operand preparation kernels (gfx950): fp64 rows -> fp32 /
// bf16 hi-lo MFMA operands, seeds and norm statistics.
#include "knn_device.h"

namespace knnk {

// ------------------------------------------------------------------ prep
// Every candidate-pass operand is centred on the train mean mu: distances
// are translation invariant (||q - x|| = ||(q - mu) - (x - mu)||), while the
// candidate pass's rounding error scales with ||x||^2 and ||q||.||x|| -- on
// min-max normalised data centring shrinks those ~20x, which is what lets
// the certification pass at d = 960.  mu only shifts the
// operands; the exact re-rank always uses the caller's fp64 rows.

// Column means, deterministic: block b sums rows [b*rpb, (b+1)*rpb) of every
// dim in row order (coalesced across threads), then one pass adds the
// per-block sums in block order.
__global__ void __launch_bounds__(256)
col_sum_kernel(const double* __restrict__ X64, int64_t n, int d, int64_t rpb,
               double* __restrict__ partial) {
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < n ? r0 + rpb : n;
  for (int c = threadIdx.x; c < d; c += 256) {
    double s = 0.0;
    for (int64_t r = r0; r < r1; ++r) s += X64[r * d + c];
    partial[(int64_t)blockIdx.x * d + c] = s;
  }
}

__global__ void __launch_bounds__(256)
col_mean_kernel(const double* __restrict__ partial, int nb, int d, int64_t n,
                double* __restrict__ mu) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= d) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += partial[(int64_t)b * d + c];
  mu[c] = s / (double)n;
}

int col_mean_blocks(int64_t n) {
  const int64_t nb = (n + 1023) / 1024;
  return (int)(nb < 2048 ? (nb > 0 ? nb : 1) : 2048);
}

void launch_col_mean(const double* X64, int64_t n, int d, double* partial, double* mu,
                     hipStream_t s) {
  const int nb = col_mean_blocks(n);
  const int64_t rpb = (n + nb - 1) / nb;
  hipLaunchKernelGGL(col_sum_kernel, dim3(nb), dim3(256), 0, s, X64, n, d, rpb, partial);
  hipLaunchKernelGGL(col_mean_kernel, dim3((d + 255) / 256), dim3(256), 0, s, partial, nb, d, n,
                     mu);
}

// max |x_i - mu_i| over the train set (fp64, non-negative -> ordered as
// u64 bits): fixes the operand scale 2^jx before any rounding to fp32.
// Also counts the non-finite train values (exponent bits all ones: a bit
// test, this file is built with -fno-honor-nans) into nonfinite[0] --
// set_train rejects such a train set (nonfinite_bits: knn_device.h).

__global__ void __launch_bounds__(256)
absmax_kernel(const double* __restrict__ X64, const double* __restrict__ mu, int64_t n, int d,
              unsigned long long* __restrict__ out, unsigned long long* __restrict__ nonfinite) {
  double m = 0.0;
  int bad = 0;
  const int64_t total = n * d;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const double x = X64[e];
    bad += nonfinite_bits(x);
    m = fmax(m, __builtin_fabs(x - mu[e % d]));
  }
  m = wave_max_d(m);
  bad = wave_sum_i(bad);
  if ((threadIdx.x & 63) == 0) {
    atomicMax(out, (unsigned long long)__double_as_longlong(m));
    if (bad) atomicAdd(nonfinite, (unsigned long long)bad);
  }
}

void launch_absmax(const double* X64, const double* mu, int64_t n, int d, unsigned long long* out,
                   unsigned long long* nonfinite, hipStream_t s) {
  int64_t blocks = (n * d + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(absmax_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X64, mu, n, d, out,
                     nonfinite);
}

// Train labels outside [0, class_cnt) (the reference indexes label_cnt[label]
// unchecked, cpp:330): counted into bad[0], set_train rejects them.
__global__ void __launch_bounds__(256)
label_check_kernel(const int32_t* __restrict__ lab, int64_t n, int class_cnt,
                   unsigned long long* __restrict__ bad) {
  int b = 0;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
    b += (lab[e] < 0 || lab[e] >= class_cnt);
  b = wave_sum_i(b);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(bad, (unsigned long long)b);
}

void launch_label_check(const int32_t* lab, int64_t n, int class_cnt, unsigned long long* bad,
                        hipStream_t s) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(label_check_kernel, dim3((unsigned)blocks), dim3(256), 0, s, lab, n, class_cnt,
                     bad);
}

// Operand scale.  Every candidate-pass operand is 2^jx (x - mu), jx putting
// max |x_i - mu_i| * 2^jx in [2^8, 2^9) (exact power-of-two scaling): the
// reduced-precision arithmetic then runs in the same range whatever the
// data's magnitude, and proxies are 2^(2 jx) (L2) / 2^jx (L1) times the
// unscaled ones (the merge unscales).  Values far below the largest may
// still leave the normal range of fp32 / fp16: the merge's absolute error
// terms cover that.

// One wave per train row: fp64 2^jx (x - mu) -> fp32 (zero padded to DP),
// fl32(||x32||^2) seeds for the L2 accumulator, 0 seeds for L1, +inf on pad
// rows; running max of the unscaled ||x - mu||_2^2 and ||x - mu||_1 (fp64,
// non-negative -> ordered as u64 bits).
__global__ void __launch_bounds__(256)
prep_train_kernel(const double* __restrict__ X64, const double* __restrict__ mu, int64_t n, int d,
                  int DP, int64_t n_pad, int jx, float* __restrict__ X32, float* __restrict__ xl2,
                  float* __restrict__ xl1, unsigned long long* __restrict__ stats,
                  const int* __restrict__ perm) {
  const int RSF = DP + 4;  // padded row: [x32 (DP) | ||x32||^2, l1 seed, 0, 0]
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  double m2 = 0.0, m1 = 0.0;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n_pad; row += wstride) {
    double s32 = 0.0, s64 = 0.0, a64 = 0.0;
    const int64_t src = src_row(perm, row, n);
    for (int c = lane; c < DP; c += 64) {
      float v = 0.0f;
      if (row < n && c < d) {
        const double x = X64[src * d + c] - mu[c];
        v = (float)__builtin_ldexp(x, jx);
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

void launch_prep_train(const double* X64, const double* mu, int64_t n, int d, int DP,
                       int64_t n_pad, int jx, float* X32, float* xl2, float* xl1,
                       unsigned long long* stats, hipStream_t s, const int* perm) {
  int64_t blocks = (n_pad + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(prep_train_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X64, mu, n, d,
                     DP, n_pad, jx, X32, xl2, xl1, stats, perm);
}

// Per query: valid[row] = 1 when every |scale * 2^jx (q_i - mu_i)| stays below
// `limit` (the operand format's safe range), else 0: the query's proxies are
// then void and the merge sends it to the exact rescan (pad rows: 1); -1
// when a coordinate is NaN or infinite (bit test): no neighbours reported.
__global__ void __launch_bounds__(256)
query_check_kernel(const double* __restrict__ Q64, const double* __restrict__ mu, int64_t m, int d,
                   int64_t m_pad, double scale, int jx, double limit, float* __restrict__ valid) {
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < m_pad; row += wstride) {
    bool ok = true, fin = true;
    if (row < m)
      for (int c = lane; c < d; c += 64) {
        const double x = Q64[row * d + c];
        fin = fin && !nonfinite_bits(x);
        ok = ok && __builtin_fabs(__builtin_ldexp(scale * (x - mu[c]), jx)) < limit;
      }
    ok = __ballot(!ok) == 0;
    fin = __ballot(!fin) == 0;
    if (lane == 0) valid[row] = !fin ? -1.0f : (ok ? 1.0f : 0.0f);
  }
}

void launch_query_check(const double* Q64, const double* mu, int64_t m, int d, int64_t m_pad,
                        double scale, int jx, double limit, float* valid, hipStream_t s) {
  int64_t blocks = (m_pad + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(query_check_kernel, dim3((unsigned)blocks), dim3(256), 0, s, Q64, mu, m, d,
                     m_pad, scale, jx, limit, valid);
}

// scale * 2^jx (q - mu) -> fp32 rows of DP (zero padded)
__global__ void __launch_bounds__(256)
prep_queries_kernel(const double* __restrict__ Q64, const double* __restrict__ mu, int64_t m,
                    int d, int DP, int64_t m_pad, double scale, int jx, float* __restrict__ Q32) {
  const int64_t total = m_pad * DP;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int64_t row = e / DP;
    const int c = (int)(e - row * DP);
    float v = 0.0f;
    if (row < m && c < d) v = (float)__builtin_ldexp(scale * (Q64[row * d + c] - mu[c]), jx);
    Q32[e] = v;
  }
}

void launch_prep_queries(const double* Q64, const double* mu, int64_t m, int d, int DP,
                         int64_t m_pad, double scale, int jx, float* Q32, hipStream_t s) {
  int64_t blocks = (m_pad * DP + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(prep_queries_kernel, dim3((unsigned)blocks), dim3(256), 0, s, Q64, mu, m, d,
                     DP, m_pad, scale, jx, Q32);
}

__global__ void __launch_bounds__(256)
prep_split_kernel(const double* __restrict__ X64, const double* __restrict__ mu, int64_t n, int d,
                  int DP, int64_t n_pad, double scale, unsigned short* __restrict__ out, int row_shorts,
                  const float* __restrict__ xl2, const float* __restrict__ xl1,
                  const int* __restrict__ perm) {
  // row r of `out` (row_shorts 16-bit words) = [hi(DP) | lo(DP) | seeds...]
  const int64_t total = n_pad * DP;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int64_t row = e / DP;
    const int c = (int)(e - row * DP);
    unsigned short hi = 0, lo = 0;
    if (row < n && c < d) split_bf16(scale * (X64[src_row(perm, row, n) * d + c] - mu[c]), hi, lo);
    out[row * row_shorts + c] = hi;
    out[row * row_shorts + DP + c] = lo;
    if (xl2 && c < 4) {  // train rows: the padded row's seed floats
      float* seed = (float*)(out + row * row_shorts + 2 * DP);
      seed[c] = c == 0 ? xl2[row] : (c == 1 ? xl1[row] : 0.0f);
    }
  }
}

void launch_prep_split(const double* X64, const double* mu, int64_t n, int d, int DP,
                       int64_t n_pad, double scale, unsigned short* out, int row_shorts,
                       const float* xl2, const float* xl1, hipStream_t s, const int* perm) {
  int64_t blocks = (n_pad * DP + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(prep_split_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X64, mu, n, d, DP,
                     n_pad, scale, out, row_shorts, xl2, xl1, perm);
}

// ---------------------------------- fp16 images (kernel metric 4, d <= 256)
// Train rows: [fp16(2^jx (x - mu)) (DP halves) | seeds (4 floats)], the seed
// fl32(||x32||^2) of the (equally scaled) fp32 copy; +inf on pad rows.  With
// max |x - mu| * 2^jx < 2^9 nothing overflows fp16; values below its normal
// range carry an absolute error the merge's bound includes.
__global__ void __launch_bounds__(256)
prep_half_train_kernel(const double* __restrict__ X64, const double* __restrict__ mu, int64_t n,
                       int d, int DP, int64_t n_pad, int jx, unsigned short* __restrict__ out,
                       const float* __restrict__ xl2, unsigned long long* __restrict__ dx2max,
                       int swz, const int* __restrict__ perm) {
  // one wave per row; the row's representation error ||h / 2^jx - (x - mu)||^2
  // is measured in fp64 (h / 2^jx - x is exact: Sterbenz, or h = 0)
  const int row_shorts = DP + 8;
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  const double sinv = __builtin_ldexp(1.0, -jx);
  double m = 0.0;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n_pad; row += wstride) {
    double e2 = 0.0;
    const int cx = swz ? xh_swz((int)(row & 15)) << 3 : 0;
    const int64_t src = src_row(perm, row, n);
    for (int c = lane; c < DP; c += 64) {
      _Float16 h = (_Float16)0.0f;
      if (row < n && c < d) {
        const double x = X64[src * d + c] - mu[c];
        h = f16_operand(x, jx);
        const double e = (double)h * sinv - x;
        e2 += e * e;
      }
      // 16-B chunk c >> 3 stored at (c >> 3) ^ xh_swz(row) (knn_device.h)
      out[row * row_shorts + (c ^ cx)] = __builtin_bit_cast(unsigned short, h);
    }
    if (lane < 4) {
      // slot 0: the row's own seed; the pad of row 4g also carries the seeds
      // of rows 4g+1 .. 4g+3 (one float4 read per 4 rows; n_pad % 4 == 0)
      float* seed = (float*)(out + row * row_shorts + DP);
      seed[lane] = (lane == 0 || (row & 3) == 0) ? xl2[row + lane] : 0.0f;
    }
    m = fmax(m, wave_sum_d(e2));
  }
  if (lane == 0) atomicMax(dx2max, (unsigned long long)__double_as_longlong(m * (1.0 + 1e-12)));
}

void launch_prep_half_train(const double* X64, const double* mu, int64_t n, int d, int DP,
                            int64_t n_pad, int jx, unsigned short* out, const float* xl2,
                            unsigned long long* dx2max, int swz, hipStream_t s, const int* perm) {
  int64_t blocks = (n_pad + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(prep_half_train_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X64, mu, n, d,
                     DP, n_pad, jx, out, xl2, dx2max, swz, perm);
}

__global__ void round_mu_kernel(double* mu, int d, int g) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= d) return;
  // |mu| 2^g >= 2^52: already a multiple of 2^-g (and no overflow)
  const double y = __builtin_ldexp(mu[c], g);
  if (__builtin_fabs(y) < 0x1p52) mu[c] = __builtin_ldexp(__builtin_rint(y), -g);
}
void launch_round_mu(double* mu, int d, int g, hipStream_t s) {
  hipLaunchKernelGGL(round_mu_kernel, dim3((d + 255) / 256), dim3(256), 0, s, mu, d, g);
}

// Query rows: fp16(-2 * 2^jx (q - mu)) (DP halves), the train set's scale;
// a query launch_query_check marked invalid (valid[row] = 0: beyond the
// fp16 range) gets zero operands, i.e. finite proxies the merge ignores.
__global__ void __launch_bounds__(256)
prep_half_queries_kernel(const double* __restrict__ Q64, const double* __restrict__ mu, int64_t m,
                         int d, int DP, int64_t m_pad, int jx, unsigned short* __restrict__ out,
                         const float* __restrict__ valid, const int* __restrict__ qperm) {
  const int64_t total = m_pad * DP;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int64_t row = e / DP;
    const int c = (int)(e - row * DP);
    _Float16 h = (_Float16)0.0f;
    const int64_t q = src_row(qperm, row, m);
    if (row < m && c < d && valid[q] > 0.0f)
      h = f16_operand(-2.0 * (Q64[q * d + c] - mu[c]), jx);
    out[e] = __builtin_bit_cast(unsigned short, h);
  }
}

void launch_prep_half_queries(const double* Q64, const double* mu, int64_t m, int d, int DP,
                              int64_t m_pad, int jx, unsigned short* out, const float* valid,
                              hipStream_t s, const int* qperm) {
  int64_t blocks = (m_pad * DP + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(prep_half_queries_kernel, dim3((unsigned)blocks), dim3(256), 0, s, Q64, mu, m,
                     d, DP, m_pad, jx, out, valid, qperm);
}

// ---------------------------------- int8 images (kernel metric 5, d <= 256)
// Integer-coded data (e.g. SIFT-like byte features scaled by a power of two,
// the reference's CSV of k/256 values): every train value is x = (c_i + k) /
// 2^s with an integer code k in [-128, 127] per dimension i.  Then q.x on
// v_mfma_i32_16x16x64_i8 is exact (int32 accumulation), twice the fp16 MFMA
// rate per element.
//
// grid_stats: per-dim min / max (fp64) and the largest number of fractional
// bits of any value (x = odd * 2^lsb -> max(0, -lsb)); two stages.
__device__ __forceinline__ int frac_bits(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const int e = (int)((b >> 52) & 0x7FF);
  const unsigned long long mant = (b & 0xFFFFFFFFFFFFFull) | (e ? (1ull << 52) : 0ull);
  if (mant == 0) return 0;                        // +-0
  if (e == 0x7FF) return 4096;                    // non-finite (refused elsewhere)
  const int lsb = (e ? e : 1) - 1075 + __builtin_ctzll(mant);
  return lsb < 0 ? -lsb : 0;
}

__global__ void __launch_bounds__(256)
grid_stats_kernel(const double* __restrict__ X64, int64_t n, int d, int64_t rpb,
                  double* __restrict__ partial, unsigned* __restrict__ frac) {
  // partial: [nb][2][d] (min | max)
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < n ? r0 + rpb : n;
  int fb = 0;
  for (int c = threadIdx.x; c < d; c += 256) {
    double lo = KNN_INF_D, hi = -KNN_INF_D;
    for (int64_t r = r0; r < r1; ++r) {
      const double x = X64[r * d + c];
      lo = fmin(lo, x);
      hi = fmax(hi, x);
      fb = max(fb, frac_bits(x));
    }
    partial[((int64_t)blockIdx.x * 2) * d + c] = lo;
    partial[((int64_t)blockIdx.x * 2 + 1) * d + c] = hi;
  }
  fb = wave_max_i(fb);
  if ((threadIdx.x & 63) == 0 && fb) atomicMax(frac, (unsigned)fb);
}

__global__ void grid_stats_final_kernel(const double* __restrict__ partial, int nb, int d,
                                        double* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= d) return;
  double lo = KNN_INF_D, hi = -KNN_INF_D;
  for (int b = 0; b < nb; ++b) {
    lo = fmin(lo, partial[(int64_t)(2 * b) * d + c]);
    hi = fmax(hi, partial[(int64_t)(2 * b + 1) * d + c]);
  }
  out[c] = lo;
  out[d + c] = hi;
}

void launch_grid_stats(const double* X64, int64_t n, int d, double* partial, double* out,
                       unsigned* frac, hipStream_t s) {
  const int nb = col_mean_blocks(n);
  const int64_t rpb = (n + nb - 1) / nb;
  hipLaunchKernelGGL(grid_stats_kernel, dim3(nb), dim3(256), 0, s, X64, n, d, rpb, partial, frac);
  hipLaunchKernelGGL(grid_stats_final_kernel, dim3((d + 255) / 256), dim3(256), 0, s, partial, nb,
                     d, out);
}

// Train rows: [int8 codes (DP bytes, 16-B chunks at (c >> 4) ^ xh_swz(row)) |
// 4 int32], codes k = x 2^s - c_i; the int32 of row 4g + j (in the pad of
// row 4g, j = 0..3) is -ceil(||k||^2 / 2), the accumulator seed: the kernel
// ends at dot(q, k) - ceil(||k||^2 / 2) = -(proxy + (||k||^2 & 1)) / 2 with
// proxy = ||k||^2 - 2 q.k, i.e. it ranks by proxy + (0 or 1).  Pad rows:
// kI8Floor (below every real accumulator: never selected).  codes_max receives max ||k||^2.
__global__ void __launch_bounds__(256)
prep_i8_train_kernel(const double* __restrict__ X64, const double* __restrict__ cent, int64_t n,
                     int d, int DP, int64_t n_pad, int s, signed char* __restrict__ out,
                     unsigned* __restrict__ codes_max, int swz, const int* __restrict__ perm) {
  const int row_bytes = DP + 16;
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  unsigned mx = 0;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n_pad; row += wstride) {
    int q2 = 0;
    const int cx = swz ? xh_swz((int)(row & 15)) << 4 : 0;
    const int64_t src = src_row(perm, row, n);
    for (int c = lane; c < DP; c += 64) {
      int k = 0;
      if (row < n && c < d) {
        k = (int)__builtin_rint(__builtin_ldexp(X64[src * d + c], s) - cent[c]);
        q2 += k * k;
      }
      out[row * row_bytes + (c ^ cx)] = (signed char)k;
    }
    q2 = wave_sum_i(q2);
    mx = max(mx, (unsigned)q2);
    const int seed = row < n ? -((q2 + 1) >> 1) : kI8Floor;
    // seeds of rows 4g .. 4g+3 in the pad of row 4g (n_pad % 4 == 0): every
    // row writes its own slot of its group leader's pad
    if (lane == 0) ((int*)(out + (row & ~3ll) * row_bytes + DP))[row & 3] = seed;
  }
  if (lane == 0 && mx) atomicMax(codes_max, mx);
}

// Sub-tile seed maxima: thread u4 = 32-row sub-tile, the max of its 32 seeds
// (pads of its rows 4g) into int slot (u4 & 3) of the pad of row 128 (u4 >>
// 2) + kI8SmaxRow, and the max of its partial seeds into the pad of row
// 128 (u4 >> 2) + kI8SmaxARow.  An all-pad sub-tile gets kI8Floor.
__global__ void __launch_bounds__(256)
prep_i8_smax_kernel(signed char* __restrict__ out, int DP, int64_t n_sub, int swz) {
  const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (u >= n_sub) return;
  const int64_t row_bytes = DP + 16;
  int mx = kI8Floor;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const int4 sd = *(const int4*)(out + (u * 32 + 4 * g) * row_bytes + DP);
    mx = max(mx, max(max(sd.x, sd.y), max(sd.z, sd.w)));
  }
  // the partial seeds: -ceil(||k_A||^2 / 2) over the first i8_part_dims(DP)
  // dims (chunk ch of 16 codes sits at ch ^ xh_swz(row & 15) in a swizzled
  // image); pad rows (all-zero codes) give 0, a valid upper bound
  const int dA = i8_part_dims(DP);
  int mxa = dA > 0 ? kI8Floor : 0;
  for (int r = 0; r < 32 && dA > 0; ++r) {
    const int64_t row = u * 32 + r;
    const signed char* p = out + row * row_bytes;
    const int sw = swz ? xh_swz((int)(row & 15)) : 0;
    int kk = 0;
    for (int ch = 0; ch < dA / 16; ++ch) {
      const int4 v = *(const int4*)(p + ((ch ^ sw) << 4));
      kk = __builtin_amdgcn_sdot4(v.x, v.x, kk, false);
      kk = __builtin_amdgcn_sdot4(v.y, v.y, kk, false);
      kk = __builtin_amdgcn_sdot4(v.z, v.z, kk, false);
      kk = __builtin_amdgcn_sdot4(v.w, v.w, kk, false);
    }
    mxa = max(mxa, -((kk + 1) >> 1));
  }
  ((int*)(out + ((u >> 2) * 128 + kI8SmaxRow) * row_bytes + DP))[u & 3] = mx;
  ((int*)(out + ((u >> 2) * 128 + kI8SmaxARow) * row_bytes + DP))[u & 3] = mxa;
}

void launch_prep_i8_train(const double* X64, const double* cent, int64_t n, int d, int DP,
                          int64_t n_pad, int s, signed char* out, unsigned* codes_max, int swz,
                          hipStream_t st, const int* perm) {
  int64_t blocks = (n_pad + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(prep_i8_train_kernel, dim3((unsigned)blocks), dim3(256), 0, st, X64, cent, n,
                     d, DP, n_pad, s, out, codes_max, swz, perm);
  // the sub-tile maxima of 128-row group g sit in the pad of its row 1: only
  // whole groups (callers pass n_pad a multiple of kRowAlign = 256; a ragged
  // tail group would place them past the image, so it gets none)
  const int64_t n_sub = n_pad / 128 * 4;
  hipLaunchKernelGGL(prep_i8_smax_kernel, dim3((unsigned)((n_sub + 255) / 256)), dim3(256), 0, st,
                     out, DP, n_sub, swz);
}

// Query rows: int8 codes clamp(rint(q 2^s - c_i), -128, 127) (DP bytes,
// plain row-major).  A value off the train set's grid or beyond the code
// range is rounded / saturated; the merge rebuilds the same code, measures
// the query's coding error and widens its bound by it (merge_rerank_kernel).
// One wave per operand row p (query q = qperm[p]), and in the same launch
// the two per-query steps that precede the candidate pass: the operand-range
// check of query_check_kernel (valid[q]: 1, 0 = void proxies / exact rescan,
// -1 = a non-finite coordinate; a void query gets zero codes) and, with gthr
// set, row p's threshold slots as launch_fill_gthr writes them -- one kernel
// instead of three (~4-6 us each at cfg2, profiles/r5_kernels_cfg2.json).
// zero[0, nzero): the region sort's block counts, read by this call's sort
// (which ran before) and cleared here for the next call's histogram; zero4:
// the call's rescan / tie counters (4 ints, read by the merge), cleared here
// instead of by a memset launch after the candidate kernel.
__global__ void __launch_bounds__(256)
prep_i8_queries_kernel(const double* __restrict__ Q64, const double* __restrict__ mu, double scale,
                       int jx, double limit, const double* __restrict__ cent, int64_t m, int d,
                       int DP, int64_t m_pad, int s, signed char* __restrict__ out,
                       float* __restrict__ valid, const int* __restrict__ qperm,
                       uint32_t* __restrict__ gthr, int active, int* __restrict__ zero,
                       int64_t nzero, int* __restrict__ zero4) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nzero; e += (int64_t)gridDim.x * 256)
    zero[e] = 0;
  if (zero4 && blockIdx.x == 0 && threadIdx.x < 4) zero4[threadIdx.x] = 0;
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < m_pad; row += wstride) {
    const int64_t q = src_row(qperm, row, m);
    bool ok = true, fin = true;
    if (row < m)
      for (int c = lane; c < d; c += 64) {
        const double x = Q64[q * d + c];
        fin = fin && !nonfinite_bits(x);
        ok = ok && __builtin_fabs(__builtin_ldexp(scale * (x - mu[c]), jx)) < limit;
      }
    ok = __ballot(!ok) == 0;
    fin = __ballot(!fin) == 0;
    const float vq = !fin ? -1.0f : (ok ? 1.0f : 0.0f);
    if (lane == 0) valid[q] = vq;  // (pad rows: q = row, valid 1)
    const bool use = row < m && vq > 0.0f;
    for (int c = lane; c < DP; c += 64) {
      int k = 0;
      if (use && c < d) {
        const double y = __builtin_ldexp(Q64[q * d + c], s) - cent[c];
        k = (int)__builtin_fmin(__builtin_fmax(__builtin_rint(y), -128.0), 127.0);
      }
      out[row * DP + c] = (signed char)k;
    }
    if (gthr && lane < kGthrSlots) gthr[row * kGthrSlots + lane] = lane < active ? kGthrInit : 0u;
  }
}

void launch_prep_i8_queries(const double* Q64, const double* mu, double scale, int jx,
                            double limit, const double* cent, int64_t m, int d, int DP,
                            int64_t m_pad, int s, signed char* out, float* valid, hipStream_t st,
                            const int* qperm, uint32_t* gthr, int active, int* zero,
                            int64_t nzero, int* zero4) {
  int64_t blocks = (m_pad + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(prep_i8_queries_kernel, dim3((unsigned)blocks), dim3(256), 0, st, Q64, mu,
                     scale, jx, limit, cent, m, d, DP, m_pad, s, out, valid, qperm, gthr, active,
                     zero, nzero, zero4);
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

__global__ void fill_gthr_kernel(uint32_t* g, int64_t n, int active) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
    g[e] = (int)(e % kGthrSlots) < active ? kGthrInit : 0u;
}
// Threshold seeding: per query, the need-th smallest proxy of the union of
// its lists from the pre-pass over a strided sample of the train rows (U
// entries; +inf entries are empty) into every active slot (0 elsewhere, as
// the fill).  tq = max over the slots then has >= need distinct rows at or
// below it whatever mix of this value and the main pass's publishes the
// slots hold (knn_api.cpp, seeded thresholds).  One wave per query.
__global__ void __launch_bounds__(256)
seed_gthr_kernel(const float* __restrict__ v, int64_t m_pad, int U, int need, int active,
                 uint32_t* __restrict__ g) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= m_pad) return;
  const float* lv = v + q * U;
  int fin = 0;
  for (int x = lane; x < U; x += 64) fin += f2key(lv[x]) < kKeyInf;
  fin = wave_sum_i(fin);
  uint32_t pre = kKeyInf;
  if (fin >= need) {
    pre = 0;  // radix select: key of the need-th smallest
    for (int b = 31; b >= 0; --b) {
      const uint32_t T = pre | ((1u << b) - 1u);
      int cnt = 0;
      for (int x = lane; x < U; x += 64) cnt += f2key(lv[x]) <= T;
      if (wave_sum_i(cnt) < need) pre |= 1u << b;
    }
  }
  if (lane < kGthrSlots) g[q * kGthrSlots + lane] = lane < active ? pre : 0u;
}
void launch_seed_gthr(const float* v, int64_t m_pad, int U, int need, int active, uint32_t* g,
                      hipStream_t s) {
  if (m_pad <= 0) return;
  hipLaunchKernelGGL(seed_gthr_kernel, dim3((unsigned)((m_pad + 3) / 4)), dim3(256), 0, s, v, m_pad,
                     U, need, active, g);
}

void launch_fill_gthr(uint32_t* g, int64_t m_pad, int active, hipStream_t s) {
  const int64_t n = m_pad * kGthrSlots;
  if (n <= 0) return;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(fill_gthr_kernel, dim3((unsigned)blocks), dim3(256), 0, s, g, n, active);
}

// ------------------------------- fp16 S3 images (DP > 256; cand_s3h_kernel)
// Tile-chunk images: block (tile of kS3R rows, chunk of 32 dims) = kS3R rows
// x 64 B, the four 16-B slots of row r (dims 0-7, 8-15, 16-23, 24-31 of the
// chunk) at slot position s3h_slot(r, s) -- the bf16x3 S3 layout with one
// fp16 k-step of 16 dims in place of each hi/lo pair and its own swizzle.  One wave per row,
// lane g < DP/8 converting dims 8g .. 8g+7 of mult * (x - mu) at scale 2^jx.
// Train (mult 1): the row's representation error ||h / 2^jx - (x - mu)||^2
// is measured as in prep_half_train, seeds fl32(||x32||^2) (+inf on pad
// rows) go to seed_out.  Queries (mult -2): zero operands for a query
// launch_query_check marked invalid.
__global__ void __launch_bounds__(256)
prep_half_tiled_kernel(const double* __restrict__ X64, const double* __restrict__ mu, int64_t n,
                       int d, int DP, int64_t n_pad, int jx, double mult,
                       unsigned short* __restrict__ out, const float* __restrict__ seed_src,
                       float* __restrict__ seed_out, const float* __restrict__ valid,
                       unsigned long long* __restrict__ dx2max, const int* __restrict__ perm) {
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  const double sinv = __builtin_ldexp(1.0, -jx);
  const int G = DP / 8, nch = DP / 32;
  double m = 0.0;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n_pad; row += wstride) {
    const bool live = row < n && (!valid || valid[row] > 0.0f);
    const int64_t tile = row / kS3R;
    const int r = (int)(row - tile * kS3R);
    const int64_t src = src_row(perm, row, n);
    double e2 = 0.0;
    for (int g = lane; g < G; g += 64) {
      unsigned short hv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int col = 8 * g + u;
        _Float16 h = (_Float16)0.0f;
        if (live && col < d) {
          const double x = X64[src * d + col] - mu[col];
          h = f16_operand(mult * x, jx);
          if (dx2max) {
            const double e = (double)h * sinv - x;
            e2 += e * e;
          }
        }
        hv[u] = __builtin_bit_cast(unsigned short, h);
      }
      uint4 v;
      v.x = hv[0] | (uint32_t)hv[1] << 16;
      v.y = hv[2] | (uint32_t)hv[3] << 16;
      v.z = hv[4] | (uint32_t)hv[5] << 16;
      v.w = hv[6] | (uint32_t)hv[7] << 16;
      unsigned char* blk = (unsigned char*)out + (((int64_t)tile * nch + (g >> 2)) * kS3R + r) * 64;
      *(uint4*)(blk + s3h_slot(r, g & 3) * 16) = v;
    }
    if (seed_out && lane == 0) seed_out[row] = row < n ? seed_src[row] : KNN_INF_F;
    if (dx2max) m = fmax(m, wave_sum_d(e2));
  }
  if (dx2max && lane == 0)
    atomicMax(dx2max, (unsigned long long)__double_as_longlong(m * (1.0 + 1e-12)));
}

void launch_prep_half_tiled(const double* X64, const double* mu, int64_t n, int d, int DP,
                            int64_t n_pad, int jx, double mult, unsigned short* out,
                            const float* seed_src, float* seed_out, const float* valid,
                            unsigned long long* dx2max, hipStream_t s, const int* perm) {
  int64_t blocks = (n_pad + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(prep_half_tiled_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X64, mu, n, d,
                     DP, n_pad, jx, mult, out, seed_src, seed_out, valid, dx2max, perm);
}

// ------------------------------- S3 images (bf16x3, DP > 256; knn_cand.hip)
// Tile-chunk images: block (tile, chunk of 16 dims) = 256 rows x 64 B, the
// four 16-B slots of row r at slot position s ^ ((r >> 2) & 3).
__global__ void __launch_bounds__(256)
prep_split_tiled_kernel(const double* __restrict__ X64, const double* __restrict__ mu, int64_t n,
                        int d, int DP, int64_t n_pad, double scale, unsigned short* __restrict__ out,
                        const float* __restrict__ seed_src, float* __restrict__ seed_out,
                        const int* __restrict__ perm) {
  const int G = DP / 8;  // 8-dim groups per row
  const int nch = DP / kS3DC;
  const int64_t total = n_pad * G;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int64_t row = e / G;
    const int g = (int)(e - row * G);
    unsigned short hi[8], lo[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int col = 8 * g + u;
      hi[u] = lo[u] = 0;
      if (row < n && col < d)
        split_bf16(scale * (X64[src_row(perm, row, n) * d + col] - mu[col]), hi[u], lo[u]);
    }
    const int64_t tile = row / kS3R;
    const int r = (int)(row - tile * kS3R);
    const int c = g >> 1, sh = g & 1;
    unsigned char* blk = (unsigned char*)out + (((int64_t)tile * nch + c) * kS3R + r) * 64;
    uint4 vh, vl;
    vh.x = hi[0] | (uint32_t)hi[1] << 16; vh.y = hi[2] | (uint32_t)hi[3] << 16;
    vh.z = hi[4] | (uint32_t)hi[5] << 16; vh.w = hi[6] | (uint32_t)hi[7] << 16;
    vl.x = lo[0] | (uint32_t)lo[1] << 16; vl.y = lo[2] | (uint32_t)lo[3] << 16;
    vl.z = lo[4] | (uint32_t)lo[5] << 16; vl.w = lo[6] | (uint32_t)lo[7] << 16;
    *(uint4*)(blk + s3_slot(r, sh) * 16) = vh;
    *(uint4*)(blk + s3_slot(r, 2 + sh) * 16) = vl;
    if (seed_out && g == 0) seed_out[row] = row < n ? seed_src[row] : KNN_INF_F;
  }
}

void launch_prep_split_tiled(const double* X64, const double* mu, int64_t n, int d, int DP,
                             int64_t n_pad, double scale, unsigned short* out,
                             const float* seed_src, float* seed_out, hipStream_t s,
                             const int* perm) {
  int64_t blocks = (n_pad * (DP / 8) + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(prep_split_tiled_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X64, mu, n, d,
                     DP, n_pad, scale, out, seed_src, seed_out, perm);
}

}  // namespace knnk
