// knn_normalize.hip -- transductive min-max normalisation on the GPU
// (reference knn_mpi.cpp cpp:229-306), bit-exact in fp64.
//
// The reference keeps per-dimension max/min over the rank's train rows and
// its test/validation shards, starting from max = -1 and min = 999999
// (cpp:239-243), with strict compares (cpp:250-251, 259-260, 270-271),
// MPI_Allreduce MAX/MIN (cpp:276-277), then rewrites every value as
// (x - min)/(max - min) on the dimensions where max - min != 0 (cpp:279-305).
//
// Here: one HBM pass per set for the statistics, one read-modify-write pass
// to apply them.  Both kernels use a grid of T = d*R threads whose stride is
// a multiple of d, so each thread owns one column (its bounds sit in
// registers) while consecutive lanes still read consecutive doubles.
// min/max are exact selections, so the reduction order cannot change the
// result (the sign of a zero extremum aside, which the reference's own
// MPI_Allreduce leaves unspecified too).  Compiled without -fno-honor-nans:
// a NaN value never wins a compare, exactly as in the reference.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "knn_kernels.h"

namespace knnk {

namespace {

constexpr int kNB = 256;  // threads per block

__global__ void __launch_bounds__(kNB)
minmax_partial_kernel(const double* __restrict__ X, int64_t total, int64_t T,
                      double* __restrict__ pmax, double* __restrict__ pmin) {
  const int64_t g = (int64_t)blockIdx.x * kNB + threadIdx.x;
  if (g >= T) return;
  // neutral elements of the strict compares: -inf never beats the final
  // "-1" start value and +inf never beats "999999", so folding them in at
  // the end gives exactly the reference's sequential result
  double mx = -INFINITY, mn = INFINITY;
  int64_t e = g;
  for (; e + 3 * T < total; e += 4 * T) {  // 4 loads in flight per thread
    const double v0 = X[e], v1 = X[e + T], v2 = X[e + 2 * T], v3 = X[e + 3 * T];
    if (v0 > mx) mx = v0;
    if (v0 < mn) mn = v0;
    if (v1 > mx) mx = v1;
    if (v1 < mn) mn = v1;
    if (v2 > mx) mx = v2;
    if (v2 < mn) mn = v2;
    if (v3 > mx) mx = v3;
    if (v3 < mn) mn = v3;
  }
  for (; e < total; e += T) {
    const double v = X[e];
    if (v > mx) mx = v;
    if (v < mn) mn = v;
  }
  pmax[g] = mx;
  pmin[g] = mn;
}

// One block per column: fold the R partials of column c (entries r*d + c)
// and then the running value (init: the reference's -1 / 999999).
__global__ void __launch_bounds__(kNB)
minmax_final_kernel(const double* __restrict__ pmax, const double* __restrict__ pmin, int d,
                    int64_t R, double* __restrict__ omax, double* __restrict__ omin, int init) {
  __shared__ double smx[kNB], smn[kNB];
  const int c = blockIdx.x, t = threadIdx.x;
  double mx = -INFINITY, mn = INFINITY;
  for (int64_t r = t; r < R; r += kNB) {
    const double a = pmax[r * d + c], b = pmin[r * d + c];
    if (a > mx) mx = a;
    if (b < mn) mn = b;
  }
  smx[t] = mx;
  smn[t] = mn;
  __syncthreads();
  for (int o = kNB / 2; o > 0; o >>= 1) {
    if (t < o) {
      if (smx[t + o] > smx[t]) smx[t] = smx[t + o];
      if (smn[t + o] < smn[t]) smn[t] = smn[t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    double cmx = init ? -1.0 : omax[c];
    double cmn = init ? 999999.0 : omin[c];
    if (smx[0] > cmx) cmx = smx[0];
    if (smn[0] < cmn) cmn = smn[0];
    omax[c] = cmx;
    omin[c] = cmn;
  }
}

__global__ void __launch_bounds__(kNB)
normalize_apply_kernel(double* __restrict__ X, int64_t total, int64_t T, int d,
                       const double* __restrict__ vmax, const double* __restrict__ vmin) {
  const int64_t g = (int64_t)blockIdx.x * kNB + threadIdx.x;
  if (g >= T) return;
  const int c = (int)(g % d);
  const double lo = vmin[c];
  const double range = vmax[c] - lo;  // cpp:284: max_value[j] - min_value[j]
  if (!(range != 0)) return;          // dimension left as is
  int64_t e = g;
  for (; e + 3 * T < total; e += 4 * T) {
    const double v0 = X[e], v1 = X[e + T], v2 = X[e + 2 * T], v3 = X[e + 3 * T];
    X[e] = (v0 - lo) / range;
    X[e + T] = (v1 - lo) / range;
    X[e + 2 * T] = (v2 - lo) / range;
    X[e + 3 * T] = (v3 - lo) / range;
  }
  for (; e < total; e += T) X[e] = (X[e] - lo) / range;
}

}  // namespace

int64_t minmax_rows_per_sweep(int64_t rows, int d, int cu_count) {
  // about 2048 threads per CU in flight, at least one row, at most all rows
  int64_t R = ((int64_t)cu_count * 2048 + d - 1) / d;
  if (R > rows) R = rows;
  return R < 1 ? 1 : R;
}

void launch_minmax(const double* X, int64_t rows, int d, int64_t R, double* partial,
                   double* out_max, double* out_min, int init, hipStream_t s) {
  const int64_t T = (int64_t)d * R;
  if (rows > 0) {
    hipLaunchKernelGGL(minmax_partial_kernel, dim3((unsigned)((T + kNB - 1) / kNB)), dim3(kNB), 0,
                       s, X, rows * d, T, partial, partial + T);
  }
  hipLaunchKernelGGL(minmax_final_kernel, dim3((unsigned)d), dim3(kNB), 0, s, partial,
                     partial + T, d, rows > 0 ? R : (int64_t)0, out_max, out_min, init);
}

void launch_normalize_apply(double* X, int64_t rows, int d, int64_t R, const double* vmax,
                            const double* vmin, hipStream_t s) {
  if (rows <= 0) return;
  const int64_t T = (int64_t)d * R;
  hipLaunchKernelGGL(normalize_apply_kernel, dim3((unsigned)((T + kNB - 1) / kNB)), dim3(kNB), 0,
                     s, X, rows * d, T, d, vmax, vmin);
}

}  // namespace knnk
