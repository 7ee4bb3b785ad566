// knn_api.cpp -- C ABI (include/knn_amd.h) over the gfx950 kernels.
//
// One knn_ctx per GPU (≙ one MPI rank of the reference, cpp:121-125).  The
// train set lives in HBM in two forms: the caller's fp64 rows (exact
// re-rank, ≙ Data_train cpp:140) and a padded fp32 copy + per-row seeds for
// the MFMA candidate pass.  Queries are classified by the pipeline in
// knn_cand.hip / knn_select.hip; there is no host compute path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/knn_amd.h"
#include "knn_api_internal.h"
#include "knn_kernels.h"

using namespace knnk;

namespace {
thread_local std::string g_err;
}

void knn_set_error(const char* fmt, const char* a, long long b) {
  char buf[512];
  snprintf(buf, sizeof buf, fmt, a, b);
  g_err = buf;
}

int knn_fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return knn_fail(KNN_ERR_DEVICE, std::string(#expr " failed: ") + hipGetErrorString(e_)); \
  } while (0)

int DevBuf::ensure(size_t bytes) {
  if (cap >= bytes && p) return KNN_OK;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  if (bytes == 0) bytes = 16;
  if (hipMalloc(&p, bytes) != hipSuccess) {
    p = nullptr;
    return knn_fail(KNN_ERR_NOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes failed");
  }
  cap = bytes;
  return KNN_OK;
}
void DevBuf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
}

static int device_guard(knn_ctx* ctx) {
  if (!ctx) return knn_fail(KNN_ERR_ARG, "null context");
  HIP_TRY(hipSetDevice(ctx->device));
  return KNN_OK;
}

extern "C" {

const char* knn_version(void) { return "mpi-knn-amd 0.1 (gfx950)"; }
const char* knn_last_error(void) { return g_err.c_str(); }

int knn_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int knn_create(knn_ctx** out, int device) {
  if (!out) return knn_fail(KNN_ERR_ARG, "null out pointer");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
    return knn_fail(KNN_ERR_DEVICE, "no HIP device available (the KNN path has no CPU fallback)");
  if (device < 0 || device >= n) return knn_fail(KNN_ERR_ARG, "device index out of range");
  HIP_TRY(hipSetDevice(device));
  knn_ctx* c = new knn_ctx();
  c->device = device;
  // a blocking stream: ordered after work the caller queued on the legacy
  // default stream (e.g. torch producing the device inputs), so device
  // pointers handed to *_device calls with stream = NULL are safe to read
  if (hipStreamCreateWithFlags(&c->stream, hipStreamDefault) != hipSuccess) {
    delete c;
    return knn_fail(KNN_ERR_DEVICE, "hipStreamCreate failed");
  }
  // per-call rescan counts, written by the device (host-mapped pinned memory)
  if (hipHostMalloc((void**)&c->h_counts, sizeof(int) * 4, hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&c->d_counts, c->h_counts, 0) != hipSuccess ||
      hipEventCreateWithFlags(&c->done_ev, hipEventDisableTiming) != hipSuccess ||
      c->totals.ensure(3 * sizeof(unsigned long long)) != KNN_OK ||
      hipMemset(c->totals.p, 0, 3 * sizeof(unsigned long long)) != hipSuccess) {
    knn_destroy(c);
    return knn_fail(KNN_ERR_DEVICE, "context setup (pinned counters / events) failed");
  }
  c->h_counts[0] = c->h_counts[1] = 0;
  if (hipDeviceGetAttribute(&c->cu_count, hipDeviceAttributeMultiprocessorCount, device) !=
          hipSuccess ||
      c->cu_count <= 0)
    c->cu_count = 256;
  if (const char* e = getenv("KNN_PRECISION")) {
    if (!strcmp(e, "fp32")) c->precision = KNN_PRECISION_FP32;
    else if (!strcmp(e, "bf16x3")) c->precision = KNN_PRECISION_BF16X3;
    else if (!strcmp(e, "fp16")) c->precision = KNN_PRECISION_FP16;
  }
  *out = c;
  return KNN_OK;
}

int knn_destroy(knn_ctx* ctx) {
  if (!ctx) return KNN_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (DevBuf* b : ctx->all_bufs()) b->release();
  for (auto& tc : ctx->ring)
    for (auto& e : tc.ev)
      if (e) (void)hipEventDestroy(e);
  if (ctx->done_ev) (void)hipEventDestroy(ctx->done_ev);
  if (ctx->h_counts) (void)hipHostFree(ctx->h_counts);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return KNN_OK;
}

}  // extern "C"

// Integer-coded train sets (knn_prep.hip, int8 images): every value x =
// (c_i + k) / 2^s with an integer code k in [-128, 127] per dimension -- the
// 8-bit grid of SIFT-like byte features, or of the reference's CSVs of
// k/256 values.  s = the largest number of fractional bits of any value; the
// centre c_i is the middle of dimension i's code range.  Sets ctx->i8_ok.
static int detect_i8(knn_ctx* ctx, const double* dX, int64_t n, int d) {
  ctx->i8_ok = false;
  if (pad_dim_i8(d) <= 0) return KNN_OK;
  int rc;
  if ((rc = ctx->i8_gs.ensure((size_t)(col_mean_blocks(n) * 2 + 2) * d * sizeof(double) + 16)))
    return rc;
  double* part = (double*)ctx->i8_gs.p;
  double* out = part + (size_t)col_mean_blocks(n) * 2 * d;
  unsigned* frac = (unsigned*)(out + 2 * d);
  HIP_TRY(hipMemsetAsync(frac, 0, sizeof(unsigned), ctx->stream));
  launch_grid_stats(dX, n, d, part, out, frac, ctx->stream);
  HIP_TRY(hipGetLastError());
  std::string buf((size_t)2 * d * sizeof(double) + sizeof(unsigned), '\0');
  HIP_TRY(hipMemcpyAsync(&buf[0], out, buf.size(), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  const double* lohi = (const double*)buf.data();
  unsigned s;
  memcpy(&s, buf.data() + 2 * d * sizeof(double), sizeof s);
  if (s > 30) return KNN_OK;
  std::string cent((size_t)2 * d * sizeof(double), '\0');
  double* c = (double*)&cent[0];
  for (int i = 0; i < d; ++i) {
    const double lo = std::ldexp(lohi[i], (int)s), hi = std::ldexp(lohi[d + i], (int)s);
    if (!(hi - lo <= 255.0) || !(std::fabs(lo) < 0x1p50) || !(std::fabs(hi) < 0x1p50)) return KNN_OK;
    c[i] = std::floor((lo + hi + 1.0) / 2.0);        // codes x 2^s - c in [-128, 127]
    c[d + i] = std::ldexp(c[i], -(int)s);            // the same centre in value units
  }
  if ((rc = ctx->i8_cent.ensure((size_t)2 * d * sizeof(double)))) return rc;
  HIP_TRY(hipMemcpy(ctx->i8_cent.p, c, (size_t)2 * d * sizeof(double), hipMemcpyHostToDevice));
  ctx->i8_s = (int)s;
  ctx->i8_ok = true;
  return KNN_OK;
}

// Region order of the train images (knn_order.hip): regions for n rows (0:
// train order).  Only where the resident kernels run (d <= 256).  Auto: 64
// regions (at most one per 16K rows) for integer-coded train sets (the int8
// pass) whose image fits the 256 MB MALL with room to spare, and for other
// sets (the fp16 pass) whose fp16 image is at most 512 MB.  With the
// order, a split's query tiles start their streams at different rows and no
// longer share the staged tiles in L2, so a larger image is re-read from
// HBM: the 12.5M x 96 shard ran 12.11 -> 13.87 ms, cfg2 1.342 -> 1.266 ms,
// 1M x 128 x 100K queries 13.16 -> 11.47 ms; the fp16 pass on continuous
// data gained nothing (2.343 / 2.342 ms; profiles/ab_log.md r4i, r4j).
// 1: on at any size, 2..64: that many regions.
constexpr int64_t kOrderMaxImage = 192ll << 20;
// Train sets that are not integer-coded (the fp16 pass, continuous data):
// auto on for fp16 images up to 512 MB.  Round 6, continuous cfg2 (272 MB
// fp16 image): candidate kernel 2.353-2.363 -> 2.170-2.197 ms, rescans 2 ->
// 1 per call, query ordering +17 us per call (profiles/ab_log.md r6h) --
// the wave-uniform fp16 test (KNN_M4_FAST) turned the tight early
// thresholds into skipped slow paths (round 4 measured 1.6 % without it).
constexpr int64_t kOrderMaxImageF16 = 512ll << 20;
// Query tiles start their streams at one of 8 phases of the region chain
// (the first region of their region's eighth), not at their own region:
// tiles of one phase share the staged tiles in L2 again -- cfg2 candidate
// 1.212 -> 1.209 ms, L2-miss traffic 1.94 -> 1.34 GB per launch; 4 phases
// 1.250 ms (profiles/ab_log.md r4p).  Tuning key "ophase": -1 auto, 0 the
// tile's own region, N phases.
constexpr int kOrderPhases = 8;
static int region_count(const knn_ctx* ctx, int64_t n, int d) {
  if (ctx->tune_order == 0 || pad_dim_fp16(d) <= 0) return 0;
  int P = (int)std::min<int64_t>(kRegionMax, n / 16384);
  if (ctx->tune_order < 0) {
    if (ctx->i8_ok && pad_dim_i8(d) > 0)
      return P >= 8 && n * (pad_dim_i8(d) + 16) <= kOrderMaxImage ? P : 0;
    const int DPh = pad_dim_fp16(d);
    return DPh > 0 && P >= 8 && n * (int64_t)(DPh / 2 + 4) * 4 <= kOrderMaxImageF16 ? P : 0;
  }
  if (ctx->tune_order >= 2) P = (int)std::min<int64_t>(ctx->tune_order, kRegionMax);
  P = (int)std::min<int64_t>(P, n / 256);
  return P >= 2 ? P : 0;
}

// k-means on a strided sample (8 Lloyd rounds), every row assigned, rows
// counting-sorted by the chain rank of their region (knn_order.hip).
static int build_order(knn_ctx* ctx, const double* dX, const double* mu, int64_t n, int d, int jx,
                       int P) {
  const int64_t ns = std::min<int64_t>(n, 65536);
  const int64_t stride = n / ns;
  const int64_t nb = region_sort_blocks(n);
  int rc;
  if ((rc = ctx->ord_cent.ensure((size_t)kRegionMax * d * sizeof(float)))) return rc;
  if ((rc = ctx->ord_cnorm.ensure(kRegionMax * sizeof(float)))) return rc;
  if ((rc = ctx->ord_img.ensure(kRegionImgBytes))) return rc;
  if ((rc = ctx->ord_rank.ensure(kRegionMax * sizeof(int)))) return rc;
  if ((rc = ctx->ord_rstart.ensure(kRegionMax * sizeof(int)))) return rc;
  if ((rc = ctx->ord_tot.ensure(kRegionMax * sizeof(int)))) return rc;
  if ((rc = ctx->ord_key.ensure((size_t)n * sizeof(int)))) return rc;
  if ((rc = ctx->ord_bcnt.ensure((size_t)nb * kRegionMax * sizeof(int)))) return rc;
  if ((rc = ctx->ord_perm.ensure((size_t)n * sizeof(int)))) return rc;
  if ((rc = ctx->ord_ipos.ensure((size_t)n * sizeof(int)))) return rc;
  float* cent = (float*)ctx->ord_cent.p;
  int* rank = (int*)ctx->ord_rank.p;
  int* key = (int*)ctx->ord_key.p;
  launch_region_kmeans(dX, mu, ns, d, stride, jx, P, 8, cent, (unsigned short*)ctx->ord_img.p,
                       (float*)ctx->ord_cnorm.p, key, rank, ctx->stream);
  launch_region_assign(dX, mu, n, d, 1, jx, (const unsigned short*)ctx->ord_img.p,
                       (const float*)ctx->ord_cnorm.p, rank, key, nullptr, ctx->stream);
  ctx->ord_bcnt_zero = 0;  // (the train sort leaves its prefix sums there)
  launch_region_sort(key, n, (int*)ctx->ord_bcnt.p, (int*)ctx->ord_tot.p, (int*)ctx->ord_perm.p,
                     (int*)ctx->ord_ipos.p, nullptr, nullptr, (int*)ctx->ord_rstart.p, ctx->stream);
  HIP_TRY(hipGetLastError());
  ctx->ord_P = P;
  return KNN_OK;
}

// Which int8 kernel: metric 6 (v_mfma_i32_32x32x32_i8, K granularity 32)
// where it issues fewer padded dims than metric 5 (16x16x64, K 64) -- d = 96
// runs 96 dims instead of 128 (configs[3]) -- and at DP = 128 (cfg2), where
// its two 4-entry lists per lane (KNN_I8W_Q4) made it the faster kernel:
// 1.278-1.290 vs 1.290-1.303 ms candidate, all phases 1.466-1.478 vs
// 1.500-1.518 ms (profiles/ab_log.md r5g; its 32x32 MFMA holds the vector
// issue for 8 of 32 cycles, the 16x16x64 one for 8 of 16).  Tuning key
// "i8w": -1 auto, 0 always 16x16x64, 1 always 32x32x32.
static int i8_kernel_d(const knn_ctx* ctx, int d) {
  if (ctx->tune_i8w >= 0) return ctx->tune_i8w > 0 && pad_dim_i8w(d) > 0 ? 6 : 5;
  const int w = pad_dim_i8w(d);
  return w > 0 && (w < pad_dim_i8(d) || w == 128) ? 6 : 5;
}
static int i8_kernel(const knn_ctx* ctx) { return i8_kernel_d(ctx, ctx->train.d); }

// Norm blocks (knn_order.hip, launch_norm_blocks): the int8 kernels bound a
// sub-tile by its largest seed instead of reading every row's seed from LDS
// (knn_cand_res.hip), which needs rows of nearly equal norm side by side.
// Auto: integer-coded train sets of more than one window at d <= 256.
static bool norm_blocks_on(const knn_ctx* ctx, int64_t n, int d) {
  if (ctx->tune_nblk == 0 || pad_dim_fp16(d) <= 0 || n < 2) return false;
  if (ctx->tune_nblk > 0) return true;
  return ctx->i8_ok && (pad_dim_i8(d) > 0 || pad_dim_i8w(d) > 0) && n > kNormWin;
}

// The windows sorted by the int8 code norm (the seeds' own; ||x - mu||^2 for
// other sets), on top of the region order when it is on.
static int build_norm_blocks(knn_ctx* ctx, const double* dX, int64_t n, int d) {
  int rc;
  if ((rc = ctx->ord_key.ensure((size_t)n * sizeof(int)))) return rc;
  if ((rc = ctx->ord_perm.ensure((size_t)n * sizeof(int)))) return rc;
  if ((rc = ctx->ord_ipos.ensure((size_t)n * sizeof(int)))) return rc;
  const int* perm0 = nullptr;
  if (ctx->ord_P) {
    if ((rc = ctx->ord_perm0.ensure((size_t)n * sizeof(int)))) return rc;
    HIP_TRY(hipMemcpyAsync(ctx->ord_perm0.p, ctx->ord_perm.p, (size_t)n * sizeof(int),
                           hipMemcpyDeviceToDevice, ctx->stream));
    perm0 = (const int*)ctx->ord_perm0.p;
  }
  const bool i8 = ctx->i8_ok;
  // norm ranks interleaved over the int8 kernel's lane lists and sub-tiles
  // spread over the window's tiles (nblk 2: the plain sorted windows, round
  // 5's layout; 3: the interleave only)
  const int il = !i8 || ctx->tune_nblk == 2 ? 0
                 : i8_kernel_d(ctx, d) | (ctx->tune_nblk == 3 ? 0 : 16);
  launch_norm_blocks(dX, i8 ? (const double*)ctx->i8_cent.p : nullptr, ctx->i8_s,
                     (const double*)ctx->mu.p, n, d, perm0, (uint32_t*)ctx->ord_key.p,
                     (int*)ctx->ord_perm.p, (int*)ctx->ord_ipos.p, il, ctx->stream);
  HIP_TRY(hipGetLastError());
  ctx->ord_nb = true;
  return KNN_OK;
}

// Builds the fp32 candidate copy + seeds + norm stats from fp64 rows that
// already sit on the device.
static int build_train(knn_ctx* ctx, const double* dX, const int32_t* dlab, int64_t n, int d,
                       int class_cnt, int64_t idx_off) {
  const int DP = pad_dim(d);
  if (!cand_supported(DP))
    return knn_fail(KNN_ERR_ARG, "dimension " + std::to_string(d) + " not supported by this build");
  const int64_t n_pad = (n + kRowAlign - 1) / kRowAlign * kRowAlign;
  int rc;
  // padded rows [payload | seeds] (+1 KiB slack: the last LDS-DMA piece of
  // the last tile may read past the final row)
  if ((rc = ctx->X32.ensure((size_t)n_pad * (DP + 4) * sizeof(float) + 1024))) return rc;
  if ((rc = ctx->xl2.ensure((size_t)n_pad * sizeof(float)))) return rc;
  if ((rc = ctx->xl1.ensure((size_t)n_pad * sizeof(float)))) return rc;
  if ((rc = ctx->stats.ensure(6 * sizeof(unsigned long long)))) return rc;
  if ((rc = ctx->mu.ensure((size_t)d * sizeof(double)))) return rc;
  if ((rc = ctx->mu_part.ensure((size_t)col_mean_blocks(n) * d * sizeof(double)))) return rc;
  launch_col_mean(dX, n, d, (double*)ctx->mu_part.p, (double*)ctx->mu.p, ctx->stream);
  HIP_TRY(hipMemsetAsync(ctx->stats.p, 0, 6 * sizeof(unsigned long long), ctx->stream));
  unsigned long long* st_d = (unsigned long long*)ctx->stats.p;
  // operand scale 2^jx: max |x_i - mu_i| * 2^jx in [2^8, 2^9) (knn_prep.hip);
  // with it, the count of non-finite values and of labels out of range
  launch_absmax(dX, (const double*)ctx->mu.p, n, d, st_d + 2, st_d + 4, ctx->stream);
  launch_label_check(dlab, n, class_cnt, st_d + 5, ctx->stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(ctx->h_stats + 2, st_d + 2, 4 * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  ctx->trained = false;
  if (ctx->h_stats[4])
    return knn_fail(KNN_ERR_ARG, "train set holds " + std::to_string(ctx->h_stats[4]) +
                                     " non-finite values (NaN / inf): distances undefined");
  if (ctx->h_stats[5])
    return knn_fail(KNN_ERR_ARG, std::to_string(ctx->h_stats[5]) +
                                     " train labels outside [0, class_cnt)");
  memcpy(&ctx->xamax, &ctx->h_stats[2], 8);
  if ((rc = detect_i8(ctx, dX, n, d))) return rc;
  int e = 0;
  if (ctx->xamax > 0.0) (void)std::frexp(ctx->xamax, &e);  // xamax < 2^e
  // |x - mu| up to 2^400 (beyond, fp32 operands could overflow); tiny data
  // is scaled up at most 2^450 (smaller values are covered by the bound's
  // absolute terms)
  if (!(ctx->xamax < std::ldexp(1.0, 400)))
    return knn_fail(KNN_ERR_ARG, "train values out of range (|x - mean| must be < 2^400 and finite)");
  const int jx = std::min(9 - e, 450);
  // centre on the 2^-(jx+2) grid: data on any coarser grid (bytes scaled by a
  // power of two, integers, ...) is then exact in the fp16 operands, whose
  // measured representation error vanishes from the bound;
  // the shift is <= 2^-11 of max |x - mu|, immaterial for the centring
  launch_round_mu((double*)ctx->mu.p, d, jx + 2, ctx->stream);
  ctx->ord_P = 0;
  ctx->ord_nb = false;
  ctx->ord_bcnt_zero = 0;
  const int P = region_count(ctx, n, d);
  if (P > 0 && (rc = build_order(ctx, dX, (const double*)ctx->mu.p, n, d, jx, P))) return rc;
  if (norm_blocks_on(ctx, n, d) && (rc = build_norm_blocks(ctx, dX, n, d))) return rc;
  const int* perm = ctx->ord_P || ctx->ord_nb ? (const int*)ctx->ord_perm.p : nullptr;
  launch_prep_train(dX, (const double*)ctx->mu.p, n, d, DP, n_pad, jx, (float*)ctx->X32.p,
                    (float*)ctx->xl2.p, (float*)ctx->xl1.p, st_d, ctx->stream, perm);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(ctx->h_stats, st_d, 2 * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  double x2, x1;
  memcpy(&x2, &ctx->h_stats[0], 8);
  memcpy(&x1, &ctx->h_stats[1], 8);
  TrainDev& t = ctx->train;
  t.X64 = dX;
  t.mu = (const double*)ctx->mu.p;
  t.lab = dlab;
  t.X32 = (const float*)ctx->X32.p;
  t.xinit_l2 = (const float*)ctx->xl2.p;
  t.xinit_l1 = (const float*)ctx->xl1.p;
  t.n = n;
  t.n_pad = n_pad;
  t.d = d;
  t.DP = DP;
  t.x2max = x2;
  t.x1max = x1;
  t.jx = jx;
  t.perm = perm;
  t.ipos = perm ? (const int*)ctx->ord_ipos.p : nullptr;
  ctx->class_cnt = class_cnt;
  ctx->idx_off = idx_off;
  ctx->DPb = 0;  // bf16x3 / fp16 copies are rebuilt lazily for the new train set
  ctx->DPh = 0;
  ctx->DPs = 0;
  ctx->DPi = 0;
  ctx->smp_kind = 0;  // the seeding sample is rebuilt for the new train set
  ctx->i8_off = false;
  ctx->fp16_off = false;
  ctx->auto_pending = false;
  ctx->trained = true;
  return KNN_OK;
}

// The bf16 hi/lo copy of the train rows for the bf16x3 L2 candidate pass,
// built on first use (same row padding as X32).
static int ensure_bf16x3(knn_ctx* ctx, hipStream_t s) {
  const TrainDev& t = ctx->train;
  const int DPb = pad_dim_bf16x3(t.d);
  if (DPb <= 0) return knn_fail(KNN_ERR_ARG, "bf16x3 path supports d <= 256");
  if (ctx->DPb == DPb) return KNN_OK;
  int rc;
  if (bf16x3_streamed(DPb)) {
    // S3 stream kernel: tile-chunk images (4 B per dim: hi + lo) + seeds,
    // rows padded to whole 256-row tiles
    const int64_t n3 = (t.n + kS3Rows - 1) / kS3Rows * kS3Rows;
    if ((rc = ctx->XB.ensure((size_t)n3 * DPb * 4))) return rc;
    if ((rc = ctx->XS.ensure((size_t)n3 * sizeof(float)))) return rc;
    launch_prep_split_tiled(t.X64, t.mu, t.n, t.d, DPb, n3, std::ldexp(1.0, t.jx), (unsigned short*)ctx->XB.p, t.xinit_l2,
                            (float*)ctx->XS.p, s, t.perm);
  } else {
    if ((rc = ctx->XB.ensure((size_t)t.n_pad * (DPb + 4) * sizeof(float) + 1024))) return rc;
    launch_prep_split(t.X64, t.mu, t.n, t.d, DPb, t.n_pad, std::ldexp(1.0, t.jx), (unsigned short*)ctx->XB.p,
                      2 * (DPb + 4), t.xinit_l2, t.xinit_l1, s, t.perm);
  }
  HIP_TRY(hipGetLastError());
  ctx->DPb = DPb;
  return KNN_OK;
}

// The fp16 copy of the train rows for kernel metric 4:
// 2^jx (x - mu) in fp16 (the operand scale of every path) + the L2 seeds;
// same row count as X32, rows of DP/2 + 4 floats.
static int ensure_fp16(knn_ctx* ctx, hipStream_t s) {
  const TrainDev& t = ctx->train;
  const int DPh = pad_dim_fp16(t.d);
  if (DPh <= 0) return knn_fail(KNN_ERR_ARG, "fp16 path supports d <= 256");
  const int swz = ctx->tune_xhswz != 0;  // chunk swizzle of the image (xh_swz)
  if (ctx->DPh == DPh && ctx->xh_swz == swz) return KNN_OK;
  int rc;
  if ((rc = ctx->XH.ensure((size_t)t.n_pad * (DPh / 2 + 4) * sizeof(float) + 1024))) return rc;
  unsigned long long* st_d = (unsigned long long*)ctx->stats.p + 3;
  HIP_TRY(hipMemsetAsync(st_d, 0, 8, s));
  launch_prep_half_train(t.X64, t.mu, t.n, t.d, DPh, t.n_pad, t.jx,
                         (unsigned short*)ctx->XH.p, t.xinit_l2, st_d, swz, s, t.perm);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(ctx->h_stats + 3, st_d, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  double dx2;
  memcpy(&dx2, &ctx->h_stats[3], 8);
  // + the fp64 rounding of x - mu itself (<= 2^-53 relative per element)
  ctx->train.dxmax = std::sqrt(dx2) * (1.0 + 1e-12) + 0x1p-50 * std::sqrt(t.x2max);
  ctx->DPh = DPh;
  ctx->xh_swz = swz;
  return KNN_OK;
}

// The int8 image for kernel metrics 5 / 6 (knn_prep.hip): codes x 2^s - c of
// every row (16-B chunks swizzled as the fp16 image for metric 5, plain for
// metric 6) + the accumulator seeds -ceil(||k||^2 / 2); rows of DP + 16
// bytes, n_pad rows.
static int ensure_i8(knn_ctx* ctx, int kmetric, hipStream_t s) {
  const TrainDev& t = ctx->train;
  const int DPi = kmetric == 6 ? pad_dim_i8w(t.d) : pad_dim_i8(t.d);
  const int swz = kmetric == 6 ? 0 : 1;
  if (!ctx->i8_ok || DPi <= 0) return knn_fail(KNN_ERR_ARG, "train set not integer-coded (int8 pass)");
  if (ctx->DPi == DPi && ctx->i8_swz == swz) return KNN_OK;
  int rc;
  if ((rc = ctx->XI.ensure((size_t)t.n_pad * (DPi + 16) + 1024))) return rc;
  unsigned* cmax = (unsigned*)((unsigned long long*)ctx->stats.p + 3);
  HIP_TRY(hipMemsetAsync(cmax, 0, 8, s));
  launch_prep_i8_train(t.X64, (const double*)ctx->i8_cent.p, t.n, t.d, DPi, t.n_pad, ctx->i8_s,
                       (signed char*)ctx->XI.p, cmax, swz, s, t.perm);
  HIP_TRY(hipGetLastError());
  unsigned cm = 0;
  HIP_TRY(hipMemcpyAsync(&cm, cmax, sizeof cm, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  ctx->i8_x2max = std::ldexp((double)cm, -2 * ctx->i8_s);
  ctx->DPi = DPi;
  ctx->i8_swz = swz;
  return KNN_OK;
}

// The fp16 S3 image (d > 256, cand_s3_kernel<R, true>): 2^jx (x - mu) in
// fp16 tile-chunk images + the L2 seeds; the representation error measured
// as for the resident copy.
// AUTO for the query-resident fp16 kernel (d > 256; profiles/ab_log.md r6v)
constexpr bool kQresAuto = false;

static int ensure_fp16_s3(knn_ctx* ctx, hipStream_t s) {
  const TrainDev& t = ctx->train;
  const int DPs = pad_dim_fp16_s3(t.d);
  if (DPs <= 0) return knn_fail(KNN_ERR_ARG, "fp16 S3 path needs d > 256");
  if (ctx->DPs == DPs) return KNN_OK;
  int rc;
  const int64_t n3 = (t.n + kS3Rows - 1) / kS3Rows * kS3Rows;
  if ((rc = ctx->XT16.ensure((size_t)n3 * DPs * 2))) return rc;
  // (+1 KB: cand_qres_kernel stages a sub-tile's 32 seeds as one 1-KB piece)
  if ((rc = ctx->XS16.ensure((size_t)n3 * sizeof(float) + 1024))) return rc;
  unsigned long long* st_d = (unsigned long long*)ctx->stats.p + 3;
  HIP_TRY(hipMemsetAsync(st_d, 0, 8, s));
  launch_prep_half_tiled(t.X64, t.mu, t.n, t.d, DPs, n3, t.jx, 1.0, (unsigned short*)ctx->XT16.p,
                         t.xinit_l2, (float*)ctx->XS16.p, nullptr, st_d, s, t.perm);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(ctx->h_stats + 3, st_d, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  double dx2;
  memcpy(&dx2, &ctx->h_stats[3], 8);
  ctx->train.dxmax = std::sqrt(dx2) * (1.0 + 1e-12) + 0x1p-50 * std::sqrt(t.x2max);
  ctx->DPs = DPs;
  return KNN_OK;
}

// Seeded thresholds (resident fp16 / int8 kernels with the global threshold).
// Workgroups of the first grid round start with no published threshold: every
// lane inserts nearly every row of its first tiles (a 10K-query batch runs
// ~3 rounds, so a third of its workgroups).  A pre-pass runs the same kernel
// over a strided sample of the train rows (its own image, built once per
// train set: identical operands and seeds for those rows, hence identical
// proxies) and seeds every query's slots with the need-th smallest proxy of
// its sample lists (launch_seed_gthr).  Measured a net loss at cfg2, one
// setting per process (profiles/ab_log.md: r3o_*): int8 candidate phase 1.40-1.43
// ms off, 1.42-1.45 with 8192 rows, 1.44-1.46 with 16384, 1.53 with 32768;
// fp16 2.28 off vs 2.47 -- the sample pass runs cold itself (every lane
// inserts) and a sample-rank threshold saves little next to the thresholds
// the first round publishes within a tile or two.  Off by default; tuning
// key "seed": 0 / -1 off, N = sample rows (experiments).

static int64_t seed_rows(const knn_ctx* ctx) {
  // (the sample image takes train rows by stride: train order only)
  if (ctx->tune_seed <= 0 || ctx->ord_P || ctx->ord_nb) return 0;
  const int64_t ns = std::min<int64_t>(ctx->tune_seed, ctx->train.n / 8) / 256 * 256;
  return ns < 4096 ? 0 : ns;
}

static int ensure_sample(knn_ctx* ctx, int kmetric, int DP, int64_t ns, hipStream_t s) {
  const TrainDev& t = ctx->train;
  if (ctx->smp_kind == kmetric && ctx->smp_dp == DP && ctx->smp_n == ns &&
      (kmetric == 5 || ctx->smp_swz == ctx->xh_swz))
    return KNN_OK;
  const int d = t.d;
  const int64_t stride = t.n / ns;  // sample row i = train row i * stride
  const size_t row_bytes = kmetric == 5 ? (size_t)DP + 16 : (size_t)(DP / 2 + 4) * 4;
  int rc;
  if ((rc = ctx->smp_x64.ensure((size_t)ns * d * sizeof(double)))) return rc;
  if ((rc = ctx->smp_xl2.ensure((size_t)ns * sizeof(float)))) return rc;
  if ((rc = ctx->smp_img.ensure((size_t)ns * row_bytes + 1024))) return rc;
  if ((rc = ctx->smp_scr.ensure(16))) return rc;
  HIP_TRY(hipMemcpy2DAsync(ctx->smp_x64.p, (size_t)d * 8, t.X64, (size_t)stride * d * 8,
                           (size_t)d * 8, (size_t)ns, hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemsetAsync(ctx->smp_scr.p, 0, 16, s));
  if (kmetric == 5) {
    launch_prep_i8_train((const double*)ctx->smp_x64.p, (const double*)ctx->i8_cent.p, ns, d, DP, ns,
                         ctx->i8_s, (signed char*)ctx->smp_img.p, (unsigned*)ctx->smp_scr.p, 1, s);
  } else {
    // the fp16 image's seeds are the rows' fl32 ||x'||^2 of the main copy
    HIP_TRY(hipMemcpy2DAsync(ctx->smp_xl2.p, 4, t.xinit_l2, (size_t)stride * 4, 4, (size_t)ns,
                             hipMemcpyDeviceToDevice, s));
    launch_prep_half_train((const double*)ctx->smp_x64.p, t.mu, ns, d, DP, ns, t.jx,
                           (unsigned short*)ctx->smp_img.p, (const float*)ctx->smp_xl2.p,
                           (unsigned long long*)ctx->smp_scr.p, ctx->xh_swz, s);
  }
  HIP_TRY(hipGetLastError());
  ctx->smp_kind = kmetric;
  ctx->smp_dp = DP;
  ctx->smp_swz = ctx->xh_swz;
  ctx->smp_n = ns;
  return KNN_OK;
}

// fp16 candidate pass (kernel metric 4): PRECISION_FP16, or AUTO -- at
// d <= 256 for batches of >= 4096 queries (8-wave workgroups of the resident
// kernel), at d > 256 (S3 kernel) always -- until a batch certifies poorly.
// Tuning key "fp16": -1 auto, 0 off, 1 on.
// (W > kQuadMaxW: the R = 4 lists of the 16x16 layouts would overflow too
// often -- AUTO keeps those for the 32x32 bf16x3 kernel with R = 8/16 lists)
constexpr int kQuadMaxW = 64;
static bool use_fp16(const knn_ctx* ctx, int metric, int64_t m, int W) {
  if (metric != KNN_METRIC_L2) return false;
  const bool streamed = pad_dim_fp16_s3(ctx->train.d) > 0;
  if (!streamed && pad_dim_fp16(ctx->train.d) <= 0) return false;
  if (ctx->tune_fp16 >= 0) return ctx->tune_fp16 > 0;
  if (ctx->precision == KNN_PRECISION_FP16) return true;
  if (ctx->precision != KNN_PRECISION_AUTO || ctx->fp16_off) return false;
  return streamed || (m >= 4096 && W <= kQuadMaxW);
}

// int8 candidate pass (kernel metric 5): integer-coded train sets (detect_i8)
// at d <= 256 for batches of >= 4096 queries, in AUTO mode only, until a
// batch sends more than 1/16 of its queries to the rescan (queries off the
// train set's grid).  Tuning key "i8": -1 auto, 0 off, 1 on (where possible);
// "fp16" = 1 (an explicit fp16 request) turns it off, "fp16" = 0 does not.
static bool use_i8(const knn_ctx* ctx, int metric, int64_t m, int W) {
  if (metric != KNN_METRIC_L2 || !ctx->i8_ok || pad_dim_i8(ctx->train.d) <= 0) return false;
  if (ctx->tune_i8 >= 0) return ctx->tune_i8 > 0;
  if (ctx->tune_fp16 == 1) return false;
  if (ctx->precision != KNN_PRECISION_AUTO || ctx->i8_off) return false;
  return m >= 4096 && W <= kQuadMaxW;
}

static bool use_bf16x3(const knn_ctx* ctx, int metric) {
  if (metric != KNN_METRIC_L2) return false;
  if (ctx->precision == KNN_PRECISION_FP32) return false;
  return pad_dim_bf16x3(ctx->train.d) > 0;  // AUTO and BF16X3 (where supported)
}

static int check_train_args(int64_t n, int d, int class_cnt) {
  if (n <= 0) return knn_fail(KNN_ERR_ARG, "n_train must be > 0");
  if (n >= (int64_t)INT32_MAX - 4096)
    return knn_fail(KNN_ERR_ARG, "n_train per context must be < 2^31 (shard the train set)");
  if (d <= 0) return knn_fail(KNN_ERR_ARG, "dim must be > 0");
  if (class_cnt <= 0) return knn_fail(KNN_ERR_ARG, "class_cnt must be > 0");
  return KNN_OK;
}

extern "C" {

int knn_set_train(knn_ctx* ctx, const double* X, const int32_t* labels, int64_t n, int32_t d,
                  int32_t class_cnt) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if ((rc = check_train_args(n, d, class_cnt))) return rc;
  if (!X || !labels) return knn_fail(KNN_ERR_ARG, "null train pointer");
  // label range check (the reference indexes label_cnt[label] unchecked, cpp:330)
  for (int64_t i = 0; i < n; i++)
    if (labels[i] < 0 || labels[i] >= class_cnt)
      return knn_fail(KNN_ERR_ARG, "train label out of [0, class_cnt) at row " + std::to_string(i));
  if ((rc = ctx->X64_own.ensure((size_t)n * d * sizeof(double)))) return rc;
  if ((rc = ctx->lab_own.ensure((size_t)n * sizeof(int32_t)))) return rc;
  HIP_TRY(hipMemcpyAsync(ctx->X64_own.p, X, (size_t)n * d * sizeof(double),
                         hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipMemcpyAsync(ctx->lab_own.p, labels, (size_t)n * sizeof(int32_t),
                         hipMemcpyHostToDevice, ctx->stream));
  return build_train(ctx, (const double*)ctx->X64_own.p, (const int32_t*)ctx->lab_own.p, n, d,
                     class_cnt, 0);
}

int knn_set_train_device(knn_ctx* ctx, const double* dX, const int32_t* dlabels, int64_t n,
                         int32_t d, int32_t class_cnt, int64_t idx_offset) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if ((rc = check_train_args(n, d, class_cnt))) return rc;
  if (!dX || !dlabels) return knn_fail(KNN_ERR_ARG, "null train pointer");
  return build_train(ctx, dX, dlabels, n, d, class_cnt, idx_offset);
}

}  // extern "C"

// Work decomposition of the candidate kernel: S train splits per 128-query
// tile, R list entries per lane.  The grid (n_qt * S workgroups) is sized so
// its last wave of workgroups is nearly full on the resident slots of this
// kernel (occupancy x CUs): a mostly-empty final round costs up to a whole
// workgroup duration.  The union of the 2S lists must hold the C re-rank
// candidates; R grows to 16 when the expected per-list share of C is large.
static void choose_geometry(knn_ctx* ctx, int metric, bool streamed, int DP, int nw, int n_qt,
                            int64_t n_tiles, int W, int C, bool s3q, int& S_out, int& R_out) {
  int S_hi = (int)std::max<int64_t>(1, std::min<int64_t>(64, n_tiles));
  int bestS = 1, bestR = 8;
  const bool quad = !streamed && metric >= 3 && metric <= 5;  // 16x16 layouts (bf16x3, fp16, int8)
  // int8 on 32x32x32: 4 lists of R = 4 per split (two per lane), or 2 of R =
  // 8 (one per lane, tuning "R" = 8)
  const bool pair4 = metric == 6;
  const bool w4 = pair4 && ctx->tune_R != 8;
  const int lps = quad || s3q || w4 ? 4 : 2;  // lists per query per split
  // S3 on 16x16x32 (s3q): R = 8 quad lists, 4 * S * 8 <= kMaxUnion entries
  if (s3q) S_hi = std::min(S_hi, kMaxUnion / (4 * 8));
  for (int R : {4, 8, 16}) {
    if (s3q && R != 8) continue;
    // kernel metrics 3, 4 (16x16x32 layout) have R = 4 only; elsewhere R = 4
    // only on request (resident kernel; tuning experiments)
    // (int8: R = 8 quad lists on request, tuning key "R")
    const bool q8 = quad && metric == 5 && ctx->tune_R == 8;
    if (pair4 ? R != (w4 ? 4 : 8) : quad ? R != (q8 ? 8 : 4)
              : (ctx->tune_R ? R != ctx->tune_R : R == 4))
      continue;
    if (R == 4 && (DP > 256 || metric == 1)) continue;
    const int64_t slots =
        (int64_t)(s3q ? s3q_blocks_per_cu() : cand_blocks_per_cu(metric, DP, R, nw)) * ctx->cu_count;
    // the union of the lists must hold the C re-rank candidates; with R = 4
    // lists (16x16 layouts) also S >= W, i.e. at most W/4S of the query's
    // top W expected per list: a list holding 5 of them (an overflow ->
    // the query fails certification) then has probability ~C(W,5)/(4S)^5
    int S_lo = std::max(1, (C + lps * R - 1) / (lps * R));
    // quad lists: S >= 2W where every split still walks >= 32 tiles (a list
    // then expects at most 1/8 of the query's top W; an overflow, 5 of them in
    // one list, fails the query's certification: 0.35 % of cfg3's 1M queries
    // at S = W, 0.05 % at 2W, 0.007 % at 4W, each an exact rescan); 4W for
    // batches of >= 128K queries, whose many workgroup rounds make the longer
    // walks of fewer splits worth nothing (cfg3: candidate +0.8 %, rescan
    // phase 11.9 -> 1.8 ms); at least S >= W
    if (q8) {
      S_lo = std::max(S_lo, W);  // an 8-entry list holding 8 of the top W: negligible
      S_hi = std::min(S_hi, kMaxUnion / (4 * 8));
    } else if (quad || pair4) {
      const int mult = n_qt >= 512 ? 4 : 2;
      S_lo = std::max(S_lo, std::max<int>(W, (int)std::min<int64_t>(mult * W, n_tiles / 32)));
    }
    // R = 8 needs an expected share of the top W per list (2S lists) of at
    // most 0.8 (S >= W / 1.6): a list overflow (9 of them in one list -> the
    // query fails certification) then has probability < 1e-6 per list; at a
    // share of 1.6 (cfg5, W = 101, S = 32) 1.6 % of the queries failed.
    // Where no such S exists R = 16 runs instead.
    if (R == 8 && !ctx->tune_R) {
      const int s8 = s3q ? (W * 5 + 15) / 16 : (W * 5 + 7) / 8;  // share W / (lps S) <= 0.8
      if (s8 > S_hi) continue;
      S_lo = std::max(S_lo, s8);
    }
    S_lo = std::min(S_hi, S_lo);
    auto eff_of = [&](int S) {
      const int64_t wg = (int64_t)n_qt * S;
      const int64_t rounds = (wg + slots - 1) / slots;
      return (double)wg / (double)(rounds * slots);
    };
    double best = -1.0;
    for (int S = S_lo; S <= S_hi; S++) best = std::max(best, eff_of(S));
    // smallest S within 2 % of the best fill: fewer, longer lists mean fewer
    // list insertions per tile (the early, insertion-heavy part of each
    // list's stream is paid once per list)
    int bS = S_lo;
    for (int S = S_lo; S <= S_hi; S++)
      if (eff_of(S) >= best - 0.02) { bS = S; break; }
    // S3: prefer a split count that lets the XCD's concurrent workgroups
    // share staged chunks (s3_map; gq 4 over 2 over none) within the same fill
    if (streamed && DP > 256) {
      const int gmax = ctx->tune_s3gq > 0 ? ctx->tune_s3gq : kS3GqMax;
      int bq = s3_group(n_qt, bS, gmax);
      for (int S = bS + 1; S <= S_hi && bq < gmax; S++)
        if (eff_of(S) >= best - 0.02 && s3_group(n_qt, S, gmax) > bq) { bS = S; bq = s3_group(n_qt, S, gmax); }
    }
    if (ctx->tune_S) bS = std::min(ctx->tune_S, S_hi);
    bestS = bS;
    bestR = R;
    break;
  }
  S_out = bestS;
  R_out = bestR;
}

// Relative factor f of the candidate-pass error bound used by the
// certification: |proxy - exact| <= f * (max||x||^2 +
// 2.1 ||q|| max||x||) for L2, f * (||q||_1 + max||x||_1) for L1.
//   kmetric 0 (fp32 MFMA, an fmaf chain of DP+1 terms): gamma_{DP+1} + 5u
//   kmetric 1 (fp32 VALU L1):                           gamma_DP + 3u
//   kmetric 2 (bf16x3): products exact, accumulation of 3DP+1 terms bounded
//     with u' = 2^-23 (covers truncating adders), + 2^-15 for the hi/lo
//     representation error (~3 * 2^-18 relative per product, x2 for -2q).
//   kmetric 4 (fp16): products of the fp16 operands exact in fp32, DP+1
//     accumulated terms with u' = 2^-23.  The operands' representation
//     error is measured (train: TrainDev::dxmax, queries: by the merge from
//     the operands themselves) and added by the merge with the seed's own
//     rounding and the fp16 subnormal-range terms.
static double err_factor(int kmetric, int DP) {
  const double u = std::ldexp(1.0, -24);
  if (kmetric == 4) {
    const double u2 = std::ldexp(1.0, -23);
    const int n = DP + 1;
    return n * u2 / (1.0 - n * u2) * 1.02;
  }
  if (kmetric == 2 || kmetric == 3) {  // bf16x3 on either MFMA shape
    const double u2 = std::ldexp(1.0, -23);
    const int n = 3 * DP + 1;
    return (n * u2 / (1.0 - n * u2) + std::ldexp(1.0, -15)) * 1.02;
  }
  const int n = kmetric == 0 ? DP + 1 : DP;
  const double gam = n * u / (1.0 - n * u);
  return (gam + (kmetric == 0 ? 5.0 : 3.0) * u) * 1.01;
}

// ---- timing ring (knn_set_timing): events of a call are read back lazily
// (mode 2: only ev[1] and ev[2], around the candidate kernel, are recorded)
static bool phase_timed(const TimedCall& tc, int p) { return tc.mode != 2 || p == 1; }
static void fold_timing(knn_ctx* ctx, TimedCall& tc) {
  if (!tc.pending) return;
  (void)hipEventSynchronize(tc.ev[tc.mode == 2 ? 2 : 4]);
  for (int p = 0; p < 4; p++) {
    float ms = 0.f;
    if (phase_timed(tc, p) && hipEventElapsedTime(&ms, tc.ev[p], tc.ev[p + 1]) == hipSuccess)
      ctx->tsum[p] += ms;
  }
  ctx->tcalls++;
  tc.pending = false;
}

static TimedCall* timing_slot(knn_ctx* ctx) {
  if (!ctx->timing) return nullptr;
  TimedCall& tc = ctx->ring[ctx->ring_next];
  fold_timing(ctx, tc);  // waits only when kTimingRing calls are still in flight
  ctx->ring_last = ctx->ring_next;
  ctx->ring_next = (ctx->ring_next + 1) % kTimingRing;
  tc.pending = true;
  tc.mode = ctx->timing;
  return &tc;
}
// the call's event e, if its timing mode records it
static hipEvent_t timing_ev(const TimedCall* tc, int e) {
  if (!tc || (tc->mode == 2 && e != 1 && e != 2)) return nullptr;
  return tc->ev[e];
}

// The deferred AUTO decision: once the last fp16 call has completed, its
// rescan count (written by the device into h_counts) decides whether the
// fp16 pass stays on for this train set.  Never waits.
static void auto_check(knn_ctx* ctx) {
  if (!ctx->auto_pending || hipEventQuery(ctx->done_ev) != hipSuccess) return;
  // AUTO retires the fp16 pass for this train set when a batch leaves more
  // than 1/16 of its queries to the rescan (data whose neighbour gaps are
  // too fine for fp16 operands): later batches take bf16x3
  if ((int64_t)ctx->h_counts[0] * 16 > ctx->auto_m) {
    if (ctx->auto_kind >= 5) ctx->i8_off = true;
    else ctx->fp16_off = true;
  }
  ctx->auto_pending = false;
}

// Core search: candidate pass + merge/re-rank/certify + the device-driven
// rescan.  Enqueue only: no host synchronisation on any path.
// Reference tie order (knn_select.hip, tie_order_kernel): which tied queries
// get the reference's own std::sort order.  Tuning key "ties": 0 none,
// 1 (default) those whose label the tie order could change (equal distances
// with different labels where two classes share the top count, or a tie
// across the k-th place within reach of the runner-up: finish_single),
// 2 every query with equal distances in its top k (neighbour indices in the
// reference's order too).
// (Partial lists stay ordered by (dist, global idx): the reference's order
// over the whole train set is restored after the merge, knn_tie_resolve_device.)
static int tie_mask_of(const knn_ctx* ctx, const Sink& sink) {
  if (sink.mode != MODE_SINGLE) return 0;
  return ctx->tune_ties;
}

// Scratch of the reference-order passes: tie_scratch_bytes per concurrent
// workgroup, at most 32 workgroups and ~512 MB (at least one: n * 20 B); the
// passes loop over their queued queries, which are rare.
static int tie_workgroups(const knn_ctx* ctx, int64_t per) {
  return (int)std::max<int64_t>(
      1, std::min<int64_t>({(int64_t)32, (int64_t)ctx->cu_count, (512ll << 20) / per}));
}

int knn_run_search(knn_ctx* ctx, const double* dQ, int64_t m, int W, int metric,
                   const Sink& sink_in, hipStream_t s) {
  const TrainDev& t = ctx->train;
  int rc;
  auto_check(ctx);
  Sink sink = sink_in;
  sink.tie_mode = tie_mask_of(ctx, sink_in);
  int64_t tie_per = 0;
  int tie_nwg = 0;
  if (sink.tie_mode) {
    // scratch for the reference-order pass: every row's distance per
    // workgroup (tied queries are rare; the pass loops over them)
    tie_per = tie_scratch_bytes(t.n, ctx->class_cnt);
    tie_nwg = tie_workgroups(ctx, tie_per);
    if ((rc = ctx->tie_q.ensure((size_t)m * sizeof(int) + 16))) return rc;
    if ((rc = ctx->tie_ws.ensure((size_t)(tie_per * tie_nwg)))) return rc;
    sink.tie_q = (int*)ctx->tie_q.p;
  }
  // candidate-pass flavour: kmetric 4 = L2 via fp16 MFMA, 2/3 = bf16x3, else fp32
  int kmetric = metric, DP = t.DP;
  const float* Xk = t.X32;
  bool s3h = false;  // fp16 on the S3 stream kernel (d > 256)
  if (use_i8(ctx, metric, m, W)) {
    kmetric = i8_kernel(ctx);
    if ((rc = ensure_i8(ctx, kmetric, s))) return rc;
    DP = ctx->DPi;
    Xk = (const float*)ctx->XI.p;
  } else if (use_fp16(ctx, metric, m, W)) {
    kmetric = 4;
    if (pad_dim_fp16(t.d) > 0) {
      if ((rc = ensure_fp16(ctx, s))) return rc;
      DP = ctx->DPh;
      Xk = (const float*)ctx->XH.p;
    } else {
      if ((rc = ensure_fp16_s3(ctx, s))) return rc;
      DP = ctx->DPs;
      s3h = true;
    }
  } else if (use_bf16x3(ctx, metric)) {
    if ((rc = ensure_bf16x3(ctx, s))) return rc;
    kmetric = 2;
    DP = ctx->DPb;
    Xk = (const float*)ctx->XB.p;
  }
  // waves per workgroup of the resident kernel: 8 (256 queries share each
  // staged tile) when there are enough queries, else 4; the large-d fp32
  // stream kernel always takes 128 queries, the bf16x3 one (S3) 256
  const bool s3 = (kmetric == 2 && bf16x3_streamed(DP)) || s3h;
  // bf16x3 on the 16x16x32 MFMA layout (resident kernel, 8 waves, DP % 32 ==
  // 0): kernel metric 3, R = 4 lists, 4 lists per split.  Tuning key
  // "mfma16": -1 auto (on for batches of >= 4096 queries), 0 off, 1 on.
  const bool m16 = ctx->tune_m16 < 0 ? m >= 4096 && W <= kQuadMaxW : ctx->tune_m16 > 0;
  if (kmetric == 2 && !s3 && m16 && DP % 32 == 0) kmetric = 3;
  int nw = 4;
  if (DP <= 256 && kmetric != 1) nw = ctx->tune_nw ? std::min(ctx->tune_nw, 8) : (m >= 4096 ? 8 : 4);
  if (kmetric >= 3) nw = 8;  // (the 16x16 layouts: fp16, bf16x3, int8)
  if (kmetric == 4 && !s3 && ctx->tune_nw) nw = ctx->tune_nw;  // 4, 8 or 16
  // int8 32x32x32: 16 waves (512 queries per staged tile) only in builds
  // with KNN_I8W_NW16 (otherwise the launch is refused: no such kernel)
  if (kmetric == 6 && ctx->tune_nw == 16) nw = 16;
  // queries per wave of the resident kernel (int8: 16 x the build's query
  // blocks); the int8 kernel with 64 queries per wave also runs 4 waves
  const int qpw = !s3 && DP <= 256 ? cand_queries_per_wave(kmetric, DP) : 32;
  if (kmetric == 5 && ctx->tune_nw) nw = ctx->tune_nw;  // 4 or 8 (16x16x64 builds have both)
  if (s3) nw = 8;
  const int qpb = s3 ? kS3Rows : (DP <= 256 ? qpw * nw : kQPB);
  const int n_qt = (int)((m + qpb - 1) / qpb);
  const int64_t m_pad = (int64_t)n_qt * qpb;
  const int64_t n_pad3 = (t.n + kS3Rows - 1) / kS3Rows * kS3Rows;
  const int64_t trows = cand_tile_rows(kmetric, DP);  // rows per tile of the launched kernel
  const int64_t n_tiles = s3 ? n_pad3 / kS3Rows : t.n_pad / trows;
  int C = (int)std::min<int64_t>(t.n, std::max(2 * W, W + 16));
  C = std::min(C, kMaxUnion);
  int S = 1, R = 8;
  // fp16 S3 on v_mfma_f32_16x16x32_f16 (quad lists of R = 8) where its lists
  // can hold the query's top W (share W / 4S <= 0.8 at S <= 32, i.e. W <= 102)
  // and the train set has that many tiles to split (else the 32x32x16 form,
  // whose R = 16 lists need fewer splits); tuning key "s3q": -1 auto, 0 off
  // (32x32x16), 1 on where feasible
  const int s3q_S = (W * 5 + 15) / 16;
  const bool s3q = s3h && ctx->tune_s3q != 0 && s3q_S <= kMaxUnion / 32 && s3q_S <= n_tiles;
  choose_geometry(ctx, kmetric, s3, DP, nw, n_qt, n_tiles, W, C, s3q, S, R);
  // the query-resident kernel in place of S3's q16 form (same images, lists
  // and thresholds; knn_cand_qres.hip); tuning key "qres": -1 auto (kQresAuto),
  // 0 off, 1 on where supported
  const bool qres = s3q && qres_supported(DP) && (ctx->tune_qres < 0 ? kQresAuto : ctx->tune_qres > 0);
  // metric 6: 4 lists of R = 4 per query per split (two per lane, one per
  // half of its rows: knn_cand_res.hip, KNN_I8W_Q4), the quad layout of the
  // 16x16 kernels; tuning "R" = 8 selects one list of 8 per lane (2 per
  // query per split, round 4's form)
  const bool w4 = kmetric == 6 && ctx->tune_R != 8;
  if (kmetric == 6) R = w4 ? 4 : 8;
  // 16x16 layouts (and w4): 4 lists per query per split
  const bool quad_lists = (!s3 && kmetric >= 3 && kmetric <= 5) || s3q || w4;
  if (quad_lists && !s3q && !(kmetric == 5 && R == 8)) R = 4;
  const int NL = (quad_lists ? 4 : 2) * S;
  C = std::min(C, NL * R);
  // rescan workspace: the fast path serves the first `cap` failed queries
  const int cap = (int)std::min<int64_t>(m, kRescanFastQueries);
  if ((rc = ctx->Q32.ensure((size_t)m_pad * DP * sizeof(float)))) return rc;
  if ((rc = ctx->qvalid.ensure((size_t)m_pad * sizeof(float)))) return rc;
  if ((rc = ctx->cand_v.ensure((size_t)m_pad * NL * R * sizeof(float)))) return rc;
  if ((rc = ctx->cand_i.ensure((size_t)m_pad * NL * R * sizeof(int)))) return rc;
  // per-query global thresholds of the resident candidate kernel
  // (tuning switch "ablate" bit 2 turns the exchange off; results stay exact)
  // gk: what the lists publish into gthr (cand_kernel, cand_s3_kernel's q16
  // form): the K-th smallest of the union of a query's lists in a workgroup,
  // 8 groups, with 8K >= W + 5 rows guaranteed below the threshold (K <= 4
  // for the resident kernel's 4-entry lists, so W <= 27; K <= 16 in S3,
  // W <= 123); else, in the resident kernel, the lists' R-th entries in 4
  // groups.  cfg2 (W = 11): K = 2, the candidate pass 3 % faster than K = 3
  // and 2-4 % faster than the list thresholds (in-process A/B,
  // profiles/ab_log.md: r2f_ab_gk, r2g_ab_pair); K = 1 (8 rows < W) sends 5 %
  // of the queries to the rescan.
  // slot groups G (resident kernel): the first grid round of a 10k batch
  // runs only ~6 of the 38 splits of each query tile, so with 8 groups group
  // 7 has published nothing until the second round and tq = max over the
  // slots stays +inf there; with 4 groups (K = (W + 5) / 4, the same G K >=
  // W + 5 rows below tq) every group has a split in round 1: cfg2 candidate
  // -0.5..0.9 %, the 12.5M x 96 shard -0.5 % (profiles/ab_log.md r5n).  Auto:
  // 4 where K stays <= 4 (W <= 11), else 8; tuning "gg" 4 / 8 forces.
  const int G = s3 ? kGthrSlots
                   : ctx->tune_gg > 0 ? ctx->tune_gg : ((W + 5 + 3) / 4 <= 4 ? 4 : kGthrSlots);
  int gk = (W + 5 + G - 1) / G;
  if (gk > (s3 ? 16 : 4)) gk = 0;
  if (ctx->tune_gk >= 0) gk = std::min(ctx->tune_gk, s3 ? 16 : 4);
  const bool use_gthr = (s3 ? s3q && gk > 0 : DP <= 256) && !(ctx->tune_ablate & 4);
  if (use_gthr && (rc = ctx->gthr.ensure((size_t)m_pad * kGthrSlots * sizeof(uint32_t))))
    return rc;
  if ((rc = ctx->rescan_q.ensure((size_t)m * sizeof(int) + 16))) return rc;
  if ((rc = ctx->rescan_tau.ensure((size_t)m * sizeof(double) + 16))) return rc;
  if ((rc = ctx->rescan_cnt.ensure(4 * sizeof(int)))) return rc;
  sink.tie_cnt = (int*)ctx->rescan_cnt.p + 2;  // zeroed with the rescan counts
  if ((rc = ctx->fr_cnt.ensure((size_t)cap * sizeof(int) + 16))) return rc;
  if ((rc = ctx->fr_buf.ensure((size_t)cap * kRescanCap * sizeof(int) + 16))) return rc;
  if ((rc = ctx->fr_q.ensure((size_t)cap * t.DP * sizeof(float) + 16))) return rc;
  if ((rc = ctx->fr_thr.ensure((size_t)cap * sizeof(float) + 16))) return rc;
  if ((rc = ctx->slow_q.ensure((size_t)m * sizeof(int) + 16))) return rc;
  if ((rc = ctx->rescan_mask.ensure((size_t)m * sizeof(unsigned long long) + 16))) return rc;
  if ((rc = ctx->rescan_nkeep.ensure((size_t)cap * sizeof(int) + 16))) return rc;

  ctx->last_kmetric = kmetric;
  ctx->geom[0] = (int64_t)(qres ? 2 * n_qt : n_qt) * S;  // (qres: workgroup tiles of 128 queries)
  ctx->geom[1] = S;
  ctx->geom[2] = R;
  ctx->last_nw = nw;
  ctx->geom[3] = C;
  if (qres)
    snprintf(ctx->last_kernel, sizeof ctx->last_kernel, "cand_qres_kernel<%d>", DP / 32);
  else if (s3)
    snprintf(ctx->last_kernel, sizeof ctx->last_kernel, "cand_s3_kernel<%d,%s,%s>", R,
             s3h ? "true" : "false", s3q ? "true" : "false");
  else if (DP <= 256)
    snprintf(ctx->last_kernel, sizeof ctx->last_kernel, "cand_kernel<%d,%d,%d,%d>", DP, R, kmetric,
             nw);
  else
    snprintf(ctx->last_kernel, sizeof ctx->last_kernel, "cand_stream_kernel<%d,%d,%d>", kStreamDC,
             R, kmetric);
  TimedCall* tc = timing_slot(ctx);
  if (hipEvent_t ev = timing_ev(tc, 0)) HIP_TRY(hipEventRecord(ev, s));
  // query operands: scale * 2^jx (q - mu), scale -2 for L2; a query whose
  // operands would leave the format's range (fp16: 65000, else 2^100) is
  // marked void and goes to the exact rescan
  const double qscale = metric == KNN_METRIC_L2 ? -2.0 : 1.0;
  float* qvalid = (float*)ctx->qvalid.p;
  // region order of the queries (resident kernels, metrics 4-6; knn_order.hip):
  // operand row p = query qperm[p], sorted by region; each query tile's
  // workgroups start their streams at the tile's region (qstart), and the
  // merge finds query q's lists at qpos[q]
  const int* qperm = nullptr;
  const int* qpos = nullptr;
  const int* qstart = nullptr;
  int64_t bcnt_clear = 0;  // block counts the int8 query builder clears after the sort
  if (ctx->ord_P > 0 && ctx->tune_order != 0 && !s3 && kmetric >= 4 && DP <= 256) {
    const int64_t nbc = region_sort_blocks(m) * kRegionMax;
    if ((rc = ctx->ord_qkey.ensure((size_t)m * sizeof(int)))) return rc;
    const size_t bcnt_cap = ctx->ord_bcnt.cap;
    if ((rc = ctx->ord_bcnt.ensure((size_t)nbc * sizeof(int)))) return rc;
    if (ctx->ord_bcnt.cap != bcnt_cap) ctx->ord_bcnt_zero = 0;  // (a new allocation)
    if ((rc = ctx->ord_qperm.ensure((size_t)m * sizeof(int)))) return rc;
    if ((rc = ctx->ord_qpos.ensure((size_t)m * sizeof(int)))) return rc;
    if ((rc = ctx->ord_qstart.ensure((size_t)m * sizeof(int)))) return rc;
    launch_region_sort_queries(dQ, t.mu, m, t.d, t.jx, (const unsigned short*)ctx->ord_img.p,
                               (const float*)ctx->ord_cnorm.p, ctx->ord_P,
                               (const int*)ctx->ord_rank.p, (const int*)ctx->ord_rstart.p,
                               std::min(ctx->tune_ophase < 0 ? kOrderPhases : ctx->tune_ophase, ctx->ord_P),
                               (int*)ctx->ord_bcnt.p,
                               (int*)ctx->ord_tot.p, (int*)ctx->ord_qkey.p, (int*)ctx->ord_qperm.p,
                               (int*)ctx->ord_qpos.p, (int*)ctx->ord_qstart.p, s,
                               ctx->ord_bcnt_zero >= nbc);
    ctx->ord_bcnt_zero = 0;
    if (kmetric >= 5) bcnt_clear = nbc;
    qperm = (const int*)ctx->ord_qperm.p;
    qpos = (const int*)ctx->ord_qpos.p;
    qstart = (const int*)ctx->ord_qstart.p;
  }
  // gthr init (slots of groups without a split stay 0, never the max); the
  // int8 query builder writes it with the operands (ablate bit 5, an
  // experiment: keep the previous call's final thresholds -- valid only for
  // a repeat of the same queries; measures what perfect seeds would save)
  const bool gthr_init = use_gthr && !(ctx->tune_ablate & 32);
  const int active = std::min(S, gk ? G : 4);
  if (kmetric < 5)
    launch_query_check(dQ, t.mu, m, t.d, m_pad, qscale, t.jx,
                       kmetric == 4 ? 65000.0 : std::ldexp(1.0, 100), qvalid, s);
  if (kmetric >= 5) {  // codes of the train set's grid; a query off it: valid 0 (rescan)
    launch_prep_i8_queries(dQ, t.mu, qscale, t.jx, DBL_MAX, (const double*)ctx->i8_cent.p, m, t.d,
                           DP, m_pad, ctx->i8_s, (signed char*)ctx->Q32.p, qvalid, s, qperm,
                           gthr_init ? (uint32_t*)ctx->gthr.p : nullptr, active,
                           (int*)ctx->ord_bcnt.p, bcnt_clear, (int*)ctx->rescan_cnt.p);
    if (bcnt_clear) ctx->ord_bcnt_zero = bcnt_clear;
  } else if (s3h)
    launch_prep_half_tiled(dQ, t.mu, m, t.d, DP, m_pad, t.jx, -2.0, (unsigned short*)ctx->Q32.p,
                           nullptr, nullptr, qvalid, nullptr, s);
  else if (s3)
    launch_prep_split_tiled(dQ, t.mu, m, t.d, DP, m_pad, std::ldexp(qscale, t.jx),
                            (unsigned short*)ctx->Q32.p, nullptr, nullptr, s);
  else if (kmetric == 4)
    launch_prep_half_queries(dQ, t.mu, m, t.d, DP, m_pad, t.jx, (unsigned short*)ctx->Q32.p,
                             qvalid, s, qperm);
  else if (kmetric == 2 || kmetric == 3)
    launch_prep_split(dQ, t.mu, m, t.d, DP, m_pad, std::ldexp(qscale, t.jx),
                      (unsigned short*)ctx->Q32.p, 2 * DP, nullptr, nullptr, s);
  else
    launch_prep_queries(dQ, t.mu, m, t.d, DP, m_pad, qscale, t.jx, (float*)ctx->Q32.p, s);
  // launch_cand records the "cand" events with the kernel's own dispatch
  // (hipExtLaunchKernelGGL), so that phase is the kernel alone (the seed pass
  // and threshold fill fall into "prep"); the streamed kernels get separate
  // event records around them
  const bool ev_ext = (!s3 || qres) && timing_ev(tc, 1) && timing_ev(tc, 2);
  if (hipEvent_t ev = timing_ev(tc, 1); ev && !ev_ext) HIP_TRY(hipEventRecord(ev, s));
  CandLaunch cl{};
  if (ev_ext) {
    cl.ev_start = timing_ev(tc, 1);
    cl.ev_stop = timing_ev(tc, 2);
  }
  cl.metric = kmetric;
  cl.DP = DP;
  cl.R = R;
  cl.S = S;
  cl.n_qt = n_qt;
  cl.n_pad = t.n_pad;
  cl.X32 = Xk;
  cl.xinit = metric == 0 ? t.xinit_l2 : t.xinit_l1;
  cl.Q32 = (const float*)ctx->Q32.p;
  cl.out_v = (float*)ctx->cand_v.p;
  cl.out_i = (int*)ctx->cand_i.p;
  cl.ablate = ctx->tune_ablate;
  cl.nw = nw;
  cl.qpb = qpb;
  cl.gthr = use_gthr ? (uint32_t*)ctx->gthr.p : nullptr;
  cl.gk = gk;
  cl.xsw = kmetric >= 5 ? ctx->i8_swz : ctx->xh_swz;
  cl.qstart = qstart;
  cl.gmask = gk ? G - 1 : 3;
  cl.qblk = ctx->tune_qblk > 0 ? std::min(ctx->tune_qblk, n_qt) : 0;
  if (gthr_init) {
    const int64_t ns = (kmetric == 4 || kmetric == 5) && !s3 ? seed_rows(ctx) : 0;
    bool seeded = false;
    if (ns > 0) {
      // seeded thresholds (see seed_rows): the pre-pass over the sample
      if ((rc = ensure_sample(ctx, kmetric, DP, ns, s))) return rc;
      const int Ss = (int)std::max<int64_t>(1, std::min<int64_t>(16, ns / trows / 4));
      const int Us = 4 * Ss * R;  // quad lists: 4 per query per split
      if ((rc = ctx->smp_v.ensure((size_t)m_pad * Us * sizeof(float)))) return rc;
      if ((rc = ctx->smp_i.ensure((size_t)m_pad * Us * sizeof(int)))) return rc;
      CandLaunch cs = cl;
      cs.X32 = (const float*)ctx->smp_img.p;
      cs.n_pad = ns;
      cs.S = Ss;
      cs.out_v = (float*)ctx->smp_v.p;
      cs.out_i = (int*)ctx->smp_i.p;
      cs.gthr = nullptr;
      cs.ablate = 0;
      cs.ev_start = cs.ev_stop = nullptr;
      if (launch_cand(cs, s)) {
        launch_seed_gthr((const float*)ctx->smp_v.p, m_pad, Us, gk ? G * gk : 4 * R, active,
                         cl.gthr, s);
        seeded = true;
      }
    }
    if (!seeded && kmetric < 5) launch_fill_gthr(cl.gthr, m_pad, active, s);
  }
  if (qres) {
    if (!launch_cand_qres((const unsigned short*)ctx->XT16.p, (const float*)ctx->XS16.p,
                          (const unsigned short*)ctx->Q32.p, DP, n_pad3, S, n_qt, cl.out_v, cl.out_i,
                          cl.gthr, gk, s, cl.ev_start, cl.ev_stop))
      return knn_fail(KNN_ERR_ARG, "no query-resident kernel for this dimension");
  } else if (s3h)
    launch_cand_s3h((const unsigned short*)ctx->XT16.p, (const float*)ctx->XS16.p,
                    (const unsigned short*)ctx->Q32.p, DP, n_pad3, R, S, n_qt, cl.out_v, cl.out_i,
                    cl.ablate, s3q, cl.gthr, gk, s, ctx->tune_s3gq > 0 ? ctx->tune_s3gq : kS3GqMax);
  else if (s3)
    launch_cand_s3((const unsigned short*)ctx->XB.p, (const float*)ctx->XS.p,
                   (const unsigned short*)ctx->Q32.p, DP, n_pad3, R, S, n_qt, cl.out_v, cl.out_i,
                   cl.ablate, s, ctx->tune_s3gq > 0 ? ctx->tune_s3gq : kS3GqMax);
  else if (!launch_cand(cl, s))
    return knn_fail(KNN_ERR_ARG, "no candidate kernel for this geometry (tuning overrides?)");
  HIP_TRY(hipGetLastError());
  if (hipEvent_t ev = timing_ev(tc, 2); ev && !ev_ext) HIP_TRY(hipEventRecord(ev, s));
  // the rescan / tie counters (the int8 query builder cleared them already)
  if (kmetric < 5) HIP_TRY(hipMemsetAsync(ctx->rescan_cnt.p, 0, 4 * sizeof(int), s));
  // per-split certification: a query failing only through some splits'
  // lists rescans just those splits' rows (knn_select.hip)
  SplitMap sm;
  sm.S = S <= 64 ? S : 0;
  sm.lps = quad_lists ? 4 : 2;
  sm.trows = trows;
  sm.cap = cap;
  sm.mask = (unsigned long long*)ctx->rescan_mask.p;
  sm.nkeep = (int*)ctx->rescan_nkeep.p;
  sm.keep = (int*)ctx->fr_buf.p;
  // the fast rescan's per-query setup, run by the merge on the queries it
  // fails (timing-only ablations leave every query uncertified: none then)
  const bool abl = ctx->tune_ablate & 27;
  RescanPrep rp;
  rp.mu = t.mu;
  rp.x2max = t.x2max;
  rp.x1max = t.x1max;
  rp.jx = t.jx;
  rp.DP = t.DP;
  rp.f_err = err_factor(metric, t.DP);
  rp.qf = (float*)ctx->fr_q.p;
  rp.thr = (float*)ctx->fr_thr.p;
  rp.fcnt = (int*)ctx->fr_cnt.p;
  rp.cap = abl ? 0 : cap;
  // the int8 rescan filter (metric 6's plain image; knn_select.hip)
  // (tuning key "i8resc": -1 / 1 auto, 0 every failed query on the fp32 filter)
  const bool i8resc = ctx->tune_i8resc != 0 && kmetric == 6 && ctx->i8_swz == 0 && DP <= 256 &&
                      DP % 16 == 0;
  if (i8resc) {
    if ((rc = ctx->rescan_qc8.ensure((size_t)cap * 256 + 16))) return rc;
    if ((rc = ctx->rescan_t8.ensure((size_t)cap * sizeof(long long) + 16))) return rc;
    rp.qc8 = (signed char*)ctx->rescan_qc8.p;
    rp.t8 = (long long*)ctx->rescan_t8.p;
  }
  if (kmetric >= 5) {
    // int8 proxies are exact up to +1 (the odd-norm half of the seed): the
    // merge sees the pass's own centre and scale (codes (x - cent/2^s) 2^s),
    // an absolute error of one code unit (DP x up / DP) and each query's
    // own coding error (off the grid / beyond the code range), measured
    TrainDev t8 = t;
    t8.mu = (const double*)ctx->i8_cent.p + t.d;
    t8.jx = ctx->i8_s;
    t8.x2max = ctx->i8_x2max;
    t8.DP = DP;
    launch_merge_rerank(metric, (const float*)ctx->cand_v.p, (const int*)ctx->cand_i.p, NL, R, t8,
                        dQ, m, W, C, 0.0,
                        ProxyScale{qvalid, 0.0, 1.0 / DP, false, (const double*)ctx->i8_cent.p, qpos,
                                   (const signed char*)ctx->XI.p, DP + 16, DP, ctx->i8_swz},
                        cl.gthr, sink,
                        (int*)ctx->rescan_q.p, (double*)ctx->rescan_tau.p, (int*)ctx->rescan_cnt.p,
                        sm, rp, s);
  } else {
    launch_merge_rerank(metric, (const float*)ctx->cand_v.p, (const int*)ctx->cand_i.p, NL, R, t,
                        dQ, m, W, C, err_factor(kmetric, DP),
                        kmetric == 4 ? ProxyScale{qvalid, 0x1p-14, 0x1p-28, true, nullptr, qpos}
                                     : ProxyScale{qvalid, 0x1p-125, 0x1p-124, false, nullptr, qpos},
                        cl.gthr, sink, (int*)ctx->rescan_q.p, (double*)ctx->rescan_tau.p,
                        (int*)ctx->rescan_cnt.p, sm, rp, s);
  }
  HIP_TRY(hipGetLastError());
  if (hipEvent_t ev = timing_ev(tc, 3)) HIP_TRY(hipEventRecord(ev, s));
  // rescan of uncertified queries, sized on the device (knn_select.hip)
  RescanBufs rb{};
  rb.q = (int*)ctx->rescan_q.p;
  rb.tau = (double*)ctx->rescan_tau.p;
  rb.cnt = (int*)ctx->rescan_cnt.p;
  rb.qf = (float*)ctx->fr_q.p;
  rb.thr = (float*)ctx->fr_thr.p;
  rb.fcnt = (int*)ctx->fr_cnt.p;
  rb.buf = (int*)ctx->fr_buf.p;
  rb.slow_q = (int*)ctx->slow_q.p;
  rb.counts = ctx->d_counts;
  rb.totals = (unsigned long long*)ctx->totals.p;
  rb.mask = sm.mask;
  rb.nkeep = sm.nkeep;
  rb.S = sm.S;
  rb.trows = sm.trows;
  rb.cus = ctx->cu_count;
  if (i8resc) {
    rb.qc8 = rp.qc8;
    rb.t8 = rp.t8;
    rb.i8img = (const signed char*)ctx->XI.p;
    rb.i8rb = DP + 16;
    rb.i8dp = DP;
  }
  launch_rescan(metric, t, dQ, rb, abl ? 0 : cap, W, err_factor(metric, t.DP), sink,
                abl ? 0 : (int)std::min<int64_t>(m, ctx->cu_count), s);
  // (without the full-scan launch nothing writes this call's counts)
  if (abl) launch_fill_i32(ctx->d_counts, 2, 0, s);
  // queries with exact distance ties: the reference's std::sort order
  if (sink.tie_mode && !abl)
    launch_tie_order(metric, t, dQ, sink.tie_q, sink.tie_cnt, ctx->class_cnt,
                     (unsigned char*)ctx->tie_ws.p, tie_per, tie_nwg, sink,
                     (unsigned long long*)ctx->totals.p + 2, s);
  HIP_TRY(hipGetLastError());
  if (hipEvent_t ev = timing_ev(tc, 4)) HIP_TRY(hipEventRecord(ev, s));
  HIP_TRY(hipEventRecord(ctx->done_ev, s));
  // the deferred AUTO decision reads done_ev and h_counts, which belong to
  // the LAST call: it is armed by an fp16 call and dropped by any other
  // (a later fp16 call re-arms it with its own count)
  ctx->auto_pending = !abl && ((kmetric == 4 && ctx->precision == KNN_PRECISION_AUTO &&
                                ctx->tune_fp16 < 0) ||
                               (kmetric >= 5 && ctx->tune_i8 < 0));
  ctx->auto_kind = kmetric;
  ctx->auto_m = m;
  return KNN_OK;
}

// k > kMaxK: the exact large-k path (knn_select.hip, large_k_kernel); the
// scratch (every row's distance per workgroup) is capped at ~8 GB.
static int run_large_k(knn_ctx* ctx, const double* dQ, int64_t m, int W, int metric,
                       const Sink& sink_in, hipStream_t s) {
  const TrainDev& t = ctx->train;
  Sink sink = sink_in;
  sink.tie_mode = tie_mask_of(ctx, sink_in);
  int rc;
  int64_t tie_per = 0;
  int tie_nwg = 0;
  if (sink.tie_mode) {  // tied queries: queued by large_k_kernel for the reference-order pass
    tie_per = tie_scratch_bytes(t.n, ctx->class_cnt);
    tie_nwg = tie_workgroups(ctx, tie_per);
    if ((rc = ctx->tie_q.ensure((size_t)m * sizeof(int) + 16))) return rc;
    if ((rc = ctx->tie_ws.ensure((size_t)(tie_per * tie_nwg)))) return rc;
    if ((rc = ctx->rescan_cnt.ensure(4 * sizeof(int)))) return rc;
    sink.tie_q = (int*)ctx->tie_q.p;
    sink.tie_cnt = (int*)ctx->rescan_cnt.p + 2;
    HIP_TRY(hipMemsetAsync(sink.tie_cnt, 0, sizeof(int), s));
  }
  const int64_t per = large_k_scratch_bytes(t.n, W, ctx->class_cnt);
  const int64_t nwg = std::max<int64_t>(
      1, std::min<int64_t>({m, 2 * (int64_t)ctx->cu_count, (8ll << 30) / per}));
  if ((rc = ctx->lk.ensure((size_t)(per * nwg)))) return rc;
  snprintf(ctx->last_kernel, sizeof ctx->last_kernel, "large_k_kernel<%d>", metric);
  ctx->last_kmetric = -1;
  launch_large_k(metric, t, dQ, m, W, ctx->class_cnt, (unsigned char*)ctx->lk.p, per, (int)nwg,
                 sink, s);
  if (sink.tie_mode)
    launch_tie_order(metric, t, dQ, sink.tie_q, sink.tie_cnt, ctx->class_cnt,
                     (unsigned char*)ctx->tie_ws.p, tie_per, tie_nwg, sink,
                     (unsigned long long*)ctx->totals.p + 2, s);
  launch_fill_i32(ctx->d_counts, 2, 0, s);  // exact path: no query fails certification
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ctx->done_ev, s));
  ctx->auto_pending = false;  // done_ev / h_counts now belong to this call
  return KNN_OK;
}

static int check_query_args(knn_ctx* ctx, int64_t m, int32_t k, int32_t metric) {
  if (!ctx->trained) return knn_fail(KNN_ERR_STATE, "classify before set_train");
  if (m < 0) return knn_fail(KNN_ERR_ARG, "m must be >= 0");
  if (m >= (int64_t)INT32_MAX) return knn_fail(KNN_ERR_ARG, "m must be < 2^31 per call");
  if (k < 0) return knn_fail(KNN_ERR_ARG, "k must be >= 0");
  if (k > ctx->train.n)
    return knn_fail(KNN_ERR_ARG, "k exceeds n_train (the reference reads past its array, cpp:328)");
  if (metric != KNN_METRIC_L2 && metric != KNN_METRIC_L1)
    return knn_fail(KNN_ERR_ARG, "metric must be 0 (L2) or 1 (L1)");
  return KNN_OK;
}

extern "C" {

int knn_classify_device(knn_ctx* ctx, const double* dQ, int64_t m, int32_t k, int32_t metric,
                        int32_t* d_labels, int64_t* d_idx, double* d_dist, int32_t* d_flags,
                        void* stream) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if ((rc = check_query_args(ctx, m, k, metric))) return rc;
  if (!d_labels) return knn_fail(KNN_ERR_ARG, "null labels output");
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  if (m == 0) return KNN_OK;
  if (!dQ) return knn_fail(KNN_ERR_ARG, "null query pointer");
  if (k == 0) {  // cpp:324: max_label stays -1
    launch_fill_i32(d_labels, m, -1, s);
    if (d_flags) launch_fill_i32(d_flags, m, 0, s);
    HIP_TRY(hipGetLastError());
    return KNN_OK;
  }
  Sink sink{};
  sink.mode = MODE_SINGLE;
  sink.k = k;
  sink.idx_off = ctx->idx_off;
  sink.labels = d_labels;
  sink.idx = d_idx;
  sink.dist = d_dist;
  sink.flags = d_flags;
  const int W = (int)std::min<int64_t>((int64_t)k + 1, ctx->train.n);
  if (k > kMaxK) return run_large_k(ctx, dQ, m, W, metric, sink, s);
  return knn_run_search(ctx, dQ, m, W, metric, sink, s);
}

int knn_classify(knn_ctx* ctx, const double* Q, int64_t m, int32_t k, int32_t metric,
                 int32_t* out_labels, int64_t* out_idx, double* out_dist, int32_t* out_flags) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if ((rc = check_query_args(ctx, m, k, metric))) return rc;
  if (!out_labels) return knn_fail(KNN_ERR_ARG, "null labels output");
  if (m == 0) return KNN_OK;
  if (!Q) return knn_fail(KNN_ERR_ARG, "null query pointer");
  const int d = ctx->train.d;
  if ((rc = ctx->Q64.ensure((size_t)m * d * sizeof(double)))) return rc;
  if ((rc = ctx->o_lab.ensure((size_t)m * sizeof(int32_t)))) return rc;
  if ((rc = ctx->o_flags.ensure((size_t)m * sizeof(int32_t)))) return rc;
  if (out_idx && (rc = ctx->o_idx.ensure((size_t)m * std::max(k, 1) * sizeof(int64_t)))) return rc;
  if (out_dist && (rc = ctx->o_dist.ensure((size_t)m * std::max(k, 1) * sizeof(double)))) return rc;
  hipStream_t s = ctx->stream;
  HIP_TRY(hipMemcpyAsync(ctx->Q64.p, Q, (size_t)m * d * sizeof(double), hipMemcpyHostToDevice, s));
  rc = knn_classify_device(ctx, (const double*)ctx->Q64.p, m, k, metric, (int32_t*)ctx->o_lab.p,
                           out_idx ? (int64_t*)ctx->o_idx.p : nullptr,
                           out_dist ? (double*)ctx->o_dist.p : nullptr,
                           (int32_t*)ctx->o_flags.p, s);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out_labels, ctx->o_lab.p, (size_t)m * sizeof(int32_t),
                         hipMemcpyDeviceToHost, s));
  if (out_flags)
    HIP_TRY(hipMemcpyAsync(out_flags, ctx->o_flags.p, (size_t)m * sizeof(int32_t),
                           hipMemcpyDeviceToHost, s));
  if (out_idx && k > 0)
    HIP_TRY(hipMemcpyAsync(out_idx, ctx->o_idx.p, (size_t)m * k * sizeof(int64_t),
                           hipMemcpyDeviceToHost, s));
  if (out_dist && k > 0)
    HIP_TRY(hipMemcpyAsync(out_dist, ctx->o_dist.p, (size_t)m * k * sizeof(double),
                           hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return KNN_OK;
}

int knn_search_partial_device(knn_ctx* ctx, const double* dQ, int64_t m, int32_t w,
                              int32_t metric, double* d_dist, int64_t* d_idx, int32_t* d_lab,
                              void* stream) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if (!ctx->trained) return knn_fail(KNN_ERR_STATE, "search before set_train");
  if (w <= 0) return knn_fail(KNN_ERR_ARG, "w must be >= 1");
  if (metric != KNN_METRIC_L2 && metric != KNN_METRIC_L1)
    return knn_fail(KNN_ERR_ARG, "metric must be 0 (L2) or 1 (L1)");
  if (m < 0 || m >= (int64_t)INT32_MAX) return knn_fail(KNN_ERR_ARG, "bad m");
  if (!d_dist || !d_idx || !d_lab) return knn_fail(KNN_ERR_ARG, "null output");
  if (m == 0) return KNN_OK;
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  Sink sink{};
  sink.mode = MODE_PARTIAL;
  sink.w = w;
  sink.idx_off = ctx->idx_off;
  sink.idx = d_idx;
  sink.dist = d_dist;
  sink.plab = d_lab;
  // a shard smaller than w yields min(w, n) entries; the tail is padded
  const int W = (int)std::min<int64_t>(w, ctx->train.n);
  if (w > kMaxK + 1) return run_large_k(ctx, dQ, m, W, metric, sink, s);
  return knn_run_search(ctx, dQ, m, W, metric, sink, s);
}

int knn_merge_vote_device(knn_ctx* ctx, const double* d_dist, const int64_t* d_idx,
                          const int32_t* d_lab, int32_t parts, int64_t m, int32_t w, int32_t k,
                          int64_t q0, int64_t mq, int32_t* d_labels, int64_t* d_out_idx,
                          double* d_out_dist, int32_t* d_flags, void* stream) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if (parts <= 0 || w <= 0 || k < 0 || k > w || (int64_t)parts * w >= INT32_MAX)
    return knn_fail(KNN_ERR_ARG, "bad merge geometry (need 0 <= k <= w)");
  if (q0 < 0 || mq < 0 || q0 + mq > m) return knn_fail(KNN_ERR_ARG, "query slice out of range");
  if (!d_labels) return knn_fail(KNN_ERR_ARG, "null labels output");
  if (mq == 0) return KNN_OK;
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  // unions beyond the LDS kernel's 4096 entries: rank merge through scratch
  if (const int64_t sb = merge_scratch_bytes(parts, w, k, mq))
    if ((rc = ctx->mrg.ensure((size_t)sb))) return rc;
  MergeTies mt;
  mt.mode = ctx->tune_ties;
  launch_merge_vote_partials(d_dist, d_idx, d_lab, parts, m, w, k, d_labels, d_out_idx,
                             d_out_dist, d_flags, s, q0, mq, 0, ctx->mrg.p, mt);
  HIP_TRY(hipGetLastError());
  return KNN_OK;
}

int knn_shard_distances_device(knn_ctx* ctx, const double* dQ, const int32_t* d_qsel,
                               int32_t nsel, int32_t metric, double* d_out, void* stream) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if (!ctx->trained) return knn_fail(KNN_ERR_STATE, "shard distances before set_train");
  if (nsel < 0 || metric < 0 || metric > 1) return knn_fail(KNN_ERR_ARG, "bad shard distance arguments");
  if (nsel == 0) return KNN_OK;
  if (!dQ || !d_out) return knn_fail(KNN_ERR_ARG, "null pointer");
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  launch_shard_dist(metric, ctx->train, dQ, d_qsel, nsel, d_out, s);
  HIP_TRY(hipGetLastError());
  return KNN_OK;
}

int knn_tie_resolve_device(knn_ctx* ctx, const double* d_D, int32_t parts, const int64_t* rows,
                           int32_t nsel, const int32_t* d_lab_all, const int32_t* d_orow,
                           int32_t k, int32_t* d_labels, int64_t* d_idx, double* d_dist,
                           int32_t* d_flags, void* stream) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if (!ctx->trained) return knn_fail(KNN_ERR_STATE, "tie resolve before set_train");
  if (parts <= 0 || parts > kMaxParts || nsel < 0 || !rows)
    return knn_fail(KNN_ERR_ARG, "bad tie resolve geometry (1 <= parts <= 64)");
  PartRows pr{};
  pr.parts = parts;
  for (int p = 0; p < parts; p++) {
    if (rows[p] < 0) return knn_fail(KNN_ERR_ARG, "negative part rows");
    pr.off[p + 1] = pr.off[p] + rows[p];
  }
  const int64_t n = pr.off[parts];
  if (n <= 0 || n >= (int64_t)INT32_MAX) return knn_fail(KNN_ERR_ARG, "total rows must be in [1, 2^31)");
  if (k <= 0 || k > n) return knn_fail(KNN_ERR_ARG, "k must be in [1, total rows]");
  if (nsel == 0) return KNN_OK;
  if (!d_D || !d_lab_all || !d_orow || !d_labels) return knn_fail(KNN_ERR_ARG, "null pointer");
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  const int64_t per = tie_scratch_bytes(n, ctx->class_cnt);
  const int nwg = std::min<int>(tie_workgroups(ctx, per), nsel);
  if ((rc = ctx->tie_ws.ensure((size_t)(per * nwg)))) return rc;
  Sink sink{};
  sink.mode = MODE_SINGLE;
  sink.k = k;
  sink.labels = d_labels;
  sink.idx = d_idx;
  sink.dist = d_dist;
  sink.flags = d_flags;
  launch_tie_resolve(d_D, pr, nsel, d_lab_all, d_orow, ctx->class_cnt,
                     (unsigned char*)ctx->tie_ws.p, per, nwg, sink,
                     (unsigned long long*)ctx->totals.p + 2, s);
  HIP_TRY(hipGetLastError());
  return KNN_OK;
}

int knn_minmax_device(knn_ctx* ctx, const double* d_X, int64_t rows, int32_t d, double* d_max,
                      double* d_min, int32_t init, void* stream) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if (rows < 0 || d <= 0 || (rows > 0 && !d_X) || !d_max || !d_min)
    return knn_fail(KNN_ERR_ARG, "bad minmax arguments");
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  const int64_t R = minmax_rows_per_sweep(rows, d, ctx->cu_count);
  if ((rc = ctx->nrm_part.ensure((size_t)2 * d * R * sizeof(double)))) return rc;
  launch_minmax(d_X, rows, d, R, (double*)ctx->nrm_part.p, d_max, d_min, init, s);
  HIP_TRY(hipGetLastError());
  return KNN_OK;
}

int knn_normalize_device(knn_ctx* ctx, double* d_X, int64_t rows, int32_t d,
                         const double* d_max, const double* d_min, void* stream) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if (rows < 0 || d <= 0 || (rows > 0 && !d_X) || !d_max || !d_min)
    return knn_fail(KNN_ERR_ARG, "bad normalize arguments");
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  launch_normalize_apply(d_X, rows, d, minmax_rows_per_sweep(rows, d, ctx->cu_count), d_max,
                         d_min, s);
  HIP_TRY(hipGetLastError());
  return KNN_OK;
}

int knn_normalize(knn_ctx* ctx, double* const* sets, const int64_t* rows, int32_t nsets,
                  int32_t d, double* out_max, double* out_min) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if (nsets < 0 || d <= 0 || (nsets > 0 && (!sets || !rows)))
    return knn_fail(KNN_ERR_ARG, "bad normalize arguments");
  int64_t total = 0;
  for (int i = 0; i < nsets; i++) {
    if (rows[i] < 0 || (rows[i] > 0 && !sets[i])) return knn_fail(KNN_ERR_ARG, "bad set");
    total += rows[i];
  }
  hipStream_t s = ctx->stream;
  if ((rc = ctx->nrm_mm.ensure((size_t)2 * d * sizeof(double)))) return rc;
  if ((rc = ctx->nrm_X.ensure((size_t)std::max<int64_t>(total, 1) * d * sizeof(double)))) return rc;
  double* dmax = (double*)ctx->nrm_mm.p;
  double* dmin = dmax + d;
  double* dX = (double*)ctx->nrm_X.p;
  int64_t off = 0;
  for (int i = 0; i < nsets; i++) {  // cpp:245-274 over every set
    double* di = dX + off * d;
    if (rows[i] > 0)
      HIP_TRY(hipMemcpyAsync(di, sets[i], (size_t)rows[i] * d * sizeof(double),
                             hipMemcpyHostToDevice, s));
    if ((rc = knn_minmax_device(ctx, di, rows[i], d, dmax, dmin, i == 0, s))) return rc;
    off += rows[i];
  }
  if (nsets == 0 && (rc = knn_minmax_device(ctx, nullptr, 0, d, dmax, dmin, 1, s))) return rc;
  off = 0;
  for (int i = 0; i < nsets; i++) {  // cpp:279-305
    double* di = dX + off * d;
    if ((rc = knn_normalize_device(ctx, di, rows[i], d, dmax, dmin, s))) return rc;
    if (rows[i] > 0)
      HIP_TRY(hipMemcpyAsync(sets[i], di, (size_t)rows[i] * d * sizeof(double),
                             hipMemcpyDeviceToHost, s));
    off += rows[i];
  }
  if (out_max) HIP_TRY(hipMemcpyAsync(out_max, dmax, d * sizeof(double), hipMemcpyDeviceToHost, s));
  if (out_min) HIP_TRY(hipMemcpyAsync(out_min, dmin, d * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return KNN_OK;
}

int knn_sync(knn_ctx* ctx) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  HIP_TRY(hipEventSynchronize(ctx->done_ev));  // the last call, on whatever stream it ran
  auto_check(ctx);
  return KNN_OK;
}

int64_t knn_last_rescan_count(knn_ctx* ctx) {
  if (!ctx || hipSetDevice(ctx->device) != hipSuccess) return -1;
  if (hipEventSynchronize(ctx->done_ev) != hipSuccess) return -1;  // the last call's counts
  auto_check(ctx);
  return ctx->h_counts[0];
}

int knn_rescan_totals(knn_ctx* ctx, int64_t out[2], int reset) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if (!out) return knn_fail(KNN_ERR_ARG, "null output");
  unsigned long long v[2];
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  HIP_TRY(hipEventSynchronize(ctx->done_ev));
  HIP_TRY(hipMemcpy(v, ctx->totals.p, sizeof v, hipMemcpyDeviceToHost));
  out[0] = (int64_t)v[0];
  out[1] = (int64_t)v[1];
  if (reset) HIP_TRY(hipMemset(ctx->totals.p, 0, sizeof v));
  auto_check(ctx);
  return KNN_OK;
}

int knn_tie_totals(knn_ctx* ctx, int64_t* out, int reset) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  if (!out) return knn_fail(KNN_ERR_ARG, "null output");
  unsigned long long v = 0;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  HIP_TRY(hipEventSynchronize(ctx->done_ev));
  HIP_TRY(hipMemcpy(&v, (unsigned long long*)ctx->totals.p + 2, sizeof v, hipMemcpyDeviceToHost));
  *out = (int64_t)v;
  if (reset) HIP_TRY(hipMemset((unsigned long long*)ctx->totals.p + 2, 0, sizeof v));
  return KNN_OK;
}

const char* knn_last_kernel_name(knn_ctx* ctx) { return ctx ? ctx->last_kernel : ""; }

int knn_set_precision(knn_ctx* ctx, int mode) {
  if (!ctx) return knn_fail(KNN_ERR_ARG, "null context");
  if (mode < KNN_PRECISION_AUTO || mode > KNN_PRECISION_FP16)
    return knn_fail(KNN_ERR_ARG, "unknown precision mode");
  ctx->precision = mode;
  return KNN_OK;
}

int knn_last_candidate_path(knn_ctx* ctx) { return ctx ? ctx->last_kmetric : -1; }

int knn_set_tuning(knn_ctx* ctx, const char* key, int64_t value) {
  if (!ctx || !key) return knn_fail(KNN_ERR_ARG, "null argument");
  if (!strcmp(key, "fp16")) {
    if (value < -1 || value > 1) return knn_fail(KNN_ERR_ARG, "fp16 must be -1, 0 or 1");
    ctx->tune_fp16 = (int)value;
  } else if (!strcmp(key, "mfma16")) {
    if (value < -1 || value > 1) return knn_fail(KNN_ERR_ARG, "mfma16 must be -1, 0 or 1");
    ctx->tune_m16 = (int)value;
  } else if (!strcmp(key, "R")) {
    if (value != 0 && value != 4 && value != 8 && value != 16)
      return knn_fail(KNN_ERR_ARG, "R must be 0 (auto), 4, 8 or 16");
    ctx->tune_R = (int)value;
  } else if (!strcmp(key, "nw")) {
    if (value != 0 && value != 4 && value != 8 && value != 16)
      return knn_fail(KNN_ERR_ARG, "nw must be 0, 4, 8 or 16 (16: fp16 16x16x32 only)");
    ctx->tune_nw = (int)value;
  } else if (!strcmp(key, "ablate")) {
    ctx->tune_ablate = (int)value;  // timing experiments only: results become invalid
  } else if (!strcmp(key, "S")) {
    if (value < 0 || value > 64) return knn_fail(KNN_ERR_ARG, "S must be 0 (auto) .. 64");
    ctx->tune_S = (int)value;
  } else if (!strcmp(key, "qres")) {
    if (value < -1 || value > 1) return knn_fail(KNN_ERR_ARG, "qres must be -1, 0 or 1");
    ctx->tune_qres = (int)value;
  } else if (!strcmp(key, "s3q")) {
    if (value < -1 || value > 1) return knn_fail(KNN_ERR_ARG, "s3q must be -1, 0 or 1");
    ctx->tune_s3q = (int)value;
  } else if (!strcmp(key, "xhswz")) {
    if (value < 0 || value > 1) return knn_fail(KNN_ERR_ARG, "xhswz must be 0 or 1");
    ctx->tune_xhswz = (int)value;
  } else if (!strcmp(key, "i8")) {
    if (value < -1 || value > 1) return knn_fail(KNN_ERR_ARG, "i8 must be -1, 0 or 1");
    ctx->tune_i8 = (int)value;
  } else if (!strcmp(key, "i8w")) {
    if (value < -1 || value > 1) return knn_fail(KNN_ERR_ARG, "i8w must be -1, 0 or 1");
    ctx->tune_i8w = (int)value;
  } else if (!strcmp(key, "seed")) {
    if (value < -1) return knn_fail(KNN_ERR_ARG, "seed must be 0 / -1 (off) or N = sample rows");
    ctx->tune_seed = value;
  } else if (!strcmp(key, "s3gq")) {
    if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8 && value != 16 && value != 32)
      return knn_fail(KNN_ERR_ARG, "s3gq must be 0 (auto) or 1, 2, 4, 8, 16, 32");
    ctx->tune_s3gq = (int)value;
  } else if (!strcmp(key, "ophase")) {
    if (value < -1 || value > kRegionMax) return knn_fail(KNN_ERR_ARG, "ophase must be -1 (auto) .. 64");
    ctx->tune_ophase = (int)value;
  } else if (!strcmp(key, "order")) {
    if (value < -1 || value > kRegionMax)
      return knn_fail(KNN_ERR_ARG, "order must be -1 (auto), 0, 1 or 2..64 regions");
    ctx->tune_order = (int)value;
  } else if (!strcmp(key, "qblk")) {
    if (value < 0 || value > 1 << 20) return knn_fail(KNN_ERR_ARG, "qblk must be 0 (split-major) or >= 1");
    ctx->tune_qblk = (int)value;
  } else if (!strcmp(key, "i8resc")) {
    if (value < -1 || value > 1) return knn_fail(KNN_ERR_ARG, "i8resc must be -1 (auto), 0 or 1");
    ctx->tune_i8resc = (int)value;
  } else if (!strcmp(key, "gg")) {
    if (value != -1 && value != 4 && value != 8) return knn_fail(KNN_ERR_ARG, "gg must be -1 (auto), 4 or 8");
    ctx->tune_gg = (int)value;
  } else if (!strcmp(key, "nblk")) {
    if (value < -1 || value > 3) return knn_fail(KNN_ERR_ARG, "nblk must be -1 (auto), 0, 1, 2 or 3");
    ctx->tune_nblk = (int)value;
  } else if (!strcmp(key, "ties")) {
    if (value < 0 || value > 2) return knn_fail(KNN_ERR_ARG, "ties must be 0, 1 or 2");
    ctx->tune_ties = (int)value;
  } else if (!strcmp(key, "gk")) {
    if (value < -1 || value > 16) return knn_fail(KNN_ERR_ARG, "gk must be -1 (auto) .. 16");
    ctx->tune_gk = (int)value;
  } else {
    return knn_fail(KNN_ERR_ARG, std::string("unknown tuning key ") + key);
  }
  return KNN_OK;
}

int knn_set_timing(knn_ctx* ctx, int enable) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  // timing-only events: no system-scope fence (cache writeback and
  // invalidate) at each record -- with it every record idled the stream
  // ~6 us (profiles/ab_log.md r5u); only the times are read back
  if (enable < 0 || enable > 2) return knn_fail(KNN_ERR_ARG, "timing must be 0, 1 or 2");
  if (enable && !ctx->ring[0].ev[0])
    for (auto& tc : ctx->ring)
      for (auto& e : tc.ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  ctx->timing = enable;
  return KNN_OK;
}

double knn_last_phase_ms(knn_ctx* ctx, int phase) {
  if (!ctx || phase < 0 || phase > 3 || ctx->ring_last < 0) return -1.0;
  if (hipSetDevice(ctx->device) != hipSuccess) return -1.0;
  TimedCall& tc = ctx->ring[ctx->ring_last];
  if (!phase_timed(tc, phase)) return -1.0;
  if (hipEventSynchronize(tc.ev[tc.mode == 2 ? 2 : 4]) != hipSuccess) return -1.0;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, tc.ev[phase], tc.ev[phase + 1]) != hipSuccess) return -1.0;
  return ms;
}

int knn_timing_totals(knn_ctx* ctx, double out_ms[4], int64_t* calls, int reset) {
  int rc;
  if ((rc = device_guard(ctx))) return rc;
  for (auto& tc : ctx->ring) fold_timing(ctx, tc);
  if (out_ms)
    for (int p = 0; p < 4; p++) out_ms[p] = ctx->tsum[p];
  if (calls) *calls = ctx->tcalls;
  if (reset) {
    for (double& v : ctx->tsum) v = 0.0;
    ctx->tcalls = 0;
  }
  return KNN_OK;
}

int knn_last_geometry(knn_ctx* ctx, int64_t out[4]) {
  if (!ctx || !out) return knn_fail(KNN_ERR_ARG, "null argument");
  for (int i = 0; i < 4; i++) out[i] = ctx->geom[i];
  return KNN_OK;
}

}  // extern "C"
