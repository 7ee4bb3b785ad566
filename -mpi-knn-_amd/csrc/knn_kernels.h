// knn_kernels.h -- internal launch interface of the HIP kernels (gfx950).
// Not part of the public ABI (see include/knn_amd.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace knnk {

constexpr int kQPB = 128;        // queries per candidate workgroup (4 waves x 32)
constexpr int kTR = 32;          // train rows per MFMA sub-tile of the resident kernel
constexpr int kResTileRows = 64; // resident kernel: train rows per staged tile (2 sub-tiles)
constexpr int kMaxUnion = 1024;  // max candidates kept per query across all lists
constexpr int kSortN = 2048;     // rows per exact-rescan chunk / reduce block
constexpr int kMaxK = 1000;      // largest k served (k+1 <= kMaxUnion)
constexpr int kStreamDC = 32;    // dims per LDS chunk in the large-d kernel
constexpr int kRowAlign = 256;   // train rows are padded to a multiple of this (<= one staged tile)

enum { MODE_SINGLE = 0, MODE_PARTIAL = 1 };

// Output sinks of a search: MODE_SINGLE writes the vote, MODE_PARTIAL the
// exact top-w list with labels (train-sharded building block).
struct Sink {
  int mode;
  int k;                 // neighbours voted / reported (single)
  int w;                 // list length (partial)
  int64_t idx_off;       // added to reported indices
  int32_t* labels;       // single: [m]
  int64_t* idx;          // single: [m*k] (nullable); partial: [m*w]
  double* dist;          // single: [m*k] (nullable); partial: [m*w]
  int32_t* flags;        // single: [m] (nullable)
  int32_t* plab;         // partial: [m*w]
  // single: tied queries appended to tie_q (count in tie_cnt[0]) for the
  // reference-order pass (launch_tie_order): tie_mode 0 none, 1 those whose
  // label the reference's tie order could change, 2 every tied query
  int tie_mode;
  int* tie_q;
  int* tie_cnt;
};

// Train-set side state resident in HBM.
struct TrainDev {
  const double* X64;     // [n][d] fp64 (reference values)
  const double* mu;      // [d] train column means: the candidate pass's centre
  const int32_t* lab;    // [n]
  const float* X32;      // [n_pad][DP+4] fp32 padded rows (payload | seeds), zero padded
  const float* xinit_l2; // [n_pad] fl32(||x32||^2); +inf on pad rows
  const float* xinit_l1; // [n_pad] 0; +inf on pad rows
  int64_t n, n_pad;
  int d, DP;
  double x2max, x1max;   // max ||x - mu||_2^2, max ||x - mu||_1 over the train rows
  double dxmax;          // max ||fp16 row / 2^jx - (x - mu)||_2 of the fp16 copy (when built)
  int jx;                // candidate operands are 2^jx (x - mu) (knn_prep.hip)
  // Region order (knn_order.hip): row p of every candidate image (X32, the
  // fp16 / bf16 / int8 copies) is train row perm[p]; ipos is the inverse.
  // Null: images in train order.  Candidate lists carry image positions; the
  // merge and the rescan report train rows.
  const int* perm = nullptr;  // [n]
  const int* ipos = nullptr;  // [n]
};

int pad_dim(int d);                 // padded dim the candidate kernels run at
int pad_dim_bf16x3(int d);          // padded dim of the bf16x3 kernel, -1 if unsupported
int pad_dim_fp16(int d);            // padded dim of the fp16 kernel (metric 4), -1 if unsupported
bool bf16x3_streamed(int DP);       // bf16x3 at this DP runs the S3 stream kernel
constexpr int kS3Rows = 256;        // S3 kernel: train rows per tile = queries per workgroup
constexpr int kS3GqMax = 4;         // S3: default largest XCD grouping of query tiles (s3_group)
int s3_blocks_per_cu(int R);
// S3 kernel (bf16x3, DP > 256): XT/QT are tile-chunk images made by
// launch_prep_split_tiled, XS the per-row seeds [n_pad]; n_pad and m_pad are
// multiples of kS3Rows.
// gq_max: the largest XCD grouping of query tiles to use (s3_group)
void launch_cand_s3(const unsigned short* XT, const float* XS, const unsigned short* QT, int DP,
                    int64_t n_pad, int R, int S, int n_qt, float* out_v, int* out_i, int ablate,
                    hipStream_t s, int gq_max = kS3GqMax);
// fp64 rows -> bf16 hi/lo tile-chunk images of scale*x (S3 layout); seed_out
// (train only, else null) receives seed_src[row] (+inf on pad rows)
void launch_prep_split_tiled(const double* X64, const double* mu, int64_t n, int d, int DP,
                             int64_t n_pad, double scale, unsigned short* out,
                             const float* seed_src, float* seed_out, hipStream_t s,
                             const int* perm = nullptr);
// fp16 S3 kernel (DP > 256, DP % 32 == 0): XT/QT made by launch_prep_half_tiled
// q16: the v_mfma_f32_16x16x32_f16 form (R = 8 quad lists: [m_pad][4S][8])
// gthr / gk: the global threshold exchange of the q16 form (null / 0: none)
void launch_cand_s3h(const unsigned short* XT, const float* XS, const unsigned short* QT, int DP,
                     int64_t n_pad, int R, int S, int n_qt, float* out_v, int* out_i, int ablate,
                     bool q16, uint32_t* gthr, int gk, hipStream_t s, int gq_max = kS3GqMax);
int s3h_blocks_per_cu(int R);
int s3q_blocks_per_cu();
// query-resident fp16 kernel for d > 256 (knn_cand_qres.hip): the S3 q16
// kernel's outputs from the same images, 2 n_qt workgroup tiles of 128
// queries; false: no instantiation for DP (run S3)
bool qres_supported(int DP);
bool launch_cand_qres(const unsigned short* XT, const float* XS, const unsigned short* QT, int DP,
                      int64_t n_pad, int S, int n_qt, float* out_v, int* out_i, uint32_t* gthr, int gk,
                      hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop);
// S3 workgroup grouping for n_qt query tiles and S splits (knn_cand.hip, s3_map)
int s3_group(int n_qt, int S, int gq_max = kS3GqMax);
int pad_dim_fp16_s3(int d);         // padded dim of the fp16 S3 image (multiple of 32, > 256)
// fp64 rows -> fp16 S3 tile-chunk images of mult * 2^jx (x - mu) (knn_prep.hip);
// train: seed_out[row] = seed_src[row] (+inf on pad rows) and the running max
// of the rows' squared representation error in dx2max; queries: seed_out =
// dx2max = null, valid[row] <= 0 -> zero operands
void launch_prep_half_tiled(const double* X64, const double* mu, int64_t n, int d, int DP,
                            int64_t n_pad, int jx, double mult, unsigned short* out,
                            const float* seed_src, float* seed_out, const float* valid,
                            unsigned long long* dx2max, hipStream_t s, const int* perm = nullptr);
bool cand_supported(int DP);
// train rows per tile of the candidate kernel serving (kernel metric, DP):
// split s of a launch walks tiles s, s + S, ... (rows (r / tile) % S == s)
int cand_tile_rows(int metric, int DP);
int cand_blocks_per_cu(int metric, int DP, int R, int nw);  // resident workgroups per CU
int cand_queries_per_wave(int metric, int DP);  // resident kernel: queries per wave

// metric: 0 = L2 fp32 MFMA, 1 = L1 fp32 VALU, 2 = L2 bf16x3 MFMA (32x32x16),
// 3 = L2 bf16x3 on 16x16x32, 4 = L2 fp16 on 16x16x32, 5 = L2 int8 on
// 16x16x64, 6 = L2 int8 on 32x32x32 (see knn_cand_res.hip)
struct CandLaunch {
  int metric, DP, R, S, n_qt;
  int64_t n_pad;
  const float* X32;
  const float* xinit;
  const float* Q32;
  float* out_v;
  int* out_i;
  int ablate;   // timing-only ablation bits (0 in production)
  int nw;       // resident kernel: waves per workgroup, 4, 8 or 16
  int qpb;      // resident kernel: queries per workgroup the host laid out (nw x
                // queries per wave; checked against the kernel before launch)
  uint32_t* gthr;  // resident kernel: per-query global thresholds [m_pad][kGthrSlots] (keys)
  int xsw;         // fp16 (metric 4): the train image's chunks are swizzled (xh_swz)
  int gk;          // what a list group publishes into gthr (see cand_kernel): 0 = the
                   // lists' R-th entries into split % 4, K = 1..4: the K-th smallest of
                   // the union of the query's lists in the workgroup into split % 8
  // resident kernel, region order: qstart[p] = the image position where the
  // region of the query at position p starts; each workgroup starts its
  // split's stream at the first of its tiles at or after qstart[first
  // query of the tile] (null: at the split's first tile)
  const int* qstart = nullptr;
  int gmask = 7;   // slot groups of gthr - 1: a split publishes into slot split & gmask
  int qblk = 0;    // workgroup order: 0 split-major, B: query blocks of B tiles (cand_kernel)
  // "cand" timing events recorded by the resident kernel's own dispatch
  // (hipExtLaunchKernelGGL), so the phase is the kernel's execution as
  // rocprofv3 times it (profiles/ab_log.md r6u); null: none
  hipEvent_t ev_start = nullptr, ev_stop = nullptr;
};
constexpr uint32_t kGthrInit = 0xFF800000u;  // order-preserving key of +inf
constexpr int kGthrSlots = 8;                // slots per query in gthr
// gthr init: slots [0, active) = +inf keys, the rest 0 (never the max)
void launch_fill_gthr(uint32_t* g, int64_t m_pad, int active, hipStream_t s);
// seeded thresholds: the need-th smallest of each query's U pre-pass list entries
void launch_seed_gthr(const float* v, int64_t m_pad, int U, int need, int active, uint32_t* g,
                      hipStream_t s);

// Candidate-pass operands are centred on the train column means mu (see knn_prep.hip).
int col_mean_blocks(int64_t n);  // rows of the `partial` scratch (x d doubles)
void launch_col_mean(const double* X64, int64_t n, int d, double* partial, double* mu,
                     hipStream_t s);
void launch_absmax(const double* X64, const double* mu, int64_t n, int d, unsigned long long* out,
                   unsigned long long* nonfinite, hipStream_t s);
void launch_label_check(const int32_t* lab, int64_t n, int class_cnt, unsigned long long* bad,
                        hipStream_t s);
// perm (every train image builder): image row p <- train row perm[p] (null: p)
void launch_prep_train(const double* X64, const double* mu, int64_t n, int d, int DP,
                       int64_t n_pad, int jx, float* X32, float* xl2, float* xl1,
                       unsigned long long* stats, hipStream_t s, const int* perm = nullptr);
void launch_query_check(const double* Q64, const double* mu, int64_t m, int d, int64_t m_pad,
                        double scale, int jx, double limit, float* valid, hipStream_t s);
void launch_prep_queries(const double* Q64, const double* mu, int64_t m, int d, int DP,
                         int64_t m_pad, double scale, int jx, float* Q32, hipStream_t s);
// false: no kernel instantiated for this (DP, R, metric, nw) -- nothing launched
bool launch_cand(const CandLaunch& c, hipStream_t s);
// gthr: the candidate kernel's per-query global thresholds ([m_pad][kGthrSlots] keys)
// or null when the kernel kept none
// failed queries are appended to rescan_q with rescan_tau = the W-th exact
// distance among their re-ranked rows (+inf if unknown)
// Proxies are in units 2^(2 t.jx) (L2) / 2^t.jx (L1).  valid[q] = 0: the
// query's operands left the format's range, its proxies are void (exact
// rescan).  ue / up: absolute error per operand element / per product in
// scaled units, for values outside the format's normal range.
// f16: the candidate pass ran on fp16 operands; the merge measures each
// query's representation error (rebuilding its operand's rounding) instead
// of assuming the format's worst case.
struct ProxyScale {
  const float* valid;
  double ue, up;
  bool f16 = false;
  // int8 pass: the per-dimension code centres (queries are coded
  // clamp(rint(q 2^s - cent), -128, 127); the merge measures the rounding)
  const double* i8c = nullptr;
  // queries in region order: query q's lists and thresholds sit at position
  // qpos[q] (null: at q)
  const int* qpos = nullptr;
  // int8 pass: the train image (rows of i8rb bytes, i8dp codes, chunks
  // swizzled when i8swz) -- the exact re-rank of a query on the train grid
  // reads it instead of the fp64 rows (merge_rerank_kernel, exact_sorted_i8)
  const signed char* i8x = nullptr;
  int i8rb = 0, i8dp = 0, i8swz = 0;
};
// Per-split certification (merge) and the targeted rescan: a query whose
// bound fails only through some splits' lists (a list holding R of its top
// W, its R-th entry inside the top W) rescans just those splits' rows.
struct SplitMap {
  int S = 0;                  // splits of the candidate launch (0: whole-set rescans only)
  int lps = 0;                // lists per query per split (4 quad, 2 otherwise)
  int64_t trows = 0;          // train rows per tile
  int cap = 0;                // failed queries the fast rescan serves
  unsigned long long* mask = nullptr;  // [m] splits each failed query rescans (~0: all rows)
  int* nkeep = nullptr;       // [cap] re-ranked rows of the other splits handed to the rescan
  int* keep = nullptr;        // [cap][kRescanCap] (the fast rescan's row buffer)
};
// The fast rescan's per-query setup, done by the merge for each query it
// fails (the first `cap`): the fp32 query operand of the rescan's X32 image
// (its centre mu, scale 2^jx, padded dim DP and norms x2max / x1max), the
// proxy threshold every row within tau passes (f_err: the fp32 error factor
// of DP) and the count of rows the merge already handed over (fcnt = nkeep).
struct RescanPrep {
  const double* mu = nullptr;
  double x2max = 0.0, x1max = 0.0, f_err = 0.0;
  float* qf = nullptr;   // [cap][DP]
  float* thr = nullptr;  // [cap]
  int* fcnt = nullptr;   // [cap]
  int jx = 0, DP = 0, cap = 0;
  // int8 pass with an unswizzled image (kernel metric 6): a failed query on
  // the train grid is filtered on the codes instead (rescan_filter_i8_kernel):
  // its codes [cap][256] and the largest exact integer squared distance
  // (code units) a row may have to reach tau; t8 < 0: the fp32 filter's
  // query (off the grid, tau unknown, or no int8 pass).  Null: none.
  signed char* qc8 = nullptr;
  long long* t8 = nullptr;
};
void launch_merge_rerank(int metric, const float* cv, const int* ci, int NL, int R,
                         const TrainDev& t, const double* Q64, int64_t m, int W, int C,
                         double f_err, ProxyScale ps, const uint32_t* gthr, const Sink& sink,
                         int* rescan_q, double* rescan_tau, int* rescan_cnt, const SplitMap& sm,
                         const RescanPrep& rp, hipStream_t s);
constexpr int kRescanCap = 1024;        // rows a fast rescan may append per query
constexpr int kRescanStageMaxDP = 256;  // fast rescan stages rows in LDS up to this DP
constexpr int kRescanFastQueries = 65536;  // failed queries per call the fast path serves
// Device-driven rescan (knn_select.hip): every buffer sized for `cap` fast-
// path queries (cap <= m); the merge fills q/tau and counts cnt[0].
struct RescanBufs {
  int* q;                    // [m] failed queries (merge)
  double* tau;               // [m] W-th exact distance among the re-ranked rows (+inf unknown)
  int* cnt;                  // [2] failed queries (merge) / passed on to the full scan
  float* qf;                 // [cap][DP] fp32 query operands of the fast path
  float* thr;                // [cap] proxy thresholds
  int* fcnt;                 // [cap] rows appended per query
  int* buf;                  // [cap][kRescanCap] appended rows
  int* slow_q;               // [m] queries for the full scan
  int* counts;               // host-mapped {cnt[0], full scans} of the call (nullable)
  unsigned long long* totals;  // device running sums of the same (nullable)
  const unsigned long long* mask;  // [m] splits to scan per failed query (null: all rows)
  const int* nkeep;          // [cap] rows the merge already put in buf (null: none)
  int S;                     // splits / tile rows of the candidate launch (mask bits)
  int64_t trows;
  int cus;                   // compute units (the staged filter's grid)
  // int8 filter (RescanPrep::qc8 / t8; null: every query on the fp32 filter):
  // the int8 image [n_pad][i8rb] bytes, codes of dims [0, i8dp) plain
  const signed char* qc8 = nullptr;
  const long long* t8 = nullptr;
  const signed char* i8img = nullptr;
  int i8rb = 0, i8dp = 0;
};
// Enqueues the rescan path (filter, exact finish, full scan; the merge did
// each fast-path query's setup, RescanPrep); every kernel reads the counts on
// the device.  f_err: the fp32 candidate
// error factor of t.DP; full_blocks: workgroups of the full-scan kernel.
void launch_rescan(int metric, const TrainDev& t, const double* Q64, const RescanBufs& rb, int cap,
                   int W, double f_err, const Sink& sink, int full_blocks, hipStream_t s);
// k-way merge + vote of [parts][m][w] sorted lists for queries [q0, q0+mq).
// Unions of up to 4096 entries sort in LDS; larger ones (any k <= n) rank
// each entry by binary searches and need merge_scratch_bytes() of device
// scratch (0 when the LDS kernel serves the geometry).
int64_t merge_scratch_bytes(int parts, int w, int k, int64_t mq);
// Reference tie order in the merge: mode as Sink::tie_mode; a query whose
// label can depend on the order among equal distances across shards gets
// kFlagTiePending and, when q is set, its output row appended to q (count in
// cnt[0]) for the train-sharded reference-order pass (launch_tie_resolve).
constexpr int kFlagTiePending = 64;  // KNN_FLAG_TIE_PENDING
struct MergeTies {
  int mode = 0;
  int* q = nullptr;
  int* cnt = nullptr;
};
void launch_merge_vote_partials(const double* dist, const int64_t* idx, const int32_t* lab,
                                int parts, int64_t m, int w, int k, int32_t* out_lab,
                                int64_t* out_idx, double* out_dist, int32_t* out_flags,
                                hipStream_t s, int64_t q0 = 0, int64_t mq = -1,
                                int64_t pstride = 0, void* scratch = nullptr,
                                const MergeTies& mt = MergeTies{});
// Train-sharded reference tie order (knn_select.hip): out[i][j] = the exact
// fp64 distance (reference operation order) of shard row j to query
// Q64[qsel[i]] (qsel null: row i), [nsel][t.n].
void launch_shard_dist(int metric, const TrainDev& t, const double* Q64, const int* qsel, int nsel,
                       double* out, hipStream_t s);
// Global row layout of the exchanged distance blocks: part p holds rows
// [off[p], off[p+1]) (parts <= kMaxParts).
constexpr int kMaxParts = 64;
struct PartRows {
  int parts;
  int64_t off[kMaxParts + 1];
};
// D = parts blocks [nsel][rows_p] at offsets nsel * off[p]; lab_all the labels
// of all off[parts] rows; outputs at sink rows orow[i] (labels, idx = global
// row, dist, flags: TIE_PENDING -> TIE_REF).  Scratch per workgroup:
// tie_scratch_bytes(off[parts], class_cnt); totals: running count (nullable).
void launch_tie_resolve(const double* D, const PartRows& pr, int nsel, const int32_t* lab_all,
                        const int* orow, int class_cnt, unsigned char* scratch, int64_t per_wg,
                        int nwg, const Sink& sink, unsigned long long* totals, hipStream_t s);
// byte stride of one part's packed [dist | idx | label] lists of m x w entries
inline int64_t packed_part_bytes(int64_t m, int w) { return (m * w * 20 + 15) / 16 * 16; }
// k beyond kMaxK (knn_select.hip, large_k_kernel): the exact path over every
// row, nwg workgroups with per_wg bytes of scratch each (large_k_scratch_bytes)
int64_t large_k_scratch_bytes(int64_t n, int W, int class_cnt);
void launch_large_k(int metric, const TrainDev& t, const double* Q64, int64_t m, int W,
                    int class_cnt, unsigned char* scratch, int64_t per_wg, int nwg,
                    const Sink& sink, hipStream_t s);
void launch_fill_i32(int32_t* p, int64_t n, int32_t v, hipStream_t s);
// int8 images (kernel metric 5, knn_prep.hip): train values x = (cent_i + k) /
// 2^s with integer codes k in [-128, 127].  grid_stats: per-dim min | max
// (out[2d]) and the largest fractional bit count (frac, atomicMax) of the
// train values; partial holds col_mean_blocks(n) x 2d doubles.
void launch_grid_stats(const double* X64, int64_t n, int d, double* partial, double* out,
                       unsigned* frac, hipStream_t s);
// swz: 16-B chunks at ch ^ xh_swz(row) (the 16x16x64 kernel's image); 0 for
// the 32x32x32 kernel's (its reads are conflict-free unswizzled)
void launch_prep_i8_train(const double* X64, const double* cent, int64_t n, int d, int DP,
                          int64_t n_pad, int s, signed char* out, unsigned* codes_max, int swz,
                          hipStream_t st, const int* perm = nullptr);
// qperm (query operand builders): operand row p <- query qperm[p] (null: p).
// The int8 builder also runs launch_query_check's test (mu, scale, jx, limit)
// into valid, with gthr set launch_fill_gthr's init of each row's slots, and
// clears zero[0, nzero) and zero4[0, 4) (when set).
void launch_prep_i8_queries(const double* Q64, const double* mu, double scale, int jx,
                            double limit, const double* cent, int64_t m, int d, int DP,
                            int64_t m_pad, int s, signed char* out, float* valid, hipStream_t st,
                            const int* qperm, uint32_t* gthr, int active, int* zero = nullptr,
                            int64_t nzero = 0, int* zero4 = nullptr);
int pad_dim_i8(int d);  // padded dim of the int8 kernel (a multiple of 64, <= 256), -1 if none
int pad_dim_i8w(int d); // padded dim of the int8 32x32x32 kernel (metric 6), -1 if none
// The reference's exact neighbour order on exact distance ties (knn_select.hip,
// "reference tie order"): libstdc++ std::sort (introsort) emulated over all
// n exact distances of each listed query, restricted to the ranges that
// reach the first k positions.  Per workgroup scratch: tie_scratch_bytes.
constexpr int kFlagTieRef = 32;  // KNN_FLAG_TIE_REF: order resolved as the reference's
int64_t tie_scratch_bytes(int64_t n, int class_cnt);
// totals: device running count of the queries re-ordered (nullable)
void launch_tie_order(int metric, const TrainDev& t, const double* Q64, const int* tie_q,
                      const int* tie_cnt, int class_cnt, unsigned char* scratch, int64_t per_wg,
                      int nwg, const Sink& sink, unsigned long long* totals, hipStream_t s);
// fp64 rows -> [hi(DP) | lo(DP)] bf16 rows of scale*x (candidate metric 2 = L2 via bf16x3)
// rows of `out` are row_shorts 16-bit words; xl2/xl1 (train only, else null)
// fill the padded row's seed floats after the 2*DP bf16 payload
// fp16 images of kernel metric 4 (knn_prep.hip): train rows of DP halves + 4
// seed floats, scaled by 2^jx; query rows of DP halves of -2 * 2^jx (q - mu)
// (zero for queries launch_query_check marked invalid)
// dx2max: running max (u64 bits of a non-negative double) of the rows'
// ||fp16 / 2^jx - (x - mu)||_2^2 (measured representation error)
// swz: store the payload chunks swizzled (xh_swz, knn_device.h)
void launch_prep_half_train(const double* X64, const double* mu, int64_t n, int d, int DP,
                            int64_t n_pad, int jx, unsigned short* out, const float* xl2,
                            unsigned long long* dx2max, int swz, hipStream_t s,
                            const int* perm = nullptr);
// mu <- mu rounded to a multiple of 2^-g (the centre then sits on any data
// grid at least as coarse, so such data is exact in the fp16 operands)
void launch_round_mu(double* mu, int d, int g, hipStream_t s);
void launch_prep_half_queries(const double* Q64, const double* mu, int64_t m, int d, int DP,
                              int64_t m_pad, int jx, unsigned short* out, const float* valid,
                              hipStream_t s, const int* qperm = nullptr);
void launch_prep_split(const double* X64, const double* mu, int64_t n, int d, int DP,
                       int64_t n_pad, double scale, unsigned short* out, int row_shorts,
                       const float* xl2, const float* xl1, hipStream_t s, const int* perm = nullptr);

// Region order (knn_order.hip).  Features are the fp32 operands 2^jx (x - mu).
constexpr int kRegionMax = 64;  // regions (k-means centroids) at most
// out[r] = rank[nearest centroid of row r * stride] (rank null: the centroid)
// Assignment on bf16 MFMA against a centroid image (launch_region_kmeans):
// out[r] = rank[nearest centroid of row r * stride] (rank null: the centroid);
// bcnt (nullable, zeroed): per-1024-row-block key counts
constexpr int kRegionImgBytes = 2 * 16 * 32 * 16 * 2;  // centroid image at d <= 256
void launch_region_assign(const double* X, const double* mu, int64_t n, int d, int64_t stride,
                          int jx, const unsigned short* img, const float* cnorm, const int* rank, int* out,
                          int* bcnt, hipStream_t s);
// k-means over ns sample rows (row i = X row i * stride): cent [P][d], img /
// cnorm the final centroids' bf16 image (kRegionImgBytes) and squared norms
// [kRegionMax], assign [ns] scratch, rank [P] = each centroid's place in the
// greedy chain
void launch_region_kmeans(const double* X, const double* mu, int64_t ns, int d, int64_t stride,
                          int jx, int P, int iters, float* cent, unsigned short* img, float* cnorm,
                          int* assign, int* rank, hipStream_t s);
// Stable counting sort of n keys in [0, kRegionMax): bcnt holds
// region_sort_blocks(n) x kRegionMax ints, tot kRegionMax; outputs (nullable)
// perm[pos] = i, ipos[i] = pos, qstart[pos] = rstart[key] (phases > 0: of
// the first key of the key's group, P keys in `phases` groups), bases[k] =
// the first position of key k
int64_t region_sort_blocks(int64_t n);
void launch_region_sort(const int* key, int64_t n, int* bcnt, int* tot, int* perm, int* ipos,
                        const int* rstart, int* qstart, int* bases, hipStream_t s, int P = 1,
                        int phases = 0);
// Per call: queries assigned to regions and counting-sorted (qperm / qpos /
// qstart as above); bcnt region_sort_blocks(m) x kRegionMax ints, cleared
// first unless bcnt_zero (already zero)
void launch_region_sort_queries(const double* Q, const double* mu, int64_t m, int d, int jx,
                                const unsigned short* img, const float* cnorm, int P, const int* rank,
                                const int* rstart, int phases, int* bcnt, int* tot, int* qkey,
                                int* qperm, int* qpos, int* qstart, hipStream_t s,
                                bool bcnt_zero = false);

// Norm blocks (knn_order.hip): every window of kNormWin image positions
// sorted by the rows' squared norm (int8 code norm with cent, else ||x -
// mu||^2): perm[p] = perm0[source] (perm0 null: train order), ipos inverse;
// key holds n uint32 of scratch.  perm0 must not alias perm / ipos.  il: the
// int8 kernel metric (5 / 6) whose lane lists the norm ranks of each 32-row
// sub-tile are interleaved over (0: sorted order).
constexpr int kNormWin = 16384;
void launch_norm_blocks(const double* X, const double* cent, int s, const double* mu, int64_t n,
                        int d, const int* perm0, uint32_t* key, int* perm, int* ipos, int il,
                        hipStream_t st);
// Int8 images carry, in the pad of row 128u + 1, the largest seed of each of
// the 32-row sub-tiles 4u .. 4u+3 (the seed-free accumulation's bound,
// knn_cand_res.hip)
constexpr int kI8SmaxRow = 1;
// ... and in the pad of row 128u + 2 the largest PARTIAL seed -ceil(||k_A||^2
// / 2) over the first i8_part_dims(DP) dims of the same sub-tiles: the
// metric-6 kernel's early prune after those dims' MFMAs (knn_cand_res.hip,
// KNN_I8_PART).  0 dims: no partial test (the pads get 0, a valid bound).
// Only for 128 <= DP <= 192: at DP = 96 the test after 64 of 96 dims prunes
// too little to pay for its tree (the 12.5M x 96 shard +21 %, ab_log r6r).
constexpr int kI8SmaxARow = 2;
constexpr int i8_part_dims(int DP) { return DP >= 128 && DP <= 192 ? DP - 32 : 0; }

// Min-max normalisation (knn_normalize.hip, cpp:229-306).  R = rows per
// grid sweep; `partial` holds 2*d*R doubles.  launch_minmax folds the set's
// per-dim max/min into out_max/out_min (init: start from -1 / 999999).
int64_t minmax_rows_per_sweep(int64_t rows, int d, int cu_count);
void launch_minmax(const double* X, int64_t rows, int d, int64_t R, double* partial,
                   double* out_max, double* out_min, int init, hipStream_t s);
void launch_normalize_apply(double* X, int64_t rows, int d, int64_t R, const double* vmax,
                            const double* vmin, hipStream_t s);

}  // namespace knnk
