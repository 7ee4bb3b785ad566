// knn_api_internal.h -- context state shared by knn_api.cpp and knn_group.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "knn_kernels.h"

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes);  // grow-only; KNN_OK or KNN_ERR_NOMEM
  void release();
};

// Per-call timing record (ring): events around the phases of one classify /
// search call, read back lazily so a call never waits for the device.
constexpr int kTimingRing = 32;
struct TimedCall {
  hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  bool pending = false;
  int mode = 1;  // knn_set_timing: 1 every phase, 2 the candidate kernel only (ev[1], ev[2])
};

struct knn_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int* h_counts = nullptr;  // pinned, device-mapped: {failed queries, full scans} of the last call
  int* d_counts = nullptr;  // device alias of h_counts
  unsigned long long h_stats[6] = {0, 0, 0, 0, 0, 0};  // train statistics read back at build
  bool trained = false;
  int class_cnt = 0;
  int64_t idx_off = 0;
  int cu_count = 0;
  int precision = 0;     // KNN_PRECISION_*
  int DPb = 0;           // padded dim of the bf16x3 copy (0 = not built)
  int DPh = 0;           // padded dim of the fp16 copy (0 = not built)
  int xh_swz = 0;        // the fp16 copy's chunks are swizzled (xh_swz)
  int DPs = 0;           // padded dim of the fp16 S3 image (0 = not built)
  double xamax = 0.0;    // max |x_i - mu_i| over the train set
  // int8 candidate pass (kernel metric 5): the train values are integer codes
  // x = (cent_i + k) / 2^i8_s, k in [-128, 127] (i8_ok, set at set_train)
  bool i8_ok = false;
  int i8_s = 0;
  int DPi = 0;           // padded dim of the int8 image (0 = not built)
  int i8_swz = 1;        // the int8 image's chunks are swizzled (16x16x64 kernel; 0: 32x32x32)
  double i8_x2max = 0.0; // max ||k||^2 / 2^(2 s) of the image
  bool i8_off = false;   // AUTO: int8 pass retired for this train set
  int auto_kind = 0;     // the pass the pending AUTO decision is about (4 fp16, 5 int8)
  bool fp16_off = false; // AUTO: fp16 candidate pass retired for this train set
                         // (a batch certified too few queries, see knn_run_search)
  // the last call, for the deferred AUTO decision: its completion event,
  // query count and whether it ran the fp16 pass (decided once it completed)
  hipEvent_t done_ev = nullptr;
  bool auto_pending = false;
  int64_t auto_m = 0;
  int tune_R = 0, tune_S = 0;  // 0 = automatic
  int tune_ablate = 0;         // timing-only kernel ablations
  int tune_nw = 0;             // resident kernel waves per workgroup (0 = auto)
  int tune_s3q = -1;           // fp16 S3 on the 16x16x32 layout: -1 auto, 0 off, 1 on
  int tune_qres = -1;          // query-resident fp16 kernel for d > 256 (knn_cand_qres.hip): -1 auto, 0 off
  int tune_gk = -1;            // what the lists publish into gthr (-1 auto, 0 list R-th, 1..16)
  int tune_xhswz = 1;          // fp16 train image chunk swizzle (xh_swz): 1 on, 0 off (A/B)
  int tune_fp16 = -1;          // fp16 candidate pass: -1 auto, 0 off, 1 on
  int tune_i8 = -1;            // int8 candidate pass: -1 auto, 0 off, 1 on (where the data allow)
  int tune_i8w = -1;           // int8 on 32x32x32 (metric 6): -1 auto (where it pads less), 0 off, 1 on
  int tune_ties = 1;           // reference tie order: 0 off, 1 vote-affecting ties, 2 all ties
  int tune_m16 = -1;           // bf16x3 on the 16x16x32 MFMA layout: -1 auto, 0 off, 1 on
  int64_t tune_seed = 0;       // seeded thresholds: 0 / -1 off, N sample rows (experiment)
  // region order (knn_order.hip): -1 auto, 0 off, 1 on, N >= 2 that many
  // regions.  The train layout is decided at set_train; a train set laid out
  // by region still serves calls with 0 (queries in call order, streams
  // starting at each split's first tile).
  int tune_order = -1;
  int ord_P = 0;               // regions of the current train layout (0: train order)
  // norm blocks (knn_order.hip): -1 auto (integer-coded train sets, d <= 256),
  // 0 off, 1 on; ord_nb: the current layout has them (ord_perm / ord_ipos valid)
  int tune_nblk = -1;
  int tune_gg = -1;            // gthr slot groups of the resident kernel: -1 auto, 4 or 8
  int tune_i8resc = -1;        // int8 rescan filter (metric 6): -1 auto (on), 0 off
  int tune_qblk = 0;           // resident kernel workgroup order: 0 split-major, B query blocks
  bool ord_nb = false;
  // ints of ord_bcnt known to be zero (the int8 query builder clears the
  // region sort's block counts after the sort read them; 0: unknown)
  int64_t ord_bcnt_zero = 0;
  int tune_s3gq = 0;           // S3 kernel: largest XCD query-tile grouping (0 = kS3GqMax)
  // query streams start at one of N phases of the region chain (P regions in
  // N groups; -1 auto = 8, 0 = at the query tile's own region)
  int tune_ophase = -1;
  // sample image of the seeding pre-pass (strided train rows in the image
  // format of kernel metric smp_kind at width smp_dp; 0 = not built)
  int smp_kind = 0, smp_dp = 0, smp_swz = -1;
  int64_t smp_n = 0;
  int last_nw = 0;
  int last_kmetric = -1; // candidate kernel metric of the last search (knn_kernels.h)
  char last_kernel[96] = {0};  // name of the last candidate kernel launched
  knnk::TrainDev train{};
  int timing = 0;  // knn_set_timing mode
  TimedCall ring[kTimingRing];
  int ring_next = 0, ring_last = -1;
  double tsum[4] = {0, 0, 0, 0};
  int64_t tcalls = 0;
  int64_t geom[4] = {0, 0, 0, 0};
  // train-side HBM
  DevBuf X64_own, lab_own, X32, xl2, xl1, stats, XB, XS, XH, XT16, XS16, mu, mu_part;
  // int8 image: codes [n_pad][DP + 16 B]; per-dim centres [code units d |
  // value units d] (the latter the merge's mu for this pass); grid stats scratch
  DevBuf XI, i8_cent, i8_gs;
  DevBuf smp_x64, smp_xl2, smp_img, smp_scr, smp_v, smp_i;
  // region order: centroids [P][d], chain ranks, region starts, image
  // position <-> train row maps; k-means / sort scratch; per-call query order
  DevBuf ord_cent, ord_cnorm, ord_img, ord_rank, ord_rstart, ord_perm, ord_ipos, ord_key, ord_bcnt, ord_tot, ord_qkey,
      ord_qperm, ord_qpos, ord_qstart, ord_perm0;
  // per-classify workspace
  DevBuf Q64, Q32, qvalid, cand_v, cand_i, gthr, rescan_q, rescan_tau, rescan_cnt, fr_cnt, fr_buf,
      fr_q, fr_thr, slow_q, totals, lk, rescan_mask, rescan_nkeep, rescan_qc8, rescan_t8;
  // train-sharded merge of unions beyond 4096 entries (rank merge scratch)
  DevBuf mrg;
  // reference tie order pass: queued queries, per-workgroup scratch
  DevBuf tie_q, tie_ws;
  // host-API outputs
  DevBuf o_lab, o_idx, o_dist, o_flags;
  // normalisation: per-thread partial max/min, bounds, host-API staging
  DevBuf nrm_part, nrm_mm, nrm_X;
  std::vector<DevBuf*> all_bufs() {
    return {&X64_own, &lab_own, &X32,   &xl2,   &xl1,    &stats,  &XB,       &XS, &XI, &i8_cent, &i8_gs,
            &XH,      &XT16,    &XS16,  &mu,      &mu_part, &Q64, &Q32,    &qvalid, &cand_v,   &cand_i,
            &gthr,    &rescan_q, &rescan_tau, &rescan_cnt, &fr_cnt, &fr_buf, &fr_q, &fr_thr,
            &slow_q,  &totals,  &lk, &mrg, &tie_q, &tie_ws, &o_lab, &o_idx, &o_dist, &o_flags, &nrm_part, &nrm_mm, &nrm_X,
            &rescan_mask, &rescan_nkeep, &rescan_qc8, &rescan_t8, &smp_x64, &smp_xl2, &smp_img, &smp_scr, &smp_v, &smp_i,
            &ord_cent, &ord_cnorm, &ord_img, &ord_rank, &ord_rstart, &ord_perm, &ord_ipos, &ord_key, &ord_bcnt, &ord_tot,
            &ord_qkey, &ord_qperm, &ord_qpos, &ord_qstart, &ord_perm0};
  }
};

int knn_fail(int code, const std::string& msg);
int knn_run_search(knn_ctx* ctx, const double* dQ, int64_t m, int W, int metric,
                   const knnk::Sink& sink, hipStream_t s);
