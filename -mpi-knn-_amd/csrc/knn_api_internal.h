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

struct knn_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int* h_count = nullptr;  // pinned
  unsigned long long h_stats[4] = {0, 0, 0, 0};  // train statistics read back at build
  bool trained = false;
  int class_cnt = 0;
  int64_t idx_off = 0;
  int64_t last_rescan = 0;       // queries that failed certification
  int64_t last_slow_rescan = 0;  // of those, queries the fast rescan passed on to the full scan
  int cu_count = 0;
  int precision = 0;     // KNN_PRECISION_*
  int DPb = 0;           // padded dim of the bf16x3 copy (0 = not built)
  int DPh = 0;           // padded dim of the fp16 copy (0 = not built)
  double xamax = 0.0;    // max |x_i - mu_i| over the train set
  bool fp16_off = false; // AUTO: fp16 candidate pass retired for this train set
                         // (a batch certified too few queries, see knn_run_search)
  int tune_R = 0, tune_S = 0;  // 0 = automatic
  int tune_ablate = 0;         // timing-only kernel ablations
  int tune_nw = 0;             // resident kernel waves per workgroup (0 = auto)
  int tune_fp16 = -1;          // fp16 candidate pass: -1 auto, 0 off, 1 on
  int tune_f16l = -1;          // fp16 MFMA layout: -1 auto, 0 16x16, 1 16x16 wide, 2 32x32
  int tune_m16 = -1;           // bf16x3 on the 16x16x32 MFMA layout: -1 auto, 0 off, 1 on
  int last_nw = 0;
  int last_kmetric = -1; // candidate kernel metric of the last search (knn_kernels.h)
  knnk::TrainDev train{};
  bool timing = false;
  hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  double phase_ms[4] = {0, 0, 0, 0};
  int64_t geom[4] = {0, 0, 0, 0};
  // train-side HBM
  DevBuf X64_own, lab_own, X32, xl2, xl1, stats, XB, XS, XH, mu, mu_part;
  // per-classify workspace
  DevBuf Q64, Q32, qvalid, cand_v, cand_i, gthr, rescan_q, rescan_tau, rescan_cnt, ra_k, ra_i, rb_k,
      rb_i, fr_cnt, fr_buf, fr_q, slow_q;
  // host-API outputs
  DevBuf o_lab, o_idx, o_dist, o_flags;
  // normalisation: per-thread partial max/min, bounds, host-API staging
  DevBuf nrm_part, nrm_mm, nrm_X;
  std::vector<DevBuf*> all_bufs() {
    return {&X64_own, &lab_own, &X32, &xl2, &xl1, &stats, &XB, &XS, &XH, &mu, &mu_part, &Q64, &Q32, &qvalid, &cand_v, &cand_i, &gthr, &rescan_tau, &fr_cnt, &fr_buf, &fr_q, &slow_q,
            &rescan_q, &rescan_cnt, &ra_k, &ra_i, &rb_k, &rb_i, &o_lab, &o_idx, &o_dist,
            &o_flags, &nrm_part, &nrm_mm, &nrm_X};
  }
};

int knn_fail(int code, const std::string& msg);
int knn_run_search(knn_ctx* ctx, const double* dQ, int64_t m, int W, int metric,
                   const knnk::Sink& sink, hipStream_t s);
