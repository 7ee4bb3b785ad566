// knn_group.cpp -- single-process multi-GPU driver over RCCL (xGMI).
//
// Replaces the reference's MPI decomposition (cpp:136-138, 224-227, 340, 383)
// with the two single-node modes of the north star:
//   mode 0, query-sharded: train rows + labels are ncclBroadcast from the
//     first GPU to all (≙ MPI_Bcast cpp:224-225); queries are split into
//     contiguous (ragged-allowed) shards (≙ MPI_Scatter cpp:226-227); each
//     GPU classifies its shard; labels land in one host array (≙ MPI_Gather
//     cpp:340/383).  No data-path collective after the broadcast.
//   mode 1, train-sharded: GPU g holds rows [n*g/G, n*(g+1)/G); queries are
//     broadcast; each GPU computes its exact local top-(k+1) (with global
//     indices and labels); ncclAllGather exchanges the lists; GPU g k-way
//     merges and votes queries [m*g/G, m*(g+1)/G).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "../../include/knn_amd.h"
#include "knn_api_internal.h"
#include "knn_kernels.h"

struct knn_group {
  int ndev = 0;
  int mode = 0;
  std::vector<int> devs;
  std::vector<knn_ctx*> ctx;
  std::vector<ncclComm_t> comms;
  std::vector<DevBuf> X, lab;                  // per-device train rows (full or shard)
  std::vector<DevBuf> Q, olab, oidx, odist, oflags;
  std::vector<DevBuf> pk, gk;                  // train-sharded packed partial / gathered lists
  std::vector<DevBuf> nX, nmm;                 // normalisation shards / per-dim bounds
  std::vector<hipEvent_t> ev0, ev1;            // per device: around the last call's device work
  int64_t n = 0;
  int d = 0;
  int class_cnt = 0;
  bool trained = false;
  double last_compute = 0.0;
};

#define HIP_G(expr)                                                                       \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return knn_fail(KNN_ERR_DEVICE, std::string(#expr " failed: ") + hipGetErrorString(e_)); \
  } while (0)
#define NCCL_G(expr)                                                                      \
  do {                                                                                    \
    ncclResult_t r_ = (expr);                                                             \
    if (r_ != ncclSuccess)                                                                \
      return knn_fail(KNN_ERR_COMM, std::string(#expr " failed: ") + ncclGetErrorString(r_)); \
  } while (0)

// Runs f(g) for every device in its own host thread; first non-zero rc wins.
template <class F>
static int for_each_dev(knn_group* g, F f) {
  std::vector<int> rc(g->ndev, 0);
  std::vector<std::string> err(g->ndev);
  std::vector<std::thread> th;
  for (int i = 0; i < g->ndev; i++)
    th.emplace_back([&, i] {
      (void)hipSetDevice(g->devs[i]);
      rc[i] = f(i);
      if (rc[i]) err[i] = knn_last_error();
    });
  for (auto& t : th) t.join();
  for (int i = 0; i < g->ndev; i++)
    if (rc[i]) return knn_fail(rc[i], "device " + std::to_string(g->devs[i]) + ": " + err[i]);
  return KNN_OK;
}

extern "C" {

int knn_group_create(knn_group** out, int ndev, const int* devs, int mode) {
  if (!out || ndev <= 0 || (mode != 0 && mode != 1))
    return knn_fail(KNN_ERR_ARG, "bad group arguments");
  *out = nullptr;
  knn_group* g = new knn_group();
  g->ndev = ndev;
  g->mode = mode;
  for (int i = 0; i < ndev; i++) g->devs.push_back(devs ? devs[i] : i);
  g->ctx.assign(ndev, nullptr);
  for (int i = 0; i < ndev; i++) {
    int rc = knn_create(&g->ctx[i], g->devs[i]);
    if (rc) {
      knn_group_destroy(g);
      return rc;
    }
  }
  g->comms.assign(ndev, nullptr);
  if (ndev > 1) {
    ncclResult_t r = ncclCommInitAll(g->comms.data(), ndev, g->devs.data());
    if (r != ncclSuccess) {
      g->comms.clear();
      knn_group_destroy(g);
      return knn_fail(KNN_ERR_COMM, std::string("ncclCommInitAll failed: ") + ncclGetErrorString(r));
    }
  }
  for (auto* v : {&g->X, &g->lab, &g->Q, &g->olab, &g->oidx, &g->odist, &g->oflags, &g->pk,
                  &g->gk, &g->nX, &g->nmm})
    v->resize(ndev);
  g->ev0.assign(ndev, nullptr);
  g->ev1.assign(ndev, nullptr);
  for (int i = 0; i < ndev; i++) {
    if (hipSetDevice(g->devs[i]) != hipSuccess || hipEventCreate(&g->ev0[i]) != hipSuccess ||
        hipEventCreate(&g->ev1[i]) != hipSuccess) {
      knn_group_destroy(g);
      return knn_fail(KNN_ERR_DEVICE, "hipEventCreate failed");
    }
  }
  *out = g;
  return KNN_OK;
}

int knn_group_destroy(knn_group* g) {
  if (!g) return KNN_OK;
  for (int i = 0; i < g->ndev; i++) {
    if (i < (int)g->ctx.size() && g->ctx[i]) {
      (void)hipSetDevice(g->devs[i]);
      (void)hipDeviceSynchronize();
    }
    for (auto* v : {&g->X, &g->lab, &g->Q, &g->olab, &g->oidx, &g->odist, &g->oflags, &g->pk,
                    &g->gk, &g->nX, &g->nmm})
      if (i < (int)v->size()) (*v)[i].release();
    for (auto* ev : {&g->ev0, &g->ev1})
      if (i < (int)ev->size() && (*ev)[i]) (void)hipEventDestroy((*ev)[i]);
  }
  for (auto c : g->comms)
    if (c) ncclCommDestroy(c);
  for (auto* c : g->ctx)
    if (c) knn_destroy(c);
  delete g;
  return KNN_OK;
}

int knn_group_set_train(knn_group* g, const double* X, const int32_t* labels, int64_t n,
                        int32_t d, int32_t class_cnt) {
  if (!g || !X || !labels || n <= 0 || d <= 0 || class_cnt <= 0)
    return knn_fail(KNN_ERR_ARG, "bad train arguments");
  for (int64_t i = 0; i < n; i++)
    if (labels[i] < 0 || labels[i] >= class_cnt)
      return knn_fail(KNN_ERR_ARG, "train label out of [0, class_cnt) at row " + std::to_string(i));
  g->n = n;
  g->d = d;
  g->class_cnt = class_cnt;
  const int G = g->ndev;
  if (g->mode == 0) {
    // root copy on the first GPU, then RCCL broadcast over xGMI (cpp:224-225)
    for (int i = 0; i < G; i++) {
      HIP_G(hipSetDevice(g->devs[i]));
      int rc;
      if ((rc = g->X[i].ensure((size_t)n * d * sizeof(double)))) return rc;
      if ((rc = g->lab[i].ensure((size_t)n * sizeof(int32_t)))) return rc;
    }
    HIP_G(hipSetDevice(g->devs[0]));
    HIP_G(hipMemcpyAsync(g->X[0].p, X, (size_t)n * d * sizeof(double), hipMemcpyHostToDevice,
                         g->ctx[0]->stream));
    HIP_G(hipMemcpyAsync(g->lab[0].p, labels, (size_t)n * sizeof(int32_t),
                         hipMemcpyHostToDevice, g->ctx[0]->stream));
    if (G > 1) {
      NCCL_G(ncclGroupStart());
      for (int i = 0; i < G; i++) {
        NCCL_G(ncclBroadcast(g->X[0].p, g->X[i].p, (size_t)n * d, ncclFloat64, 0, g->comms[i],
                             g->ctx[i]->stream));
        NCCL_G(ncclBroadcast(g->lab[0].p, g->lab[i].p, (size_t)n, ncclInt32, 0, g->comms[i],
                             g->ctx[i]->stream));
      }
      NCCL_G(ncclGroupEnd());
    }
    int rc = for_each_dev(g, [&](int i) {
      return knn_set_train_device(g->ctx[i], (const double*)g->X[i].p,
                                  (const int32_t*)g->lab[i].p, n, d, class_cnt, 0);
    });
    if (rc) return rc;
  } else {
    // train-sharded: contiguous row shards, global index offsets
    int rc = for_each_dev(g, [&](int i) {
      const int64_t r0 = n * i / G, r1 = n * (i + 1) / G;
      const int64_t ni = r1 - r0;
      if (ni <= 0) return knn_fail(KNN_ERR_ARG, "more GPUs than train rows");
      int e;
      if ((e = g->X[i].ensure((size_t)ni * d * sizeof(double)))) return e;
      if ((e = g->lab[i].ensure((size_t)ni * sizeof(int32_t)))) return e;
      hipStream_t s = g->ctx[i]->stream;
      if (hipMemcpyAsync(g->X[i].p, X + r0 * d, (size_t)ni * d * sizeof(double),
                         hipMemcpyHostToDevice, s) != hipSuccess ||
          hipMemcpyAsync(g->lab[i].p, labels + r0, (size_t)ni * sizeof(int32_t),
                         hipMemcpyHostToDevice, s) != hipSuccess)
        return knn_fail(KNN_ERR_DEVICE, "H2D of train shard failed");
      return knn_set_train_device(g->ctx[i], (const double*)g->X[i].p,
                                  (const int32_t*)g->lab[i].p, ni, d, class_cnt, r0);
    });
    if (rc) return rc;
  }
  g->trained = true;
  return KNN_OK;
}

int knn_group_classify(knn_group* g, const double* Q, int64_t m, int32_t k, int32_t metric,
                       int32_t* out_labels, int64_t* out_idx, double* out_dist,
                       int32_t* out_flags) {
  if (!g || !g->trained) return knn_fail(KNN_ERR_STATE, "group classify before set_train");
  if (m < 0 || !out_labels || (m > 0 && !Q)) return knn_fail(KNN_ERR_ARG, "bad classify arguments");
  if (k < 0 || k > g->n) return knn_fail(KNN_ERR_ARG, "bad k");
  if (m == 0) return KNN_OK;
  const int G = g->ndev;
  const int d = g->d;
  // Every step of a call is enqueued from this thread on the devices'
  // context streams (H2D, compute, collectives, D2H: all asynchronous) and
  // the host waits once per device at the end; the compute span is read
  // from events around the device work (max over devices).
  auto slice = [&](int i, int64_t& q0, int64_t& mi) {
    q0 = m * i / G;
    mi = m * (i + 1) / G - q0;
  };
  auto d2h = [&](int i, int64_t q0, int64_t mi) -> int {
    hipStream_t s = g->ctx[i]->stream;
    HIP_G(hipMemcpyAsync(out_labels + q0, g->olab[i].p, mi * sizeof(int32_t),
                         hipMemcpyDeviceToHost, s));
    if (out_flags)
      HIP_G(hipMemcpyAsync(out_flags + q0, g->oflags[i].p, mi * sizeof(int32_t),
                           hipMemcpyDeviceToHost, s));
    if (out_idx && k > 0)
      HIP_G(hipMemcpyAsync(out_idx + q0 * k, g->oidx[i].p, mi * k * sizeof(int64_t),
                           hipMemcpyDeviceToHost, s));
    if (out_dist && k > 0)
      HIP_G(hipMemcpyAsync(out_dist + q0 * k, g->odist[i].p, mi * k * sizeof(double),
                           hipMemcpyDeviceToHost, s));
    return KNN_OK;
  };
  auto finish = [&]() -> int {
    double span = 0.0;
    for (int i = 0; i < G; i++) {
      HIP_G(hipSetDevice(g->devs[i]));
      HIP_G(hipStreamSynchronize(g->ctx[i]->stream));
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, g->ev0[i], g->ev1[i]) == hipSuccess)
        span = std::max(span, (double)ms * 1e-3);
    }
    g->last_compute = span;
    return KNN_OK;
  };
  int rc;
  if (g->mode == 0) {
    // query shards: [m*i/G, m*(i+1)/G)  (ragged shards allowed, unlike cpp:127-129)
    for (int i = 0; i < G; i++) {
      int64_t q0, mi;
      slice(i, q0, mi);
      HIP_G(hipSetDevice(g->devs[i]));
      hipStream_t s = g->ctx[i]->stream;
      if (mi <= 0) {
        HIP_G(hipEventRecord(g->ev0[i], s));
        HIP_G(hipEventRecord(g->ev1[i], s));
        continue;
      }
      if ((rc = g->Q[i].ensure((size_t)mi * d * sizeof(double)))) return rc;
      if ((rc = g->olab[i].ensure((size_t)mi * sizeof(int32_t)))) return rc;
      if ((rc = g->oflags[i].ensure((size_t)mi * sizeof(int32_t)))) return rc;
      if ((rc = g->oidx[i].ensure((size_t)mi * std::max(k, 1) * sizeof(int64_t)))) return rc;
      if ((rc = g->odist[i].ensure((size_t)mi * std::max(k, 1) * sizeof(double)))) return rc;
      HIP_G(hipMemcpyAsync(g->Q[i].p, Q + q0 * d, (size_t)mi * d * sizeof(double),
                           hipMemcpyHostToDevice, s));
      HIP_G(hipEventRecord(g->ev0[i], s));
      if ((rc = knn_classify_device(g->ctx[i], (const double*)g->Q[i].p, mi, k, metric,
                                    (int32_t*)g->olab[i].p,
                                    out_idx ? (int64_t*)g->oidx[i].p : nullptr,
                                    out_dist ? (double*)g->odist[i].p : nullptr,
                                    (int32_t*)g->oflags[i].p, s)))
        return rc;
      HIP_G(hipEventRecord(g->ev1[i], s));
    }
    // the copies back only once every device has its work queued (a copy
    // into pageable host memory may hold this thread until it completes)
    for (int i = 0; i < G; i++) {
      int64_t q0, mi;
      slice(i, q0, mi);
      HIP_G(hipSetDevice(g->devs[i]));
      if (mi > 0 && (rc = d2h(i, q0, mi))) return rc;
    }
    return finish();
  }

  // ---- train-sharded
  if (k == 0) {
    for (int64_t q = 0; q < m; q++) out_labels[q] = -1;
    if (out_flags)
      for (int64_t q = 0; q < m; q++) out_flags[q] = 0;
    return KNN_OK;
  }
  // each GPU's exact local top-w (w <= its shard: padded with idx -1); any
  // K <= N_train like cpp:328 (unions beyond 4096 entries: the rank merge)
  const int w = (int)std::min<int64_t>((int64_t)k + 1, g->n);
  const int64_t PB = knnk::packed_part_bytes(m, w);
  for (int i = 0; i < G; i++) {
    int64_t q0, mi;
    slice(i, q0, mi);
    HIP_G(hipSetDevice(g->devs[i]));
    if ((rc = g->Q[i].ensure((size_t)m * d * sizeof(double)))) return rc;
    // this GPU's lists packed [dist | idx | label] (one all-gather per step)
    if ((rc = g->pk[i].ensure((size_t)PB))) return rc;
    if (G > 1 && (rc = g->gk[i].ensure((size_t)G * PB))) return rc;
    if ((rc = g->olab[i].ensure((size_t)std::max<int64_t>(mi, 1) * sizeof(int32_t)))) return rc;
    if ((rc = g->oflags[i].ensure((size_t)std::max<int64_t>(mi, 1) * sizeof(int32_t)))) return rc;
    if ((rc = g->oidx[i].ensure((size_t)std::max<int64_t>(mi, 1) * k * sizeof(int64_t)))) return rc;
    if ((rc = g->odist[i].ensure((size_t)std::max<int64_t>(mi, 1) * k * sizeof(double)))) return rc;
    if (const int64_t sb = knnk::merge_scratch_bytes(G, w, k, mi))
      if ((rc = g->ctx[i]->mrg.ensure((size_t)sb))) return rc;
  }
  // queries to the first GPU, RCCL broadcast to the rest
  HIP_G(hipSetDevice(g->devs[0]));
  HIP_G(hipMemcpyAsync(g->Q[0].p, Q, (size_t)m * d * sizeof(double), hipMemcpyHostToDevice,
                       g->ctx[0]->stream));
  for (int i = 0; i < G; i++) {
    HIP_G(hipSetDevice(g->devs[i]));
    HIP_G(hipEventRecord(g->ev0[i], g->ctx[i]->stream));
  }
  if (G > 1) {
    NCCL_G(ncclGroupStart());
    for (int i = 0; i < G; i++)
      NCCL_G(ncclBroadcast(g->Q[0].p, g->Q[i].p, (size_t)m * d, ncclFloat64, 0, g->comms[i],
                           g->ctx[i]->stream));
    NCCL_G(ncclGroupEnd());
  }
  for (int i = 0; i < G; i++) {
    unsigned char* pb = (unsigned char*)g->pk[i].p;
    if ((rc = knn_search_partial_device(g->ctx[i], (const double*)g->Q[i].p, m, w, metric,
                                        (double*)pb, (int64_t*)(pb + 8 * m * w),
                                        (int32_t*)(pb + 16 * m * w), nullptr)))
      return rc;
  }
  if (G > 1) {  // one all-gather of the packed lists (≙ the reference's MPI_Gather, cpp:340)
    NCCL_G(ncclGroupStart());
    for (int i = 0; i < G; i++)
      NCCL_G(ncclAllGather(g->pk[i].p, g->gk[i].p, (size_t)PB, ncclUint8, g->comms[i],
                           g->ctx[i]->stream));
    NCCL_G(ncclGroupEnd());
  }
  for (int i = 0; i < G; i++) {
    int64_t q0, mi;
    slice(i, q0, mi);
    HIP_G(hipSetDevice(g->devs[i]));
    hipStream_t s = g->ctx[i]->stream;
    if (mi > 0) {
      const double* sk = (const double*)(G > 1 ? g->gk[i].p : g->pk[i].p);
      knnk::launch_merge_vote_partials(sk, nullptr, nullptr, G, m, w, k, (int32_t*)g->olab[i].p,
                                       (int64_t*)g->oidx[i].p, (double*)g->odist[i].p,
                                       (int32_t*)g->oflags[i].p, s, q0, mi, PB, g->ctx[i]->mrg.p);
      HIP_G(hipGetLastError());
    }
    HIP_G(hipEventRecord(g->ev1[i], s));
  }
  for (int i = 0; i < G; i++) {
    int64_t q0, mi;
    slice(i, q0, mi);
    HIP_G(hipSetDevice(g->devs[i]));
    if (mi > 0 && (rc = d2h(i, q0, mi))) return rc;
  }
  return finish();
}

double knn_group_last_compute_seconds(knn_group* g) { return g ? g->last_compute : -1.0; }

int knn_group_normalize(knn_group* g, double* const* sets, const int64_t* rows, int32_t nsets,
                        int32_t d) {
  if (!g || nsets < 0 || d <= 0 || (nsets > 0 && (!sets || !rows)))
    return knn_fail(KNN_ERR_ARG, "bad normalize arguments");
  for (int s = 0; s < nsets; s++)
    if (rows[s] < 0 || (rows[s] > 0 && !sets[s])) return knn_fail(KNN_ERR_ARG, "bad set");
  const int G = g->ndev;
  // shard s of device i: rows [rows[s]*i/G, rows[s]*(i+1)/G) (≙ the rank's
  // batch_train / batch_test / batch_val rows, cpp:245-274)
  auto shard = [&](int s, int i, int64_t& r0, int64_t& r1) {
    r0 = rows[s] * i / G;
    r1 = rows[s] * (i + 1) / G;
  };
  int rc = for_each_dev(g, [&](int i) {
    int64_t total = 0, r0, r1;
    for (int s = 0; s < nsets; s++) {
      shard(s, i, r0, r1);
      total += r1 - r0;
    }
    int e;
    if ((e = g->nX[i].ensure((size_t)std::max<int64_t>(total, 1) * d * sizeof(double)))) return e;
    if ((e = g->nmm[i].ensure((size_t)2 * d * sizeof(double)))) return e;
    knn_ctx* c = g->ctx[i];
    double* mx = (double*)g->nmm[i].p;
    int64_t off = 0;
    for (int s = 0; s < nsets; s++) {
      shard(s, i, r0, r1);
      double* dX = (double*)g->nX[i].p + off * d;
      if (r1 > r0 && hipMemcpyAsync(dX, sets[s] + r0 * d, (size_t)(r1 - r0) * d * sizeof(double),
                                    hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return knn_fail(KNN_ERR_DEVICE, "H2D of normalisation shard failed");
      if ((e = knn_minmax_device(c, dX, r1 - r0, d, mx, mx + d, s == 0, nullptr))) return e;
      off += r1 - r0;
    }
    if (nsets == 0) return knn_minmax_device(c, nullptr, 0, d, mx, mx + d, 1, nullptr);
    return KNN_OK;
  });
  if (rc) return rc;
  if (G > 1) {  // ≙ MPI_Allreduce MAX / MIN, cpp:276-277
    NCCL_G(ncclGroupStart());
    for (int i = 0; i < G; i++) {
      double* mx = (double*)g->nmm[i].p;
      NCCL_G(ncclAllReduce(mx, mx, d, ncclFloat64, ncclMax, g->comms[i], g->ctx[i]->stream));
      NCCL_G(ncclAllReduce(mx + d, mx + d, d, ncclFloat64, ncclMin, g->comms[i],
                           g->ctx[i]->stream));
    }
    NCCL_G(ncclGroupEnd());
  }
  return for_each_dev(g, [&](int i) {  // cpp:279-305 on each shard, back to the host
    knn_ctx* c = g->ctx[i];
    const double* mx = (const double*)g->nmm[i].p;
    int64_t off = 0, r0, r1;
    for (int s = 0; s < nsets; s++) {
      shard(s, i, r0, r1);
      double* dX = (double*)g->nX[i].p + off * d;
      int e;
      if ((e = knn_normalize_device(c, dX, r1 - r0, d, mx, mx + d, nullptr))) return e;
      if (r1 > r0 && hipMemcpyAsync(sets[s] + r0 * d, dX, (size_t)(r1 - r0) * d * sizeof(double),
                                    hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        return knn_fail(KNN_ERR_DEVICE, "D2H of normalised shard failed");
      off += r1 - r0;
    }
    return hipStreamSynchronize(c->stream) == hipSuccess
               ? KNN_OK
               : knn_fail(KNN_ERR_DEVICE, "normalisation failed");
  });
}

}  // extern "C"
