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
//     merges and votes queries [m*g/G, m*(g+1)/G).  Queries whose label the
//     reference's order among equal distances decides (its std::sort over
//     the whole train set, cpp:366) are rare: their exact distances to every
//     shard's rows go to the owner by ncclSend/ncclRecv, which re-sorts them
//     as the reference does (knn_tie_resolve_device).
// Transport (knn_group_transport): RCCL between distinct devices, also at
// G = 1 on request (KNN_GROUP_RCCL: a one-rank communicator, every
// collective of the path through RCCL); ranks sharing a device (repeated
// entries in devs) exchange by stream-ordered device copies ("loopback"):
// the whole G-rank decomposition, offsets and merges on fewer GPUs.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/knn_amd.h"
#include "knn_api_internal.h"
#include "knn_kernels.h"

enum { XPORT_NONE = 0, XPORT_RCCL = 1, XPORT_LOOPBACK = 2 };

struct knn_group {
  int ndev = 0;
  int mode = 0;
  int transport = XPORT_NONE;
  std::vector<int> devs;
  std::vector<knn_ctx*> ctx;
  std::vector<ncclComm_t> comms;
  std::vector<DevBuf> X, lab;                  // per-device train rows (full or shard)
  std::vector<DevBuf> labA;                    // mode 1: every train label (reference tie order)
  std::vector<DevBuf> Q, olab, oidx, odist, oflags;
  std::vector<DevBuf> pk, gk;                  // train-sharded packed partial / gathered lists
  std::vector<DevBuf> tq, tcnt, tsel, trow, tsend, trecv;  // reference tie order exchange
  std::vector<DevBuf> nX, nmm;                 // normalisation shards / per-dim bounds
  std::vector<hipEvent_t> ev0, ev1;            // per device: around the last call's device work
  std::vector<hipEvent_t> evx;                 // loopback: cross-rank stream ordering
  int64_t n = 0;
  int d = 0;
  int class_cnt = 0;
  bool trained = false;
  double last_compute = 0.0;
  int64_t last_ties = 0;                       // mode 1: queries resolved by the exchange (last call)
};

#define HIP_G(expr)                                                                       \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return knn_fail(KNN_ERR_DEVICE, std::string(#expr " failed: ") + hipGetErrorString(e_)); \
  } while (0)
// An RCCL failure names the call, the collective it belongs to and the ranks
// (and devices) involved: a G > 1 failure on the first multi-GPU run must be
// attributable from its message alone (the driver exits 1 with it).
#define NCCL_G(expr) NCCL_AT(expr, std::string())
#define NCCL_AT(expr, where)                                                              \
  do {                                                                                    \
    ncclResult_t r_ = (expr);                                                             \
    if (r_ != ncclSuccess)                                                                \
      return knn_fail(KNN_ERR_COMM, std::string(#expr " failed") + (where) + ": " +      \
                                        ncclGetErrorString(r_));                           \
  } while (0)

// " in <what>, rank i (device d) of G" / " in <what>, ranks 0..G-1 (devices ...)"
static std::string ranks_of(const knn_group* g, const char* what, int i = -1);

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

static hipStream_t stream_of(knn_group* g, int i) { return g->ctx[i]->stream; }

// Waits for rank i's stream.  With RCCL the wait polls: an asynchronous RCCL
// error on any rank, or no progress within KNN_GROUP_TIMEOUT_S seconds
// (default 600), aborts the communicators and fails naming the step and the
// rank -- a hang of a G > 1 collective ends the driver (exit 1) instead of
// holding the GPUs.
static int sync_rank(knn_group* g, int i, const char* what) {
  if (hipSetDevice(g->devs[i]) != hipSuccess)
    return knn_fail(KNN_ERR_DEVICE, std::string("hipSetDevice failed") + ranks_of(g, what, i));
  hipStream_t st = stream_of(g, i);
  if (g->transport != XPORT_RCCL) {
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess)
      return knn_fail(KNN_ERR_DEVICE, std::string("stream of ") + ranks_of(g, what, i).substr(4) +
                                          " failed: " + hipGetErrorString(e));
    return KNN_OK;
  }
  static const double limit = [] {
    const char* e = getenv("KNN_GROUP_TIMEOUT_S");
    const double v = e ? atof(e) : 0.0;
    return v > 0 ? v : 600.0;
  }();
  const auto t0 = std::chrono::steady_clock::now();
  for (int polls = 0;; ++polls) {
    hipError_t e = hipStreamQuery(st);
    if (e == hipSuccess) return KNN_OK;
    if (e != hipErrorNotReady)
      return knn_fail(KNN_ERR_DEVICE, std::string("stream of ") + ranks_of(g, what, i).substr(4) +
                                          " failed: " + hipGetErrorString(e));
    for (int r = 0; r < g->ndev; r++) {
      ncclResult_t ae = ncclSuccess;
      if (g->comms[r] && ncclCommGetAsyncError(g->comms[r], &ae) == ncclSuccess &&
          ae != ncclSuccess && ae != ncclInProgress) {
        for (auto c : g->comms)
          if (c) ncclCommAbort(c);
        g->comms.assign(g->ndev, nullptr);
        return knn_fail(KNN_ERR_COMM, std::string("RCCL asynchronous error") + ranks_of(g, what, r) +
                                          ": " + ncclGetErrorString(ae));
      }
    }
    const double el =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > limit) {
      for (auto c : g->comms)
        if (c) ncclCommAbort(c);
      g->comms.assign(g->ndev, nullptr);
      return knn_fail(KNN_ERR_COMM, "no progress for " + std::to_string((int)el) +
                                        " s waiting for" + ranks_of(g, what, i).substr(3) +
                                        " (communicators aborted; KNN_GROUP_TIMEOUT_S)");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(polls < 1000 ? 20 : 200));
  }
}

static std::string ranks_of(const knn_group* g, const char* what, int i) {
  std::string s = std::string(" in ") + what + ", ";
  if (i >= 0)
    return s + "rank " + std::to_string(i) + " (device " + std::to_string(g->devs[i]) + ") of " +
           std::to_string(g->ndev);
  s += "ranks 0.." + std::to_string(g->ndev - 1) + " (devices";
  for (int d : g->devs) s += " " + std::to_string(d);
  return s + ")";
}

// ---- collectives of the group (one call covers every rank)

// loopback: every rank's stream waits for what every other rank's stream
// has queued so far (before a copy: its sources are complete; after: no
// rank overwrites a source another rank is still reading)
static int lb_barrier(knn_group* g) {
  for (int i = 0; i < g->ndev; i++) {
    HIP_G(hipSetDevice(g->devs[i]));
    HIP_G(hipEventRecord(g->evx[i], stream_of(g, i)));
  }
  for (int i = 0; i < g->ndev; i++) {
    HIP_G(hipSetDevice(g->devs[i]));
    for (int j = 0; j < g->ndev; j++)
      if (j != i) HIP_G(hipStreamWaitEvent(stream_of(g, i), g->evx[j], 0));
  }
  return KNN_OK;
}

// buf[i] <- buf[root] for every rank i (count elements of `type`, esize B each)
static int coll_bcast(knn_group* g, const std::vector<void*>& buf, size_t count,
                      ncclDataType_t type, size_t esize, int root) {
  if (g->transport == XPORT_RCCL) {
    NCCL_AT(ncclGroupStart(), ranks_of(g, "broadcast"));
    for (int i = 0; i < g->ndev; i++)
      NCCL_AT(ncclBroadcast(buf[root], buf[i], count, type, root, g->comms[i], stream_of(g, i)),
              ranks_of(g, "broadcast", i));
    NCCL_AT(ncclGroupEnd(), ranks_of(g, "broadcast"));
  } else if (g->transport == XPORT_LOOPBACK) {
    int rc;
    if ((rc = lb_barrier(g))) return rc;
    for (int i = 0; i < g->ndev; i++) {
      if (i == root) continue;
      HIP_G(hipSetDevice(g->devs[i]));
      HIP_G(hipMemcpyAsync(buf[i], buf[root], count * esize, hipMemcpyDeviceToDevice,
                           stream_of(g, i)));
    }
    return lb_barrier(g);
  }
  return KNN_OK;
}

// recv[i][j * bytes ..] <- send[j] for every rank pair
static int coll_allgather(knn_group* g, const std::vector<void*>& send,
                          const std::vector<void*>& recv, size_t bytes) {
  if (g->transport == XPORT_RCCL) {
    NCCL_AT(ncclGroupStart(), ranks_of(g, "all-gather"));
    for (int i = 0; i < g->ndev; i++)
      NCCL_AT(ncclAllGather(send[i], recv[i], bytes, ncclUint8, g->comms[i], stream_of(g, i)),
              ranks_of(g, "all-gather", i));
    NCCL_AT(ncclGroupEnd(), ranks_of(g, "all-gather"));
  } else if (g->transport == XPORT_LOOPBACK) {
    int rc;
    if ((rc = lb_barrier(g))) return rc;
    for (int i = 0; i < g->ndev; i++) {
      HIP_G(hipSetDevice(g->devs[i]));
      for (int j = 0; j < g->ndev; j++)
        HIP_G(hipMemcpyAsync((unsigned char*)recv[i] + j * bytes, send[j], bytes,
                             hipMemcpyDeviceToDevice, stream_of(g, i)));
    }
    return lb_barrier(g);
  }
  return KNN_OK;
}

// mm[i] = [max | min] (2d doubles): MAX over ranks of the first d, MIN of the
// rest (≙ the two MPI_Allreduce of cpp:276-277)
static int coll_allreduce_maxmin(knn_group* g, const std::vector<double*>& mm, int d) {
  if (g->transport == XPORT_RCCL) {
    NCCL_AT(ncclGroupStart(), ranks_of(g, "normalisation all-reduce"));
    for (int i = 0; i < g->ndev; i++) {
      NCCL_AT(ncclAllReduce(mm[i], mm[i], d, ncclFloat64, ncclMax, g->comms[i], stream_of(g, i)),
              ranks_of(g, "normalisation all-reduce (MAX)", i));
      NCCL_AT(ncclAllReduce(mm[i] + d, mm[i] + d, d, ncclFloat64, ncclMin, g->comms[i],
                            stream_of(g, i)),
              ranks_of(g, "normalisation all-reduce (MIN)", i));
    }
    NCCL_AT(ncclGroupEnd(), ranks_of(g, "normalisation all-reduce"));
  } else if (g->transport == XPORT_LOOPBACK) {
    // (test transport) folded on the host in rank order with strict compares
    std::vector<double> acc((size_t)2 * d), v((size_t)2 * d);
    for (int i = 0; i < g->ndev; i++) {
      HIP_G(hipSetDevice(g->devs[i]));
      HIP_G(hipMemcpyAsync(v.data(), mm[i], v.size() * 8, hipMemcpyDeviceToHost, stream_of(g, i)));
      HIP_G(hipStreamSynchronize(stream_of(g, i)));
      for (int c = 0; c < 2 * d; c++)
        if (i == 0 || (c < d ? v[c] > acc[c] : v[c] < acc[c])) acc[c] = v[c];
    }
    for (int i = 0; i < g->ndev; i++) {
      HIP_G(hipSetDevice(g->devs[i]));
      HIP_G(hipMemcpyAsync(mm[i], acc.data(), acc.size() * 8, hipMemcpyHostToDevice, stream_of(g, i)));
      HIP_G(hipStreamSynchronize(stream_of(g, i)));
    }
  }
  return KNN_OK;
}

// All-to-all of doubles: rank a sends cnt[a][b] doubles from send[a] + soff[a][b]
// to rank b, which receives them at recv[b] + roff[b][a].
static int coll_alltoallv(knn_group* g, const std::vector<double*>& send,
                          const std::vector<double*>& recv,
                          const std::vector<std::vector<int64_t>>& cnt,
                          const std::vector<std::vector<int64_t>>& soff,
                          const std::vector<std::vector<int64_t>>& roff) {
  const int G = g->ndev;
  if (g->transport == XPORT_LOOPBACK) {
    int rc;
    if ((rc = lb_barrier(g))) return rc;
  }
  // without RCCL (loopback, or no transport): every block a device copy
  if (g->transport != XPORT_RCCL)
    for (int a = 0; a < G; a++)
      for (int b = 0; b < G; b++) {
        if (cnt[a][b] <= 0) continue;
        HIP_G(hipSetDevice(g->devs[b]));
        HIP_G(hipMemcpyAsync(recv[b] + roff[b][a], send[a] + soff[a][b], cnt[a][b] * 8,
                             hipMemcpyDeviceToDevice, stream_of(g, b)));
      }
  // RCCL: every block, a rank's own included (send to self inside the group:
  // the one-rank communicator of KNN_GROUP_RCCL then runs this exchange's
  // ncclSend / ncclRecv on a single GPU)
  if (g->transport == XPORT_RCCL) {
    NCCL_AT(ncclGroupStart(), ranks_of(g, "tie all-to-all"));
    for (int a = 0; a < G; a++)
      for (int b = 0; b < G; b++) {
        if (cnt[a][b] > 0)
          NCCL_AT(ncclSend(send[a] + soff[a][b], (size_t)cnt[a][b], ncclFloat64, b, g->comms[a],
                           stream_of(g, a)),
                  ranks_of(g, ("tie all-to-all, to rank " + std::to_string(b)).c_str(), a));
        if (cnt[b][a] > 0)
          NCCL_AT(ncclRecv(recv[a] + roff[a][b], (size_t)cnt[b][a], ncclFloat64, b, g->comms[a],
                           stream_of(g, a)),
                  ranks_of(g, ("tie all-to-all, from rank " + std::to_string(b)).c_str(), a));
      }
    NCCL_AT(ncclGroupEnd(), ranks_of(g, "tie all-to-all"));
  }
  if (g->transport == XPORT_LOOPBACK) return lb_barrier(g);
  return KNN_OK;
}

extern "C" {

int knn_group_create(knn_group** out, int ndev, const int* devs, int mode) {
  const int base = mode & 0xff;
  if (!out || ndev <= 0 || (base != 0 && base != 1) || (mode & ~(0xff | KNN_GROUP_RCCL)))
    return knn_fail(KNN_ERR_ARG, "bad group arguments");
  if (ndev > knnk::kMaxParts) return knn_fail(KNN_ERR_ARG, "at most 64 ranks per group");
  *out = nullptr;
  knn_group* g = new knn_group();
  g->ndev = ndev;
  g->mode = base;
  for (int i = 0; i < ndev; i++) g->devs.push_back(devs ? devs[i] : i);
  bool shared = false;
  for (int i = 0; i < ndev; i++)
    for (int j = 0; j < i; j++) shared |= g->devs[i] == g->devs[j];
  const char* env = getenv("KNN_GROUP_RCCL");
  const bool force = (mode & KNN_GROUP_RCCL) || (env && !strcmp(env, "1"));
  g->transport = shared ? XPORT_LOOPBACK : (ndev > 1 || force) ? XPORT_RCCL : XPORT_NONE;
  g->ctx.assign(ndev, nullptr);
  for (int i = 0; i < ndev; i++) {
    int rc = knn_create(&g->ctx[i], g->devs[i]);
    if (rc) {
      knn_group_destroy(g);
      return rc;
    }
  }
  g->comms.assign(ndev, nullptr);
  if (g->transport == XPORT_RCCL) {
    ncclResult_t r = ncclCommInitAll(g->comms.data(), ndev, g->devs.data());
    if (r != ncclSuccess) {
      g->comms.clear();
      knn_group_destroy(g);
      std::string devl;
      for (int i = 0; i < ndev; i++) devl += " " + std::to_string(devs ? devs[i] : i);
      return knn_fail(KNN_ERR_COMM, "ncclCommInitAll over ranks 0.." + std::to_string(ndev - 1) +
                                        " (devices" + devl + ") failed: " + ncclGetErrorString(r));
    }
  }
  for (auto* v : {&g->X, &g->lab, &g->labA, &g->Q, &g->olab, &g->oidx, &g->odist, &g->oflags,
                  &g->pk, &g->gk, &g->tq, &g->tcnt, &g->tsel, &g->trow, &g->tsend, &g->trecv,
                  &g->nX, &g->nmm})
    v->resize(ndev);
  g->ev0.assign(ndev, nullptr);
  g->ev1.assign(ndev, nullptr);
  g->evx.assign(ndev, nullptr);
  for (int i = 0; i < ndev; i++) {
    if (hipSetDevice(g->devs[i]) != hipSuccess || hipEventCreate(&g->ev0[i]) != hipSuccess ||
        hipEventCreate(&g->ev1[i]) != hipSuccess ||
        hipEventCreateWithFlags(&g->evx[i], hipEventDisableTiming) != hipSuccess) {
      knn_group_destroy(g);
      return knn_fail(KNN_ERR_DEVICE, "hipEventCreate failed");
    }
  }
  *out = g;
  return KNN_OK;
}

int knn_group_transport(knn_group* g) { return g ? g->transport : -1; }

int knn_group_set_precision(knn_group* g, int mode) {
  if (!g) return knn_fail(KNN_ERR_ARG, "null group");
  for (auto* c : g->ctx) {
    int rc = knn_set_precision(c, mode);
    if (rc) return rc;
  }
  return KNN_OK;
}

int knn_group_set_tuning(knn_group* g, const char* key, int64_t value) {
  if (!g) return knn_fail(KNN_ERR_ARG, "null group");
  for (auto* c : g->ctx) {
    int rc = knn_set_tuning(c, key, value);
    if (rc) return rc;
  }
  return KNN_OK;
}

int knn_group_destroy(knn_group* g) {
  if (!g) return KNN_OK;
  for (int i = 0; i < g->ndev; i++) {
    if (i < (int)g->ctx.size() && g->ctx[i]) {
      (void)hipSetDevice(g->devs[i]);
      (void)hipDeviceSynchronize();
    }
    for (auto* v : {&g->X, &g->lab, &g->labA, &g->Q, &g->olab, &g->oidx, &g->odist, &g->oflags,
                    &g->pk, &g->gk, &g->tq, &g->tcnt, &g->tsel, &g->trow, &g->tsend, &g->trecv,
                    &g->nX, &g->nmm})
      if (i < (int)v->size()) (*v)[i].release();
    for (auto* ev : {&g->ev0, &g->ev1, &g->evx})
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
  g->trained = false;
  const int G = g->ndev;
  if (g->mode == 0) {
    // root copy on the first GPU, then a broadcast over xGMI (cpp:224-225)
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
    std::vector<void*> xb(G), lb(G);
    for (int i = 0; i < G; i++) {
      xb[i] = g->X[i].p;
      lb[i] = g->lab[i].p;
    }
    int rc;
    if ((rc = coll_bcast(g, xb, (size_t)n * d, ncclFloat64, 8, 0))) return rc;
    if ((rc = coll_bcast(g, lb, (size_t)n, ncclInt32, 4, 0))) return rc;
    for (int i = 0; i < G; i++)  // (the watchdog: a hung broadcast fails here, naming the rank)
      if ((rc = sync_rank(g, i, "train broadcast"))) return rc;
    rc = for_each_dev(g, [&](int i) {
      return knn_set_train_device(g->ctx[i], (const double*)g->X[i].p,
                                  (const int32_t*)g->lab[i].p, n, d, class_cnt, 0);
    });
    if (rc) return rc;
  } else {
    // train-sharded: contiguous row shards, global index offsets; every
    // label on every device for the reference-order pass (4 B per row)
    if (n < G) return knn_fail(KNN_ERR_ARG, "more ranks than train rows");
    int rc = for_each_dev(g, [&](int i) {
      const int64_t r0 = n * i / G, r1 = n * (i + 1) / G;
      const int64_t ni = r1 - r0;
      int e;
      if ((e = g->X[i].ensure((size_t)ni * d * sizeof(double)))) return e;
      if ((e = g->lab[i].ensure((size_t)ni * sizeof(int32_t)))) return e;
      if ((e = g->labA[i].ensure((size_t)n * sizeof(int32_t)))) return e;
      hipStream_t s = g->ctx[i]->stream;
      if (hipMemcpyAsync(g->X[i].p, X + r0 * d, (size_t)ni * d * sizeof(double),
                         hipMemcpyHostToDevice, s) != hipSuccess ||
          hipMemcpyAsync(g->lab[i].p, labels + r0, (size_t)ni * sizeof(int32_t),
                         hipMemcpyHostToDevice, s) != hipSuccess ||
          hipMemcpyAsync(g->labA[i].p, labels, (size_t)n * sizeof(int32_t),
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

}  // extern "C"

// Train-sharded: the queries the merges flagged KNN_FLAG_TIE_PENDING (their
// label depends on the reference's order among equal distances over the
// whole train set) get the reference's order.  The host reads the owners'
// queues (one small copy per device; the call waits for its devices at the
// end anyway), then per batch: every shard computes the batch's exact
// distances to its rows, an all-to-all moves each owner's blocks to it, and
// the owner re-sorts and votes (knn_tie_resolve_device).
static int resolve_ties(knn_group* g, int64_t m, int k, int metric) {
  int rc;
  const int G = g->ndev;
  const int64_t n = g->n;
  g->last_ties = 0;
  std::vector<int> hc(G, 0);
  for (int i = 0; i < G; i++) {
    HIP_G(hipSetDevice(g->devs[i]));
    HIP_G(hipMemcpyAsync(&hc[i], g->tcnt[i].p, sizeof(int), hipMemcpyDeviceToHost,
                         stream_of(g, i)));
  }
  int64_t total = 0;
  for (int i = 0; i < G; i++) {
    HIP_G(hipSetDevice(g->devs[i]));
    if ((rc = sync_rank(g, i, "tie exchange (counts)"))) return rc;
    total += hc[i];
  }
  if (total == 0) return KNN_OK;
  std::vector<std::vector<int>> own(G);  // owner's queued output rows (slice-local)
  for (int i = 0; i < G; i++) {
    own[i].resize(hc[i]);
    if (!hc[i]) continue;
    HIP_G(hipSetDevice(g->devs[i]));
    HIP_G(hipMemcpy(own[i].data(), g->tq[i].p, hc[i] * sizeof(int), hipMemcpyDeviceToHost));
    std::sort(own[i].begin(), own[i].end());
  }
  std::vector<int64_t> rows(G), r0(G);
  for (int i = 0; i < G; i++) {
    r0[i] = n * i / G;
    rows[i] = n * (i + 1) / G - r0[i];
  }
  // queries per batch: the owner receives up to B x n distances (<= 1 GB)
  const int64_t B = std::max<int64_t>(1, std::min<int64_t>(4096, (1ll << 30) / (8 * n)));
  std::vector<size_t> pos(G, 0);
  while (true) {
    std::vector<int64_t> cnt(G, 0);
    std::vector<int> sel;
    std::vector<std::vector<int>> orow(G);
    for (int r = 0; r < G && (int64_t)sel.size() < B; r++)
      while (pos[r] < own[r].size() && (int64_t)sel.size() < B) {
        const int qo = own[r][pos[r]++];
        sel.push_back((int)(m * r / G) + qo);  // global query row
        orow[r].push_back(qo);
        cnt[r]++;
      }
    const int Bt = (int)sel.size();
    if (Bt == 0) break;
    for (int i = 0; i < G; i++) {
      HIP_G(hipSetDevice(g->devs[i]));
      if ((rc = g->tsel[i].ensure((size_t)B * sizeof(int)))) return rc;
      if ((rc = g->trow[i].ensure((size_t)B * sizeof(int)))) return rc;
      if ((rc = g->tsend[i].ensure((size_t)B * rows[i] * sizeof(double)))) return rc;
      if ((rc = g->trecv[i].ensure((size_t)B * n * sizeof(double)))) return rc;
      hipStream_t s = stream_of(g, i);
      HIP_G(hipMemcpyAsync(g->tsel[i].p, sel.data(), Bt * sizeof(int), hipMemcpyHostToDevice, s));
      if (cnt[i])
        HIP_G(hipMemcpyAsync(g->trow[i].p, orow[i].data(), cnt[i] * sizeof(int),
                             hipMemcpyHostToDevice, s));
      if ((rc = knn_shard_distances_device(g->ctx[i], (const double*)g->Q[i].p,
                                           (const int32_t*)g->tsel[i].p, Bt, metric,
                                           (double*)g->tsend[i].p, s)))
        return rc;
    }
    // shard a's block for owner b: [cnt_b][rows_a] at (sum of earlier owners'
    // counts) x rows_a; it lands at cnt_b x r0_a on b (parts in row order)
    std::vector<std::vector<int64_t>> c2(G, std::vector<int64_t>(G)), so(G, std::vector<int64_t>(G)),
        ro(G, std::vector<int64_t>(G));
    for (int a = 0; a < G; a++) {
      int64_t before = 0;
      for (int b = 0; b < G; b++) {
        c2[a][b] = cnt[b] * rows[a];
        so[a][b] = before * rows[a];
        before += cnt[b];
      }
    }
    for (int b = 0; b < G; b++)
      for (int a = 0; a < G; a++) ro[b][a] = cnt[b] * r0[a];
    std::vector<double*> sb(G), rb(G);
    for (int i = 0; i < G; i++) {
      sb[i] = (double*)g->tsend[i].p;
      rb[i] = (double*)g->trecv[i].p;
    }
    if ((rc = coll_alltoallv(g, sb, rb, c2, so, ro))) return rc;
    for (int b = 0; b < G; b++) {
      if (!cnt[b]) continue;
      HIP_G(hipSetDevice(g->devs[b]));
      if ((rc = knn_tie_resolve_device(g->ctx[b], (const double*)g->trecv[b].p, G, rows.data(),
                                       (int)cnt[b], (const int32_t*)g->labA[b].p,
                                       (const int32_t*)g->trow[b].p, k, (int32_t*)g->olab[b].p,
                                       (int64_t*)g->oidx[b].p, (double*)g->odist[b].p,
                                       (int32_t*)g->oflags[b].p, stream_of(g, b))))
        return rc;
    }
    for (int i = 0; i < G; i++) {  // the host lists of this batch are reused
      HIP_G(hipSetDevice(g->devs[i]));
      if ((rc = sync_rank(g, i, "tie exchange (resolve)"))) return rc;
    }
    g->last_ties += Bt;
  }
  return KNN_OK;
}

extern "C" {

int knn_group_classify(knn_group* g, const double* Q, int64_t m, int32_t k, int32_t metric,
                       int32_t* out_labels, int64_t* out_idx, double* out_dist,
                       int32_t* out_flags) {
  if (!g || !g->trained) return knn_fail(KNN_ERR_STATE, "group classify before set_train");
  if (m < 0 || !out_labels || (m > 0 && !Q)) return knn_fail(KNN_ERR_ARG, "bad classify arguments");
  if (k < 0 || k > g->n) return knn_fail(KNN_ERR_ARG, "bad k");
  if (m >= (int64_t)INT32_MAX) return knn_fail(KNN_ERR_ARG, "m must be < 2^31 per call");
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
      if (int e = sync_rank(g, i, "classify")) return e;
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
  g->last_ties = 0;
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
  const int ties = g->ctx[0]->tune_ties;
  for (int i = 0; i < G; i++) {
    int64_t q0, mi;
    slice(i, q0, mi);
    HIP_G(hipSetDevice(g->devs[i]));
    if ((rc = g->Q[i].ensure((size_t)m * d * sizeof(double)))) return rc;
    // this GPU's lists packed [dist | idx | label] (one all-gather per step)
    if ((rc = g->pk[i].ensure((size_t)PB))) return rc;
    if (g->transport != XPORT_NONE && (rc = g->gk[i].ensure((size_t)G * PB))) return rc;
    if ((rc = g->olab[i].ensure((size_t)std::max<int64_t>(mi, 1) * sizeof(int32_t)))) return rc;
    if ((rc = g->oflags[i].ensure((size_t)std::max<int64_t>(mi, 1) * sizeof(int32_t)))) return rc;
    if ((rc = g->oidx[i].ensure((size_t)std::max<int64_t>(mi, 1) * k * sizeof(int64_t)))) return rc;
    if ((rc = g->odist[i].ensure((size_t)std::max<int64_t>(mi, 1) * k * sizeof(double)))) return rc;
    if ((rc = g->tq[i].ensure((size_t)std::max<int64_t>(mi, 1) * sizeof(int)))) return rc;
    if ((rc = g->tcnt[i].ensure(sizeof(int)))) return rc;
    if (const int64_t sb = knnk::merge_scratch_bytes(G, w, k, mi))
      if ((rc = g->ctx[i]->mrg.ensure((size_t)sb))) return rc;
  }
  // queries to the first GPU, broadcast to the rest
  HIP_G(hipSetDevice(g->devs[0]));
  HIP_G(hipMemcpyAsync(g->Q[0].p, Q, (size_t)m * d * sizeof(double), hipMemcpyHostToDevice,
                       g->ctx[0]->stream));
  for (int i = 0; i < G; i++) {
    HIP_G(hipSetDevice(g->devs[i]));
    HIP_G(hipEventRecord(g->ev0[i], g->ctx[i]->stream));
  }
  std::vector<void*> qb(G), sp(G), rp(G);
  for (int i = 0; i < G; i++) {
    qb[i] = g->Q[i].p;
    sp[i] = g->pk[i].p;
    rp[i] = g->gk[i].p;
  }
  if ((rc = coll_bcast(g, qb, (size_t)m * d, ncclFloat64, 8, 0))) return rc;
  for (int i = 0; i < G; i++) {
    HIP_G(hipSetDevice(g->devs[i]));
    unsigned char* pb = (unsigned char*)g->pk[i].p;
    if ((rc = knn_search_partial_device(g->ctx[i], (const double*)g->Q[i].p, m, w, metric,
                                        (double*)pb, (int64_t*)(pb + 8 * m * w),
                                        (int32_t*)(pb + 16 * m * w), nullptr)))
      return rc;
  }
  // one all-gather of the packed lists (≙ the reference's MPI_Gather, cpp:340)
  if ((rc = coll_allgather(g, sp, rp, (size_t)PB))) return rc;
  for (int i = 0; i < G; i++) {
    int64_t q0, mi;
    slice(i, q0, mi);
    HIP_G(hipSetDevice(g->devs[i]));
    hipStream_t s = g->ctx[i]->stream;
    if (mi > 0) {
      const double* sk = (const double*)(g->transport != XPORT_NONE ? g->gk[i].p : g->pk[i].p);
      knnk::MergeTies mt;
      mt.mode = ties;
      mt.q = (int*)g->tq[i].p;
      mt.cnt = (int*)g->tcnt[i].p;
      HIP_G(hipMemsetAsync(mt.cnt, 0, sizeof(int), s));
      knnk::launch_merge_vote_partials(sk, nullptr, nullptr, G, m, w, k, (int32_t*)g->olab[i].p,
                                       (int64_t*)g->oidx[i].p, (double*)g->odist[i].p,
                                       (int32_t*)g->oflags[i].p, s, q0, mi, PB, g->ctx[i]->mrg.p,
                                       mt);
      HIP_G(hipGetLastError());
    } else {
      HIP_G(hipMemsetAsync(g->tcnt[i].p, 0, sizeof(int), s));
    }
  }
  if (ties && (rc = resolve_ties(g, m, k, metric))) return rc;
  for (int i = 0; i < G; i++) {
    HIP_G(hipSetDevice(g->devs[i]));
    HIP_G(hipEventRecord(g->ev1[i], g->ctx[i]->stream));
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

int64_t knn_group_last_tie_count(knn_group* g) { return g ? g->last_ties : -1; }

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
  std::vector<double*> mm(G);
  for (int i = 0; i < G; i++) mm[i] = (double*)g->nmm[i].p;
  if ((rc = coll_allreduce_maxmin(g, mm, d))) return rc;  // ≙ MPI_Allreduce, cpp:276-277
  for (int i = 0; i < G; i++)
    if ((rc = sync_rank(g, i, "normalisation all-reduce"))) return rc;
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
