/* knn_amd.h -- C ABI of the MI355X-native brute-force KNN classifier.
 *
 * This is the drop-in boundary for the hot path of Jason-Woo/-MPI-KNN-
 * (/root/reference/knn_mpi.cpp, cited "cpp:N").  The reference has no
 * library interface: its hot path is inlined in main() (cpp:308-381), fed by
 * the constant block (cpp:108-119) and the MPI collectives (cpp:224-227,
 * 340, 383).  Each entry point below replaces one piece of that:
 *
 *   knn_set_train*      MPI_Bcast of Data_train/Train_label (cpp:224-225) and
 *                       the train side of the config block (N_train, dim,
 *                       class_cnt: cpp:108-113)
 *   knn_classify*       the query loop: per-pair Euclidean_D/Manhattan_D
 *                       (cpp:33-67) -> std::sort of all N_train records
 *                       (cpp:323/366) -> first-to-max vote over K
 *                       (cpp:324-337/367-380) -> Val/Test_label_buffer
 *   knn_search_partial  train-sharded variant (new; north_star mode b):
 *                       exact local top-w per query with global indices
 *   knn_merge_vote      k-way merge of per-shard lists + the vote (cpp:324-337)
 *   knn_group_*         single-process multi-GPU driver over RCCL/xGMI that
 *                       replaces MPI_Bcast/Scatter/Gather (cpp:224-227, 383)
 *
 * Semantics (identical to the reference on the same fp64 inputs):
 *   - distances are the reference's fp64 values: sqrt of the sequential
 *     sum of (q_i - x_i)^2 (no FMA) for metric 0, sum of |q_i - x_i| for
 *     metric 1;
 *   - neighbours are ordered by ascending distance.  Among exactly equal
 *     distances the reference's order is whatever its std::sort (libstdc++
 *     introsort) leaves; queries where that order can change the label
 *     (KNN_FLAG_TIE_VOTE / KNN_FLAG_TIE_BOUNDARY) are re-ordered exactly as
 *     the reference's std::sort orders them (KNN_FLAG_TIE_REF), other ties
 *     are ordered by train index (KNN_FLAG_TIE_ORDER; tuning key "ties" = 2
 *     re-orders those too);
 *   - label = first label whose running count strictly exceeds the running
 *     maximum while scanning the k nearest in order; -1 when k == 0.
 *   - the GPU computes a certified candidate set on MFMA (by default exact
 *     int8 codes on v_mfma_i32_16x16x64_i8 / 32x32x32_i8 for integer-coded
 *     train sets,
 *     else fp16 operands on v_mfma_f32_16x16x32_f16; bf16x3 or fp32 by
 *     precision mode, see knn_set_precision) and re-ranks it in fp64; queries whose
 *     candidate set cannot be certified are re-run exactly (fp64 over all
 *     rows).  No CPU fallback exists: without a usable HIP device every call
 *     fails with KNN_ERR_DEVICE.
 *
 * Conventions: plain pointers and sizes; return 0 on success, a negative
 * KNN_ERR_* code on failure (message via knn_last_error(), thread-local).
 * A host driver maps non-zero to exit(1), like MPI_Abort(..., 1)
 * (cpp:127-129).  One host thread per context; contexts are independent.
 * "Host" pointers are ordinary CPU memory; "_device" variants take device
 * pointers on the context's GPU and an optional hipStream_t (NULL = the
 * context's own stream, which is ordered after work on the device's legacy
 * default stream; work on other streams must be synchronised by the caller).
 */
#ifndef KNN_AMD_H
#define KNN_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KNN_OK 0
#define KNN_ERR_ARG -1     /* bad argument (sizes, k > n_train, label range) */
#define KNN_ERR_DEVICE -2  /* no HIP device / HIP runtime error */
#define KNN_ERR_STATE -3   /* e.g. classify before set_train */
#define KNN_ERR_NOMEM -4   /* device allocation failed */
#define KNN_ERR_COMM -5    /* RCCL failure */

#define KNN_METRIC_L2 0 /* Euclidean_distance = true  (cpp:114, 320, 363) */
#define KNN_METRIC_L1 1 /* Euclidean_distance = false (cpp:114, 321, 364) */

/* out_flags bits (per query) */
#define KNN_FLAG_EXACT_RESCAN 1 /* candidate set not certified; exact fp64 rescan used */
#define KNN_FLAG_TIE_BOUNDARY 2 /* dist[k-1] == dist[k]: membership tie at the k-th */
#define KNN_FLAG_TIE_VOTE 4     /* equal distances with different labels inside top-k */
#define KNN_FLAG_TIE_ORDER 8    /* equal distances inside top-k (order unspecified in
                                   the reference's std::sort; ours: by train index) */
#define KNN_FLAG_NONFINITE 16   /* the query has a NaN / inf coordinate: label -1, no
                                   neighbours (idx -1, dist NaN); the reference's
                                   distances are undefined there */
#define KNN_FLAG_TIE_REF 32     /* a tied query re-ordered as the reference's std::sort
                                   orders it (libstdc++ introsort emulated over all
                                   n distances): label, indices and their order are
                                   the reference's (knn_set_tuning "ties") */
#define KNN_FLAG_TIE_PENDING 64 /* knn_merge_vote_device: the label can depend on the
                                   reference's order among equal distances ACROSS
                                   shards; knn_shard_distances_device +
                                   knn_tie_resolve_device give the reference's order
                                   (knn_group mode 1 does this itself) */

typedef struct knn_ctx knn_ctx;
typedef struct knn_group knn_group;

/* Version string of the library build. */
const char* knn_version(void);
/* Last error message of the calling thread ("" if none). */
const char* knn_last_error(void);
/* Number of visible HIP devices (0 if none). */
int knn_device_count(void);

/* Context on HIP device `device` (replaces MPI_Init + per-rank state, cpp:123-125). */
int knn_create(knn_ctx** out, int device);
int knn_destroy(knn_ctx* ctx);

/* Train set from host memory: X row-major n x d fp64 (Data_train, cpp:140),
 * labels (Train_label, cpp:141) with 0 <= label < class_cnt.  The library
 * copies both to HBM (≙ MPI_Bcast cpp:224-225).  KNN_ERR_ARG for a label out
 * of range or a non-finite value (NaN / inf) anywhere in X. */
int knn_set_train(knn_ctx* ctx, const double* X, const int32_t* labels, int64_t n,
                  int32_t d, int32_t class_cnt);
/* Same from device memory on ctx's GPU (e.g. after an RCCL broadcast).
 * dX/dlabels are borrowed and must stay valid until the next set_train or
 * destroy.  idx_offset is added to every reported neighbour index (train
 * sharding: global index of this shard's first row).  Labels and values are
 * checked on the device (same errors as knn_set_train).  The work runs on
 * the context's stream, which is ordered after the device's legacy default
 * stream: producers on other streams must be synchronised by the caller. */
int knn_set_train_device(knn_ctx* ctx, const double* dX, const int32_t* dlabels, int64_t n,
                         int32_t d, int32_t class_cnt, int64_t idx_offset);

/* Classify m queries Q (row-major m x d fp64, same d as the train set).
 * out_labels[m] (Test_label_buffer, cpp:380) required; out_idx[m*k]
 * (global train indices) and out_dist[m*k] (fp64 reference distances) and
 * out_flags[m] nullable.  Host pointers.  0 <= k <= n_train (k > 1000 runs
 * the exact large-k path). */
int knn_classify(knn_ctx* ctx, const double* Q, int64_t m, int32_t k, int32_t metric,
                 int32_t* out_labels, int64_t* out_idx, double* out_dist,
                 int32_t* out_flags);
/* Device-pointer variant; enqueued on `stream` (hipStream_t, NULL = ctx
 * stream) and returns without waiting for the device on every path: the
 * exact rescan of uncertified queries is enqueued too and sized on the
 * device.  Outputs are complete once the stream reaches the end of the call
 * (knn_sync, or any later work on the same stream).  One stream at a time
 * per context (the context's workspace is shared by its calls). */
int knn_classify_device(knn_ctx* ctx, const double* dQ, int64_t m, int32_t k, int32_t metric,
                        int32_t* d_labels, int64_t* d_idx, double* d_dist, int32_t* d_flags,
                        void* stream);

/* Train-sharded building block: exact top-w of THIS context's shard for
 * each query, sorted by (dist, global idx), with each neighbour's label.
 * Rows beyond the shard size are padded with dist=+inf, idx=-1, label=-1.
 * Device pointers: d_dist[m*w], d_idx[m*w], d_lab[m*w]. */
int knn_search_partial_device(knn_ctx* ctx, const double* dQ, int64_t m, int32_t w,
                              int32_t metric, double* d_dist, int64_t* d_idx,
                              int32_t* d_lab, void* stream);
/* k-way merge of `parts` sorted lists per query, laid out [parts][m][w]
 * (the layout an all-gather of knn_search_partial outputs produces), then
 * the reference vote over the first k of the merged order, for queries
 * [q0, q0+mq) (a rank's slice; q0=0, mq=m for all).  Outputs are indexed
 * from 0 (row q-q0).  Device pointers; d_out_idx/d_out_dist/d_flags nullable.
 * Within exact distance ties the merged order is (dist, global idx); a query
 * whose label that order could decide (tuning "ties" of ctx: 1 vote-affecting
 * ties, 2 every tie, 0 none) gets KNN_FLAG_TIE_PENDING in d_flags.  A query
 * no shard listed a neighbour for (non-finite) gets label -1,
 * KNN_FLAG_NONFINITE, idx -1, dist NaN; with fewer than k rows in all, the
 * empty slots are idx -1, dist +inf. */
int knn_merge_vote_device(knn_ctx* ctx, const double* d_dist, const int64_t* d_idx,
                          const int32_t* d_lab, int32_t parts, int64_t m, int32_t w, int32_t k,
                          int64_t q0, int64_t mq, int32_t* d_labels, int64_t* d_out_idx,
                          double* d_out_dist, int32_t* d_flags, void* stream);

/* ---- train-sharded reference tie order (cpp:323/366 over the WHOLE train
 * set, whose std::sort order among equal distances depends on every row).
 * For the KNN_FLAG_TIE_PENDING queries of all ranks (rare):
 * 1. every shard: knn_shard_distances_device -- d_out[i][j] = the exact fp64
 *    distance (cpp:33-67 operation order) of shard row j to query
 *    dQ[d_qsel[i]] (d_qsel NULL: query i), [nsel][n_shard];
 * 2. an all-to-all moves each owner's [nsel_r][n_shard] block to it;
 * 3. the owner: knn_tie_resolve_device over d_D = parts blocks in global row
 *    order, block p = [nsel][rows[p]] at offset nsel * (rows[0] + ... +
 *    rows[p-1]) (what the all-to-all delivers), d_lab_all = the labels of all
 *    rows (global order); runs libstdc++'s introsort as the reference does
 *    and the vote, and rewrites output row d_orow[i] of d_labels / d_idx /
 *    d_dist (k per row) / d_flags (TIE_PENDING -> TIE_REF).  parts <= 64,
 *    sum(rows) < 2^31.  Scratch: ~20 B per row per concurrent query. */
int knn_shard_distances_device(knn_ctx* ctx, const double* dQ, const int32_t* d_qsel,
                               int32_t nsel, int32_t metric, double* d_out, void* stream);
int knn_tie_resolve_device(knn_ctx* ctx, const double* d_D, int32_t parts, const int64_t* rows,
                           int32_t nsel, const int32_t* d_lab_all, const int32_t* d_orow,
                           int32_t k, int32_t* d_labels, int64_t* d_idx, double* d_dist,
                           int32_t* d_flags, void* stream);

/* ---- min-max normalisation (replaces cpp:229-306, bit-exact in fp64) -----
 * Transductive, like the reference: per-dimension max/min over the train
 * rows AND every query set, starting from max = -1 / min = 999999
 * (cpp:239-243, strict compares), then x = (x - min)/(max - min) on the
 * dimensions where max - min != 0.
 * knn_minmax_device folds one device set [rows x d] (fp64, row-major) into
 *   d_max/d_min (device, d doubles each); init != 0 starts from -1/999999
 *   (the first set), 0 folds into the current values (later sets, or the
 *   result of an all-reduce over ranks, ≙ MPI_Allreduce cpp:276-277).
 * knn_normalize_device applies the bounds to a device set in place.
 * knn_normalize runs both on host sets in place (sets[i] has rows[i] rows;
 *   e.g. {train, test, val}); out_max/out_min (nullable) receive the bounds. */
int knn_minmax_device(knn_ctx* ctx, const double* d_X, int64_t rows, int32_t d, double* d_max,
                      double* d_min, int32_t init, void* stream);
int knn_normalize_device(knn_ctx* ctx, double* d_X, int64_t rows, int32_t d,
                         const double* d_max, const double* d_min, void* stream);
int knn_normalize(knn_ctx* ctx, double* const* sets, const int64_t* rows, int32_t nsets,
                  int32_t d, double* out_max, double* out_min);

/* Per-phase device timing with HIP events recorded on the stream the
 * kernels run on (off by default).  Phases: 0 = query prep, 1 = candidate
 * kernel (fused MFMA distance + top-R), 2 = merge/re-rank/vote, 3 = exact
 * rescan.  knn_last_phase_ms: the last classify/search call (waits for it;
 * -1 if none).  knn_timing_totals: per-phase sums over every timed call
 * since the last reset, and their number (waits for them); reset != 0
 * starts a new sum.  Recording never makes a call wait.  enable: 0 off, 1
 * every phase (5 events per call), 2 the candidate kernel only (2 events:
 * each event record holds the stream ~6 us, profiles/ab_log.md r5u; the
 * other phases then read -1 / 0).  Behaviour change (round 5): any other
 * value of enable (earlier builds took every non-zero value as "on") is
 * refused with KNN_ERR_ARG and leaves the timing state unchanged. */
#define KNN_PHASE_PREP 0
#define KNN_PHASE_CANDIDATE 1
#define KNN_PHASE_RERANK 2
#define KNN_PHASE_RESCAN 3
int knn_set_timing(knn_ctx* ctx, int enable);
double knn_last_phase_ms(knn_ctx* ctx, int phase);
int knn_timing_totals(knn_ctx* ctx, double out_ms[4], int64_t* calls, int reset);
/* Geometry of the last candidate launch: out[0]=workgroups, out[1]=splits
 * per query tile, out[2]=list entries per lane (R), out[3]=re-rank count C. */
int knn_last_geometry(knn_ctx* ctx, int64_t out[4]);

/* Candidate-pass precision for L2 (the result is the exact fp64 top-k in
 * every mode; this only selects how candidates are found):
 *   AUTO (default): for batches of >= 4096 queries at d <= 256, int8 when
 *         the train set is integer-coded (every value c / 2^s with the
 *         codes of each dimension spanning <= 255, e.g. byte features),
 *         else fp16 (either until a batch of this train set leaves > 1/16
 *         of its queries to the rescan); otherwise bf16x3 (d > 256 on the
 *         streamed kernel);
 *   FP32: v_mfma_f32_32x32x2_f32 on fp32 copies;
 *   BF16X3: q.x as qh.xh + ql.xh + qh.xl on bf16 MFMA
 *           (hi/lo bf16 split of the fp64 values, ~2^-16 relative error);
 *   FP16: q.x on v_mfma_f32_16x16x32_f16 with both operands in fp16 under
 *         power-of-two scales (~2^-10 relative error), d <= 256.
 * The int8 pass (kernel paths 5 and 6) is exact: v_mfma_i32_16x16x64_i8
 * (dims padded to 64) or v_mfma_i32_32x32x32_i8 (dims padded to 32, chosen
 * where that pads fewer dims, e.g. d = 96) on the codes, centred per
 * dimension; a query off the train set's grid or beyond the codes' range
 * goes to the exact rescan.  It has no precision mode of its own (tuning
 * keys "i8", "i8w").
 * Environment override at knn_create: KNN_PRECISION=fp32|bf16x3|fp16. */
#define KNN_PRECISION_AUTO 0
#define KNN_PRECISION_FP32 1
#define KNN_PRECISION_BF16X3 2
#define KNN_PRECISION_FP16 3
int knn_set_precision(knn_ctx* ctx, int mode);
/* Candidate kernel flavour of the last search: 0 fp32 L2, 1 fp32 L1, 2 bf16x3
 * L2 (32x32x16 MFMA), 3 bf16x3 L2 (16x16x32), 4 fp16 L2 (16x16x32), 5 int8
 * L2 (16x16x64, exact integer dot products), 6 int8 L2 (32x32x32). */
int knn_last_candidate_path(knn_ctx* ctx);
/* Name of the last candidate kernel launched, as rocprofv3 reports it
 * without namespace, spaces and argument list (e.g. "cand_kernel<128,4,4,8>"). */
const char* knn_last_kernel_name(knn_ctx* ctx);

/* Tuning overrides for experiments (0 = automatic): "R" list entries per
 * lane (4, 8, 16), "S" train splits per query tile (1..64), "nw" waves per
 * candidate workgroup (4, 8 or 16 where the kernel has the variant), "ablate"
 * (bits 0/1/3/4: timing-only kernel ablations -- no staging, no selection,
 * L2-resident staging, no workgroup barrier -- results invalid; bit 2: no
 * per-query global threshold exchange, results stay exact); -1 = auto for "fp16" (fp16
 * candidate pass: 0 off, 1 on), "i8" (the int8 candidate pass where the
 * train set is integer-coded: 0 off, 1 on at every batch size), "i8w" (int8
 * kernel: -1 auto, 0 the 16x16x64 one, 1 the 32x32x32 one; also read by
 * knn_set_train*, whose norm blocks interleave the rows over that kernel's
 * lane lists -- set it before the train set: a later change keeps results
 * exact but loses the interleave's certification odds), "mfma16" (bf16x3 on the 16x16x32 layout: 0
 * off, 1 on), "s3q" (the fp16 d > 256 kernel on 16x16x32: 0 off, 1 on), "qres"
 * (1: where "s3q" runs and d pads to 32 x {9, 10, 12, 14, 16, 18, 20, 24,
 * 25, 28, 30}, the query-resident kernel replaces it -- queries held in
 * registers, rows streamed; 0 off: S3; -1 auto) and
 * "gk" (what the global threshold exchange publishes: 0 the lists' R-th
 * entries (resident kernel) / no exchange (S3), K = 1..16 the K-th smallest
 * of a workgroup's union of a query's lists; results stay exact); "ties"
 * (the reference's std::sort order for tied queries: 0 off, 1 (default) the
 * queries whose label it can change, 2 every query with a tie in its top k);
 * "seed" (experiment: seeded global thresholds of the fp16 / int8 resident
 * kernels from a pre-pass over N strided train rows; 0 / -1 off, the
 * default -- measured slower; results stay exact); "order" (region order of
 * the train images, read by knn_set_train*: -1 auto -- on for integer-coded
 * train sets (the int8 pass) whose int8 image (n x (padded d + 16) bytes) is
 * at most 192 MB and for other sets whose fp16 image (n x (2 padded d + 16)
 * bytes) is at most 512 MB, with P = min(64, n / 16384) regions and at
 * least 8 of them -- 0 off, 1 on with P = min(64, n / 16384) regions (stays
 * off below n = 32768, where P < 2), 2..64 that many regions (at most n /
 * 256); queries of the resident fp16 / int8 kernels are then sorted by
 * region and each query tile's stream starts at its region -- "ophase": -1
 * auto (at the first region of its region's eighth of the chain, so 8
 * groups of query tiles share their streams), 0 its own region, N phases);
 * "nblk" (norm blocks of the train images, read by knn_set_train*: every
 * 16384-row window of the image order sorted by the rows' squared norm, so
 * the int8 kernels' per-sub-tile seed bound is tight; -1 auto -- on for
 * integer-coded train sets of more than 16384 rows at d <= 256 -- 0 off, 1
 * on, 2 on as plain sorted windows, 3 on with the interleave only: by
 * default the norm ranks of each 32-row sub-tile are spread over the int8
 * kernel's per-lane lists and the sub-tiles over the window's tiles, so rows
 * of adjacent norm share neither a list nor a split); "s3gq" (the fp16 d > 256 kernel's largest XCD grouping of query
 * tiles, 0 = 4); "xhswz" (the fp16 image's chunk swizzle: 1 on, 0 off);
 * "i8resc" (the fast rescan of failed queries on the train grid filters the
 * int8 32x32x32 kernel's image exactly on the codes: -1 auto = on, 0 every
 * failed query on the fp32 filter);
 * all of them leave results exact. */
int knn_set_tuning(knn_ctx* ctx, const char* key, int64_t value);

/* Synchronise the context's stream. */
int knn_sync(knn_ctx* ctx);
/* Last classify's count of queries that needed the exact rescan (waits for
 * that call; -1 on error). */
int64_t knn_last_rescan_count(knn_ctx* ctx);
/* Rescan counts summed over calls since the last reset: out[0] = queries
 * that failed certification, out[1] = of those, queries finished by the full
 * exact scan.  Waits for the context's work; reset != 0 zeroes the sums. */
int knn_rescan_totals(knn_ctx* ctx, int64_t out[2], int reset);
/* Queries re-ordered as the reference's std::sort orders them
 * (KNN_FLAG_TIE_REF) summed over calls since the last reset.  Waits for the
 * context's work; reset != 0 zeroes the sum. */
int knn_tie_totals(knn_ctx* ctx, int64_t* out, int reset);

/* ---- single-process multi-GPU group over RCCL (xGMI) ---------------------
 * mode 0 = query-sharded: the train set is RCCL-broadcast from device
 *          devs[0] to every GPU (≙ MPI_Bcast cpp:224-225); queries are
 *          split into contiguous shards (≙ MPI_Scatter cpp:226-227, ragged
 *          shards allowed); labels land in one host array (≙ MPI_Gather
 *          cpp:340/383).
 * mode 1 = train-sharded: every GPU holds n/G rows; each computes the exact
 *          local top-(k+1) for all queries; ncclAllGather exchanges the lists;
 *          each GPU k-way merges and votes its slice of the queries; queries
 *          whose label the reference's tie order decides (KNN_FLAG_TIE_PENDING)
 *          get it from an RCCL send/recv exchange of their exact distances
 *          (knn_tie_resolve_device), so every mode gives the same labels.
 * Transport: RCCL whenever G > 1 and the devices are distinct.
 *   | KNN_GROUP_RCCL: RCCL also at G = 1 (a one-rank communicator: every
 *     collective of the path runs through RCCL; env KNN_GROUP_RCCL=1 too).
 *   Repeated devices in devs (e.g. {0, 0, 0}): several ranks share a GPU and
 *     the collectives run as stream-ordered device copies (loopback) -- the
 *     whole G-rank decomposition on fewer GPUs, for tests. */
#define KNN_GROUP_RCCL 0x100
int knn_group_create(knn_group** out, int ndev, const int* devs, int mode);
/* Transport of a group: 0 none (G = 1), 1 RCCL, 2 loopback copies. */
int knn_group_transport(knn_group* g);
/* knn_set_precision / knn_set_tuning on every rank's context. */
int knn_group_set_precision(knn_group* g, int mode);
int knn_group_set_tuning(knn_group* g, const char* key, int64_t value);
int knn_group_destroy(knn_group* g);
int knn_group_set_train(knn_group* g, const double* X, const int32_t* labels, int64_t n,
                        int32_t d, int32_t class_cnt);
int knn_group_classify(knn_group* g, const double* Q, int64_t m, int32_t k, int32_t metric,
                       int32_t* out_labels, int64_t* out_idx, double* out_dist,
                       int32_t* out_flags);
/* Seconds of the last group classify spent between the first enqueue and
 * the last device completion (device-resident inputs, excludes H2D/D2H). */
double knn_group_last_compute_seconds(knn_group* g);
/* Mode 1: queries of the last classify that took the cross-shard reference
 * tie order (KNN_FLAG_TIE_PENDING -> KNN_FLAG_TIE_REF). */
int64_t knn_group_last_tie_count(knn_group* g);
/* Normalisation over the group (cpp:229-306 with the reference's own
 * decomposition): GPU g takes rows [r*g/G, r*(g+1)/G) of every host set,
 * reduces its max/min, ncclAllReduce MAX/MIN combines them (≙ MPI_Allreduce
 * cpp:276-277), and each GPU rewrites its rows in place. */
int knn_group_normalize(knn_group* g, double* const* sets, const int64_t* rows, int32_t nsets,
                        int32_t d);

#ifdef __cplusplus
}
#endif
#endif /* KNN_AMD_H */
