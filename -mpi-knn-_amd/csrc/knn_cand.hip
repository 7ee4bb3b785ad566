// knn_cand.hip -- MI355X (gfx950, CDNA4) candidate kernels of the KNN classify path.
//
// Pipeline per classify call (reference loop: cpp:308-381):
//   1. prep_queries      fp64 queries -> fp32 (x -2 for L2) MFMA operands
//   2. cand_kernel       fused distance + per-lane top-R selection.
//        L2: -2 q.x^T on v_mfma_f32_32x32x2_f32 with the accumulator seeded by
//            ||x||^2, so the chain ends at ||x||^2 - 2 q.x (the rank-equivalent
//            of ||q - x||^2 for a fixed query; cpp:33-50).
//        L1: sum |q - x| on the VALU (cpp:51-67; no GEMM identity exists).
//        The distance matrix is never materialised: each lane keeps a sorted
//        register list of its R best rows and a threshold filter.
//   3. merge_rerank      per query: union of all lists -> best C by the fp32
//        proxy -> exact fp64 reference distances for those C (sequential sum,
//        no FMA, correctly rounded sqrt) -> sort by (dist, idx) -> certify
//        that no excluded row can enter the top-w (rigorous fp32 error
//        bound) -> first-to-max vote (cpp:324-337) or partial list output.
//   4. rescan (rare)     queries that fail certification get an exact fp64
//        scan over every row (chunked sort + tree reduce).
// The result is the reference's fp64 top-k with ties ordered by train index.
//
// This TU: the large-d fp32 stream kernel, the bf16x3 large-d S3 kernel and
// the dispatch over all candidate kernels (the register-resident kernel is
// instantiated in knn_cand_res.hip, one object per group of dimensions).
#include "knn_device.h"

namespace knnk {

#define KNN_DECL(v)                                          \
  bool launch_res_##v(const CandLaunch& c, hipStream_t s);   \
  int blocks_res_##v(int R, int metric, int nw);             \
  int qpw_res_##v(int metric);                               \
  int trows_res_##v(int metric);
KNN_DP_LIST(KNN_DECL)
#undef KNN_DECL

// Large-dimension variant (DP > 256, e.g. the reference's MNIST default
// d=784): the query tile no longer fits in VGPRs, so both operands are staged
// through LDS in chunks of DC dims.  Workgroup tile = 128 queries x 128 train
// rows (4 waves x (32 queries x 4 row blocks)); per chunk each wave issues
// 4 x DC/2 MFMAs reading its B fragment once per 8 dims and reusing it over
// the 4 row blocks.  LDS: 2 buffers x (A 128xDC + B 128xDC), rows padded by
// 16 B (DC/4 + 1 odd -> conflict-free ds_read_b128).  Same selection epilogue
// after the last chunk of a tile.
template <int DC, int R, int METRIC>
__global__ void __launch_bounds__(256)
cand_stream_kernel(const float* __restrict__ X32, const float* __restrict__ xinit,
                   const float* __restrict__ Q32, int DP, int n_tiles, int S, int n_qt,
                   float* __restrict__ out_v, int* __restrict__ out_i) {
  constexpr int TRS = 128;          // train rows per tile
  constexpr int LS = DC + 4;        // LDS row stride (floats)
  constexpr int OP = TRS * LS;      // floats per operand image
  constexpr int CPR = DC / 4;       // float4 per row chunk
  constexpr int NCH = TRS * CPR;    // float4 per operand chunk
  constexpr int CPT = NCH / 256;    // per thread
  static_assert(CPT == 4, "staging below is written for 4 float4 per operand");
  __shared__ __attribute__((aligned(16))) float lds[2 * 2 * OP + 2 * TRS];
  float* ldsn = lds + 4 * OP;

  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / n_qt;
  const int qt = bid - split * n_qt;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t qg = (int64_t)qt * kQPB + wv * 32 + j;
  const int nch = DP / DC;

  float L[R];
  int I[R];
#pragma unroll
  for (int t = 0; t < R; ++t) { L[t] = KNN_INF_F; I[t] = -1; }
  float thr = KNN_INF_F;

  const int my_nt = split < n_tiles ? (n_tiles - split + S - 1) / S : 0;
  const int total = my_nt * nch;

  float4 a0, a1, a2, a3, b0, b1, b2, b3;
  float4 stn = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* qbase = Q32 + (int64_t)qt * kQPB * DP;
#define KNN_SLOAD(st_)                                                                  \
  do {                                                                                  \
    const int it_ = (st_) / nch, c_ = (st_) - it_ * nch;                                \
    const int t_ = split + it_ * S;                                                     \
    const float* xs_ = X32 + (int64_t)t_ * TRS * (DP + 4) + c_ * DC;                    \
    const float* qs_ = qbase + c_ * DC;                                                 \
    int e_ = tid;                                                                       \
    a0 = *(const float4*)(xs_ + (e_ / CPR) * (DP + 4) + (e_ % CPR) * 4);                \
    b0 = *(const float4*)(qs_ + (e_ / CPR) * DP + (e_ % CPR) * 4);                      \
    e_ += 256;                                                                          \
    a1 = *(const float4*)(xs_ + (e_ / CPR) * (DP + 4) + (e_ % CPR) * 4);                \
    b1 = *(const float4*)(qs_ + (e_ / CPR) * DP + (e_ % CPR) * 4);                      \
    e_ += 256;                                                                          \
    a2 = *(const float4*)(xs_ + (e_ / CPR) * (DP + 4) + (e_ % CPR) * 4);                \
    b2 = *(const float4*)(qs_ + (e_ / CPR) * DP + (e_ % CPR) * 4);                      \
    e_ += 256;                                                                          \
    a3 = *(const float4*)(xs_ + (e_ / CPR) * (DP + 4) + (e_ % CPR) * 4);                \
    b3 = *(const float4*)(qs_ + (e_ / CPR) * DP + (e_ % CPR) * 4);                      \
    if (c_ == 0 && tid < TRS / 4) stn = ((const float4*)(xinit + (int64_t)t_ * TRS))[tid]; \
  } while (0)
#define KNN_SSTORE(st_, buf_)                                                           \
  do {                                                                                  \
    float* A_ = lds + (buf_) * 2 * OP;                                                  \
    float* B_ = A_ + OP;                                                                \
    int e_ = tid;                                                                       \
    *(float4*)(A_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = a0;                             \
    *(float4*)(B_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = b0;                             \
    e_ += 256;                                                                          \
    *(float4*)(A_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = a1;                             \
    *(float4*)(B_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = b1;                             \
    e_ += 256;                                                                          \
    *(float4*)(A_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = a2;                             \
    *(float4*)(B_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = b2;                             \
    e_ += 256;                                                                          \
    *(float4*)(A_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = a3;                             \
    *(float4*)(B_ + (e_ / CPR) * LS + (e_ % CPR) * 4) = b3;                             \
    const int c_ = (st_) % nch;                                                         \
    if (c_ == 0 && tid < TRS / 4) *(float4*)(ldsn + (buf_) * TRS + 4 * tid) = stn;      \
  } while (0)

  if (total > 0) {
    KNN_SLOAD(0);
    KNN_SSTORE(0, 0);
  }
  __syncthreads();

  f32x16 acc0, acc1, acc2, acc3;
  for (int st = 0; st < total; ++st) {
    const int it = st / nch, c = st - it * nch;
    const int t = split + it * S;
    const bool more = st + 1 < total;
    if (more) KNN_SLOAD(st + 1);
    const float* A = lds + (st & 1) * 2 * OP;
    const float* B = A + OP;
    if (c == 0) {
      // the norms were staged with chunk 0 of this tile into buffer (st & 1)
      const float* nb = ldsn + (st & 1) * TRS;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 n0 = *(const float4*)(nb + 0 * 32 + 8 * g + 4 * h);
        const float4 n1 = *(const float4*)(nb + 1 * 32 + 8 * g + 4 * h);
        const float4 n2 = *(const float4*)(nb + 2 * 32 + 8 * g + 4 * h);
        const float4 n3 = *(const float4*)(nb + 3 * 32 + 8 * g + 4 * h);
        acc0[4 * g] = n0.x; acc0[4 * g + 1] = n0.y; acc0[4 * g + 2] = n0.z; acc0[4 * g + 3] = n0.w;
        acc1[4 * g] = n1.x; acc1[4 * g + 1] = n1.y; acc1[4 * g + 2] = n1.z; acc1[4 * g + 3] = n1.w;
        acc2[4 * g] = n2.x; acc2[4 * g + 1] = n2.y; acc2[4 * g + 2] = n2.z; acc2[4 * g + 3] = n2.w;
        acc3[4 * g] = n3.x; acc3[4 * g + 1] = n3.y; acc3[4 * g + 2] = n3.z; acc3[4 * g + 3] = n3.w;
      }
    }
    if constexpr (METRIC == 0) {
      const float* brow = B + (wv * 32 + j) * LS + 4 * h;
      const float* arow = A + j * LS + 4 * h;
#pragma unroll
      for (int g = 0; g < DC / 8; ++g) {
        const float4 b = *(const float4*)(brow + 8 * g);
        const float4 x0 = *(const float4*)(arow + 0 * 32 * LS + 8 * g);
        const float4 x1 = *(const float4*)(arow + 1 * 32 * LS + 8 * g);
        const float4 x2 = *(const float4*)(arow + 2 * 32 * LS + 8 * g);
        const float4 x3 = *(const float4*)(arow + 3 * 32 * LS + 8 * g);
#define KNN_MF4(acc_, x_)                                                               \
  acc_ = __builtin_amdgcn_mfma_f32_32x32x2f32(x_.x, b.x, acc_, 0, 0, 0);                \
  acc_ = __builtin_amdgcn_mfma_f32_32x32x2f32(x_.y, b.y, acc_, 0, 0, 0);                \
  acc_ = __builtin_amdgcn_mfma_f32_32x32x2f32(x_.z, b.z, acc_, 0, 0, 0);                \
  acc_ = __builtin_amdgcn_mfma_f32_32x32x2f32(x_.w, b.w, acc_, 0, 0, 0);
        KNN_MF4(acc0, x0) KNN_MF4(acc1, x1) KNN_MF4(acc2, x2) KNN_MF4(acc3, x3)
#undef KNN_MF4
      }
    } else {
      const float* brow = B + (wv * 32 + j) * LS;
#pragma unroll 2
      for (int g = 0; g < DC / 4; ++g) {
        const float4 qv = *(const float4*)(brow + 4 * g);
#define KNN_L1B(acc_, blk_)                                                             \
  _Pragma("unroll") for (int i = 0; i < 16; ++i) {                                      \
    const int r = (blk_) * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;                         \
    const float4 xv = *(const float4*)(A + r * LS + 4 * g);                             \
    float a = acc_[i];                                                                  \
    a = a + __builtin_fabsf(qv.x - xv.x);                                               \
    a = a + __builtin_fabsf(qv.y - xv.y);                                               \
    a = a + __builtin_fabsf(qv.z - xv.z);                                               \
    a = a + __builtin_fabsf(qv.w - xv.w);                                               \
    acc_[i] = a;                                                                        \
  }
        KNN_L1B(acc0, 0) KNN_L1B(acc1, 1) KNN_L1B(acc2, 2) KNN_L1B(acc3, 3)
#undef KNN_L1B
      }
    }
    if (c == nch - 1) {
      select_block<R>(acc0, t * TRS + 0, h, L, I, thr, KNN_INF_F);
      select_block<R>(acc1, t * TRS + 32, h, L, I, thr, KNN_INF_F);
      select_block<R>(acc2, t * TRS + 64, h, L, I, thr, KNN_INF_F);
      select_block<R>(acc3, t * TRS + 96, h, L, I, thr, KNN_INF_F);
    }
    if (more) KNN_SSTORE(st + 1, (st + 1) & 1);
    __syncthreads();
  }
  write_lists<R>(out_v, out_i, qg, S, split, h, L, I);
#undef KNN_SLOAD
#undef KNN_SSTORE
}

// -------------------------------------- bf16x3 large-dimension kernel (S3)
// For DP > 256 with the bf16x3 L2 candidate pass (cfg5: d = 960, k = 100;
// the reference's MNIST default d = 784).  Neither operand fits in VGPRs, so
// both are staged per chunk of 16 dims (one 32x32x16 k-step).  Workgroup =
// 8 waves, tile = 256 queries x 256 train rows; wave w owns queries
// 32w..32w+31 against all 256 rows as 8 accumulator blocks (128 acc
// registers), so one staged chunk (32 KiB: 16 KiB of rows + 16 KiB of
// queries) feeds 8 x 24 MFMAs -- 98 MACs per staged byte, a third of what the
// XCD L2 can deliver at the full MFMA rate.  The epilogue (the same register
// top-R lists as cand_kernel) runs once per tile, i.e. every DP/16 chunks.
//
// HBM images are pre-laid out exactly as the LDS images, so LDS-DMA copies
// them linearly: block (tile, chunk) = 256 rows x 64 B, row r holding the
// four 16-B slots {hi k0-7, hi k8-15, lo k0-7, lo k8-15} at slot position
// s ^ ((r >> 2) & 3).  That XOR makes every 16-lane group of a ds_read_b128
// (lanes on rows {0-3,12-15,20-27} etc.) touch 16 distinct 16-B bank groups.
// Seeds (fl32 ||x32||^2, +inf on pad rows) travel as one 1-KiB piece with
// chunk 0 of each tile.
//
// F16 (cand_s3h_kernel, the fp16 candidate pass at d > 256): the same images
// with a chunk of 32 dims in fp16 -- slots {k0-7, k8-15, k16-23, k24-31} --
// and two v_mfma_f32_32x32x16_f16 per block and chunk (one per 16 dims,
// products exact in fp32) instead of three bf16 ones per 16 dims: 3x fewer
// MFMAs per algorithmic flop and half the staged bytes per MFMA.
#ifndef KNN_S3_NB
#define KNN_S3_NB 4
#endif
// Q16: A-fragment ring depth (LDS reads in flight behind the MFMAs) and
// whether the MFMA / read interleave is pinned with sched_group_barrier
#ifndef KNN_S3_RING
#define KNN_S3_RING 3
#endif
#ifndef KNN_S3_SCHED
#define KNN_S3_SCHED 1
#endif
// one 8-wave workgroup per CU (the 4-deep LDS ring takes 132 KiB): 2 waves
// per SIMD, so up to 256 registers each for fragments in flight
#ifndef KNN_S3_WPE
#define KNN_S3_WPE 2
#endif
// s_waitcnt vmcnt(n) + s_barrier with a run-time n (vmcnt takes an immediate)
__device__ __forceinline__ void s3_wait_barrier(int n) {
  switch (n) {
#define KNN_W(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")\n\ts_barrier" ::: "memory"); break;
    KNN_W(1) KNN_W(2) KNN_W(3) KNN_W(4) KNN_W(5) KNN_W(6) KNN_W(7) KNN_W(8) KNN_W(9) KNN_W(10)
    KNN_W(11) KNN_W(12) KNN_W(13) KNN_W(14) KNN_W(15)
#undef KNN_W
    default: asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
}

// Workgroup -> (query tile, split) of the S3 kernel.  gq = 0: XCD-contiguous
// ranges (xcd_remap), splits outer.  gq in {1, 2, 4, 8, 16, 32} (n_qt % gq == 0 and
// S % (32 / gq) == 0): the 32 workgroups an XCD runs at once (one per CU,
// workgroup w on XCD w % 8) form one group of gq query tiles x 32/gq splits,
// so each step's staged chunks are shared in the XCD's L2 -- a row chunk by
// gq workgroups, a query chunk by 32/gq -- instead of each workgroup's query
// images streaming through L2 on their own (32 query tiles per XCD with
// gq = 0: the query images are re-fetched for every train tile).
__device__ __forceinline__ void s3_map(int b, int nwg, int n_qt, int gq, int& qt, int& split) {
  if (gq == 0) {
    const int l = xcd_remap(b, nwg);
    split = l / n_qt;
    qt = l - split * n_qt;
    return;
  }
  // group index g: rounds of 256 workgroups (32 per XCD), XCD-major inside
  // a round; the tail of an incomplete round keeps its own order
  const int full = nwg & ~255;
  const int l = b < full ? (((b >> 3) >> 5) * 8 + (b & 7)) * 32 + ((b >> 3) & 31) : b;
  const int gs = 32 / gq;
  const int g = l >> 5, r = l & 31;
  const int ngq = n_qt / gq;  // groups along the query tiles
  const int sb = g / ngq, qb = g - sb * ngq;
  qt = qb * gq + r % gq;
  split = sb * gs + r / gq;
}

// Q16 (fp16 only): the same staging on v_mfma_f32_16x16x32_f16 -- wave w's
// 32 queries as 2 blocks of 16 against the tile's 256 rows as 16 blocks of
// 16 (32 accumulators of 4), one MFMA per block pair and chunk.  Lane l reads
// 16 B of row (or query) 16b + (l & 15), dims 8(l >> 4) .. +7 of the chunk;
// the fp16 image swizzle (s3h_slot) keeps those reads conflict-free as well
// as the 32x32 ones.  The output D holds rows 4(l >> 4) + i of a block for
// query l & 15, so the 4 lanes l & 15 + 16r keep one list each: 4 lists per
// query per split (the merge's quad layout, as cand_kernel's 16x16 paths).
// At the chip's power-limited clock the 16x16x32 shape sustains more FLOP/s
// than 32x32x16 for the same cycles per FLOP (MI355X_MICROARCH.md, DVFS
// give-back item 7).
template <int R, bool F16, bool Q16>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(KNN_S3_WPE, KNN_S3_WPE)))
cand_s3_kernel(const unsigned short* XT, const float* XS, const unsigned short* QT, int nch,
               int n_tiles, int S, int n_qt, float* __restrict__ out_v, int* __restrict__ out_i,
               int abl, int gq, uint32_t* gthr, int gk) {
#if !KNN_ABLATIONS
  abl = 0;  // (folds every ablation check below)
#endif
  static_assert(F16 || !Q16, "the 16x16x32 S3 layout is fp16 only");
  // gthr / gk (Q16 only; null / 0: none): the per-query global threshold of
  // cand_kernel -- at tiles 0, 1, 2, 4 and every 4th tile each workgroup
  // publishes, per query, the gk-th smallest of the union of the query's 4
  // lists (quad_union_kth16) into slot split % 8 (atomicMin) and fetches the
  // 8 slots by LDS-DMA; the max over them has >= 8 gk rows at or below it and
  // joins the quad's filter at the tile's epilogue.
  // abl: timing-only ablations as in cand_kernel (bit0 no staging after the
  // first steps, bit1 no selection epilogue); 0 in production.
  constexpr int BLK = kS3R * 64;        // bytes of one operand image
  constexpr int BUFB = 2 * BLK + 1024;  // A (rows) | B (queries) | seeds
  constexpr int NB = KNN_S3_NB;  // LDS buffers: prefetch distance NB - 1 steps
  constexpr int PD = NB - 1;
  static_assert(4 * (PD - 1) + PD <= 15, "vmcnt wait range");
  __shared__ __attribute__((aligned(16))) unsigned char lds[NB * BUFB];
  __shared__ __attribute__((aligned(16))) u32x4 gls[Q16 ? 8 * 64 : 1];

  int qt, split;
  s3_map(blockIdx.x, gridDim.x, n_qt, gq, qt, split);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, h = lane >> 5;
  const int64_t qg = (int64_t)qt * kS3Q + wv * 32 + j;
  // fragment byte offsets inside an image (the swizzle depends on j only:
  // rows 32b + j and 32w + j share (r >> 2) & 3)
  const int sw = F16 ? s3h_swz(j >> 2) : (j >> 2) & 3;
  const int off_hi = j * 64 + ((h ^ sw) << 4);
  const int off_lo = j * 64 + (((2 + h) ^ sw) << 4);
  const int off_q = wv * 32 * 64;
  // Q16: row/query (l & 15) of a 16-block, slot l >> 4
  const int c16 = lane & 15, g16 = lane >> 4;
  const int off_16 = c16 * 64 + ((g16 ^ s3h_swz(c16 >> 2)) << 4);

  const int my_nt = split < n_tiles ? (n_tiles - split + S - 1) / S : 0;
  const int total = my_nt * nch;
  const uint32_t lds_base =
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds;

  // issue cursor (chunk, tile, buffer) of the next step to stage
  int ic = 0, itile = split, ib = 0;
  auto issue = [&]() {
    const char* gA = (const char*)XT + ((int64_t)itile * nch + ic) * BLK + lane * 16;
    const char* gB = (const char*)QT + ((int64_t)qt * nch + ic) * BLK + lane * 16;
    const uint32_t l = lds_base + (uint32_t)(ib * BUFB);
    glds16(gA + wv * 1024, l + wv * 1024);
    glds16(gA + (wv + 8) * 1024, l + (wv + 8) * 1024);
    glds16(gB + wv * 1024, l + BLK + wv * 1024);
    glds16(gB + (wv + 8) * 1024, l + BLK + (wv + 8) * 1024);
    if (ic == 0 && wv == 0)
      glds16((const char*)(XS + (int64_t)itile * kS3R) + lane * 16, l + 2 * BLK);
    if (++ic == nch) { ic = 0; itile += (abl & 8) ? 0 : S; }  // abl bit 3: see cand_kernel
    if (++ib == NB) ib = 0;
  };

  constexpr int NQL = Q16 ? 2 : 1;  // lists per lane (Q16: one per query block)
  float L[NQL][R];
  int I[NQL][R];
  float thr[NQL];
#pragma unroll
  for (int b = 0; b < NQL; ++b) {
#pragma unroll
    for (int t = 0; t < R; ++t) { L[b][t] = KNN_INF_F; I[b][t] = -1; }
    thr[b] = KNN_INF_F;
  }

  // Q16 global threshold state (see above); the exchange's ops stay in flight
  // across PD barriers (counted into their waits) and the slots are read
  // after the barrier that retires them
  const bool gx = Q16 && gthr && gk > 0;
  const uint32_t goff = (uint32_t)(((int64_t)qt * kS3Q + wv * 32 + (lane & 31)) * (4 * kGthrSlots));
  const uint32_t gls_addr =
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) u32x4*)gls + wv * 1024;
  float tq[2] = {KNN_INF_F, KNN_INF_F};
  uint32_t last_pub = kKeyInf;
  int x_ops = 0, x_age = -1;
  if (gx && KNN_X_START && total > 0) {
    // the slots as they stand now (published by earlier grid rounds), fetched
    // before step 0's pieces: step 0's wait retires them and they are read
    // right after it (x_age = PD + 1 there, no extra count)
    glds16((const char*)gthr + goff + 16 * h, gls_addr);
    x_age = PD;
  }
#pragma unroll
  for (int p = 0; p < PD; ++p)
    if (total > p) issue();

  f32x16 acc[8];
  f32x4 aq[16][2];  // Q16: [row block][query block]
  int c = 0, t = split, cb = 0, ti = 0;
  for (int st = 0; st < total; ++st) {
    // own pieces of step st landed (those of st+1 may still be in flight),
    // then the barrier publishes every wave's pieces and retires all reads
    // of the buffer that the issue below refills.
    // (the younger steps st+1 .. st+y stay in flight: 4 pieces each, wave 0
    // one more -- the seeds -- for a step that opens a tile)
    {
      const int y = min(PD - 1, total - 1 - st);
      int n = 4 * y;
      if (wv == 0)
        for (int jj = 1; jj <= y; ++jj) n += (c + jj) % nch == 0;
      if (abl & 1) n = 0;
      if (x_age >= 0) ++x_age;
      if (x_age >= 1 && x_age <= PD) n += x_ops;
      // (wave-uniform: scalar branches to the right immediate, not an
      // exec-masked tree -- the divergence analysis cannot prove it)
      s3_wait_barrier(__builtin_amdgcn_readfirstlane(n));
    }
    __builtin_amdgcn_sched_barrier(0);
    if (st + PD < total && !(abl & 1)) issue();
    if constexpr (Q16) {
      if (gx) {
        if (x_age == PD + 1) {
#pragma unroll
          for (int qb = 0; qb < 2; ++qb) {
            const u32x4 g0 = gls[wv * 64 + 16 * qb + c16], g1 = gls[wv * 64 + 16 * qb + c16 + 32];
            tq[qb] = key2f(max(max(max(g0.x, g0.y), max(g0.z, g0.w)),
                               max(max(g1.x, g1.y), max(g1.z, g1.w))));
          }
          x_age = -1;
        }
        if (x_age < 0 && c == 0 && st + PD < total &&
            (ti < 4 ? ti != 3 : (ti & 3) == 0)) {
          const float m0 = quad_union_kth16(L[0], gk), m1 = quad_union_kth16(L[1], gk);
          const uint32_t pk = f2key(g16 == 0 ? m0 : m1);
          const bool pub = g16 < 2 && pk < last_pub;
          x_ops = 1;
          if (__ballot(pub)) {
            if (pub)
              asm volatile("global_atomic_umin %0, %1, %2" ::"v"(goff), "v"(pk),
                           "s"(gthr + (split & 7))
                           : "memory");
            x_ops = 2;
          }
          if (pub) last_pub = pk;
          glds16((const char*)gthr + goff + 16 * h, gls_addr);
          x_age = 0;
        }
      }
    }

    const unsigned char* buf = lds + cb * BUFB;
    if constexpr (Q16) {
      if (c == 0) {
        const float* seed = (const float*)(buf + 2 * BLK);
#pragma unroll
        for (int rb = 0; rb < 16; ++rb) {
          const float4 s4 = *(const float4*)(seed + 16 * rb + 4 * g16);
          aq[rb][0] = aq[rb][1] = f32x4{s4.x, s4.y, s4.z, s4.w};
        }
      }
      const f16x8 b0 = *(const f16x8*)(buf + BLK + off_q + off_16);
      const f16x8 b1 = *(const f16x8*)(buf + BLK + off_q + 16 * 64 + off_16);
      // A fragments through a ring of KNN_S3_RING registers: the read of row
      // block rb + RING is issued as block rb's two MFMAs go out, so RING - 1
      // reads are in flight behind the MFMAs instead of the one or two the
      // compiler's own schedule keeps (its just-in-time reads left each wave
      // waiting on LDS latency every two MFMAs, with only two waves per SIMD
      // to cover it)
      constexpr int RING = KNN_S3_RING;
      f16x8 ar[RING];
#pragma unroll
      for (int i = 0; i < RING; ++i) ar[i] = *(const f16x8*)(buf + i * 16 * 64 + off_16);
#if KNN_S3_SCHED
      __builtin_amdgcn_sched_group_barrier(0x100, RING + 2, 0);  // B pair + ring fill first
#endif
#pragma unroll
      for (int rb = 0; rb < 16; ++rb) {
        const f16x8 a = ar[rb % RING];
        aq[rb][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b0, aq[rb][0], 0, 0, 0);
        aq[rb][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b1, aq[rb][1], 0, 0, 0);
        if (rb + RING < 16) ar[rb % RING] = *(const f16x8*)(buf + (rb + RING) * 16 * 64 + off_16);
#if KNN_S3_SCHED
        // pin the order: 2 MFMAs, then the ring refill
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
#endif
      }
      if (c == nch - 1) {
        if (!(abl & 2)) {
#pragma unroll
          for (int qb = 0; qb < 2; ++qb) {
            // the quad's shared filter once per tile (min over its 4 lists'
            // R-th entries: anything dropped is >= some list's final R-th)
            const float tf = __builtin_fminf(quad_min(L[qb][R - 1]), tq[qb]);
#pragma unroll
            for (int rb = 0; rb < 16; rb += 2)
              select_quad_f<R>(aq[rb][qb], aq[rb + 1][qb], t * kS3R + 16 * rb + 4 * g16, L[qb],
                               I[qb], tf);
          }
        } else if (aq[0][0][0] == 1234.5f && aq[15][1][3] == 1234.5f) {
          thr[0] = aq[7][0][2];  // keep the accumulators live
        }
      }
      if (++c == nch) { c = 0; t += S; ++ti; }
      if (++cb == NB) cb = 0;
      continue;
    }
    if (c == 0) {
      const float* seed = (const float*)(buf + 2 * BLK);
#pragma unroll
      for (int bb = 0; bb < 8; ++bb) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 s4 = *(const float4*)(seed + 32 * bb + 8 * g + 4 * h);
          acc[bb][4 * g] = s4.x;
          acc[bb][4 * g + 1] = s4.y;
          acc[bb][4 * g + 2] = s4.z;
          acc[bb][4 * g + 3] = s4.w;
        }
      }
    }
    if constexpr (F16) {
      // k-step 0 = dims 0-15 of the chunk (slots 0, 1), k-step 1 = 16-31 (2, 3)
      const f16x8 b0 = *(const f16x8*)(buf + BLK + off_q + off_hi);
      const f16x8 b1 = *(const f16x8*)(buf + BLK + off_q + off_lo);
#pragma unroll
      for (int bb = 0; bb < 8; ++bb) {
        const f16x8 a0 = *(const f16x8*)(buf + bb * 32 * 64 + off_hi);
        const f16x8 a1 = *(const f16x8*)(buf + bb * 32 * 64 + off_lo);
        acc[bb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc[bb], 0, 0, 0);
        acc[bb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, acc[bb], 0, 0, 0);
      }
    } else {
      const bf16x8 bh = *(const bf16x8*)(buf + BLK + off_q + off_hi);
      const bf16x8 bl = *(const bf16x8*)(buf + BLK + off_q + off_lo);
#pragma unroll
      for (int bb = 0; bb < 8; ++bb) {
        const bf16x8 ah = *(const bf16x8*)(buf + bb * 32 * 64 + off_hi);
        const bf16x8 al = *(const bf16x8*)(buf + bb * 32 * 64 + off_lo);
        acc[bb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[bb], 0, 0, 0);
        acc[bb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[bb], 0, 0, 0);
        acc[bb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[bb], 0, 0, 0);
      }
    }
    if (c == nch - 1) {
      if (!(abl & 2)) {
#pragma unroll
        for (int bb = 0; bb < 8; ++bb)
          select_block<R>(acc[bb], t * kS3R + 32 * bb, h, L[0], I[0], thr[0], KNN_INF_F);
      } else if (acc[0][0] == 1234.5f && acc[7][15] == 1234.5f) {
        thr[0] = acc[3][7];  // keep the accumulators live
      }
    }
    if (++c == nch) { c = 0; t += S; }
    if (++cb == NB) cb = 0;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (Q16) {
    // [query][4S][R], as cand_kernel's 16x16 layouts
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int64_t q = (int64_t)qt * kS3Q + wv * 32 + 16 * qb + c16;
      const int64_t o = (q * (4 * S) + split * 4 + g16) * R;
#pragma unroll
      for (int e = 0; e < R; e += 4) {
        *(float4*)(out_v + o + e) = make_float4(L[qb][e], L[qb][e + 1], L[qb][e + 2], L[qb][e + 3]);
        *(int4*)(out_i + o + e) = make_int4(I[qb][e], I[qb][e + 1], I[qb][e + 2], I[qb][e + 3]);
      }
    }
  } else {
    write_lists<R>(out_v, out_i, qg, S, split, h, L[0], I[0]);
  }
}


int pad_dim(int d) {
#define KNN_CASE(v) if (d <= v) return v;
  KNN_DP_LIST(KNN_CASE)
#undef KNN_CASE
  return (d + kStreamDC - 1) / kStreamDC * kStreamDC;  // streamed kernel
}

bool cand_supported(int DP) { return DP > 0 && pad_dim(DP) == DP; }

// bf16x3 path: resident kernel for DP <= 256 (a multiple of 16 in the
// resident list), the S3 stream kernel above it (any multiple of 16).
int pad_dim_bf16x3(int d) {
  const int d16 = (d + 15) / 16 * 16;
  if (d16 > 256) return d16;
  const int DP = pad_dim(d16);
  return (DP <= 256 && DP % 16 == 0) ? DP : -1;
}

bool bf16x3_streamed(int DP) { return DP > 256; }

// fp16 path: resident 16x16x32 kernel, DP % 32 == 0 and <= 256.
int pad_dim_fp16(int d) {
  const int DP = pad_dim((d + 31) / 32 * 32);
  return (DP <= 256 && DP % 32 == 0) ? DP : -1;
}

// int8 path: the resident 16x16x64 kernel, DP a multiple of 64, <= 256
int pad_dim_i8(int d) {
  const int DP = (d + 63) / 64 * 64;
  return DP <= 256 ? DP : -1;
}

// int8 on the 32x32x32 kernel (metric 6): the smallest resident DP >= d
// that is a multiple of 32 (d = 96 -> 96, where 16x16x64 pads to 128)
int pad_dim_i8w(int d) {
  for (int DP : {32, 64, 96, 128, 160, 192, 256})
    if (DP >= d) return DP;
  return -1;
}

// fp16 S3 kernel above 256 dims: any multiple of 32
int pad_dim_fp16_s3(int d) {
  const int DP = (d + 31) / 32 * 32;
  return DP > 256 ? DP : -1;
}

int s3_blocks_per_cu(int R) {
  return R == 8 ? occupancy_of(cand_s3_kernel<8, false, false>, 512)
                : occupancy_of(cand_s3_kernel<16, false, false>, 512);
}

int s3h_blocks_per_cu(int R) {
  return R == 8 ? occupancy_of(cand_s3_kernel<8, true, false>, 512)
                : occupancy_of(cand_s3_kernel<16, true, false>, 512);
}

// the S3 grouping (s3_map) that n_qt and S admit, the largest up to gq_max
// (a row chunk then serves gq workgroups of the XCD, a query chunk 32 / gq):
// 32, 16, 8, 4, 2, 1, else 0
int s3_group(int n_qt, int S, int gq_max) {
  for (int gq : {32, 16, 8, 4, 2, 1})
    if (gq <= gq_max && n_qt % gq == 0 && S % (32 / gq) == 0) return gq;
  return 0;
}

void launch_cand_s3(const unsigned short* XT, const float* XS, const unsigned short* QT, int DP,
                    int64_t n_pad, int R, int S, int n_qt, float* out_v, int* out_i, int ablate,
                    hipStream_t s, int gq_max) {
  const int gq = s3_group(n_qt, S, gq_max);
  const int nch = DP / kS3DC;
  const int n_tiles = (int)(n_pad / kS3R);
  if (R == 8)
    hipLaunchKernelGGL((cand_s3_kernel<8, false, false>), dim3((unsigned)(n_qt * S)), dim3(512), 0, s, XT,
                       XS, QT, nch, n_tiles, S, n_qt, out_v, out_i, ablate, gq, nullptr, 0);
  else
    hipLaunchKernelGGL((cand_s3_kernel<16, false, false>), dim3((unsigned)(n_qt * S)), dim3(512), 0, s, XT,
                       XS, QT, nch, n_tiles, S, n_qt, out_v, out_i, ablate, gq, nullptr, 0);
}

void launch_cand_s3h(const unsigned short* XT, const float* XS, const unsigned short* QT, int DP,
                     int64_t n_pad, int R, int S, int n_qt, float* out_v, int* out_i, int ablate,
                     bool q16, uint32_t* gthr, int gk, hipStream_t s, int gq_max) {
  const int gq = s3_group(n_qt, S, gq_max);
  const int nch = DP / 32;
  const int n_tiles = (int)(n_pad / kS3R);
  const dim3 g((unsigned)(n_qt * S)), b(512);
  if (q16)
    hipLaunchKernelGGL((cand_s3_kernel<8, true, true>), g, b, 0, s, XT, XS, QT, nch, n_tiles, S,
                       n_qt, out_v, out_i, ablate, gq, q16 ? gthr : nullptr, q16 ? gk : 0);
  else if (R == 8)
    hipLaunchKernelGGL((cand_s3_kernel<8, true, false>), g, b, 0, s, XT, XS, QT, nch, n_tiles, S,
                       n_qt, out_v, out_i, ablate, gq, q16 ? gthr : nullptr, q16 ? gk : 0);
  else
    hipLaunchKernelGGL((cand_s3_kernel<16, true, false>), g, b, 0, s, XT, XS, QT, nch, n_tiles, S,
                       n_qt, out_v, out_i, ablate, gq, q16 ? gthr : nullptr, q16 ? gk : 0);
}

int s3q_blocks_per_cu() { return occupancy_of(cand_s3_kernel<8, true, true>, 512); }

template <int R, int METRIC>
static void launch_str(const CandLaunch& c, hipStream_t s) {
  hipLaunchKernelGGL((cand_stream_kernel<kStreamDC, R, METRIC>), dim3((unsigned)(c.n_qt * c.S)),
                     dim3(256), 0, s, c.X32, c.xinit, c.Q32, c.DP, (int)(c.n_pad / 128), c.S,
                     c.n_qt, c.out_v, c.out_i);
}

int cand_blocks_per_cu(int metric, int DP, int R, int nw) {
  if (metric == 2 && bf16x3_streamed(DP)) return s3_blocks_per_cu(R);
  if (metric == 4 && DP > 256) return s3h_blocks_per_cu(R);
#define KNN_CASE(v) if (DP == v) return blocks_res_##v(R, metric, nw);
  KNN_DP_LIST(KNN_CASE)
#undef KNN_CASE
  int out = 1;
  if (R == 8)
    out = occupancy_of(metric == 1 ? cand_stream_kernel<kStreamDC, 8, 1>
                                   : cand_stream_kernel<kStreamDC, 8, 0>, 256);
  else
    out = occupancy_of(metric == 1 ? cand_stream_kernel<kStreamDC, 16, 1>
                                   : cand_stream_kernel<kStreamDC, 16, 0>, 256);
  return out;
}

// queries per wave of the resident kernel serving (metric, DP), from the
// object that holds that kernel (a variant build's KNN_I8_QB)
int cand_queries_per_wave(int metric, int DP) {
#define KNN_CASE(v) if (DP == v) return qpw_res_##v(metric);
  KNN_DP_LIST(KNN_CASE)
#undef KNN_CASE
  return 32;
}

int cand_tile_rows(int metric, int DP) {
  if ((metric == 2 && bf16x3_streamed(DP)) || (metric == 4 && DP > 256)) return kS3R;
#define KNN_CASE(v) if (DP == v) return trows_res_##v(metric);
  KNN_DP_LIST(KNN_CASE)
#undef KNN_CASE
  return 128;  // cand_stream_kernel
}

bool launch_cand(const CandLaunch& c, hipStream_t s) {
#define KNN_CASE(v) \
  if (c.DP == v) return launch_res_##v(c, s);
  KNN_DP_LIST(KNN_CASE)
#undef KNN_CASE
  if (c.ev_start) (void)hipEventRecord(c.ev_start, s);
  if (c.R == 8) {
    if (c.metric == 1) launch_str<8, 1>(c, s);
    else launch_str<8, 0>(c, s);
  } else {
    if (c.metric == 1) launch_str<16, 1>(c, s);
    else launch_str<16, 0>(c, s);
  }
  if (c.ev_stop) (void)hipEventRecord(c.ev_stop, s);
  return true;
}

}  // namespace knnk
