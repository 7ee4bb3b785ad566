// knn_cand_res.hip -- the register-resident candidate kernel (d <= 256),
// compiled once per group of padded dimensions (-DKNN_GROUP=0..3) so the
// many (DP, R, metric, waves) instantiations build in parallel.
#include "knn_device.h"

#include <hip/hip_ext.h>

// Staging geometry (build-time; tools/build_variant.sh overrides for A/B):
// 2 LDS buffers of 64-row tiles (two 32-row MFMA sub-tiles per barrier).
// Measured against 3 buffers of 32-row tiles: -5.5 % (bf16x3) / -3 % (fp32).
#ifndef KNN_RES_NB
#define KNN_RES_NB 2
#endif
#ifndef KNN_RES_TPB
#define KNN_RES_TPB 2
#endif
static_assert(KNN_RES_TPB * knnk::kTR == knnk::kResTileRows || KNN_RES_TPB != 2,
              "default tile rows must match kResTileRows");
// fp16 kernel (METRIC 4) experiments: sub-tiles per staged tile, per-tile
// cached quad thresholds, seeds read as one float4 per 4 rows
#ifndef KNN_M4_TPB
#define KNN_M4_TPB 4
#endif
#ifndef KNN_M4_TE_CACHE
#define KNN_M4_TE_CACHE 1
#endif
#ifndef KNN_SETPRIO
#define KNN_SETPRIO 0
#endif
#ifndef KNN_M4_SEED4
#define KNN_M4_SEED4 1
#endif
// fp16 kernel: the selection of sub-tile s runs after the MFMAs of sub-tile
// s+1 are issued (its accumulators are complete by then), so a wave never
// waits for its own MFMA chains to drain before its min-trees
#ifndef KNN_M4_PIPE
#define KNN_M4_PIPE 1
#endif
// fp16 kernel: A-fragment reads kept KNN_M4_SCHED ahead of the MFMAs by
// sched_group_barrier (0: the compiler's own schedule)
#ifndef KNN_M4_SCHED
#define KNN_M4_SCHED 0
#endif
#ifndef KNN_RFL
#define KNN_RFL 1
#endif
// int8 kernel: 32-row sub-tiles per staged tile (8: 256-row tiles, half the
// barriers and per-tile work per MFMA of 128-row tiles, and a 256-row lead
// for the streamed rows; n_pad is a multiple of kRowAlign = 256): cfg2
// candidate pass 1.636 -> 1.50 ms against 4 (profiles/ab_log.md: r3c_ab_*), where
// a third LDS buffer of 128-row tiles measured +4 % and 64 queries per wave
// +12 %
#ifndef KNN_I8_TPB
#define KNN_I8_TPB 8
#endif
// int8 kernel: all A-fragment reads of a sub-tile issued before its MFMAs
#ifndef KNN_I8_SCHED
#define KNN_I8_SCHED 1
#endif
// int8 kernel: 16-query blocks per wave (2: 32 queries per wave as the fp16
// kernel; 4: 64 queries, each A fragment read from LDS feeds 4 MFMAs) and
// the waves-per-SIMD target of the 4-block form (its registers exceed 128)
// int8 kernel: LDS buffers (2: tile it+1 streams in behind tile it's
// compute; 3: two tiles of lead -- the int8 tile's compute is half the
// fp16 one's, too short to cover an HBM fetch)
#ifndef KNN_I8_NB
#define KNN_I8_NB 2
#endif
#ifndef KNN_I8_QB
#define KNN_I8_QB 2
#endif
#ifndef KNN_I8_WPE
#define KNN_I8_WPE 2
#endif
// int8 kernels: seed-free accumulation.  The accumulators start at zero (no
// LDS read of the rows' seeds per sub-tile: 4 of the 7 ds_read_b128 per
// metric-6 sub-tile, 2 of 6 at metric 5) and a sub-tile's no-candidate test
// adds the largest seed of its 32 rows (kI8SmaxRow pads, 2 reads per staged
// tile); only a wave whose bound passes reads the exact seeds and runs the
// exact selection.  The bound is tight on norm-blocked images (knn_order.hip):
// 7.6 % of metric-6 sub-tile tests pass it at cfg2 against 7.56 % passing
// exactly (profiles/ab_log.md r5e).  Metric 6 (KNN_I8_SMAX): the 12.5M x 96
// shard 12.06 -> 11.72 ms (r5d4; bare MFMA + LDS loop 9.84 -> 9.25 ms, r5c4).
// Metric 5 (KNN_I8_SMAX5, off): that loop is not LDS-bound (bare loop 0.912 vs
// 0.913 ms, r5b) but issue-bound -- a 16x16x64 MFMA holds the SIMD's vector
// issue for 8 of its 16 cycles and the selection already spends ~4 VALU per
// MFMA -- so the bound's extra VALU made cfg2 slower (1.41 vs 1.26-1.29 ms, r5d).
#ifndef KNN_I8_SMAX
#define KNN_I8_SMAX 1
#endif
#ifndef KNN_I8_SMAX5
#define KNN_I8_SMAX5 0
#endif
// int8 on 32x32x32 (metric 6) with R = 4: each lane keeps TWO lists of 4,
// one per half of its 16 rows (i < 8: rows (i&3) + 8(i>>2), c = 0, 1; i >= 8:
// c = 2, 3) -- 4 lists of 4 per query per split, the merge's quad layout of
// the 16x16 kernels -- instead of one list of 8: an insertion then shifts 4
// entries instead of 8 (the selection's slow path is most of its cost,
// profiles/ab_log.md r5e) at the 16x16 kernels' certification odds.
#ifndef KNN_I8W_Q4
#define KNN_I8W_Q4 1
#endif
// metric 6: issue priority of a wave inside its selection slow path (0:
// none).  At 2: cfg2 candidate -1.1 %, the 12.5M x 96 shard -0.6 % in every
// interleaved pair (profiles/ab_log.md r5ag)
#ifndef KNN_SLOWPRIO
#define KNN_SLOWPRIO 2
#endif
// metric 6: waves NW/2 .. NW-1 walk a staged tile's sub-tiles rotated by
// TPB/2 (a stagger, MI355X_MICROARCH.md "Two waves per SIMD" item 9): the
// two halves' LDS bursts and selection slow paths then fall on different
// sub-tiles instead of in lockstep
#ifndef KNN_STAGGER
#define KNN_STAGGER 0
#endif
#ifndef KNN_STAGGER4
#define KNN_STAGGER4 0
#endif
// metric 6: the exact seeds of a staged tile's last sub-tile (its selection
// runs after the next tile's barrier, when the buffer may be refilled) are
// read in the rare slow path from the image in HBM / L2 by wave-uniform
// scalar loads (32 seeds per sub-tile, 8 x s_load_dwordx4) instead of being
// held in 16 VGPRs from the sub-tile's LDS reads
#ifndef KNN_SPRE_GLB
#define KNN_SPRE_GLB 0
#endif
#ifndef KNN_I8W_PF
#define KNN_I8W_PF 0
#endif
// metric 6: early prune on a partial distance.  After the MFMAs of the first
// i8_part_dims(DP) dims of a sub-tile (all but the last 32), the partial
// accumulators q_A.k_A plus the sub-tile's largest partial seed bound every
// full accumulator from above, up to the query's remaining norm:
//   q.k - ceil(|k|^2/2) <= (q_A.k_A - ceil(|k_A|^2/2)) + (|q_B|^2 + 1) / 2
// (|q_B - k_B|^2 >= 0), so a wave none of whose values passes tn - hq, hq =
// ceil((|q_B|^2 + 1) / 2), has no candidate in the sub-tile and skips its
// last MFMA; its pending selection then never passes (smx = kI8Pruned).
#ifndef KNN_I8_PART
#define KNN_I8_PART 0
#endif
// metric 6 (experiment): also a 16-wave form (512 queries per staged tile:
// half the L2 -> LDS staging bytes per MFMA; one workgroup per CU), selected
// with tuning "nw" 16
#ifndef KNN_I8W_NW16
#define KNN_I8W_NW16 0
#endif
// metric 6: barrier-free staging (experiment).  Instead of one s_barrier per
// staged tile, each buffer carries two LDS counters: ready (waves whose
// pieces of the buffer's tile have landed) and done (waves that finished
// reading it).  A wave starts tile it once every wave's pieces of it have
// landed, and issues its pieces of tile it+1 into the other buffer as soon
// as every wave has finished tile it-1 (polled after each sub-tile) -- so a
// wave may run up to a tile ahead of the slowest one instead of waiting for
// it at every tile (the no-barrier ablation: -16 %, round 5 r5e).
#ifndef KNN_I8_CTR
#define KNN_I8_CTR 0
#endif
// (KNN_I8_CTR) sub-tiles after issuing its pieces of the next tile at which a
// wave waits for them (vmcnt) and counts them ready -- early enough that the
// other waves need not wait for it to finish its tile, late enough that the
// pieces have landed from L2 / HBM
#ifndef KNN_CTR_SIGD
#define KNN_CTR_SIGD 4
#endif
// metric 6: the no-candidate test's max over 16 values as 7 v_max3 + 1 v_max
#ifndef KNN_MAX3T
#define KNN_MAX3T 0
#endif


namespace knnk {

#if KNN_COUNT_SEL
__device__ unsigned long long knn_sel_cnt[8];
#endif

// (lgkmcnt(0): every LDS read of the wave -- the int8 kernels' seed reads of
// a staged tile's last sub-tile among them -- has completed before any wave
// refills that tile's buffer after the barrier)
template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// The wait count plus `extra` younger exchange ops (see cand_kernel).
template <int BASE, int XMAX = 2>
__device__ __forceinline__ void wait_barrier_x(int extra) {
  if (XMAX >= 3 && extra == 3) wait_barrier<BASE + 3>();
  else if (extra == 2) wait_barrier<BASE + 2>();
  else if (extra == 1) wait_barrier<BASE + 1>();
  else wait_barrier<BASE>();
}

// (KNN_I8_CTR) wait until the LDS counter *p reaches target; bounded (a
// protocol error ends the wait after ~2^22 sleeps instead of hanging the GPU;
// the parity gate then sees wrong answers)
__device__ __forceinline__ void ctr_wait(int* p, int target) {
  for (int n = 0; n < (1 << 22); ++n) {
    if (__builtin_amdgcn_readfirstlane(*(volatile int*)p) >= target) break;
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

#ifndef KNN_PUB_EVERY
#define KNN_PUB_EVERY 8
#endif
constexpr int kPubEvery = KNN_PUB_EVERY;  // tiles between global-threshold exchanges (power of 2)
// Early exchanges (KNN_EARLY_X): also at tiles 0, 1, 2 and 4.  The fetch at
// tile 0 hands a workgroup of a later grid round the thresholds the earlier
// rounds already published, and the early publishes shorten every list's
// cold start -- the insertion-heavy tiles before a filter threshold exists,
// where some lane of the wave inserts on nearly every value.
#ifndef KNN_EARLY_X
#define KNN_EARLY_X 1
#endif
__device__ __forceinline__ bool exchange_tile(int it) {
  if (KNN_EARLY_X && it < 8 && kPubEvery >= 4) return it == 0 || it == 1 || it == 2 || it == 4;
  return (it & (kPubEvery - 1)) == kPubEvery - 1;
}

// waves per SIMD the resident kernel is compiled for: 4 (<= 128 VGPRs, two
// 8-wave workgroups per CU) where its registers fit
template <int DP, int R, int METRIC>
constexpr int res_wpe() {
  if (METRIC == 5 && KNN_I8_QB > 2) return KNN_I8_WPE;
  return (METRIC >= 5 ? DP / 4 : METRIC == 4 ? DP / 2 : DP) <= 160 && R <= 8 ? 4 : 1;
}

// queries per wave: 16 per query block (the 16x16 layouts), 32 otherwise
template <int METRIC>
constexpr int res_qpw() {
  return METRIC == 5 ? 16 * KNN_I8_QB : 32;
}

template <int METRIC>
constexpr int res_tpb() {
  return METRIC >= 5 ? KNN_I8_TPB : METRIC == 4 ? KNN_M4_TPB : KNN_RES_TPB;
}

// Train rows in HBM (X32 for fp32/L1, XB for bf16x3) share one padded row
// format of RSF = DP + 4 floats: [payload (DP floats) | ||x32||^2, l1 seed,
// 0, 0], where payload is DP fp32 values or [hi(DP) | lo(DP)] bf16.  A tile
// is 32 consecutive rows = one contiguous block, copied linearly into LDS;
// the odd 16-B row stride (DP/4 + 1 chunks) makes the A-fragment reads
// (ds_read_b128, 16-lane groups on distinct rows) bank-conflict free, and the
// accumulator seeds come from the same rows.  Pad rows carry +inf seeds.
//
// Workgroup = 4 waves = 128 queries; it streams the 32-row train tiles
// split, split+S, split+2S, ... (round-robin so a run of similar rows is
// spread over all splits).  Lane (j = lane&31, h = lane>>5) of wave w owns
// query j of the wave and the train rows rho(i,h) = (i&3) + 8(i>>2) + 4h of
// every tile (the 32x32 MFMA C/D layout with train rows on A, queries on B).
//
// METRIC 0, per tile and wave: DP/2 MFMAs 32x32x2 f32; lane (r, h) reads
// float4 X[r][8c+4h ..] for the four k-steps of group c.  METRIC 2: 3*DP/16
// MFMAs 32x32x16 bf16 (see below).  The B operand (queries, -2 q) stays in
// VGPRs for the whole kernel.  Accumulators start at ||x_row||^2, so
// acc = ||x||^2 - 2 q.x.
//
// NW waves (32 queries each) share every staged tile: NW = 8 halves the
// staging instructions and L2 traffic per MFMA relative to NW = 4.
//
// Staging: global_load_lds (LDS-DMA, no VGPRs) into NB = KNN_RES_NB LDS
// buffers (2 by default): tile it+NB-1 is issued right after the barrier
// that opens tile it, and each wave waits with a counted vmcnt for its own
// pieces of tile it before that barrier -- NB-1 tiles of latency hidden, one
// barrier per tile.  (A register-staged variant measured the same or
// slower; removed.)
// waves_per_eu(4): 4 waves per SIMD (<= 128 VGPRs), so two 8-wave workgroups
// share a CU and one's barrier/epilogue gaps are filled by the other's MFMAs
// (not for R = 16 lists or DP > 160, whose registers do not fit: spills).
template <int DP, int R, int METRIC, int NW>
__global__ void __launch_bounds__(NW * 64)
__attribute__((amdgpu_waves_per_eu(res_wpe<DP, R, METRIC>())))
cand_kernel(const float* __restrict__ Xr, const float* Q32, int n_tiles, int S,
            int n_qt, float* __restrict__ out_v, int* __restrict__ out_i, int abl,
            uint32_t* gthr, int gk, int xsw, const int* __restrict__ qstart, int gmask, int qblk) {
#if !KNN_ABLATIONS
  abl = 0;  // (folds every ablation check below)
#endif
#if KNN_SETPRIO
  // the second-dispatched half of the workgroup at priority 1 (MI355X_MICROARCH
  // "Two waves per SIMD", item 4)
  if ((threadIdx.x >> 6) >= NW / 2) __builtin_amdgcn_s_setprio(1);
#endif
  // Q32 is deliberately not __restrict__: with it hipcc treats the query
  // fragments as invariant and re-loads them inside the tile loop instead of
  // keeping them in VGPRs (its waits would then also drain the LDS-DMA queue).
  // abl: timing-only ablations (results invalid): bit0 = no staging loads
  // after the first tiles, bit1 = no selection epilogue, bit3 = staging
  // pieces always of an L2-resident tile, bit4 = no workgroup barrier (own
  // vmcnt wait only).  0 in production.
  // fp16 operands: METRIC 4 on the 16x16x32 layout; int8 codes: METRIC 5 on
  // v_mfma_i32_16x16x64_i8, the same fragment layout with 64 dims per MFMA
  constexpr bool F16 = METRIC == 4;
  constexpr bool I8 = METRIC == 5;
  // int8 codes on v_mfma_i32_32x32x32_i8 (METRIC 6): the 32x32 layout of
  // METRIC 0 (lane (j, h): query j, rows (i&3) + 8(i>>2) + 4h) with 32 dims
  // per MFMA, so d = 96, 160, 224 issue no padded dims (16x16x64 pads them
  // to a multiple of 64)
  constexpr bool I8W = METRIC == 6;
  constexpr bool I8A = I8 || I8W;  // either int8 form: int accumulators, seeds, int lists
  constexpr bool TEC = (F16 || I8A) && KNN_M4_TE_CACHE;
  constexpr int DPF = I8A ? DP / 4 : (F16 ? DP / 2 : DP);  // payload floats per row
  constexpr int RSF = DPF + 4;              // row stride (floats), HBM and LDS
  constexpr int TPB = res_tpb<METRIC>();    // 32-row sub-tiles per staged tile
  constexpr int TBY = kTR * TPB * RSF * 4;  // tile bytes
  constexpr int NG = (TBY + 1023) / 1024;   // 1-KiB LDS-DMA pieces per tile
  constexpr int NB = I8A ? KNN_I8_NB : KNN_RES_NB;  // LDS buffers (prefetch distance NB - 1)
  constexpr int BUFF = NG * 256;            // floats per buffer
  constexpr int SEED = METRIC == 1 ? DP + 1 : DPF;  // seed float within a row
  __shared__ __attribute__((aligned(16))) float lds[NB * BUFF];

  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  // workgroup -> (split, query tile): split-major (qblk 0: the XCD's
  // concurrent workgroups are one split's consecutive query tiles), or query
  // blocks of qblk tiles, splits outer inside a block (the first grid round
  // then holds most splits of the first blocks' queries)
  int split, qt;
  if (qblk > 0) {
    const int blk = bid / (qblk * S);
    const int qt0 = blk * qblk;
    const int bb = min(qblk, n_qt - qt0);
    const int w = bid - blk * qblk * S;
    split = w / bb;
    qt = qt0 + (w - split * bb);
  } else {
    split = bid / n_qt;
    qt = bid - split * n_qt;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, h = lane >> 5;
  // (KNN_STAGGER: this wave's sub-tile rotation, wave-uniform)
  // (KNN_STAGGER4: the same for the fp16 kernel, metric 4)
  const int rot = (((KNN_STAGGER && METRIC == 6) || (KNN_STAGGER4 && METRIC == 4)) && wv >= NW / 2)
                      ? res_tpb<METRIC>() / 2 : 0;
  const int64_t qg = (int64_t)qt * (NW * 32) + wv * 32 + j;
  const float* qrow = Q32 + qg * DP;
  // METRIC 3 (bf16x3 on 16x16x32) and 4 (fp16 on 16x16x32): lane l holds
  // queries wv*32 + qb*16 + (l&15), qb = 0, 1, against rows 4*(l>>4) + i of
  // each 16-row block
  constexpr bool M16 = METRIC == 3 || METRIC == 4 || I8;
  constexpr int QB = I8 ? KNN_I8_QB : 2;   // 16-query blocks per wave (M16)
  constexpr int QW = M16 ? 16 * QB : 32;   // queries per wave
  static_assert(QW == res_qpw<METRIC>(), "queries per wave: kernel and host disagree");
  const int c16 = lane & 15, g16 = lane >> 4;
  const int64_t qb0 = (int64_t)qt * (NW * QW) + wv * QW + c16;  // query of block 0 (+16 qb: block qb)

  // B operand resident in VGPRs for the whole kernel.  METRIC 0: fp32 -2q,
  // float4 c holds dims 8c+4h..8c+4h+3 (four 32x32x2 k-steps).  METRIC 2:
  // the row is [qh | ql] in bf16 (-2q split hi/lo); float4 t (t < DP/16) is
  // qh dims 16t+8h..16t+8h+7, float4 DP/16+t the same dims of ql.
  // METRIC 4: fp16 -2q (the train set's power-of-two scale), float4 qb*(DP/32)+ks
  // = dims 32ks + 8*g16 .. +7 of query block qb.
  // METRIC 5: int8 codes, float4 qb*(DP/64)+ks = dims 64ks + 16*g16 .. +15
  // METRIC 6: int8 codes, float4 ks = dims 32ks + 16h .. +15 of query j
  constexpr int NQF = METRIC == 1 ? 1 : I8W ? DP / 32 : (I8 ? QB * DP / 64 : (F16 ? QB * DP / 32 : DP / 8));
  float4 qf[NQF];
  if constexpr (METRIC != 1) {
    // Loaded with inline asm (loads + their vmcnt(0) in one statement): with
    // ordinary loads hipcc places the vmcnt waits for these registers at
    // their first MFMA use INSIDE the tile loop, where each executes every
    // tile and -- counting all vector-memory ops -- drains the in-flight
    // LDS-DMA pieces of the staging pipeline.
#pragma unroll
    for (int c0 = 0; c0 < NQF; c0 += 4) {
      const float* p[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = c0 + u < NQF ? c0 + u : c0;
        if constexpr (I8W) {
          p[u] = Q32 + qg * (DP / 4) + 8 * c + 4 * h;
        } else if constexpr (I8) {
          const int ks = c % (DP / 64), qb = c / (DP / 64);
          p[u] = Q32 + (qb0 + 16 * qb) * (DP / 4) + 16 * ks + 4 * g16;
        } else if constexpr (F16) {
          const int ks = c % (DP / 32), qb = c / (DP / 32);
          p[u] = Q32 + (qb0 + 16 * qb) * (DP / 2) + 16 * ks + 4 * g16;
        } else if constexpr (M16) {
          // c = (qb*2 + part)*(DP/32) + ks: dims 32ks + 8*g16 .. +7 of part
          const int ks = c % (DP / 32), pp = (c / (DP / 32)) & 1, qb = c / (DP / 16);
          p[u] = Q32 + (qb0 + 16 * qb) * DP + pp * (DP / 2) + 16 * ks + 4 * g16;
        } else {
          const int off = METRIC == 0 ? 8 * c : (c < DP / 16 ? 8 * c : DP / 2 + 8 * (c - DP / 16));
          p[u] = qrow + off + 4 * h;
        }
      }
      float4 v0, v1, v2, v3;
      asm volatile(
          "global_load_dwordx4 %0, %4, off\n\t"
          "global_load_dwordx4 %1, %5, off\n\t"
          "global_load_dwordx4 %2, %6, off\n\t"
          "global_load_dwordx4 %3, %7, off\n\t"
          "s_waitcnt vmcnt(0)"
          : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
          : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3])
          : "memory");
      qf[c0] = v0;
      if (c0 + 1 < NQF) qf[c0 + 1] = v1;
      if (c0 + 2 < NQF) qf[c0 + 2] = v2;
      if (c0 + 3 < NQF) qf[c0 + 3] = v3;
    }
  }

  constexpr int NQL = M16 ? QB : 1;  // queries (lists) per lane
  // int8: lists of the accumulators themselves (KNN_I8_ILIST, knn_device.h)
  constexpr bool ILIST = I8A && KNN_I8_ILIST;
  using LT = std::conditional_t<ILIST, int, float>;
  LT L[NQL][R];
  int I[NQL][R];
  float thr[NQL];
#pragma unroll
  for (int b = 0; b < NQL; ++b) {
#pragma unroll
    for (int t = 0; t < R; ++t) {
      if constexpr (ILIST) L[b][t] = kI8Floor;
      else L[b][t] = KNN_INF_F;
      I[b][t] = -1;
    }
    thr[b] = KNN_INF_F;
  }
  // W4 (KNN_I8W_Q4, metric 6 at R = 4): the lane's second list (rows of its
  // values i >= 8); L[0] holds i < 8
  constexpr bool W4 = I8W && R == 4 && KNN_I8W_Q4 && ILIST && KNN_I8_SMAX;
  int L2[W4 ? R : 1], I2[W4 ? R : 1];
#pragma unroll
  for (int t = 0; t < (W4 ? R : 1); ++t) {
    L2[t] = kI8Floor;
    I2[t] = -1;
  }
  // the lane's lists' threshold (the smaller R-th proxy of the two under W4:
  // the merge bounds dropped rows by the min over a split's lists)
  auto lane_thr = [&]() {
    if constexpr (W4) return __builtin_fminf(lval(L[0][R - 1]), lval(L2[R - 1]));
    else return lval(L[0][R - 1]);
  };
  // the int8 selection on either list form
  auto select_i8 = [&](const auto& a, const auto& b, int row0, auto& Lq, auto& Iq, float& teq,
                       int& tnq, SelCount& sc) {
    if constexpr (ILIST && KNN_I8_SLOW == 2) select_quad_i8t<R>(a, b, row0, Lq, Iq, tnq, sc);
    else if constexpr (ILIST) select_quad_i8i<R>(a, b, row0, Lq, Iq, tnq, sc);
    else select_quad_i8<R>(a, b, row0, Lq, Iq, teq, tnq, sc);
  };

  // Global per-query threshold.  The query's lists are spread over S
  // workgroups; they form G groups by split % G (disjoint row sets), and slot
  // g of gthr[query] (kGthrSlots keys) holds the min over group g's published
  // values (order-preserving keys, atomicMin).  gk = 0 (G = 4): a value is a
  // list's R-th entry, so group g has R rows at or below its slot.  gk = K in
  // 1..4 (G = 8): a value is the K-th smallest of the union of the query's
  // lists in this workgroup (its 2 or 4 lanes), so group g has K rows at or
  // below its slot -- a far smaller value than any one list's R-th entry
  // (the K-th of a whole split against the R-th of a quarter of it).  Either
  // way tq = max over the slots has >= G x (R or K) distinct rows at or below
  // it: any row above tq is outside the query's best G x (R or K) and may be
  // dropped.  The merge bounds dropped rows by the final tq.  Lists then stop
  // filling with rows only a cold list would keep -- the insertions (64
  // independent lists per wave) that dominate the epilogue.
  // Lanes l and l+32 (same query) fetch slots 0-3 and 4-7 by LDS-DMA into this
  // wave's 1-KiB area of gls (16 B per lane); they are read after the next
  // barrier: a plain load into VGPRs would be consumed (or copied) by
  // compiler code before it lands.
  // (64 queries per wave: lane l fetches both halves of query l's slots,
  // into this wave's 2-KiB area)
  constexpr int GW = QW > 32 ? 128 : 64;  // gls entries per wave
  constexpr int XMAX = GW == 128 ? 3 : 2;  // exchange ops in flight at most
  __shared__ __attribute__((aligned(16))) u32x4 gls[NW * GW];
  // (KNN_I8_CTR) ready[2] | done[2] counters of the two staging buffers
  constexpr bool CTR = METRIC == 6 && KNN_I8_CTR && KNN_I8_NB == 2;
  __shared__ int s_ctr[CTR ? 4 : 1];
  if constexpr (CTR) {
    if (threadIdx.x < 4) s_ctr[threadIdx.x] = 0;
    __syncthreads();
  }
  const uint32_t gls_addr =
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) u32x4*)gls + wv * GW * 16;
  // An exchange at tile e issues (after that tile's DMA pieces) an atomic
  // (only if some lane improved) and the slot fetch; the barriers of tiles
  // e+1 .. e+PD-1 leave those x ops in flight (counted wait + x), the
  // barrier of tile e+PD retires them and the slots are read after it -- no
  // barrier ever waits on a (contended) atomic.
  // byte offset of gthr[query][0]: the lane's query, or for METRIC 3/4 query
  // (l & 31) of the wave (lanes 0-15 block 0, 16-31 block 1; 32-63 repeat)
  const uint32_t goff =
      M16 ? (uint32_t)(((int64_t)qt * (NW * QW) + wv * QW + (lane & (QW - 1))) * (4 * kGthrSlots))
          : (uint32_t)(qg * (4 * kGthrSlots));
  // slot group of this split: split % G, G = gmask + 1 (8 with gk > 0 by
  // default, 4 for the lists' R-th entries; the host may use 4 with gk > 0)
  const uint32_t* gslot = gthr + (split & gmask);
  float tq[NQL], te[NQL];
  int tn[NQL];  // int8: i8_neg_half(te), the filter on the accumulators
#pragma unroll
  for (int b = 0; b < NQL; ++b) {
    tq[b] = te[b] = KNN_INF_F;
    tn[b] = kI8Floor;
  }
  uint32_t last_pub = kKeyInf;
  int x_ops = 0, x_age = -1;  // ops of the pending exchange, tiles since it

  const int my_nt = split < n_tiles ? (n_tiles - split + S - 1) / S : 0;
  // Region order (knn_order.hip): the split's stream starts at its first tile
  // at or after the start of the query tile's region (the query tile's own
  // neighbourhood first, thresholds tight from the first tiles) and wraps.
  // The split's set of tiles is unchanged.
  int it0 = 0;
  if (qstart && my_nt > 1) {
    const int t0 = __builtin_amdgcn_readfirstlane(qstart[(int64_t)qt * (NW * QW)]) / (kTR * TPB);
    it0 = t0 > split ? (t0 - split + S - 1) / S : 0;
    if (it0 >= my_nt) it0 = my_nt - 1;
  }
  auto tile_at = [&](int i) {  // i < 2 my_nt
    int r = i + it0;
    if (r >= my_nt) r -= my_nt;
    return split + r * S;
  };
  constexpr bool PIPE = TEC && KNN_M4_PIPE && DP <= 192;  // DP 256: no registers to spare
  using AccT = std::conditional_t<I8A, i32x4, f32x4>;
  // PIPE: the previous sub-tile's accumulators; before the first sub-tile
  // they hold values no filter passes (int8: kI8Floor, fp16: +inf), so the
  // pipelined selection needs no first-sub-tile check
  AccT accp[2][QB];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      if constexpr (I8A) accp[rb][qb] = i32x4{kI8Floor, kI8Floor, kI8Floor, kI8Floor};
      else accp[rb][qb] = f32x4{KNN_INF_F, KNN_INF_F, KNN_INF_F, KNN_INF_F};
    }
  // METRIC 6: the previous sub-tile's 32x32 accumulators
  i32x16 accw;
  if constexpr (I8W) {
#pragma unroll
    for (int i = 0; i < 16; ++i) accw[i] = kI8Floor;
  }
  int rowp = 0;
  int rowp_s = 0;  // (KNN_SPRE_GLB) the pending sub-tile's first image row, wave-uniform
  SelCount selc;
  // Seed-free int8 accumulation (KNN_I8_SMAX): a holds q.k of a sub-tile,
  // smx the largest seed of its rows.  Every value's exact accumulator q.k +
  // seed is at most q.k + smx, so a wave none of whose lanes passes tn - smx
  // has no candidate; otherwise the exact seeds are added (sd(c): the seed
  // group c of the lane's rows -- from the sub-tile's LDS rows, or from
  // registers) and the exact selection runs.
  constexpr bool SMX = (I8W && KNN_I8_SMAX) || (I8 && KNN_I8_SMAX5);
  constexpr int NSG = I8W ? 4 : 2;  // i32x4 seed groups per lane and sub-tile
  // seed group c of the sub-tile whose LDS rows start at sb: metric 5 rows
  // 16c + 4 g16 (block c), metric 6 rows 8c + 4h
  auto seed_lds = [&](const float* sb, int c) {
    return __builtin_bit_cast(i32x4, *(const float4*)(sb + (I8W ? 8 * c + 4 * h : 16 * c + 4 * g16) * RSF + SEED));
  };
  int smxp = 0;  // PIPE: smx of the pending sub-tile
  // KNN_I8_PART: the partial-distance prune (metric 6, PIPE, >= 2 k-steps)
  constexpr bool PART = I8W && SMX && PIPE && KNN_I8_PART && i8_part_dims(DP) > 0;
  constexpr int KA = PART ? i8_part_dims(DP) / 32 : DP / 32;  // k-steps before the test
  constexpr int kI8Pruned = -(1 << 25);  // smx of a pruned sub-tile: tn - smx exceeds any q.k
  static_assert(!PART || !(KNN_SPRE_GLB), "the partial prune selects the pending sub-tile with spre");
  int hq = 0;  // ceil((|q_B|^2 + 1) / 2) of the lane's query (the dims after KA k-steps)
  if constexpr (PART) {
    int qb2 = 0;
#pragma unroll
    for (int ks = KA; ks < DP / 32; ++ks) {
      const i32x4 v = __builtin_bit_cast(i32x4, qf[ks]);
      qb2 = __builtin_amdgcn_sdot4(v.x, v.x, qb2, false);
      qb2 = __builtin_amdgcn_sdot4(v.y, v.y, qb2, false);
      qb2 = __builtin_amdgcn_sdot4(v.z, v.z, qb2, false);
      qb2 = __builtin_amdgcn_sdot4(v.w, v.w, qb2, false);
    }
    qb2 += __shfl_xor(qb2, 32, 64);  // lanes j and j + 32 hold the two halves of query j
    hq = (qb2 + 2) >> 1;
  }
  [[maybe_unused]] int cnt_it = 0;  // (KNN_COUNT_SEL: the staged tile being selected)
  auto sel5 = [&](const auto& a, int row0, int smx, auto&& sd) {  // a: i32x4 [2][QB]
   if constexpr (SMX) {
    bool pass = false;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      const i32x4 x = a[0][qb], y = a[1][qb];
      const int mx = max(max(max(x[0], x[1]), max(x[2], x[3])), max(max(y[0], y[1]), max(y[2], y[3])));
      pass = pass || mx > tn[qb] - smx;
    }
#if KNN_COUNT_SEL
    selc.bcalls++;
    selc.bpass += __builtin_amdgcn_ballot_w64(pass) != 0;
#endif
    if (__builtin_amdgcn_ballot_w64(pass)) {
      const i32x4 s0 = sd(0), s1 = sd(1);
#pragma unroll
      for (int qb = 0; qb < QB; ++qb)
        select_i8(a[0][qb] + s0, a[1][qb] + s1, row0, L[qb], I[qb], te[qb], tn[qb], selc);
    }
   }
  };
  auto sel6 = [&](const auto& a, int row0, int smx, auto&& sd) {  // a: i32x16
   if constexpr (SMX && I8W) {
#if KNN_MAX3T
    // (each max(max(x, y), z) is one v_max3_i32)
    auto m3 = [](int x, int y, int z) { return max(max(x, y), z); };
    const int mx = max(m3(m3(a[0], a[1], a[2]), m3(a[3], a[4], a[5]), m3(a[6], a[7], a[8])),
                       m3(m3(a[9], a[10], a[11]), m3(a[12], a[13], a[14]), a[15]));
#else
    const int mx = max(max(max(max(a[0], a[1]), max(a[2], a[3])), max(max(a[4], a[5]), max(a[6], a[7]))),
                       max(max(max(a[8], a[9]), max(a[10], a[11])), max(max(a[12], a[13]), max(a[14], a[15]))));
#endif
#if KNN_COUNT_SEL
    selc.bcalls++;
    selc.bpass += __builtin_amdgcn_ballot_w64(mx > tn[0] - smx) != 0;
    if (!(KNN_I8_PART)) {  // (with the partial prune these two count its tests)
      selc.bcold += cnt_it < 2;
      selc.bpcold += cnt_it < 2 && __builtin_amdgcn_ballot_w64(mx > tn[0] - smx) != 0;
    }
#endif
    if (__builtin_amdgcn_ballot_w64(mx > tn[0] - smx)) {
#if KNN_SLOWPRIO
      // the slow path at a raised issue priority: the other 7 waves of the
      // workgroup wait for it at the next barrier
      __builtin_amdgcn_s_setprio(KNN_SLOWPRIO);
#endif
      i32x16 b = a;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const i32x4 g = sd(c);
#pragma unroll
        for (int e = 0; e < 4; ++e) b[4 * c + e] = a[4 * c + e] + g[e];
      }
      if constexpr (W4) select_block_i8w4<R>(b, row0, L[0], I[0], L2, I2, tn[0], selc);
      else select_block_i8<R>(b, row0, L[0], I[0], tn[0], selc);
#if KNN_SLOWPRIO
      __builtin_amdgcn_s_setprio(0);
#endif
    }
   }
  };
  // SMX: the largest seeds of the staged tile's sub-tiles (wave-uniform);
  // spre: the exact seeds of the staged tile's last sub-tile, read with its
  // A fragments -- its selection runs after the next tile's first MFMAs,
  // when the buffer may be refilled (a pending sub-tile starts empty: raw
  // accumulators kI8Floor and smx 0 never pass)
  int smt[SMX ? TPB : 1];
  int smtA[PART ? TPB : 1];  // (KNN_I8_PART) the sub-tiles' largest partial seeds
  constexpr bool SPG = I8W && SMX && KNN_SPRE_GLB;  // last sub-tile's seeds by scalar loads
  // metric 6 (KNN_I8W_PF): the next sub-tile's A fragments in flight behind
  // the current sub-tile's MFMAs (its LDS latency no longer ahead of them)
  constexpr bool I8PF = I8W && KNN_I8W_PF;
  i32x4 afn[I8PF ? DP / 32 : 1];
  i32x4 spre[SMX && !SPG ? NSG : 1];
  // (SPG) seed group c of the lane's rows of the sub-tile at image row r0s
  // (wave-uniform): groups 2c and 2c + 1 by scalar loads, the lane's by h
  // (inline asm: a plain load of a uniform address becomes a vector load,
  // and its vmcnt wait would drain the staging pipeline's LDS-DMA pieces;
  // scalar loads are waited for with lgkmcnt)
  auto seed_glb = [&](int r0s, int c) {
    const float* p = Xr + ((int64_t)r0s + 8 * c) * RSF + SEED;
    const float* q = p + 4 * RSF;
    i32x4 a, b;
    asm volatile("s_load_dwordx4 %0, %2, 0x0\n\ts_load_dwordx4 %1, %3, 0x0\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b)
                 : "s"(p), "s"(q)
                 : "memory");
    return h ? b : a;
  };
#pragma unroll
  for (int c = 0; c < (SMX && !SPG ? NSG : 1); ++c) spre[c] = i32x4{0, 0, 0, 0};
  static_assert(!SMX || (TPB % 4 == 0 && kTR * 4 == 128), "sub-tile maxima are stored per 128-row group");

  // ---- staging: this wave's LDS-DMA pieces i = wv, wv+NW, ... of tile t ->
  // buffer b.  The last piece may read past the tile (and past the last row:
  // the HBM allocation carries 1 KiB of slack); it lands in the buffer tail.
  constexpr int G_HI = (NG + NW - 1) / NW, G_LO = NG / NW;
  constexpr int PD = NB - 1;  // prefetch distance in tiles
  static_assert(G_HI * (PD - 1) <= 63, "vmcnt range");
  // tiles an exchange's ops stay in flight (the slots are read after the
  // barrier of tile e + XPD); KNN_XPD_MIN = 2 lets them pass the barrier of
  // tile e + 1 even at PD = 1 (counted as younger than its pieces), but the
  // thresholds then arrive a tile later: int8 cfg2 candidate +2.5 %
  // (profiles/ab_log.md: r3e_ab_*), so the default waits at tile e + 1
#ifndef KNN_XPD_MIN
#define KNN_XPD_MIN 1
#endif
  constexpr int XPD = PD < KNN_XPD_MIN ? KNN_XPD_MIN : PD;
  // LDS byte address of the staging array (wave-uniform)
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds;
#define KNN_ISSUE(t_, b_)                                                              \
  do {                                                                                 \
    const char* g_ = (const char*)Xr + (int64_t)(t_) * TBY + lane * 16;                \
    const uint32_t l_ = lds_base + (uint32_t)((b_) * BUFF * 4);                        \
    for (int i_ = wv; i_ < NG; i_ += NW) glds16(g_ + i_ * 1024, l_ + (uint32_t)(i_ * 1024)); \
  } while (0)

  if (gthr && KNN_X_START && my_nt > 0) {
    // the slots as they stand now, fetched before tile 0's pieces: tile 0's
    // wait retires them (x_age reaches XPD there, no extra count) and its
    // selection filters with them
    if constexpr (GW == 128) {
      glds16((const char*)gthr + goff, gls_addr);
      glds16((const char*)gthr + goff + 16, gls_addr + 1024);
    } else {
      glds16((const char*)gthr + goff + 16 * h, gls_addr);
    }
    x_age = XPD - 1;
  }
#pragma unroll
  for (int p = 0; p < PD; ++p)
    if (my_nt > p) KNN_ISSUE(tile_at(p), p);

  const bool g_hi = wv < NG % NW || NG % NW == 0;
  int cur = 0, nxt = PD;  // buffer of tile it, buffer that tile it+PD goes to
  // (CTR) whether this wave has issued its pieces of tile it / it+1 (tile 0:
  // by the prologue)
  bool issued_cur = true, issued_next = false;
  bool signalled_cur = false, signalled_next = false;  // (CTR) counted ready
  int sig_at = TPB;  // (CTR) the sub-tile at which to count the next tile's pieces ready
  for (int it = 0; it < my_nt; ++it) {
    const int t = tile_at(it);
#if KNN_COUNT_SEL
    cnt_it = it;
#endif
    if constexpr (TEC) {
#pragma unroll
      for (int b = 0; b < NQL; ++b) thr[b] = lval(L[b][R - 1]);  // for the exchange below
      if constexpr (W4) thr[0] = lane_thr();
    }
    {
      // this wave's pieces of tile `it` have landed once at most the pieces
      // of the (up to PD-1) later tiles already issued remain outstanding;
      // the barrier then publishes all waves' pieces and retires every read
      // of buffer (it-1)%NB before it is refilled with tile it+PD.
      // wait + barrier in ONE asm statement with a memory clobber, so no LDS
      // read can be hoisted above the barrier (a bare s_barrier builtin does
      // not order memory) and no vmcnt(0) drains the in-flight tiles.
      const int ahead = min(PD - 1, my_nt - 1 - it);
      if (x_age >= 0) ++x_age;
      // (wave-uniform; readfirstlane keeps the dispatch below on scalar branches)
#if KNN_RFL
      const int extra = __builtin_amdgcn_readfirstlane((x_age >= 1 && x_age <= XPD - 1) ? x_ops : 0);
#else
      const int extra = (x_age >= 1 && x_age <= XPD - 1) ? x_ops : 0;
#endif
      if constexpr (CTR) {
        if (!issued_cur) {  // (this wave could not issue them during the previous tile)
          ctr_wait(&s_ctr[2 + cur], NW * (it / 2));
          KNN_ISSUE(tile_at(it), cur);
        }
        if (!signalled_cur) {
          // this wave's pieces of tile it landed (and every older op)
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (lane == 0) atomicAdd(&s_ctr[cur], 1);
        }
        ctr_wait(&s_ctr[cur], NW * (it / 2 + 1));  // every wave's pieces landed
        issued_next = signalled_next = false;
        sig_at = TPB;
      } else if (abl & 16) {
        // timing-only ablation: this wave's own waits, no workgroup barrier
        // (other waves' pieces may not have landed: results invalid)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (ahead >= 2 && PD >= 3) {
        if (g_hi) wait_barrier_x<2 * G_HI, XMAX>(extra); else wait_barrier_x<2 * G_LO, XMAX>(extra);
      } else if (ahead == 1) {
        if (g_hi) wait_barrier_x<G_HI, XMAX>(extra); else wait_barrier_x<G_LO, XMAX>(extra);
      } else {
        wait_barrier_x<0, XMAX>(extra);
      }
      __builtin_amdgcn_sched_barrier(0);
      // (abl bit 3: the same pieces, always of the split's first tile -- DMA
      // issue cost without the data stream; timing only)
      if (CTR) {
        // the next tile into the other buffer right away when every wave is
        // done with it (always for tile 1)
        if (it + 1 < my_nt &&
            __builtin_amdgcn_readfirstlane(*(volatile int*)&s_ctr[2 + nxt]) >= NW * ((it + 1) / 2)) {
          KNN_ISSUE(tile_at(it + 1), nxt);
          issued_next = true;
          sig_at = KNN_CTR_SIGD;
        }
      } else if (it + PD < my_nt && !(abl & 1)) {
        KNN_ISSUE((abl & 8) ? tile_at(0) : tile_at(it + PD), nxt);
      }
      if (gthr) {
        if (x_age == XPD) {
#pragma unroll
          for (int b = 0; b < NQL; ++b) {
            // slots 0-3 as fetched by lane qi, 4-7 by lane qi + 32
            const int qi = M16 ? 16 * b + c16 : j;
            const u32x4 g0 = gls[wv * GW + qi], g1 = gls[wv * GW + qi + GW / 2];
            tq[b] = key2f(max(max(max(g0.x, g0.y), max(g0.z, g0.w)),
                              max(max(g1.x, g1.y), max(g1.z, g1.w))));
          }
          x_age = -1;
        }
        if (x_age < 0 && exchange_tile(it) && it + XPD < my_nt) {
          // publish the best list threshold of the query's lanes in this wave
          // (one lane per query, only when it improved), fetch its 4 slots
          uint32_t pk;
          bool pub;
          if constexpr (M16) {
            // lane group g16 publishes for query block g16 (QB of the 4)
            float mb[QB];
            if (gk) {
#pragma unroll
              for (int b = 0; b < QB; ++b) {
                float u[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) u[e] = lval(L[b][e]);
                mb[b] = union_kth<4>(u, gk);
              }
            } else {
#pragma unroll
              for (int b = 0; b < QB; ++b) mb[b] = quad_min(thr[b]);
            }
            float mq = mb[QB - 1];
#pragma unroll
            for (int b = QB - 2; b >= 0; --b) mq = g16 == b ? mb[b] : mq;
            pk = f2key(mq);
            pub = g16 < QB && pk < last_pub;
          } else {
            float m;
            if (gk) {
              float u[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) u[e] = lval(L[0][e]);
              if constexpr (W4) {
                float u2[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) u2[e] = lval(L2[e]);
                merge_top4(u, u2);  // the lane's 4 best over both lists
              }
              m = union_kth<2>(u, gk);
            } else {
              const auto sw = __builtin_amdgcn_permlane32_swap(
                  __float_as_uint(thr[0]), __float_as_uint(thr[0]), false, false);
              m = fminf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
            }
            pk = f2key(m);
            pub = h == 0 && pk < last_pub;
          }
          x_ops = 1;
          if (__ballot(pub)) {
            if (pub)
              asm volatile("global_atomic_umin %0, %1, %2" ::"v"(goff), "v"(pk), "s"(gslot)
                           : "memory");
            x_ops = 2;
          }
          if (pub) last_pub = pk;
          if constexpr (GW == 128) {
            glds16((const char*)gthr + goff, gls_addr);
            glds16((const char*)gthr + goff + 16, gls_addr + 1024);
            ++x_ops;
          } else {
            glds16((const char*)gthr + goff + 16 * h, gls_addr);
          }
          x_age = 0;
        }
      }
    }
    if constexpr (TEC) {
      // the quad's shared filter, refreshed once per staged tile (a stale,
      // larger value only admits more insertions)
#pragma unroll
      for (int b = 0; b < NQL; ++b) {
        te[b] = __builtin_fminf(I8W ? pair_min(thr[b]) : quad_min(thr[b]), tq[b]);
        if constexpr (I8A) tn[b] = i8_neg_half(te[b]);
      }
    }
    if constexpr (SMX) {
#pragma unroll
      for (int u = 0; u < TPB / 4; ++u) {
        const int uu = rot ? (u + rot / 4) % (TPB / 4) : u;  // (KNN_STAGGER: rotated with the sub-tiles)
        const i32x4 v = __builtin_bit_cast(
            i32x4, *(const float4*)(lds + cur * BUFF + (128 * uu + kI8SmaxRow) * RSF + SEED));
#pragma unroll
        for (int e = 0; e < 4; ++e) smt[4 * u + e] = __builtin_amdgcn_readfirstlane(v[e]);
        if constexpr (PART) {
          const i32x4 va = __builtin_bit_cast(
              i32x4, *(const float4*)(lds + cur * BUFF + (128 * uu + kI8SmaxARow) * RSF + SEED));
#pragma unroll
          for (int e = 0; e < 4; ++e) smtA[4 * u + e] = __builtin_amdgcn_readfirstlane(va[e]);
        }
      }
    }
#pragma unroll
    for (int sub = 0; sub < TPB; ++sub) {
    // ps: the staged sub-tile processed at step sub (KNN_STAGGER rotates it)
    const int ps = (I8W && KNN_STAGGER) || (F16 && KNN_STAGGER4) ? (sub + rot) & (TPB - 1) : sub;
    const float* base = lds + cur * BUFF + ps * kTR * RSF;
    const float* base_prev = lds + cur * BUFF + ((I8W && KNN_STAGGER ? (sub - 1 + rot) & (TPB - 1) : sub - 1)) * kTR * RSF;

    if constexpr (I8W) {
      // int8 codes on v_mfma_i32_32x32x32_i8, exact: lane (j, h) holds query
      // j against rows (i&3) + 8(i>>2) + 4h; the accumulators start at the
      // rows' seeds -ceil(||k||^2 / 2) (the pad of row 4g carries rows 4g ..
      // 4g+3: groups 2c + h, c = i >> 2) and end at q.k - ceil(||k||^2 / 2)
      i32x16 acc = {};  // (SMX: the first MFMA's C operand is the inline zero)
      if constexpr (!SMX) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const i32x4 sd = __builtin_bit_cast(i32x4, *(const float4*)(base + (8 * c + 4 * h) * RSF + SEED));
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[4 * c + e] = sd[e];
        }
      }
      // A fragment of k-step ks: row j, dims 32ks + 16h .. +15 (the image of
      // this kernel is not chunk-swizzled: the 32x32 reads are conflict-free)
      i32x4 af[DP / 32];
      if (!I8PF || sub == 0) {
#pragma unroll
        for (int ks = 0; ks < DP / 32; ++ks)
          af[ks] = __builtin_bit_cast(i32x4, *(const float4*)(base + j * RSF + 8 * ks + 4 * h));
      } else {
#pragma unroll
        for (int ks = 0; ks < DP / 32; ++ks) af[ks] = afn[ks];
      }
      if (I8PF && sub + 1 < TPB) {
        // (KNN_I8W_PF) the next sub-tile's A fragments, read behind this one's MFMAs
        const float* bn =
            lds + cur * BUFF + ((KNN_STAGGER ? (sub + 1 + rot) & (TPB - 1) : sub + 1)) * kTR * RSF;
#pragma unroll
        for (int ks = 0; ks < DP / 32; ++ks)
          afn[ks] = __builtin_bit_cast(i32x4, *(const float4*)(bn + j * RSF + 8 * ks + 4 * h));
      }
      if constexpr (SMX && PIPE && !SPG) {
        if (sub == TPB - 1) {
#pragma unroll
          for (int c = 0; c < NSG; ++c) spre[c] = seed_lds(base, c);
        }
      }
#if KNN_I8_SCHED
      __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
      for (int ks = 0; ks < KA; ++ks)
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[ks], __builtin_bit_cast(i32x4, qf[ks]),
                                                    SMX && ks == 0 ? i32x16{} : acc, 0, 0, 0);
      if constexpr (PART) {
        // the pending sub-tile's selection first (it covers these MFMAs'
        // latency), then the partial test, then the last k-steps or none
        // (a pruned pending sub-tile skips its full test altogether: smxp is
        // wave-uniform, so this is a scalar branch)
        if (smxp != kI8Pruned) {
          if (sub > 0) sel6(accw, rowp, smxp, [&](int c) { return seed_lds(base_prev, c); });
          else sel6(accw, rowp, smxp, [&](int c) { return spre[c]; });
        }
        auto m3 = [](int x, int y, int z) { return max(max(x, y), z); };
        const int mxa = max(m3(m3(acc[0], acc[1], acc[2]), m3(acc[3], acc[4], acc[5]), m3(acc[6], acc[7], acc[8])),
                            m3(m3(acc[9], acc[10], acc[11]), m3(acc[12], acc[13], acc[14]), acc[15]));
#if KNN_COUNT_SEL
        // (partial tests and the waves passing them in the "cold" counters)
        selc.bcold++;
        selc.bpcold += __builtin_amdgcn_ballot_w64(mxa > tn[0] - hq - smtA[sub]) != 0;
#endif
        if (__builtin_amdgcn_ballot_w64(mxa > tn[0] - hq - smtA[sub])) {
#pragma unroll
          for (int ks = KA; ks < DP / 32; ++ks)
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[ks], __builtin_bit_cast(i32x4, qf[ks]), acc, 0, 0, 0);
          smxp = smt[sub];
        } else {
          smxp = kI8Pruned;
        }
      }
      if constexpr (CTR) {
        // (poll) the next tile's pieces as soon as every wave is done with
        // the tile before this one; SIGD sub-tiles later, counted ready
        if (!issued_next) {
          if (it + 1 < my_nt &&
              __builtin_amdgcn_readfirstlane(*(volatile int*)&s_ctr[2 + nxt]) >= NW * ((it + 1) / 2)) {
            KNN_ISSUE(tile_at(it + 1), nxt);
            issued_next = true;
            sig_at = sub + 1 + KNN_CTR_SIGD;
          }
        } else if (!signalled_next && sub >= sig_at) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (lane == 0) atomicAdd(&s_ctr[nxt], 1);
          signalled_next = true;
        }
      }
      const int row0 = (t * TPB + ps) * kTR + 4 * h;
      if constexpr (SMX) {
        // the pending sub-tile's selection after this one's MFMAs (seeds of
        // the previous staged tile's last sub-tile from spre)
        if (!(abl & 2)) {
          if constexpr (PART) {
            accw = acc;  // (selected, tested and completed above)
            rowp = row0;
          } else if constexpr (PIPE) {
            if (sub > 0) sel6(accw, rowp, smxp, [&](int c) { return seed_lds(base_prev, c); });
            else if constexpr (SPG) sel6(accw, rowp, smxp, [&](int c) { return seed_glb(rowp_s, c); });
            else sel6(accw, rowp, smxp, [&](int c) { return spre[c]; });
            accw = acc;
            rowp = row0;
            rowp_s = __builtin_amdgcn_readfirstlane((t * TPB + ps) * kTR);
            smxp = smt[sub];
          } else {
            sel6(acc, row0, smt[sub], [&](int c) { return seed_lds(base, c); });
          }
        } else if (acc[0] == 12345 && acc[15] == 12345) {
          thr[0] = (float)acc[7];  // keep the accumulators live
        }
      } else if constexpr (PIPE) {
        if (!(abl & 2)) {
          select_block_i8<R>(accw, rowp, L[0], I[0], tn[0], selc);
          accw = acc;
          rowp = row0;
        } else if (acc[0] == 12345 && acc[15] == 12345) {
          thr[0] = (float)acc[7];  // keep the accumulators live
        }
      } else if (!(abl & 2)) {
        select_block_i8<R>(acc, row0, L[0], I[0], tn[0], selc);
      } else if (acc[0] == 12345 && acc[15] == 12345) {
        thr[0] = (float)acc[7];
      }
    } else if constexpr (I8) {
      // int8 codes on v_mfma_i32_16x16x64_i8, exact: the accumulators start
      // at -ceil(||k||^2 / 2) (the pad of row 4g carries rows 4g .. 4g+3)
      // and end at q.k - ceil(||k||^2 / 2); one MFMA per 64 dims
      // every A fragment of the sub-tile (DP / 32 reads) is read before its
      // MFMAs, fenced (KNN_I8_SCHED): the registers are there (the query
      // image is half the fp16 one), and the compiler's own schedule would
      // wait on each read just before its two MFMAs
      i32x4 acc[2][QB] = {};
      if constexpr (!SMX) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const i32x4 sd = __builtin_bit_cast(i32x4, *(const float4*)(base + (rb * 16 + 4 * g16) * RSF + SEED));
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) acc[rb][qb] = sd;
        }
      }
      const int g16s = g16 ^ (xsw ? xh_swz(c16) : 0);
      i32x4 af[DP / 64][2];
#pragma unroll
      for (int ks = 0; ks < DP / 64; ++ks)
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
          af[ks][rb] = __builtin_bit_cast(
              i32x4, *(const float4*)(base + (rb * 16 + c16) * RSF + 16 * ks + 4 * g16s));
      if constexpr (SMX && PIPE) {
        if (sub == TPB - 1) {
#pragma unroll
          for (int c = 0; c < NSG; ++c) spre[c] = seed_lds(base, c);
        }
      }
#if KNN_I8_SCHED
      __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
      for (int ks = 0; ks < DP / 64; ++ks) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const i32x4 a = af[ks][rb];
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) {
            const i32x4 b = __builtin_bit_cast(i32x4, qf[qb * (DP / 64) + ks]);
            acc[rb][qb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                a, b, SMX && ks == 0 ? i32x4{} : acc[rb][qb], 0, 0, 0);
          }
        }
      }
      const int row0 = (t * TPB + sub) * kTR + 4 * g16;
      if constexpr (SMX) {
        // as metric 6
        if (!(abl & 2)) {
          if constexpr (PIPE) {
            if (sub > 0) sel5(accp, rowp, smxp, [&](int c) { return seed_lds(base - kTR * RSF, c); });
            else sel5(accp, rowp, smxp, [&](int c) { return spre[c]; });
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
              for (int qb = 0; qb < QB; ++qb) accp[rb][qb] = acc[rb][qb];
            rowp = row0;
            smxp = smt[sub];
          } else {
            sel5(acc, row0, smt[sub], [&](int c) { return seed_lds(base, c); });
          }
        } else if (acc[0][0][0] == 12345 && acc[1][1][3] == 12345) {
          thr[0] = (float)acc[0][1][2];  // keep the accumulators live
        }
      } else if constexpr (PIPE) {
        if (!(abl & 2)) {
#pragma unroll
          for (int qb = 0; qb < QB; ++qb)
            select_i8(accp[0][qb], accp[1][qb], rowp, L[qb], I[qb], te[qb], tn[qb], selc);
#pragma unroll
          for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) accp[rb][qb] = acc[rb][qb];
          rowp = row0;
        } else if (acc[0][0][0] == 12345 && acc[1][1][3] == 12345) {
          thr[0] = (float)acc[0][1][2];  // keep the accumulators live
        }
      } else if (!(abl & 2)) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
          select_i8(acc[0][qb], acc[1][qb], row0, L[qb], I[qb], te[qb], tn[qb], selc);
      } else if (acc[0][0][0] == 12345 && acc[1][1][3] == 12345) {
        thr[0] = (float)acc[0][1][2];  // keep the accumulators live
      }
    } else if constexpr (M16) {
      // bf16x3 on v_mfma_f32_16x16x32_bf16: 2 row blocks x 2 query blocks of
      // 16; lane l: A = row rb*16 + (l&15), B = query qb*16 + (l&15), k-group
      // l>>4; D = rows rb*16 + 4(l>>4) + i, column l&15
      f32x4 acc[2][QB];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        if constexpr (F16 && KNN_M4_SEED4) {
          // the pad of row 4g carries the seeds of rows 4g .. 4g+3
          const float4 sd = *(const float4*)(base + (rb * 16 + 4 * g16) * RSF + SEED);
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) acc[rb][qb] = f32x4{sd.x, sd.y, sd.z, sd.w};
        } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float sd = base[(rb * 16 + 4 * g16 + i) * RSF + SEED];
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) acc[rb][qb][i] = sd;
        }
        }
      }
      if constexpr (F16) {
        // fp16 x fp16 products are exact in fp32: one MFMA per 32 dims; the
        // lane's chunk 4ks + g16 sits at 4ks + (g16 ^ xh_swz(row)) (rows of a
        // sub-tile start at multiples of 32, so row & 15 = c16)
        const int g16s = g16 ^ (xsw ? xh_swz(c16) : 0);
#if KNN_M4_SCHED
        // the seed reads and the first KNN_M4_SCHED A fragments first, then
        // each fragment's two MFMAs followed by the next fragment's read
        __builtin_amdgcn_sched_group_barrier(0x100, KNN_M4_SCHED + 2, 0);
#endif
#pragma unroll
        for (int ks = 0; ks < DP / 32; ++ks) {
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            const float* ar = base + (rb * 16 + c16) * RSF + 16 * ks + 4 * g16s;
            const f16x8 a = __builtin_bit_cast(f16x8, *(const float4*)ar);
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) {
              const f16x8 b = __builtin_bit_cast(f16x8, qf[qb * (DP / 32) + ks]);
              acc[rb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[rb][qb], 0, 0, 0);
            }
#if KNN_M4_SCHED
            __builtin_amdgcn_sched_group_barrier(0x008, QB, 0);
            if (2 * ks + rb + KNN_M4_SCHED < DP / 16)
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#endif
          }
        }
      } else {
#pragma unroll
      for (int ks = 0; ks < DP / 32; ++ks) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const float* ar = base + (rb * 16 + c16) * RSF + 16 * ks + 4 * g16;
          const bf16x8 ah = __builtin_bit_cast(bf16x8, *(const float4*)ar);
          const bf16x8 al = __builtin_bit_cast(bf16x8, *(const float4*)(ar + DP / 2));
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) {
            const bf16x8 bh = __builtin_bit_cast(bf16x8, qf[(qb * 2 + 0) * (DP / 32) + ks]);
            const bf16x8 bl = __builtin_bit_cast(bf16x8, qf[(qb * 2 + 1) * (DP / 32) + ks]);
            acc[rb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc[rb][qb], 0, 0, 0);
            acc[rb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc[rb][qb], 0, 0, 0);
            acc[rb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc[rb][qb], 0, 0, 0);
          }
        }
      }
      }
      const int row0 = (t * TPB + ps) * kTR + 4 * g16;
      if constexpr (PIPE) {
        if (!(abl & 2)) {
#pragma unroll
          for (int qb = 0; qb < QB; ++qb)
            select_quad_te<R>(accp[0][qb], accp[1][qb], rowp, L[qb], I[qb], te[qb]);
#pragma unroll
          for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) accp[rb][qb] = acc[rb][qb];
          rowp = row0;
        } else if (acc[0][0][0] == 1234.5f && acc[1][1][3] == 1234.5f) {
          thr[0] = acc[0][1][2];  // keep the accumulators live
        }
      } else if (!(abl & 2)) {
        if constexpr (TEC) {
#pragma unroll
          for (int qb = 0; qb < QB; ++qb)
            select_quad_te<R>(acc[0][qb], acc[1][qb], row0, L[qb], I[qb], te[qb]);
        } else {
#pragma unroll
          for (int qb = 0; qb < QB; ++qb)
            select_quad<R>(acc[0][qb], acc[1][qb], row0, L[qb], I[qb], thr[qb], tq[qb]);
        }
      } else if (acc[0][0][0] == 1234.5f && acc[1][1][3] == 1234.5f) {
        thr[0] = acc[0][1][2];  // keep the accumulators live
      }
    } else {
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = base[((i & 3) + 8 * (i >> 2) + 4 * h) * RSF + SEED];
    if constexpr (METRIC == 0) {
      const float* arow = base + j * RSF + 4 * h;
#pragma unroll
      for (int c = 0; c < DP / 8; ++c) {
        const float4 a = *(const float4*)(arow + 8 * c);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, qf[c].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, qf[c].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, qf[c].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, qf[c].w, acc, 0, 0, 0);
      }
    } else if constexpr (METRIC == 2) {
      // bf16x3 split product on v_mfma_f32_32x32x16_bf16:
      //   q.x ~= qh.xh + ql.xh + qh.xl   (train row payload = [xh | xl])
      // i.e. one bf16 GEMM with K = 3*DP; ~2^-16 relative product error,
      // 16x the f32 MFMA rate per instruction -> 5.3x per fp32-equivalent flop.
      const float* arow = base + j * RSF + 4 * h;
#pragma unroll
      for (int tt = 0; tt < DP / 16; ++tt) {
        const bf16x8 ah = __builtin_bit_cast(bf16x8, *(const float4*)(arow + 8 * tt));
        const bf16x8 al = __builtin_bit_cast(bf16x8, *(const float4*)(arow + DP / 2 + 8 * tt));
        const bf16x8 bh = __builtin_bit_cast(bf16x8, qf[tt]);
        const bf16x8 bl = __builtin_bit_cast(bf16x8, qf[DP / 16 + tt]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
      }
    } else {
      // L1 on the VALU: lane's query against its 16 rows, dims in chunks of 4.
#pragma unroll 2
      for (int c = 0; c < DP / 4; ++c) {
        const float4 qv = *(const float4*)(qrow + 4 * c);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int r = (i & 3) + 8 * (i >> 2) + 4 * h;
          const float4 xv = *(const float4*)(base + r * RSF + 4 * c);
          float a = acc[i];
          a = a + __builtin_fabsf(qv.x - xv.x);
          a = a + __builtin_fabsf(qv.y - xv.y);
          a = a + __builtin_fabsf(qv.z - xv.z);
          a = a + __builtin_fabsf(qv.w - xv.w);
          acc[i] = a;
        }
      }
    }

    if (!(abl & 2)) select_block<R>(acc, (t * TPB + sub) * kTR, h, L[0], I[0], thr[0], tq[0]);
    else if (acc[0] == 1234.5f && acc[15] == 1234.5f) thr[0] = acc[7];  // keep acc live
    }
    }
    if constexpr (CTR) {
      // every read of this tile's buffer done (the last sub-tile's seeds are
      // in spre), then counted: its refill may be issued
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) atomicAdd(&s_ctr[2 + cur], 1);
      issued_cur = issued_next;
      signalled_cur = signalled_next;
    }
    if (++cur == NB) cur = 0;
    if (++nxt == NB) nxt = 0;

  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (SMX && PIPE) {
    // the last tile's last sub-tile, seeds from spre
    if (!(abl & 2)) {
      if constexpr (SPG) sel6(accw, rowp, smxp, [&](int c) { return seed_glb(rowp_s, c); });
      else if constexpr (I8W) sel6(accw, rowp, smxp, [&](int c) { return spre[c]; });
      else sel5(accp, rowp, smxp, [&](int c) { return spre[c]; });
    }
  } else if constexpr (PIPE && I8W) {
    if (!(abl & 2)) select_block_i8<R>(accw, rowp, L[0], I[0], tn[0], selc);
  } else if constexpr (PIPE) {
    if (!(abl & 2)) {
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        if constexpr (I8)
          select_i8(accp[0][qb], accp[1][qb], rowp, L[qb], I[qb], te[qb], tn[qb], selc);
        else
          select_quad_te<R>(accp[0][qb], accp[1][qb], rowp, L[qb], I[qb], te[qb]);
      }
    }
  }

#if KNN_COUNT_SEL
  if constexpr (I8A) {
    atomicAdd(&knn_sel_cnt[0], (unsigned long long)selc.calls);
    atomicAdd(&knn_sel_cnt[1], (unsigned long long)selc.lane_pass);
    if (lane == 0) atomicAdd(&knn_sel_cnt[2], (unsigned long long)selc.wave_pass);
    atomicAdd(&knn_sel_cnt[3], (unsigned long long)selc.inserts);
    if (lane == 0) atomicAdd(&knn_sel_cnt[4], (unsigned long long)selc.bcalls);
    if (lane == 0) atomicAdd(&knn_sel_cnt[5], (unsigned long long)selc.bpass);
    if (lane == 0) atomicAdd(&knn_sel_cnt[6], (unsigned long long)selc.bcold);
    if (lane == 0) atomicAdd(&knn_sel_cnt[7], (unsigned long long)selc.bpcold);
  }
#endif
  if constexpr (M16) {
    // 4 lists per query per split (lane groups l>>4): [query][4S][R]
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      const int64_t o = ((qb0 + 16 * qb) * (4 * S) + split * 4 + g16) * R;
#pragma unroll
      for (int t = 0; t < R; t += 4) {
        *(float4*)(out_v + o + t) = make_float4(lval(L[qb][t]), lval(L[qb][t + 1]),
                                                lval(L[qb][t + 2]), lval(L[qb][t + 3]));
        *(int4*)(out_i + o + t) = make_int4(I[qb][t], I[qb][t + 1], I[qb][t + 2], I[qb][t + 3]);
      }
    }
  } else if constexpr (W4) {
    // 4 lists per query per split, [query][4S][R]: list 2h + half
#pragma unroll
    for (int li = 0; li < 2; ++li) {
      const int64_t o = (qg * (4 * S) + split * 4 + 2 * h + li) * R;
      const int* Ls = li ? L2 : L[0];
      const int* Is = li ? I2 : I[0];
      *(float4*)(out_v + o) = make_float4(lval(Ls[0]), lval(Ls[1]), lval(Ls[2]), lval(Ls[3]));
      *(int4*)(out_i + o) = make_int4(Is[0], Is[1], Is[2], Is[3]);
    }
  } else if constexpr (ILIST) {
    float Lf[R];
#pragma unroll
    for (int t = 0; t < R; ++t) Lf[t] = lval(L[0][t]);
    write_lists<R>(out_v, out_i, qg, S, split, h, Lf, I[0]);
  } else {
    write_lists<R>(out_v, out_i, qg, S, split, h, L[0], I[0]);
  }
#undef KNN_ISSUE
}

// Compile-time dispatch over (R, METRIC): R in {4, 8, 16}; METRIC 0..4
// (2 = bf16x3 with DP % 16 == 0; 3 = bf16x3 and 4 = fp16 on the 16x16x32
// layout, DP % 32 == 0, R = 4, 8 waves).
template <class F>
static void with_R(int R, F f) {
  if (R == 4) f(std::integral_constant<int, 4>{});
  else if (R == 8) f(std::integral_constant<int, 8>{});
  else f(std::integral_constant<int, 16>{});
}
template <class F>
static void with_M(int M, F f) {
  if (M == 0) f(std::integral_constant<int, 0>{});
  else if (M == 1) f(std::integral_constant<int, 1>{});
  else if (M == 2) f(std::integral_constant<int, 2>{});
  else if (M == 3) f(std::integral_constant<int, 3>{});
  else if (M == 4) f(std::integral_constant<int, 4>{});
  else if (M == 5) f(std::integral_constant<int, 5>{});
  else f(std::integral_constant<int, 6>{});
}

template <int DP, int R, int METRIC, int NW>
static void launch_res(const CandLaunch& c, hipStream_t s) {
  const int nt = (int)(c.n_pad / (kTR * res_tpb<METRIC>()));
  if (c.ev_start)
    hipExtLaunchKernelGGL((cand_kernel<DP, R, METRIC, NW>), dim3((unsigned)(c.n_qt * c.S)),
                          dim3(NW * 64), 0, s, c.ev_start, c.ev_stop, 0, c.X32, c.Q32, nt, c.S,
                          c.n_qt, c.out_v, c.out_i, c.ablate, c.gthr, c.gk, c.xsw, c.qstart,
                          c.gmask, c.qblk);
  else
    hipLaunchKernelGGL((cand_kernel<DP, R, METRIC, NW>), dim3((unsigned)(c.n_qt * c.S)),
                       dim3(NW * 64), 0, s, c.X32, c.Q32, nt, c.S, c.n_qt,
                       c.out_v, c.out_i, c.ablate, c.gthr, c.gk, c.xsw, c.qstart, c.gmask, c.qblk);
}

// Instantiated variants: R in {4, 8, 16}; METRIC 0/2 with NW in {4, 8};
// METRIC 4 also with NW = 16 (512 queries share each staged tile); METRIC 5
// (int8) with R = 4 (8 on request), NW = 8 or 4 at DP % 64 == 0;
// METRIC 1 (L1, not perf-graded) with NW = 4 and R in {8, 16}; METRIC 2
// needs DP % 16 == 0.
// Metric 6 at R = 4 writes 4 lists per query per split (W4 above) only with
// KNN_I8W_Q4, KNN_I8_ILIST and KNN_I8_SMAX all on; the host's merge then
// reads that quad layout (knn_api.cpp: w4).  A build with any of them off
// has no R = 4 metric-6 kernel, so the host's launch is refused ("no
// candidate kernel for this geometry") instead of the merge reading 2 lists
// per split as 4 (stale entries).
constexpr bool kI8WQuad = KNN_I8W_Q4 && KNN_I8_ILIST && KNN_I8_SMAX;

template <int DP, int R, int M, int NW>
constexpr bool res_variant() {
  return (M != 6 || R != 4 || kI8WQuad) && (M != 2 || DP % 16 == 0) && (M != 1 || (NW == 4 && R != 4)) &&
         (M < 3 || (DP % 32 == 0 && (R == 4 || (M >= 5 && R == 8)) && (NW == 8 || M >= 4))) &&
         (NW != 16 || M == 4 || (M == 6 && KNN_I8W_NW16 && R == 4 && DP <= 128)) &&
         (M != 5 || (DP % 64 == 0 && (NW == 8 || NW == 4))) &&
         (M != 6 || ((NW == 8 || (NW == 16 && KNN_I8W_NW16)) && (R == 4 || R == 8)));
}

template <int DP>
static int blocks_per_cu_res(int R, int metric, int nw) {
  int out = 1;
  with_R(R, [&](auto Rc) {
    with_M(metric, [&](auto Mc) {
      if (nw == 16) {
        if constexpr (res_variant<DP, Rc.value, Mc.value, 16>())
          out = occupancy_of(cand_kernel<DP, Rc.value, Mc.value, 16>, 1024);
      } else if (nw == 8) {
        if constexpr (res_variant<DP, Rc.value, Mc.value, 8>())
          out = occupancy_of(cand_kernel<DP, Rc.value, Mc.value, 8>, 512);
      } else {
        if constexpr (res_variant<DP, Rc.value, Mc.value, 4>())
          out = occupancy_of(cand_kernel<DP, Rc.value, Mc.value, 4>, 256);
      }
    });
  });
  return out;
}

template <int DP>
static bool launch_res_dp(const CandLaunch& c, hipStream_t s) {
  bool launched = false;  // false: no instantiated variant (caller reports it)
  with_R(c.R, [&](auto Rc) {
    with_M(c.metric, [&](auto Mc) {
      // the host's query tile must be this kernel's (nw x queries per
      // wave): a mismatch would index queries past the operand buffers
      if (c.qpb != c.nw * res_qpw<Mc.value>()) return;
      if (c.nw == 16) {
        if constexpr (res_variant<DP, Rc.value, Mc.value, 16>())
          launch_res<DP, Rc.value, Mc.value, 16>(c, s), launched = true;
      } else if (c.nw == 8) {
        if constexpr (res_variant<DP, Rc.value, Mc.value, 8>())
          launch_res<DP, Rc.value, Mc.value, 8>(c, s), launched = true;
      } else {
        if constexpr (res_variant<DP, Rc.value, Mc.value, 4>())
          launch_res<DP, Rc.value, Mc.value, 4>(c, s), launched = true;
      }
    });
  });
  return launched;
}

#if KNN_GROUP == 0
#define KNN_GROUP_DPS(X) X(8) X(16) X(24) X(32) X(48) X(64)
#elif KNN_GROUP == 1
#define KNN_GROUP_DPS(X) X(96) X(128)
#elif KNN_GROUP == 2
#define KNN_GROUP_DPS(X) X(160) X(192)
#elif KNN_GROUP == 3
#define KNN_GROUP_DPS(X) X(256)
#else
#error "KNN_GROUP must be 0..3"
#endif

#define KNN_DEF(v)                                                                 \
  bool launch_res_##v(const CandLaunch& c, hipStream_t s) { return launch_res_dp<v>(c, s); } \
  int blocks_res_##v(int R, int metric, int nw) { return blocks_per_cu_res<v>(R, metric, nw); } \
  int qpw_res_##v(int metric) { return metric == 5 ? res_qpw<5>() : res_qpw<0>(); } \
  int trows_res_##v(int metric) {                                                        \
    return kTR * (metric >= 5 ? res_tpb<5>() : metric == 4 ? res_tpb<4>() : res_tpb<0>()); \
  }
KNN_GROUP_DPS(KNN_DEF)
#undef KNN_DEF

#if KNN_GROUP == 1
// Experiment hook (no C-ABI entry; tools call it by its symbol): the int8
// selection counts of a KNN_COUNT_SEL build (DP 96 / 128), zeros otherwise.
int res_sel_counters(unsigned long long* out, int reset) {
#if KNN_COUNT_SEL
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(knn_sel_cnt), 8 * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  if (reset) {
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(knn_sel_cnt), z, sizeof z) != hipSuccess) return -1;
  }
#else
  (void)reset;
  for (int i = 0; i < 8; ++i) out[i] = 0;
#endif
  return 0;
}
#endif

}  // namespace knnk
