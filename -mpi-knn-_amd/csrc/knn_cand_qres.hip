// knn_cand_qres.hip -- the query-resident fp16 candidate kernel for d > 256
// (cfg5: d = 960, k = 100; cpp:33-50 per query against every train row).
//
// The S3 kernel (knn_cand.hip) streams both operands through LDS in 32-dim
// chunks, so every query chunk is re-read for every 256-row train tile
// (32.7 GB of L2 misses per cfg5 launch, profiles/r5f_traffic_cfg5.json).
// Here each wave keeps its 32 queries' fp16 operands for the whole kernel in
// AGPRs (32 queries x DP dims: DP / 4 registers per lane, 240 at d = 960;
// MFMA srcB reads AGPRs directly), one wave per SIMD, 4 waves = 128 queries
// per workgroup and one workgroup per CU (two 60-KB LDS buffers).  Only the
// train rows stream: 32-row sub-tiles of all DP dims, straight from the S3
// tile-chunk image (XT16: a chunk of 32 rows is 2 KB contiguous, two LDS-DMA
// pieces; its swizzle keeps the 16x16 fragment reads conflict-free) plus
// their 32 seeds, one barrier per sub-tile.  The workgroup's XCD neighbours
// (xcd_remap: consecutive query tiles of one split) share the row stream in
// L2, and the queries are read once.
//
// Measured (profiles/ab_log.md r6v-r6w): SLOWER than S3 at cfg5 -- 24.0 ms
// against 19.9-20.1 ms in the same process, although its bare loop (no
// selection) runs 16.6 ms.  With one wave per SIMD nothing hides the
// selection's VALU work (k = 100: 4 lists of 8 per query per split), which
// S3's second wave per SIMD overlaps with MFMAs.  Opt-in (tuning "qres" 1;
// AUTO off, kQresAuto in knn_api.cpp); parity-tested like every path.
//
// Outputs are the S3 q16 kernel's exactly: the 16x16 layout's quad lists of
// R = 8 per query per split (split s = 256-row tiles s, s + S, ...: the same
// row sets, so the merge, the certification and the targeted rescan are
// unchanged), the per-query global threshold exchange (gthr, gk) included.
#include "knn_device.h"

#include <hip/hip_ext.h>

namespace knnk {

// A-fragment reads software-pipelined in chunks of KC k-steps (one wave per
// SIMD: no other wave hides their latency).  Measured on the bare loop
// (tools/exp/res960.hip, profiles/ab_log.md r6v): KC 2 / 3 / 5 -> 16.3 / 16.6 /
// 16.9 ms at cfg5 shape
// Selection (experiments; KNN_QRES_SEL): 1 after each sub-tile's MFMAs; 2
// pipelined -- the previous sub-tile's no-candidate test (min tree, filter)
// issued among this sub-tile's first MFMAs, its insertions (if any lane
// passes) after them: with one wave per SIMD nothing else hides the
// selection's VALU work; 0 none (timing only, results invalid)
#ifndef KNN_QRES_SEL
#define KNN_QRES_SEL 1
#endif
// workgroup order: 2 (S % 8 == 0; else 1) XCD x runs splits x, x + 8, x +
// 16, ... -- split-major over the query tiles, so its concurrent workgroups
// share one split's row stream in its L2, and every query tile's first
// workgroups cover all 8 slot groups of the global threshold (split % 8) at
// once: its threshold is finite after their first exchanges, and later
// workgroups start with it (KNN_X_START); 1 xcd_remap (an XCD's range of
// consecutive logical ids: the first rounds hold only splits = 0 or 4 mod 8,
// no query's threshold is finite until every group has run); 0 dispatch order
#ifndef KNN_QRES_REMAP
#define KNN_QRES_REMAP 2
#endif

template <int NCH>
constexpr int qres_kc() {
  return NCH % 3 == 0 ? 3 : NCH % 2 == 0 ? 2 : NCH % 5 == 0 ? 5 : 1;
}

template <int NCH>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
cand_qres_kernel(const unsigned short* XT, const float* XS, const unsigned short* QT, int n_tiles,
                 int S, int n_qt, float* __restrict__ out_v, int* __restrict__ out_i, uint32_t* gthr,
                 int gk) {
  constexpr int R = 8;
  constexpr int SUBB = NCH * 2048 + 1024;  // LDS buffer: [chunk][32 rows][64 B] | 32 seeds (+pad)
  constexpr int NP = 2 * NCH + 1;          // LDS-DMA pieces per sub-tile (the last: seeds)
  constexpr int KC = qres_kc<NCH>(), NC = NCH / KC;
  static_assert(NC * KC == NCH, "chunking");
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * SUBB];
  __shared__ __attribute__((aligned(16))) u32x4 gls[4 * 64];

  int split, qt;
  if (KNN_QRES_REMAP == 2 && (S & 7) == 0) {
    const int r = blockIdx.x >> 3, j = r / n_qt;  // (gridDim.x = n_qt S, a multiple of 8)
    qt = r - j * n_qt;
    split = 8 * j + (blockIdx.x & 7);
  } else {
    const int bid = KNN_QRES_REMAP ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    split = bid / n_qt;
    qt = bid - split * n_qt;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, g16 = lane >> 4, h = lane >> 5;
  // fragment offset of row (or query) c16 of a 16-block, slot g16 (the
  // image's swizzle depends on (row >> 2) & 3 = c16 >> 2 here)
  const int off_16 = c16 * 64 + ((g16 ^ s3h_swz(c16 >> 2)) << 4);

  // this wave's queries: rows 16 qb + c16 of its 32 in the S3 query image
  // (256-query tiles: this 128-query tile is half qt & 1 of tile qt >> 1)
  const int64_t qbase = ((int64_t)(qt >> 1) * NCH) * kS3R * 64 + (int64_t)((qt & 1) * 128 + wv * 32) * 64;
  float4 qf[2 * NCH];  // [qb][chunk], in AGPRs
#pragma unroll
  for (int c0 = 0; c0 < 2 * NCH; c0 += 4) {
    const char* p[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + u < 2 * NCH ? c0 + u : c0;
      const int qb = c / NCH, ks = c % NCH;
      p[u] = (const char*)QT + qbase + (int64_t)ks * kS3R * 64 + qb * 16 * 64 + off_16;
    }
    float4 v0, v1, v2, v3;
    // loads and their wait in one statement, straight into AGPRs: the
    // compiler's own waits for these would sit inside the tile loop (and
    // drain the LDS-DMA pieces in flight)
    asm volatile(
        "global_load_dwordx4 %0, %4, off\n\t"
        "global_load_dwordx4 %1, %5, off\n\t"
        "global_load_dwordx4 %2, %6, off\n\t"
        "global_load_dwordx4 %3, %7, off\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&a"(v0), "=&a"(v1), "=&a"(v2), "=&a"(v3)
        : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3])
        : "memory");
    qf[c0] = v0;
    if (c0 + 1 < 2 * NCH) qf[c0 + 1] = v1;
    if (c0 + 2 < 2 * NCH) qf[c0 + 2] = v2;
    if (c0 + 3 < 2 * NCH) qf[c0 + 3] = v3;
  }

  float L[2][R];
  int I[2][R];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int t = 0; t < R; ++t) { L[b][t] = KNN_INF_F; I[b][t] = -1; }

  // global per-query threshold (as cand_s3_kernel's q16 form): at the first
  // sub-tile of tiles 0, 1, 2, 4, 8, 12, ... each workgroup publishes, per
  // query, the gk-th smallest of the union of its 4 lists into slot split % 8
  // and fetches the 8 slots by LDS-DMA; every barrier here waits for all
  // vector memory ops, so the slots are read after the next one
  const bool gx = gthr && gk > 0;
  const int64_t q_lane = (int64_t)qt * 128 + wv * 32 + (lane & 31);
  const uint32_t goff = (uint32_t)(q_lane * (4 * kGthrSlots));
  const uint32_t gls_addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) u32x4*)gls + wv * 1024;
  float tq[2] = {KNN_INF_F, KNN_INF_F};
  uint32_t last_pub = kKeyInf;
  bool x_pending = false;

  const int my_nt = split < n_tiles ? (n_tiles - split + S - 1) / S : 0;
  const int total = my_nt * (kS3R / 32);  // 32-row sub-tiles
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds;
  // this wave's pieces of sub-tile st into buffer b: pieces wv, wv + 4, ...
  // (piece 2c + e = rows 16e .. 16e + 15 of chunk c; piece 2 NCH = the seeds,
  // 1 KB from the sub-tile's first seed: the XS16 allocation has the slack)
  auto issue = [&](int st, int b) {
    const int64_t T = split + (int64_t)(st >> 3) * S;
    const int u = st & 7;
    const uint32_t l = lds_base + (uint32_t)(b * SUBB) + lane * 16;
    for (int pc = wv; pc < NP; pc += 4) {
      if (pc < 2 * NCH) {
        const int c = pc >> 1, e = pc & 1;
        glds16((const char*)XT + ((T * NCH + c) * kS3R + 32 * u + 16 * e) * 64 + lane * 16,
               l + (uint32_t)((c * 32 + 16 * e) * 64));
      } else {
        glds16((const char*)(XS + T * kS3R + 32 * u) + lane * 16, l + (uint32_t)(NCH * 2048));
      }
    }
  };
  if (gx && KNN_X_START && total > 0) {
    glds16((const char*)gthr + goff + 16 * h, gls_addr);
    x_pending = true;
  }
  if (total > 0) issue(0, 0);
  // (KNN_QRES_SEL 2) the pending sub-tile: its accumulators (+inf before the
  // first: no value passes), first row, filters and test result
  f32x4 accp[2][2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) accp[rb][qb] = f32x4{KNN_INF_F, KNN_INF_F, KNN_INF_F, KNN_INF_F};
  int row0p = 0;
  float tfp[2] = {KNN_INF_F, KNN_INF_F};
  bool passp = false;

  for (int st = 0; st < total; ++st) {
    const int cb = st & 1;
    // every wave's pieces of sub-tile st (and any exchange ops) have landed;
    // every read of the other buffer (sub-tile st - 1) has retired
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (st + 1 < total) issue(st + 1, cb ^ 1);
    const int ti = st >> 3, u = st & 7;
    if (gx) {
      if (x_pending) {
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          const u32x4 g0 = gls[wv * 64 + 16 * qb + c16], g1 = gls[wv * 64 + 16 * qb + c16 + 32];
          tq[qb] = key2f(max(max(max(g0.x, g0.y), max(g0.z, g0.w)), max(max(g1.x, g1.y), max(g1.z, g1.w))));
        }
        x_pending = false;
      }
      if (u == 0 && st + 1 < total && (ti < 4 ? ti != 3 : (ti & 3) == 0)) {
        const float m0 = quad_union_kth16(L[0], gk), m1 = quad_union_kth16(L[1], gk);
        const uint32_t pk = f2key(g16 == 0 ? m0 : m1);
        const bool pub = g16 < 2 && pk < last_pub;
        if (__ballot(pub)) {
          if (pub)
            asm volatile("global_atomic_umin %0, %1, %2" ::"v"(goff), "v"(pk), "s"(gthr + (split & 7))
                         : "memory");
        }
        if (pub) last_pub = pk;
        glds16((const char*)gthr + goff + 16 * h, gls_addr);
        x_pending = true;
      }
    }

    const unsigned char* buf = lds + cb * SUBB;
    // accumulators start at the rows' seeds fl32(||x||^2) (+inf on pad rows):
    // rows 16 rb + 4 g16 + i
    f32x4 acc[2][2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const float4 s4 = *(const float4*)(buf + NCH * 2048 + (16 * rb + 4 * g16) * 4);
      acc[rb][0] = acc[rb][1] = f32x4{s4.x, s4.y, s4.z, s4.w};
    }
    float4 af[2][KC][2];
    auto rd = [&](int c, int bsel) {
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
          af[bsel][k][rb] = *(const float4*)(buf + (c * KC + k) * 2048 + rb * 1024 + off_16);
    };
    rd(0, 0);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (c + 1 < NC) rd(c + 1, (c + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const int ks = c * KC + k;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const f16x8 a = __builtin_bit_cast(f16x8, af[c & 1][k][rb]);
#pragma unroll
          for (int qb = 0; qb < 2; ++qb)
            acc[rb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, __builtin_bit_cast(f16x8, qf[qb * NCH + ks]),
                                                                acc[rb][qb], 0, 0, 0);
        }
      }
      if (KNN_QRES_SEL == 2 && c == 0) {
        // the pending sub-tile's no-candidate test, among these MFMAs
        passp = false;
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          tfp[qb] = __builtin_fminf(quad_min(L[qb][R - 1]), tq[qb]);
          const f32x4 x = accp[0][qb], y = accp[1][qb];
          const float mn = __builtin_fminf(__builtin_fminf(__builtin_fminf(x[0], x[1]), __builtin_fminf(x[2], x[3])),
                                           __builtin_fminf(__builtin_fminf(y[0], y[1]), __builtin_fminf(y[2], y[3])));
          passp = passp || mn < __builtin_fminf(tfp[qb], L[qb][R - 1]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // the quad's shared filter (min over its 4 lists' R-th entries and the
    // global threshold) and this lane's lists; rows 32 u + 16 rb + 4 g16 + i
    // of tile T
    const int row0 = (int)((split + (int64_t)ti * S) * kS3R) + 32 * u + 4 * g16;
    if constexpr (KNN_QRES_SEL == 2) {
      if (__builtin_amdgcn_ballot_w64(passp)) {
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) select_quad_f<R>(accp[0][qb], accp[1][qb], row0p, L[qb], I[qb], tfp[qb]);
      }
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) accp[rb][qb] = acc[rb][qb];
      row0p = row0;
    } else if constexpr (KNN_QRES_SEL == 1) {
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const float tf = __builtin_fminf(quad_min(L[qb][R - 1]), tq[qb]);
        select_quad_f<R>(acc[0][qb], acc[1][qb], row0, L[qb], I[qb], tf);
      }
    } else if (acc[0][0][0] == 1234.5f && acc[1][1][3] == 1234.5f) {
      L[0][0] = acc[0][1][2];  // (timing only: keep the accumulators live)
    }
  }
  if constexpr (KNN_QRES_SEL == 2) {
    // the last sub-tile's selection
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const float tf = __builtin_fminf(quad_min(L[qb][R - 1]), tq[qb]);
      select_quad_f<R>(accp[0][qb], accp[1][qb], row0p, L[qb], I[qb], tf);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // [query][4S][R]: the S3 q16 layout
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int64_t q = (int64_t)qt * 128 + wv * 32 + 16 * qb + c16;
    const int64_t o = (q * (4 * S) + split * 4 + g16) * R;
#pragma unroll
    for (int e = 0; e < R; e += 4) {
      *(float4*)(out_v + o + e) = make_float4(L[qb][e], L[qb][e + 1], L[qb][e + 2], L[qb][e + 3]);
      *(int4*)(out_i + o + e) = make_int4(I[qb][e], I[qb][e + 1], I[qb][e + 2], I[qb][e + 3]);
    }
  }
}

// Padded dimensions with an instantiation (DP = 32 NCH); other d > 256 run S3
// (d = 288 .. 960 in steps that cover the usual widths: 300 -> 10, 512 ->
// 16, 784 (MNIST) -> 25, 960 (cfg5) -> 30)
#define KNN_QRES_LIST(X) X(9) X(10) X(12) X(14) X(16) X(18) X(20) X(24) X(25) X(28) X(30)

bool qres_supported(int DP) {
  if (DP % 32) return false;
#define KNN_CASE(v) if (DP / 32 == v) return true;
  KNN_QRES_LIST(KNN_CASE)
#undef KNN_CASE
  return false;
}

// n_qt: 256-query tiles of the S3 geometry (the kernel runs 2 n_qt tiles of
// 128); n_pad: train rows padded to 256.  false: no instantiation for DP.
bool launch_cand_qres(const unsigned short* XT, const float* XS, const unsigned short* QT, int DP,
                      int64_t n_pad, int S, int n_qt, float* out_v, int* out_i, uint32_t* gthr, int gk,
                      hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
  const int n_tiles = (int)(n_pad / kS3R);
  const dim3 g((unsigned)(2 * n_qt * S)), b(256);
#define KNN_CASE(v)                                                                                  \
  if (DP / 32 == v && DP % 32 == 0) {                                                                \
    hipExtLaunchKernelGGL((cand_qres_kernel<v>), g, b, 0, s, ev_start, ev_stop, 0, XT, XS, QT, n_tiles, \
                          S, 2 * n_qt, out_v, out_i, gthr, gk);                                       \
    return true;                                                                                     \
  }
  KNN_QRES_LIST(KNN_CASE)
#undef KNN_CASE
  return false;
}

}  // namespace knnk
