// knn_order.hip -- the order in which the candidate pass streams the train
// rows ("regions"), and the matching order of the queries.
//
// The candidate kernels filter each row against per-query thresholds that
// tighten as the stream goes on; the rows a split sees before its thresholds
// are tight are the ones that pay list insertions and the divergent slow
// path of the selection.  Nothing in the result depends on
// the order (the pass is certified and re-ranked exactly, ties by train
// index), so the train image is laid out by region:
//   1. k-means (Lloyd) on a strided sample of the rows, P <= 64 centroids;
//   2. the centroids chained greedily (each next one the nearest unvisited),
//      so regions adjacent in the chain are near each other;
//   3. every row assigned to its nearest centroid and the rows stably
//      counting-sorted by the chain rank of their region: image position
//      p holds train row perm[p] (ipos is the inverse).
// Per classify call the queries get the same treatment (assign, sort), and
// each query tile's workgroups start their streams at the tile's
// neighbourhood in the chain (cand_kernel, qstart: the first region of the
// tile's region's phase, 8 phases by default, so the tiles of one phase
// still share staged tiles in L2); its thresholds are tight from the first
// tiles on.  Everything here is deterministic (integer counts, fixed
// summation orders), so the same train set always gets the same layout.
#include "knn_device.h"
#include "knn_kernels.h"

namespace knnk {

// Centroid image of the assignment kernel: the P <= 64 centroids (fp32,
// 2^jx-scaled) as bf16 A fragments of v_mfma_f32_32x32x16_bf16, [block b of
// 32 centroids][k-step s of 16 dims][row r][16 dims] (zero past P and d),
// and their fp32 squared norms (+inf past P).  One wave, lane = centroid.
__global__ void __launch_bounds__(64)
region_image_kernel(const float* __restrict__ cent, int P, int d, __bf16* __restrict__ img,
                    float* __restrict__ cnorm) {
  const int p = threadIdx.x, b = p >> 5, r = p & 31;
  const int DS = (d + 15) / 16;
  float s = 0.0f;
  for (int c = 0; c < DS * 16; ++c) {
    const float v = p < P && c < d ? cent[(int64_t)p * d + c] : 0.0f;
    s = __builtin_fmaf(v, v, s);
    img[((b * DS + (c >> 4)) * 32 + r) * 16 + (c & 15)] = (__bf16)v;
  }
  cnorm[p] = p < P ? s : KNN_INF_F;
}

// Nearest centroid of rows r = 0..n-1 (source row r * stride of X), as the
// fp32 operands 2^jx (x - mu) of every candidate path rounded to bf16 -- any
// assignment is valid, only locality matters, so the scores
// ||c||^2 - 2 x.c run on the matrix cores.  Block = 32 rows, 2 waves: the
// rows are staged into LDS as bf16 first (coalesced loads, all of a
// thread's in flight at once), then wave b multiplies them (B operand: lane (j, h) row j, dims
// 16s + 8h .. +7 of k-step s) with centroid block b (A: 32 centroids); lane
// (j, h) of wave b ends with the scores of centroids 32b + (i & 3) +
// 8 (i >> 2) + 4h (the 32x32 C layout); the lowest over both lanes of row j
// and both waves wins, the lowest centroid on ties.  out[r] = rank[p] (rank
// null: p); bcnt (nullable, zeroed): per 1024-row block, the count of each
// output key (the counting sort's histogram).
// DS = k-steps of 16 dims (compile time: the staging and the MFMA loop
// unroll completely, every load in flight at once).
constexpr int kAsgRows = 32;
constexpr int kAsgStride = 256 + 8;  // bf16 per staged row (d <= 256; 16-B aligned, conflict-reducing pad)
template <int DS>
__global__ void __launch_bounds__(128)
region_assign_kernel(const double* __restrict__ X, const double* __restrict__ mu, int64_t n, int d,
                     int64_t stride, int jx, const __bf16* __restrict__ img,
                     const float* __restrict__ cnorm, const int* __restrict__ rank,
                     int* __restrict__ out, int* __restrict__ bcnt) {
  __shared__ __attribute__((aligned(16))) __bf16 xs[kAsgRows * kAsgStride];
  __shared__ float bs[2][kAsgRows];
  __shared__ int bpi[2][kAsgRows];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  constexpr int dp = DS * 16;
  const int64_t r0 = (int64_t)blockIdx.x * kAsgRows;
  constexpr int total = kAsgRows * dp;  // a multiple of 128
  // (a constant trip count: the loop unrolls and every load is in flight
  // before the first conversion)
#pragma unroll
  for (int i = 0; i < total / 128; ++i) {
    const int e = tid + 128 * i;
    const int rr = e / dp, c = e - rr * dp;
    // unconditional loads at clamped addresses (no branch per load: all of
    // them issue before the first wait), the padding zeroed after
    const bool ok = r0 + rr < n && c < d;
    const int64_t ri = r0 + rr < n ? r0 + rr : n - 1;
    const int ci = c < d ? c : d - 1;
    const float v = (float)__builtin_ldexp(X[ri * stride * d + ci] - mu[ci], jx);
    xs[rr * kAsgStride + c] = (__bf16)(ok ? v : 0.0f);
  }
  // this lane's 16 centroid norms, loaded before the MFMAs
  float cn[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) cn[i] = cnorm[32 * wv + (i & 3) + 8 * (i >> 2) + 4 * h];
  __syncthreads();
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  const bf16x8* A = (const bf16x8*)img;  // 16-B fragments: [b][s][r][2]
#pragma unroll
  for (int st = 0; st < DS; ++st) {
    const bf16x8 bq = *(const bf16x8*)(xs + j * kAsgStride + 16 * st + 8 * h);
    const bf16x8 a = A[((wv * DS + st) * 32 + j) * 2 + h];
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bq, acc, 0, 0, 0);
  }
  float best = KNN_INF_F;
  int bp = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int p = 32 * wv + (i & 3) + 8 * (i >> 2) + 4 * h;
    const float sc = cn[i] - 2.0f * acc[i];
    if (sc < best || (sc == best && p < bp)) {
      best = sc;
      bp = p;
    }
  }
  const float ob = __shfl_xor(best, 32, 64);
  const int op = __shfl_xor(bp, 32, 64);
  if (ob < best || (ob == best && op < bp)) {
    best = ob;
    bp = op;
  }
  if (h == 0) {
    bs[wv][j] = best;
    bpi[wv][j] = bp;
  }
  __syncthreads();
  const int64_t row = r0 + j;
  if (wv == 0 && h == 0 && row < n) {
    if (bpi[1][j] != 0x7fffffff && (bp == 0x7fffffff || bs[1][j] < best)) bp = bpi[1][j];
    if (bp == 0x7fffffff) bp = 0;  // no finite score (a query beyond fp32 range)
    const int key = rank ? rank[bp] : bp;
    out[row] = key;
    if (bcnt) atomicAdd(&bcnt[(row >> 10) * kRegionMax + key], 1);
  }
}

// Lloyd update: centroid p = mean of the sample rows assigned to it (fp64
// sums in row order: deterministic); an empty centroid keeps its value.
// Grid = P blocks, thread = dimension (d <= 256).  Per chunk of 256 sample
// rows the members' offsets are compacted (in row order) into LDS first, so
// their loads go out 8 at a time instead of one dependent load per member.
__global__ void __launch_bounds__(256)
region_update_kernel(const double* __restrict__ X, const double* __restrict__ mu, int64_t ns,
                     int d, int64_t stride, int jx, const int* __restrict__ assign,
                     float* __restrict__ cent) {
  __shared__ int mem[256];
  __shared__ int wcnt[4];
  const int p = blockIdx.x, c = threadIdx.x, lane = c & 63, wv = c >> 6;
  const double mc = c < d ? mu[c] : 0.0;
  const int cc = c < d ? c : 0;
  double s = 0.0;
  int64_t cnt = 0;
  for (int64_t i0 = 0; i0 < ns; i0 += 256) {
    const bool is = i0 + c < ns && assign[i0 + c] == p;
    const unsigned long long bal = __ballot(is);
    __syncthreads();  // the previous chunk's reads of mem are done
    if (lane == 0) wcnt[wv] = __popcll(bal);
    __syncthreads();
    int before = 0, nm = 0;
    for (int w = 0; w < 4; ++w) {
      before += w < wv ? wcnt[w] : 0;
      nm += wcnt[w];
    }
    if (is)
      mem[before + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                             __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0))] = c;
    __syncthreads();
    cnt += nm;
    int k = 0;
    for (; k + 8 <= nm; k += 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = X[(i0 + mem[k + u]) * stride * d + cc];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += __builtin_ldexp(v[u] - mc, jx);
    }
    for (; k < nm; ++k) s += __builtin_ldexp(X[(i0 + mem[k]) * stride * d + cc] - mc, jx);
  }
  if (c < d && cnt > 0) cent[(int64_t)p * d + c] = (float)(s / (double)cnt);
}

// Initial centroids: sample rows p * ns / P (centred).
__global__ void region_init_kernel(const double* __restrict__ X, const double* __restrict__ mu,
                                   int64_t ns, int d, int64_t stride, int jx, int P,
                                   float* __restrict__ cent) {
  const int p = blockIdx.x;
  const int64_t r = (int64_t)p * ns / P;
  for (int c = threadIdx.x; c < d; c += blockDim.x)
    cent[(int64_t)p * d + c] = (float)__builtin_ldexp(X[r * stride * d + c] - mu[c], jx);
}

// Greedy chain over the P centroids (one wave, lane = centroid): start at
// the centroid farthest from centroid 0, then repeatedly the nearest
// unvisited one; rank[p] = its position in the chain.  The centroids are
// staged in LDS first ([p][d + 1]: conflict-free per-lane rows).
__global__ void __launch_bounds__(64)
region_chain_kernel(const float* __restrict__ cent, int P, int d, int* __restrict__ rank) {
  __shared__ float cs[kRegionMax * 257];
  const int p = threadIdx.x;
  for (int e = p; e < P * d; e += 64) {
    const int r = e / d, c = e - r * d;
    cs[r * (d + 1) + c] = cent[e];
  }
  __syncthreads();
  auto dist_to = [&](int cur) {
    float s = KNN_INF_F;
    if (p < P) {
      s = 0.0f;
      for (int c = 0; c < d; ++c) {
        const float t = cs[p * (d + 1) + c] - cs[cur * (d + 1) + c];
        s = __builtin_fmaf(t, t, s);
      }
    }
    return s == s ? s : 3e38f;  // (NaN: far)
  };
  // argmax / argmin over the wave, lowest index on ties
  auto pick = [&](float v, bool want_max) {
    float best = v;
    int bi = p;
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      const bool take = want_max ? (ov > best || (ov == best && oi < bi))
                                 : (ov < best || (ov == best && oi < bi));
      if (take) {
        best = ov;
        bi = oi;
      }
    }
    return bi;
  };
  float d0 = dist_to(0);
  int cur = pick(p < P ? d0 : -1.0f, true);
  bool visited = false;
  for (int step = 0; step < P; ++step) {
    if (p == cur) {
      visited = true;
      rank[p] = step;
    }
    if (step + 1 == P) break;
    const float dc = dist_to(cur);
    cur = pick(visited || p >= P ? KNN_INF_F : dc, false);
  }
}

// ------------------------------------------------------------ counting sort
// Stable sort of n keys in [0, kRegionMax) (key < 0: not sorted), in
// blocks of 1024 elements: per-block counts, per-key exclusive scans over
// the blocks, then a scatter that ranks equal keys within a block in index
// order (wave ballots on the key bits).
constexpr int kSortB = 1024;

__global__ void __launch_bounds__(kSortB)
sort_hist_kernel(const int* __restrict__ key, int64_t n, int* __restrict__ bcnt) {
  __shared__ int cnt[kRegionMax];
  if (threadIdx.x < kRegionMax) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kSortB + threadIdx.x;
  if (i < n) {
    const int k = key[i];
    if (k >= 0) atomicAdd(&cnt[k], 1);
  }
  __syncthreads();
  if (threadIdx.x < kRegionMax) bcnt[(int64_t)blockIdx.x * kRegionMax + threadIdx.x] = cnt[threadIdx.x];
}

// Grid = kRegionMax blocks (one per key): bcnt[b][k] <- exclusive prefix over
// blocks b, tot[k] <- the key's total.
__global__ void __launch_bounds__(kSortB)
sort_scan_kernel(int* __restrict__ bcnt, int64_t nb, int* __restrict__ tot) {
  __shared__ int ws[kSortB / 64];
  __shared__ int carry;
  const int k = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += kSortB) {
    __syncthreads();
    const int64_t b = b0 + tid;
    const int v = b < nb ? bcnt[b * kRegionMax + k] : 0;
    // inclusive scan within the wave
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) ws[wv] = x;
    __syncthreads();
    int before = carry;
    for (int w = 0; w < wv; ++w) before += ws[w];
    if (b < nb) bcnt[b * kRegionMax + k] = before + x - v;
    __syncthreads();
    if (tid == kSortB - 1) carry = before + x;
  }
  __syncthreads();
  if (tid == 0) tot[k] = carry;
}

// pos = (keys before k in total) + (key k in earlier blocks) + (key k
// earlier in this block).  inl > 0: bcnt holds the blocks' plain counts
// (nb = inl blocks, the query sort): each block sums the earlier blocks'
// counts and the totals itself instead of reading sort_scan_kernel's
// prefixes.  Outputs (each nullable): perm[pos] = i,
// ipos[i] = pos, qstart[pos] = rstart[k] (phases > 0: rstart of the first
// key of k's group, keys split into `phases` groups of P / phases: query
// tiles of one group share their streams' start); bases (block 0) = the
// exclusive prefix of tot (the start position of each key).
__global__ void __launch_bounds__(kSortB)
sort_scatter_kernel(const int* __restrict__ key, int64_t n, const int* __restrict__ bcnt,
                    const int* __restrict__ tot, int* __restrict__ perm, int* __restrict__ ipos,
                    const int* __restrict__ rstart, int* __restrict__ qstart, int* __restrict__ bases,
                    int P, int phases, int inl) {
  __shared__ int base[kRegionMax];
  __shared__ int boff[kRegionMax];
  __shared__ int wc[kSortB / 64][kRegionMax];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid < 64) {
    int v;
    if (inl > 0) {
      int before = 0, all = 0;
#pragma unroll 8
      for (int b = 0; b < inl; ++b) {
        const int c = bcnt[(int64_t)b * kRegionMax + tid];
        all += c;
        before += b < (int)blockIdx.x ? c : 0;
      }
      boff[tid] = before;
      v = all;
    } else {
      v = tot[tid];
      boff[tid] = bcnt[(int64_t)blockIdx.x * kRegionMax + tid];
    }
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (tid < kRegionMax) {
      base[tid] = x - v;
      if (bases && blockIdx.x == 0) bases[tid] = x - v;
    }
  }
  for (int e = tid; e < (kSortB / 64) * kRegionMax; e += kSortB) (&wc[0][0])[e] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kSortB + tid;
  const int k = i < n ? key[i] : -1;
  const bool valid = k >= 0;
  unsigned long long m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 6; ++b) {
    const bool bit = valid && ((k >> b) & 1);
    const unsigned long long bal = __ballot(bit);
    m &= bit ? bal : ~bal;
  }
  const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
  if (valid && r == 0) wc[wv][k] = __popcll(m);
  __syncthreads();
  if (!valid) return;
  int pos = base[k] + boff[k] + r;
  for (int w = 0; w < wv; ++w) pos += wc[w][k];
  if (perm) perm[pos] = (int)i;
  if (ipos) ipos[i] = pos;
  if (qstart) qstart[pos] = rstart[phases > 0 ? ((k * phases / P) * P + phases - 1) / phases : k];
}

int64_t region_sort_blocks(int64_t n) { return (n + kSortB - 1) / kSortB; }

// ------------------------------------------------------------ norm blocks
// The int8 candidate kernels start their accumulators at zero and test a
// 32-row sub-tile against the largest seed of its rows (the seed -ceil(||k||^2
// / 2) then leaves the LDS port: knn_cand_res.hip); that bound is tight only
// when the rows of a sub-tile have nearly equal norms.  So the image order is
// refined once more: every window of kNormWin consecutive image positions
// (the region order's, or train order) is sorted by the rows' squared norm.
// A window spans 64 staged tiles of 256 rows, i.e. a split sees at most a
// few tiles of one window: its stream stays in the window order's (region /
// train) sequence, only the rows within a window move.
//
// key[p] = the squared norm of image row p's train row perm0[p] (perm0 null:
// p): with cent (int8-coded set) the integer ||k||^2 of its codes k =
// rint(x 2^s - cent_i), the seed's own norm; otherwise the bits of the float
// ||x - mu||^2 (non-negative floats order as their bits).  One wave per row.
__global__ void __launch_bounds__(256)
norm_key_kernel(const double* __restrict__ X, const double* __restrict__ cent, int s,
                const double* __restrict__ mu, int64_t n, int d, const int* __restrict__ perm0,
                uint32_t* __restrict__ key) {
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); p < n; p += wstride) {
    const int64_t r = perm0 ? perm0[p] : p;
    if (cent) {
      int q2 = 0;
      for (int c = lane; c < d; c += 64) {
        const int k = (int)__builtin_rint(__builtin_ldexp(X[r * d + c], s) - cent[c]);
        q2 += k * k;
      }
      q2 = wave_sum_i(q2);
      if (lane == 0) key[p] = (uint32_t)q2;
    } else {
      double q2 = 0.0;
      for (int c = lane; c < d; c += 64) {
        const double t = X[r * d + c] - mu[c];
        q2 += t * t;
      }
      q2 = wave_sum_d(q2);
      if (lane == 0) key[p] = __float_as_uint((float)q2);
    }
  }
}

// Interleave of the norm ranks inside each 32-row sub-tile (il = the int8
// kernel's metric, 0: none): norm ranks 4a + b go to rows of the lane lists
// b = 0..3 of the query in the kernel's accumulator layout, so 4 rows of
// consecutive norm -- where a query's nearest neighbours cluster -- land in 4
// different lists.  Uninterleaved, a run of 4 adjacent rows shares a list, and
// one list holding 4 of a query's top W is what fails certification (an exact
// rescan): cfg2 sent 2 queries per 10k batch to it (~40 us per call).  The
// sub-tile's set of rows, hence its largest seed, does not change.
//   metric 6 (32x32: lane (j, h) list 0 = rows (i&3) + 8(i>>2) + 4h, i < 8,
//            list 1 the same + 16): list b = 2h + half at rows
//            16 half + 8x + 4h + y
//   metric 5 (16x16: lane group g16 = rows 4 g16 + i of each 16-row block)
__device__ __forceinline__ int norm_il(int r, int il) {
  const int a = r >> 2, b = r & 3;
  if (il == 6) return (b & 1) * 16 + (a >> 2) * 8 + (b >> 1) * 4 + (a & 3);
  if (il == 5) return (a >> 2) * 16 + b * 4 + (a & 3);
  return r;
}

// Spread of the sub-tiles over the window's staged tiles (il & 16, whole
// windows): the 512 sub-tiles of 32 rows, in norm order u = 64 a + b, go to
// tile b, slot a -- sub-tiles of adjacent norm lie in adjacent tiles, i.e.
// in different splits (tile t streams in split t mod S).  A query's nearest
// neighbours are near one another, hence of nearly equal norm: sorted
// windows put them into one tile of one split, where the interleave alone
// still let 4 of a cfg2 query's top 7 share a list (profiles/ab_log.md r5w).
// Each sub-tile keeps its rows, so its seed bound is unchanged.
constexpr int kNormSub = kNormWin / 32;            // sub-tiles per window
constexpr int kNormTiles = kNormWin / 256;          // staged tiles per window (256 rows)
__device__ __forceinline__ int norm_spread(int u) {
  return (u % kNormTiles) * (kNormSub / kNormTiles) + u / kNormTiles;
}

// One workgroup per window: (key, position) pairs bitonic-sorted in LDS
// (unique, so the order is deterministic), then perm[p] = perm0[source] and
// ipos[perm[p]] = p, p the sorted rank, interleaved within whole 32-row
// sub-tiles (norm_il, il & 15) and, il & 16, the sub-tiles spread over the
// window's tiles (norm_spread).  perm0 and perm are distinct buffers.
constexpr int kNormSortT = 1024;
__global__ void __launch_bounds__(kNormSortT)
norm_block_sort_kernel(const uint32_t* __restrict__ key, int64_t n, const int* __restrict__ perm0,
                       int* __restrict__ perm, int* __restrict__ ipos, int il) {
  __shared__ unsigned long long sk[kNormWin];  // 128 KiB
  const int tid = threadIdx.x;
  const int64_t w0 = (int64_t)blockIdx.x * kNormWin;
  const int cnt = (int)(n - w0 < kNormWin ? n - w0 : kNormWin);
  for (int i = tid; i < kNormWin; i += kNormSortT)
    sk[i] = i < cnt ? ((unsigned long long)key[w0 + i] << 32) | (unsigned)i : ~0ull;
  for (int size = 2; size <= kNormWin; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int t = tid; t < kNormWin / 2; t += kNormSortT) {
        const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
        const unsigned long long a = sk[lo], b = sk[hi];
        if (((lo & size) == 0) == (b < a)) {
          sk[lo] = b;
          sk[hi] = a;
        }
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < cnt; i += kNormSortT) {
    const int64_t src = w0 + (int64_t)(unsigned)(sk[i] & 0xFFFFFFFFu);
    const int r = perm0 ? perm0[src] : (int)src;
    int p = (i | 31) < cnt ? (i & ~31) | norm_il(i & 31, il & 15) : i;
    if ((il & 16) && cnt == kNormWin) p = norm_spread(p >> 5) * 32 + (p & 31);
    perm[w0 + p] = r;
    ipos[r] = (int)(w0 + p);
  }
}

void launch_norm_blocks(const double* X, const double* cent, int s, const double* mu, int64_t n,
                        int d, const int* perm0, uint32_t* key, int* perm, int* ipos, int il,
                        hipStream_t st) {
  if (n <= 0) return;
  int64_t blocks = (n + 3) / 4;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(norm_key_kernel, dim3((unsigned)blocks), dim3(256), 0, st, X, cent, s, mu, n, d,
                     perm0, key);
  hipLaunchKernelGGL(norm_block_sort_kernel, dim3((unsigned)((n + kNormWin - 1) / kNormWin)),
                     dim3(kNormSortT), 0, st, key, n, perm0, perm, ipos, il);
}

void launch_region_assign(const double* X, const double* mu, int64_t n, int d, int64_t stride,
                          int jx, const unsigned short* img, const float* cnorm, const int* rank, int* out,
                          int* bcnt, hipStream_t s) {
  if (n <= 0) return;
  const dim3 g((unsigned)((n + kAsgRows - 1) / kAsgRows)), b(128);
  const __bf16* im = (const __bf16*)img;
  switch ((d + 15) / 16) {
#define KNN_ASG(D_) \
    case D_: hipLaunchKernelGGL(region_assign_kernel<D_>, g, b, 0, s, X, mu, n, d, stride, jx, im, cnorm, rank, out, bcnt); break;
    KNN_ASG(1) KNN_ASG(2) KNN_ASG(3) KNN_ASG(4) KNN_ASG(5) KNN_ASG(6) KNN_ASG(7) KNN_ASG(8)
    KNN_ASG(9) KNN_ASG(10) KNN_ASG(11) KNN_ASG(12) KNN_ASG(13) KNN_ASG(14) KNN_ASG(15) KNN_ASG(16)
#undef KNN_ASG
    default: break;  // (d > 256: no region order, region_count)
  }
}

void launch_region_kmeans(const double* X, const double* mu, int64_t ns, int d, int64_t stride,
                          int jx, int P, int iters, float* cent, unsigned short* img_u, float* cnorm,
                          int* assign, int* rank, hipStream_t s) {
  __bf16* img = (__bf16*)img_u;
  hipLaunchKernelGGL(region_init_kernel, dim3(P), dim3(256), 0, s, X, mu, ns, d, stride, jx, P,
                     cent);
  for (int it = 0; it < iters; ++it) {
    hipLaunchKernelGGL(region_image_kernel, dim3(1), dim3(64), 0, s, cent, P, d, img, cnorm);
    launch_region_assign(X, mu, ns, d, stride, jx, img_u, cnorm, nullptr, assign, nullptr, s);
    hipLaunchKernelGGL(region_update_kernel, dim3(P), dim3(256), 0, s, X, mu, ns, d, stride, jx,
                       assign, cent);
  }
  hipLaunchKernelGGL(region_image_kernel, dim3(1), dim3(64), 0, s, cent, P, d, img, cnorm);
  hipLaunchKernelGGL(region_chain_kernel, dim3(1), dim3(64), 0, s, cent, P, d, rank);
}

void launch_region_sort(const int* key, int64_t n, int* bcnt, int* tot, int* perm, int* ipos,
                        const int* rstart, int* qstart, int* bases, hipStream_t s, int P,
                        int phases) {
  if (n <= 0) return;
  const int64_t nb = region_sort_blocks(n);
  hipLaunchKernelGGL(sort_hist_kernel, dim3((unsigned)nb), dim3(kSortB), 0, s, key, n, bcnt);
  hipLaunchKernelGGL(sort_scan_kernel, dim3(kRegionMax), dim3(kSortB), 0, s, bcnt, nb, tot);
  hipLaunchKernelGGL(sort_scatter_kernel, dim3((unsigned)nb), dim3(kSortB), 0, s, key, n, bcnt, tot,
                     perm, ipos, rstart, qstart, bases, P, phases, 0);
}

// The per-call query order: assignment with the sort's histogram fused in,
// then the scatter (which sums the block counts itself up to 64 blocks, i.e.
// 64K queries; beyond, the scan kernel runs between).
void launch_region_sort_queries(const double* Q, const double* mu, int64_t m, int d, int jx,
                                const unsigned short* img, const float* cnorm, int P, const int* rank,
                                const int* rstart, int phases, int* bcnt, int* tot, int* qkey,
                                int* qperm, int* qpos, int* qstart, hipStream_t s,
                                bool bcnt_zero) {
  if (m <= 0) return;
  const int64_t nb = region_sort_blocks(m);
  if (!bcnt_zero) launch_fill_i32(bcnt, nb * kRegionMax, 0, s);
  launch_region_assign(Q, mu, m, d, 1, jx, img, cnorm, rank, qkey, bcnt, s);
  int inl = (int)nb;
  if (nb > 64) {
    hipLaunchKernelGGL(sort_scan_kernel, dim3(kRegionMax), dim3(kSortB), 0, s, bcnt, nb, tot);
    inl = 0;
  }
  hipLaunchKernelGGL(sort_scatter_kernel, dim3((unsigned)nb), dim3(kSortB), 0, s, qkey, m, bcnt, tot,
                     qperm, qpos, rstart, qstart, nullptr, P, phases, inl);
}

}  // namespace knnk
