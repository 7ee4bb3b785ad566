// scan_probe.hip -- standalone timing of the fp16 threshold-scan kernel
// (knn_scan.hip) on random Gaussian fp16 operands; no correctness check (the
// parity suite covers the kernel through the library).  Timing tool only.
//   scan_probe <n> <m> <S> <abl> <chi> <reps>
// chi: threshold T_q = 2 sigma^2 chi - ||q||^2 (the chi^2_DP quantile that
// sets how many rows pass); prints ms per launch and rows appended per query.
#include "../-mpi-knn-_amd/csrc/knn_scan.hip"

#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

using namespace knnk;

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
      return 1;                                                           \
    }                                                                     \
  } while (0)

static uint32_t h_f2key(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u ^ ((u >> 31) ? 0xFFFFFFFFu : 0x80000000u);
}

int main(int argc, char** argv) {
  const int DP = 128;
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
  const int64_t m = argc > 2 ? atoll(argv[2]) : 10240;
  const int S = argc > 3 ? atoi(argv[3]) : 12;
  const int abl = argc > 4 ? atoi(argv[4]) : 0;
  const double chi = argc > 5 ? atof(argv[5]) : 75.0;
  const int reps = argc > 6 ? atoi(argv[6]) : 10;
  const int cap = 64;
  const int64_t n_pad = (n + 127) / 128 * 128;
  const int n_qt = (int)((m + kScanQ - 1) / kScanQ);
  const int64_t m_pad = (int64_t)n_qt * kScanQ;
  const double sigma = 64.0;
  std::mt19937_64 rng(1234);
  std::normal_distribution<float> nd(0.f, (float)sigma);
  const int RSH = DP + 8;  // shorts per train row
  std::vector<_Float16> xh((size_t)n_pad * RSH + 512, (_Float16)0.f);
  std::vector<float> seed(n_pad);
  for (int64_t r = 0; r < n_pad; r++) {
    double s2 = 0;
    for (int c = 0; c < DP; c++) {
      const _Float16 h = r < n ? (_Float16)nd(rng) : (_Float16)0.f;
      xh[r * RSH + c] = h;
      s2 += (double)h * (double)h;
    }
    seed[r] = r < n ? (float)s2 : INFINITY;
  }
  for (int64_t r = 0; r < n_pad; r++) {
    float* sp = (float*)&xh[r * RSH + DP];
    for (int l = 0; l < 4; l++) sp[l] = (l == 0 || (r & 3) == 0) ? seed[r + l] : 0.f;
  }
  std::vector<_Float16> qh((size_t)m_pad * DP);
  std::vector<uint32_t> tk(m_pad);
  for (int64_t q = 0; q < m_pad; q++) {
    double q2 = 0;
    for (int c = 0; c < DP; c++) {
      const float v = nd(rng);
      const _Float16 h = (_Float16)v;
      q2 += (double)h * (double)h;
      qh[q * DP + c] = (_Float16)(-2.0f * (float)h);
    }
    tk[q] = h_f2key((float)(2 * sigma * sigma * chi - q2));
  }
  float* dX;
  unsigned short* dQ;
  uint32_t* dT;
  int* dC;
  int2* dB;
  CK(hipMalloc(&dX, xh.size() * 2));
  CK(hipMalloc(&dQ, qh.size() * 2));
  CK(hipMalloc(&dT, tk.size() * 4));
  CK(hipMalloc(&dC, (size_t)m_pad * S * 4));
  CK(hipMalloc(&dB, (size_t)m_pad * S * cap * 8));
  CK(hipMemcpy(dX, xh.data(), xh.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dQ, qh.data(), qh.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dT, tk.data(), tk.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch_scan(DP, dX, dQ, n_pad, S, n_qt, dT, cap, dC, dB, abl, 0);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; i++) launch_scan(DP, dX, dQ, n_pad, S, n_qt, dT, cap, dC, dB, abl, 0);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  std::vector<int> cnt((size_t)m_pad * S);
  CK(hipMemcpy(cnt.data(), dC, cnt.size() * 4, hipMemcpyDeviceToHost));
  double tot = 0;
  int mx = 0, ovf = 0;
  for (int64_t q = 0; q < m; q++)
    for (int s = 0; s < S; s++) {
      const int c = cnt[q * S + s];
      tot += c;
      mx = std::max(mx, c);
      ovf += c > cap;
    }
  const double fl = 2.0 * n * m * 128;
  printf("RB=%d S=%d grid=%d blocks/CU=%d abl=%d chi=%.1f: %.3f ms  %.3f PF (%.3f of 2.5)  "
         "appended/query %.1f  max/seg %d  overflowed segs %d\n",
         scan_rb(DP), S, n_qt * S, scan_blocks_per_cu(DP), abl, chi, ms, fl / ms * 1e-12,
         fl / ms * 1e-12 / 2500.0, tot / m, mx, ovf);
  return 0;
}
