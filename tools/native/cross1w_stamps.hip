// Diagnostic build of the one-wave MX-fp8 cross kernel (cross1w_kernel,
// csrc/kernels/cross_gemm.hip) with s_memtime stamps (DTFS_CROSS1W_STAMPS):
// where does one 128-deep K tile spend its cycles - step 0 (fragment waits,
// G3 W loads, fragments 6 / 7), step 1 (G0: W + A DMAs), step 2 (G1), the
// barrier, step 3 (G2 + the next tile's fragments) - against the 64 x 32 =
// 2048 MFMA cycles it carries? DCN-v2 cross shape: N = 2752, K = 2816.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I ../../csrc/kernels -o cross1w_stamps cross1w_stamps.hip
// Arguments: M values (default 2048 16384).
#define DTFS_CROSS1W_STAMPS 1
#include "cross_gemm_1w.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

static void fill_bytes(void* p, size_t n, uint32_t seed, uint8_t mask) {
  std::vector<uint8_t> h(n);
  uint32_t x = seed;
  for (size_t i = 0; i < n; ++i) {
    x = x * 1664525u + 1013904223u;
    h[i] = uint8_t(x >> 24) & mask;  // e4m3 with the top exponent bits clear: finite, small
  }
  (void)hipMemcpy(p, h.data(), n, hipMemcpyHostToDevice);
}

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  std::vector<int> Ms;
  for (int i = 1; i < argc; ++i) Ms.push_back(std::atoi(argv[i]));
  if (Ms.empty()) Ms = {2048, 16384};
  const int N = 2752, K = 2816, Mmax = 16384;
  void *A, *Wp, *Z, *X0;
  float *bias, *sa, *sw, *hw, *dot;
  (void)hipMalloc(&A, size_t(Mmax) * K);
  (void)hipMalloc(&Wp, size_t(N) * K);
  (void)hipMalloc(&Z, size_t(Mmax) * N * 2);
  (void)hipMalloc(&X0, size_t(Mmax) * N * 2);
  (void)hipMalloc(&bias, N * 4);
  (void)hipMalloc(&sa, Mmax * 4);
  (void)hipMalloc(&sw, N * 4);
  (void)hipMalloc(&hw, N * 4);
  (void)hipMalloc(&dot, size_t(8) * Mmax * 4);
  fill_bytes(A, size_t(Mmax) * K, 3, 0xb7);
  fill_bytes(Wp, size_t(N) * K, 5, 0xb7);
  fill_bytes(X0, size_t(Mmax) * N * 2, 7, 0x3b);
  (void)hipMemset(bias, 0, N * 4);
  {
    std::vector<float> one(std::max(Mmax, N), 0.01f);
    (void)hipMemcpy(sa, one.data(), Mmax * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(sw, one.data(), N * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(hw, one.data(), N * 4, hipMemcpyHostToDevice);
  }
  for (int M : Ms) {
    if (M < 1 || M > Mmax) continue;
    dtfs::CrossGemmArgs a{};
    a.A = A;
    a.lda = K;
    a.sa = sa;
    a.sw = sw;
    a.bias = bias;
    a.Z = Z;
    a.ldz = N;
    a.X0 = X0;
    a.XL = X0;
    a.ldx = N;
    a.M = M;
    a.N = N;
    a.K = K;
    auto run = [&] { return dtfs::launch_cross1w(a, Wp, nullptr); };
    for (int i = 0; i < 20; ++i)
      if (run() != hipSuccess) {
        printf("launch failed\n");
        return 1;
      }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) (void)run();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)run();  // the stamped dispatch (last one wins)
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("kernel failed\n");
      return 1;
    }
    const int nb = ((M + 127) / 128) * dtfs::cross1w_tiles_n(N);
    std::vector<unsigned long long> st(size_t(4096) * 4 * 10);
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(dtfs::kern::g_cross1w_stamps), st.size() * 8);
    std::vector<double> pro, loop, epi, tile, seg[5];
    for (int b = 0; b < std::min(nb, 4096); ++b)
      for (int w = 0; w < 4; ++w) {
        const unsigned long long* t = &st[(size_t(b) * 4 + w) * 10];
        pro.push_back(double(t[1] - t[0]));
        loop.push_back(double(t[8] - t[1]));
        epi.push_back(double(t[9] - t[8]));
        tile.push_back(double(t[7] - t[2]));
        for (int k = 0; k < 5; ++k) seg[k].push_back(double(t[3 + k] - t[2 + k]));
      }
    std::vector<unsigned long long> tt(size_t(4096) * 4 * 32);
    (void)hipMemcpyFromSymbol(tt.data(), HIP_SYMBOL(dtfs::kern::g_cross1w_tiles), tt.size() * 8);
    const int KT = K / 128;
    std::string per_tile;
    for (int t = 0; t + 1 < KT && t < 31; ++t) {
      std::vector<double> d;
      for (int b = 0; b < std::min(nb, 4096); ++b)
        for (int w = 0; w < 4; ++w) {
          const unsigned long long* x = &tt[(size_t(b) * 4 + w) * 32];
          d.push_back(double(x[t + 1] - x[t]));
        }
      per_tile += (t ? ", " : "") + std::to_string(int(med(d)));
    }
    {  // the last tile: its top to the loop end
      std::vector<double> d;
      for (int b = 0; b < std::min(nb, 4096); ++b)
        for (int w = 0; w < 4; ++w) d.push_back(double(st[(size_t(b) * 4 + w) * 10 + 8] - tt[(size_t(b) * 4 + w) * 32 + KT - 1]));
      per_tile += ", " + std::to_string(int(med(d)));
    }
    printf("{\"M\": %d, \"median_cycles_per_k_tile\": [%s]}\n", M, per_tile.c_str());
    const double flops = 2.0 * M * N * K;
    printf("{\"kernel\": \"cross1w\", \"M\": %d, \"N\": %d, \"K\": %d, \"blocks\": %d, \"event_us\": %.2f, "
           "\"pflops\": %.2f, \"median_cycles\": {\"prologue\": %.0f, \"loop\": %.0f, \"loop_per_k_tile\": %.0f, "
           "\"epilogue\": %.0f, \"sampled_tile\": %.0f, \"step0\": %.0f, \"step1\": %.0f, \"step2\": %.0f, "
           "\"barrier\": %.0f, \"step3\": %.0f}}\n",
           M, N, K, nb, ms * 1e3 / 20, flops / (ms * 1e-3 / 20) / 1e15, med(pro), med(loop), med(loop) / (K / 128),
           med(epi), med(tile), med(seg[0]), med(seg[1]), med(seg[2]), med(seg[3]), med(seg[4]));
  }
  return 0;
}
