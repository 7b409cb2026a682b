// Diagnostic build of the one-launch DeepFM tower (gather_mlp_kernel,
// csrc/kernels/gather_mlp.hip) with s_memtime stamps (DTFS_GM_STAMPS): the
// prologue, the K loop (and the six parts of one K tile in its middle against
// its 64 x 32 = 2048 MFMA cycles), the h1 store, GEMM2, the h2 store and
// GEMM3 + head, per wave, median over waves.
// DeepFM: F = 43 fields x 64 dims -> 1024 -> 512 -> 256 -> score, FM on.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -o gm_stamps gm_stamps.hip
// Argument "hot": every row from the first 256 table rows (L2-resident).
// The prologue includes the rows' resolve (int32 row ids + fp32 weights here).
#define DTFS_GM_STAMPS 1
#include "../../csrc/kernels/gather_mlp.hip"

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

static void fill_bf16(void* p, size_t n, uint32_t seed) {
  std::vector<uint16_t> h(n);
  uint32_t x = seed;
  for (size_t i = 0; i < n; ++i) {
    x = x * 1664525u + 1013904223u;
    h[i] = uint16_t(0x3c00 + ((x >> 20) & 0x3ff)) ^ uint16_t((x >> 4) & 0x8000);  // |v| in [2^-7, 2^-6)
  }
  (void)hipMemcpy(p, h.data(), n * 2, hipMemcpyHostToDevice);
}

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  const bool hot = argc > 1 && std::string(argv[1]) == "hot";
  const int F = 43, V = 1 << 20, K = F * 64;
  void *table, *W1, *W2, *W3;
  float *b1, *b2, *b3, *hw, *y, *wts;
  int32_t* rows;
  const int Mmax = 16384;
  (void)hipMalloc(&table, size_t(V) * 128);
  (void)hipMalloc(&W1, size_t(1024) * K * 2);
  (void)hipMalloc(&W2, size_t(512) * 1024 * 2);
  (void)hipMalloc(&W3, size_t(256) * 512 * 2);
  (void)hipMalloc(&b1, 1024 * 4);
  (void)hipMalloc(&b2, 512 * 4);
  (void)hipMalloc(&b3, 256 * 4);
  (void)hipMalloc(&hw, 256 * 4);
  (void)hipMalloc(&y, size_t(Mmax) * 4);
  (void)hipMalloc(&rows, size_t(F) * Mmax * 4);
  (void)hipMalloc(&wts, size_t(F) * Mmax * 4);
  fill_bf16(table, size_t(V) * 64, 7);
  fill_bf16(W1, size_t(1024) * K, 11);  // timing only: any bytes serve as packed fragments
  fill_bf16(W2, size_t(512) * 1024, 13);
  fill_bf16(W3, size_t(256) * 512, 17);
  (void)hipMemset(b1, 0, 1024 * 4);
  (void)hipMemset(b2, 0, 512 * 4);
  (void)hipMemset(b3, 0, 256 * 4);
  (void)hipMemset(hw, 0, 256 * 4);
  {
    std::vector<int32_t> r(size_t(F) * Mmax);
    std::vector<float> w(size_t(F) * Mmax);
    uint32_t x = 3;
    for (size_t i = 0; i < r.size(); ++i) {
      x = x * 1664525u + 1013904223u;
      r[i] = int32_t(x % uint32_t(hot ? 256 : V));
      w[i] = 0.5f + float((x >> 8) & 0xff) / 512.f;
    }
    (void)hipMemcpy(rows, r.data(), r.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(wts, w.data(), w.size() * 4, hipMemcpyHostToDevice);
  }
  for (int M : {8192, 16384}) {
    dtfs::EmbedArgs a;  // int32 row ids [M][F] + fp32 weights (the resolve runs in the kernel's prologue)
    a.table = table;
    a.V = V;
    a.ids = rows;
    a.ids64 = false;
    a.ids_ld = F;
    a.wts = wts;
    a.wts_ld = F;
    a.B = M;
    a.F = F;
    a.D = 64;
    a.modulo = V;
    auto run = [&] {
      return dtfs::launch_gather_mlp(a, W1, b1, W2, b2, 1, W3, b3, 1, hw, 0.f, true, 2, y, nullptr);
    };
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
    const int nb = M / 64;
    std::vector<unsigned long long> st(size_t(1024) * 4 * 16);
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(dtfs::kern::g_gm_stamps), st.size() * 8);
    std::vector<double> seg[13];
    for (int b = 0; b < std::min(nb, 1024); ++b)
      for (int w = 0; w < 4; ++w) {
        const unsigned long long* t = &st[(size_t(b) * 4 + w) * 16];
        seg[0].push_back(double(t[1] - t[0]));   // prologue
        seg[1].push_back(double(t[8] - t[1]));   // K loop
        seg[2].push_back(double(t[7] - t[2]));   // sampled tile (wait .. end of step 3)
        for (int k = 0; k < 5; ++k) seg[3 + k].push_back(double(t[3 + k] - t[2 + k]));
        seg[8].push_back(double(t[9] - t[8]));    // h1 store
        seg[9].push_back(double(t[10] - t[9]));   // GEMM2
        seg[10].push_back(double(t[11] - t[10])); // h2 store
        seg[11].push_back(double(t[12] - t[11])); // GEMM3 + head
        seg[12].push_back(double(t[12] - t[0]));  // total
      }
    printf("{\"kernel\": \"gather_mlp (FM%s)\", \"M\": %d, \"F\": %d, \"blocks\": %d, \"event_us\": %.2f, "
           "\"median_cycles\": {\"prologue\": %.0f, \"loop\": %.0f, \"loop_per_k_tile\": %.0f, \"sampled_tile\": %.0f, "
           "\"step0\": %.0f, \"step1\": %.0f, \"step2\": %.0f, \"barrier\": %.0f, \"step3\": %.0f, "
           "\"h1_store\": %.0f, \"gemm2\": %.0f, \"h2_store\": %.0f, \"gemm3_head\": %.0f, \"total\": %.0f}}\n",
           hot ? ", L2-hot rows" : "", M, F, nb, ms * 1e3 / 20, med(seg[0]), med(seg[1]), med(seg[1]) / F, med(seg[2]),
           med(seg[3]), med(seg[4]), med(seg[5]), med(seg[6]), med(seg[7]), med(seg[8]), med(seg[9]), med(seg[10]),
           med(seg[11]), med(seg[12]));
  }
  return 0;
}
