// Diagnostic build of the gather-GEMM (gemm_gather_kernel, csrc/kernels/gemm.hip)
// with per-phase s_memtime stamps (DTFS_GG_STAMPS): where does a K tile of the
// gather-GEMM spend its cycles - the read / DMA-issue / counted-wait / barrier
// segment of each of the 8-phase schedule's 4 phases, or the MFMA segment after
// it - and how does its loop compare with the dense 8-phase GEMM of the same
// shape (DTFS_8PH_STAMPS: prologue / loop / epilogue)?
// DeepFM's first layer: F = 43 fields x 64 dims -> 1024, rows drawn uniformly
// from a 1M-row table (the gather's time does not depend on row locality,
// profiles/r04_gather_locality.md).
// Build: hipcc --offload-arch=gfx950 -O3 -I../../csrc -o gg_stamps gg_stamps.hip
// Ablations (timing only, the results are wrong): -DDTFS_GG_NO_SCALE drops the
// scale pass; argument "wdl" runs without the FM term (EXTRA 0).
#define DTFS_GG_STAMPS 1
#define DTFS_8PH_STAMPS 1
#include "../../csrc/kernels/gemm.hip"

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
  const bool wdl = argc > 1 && std::string(argv[1]) == "wdl";
  const int F = 43, N = 1024, V = 1 << 20, K = F * 64;
  void *table, *W, *C;
  float *bias, *fm, *wts;
  int32_t* rows;
  const int Mmax = 16384;
  (void)hipMalloc(&table, size_t(V) * 128);
  (void)hipMalloc(&W, size_t(N) * K * 2);
  (void)hipMalloc(&C, size_t(Mmax) * N * 2);
  (void)hipMalloc(&bias, N * 4);
  (void)hipMalloc(&fm, size_t(2) * Mmax * 4);
  (void)hipMalloc(&rows, size_t(F) * Mmax * 4);
  (void)hipMalloc(&wts, size_t(F) * Mmax * 4);
  fill_bf16(table, size_t(V) * 64, 7);
  fill_bf16(W, size_t(N) * K, 11);
  (void)hipMemset(bias, 0, N * 4);
  {
    std::vector<int32_t> r(size_t(F) * Mmax);
    std::vector<float> w(size_t(F) * Mmax);
    uint32_t x = 3;
    for (size_t i = 0; i < r.size(); ++i) {
      x = x * 1664525u + 1013904223u;
      r[i] = int32_t(x % uint32_t(V));
      w[i] = 0.5f + float((x >> 8) & 0xff) / 512.f;
    }
    (void)hipMemcpy(rows, r.data(), r.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(wts, w.data(), w.size() * 4, hipMemcpyHostToDevice);
  }
  for (int M : {2048, 16384}) {
    // rows_t / wts_t are field-major [F][Mp] with Mp = M here (a multiple of 256)
    auto gather = [&] {
      return dtfs::launch_gemm_gather(table, V, rows, wts, M, F, W, bias, C, N, wdl ? nullptr : fm, M, N, 1, nullptr,
                                      nullptr, nullptr, 0);
    };
    auto dense = [&] {  // the same GEMM with x already in HBM (C's rows stand in for x; timing only)
      return dtfs::launch_gemm(table, K, W, K, bias, nullptr, nullptr, C, N, false, nullptr, nullptr, 0, M, N, K, 1,
                               false, 0, 17, nullptr);
    };
    for (int which = 0; which < 2; ++which) {
      for (int i = 0; i < 20; ++i)
        if ((which ? dense() : gather()) != hipSuccess) {
          printf("launch failed\n");
          return 1;
        }
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      for (int i = 0; i < 20; ++i) (void)(which ? dense() : gather());
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      (void)(which ? dense() : gather());  // the stamped dispatch (last one wins)
      (void)hipDeviceSynchronize();
      const int nb = (M / 256) * (N / 256);
      if (which == 0) {
        std::vector<unsigned long long> st(size_t(4096) * 8 * 16);
        (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(dtfs::kern::g_gg_stamps), st.size() * 8);
        std::vector<double> pro, loop, epi, tile, seg[8];
        for (int b = 0; b < std::min(nb, 4096); ++b)
          for (int w = 0; w < 8; ++w) {
            const unsigned long long* t = &st[(size_t(b) * 8 + w) * 16];
            pro.push_back(double(t[1] - t[0]));
            loop.push_back(double(t[11] - t[1]));
            epi.push_back(double(t[12] - t[11]));
            tile.push_back(double(t[10] - t[2]));
            for (int k = 0; k < 8; ++k) seg[k].push_back(double(t[3 + k] - t[2 + k]));
          }
        printf("{\"kernel\": \"gemm_gather (%s%s)\", \"M\": %d, \"N\": %d, \"F\": %d, \"blocks\": %d, \"event_us\": %.2f, "
               "\"median_cycles\": {\"prologue\": %.0f, \"loop\": %.0f, \"loop_per_k_tile\": %.0f, \"epilogue\": %.0f, "
               "\"sampled_tile\": %.0f, \"phases\": [",
               wdl ? "no FM" : "FM",
#ifdef DTFS_GG_NO_SCALE
               ", no scale pass",
#else
               "",
#endif
               M, N, F, nb, ms * 1e3 / 20, med(pro), med(loop), med(loop) / F, med(epi), med(tile));
        for (int p = 0; p < 4; ++p)
          printf("%s{\"wait\": %.0f, \"mma\": %.0f}", p ? ", " : "", med(seg[2 * p]), med(seg[2 * p + 1]));
        printf("]}}\n");
      } else {
        std::vector<unsigned long long> st(size_t(4096) * 8 * 4);
        (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(dtfs::kern::g_8ph_stamps), st.size() * 8);
        std::vector<double> pro, loop, epi;
        for (int b = 0; b < std::min(nb, 4096); ++b)
          for (int w = 0; w < 8; ++w) {
            const unsigned long long* t = &st[(size_t(b) * 8 + w) * 4];
            pro.push_back((t[1] - t[0]) * 0.01);
            loop.push_back((t[2] - t[1]) * 0.01);
            epi.push_back((t[3] - t[2]) * 0.01);
          }
        printf("{\"kernel\": \"gemm_8ph (dense, same shape)\", \"M\": %d, \"N\": %d, \"K\": %d, \"blocks\": %d, "
               "\"event_us\": %.2f, \"median_us\": {\"prologue\": %.2f, \"loop\": %.2f, \"loop_per_k_tile\": %.3f, "
               "\"epilogue\": %.2f}}\n",
               M, N, K, nb, ms * 1e3 / 20, med(pro), med(loop), med(loop) / (K / 64), med(epi));
      }
    }
  }
  return 0;
}
