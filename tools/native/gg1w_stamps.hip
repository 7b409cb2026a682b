// Diagnostic build of the one-wave-per-SIMD gather-GEMM (gemm_gather1w_kernel,
// csrc/kernels/gather_gemm.hip) with s_memtime stamps (DTFS_GG1W_STAMPS): where
// does one K tile spend its cycles - step 0 (fragment waits, scale reads, A
// DMAs), step 1 (scale writes, A DMAs), step 2 (scale writes, rows), the
// barrier, step 3 (MFMAs + next tile's fragment reads, then W loads + ring DMA)
// - against the 64 x 32 = 2048 MFMA cycles it carries?
// DeepFM's first layer: F = 43 fields x 64 dims -> 1024, FM on.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o gg1w_stamps gg1w_stamps.hip
// Arguments: "hot" draws every row from the first 256 table rows (L2-resident)
// instead of uniformly from the 1M-row table.
#define DTFS_GG1W_STAMPS 1
#include "../../csrc/kernels/gather_gemm.hip"

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
  // "graph": the launches go through a captured HIP graph on a non-blocking
  // stream (the served step's way; the kernel's scratch use is reported)
  const bool graph = argc > 1 && std::string(argv[1]) == "graph";
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
  fill_bf16(W, size_t(N) * K, 11);  // timing only: any bytes serve as packed fragments
  (void)hipMemset(bias, 0, N * 4);
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
  if (graph) {
    hipFuncAttributes fa{};
    (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&dtfs::kern::gemm_gather1w_kernel<true>));
    printf("{\"kernel\": \"gemm_gather1w<FM>\", \"scratch_bytes_per_lane\": %zu}\n", fa.localSizeBytes);
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
    for (int i = 0; i < 4; ++i)
      (void)dtfs::launch_gemm_gather1w(table, V, rows, wts, 16384, F, W, bias, C, N, fm, 16384, N, 1, st);
    (void)hipStreamEndCapture(st, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int i = 0; i < 5; ++i) (void)hipGraphLaunch(ge, st);
    const hipError_t e = hipStreamSynchronize(st);
    printf("{\"graph_replays\": 5, \"status\": \"%s\"}\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
  }
  for (int M : {2048, 16384}) {
    auto run = [&] {
      return dtfs::launch_gemm_gather1w(table, V, rows, wts, M, F, W, bias, C, N, fm, M, N, 1, nullptr);
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
    (void)hipDeviceSynchronize();
    const int nb = (M / 128) * (N / 512);
    std::vector<unsigned long long> st(size_t(4096) * 4 * 12);
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(dtfs::kern::g_gg1w_stamps), st.size() * 8);
    std::vector<double> pro, loop, epi, tile, seg[6];
    for (int b = 0; b < std::min(nb, 4096); ++b)
      for (int w = 0; w < 4; ++w) {
        const unsigned long long* t = &st[(size_t(b) * 4 + w) * 12];
        pro.push_back(double(t[1] - t[0]));
        loop.push_back(double(t[9] - t[1]));
        epi.push_back(double(t[10] - t[9]));
        tile.push_back(double(t[8] - t[2]));
        for (int k = 0; k < 6; ++k) seg[k].push_back(double(t[3 + k] - t[2 + k]));
      }
    printf("{\"kernel\": \"gemm_gather1w (FM%s)\", \"M\": %d, \"N\": %d, \"F\": %d, \"blocks\": %d, \"event_us\": %.2f, "
           "\"median_cycles\": {\"prologue\": %.0f, \"loop\": %.0f, \"loop_per_k_tile\": %.0f, \"epilogue\": %.0f, "
           "\"sampled_tile\": %.0f, \"step0\": %.0f, \"step1\": %.0f, \"step2\": %.0f, \"barrier\": %.0f, "
           "\"step3\": %.0f, \"unused\": %.0f}}\n",
           hot ? ", L2-hot rows" : "", M, N, F, nb, ms * 1e3 / 20, med(pro), med(loop), med(loop) / F, med(epi),
           med(tile), med(seg[0]), med(seg[1]), med(seg[2]), med(seg[3]), med(seg[4]), med(seg[5]));
  }
  return 0;
}
