// Diagnostic build of the 8-phase GEMM with s_memrealtime stamps
// (DTFS_8PH_STAMPS, csrc/kernels/gemm.hip): where does a dispatch spend its
// time - block start skew, prologue (first tiles' DMA), main loop, epilogue?
// Read the SHARES, not the absolute length (the stamps' waits add a little).
// Build: hipcc --offload-arch=gfx950 -O3 -I../csrc -o g8ph_stamps g8ph_stamps.hip
#define DTFS_8PH_STAMPS 1
#include "../csrc/kernels/gemm.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

static void fill(void* p, size_t bytes, bool fp8) {
  std::vector<uint8_t> h(bytes);
  uint32_t x = 12345;
  for (size_t i = 0; i < bytes; ++i) {
    x = x * 1664525u + 1013904223u;
    h[i] = uint8_t(x >> 24) & (fp8 ? 0x77 : 0x3f);  // no NaN / inf patterns
  }
  (void)hipMemcpy(p, h.data(), bytes, hipMemcpyHostToDevice);
}

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main() {
  struct Cfg { int M, N, K; bool fp8; bool nobias; };
  const Cfg cfgs[] = {{256, 256, 128, false, false}, {256, 256, 2816, false, false},
                      {16384, 1024, 128, false, false}, {16384, 1024, 576, false, false},
                      {16384, 1024, 1024, false, false}, {16384, 1024, 2816, false, false},
                      {16384, 1024, 2816, true, false}, {16384, 2752, 2816, true, false}};
  for (const Cfg& c : cfgs) {
    const int eb = c.fp8 ? 1 : 2;
    void *A, *W, *C;
    float *bias, *sa, *sw;
    (void)hipMalloc(&A, size_t(c.M) * c.K * eb);
    (void)hipMalloc(&W, size_t(c.N) * c.K * eb);
    (void)hipMalloc(&C, size_t(c.M) * c.N * 2);
    (void)hipMalloc(&bias, c.N * 4);
    (void)hipMalloc(&sa, c.M * 4);
    (void)hipMalloc(&sw, c.N * 4);
    fill(A, size_t(c.M) * c.K * eb, c.fp8);
    fill(W, size_t(c.N) * c.K * eb, c.fp8);
    (void)hipMemset(bias, 0, c.N * 4);
    std::vector<float> ones(std::max(c.M, c.N), 1.f);
    (void)hipMemcpy(sa, ones.data(), c.M * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(sw, ones.data(), c.N * 4, hipMemcpyHostToDevice);
    auto launch = [&] {
      return dtfs::launch_gemm(A, c.K, W, c.K, c.nobias ? nullptr : bias, c.fp8 ? sa : nullptr, c.fp8 ? sw : nullptr, C, c.N, false, nullptr,
                               nullptr, 0, c.M, c.N, c.K, 1, c.fp8, 0, 17, nullptr);
    };
    for (int i = 0; i < 20; ++i)
      if (launch() != hipSuccess) { printf("launch failed\n"); return 1; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) (void)launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)launch();  // the stamped dispatch (last one wins)
    (void)hipDeviceSynchronize();
    const int nb = ((c.M + 255) / 256) * ((c.N + 255) / 256);
    std::vector<unsigned long long> st(size_t(4096) * 8 * 4);
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(dtfs::kern::g_8ph_stamps), st.size() * 8);
    unsigned long long t_min = ~0ull, t_max = 0;
    std::vector<double> pro, loop, epi, start;
    for (int b = 0; b < std::min(nb, 4096); ++b)
      for (int w = 0; w < 8; ++w) {
        const unsigned long long* t = &st[(size_t(b) * 8 + w) * 4];
        t_min = std::min(t_min, t[0]);
        t_max = std::max(t_max, t[3]);
        pro.push_back((t[1] - t[0]) * 0.01);
        loop.push_back((t[2] - t[1]) * 0.01);
        epi.push_back((t[3] - t[2]) * 0.01);
      }
    for (int b = 0; b < std::min(nb, 4096); ++b) start.push_back((st[size_t(b) * 32] - t_min) * 0.01);
    printf("{\"nobias\": %d, \"M\": %d, \"N\": %d, \"K\": %d, \"fp8\": %d, \"blocks\": %d, \"event_us\": %.2f, \"stamped_span_us\": %.2f, "
           "\"median_prologue_us\": %.2f, \"median_loop_us\": %.2f, \"median_epilogue_us\": %.2f, "
           "\"max_block_start_us\": %.2f}\n",
           int(c.nobias), c.M, c.N, c.K, int(c.fp8), nb, ms * 1e3 / 20, (t_max - t_min) * 0.01, med(pro), med(loop), med(epi),
           *std::max_element(start.begin(), start.end()));
    (void)hipFree(A);
    (void)hipFree(W);
    (void)hipFree(C);
    (void)hipFree(bias);
    (void)hipFree(sa);
    (void)hipFree(sw);
  }
  return 0;
}
