// Timing-only ablations of the fused MLP tail (csrc/kernels/mlp_tail.hip,
// TAIL_ABL): which part bounds it at 16384 x 1024 -> 512 -> 256 -> score?
// Build one binary per TAIL_ABL value:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc -DTAIL_ABL=<bits> -o tail_ablate tail_ablate.hip
#include "../../csrc/kernels/mlp_tail.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

int main() {
  const int M = 16384, K1 = 1024, N2 = 512, N3 = 256;
  void *X, *W2p, *W3p;
  float *b2, *b3, *hw, *y;
  (void)hipMalloc(&X, size_t(M) * K1 * 2);
  (void)hipMalloc(&W2p, size_t(N2) * K1 * 2);
  (void)hipMalloc(&W3p, size_t(N3) * N2 * 2);
  (void)hipMalloc(&b2, N2 * 4);
  (void)hipMalloc(&b3, N3 * 4);
  (void)hipMalloc(&hw, N3 * 4);
  (void)hipMalloc(&y, M * 4);
  (void)hipMemset(X, 0x3c, size_t(M) * K1 * 2);
  (void)hipMemset(W2p, 0x3c, size_t(N2) * K1 * 2);
  (void)hipMemset(W3p, 0x3c, size_t(N3) * N2 * 2);
  (void)hipMemset(b2, 0, N2 * 4);
  (void)hipMemset(b3, 0, N3 * 4);
  (void)hipMemset(hw, 0, N3 * 4);
  auto run = [&] {
    return dtfs::launch_mlp_tail(X, K1, M, K1, W2p, b2, 1, N2, W3p, b3, 1, N3, hw, 0.f, nullptr, 0, 0, 2, y, nullptr);
  };
  for (int i = 0; i < 50; ++i)
    if (run() != hipSuccess) {
      printf("launch failed\n");
      return 1;
    }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  std::vector<float> r;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0);
    for (int i = 0; i < 50; ++i) (void)run();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    r.push_back(ms * 1e3f / 50);
  }
  std::sort(r.begin(), r.end());
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("{\"tail_abl\": %d, \"us\": %.2f}\n", TAIL_ABL, r[2]);
  return 0;
}
