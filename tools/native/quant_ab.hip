// quant_rows_kernel (8 columns per lane, 8-byte stores) vs quant_rows16_kernel
// (16 columns per lane, 16-byte stores) at DCN-v2's shape (16384 x 2752 ->
// e4m3 [16384, 2816]): bit equality and interleaved timing.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc -o quant_ab quant_ab.hip
#include "../../csrc/kernels/interaction.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

int main() {
  const int M = 16384, K = 2752, Kq = 2816;
  void *x, *q1, *q2;
  float *s1, *s2;
  (void)hipMalloc(&x, size_t(M) * K * 2);
  (void)hipMalloc(&q1, size_t(M) * Kq);
  (void)hipMalloc(&q2, size_t(M) * Kq);
  (void)hipMalloc(&s1, M * 4);
  (void)hipMalloc(&s2, M * 4);
  {
    std::vector<uint16_t> h(size_t(M) * K);
    uint32_t r = 1;
    for (auto& v : h) {
      r = r * 1664525u + 1013904223u;
      v = uint16_t(0x3800 + ((r >> 12) & 0x7ff)) ^ uint16_t(r & 0x8000);
    }
    (void)hipMemcpy(x, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  }
  const auto* xi = static_cast<const dtfs::kern::bf16*>(x);
  dim3 grid((M + 3) / 4), block(256);
  auto old_k = [&] {
    hipLaunchKernelGGL(dtfs::kern::quant_rows_kernel<6>, grid, block, 0, nullptr, xi, int64_t(K), M, K,
                       static_cast<uint8_t*>(q1), int64_t(Kq), s1, Kq);
  };
  auto new_k = [&] {
    hipLaunchKernelGGL(dtfs::kern::quant_rows16_kernel<3>, grid, block, 0, nullptr, xi, int64_t(K), M, K,
                       static_cast<uint8_t*>(q2), int64_t(Kq), s2, Kq);
  };
  old_k();
  new_k();
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::vector<uint8_t> a(size_t(M) * Kq), b(size_t(M) * Kq);
  std::vector<float> sa(M), sb(M);
  (void)hipMemcpy(a.data(), q1, a.size(), hipMemcpyDeviceToHost);
  (void)hipMemcpy(b.data(), q2, b.size(), hipMemcpyDeviceToHost);
  (void)hipMemcpy(sa.data(), s1, M * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(sb.data(), s2, M * 4, hipMemcpyDeviceToHost);
  const bool same = a == b && sa == sb;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto time = [&](auto&& fn) {
    (void)hipEventRecord(e0);
    for (int i = 0; i < 50; ++i) fn();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e3f / 50;
  };
  std::vector<float> to, tn;
  for (int r = 0; r < 7; ++r) {
    to.push_back(time(old_k));
    tn.push_back(time(new_k));
  }
  std::sort(to.begin(), to.end());
  std::sort(tn.begin(), tn.end());
  printf("{\"bit_equal\": %s, \"old_us\": %.2f, \"new_us\": %.2f}\n", same ? "true" : "false", to[3], tn[3]);
  return same ? 0 : 1;
}
