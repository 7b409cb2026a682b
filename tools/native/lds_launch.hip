// Per-launch cost vs static LDS size: an almost empty kernel (each thread
// touches its LDS once) with 16..160 KiB of LDS, 1 and 256 workgroups of 512
// threads, 200 back-to-back launches timed with events. Checks whether a large
// LDS allocation (the 8-phase GEMM's 128 KiB) adds a fixed per-launch cost.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int KB>
__global__ void __launch_bounds__(512) touch(float* out) {
  __shared__ float s[KB * 256];
  s[threadIdx.x * (KB * 256 / 512)] = float(threadIdx.x);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s[(blockIdx.x * 7) % (KB * 256)];
}

template <int KB>
static void run(float* d, int blocks) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(touch<KB>, dim3(blocks), dim3(512), 0, 0, d);
  (void)hipEventRecord(e0);
  const int n = 200;
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(touch<KB>, dim3(blocks), dim3(512), 0, 0, d);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("{\"lds_kib\": %d, \"blocks\": %d, \"us_per_launch\": %.2f}\n", KB, blocks, ms * 1e3f / n);
}

int main() {
  float* d;
  if (hipMalloc(&d, 4096 * sizeof(float)) != hipSuccess) return 1;
  for (int blocks : {1, 256, 1024}) {
    run<16>(d, blocks);
    run<64>(d, blocks);
    run<65>(d, blocks);
    run<96>(d, blocks);
    run<128>(d, blocks);
    run<160>(d, blocks);
  }
  (void)hipFree(d);
  return 0;
}
