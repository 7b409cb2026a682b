// Cycles per MFMA on one SIMD (one wave per SIMD, 4 independent accumulators,
// operands in registers): bf16 16x16x32 vs plain fp8 16x16x32 vs block-scaled
// MX-fp8 16x16x128 - checks the per-dtype rates the fp8 GEMM design assumes
// (MI355X_MICROARCH.md § Matrix cores). Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef long i64x1;

constexpr int N = 65536;  // ~4 ms per launch: long enough for the clock to settle under load

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

template <int KIND>
__global__ void __launch_bounds__(256) loop(float* out, long long* cyc, int scale, int rnd) {
  f32x4 c0{0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  const int l = threadIdx.x;
  bf16x8 a, b;
  i32x8 x, y;
  long fa = 0x3c003c00 + l, fb = 0x3c003c01 + l;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (l + i));
    b[i] = (__bf16)(0.002f * (l - i));
    x[i] = 0x38383838 + l + i;
    y[i] = 0x30303030 + l - i;
    if (rnd) {  // random operands: every mantissa bit toggles (the DVFS-relevant case)
      const unsigned h0 = hash32(blockIdx.x * 4096u + l * 16u + i), h1 = hash32(h0 + 0x9e3779b9u);
      a[i] = (__bf16)((int(h0 & 0xffff) - 32768) * (1.f / 32768.f));
      b[i] = (__bf16)((int(h1 & 0xffff) - 32768) * (1.f / 32768.f));
      x[i] = int(h0 & 0x77777777u);  // e4m3 bytes without NaN patterns
      y[i] = int(h1 & 0x77777777u);
    }
  }
  if (rnd) {
    fa = (long(hash32(l * 7u + 1)) << 32 | hash32(l * 7u + 2)) & 0x7777777777777777L;
    fb = (long(hash32(l * 7u + 3)) << 32 | hash32(l * 7u + 4)) & 0x7777777777777777L;
  }
  __syncthreads();
  const long long t0 = clock64();
  for (int it = 0; it < N; ++it) {
    if constexpr (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c3, 0, 0, 0);
    } else if constexpr (KIND == 1) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(fa, fb, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(fa, fb, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(fa, fb, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(fa, fb, c3, 0, 0, 0);
    } else {
      c0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(x, y, c0, 0, 0, 0, scale, 0, scale);
      c1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(x, y, c1, 0, 0, 0, scale, 0, scale);
      c2 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(x, y, c2, 0, 0, 0, scale, 0, scale);
      c3 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(x, y, c3, 0, 0, 0, scale, 0, scale);
    }
  }
  const long long t1 = clock64();
  out[blockIdx.x * blockDim.x + l] = c0[0] + c1[1] + c2[2] + c3[3];
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 256 * 256 * sizeof(float));
  hipMalloc(&cyc, 256 * sizeof(long long));
  const char* names[3] = {"bf16 16x16x32", "fp8 16x16x32", "MX-fp8 16x16x128 (scaled)"};
  const double flop[3] = {2.0 * 16 * 16 * 32, 2.0 * 16 * 16 * 32, 2.0 * 16 * 16 * 128};
  for (int rnd = 0; rnd < 2; ++rnd)
  for (int k = 0; k < 3; ++k) {
    for (int rep = 0; rep < 4; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      // 256 blocks x 256 threads = one wave per SIMD on every CU
      if (k == 0) hipLaunchKernelGGL(loop<0>, dim3(256), dim3(256), 0, 0, out, cyc, 127, rnd);
      if (k == 1) hipLaunchKernelGGL(loop<1>, dim3(256), dim3(256), 0, 0, out, cyc, 127, rnd);
      if (k == 2) hipLaunchKernelGGL(loop<2>, dim3(256), dim3(256), 0, 0, out, cyc, 127, rnd);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      long long c[256];
      hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
      double avg = 0;
      for (int i = 0; i < 256; ++i) avg += double(c[i]);
      avg /= 256;
      const double per = avg / (4.0 * N);
      const double tf = flop[k] * 4.0 * N * 1024 / (ms * 1e-3) / 1e12;  // 1024 waves
      if (rep == 3)
        printf("{\"mfma\": \"%s\", \"operands\": \"%s\", \"cycles_per_mfma\": %.2f, \"wall_ms\": %.3f, \"tflops\": %.1f}\n",
               names[k], rnd ? "random" : "structured", per, ms, tf);
    }
  }
  return 0;
}
