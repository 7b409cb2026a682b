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

constexpr int N = 4096;

template <int KIND>
__global__ void __launch_bounds__(256) loop(float* out, long long* cyc, int scale) {
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
  for (int k = 0; k < 3; ++k) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      // 256 blocks x 256 threads = one wave per SIMD on every CU
      if (k == 0) hipLaunchKernelGGL(loop<0>, dim3(256), dim3(256), 0, 0, out, cyc, 127);
      if (k == 1) hipLaunchKernelGGL(loop<1>, dim3(256), dim3(256), 0, 0, out, cyc, 127);
      if (k == 2) hipLaunchKernelGGL(loop<2>, dim3(256), dim3(256), 0, 0, out, cyc, 127);
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
      if (rep == 1)
        printf("{\"mfma\": \"%s\", \"cycles_per_mfma\": %.2f, \"wall_ms\": %.3f, \"tflops\": %.1f}\n", names[k], per, ms,
               tf);
    }
  }
  return 0;
}
