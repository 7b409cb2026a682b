// Probe of the 16x16x128 block-scaled fp8 MFMA operand layout on gfx950:
// which logical K position a (lane, byte) of an operand lands on, and which
// lane's scale byte scales it. A = one e4m3 1.0 at (lane la, byte j), B = all
// ones, scale_b(lane) = 127 + lane: D[row][col] = 2^(index of the scale lane).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(int la, int j, int mode, float* out) {
  const int lane = threadIdx.x;
  i32x8 a, b;
  for (int v = 0; v < 8; ++v) {
    a[v] = 0;
    b[v] = 0x38383838;  // e4m3 1.0
  }
  if (lane == la) a[j / 4] = 0x38 << (8 * (j % 4));
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  if (mode == 0)  // scales on b
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127 + lane);
  else  // scales on a
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127 + lane, 0, 127);
  // C layout: col = lane & 15, row = 4 * (lane >> 4) + r
  for (int r = 0; r < 4; ++r) out[(4 * (lane >> 4) + r) * 16 + (lane & 15)] = c[r];
}

int main() {
  float* d;
  if (hipMalloc(&d, 256 * sizeof(float)) != hipSuccess) return 1;
  float h[256];
  const int las[] = {0, 5, 16, 32, 48};
  const int js[] = {0, 15, 16, 31};
  for (int mode = 0; mode < 2; ++mode)
    for (int la : las)
      for (int j : js) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, la, j, mode, d);
        if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
        // print the nonzero entries as row,col:log2
        printf("{\"mode\": \"%s\", \"la\": %d, \"j\": %d, \"nz\": \"", mode ? "scale_a" : "scale_b", la, j);
        int shown = 0;
        for (int i = 0; i < 256; ++i)
          if (h[i] != 0.f && shown < 6) {
            printf("%s%d,%d:%g", shown ? " " : "", i / 16, i % 16, std::log2(h[i]));
            ++shown;
          }
        int nz = 0;
        for (int i = 0; i < 256; ++i) nz += h[i] != 0.f;
        printf("\", \"count\": %d}\n", nz);
      }
  (void)hipFree(d);
  return 0;
}
