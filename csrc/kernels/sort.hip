// K7: score ranking. The reference sorts the gathered CTR list ascending with
// Collections.sort on boxed Floats and in doing so loses which candidate each
// score belongs to (reference DCNClient.java:195). Here one workgroup sorts up
// to 8192 (score, candidate) pairs in LDS with a bitonic network and returns
// both the sorted scores and the permutation; top-k is a prefix of it.
#include "common.h"
#include "launchers.h"

namespace dtfs {
namespace kern {

constexpr int kSortMax = 8192;

__global__ void __launch_bounds__(1024) bitonic_sort_kernel(const float* __restrict__ in, int n, int descending,
                                                            float* __restrict__ out, int64_t* __restrict__ perm,
                                                            int k_out) {
  __shared__ float key[kSortMax];
  __shared__ int idx[kSortMax];
  int p2 = 1;
  while (p2 < n) p2 <<= 1;
  // Always sort ascending on a transformed key (negated for descending), so
  // ties break by candidate index in both modes; padding and NaN rank last.
  for (int i = threadIdx.x; i < p2; i += blockDim.x) {
    float v = i < n ? in[i] : INFINITY;
    if (v != v) v = INFINITY;
    else if (descending && i < n) v = -v;
    key[i] = v;
    idx[i] = i < n ? i : 0x7fffffff;
  }
  __syncthreads();
  for (int size = 2; size <= p2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < p2 / 2; i += blockDim.x) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const float a = key[lo], b = key[hi];
        const int ia = idx[lo], ib = idx[hi];
        // total order: by key, ties by candidate index (stable)
        const bool gt = (a > b) || (a == b && ia > ib);
        if (gt == up) {
          key[lo] = b;
          key[hi] = a;
          idx[lo] = ib;
          idx[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < k_out; i += blockDim.x) {
    const float v = key[i];
    out[i] = (descending && v != INFINITY) ? -v : v;
    if (perm) perm[i] = idx[i];
  }
}

}  // namespace kern

using namespace kern;

int sort_max_elems() { return kSortMax; }

hipError_t launch_sort_scores(const float* in, int n, bool descending, float* out, int64_t* perm, int k_out,
                              hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (n > kSortMax || k_out > n) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bitonic_sort_kernel, dim3(1), dim3(1024), 0, st, in, n, descending ? 1 : 0, out, perm, k_out);
  return hipGetLastError();
}

}  // namespace dtfs
