// What a served step's device-side wait on its request copy costs at the
// step boundary, natively (tools/studies/step_gap_study.py measured +9.6 us
// per launch from Python): a ~100 us L2-resident kernel back to back on one
// stream, fed three ways, 200 launches timed with events:
//   plain     nothing between the launches
//   wait_h2d  a 5 MB pinned H2D per launch on a copy stream (ring of 4
//             buffers), the compute stream waits on its event (StepRunner's
//             default, step_runner.cpp h2d_copies)
//   host_fed  the same copies issued ahead by a copier thread; the launching
//             thread polls each copy's event and only then enqueues the kernel
//             (no cross-queue wait packet on the compute queue)
// The kernel reads its copy's buffer (first 64 KiB) so host_fed also shows
// whether a kernel enqueued after a host-observed copy sees the copied bytes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/native/bin/step_gap tools/native/step_gap.hip -lpthread
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

constexpr int kBlocks = 256, kThreads = 256;
constexpr size_t kCopy = 5u << 20, kW = 4u << 20;

// each block sums a 16 KiB slice of a 4 MiB "weight" buffer `reps` times (L2
// traffic like the tower's W stream) plus the first words of its step's copy
__global__ void __launch_bounds__(kThreads) busy(const float4* __restrict__ w, const uint32_t* __restrict__ in,
                                                 float* __restrict__ out, uint32_t* __restrict__ seen, int reps) {
  const int slice = (blockIdx.x * 1024) % int(kW / 16);
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < reps; ++r)
    for (int i = threadIdx.x; i < 1024; i += kThreads) {
      const float4 v = w[slice + ((i + r * 37) & 1023)];
      acc.x += v.x;
      acc.y += v.y * 0.5f;
      acc.z += v.z;
      acc.w += v.w * 0.25f;
    }
  out[blockIdx.x * kThreads + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
  if (blockIdx.x == 0 && threadIdx.x == 0) seen[0] = in[0];
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 200;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 600;
  float4* w;
  float* out;
  uint32_t* seen;
  CK(hipMalloc(&w, kW));
  CK(hipMemset(w, 0, kW));
  CK(hipMalloc(&out, kBlocks * kThreads * 4));
  CK(hipMalloc(&seen, 4 * n));
  std::vector<uint8_t*> dev(4), host(4);
  for (int b = 0; b < 4; ++b) {
    CK(hipMalloc(&dev[b], kCopy));
    CK(hipHostMalloc(&host[b], kCopy, hipHostMallocDefault));
    std::memset(host[b], 0, kCopy);
  }
  hipStream_t comp, copy;
  CK(hipStreamCreateWithFlags(&comp, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&copy, hipStreamNonBlocking));
  std::vector<hipEvent_t> h2d(n), done(n);
  for (int i = 0; i < n; ++i) {
    CK(hipEventCreateWithFlags(&h2d[i], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
  }
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  auto launch = [&](int i) {
    hipLaunchKernelGGL(busy, dim3(kBlocks), dim3(kThreads), 0, comp, w, reinterpret_cast<const uint32_t*>(dev[i & 3]),
                       out, seen + i, reps);
    CK(hipEventRecord(done[i], comp));
  };
  auto issue_copy = [&](int i) {
    uint32_t tag = 0x5eed0000u + uint32_t(i);
    std::memcpy(host[i & 3], &tag, 4);  // the host buffer is free: its previous copy landed
    CK(hipMemcpyAsync(dev[i & 3], host[i & 3], kCopy, hipMemcpyHostToDevice, copy));
    CK(hipEventRecord(h2d[i], copy));
  };
  const char* names[] = {"plain", "wait_h2d", "host_fed"};
  for (int round = 0; round < 3; ++round)
    for (int v = 0; v < 3; ++v) {
      CK(hipDeviceSynchronize());
      CK(hipMemset(seen, 0, 4 * n));
      launch(0);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(t0, comp));
      if (v == 0) {
        for (int i = 0; i < n; ++i) launch(i);
      } else if (v == 1) {
        for (int i = 0; i < n; ++i) {
          if (i >= 4) CK(hipEventSynchronize(done[i - 4]));  // WAR on the ring slot (host buffer + device buffer)
          issue_copy(i);
          CK(hipStreamWaitEvent(comp, h2d[i], 0));
          launch(i);
        }
      } else {
        std::atomic<int> issued{0}, launched{0};
        std::thread copier([&] {
          for (int i = 0; i < n; ++i) {
            if (i >= 4) {
              while (launched.load(std::memory_order_acquire) <= i - 4) std::this_thread::yield();
              CK(hipEventSynchronize(done[i - 4]));
            }
            issue_copy(i);
            issued.store(i + 1, std::memory_order_release);
          }
        });
        for (int i = 0; i < n; ++i) {
          while (issued.load(std::memory_order_acquire) <= i) std::this_thread::yield();
          for (;;) {
            const hipError_t e = hipEventQuery(h2d[i]);
            if (e == hipSuccess) break;
            if (e != hipErrorNotReady) CK(e);
            std::this_thread::yield();
          }
          launch(i);
          launched.store(i + 1, std::memory_order_release);
        }
        copier.join();
      }
      CK(hipEventRecord(t1, comp));
      CK(hipEventSynchronize(t1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, t0, t1));
      int stale = 0;
      if (v > 0) {
        std::vector<uint32_t> s(n);
        CK(hipMemcpy(s.data(), seen, 4 * n, hipMemcpyDeviceToHost));
        for (int i = 0; i < n; ++i) stale += s[i] != 0x5eed0000u + uint32_t(i);
      }
      std::printf("{\"round\": %d, \"variant\": \"%s\", \"us_per_launch\": %.2f, \"stale_reads\": %d}\n", round,
                  names[v], ms * 1e3f / n, stale);
      std::fflush(stdout);
    }
  return 0;
}
