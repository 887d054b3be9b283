// Same-address 64-bit atomicAdd throughput on MI355X: one returning atomic per wave from W waves,
// all on one counter, or spread over K counters (wave w -> counter (block % K), one per 256 B),
// timed with events.  The SHORTEST chain's appends are exactly this (one per wave tile).
// Build: hipcc --offload-arch=gfx950 -O2 tools/atomic_probe.hip -o tools/atomic_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_atomic(unsigned long long* ctr, int k, int reps, unsigned long long* sink) {
  const int lane = threadIdx.x & 63;
  unsigned long long* c = ctr + (size_t)(blockIdx.x % k) * 32;   // 256 B apart
  unsigned long long acc = 0;
  for (int r = 0; r < reps; ++r) {
    unsigned long long old = 0;
    if (lane == 0) old = atomicAdd(c, 1ull);
    acc += __shfl(old, 0, 64);   // (returning: the wave waits for the value, as an append does)
  }
  if (lane == 0 && acc == 0xFFFFFFFFFFFFFFFFull) *sink = acc;
}

int main() {
  unsigned long long *ctr, *sink;
  CK(hipMalloc((void**)&ctr, 4096 * 256));
  CK(hipMalloc((void**)&sink, 8));
  CK(hipMemset(ctr, 0, 4096 * 256));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  printf("{\"probe\": \"same-address returning atomicAdd, one per wave\", \"rows\": [\n");
  bool first = true;
  for (int blocks : {128, 512, 2048}) {
    for (int k : {1, 8, 64}) {
      for (int reps : {1, 4}) {
        std::vector<float> ms;
        for (int it = 0; it < 12; ++it) {
          CK(hipEventRecord(a, 0));
          hipLaunchKernelGGL(k_atomic, dim3(blocks), dim3(256), 0, 0, ctr, k, reps, sink);
          CK(hipEventRecord(b, 0));
          CK(hipEventSynchronize(b));
          float t = 0;
          CK(hipEventElapsedTime(&t, a, b));
          if (it >= 2) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double us = ms[ms.size() / 2] * 1e3, n = (double)blocks * 4 * reps;
        printf("%s {\"workgroups\": %d, \"waves\": %d, \"counters\": %d, \"atomics_per_wave\": %d, \"us\": %.2f, \"ns_per_atomic\": %.2f}",
               first ? "" : ",\n", blocks, blocks * 4, k, reps, us, us * 1e3 / n);
        first = false;
      }
    }
  }
  // the floor: the same launch with no atomics
  printf("\n]}\n");
  return 0;
}
