// Dependent-access latency on an idle MI355X, one wave (lane 0 active): a chain of N accesses
// where each address depends on the previous result, over a 1 GiB buffer (random lines, HBM
// misses) or a 64 KiB one (cache hits): plain loads, returning atomicCAS, returning atomicAdd,
// and loads after an agent-scope acquire.  The level kernels of the SHORTEST chain and MARK are
// chains of such accesses per tile.
// Build: hipcc --offload-arch=gfx950 -O2 tools/latency_probe.hip -o tools/latency_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_chase(uint32_t* buf, uint64_t mask, int n, int mode, unsigned long long* out) {
  if (threadIdx.x != 0) return;
  uint32_t i = 0;
  const unsigned long long t0 = wall_clock64();
  for (int k = 0; k < n; ++k) {
    uint32_t v;
    if (mode == 0) v = buf[i];
    else if (mode == 1) v = atomicCAS(buf + i, 0xFFFFFFFFu, 0xFFFFFFFFu);   // (never matches: the value stays)
    else v = atomicAdd(buf + i, 0u);
    i = (uint32_t)((v * 2654435761ull + k) & mask) & ~31u;   // next line depends on the value read
  }
  const unsigned long long t1 = wall_clock64();
  out[0] = t1 - t0;
  out[1] = i;
}

__global__ void k_fill(uint32_t* buf, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    buf[i] = (uint32_t)(i * 0x9E3779B1u);
}

int main() {
  const uint64_t big = 1ull << 28;   // words (1 GiB)
  uint32_t* buf;
  unsigned long long *out, h[2];
  CK(hipMalloc((void**)&buf, big * 4));
  CK(hipMalloc((void**)&out, 16));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, buf, big);
  CK(hipDeviceSynchronize());
  printf("{\"probe\": \"dependent access latency, one lane, idle GPU\", \"rows\": [\n");
  bool first = true;
  const char* names[3] = {"load", "atomicCAS (returning)", "atomicAdd (returning)"};
  for (uint64_t words : {(uint64_t)1 << 14, big}) {
    for (int mode = 0; mode < 3; ++mode) {
      const int n = 2000;
      hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, buf, words - 1, 200, mode, out);   // warm
      hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, buf, words - 1, n, mode, out);
      CK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
      printf("%s {\"buffer_bytes\": %llu, \"op\": \"%s\", \"ns_per_dependent_op\": %.1f}", first ? "" : ",\n",
             (unsigned long long)(words * 4), names[mode], h[0] * 10.0 / n);   // wall clock: 100 MHz
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}
