// Small device->host result copies: hipMemcpyAsync into pinned memory vs a kernel storing into
// mapped pinned memory, round trip (enqueue -> host sees the data) per size.
// Build: hipcc --offload-arch=gfx950 -O2 tools/d2h_probe.hip -o gpurun_out/d2h_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_touch(unsigned long long* d, size_t n) {
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) d[i] += 1;
}
__global__ void k_store(const unsigned long long* __restrict__ d, unsigned long long* h, size_t n) {
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) h[i] = d[i];
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t maxb = 1 << 20;
  unsigned long long *d, *h, *hc;
  CK(hipMalloc((void**)&d, maxb));
  CK(hipMemset(d, 0, maxb));
  CK(hipHostMalloc((void**)&h, maxb, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&hc, maxb, hipHostMallocMapped | hipHostMallocCoherent));
  unsigned long long* hcd = nullptr;
  CK(hipHostGetDevicePointer((void**)&hcd, hc, 0));
  const int reps = 400;
  printf("{\"probe\": \"small D2H result copies\", \"rows\": [\n");
  bool first = true;
  for (size_t bytes : {64ul, 2048ul, 8192ul, 10240ul, 12288ul, 14336ul, 16384ul, 17408ul, 65536ul, 262144ul}) {
    const size_t n = bytes / 8;
    for (int mode = 0; mode < 3; ++mode) {
      std::vector<double> us;
      for (int r = 0; r < reps; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_touch, dim3(1), dim3(256), 0, s, d, n);
        if (mode == 0) CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
        else if (mode == 1) hipLaunchKernelGGL(k_store, dim3(1), dim3(256), 0, s, d, hcd, n);
        // mode 2: the kernel alone (the floor)
        CK(hipStreamSynchronize(s));
        auto t1 = std::chrono::steady_clock::now();
        if (r >= 20) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      }
      std::sort(us.begin(), us.end());
      printf("%s {\"bytes\": %zu, \"mode\": \"%s\", \"p50_us\": %.2f, \"p90_us\": %.2f}", first ? "" : ",\n", bytes,
             mode == 0 ? "touch+hipMemcpyAsync(pinned)" : mode == 1 ? "touch+kernel store to mapped" : "touch only",
             us[us.size() / 2], us[us.size() * 9 / 10]);
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}
