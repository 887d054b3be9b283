// Large device->host copies (the host-delivered rows path): GB/s of hipMemcpyAsync and of a
// kernel's stores into each kind of host memory, per copy size.
// Build: hipcc --offload-arch=gfx950 -O2 tools/d2h_bw_probe.hip -o tools/d2h_bw_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_store(const uint4* __restrict__ d, uint4* h, size_t n16) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) h[i] = d[i];
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t maxb = 384ull << 20;
  void* d = nullptr;
  CK(hipMalloc(&d, maxb));
  CK(hipMemset(d, 1, maxb));
  struct Kind { const char* name; void* h; };
  std::vector<Kind> kinds;
  void* p = nullptr;
  CK(hipHostMalloc(&p, maxb, hipHostMallocDefault)); kinds.push_back({"hipHostMalloc(Default)", p});
  CK(hipHostMalloc(&p, maxb, hipHostMallocNonCoherent)); kinds.push_back({"hipHostMalloc(NonCoherent)", p});
  CK(hipHostMalloc(&p, maxb, hipHostMallocCoherent | hipHostMallocMapped)); kinds.push_back({"hipHostMalloc(Coherent|Mapped)", p});
  p = aligned_alloc(4096, maxb);
  for (size_t i = 0; i < maxb; i += 4096) static_cast<char*>(p)[i] = 0;
  CK(hipHostRegister(p, maxb, hipHostRegisterDefault)); kinds.push_back({"malloc+hipHostRegister", p});
  printf("{\"probe\": \"large D2H copies into host memory kinds\", \"rows\": [\n");
  bool first = true;
  for (size_t bytes : {1ull << 20, 16ull << 20, 352ull << 20}) {
    for (auto& k : kinds) {
      for (int mode = 0; mode < 2; ++mode) {
        void* hd = nullptr;
        if (mode == 1 && (hipHostGetDevicePointer(&hd, k.h, 0) != hipSuccess || !hd)) continue;
        const int reps = bytes >= (64ull << 20) ? 6 : 30;
        std::vector<double> gbs;
        for (int r = 0; r < reps + 1; ++r) {
          auto t0 = std::chrono::steady_clock::now();
          if (mode == 0) CK(hipMemcpyAsync(k.h, d, bytes, hipMemcpyDeviceToHost, s));
          else hipLaunchKernelGGL(k_store, dim3(2048), dim3(256), 0, s, (const uint4*)d, (uint4*)hd, bytes / 16);
          CK(hipStreamSynchronize(s));
          auto t1 = std::chrono::steady_clock::now();
          if (r) gbs.push_back(bytes / std::chrono::duration<double>(t1 - t0).count() / 1e9);
        }
        std::sort(gbs.begin(), gbs.end());
        printf("%s {\"bytes\": %zu, \"host\": \"%s\", \"mode\": \"%s\", \"median_GBs\": %.2f, \"max_GBs\": %.2f}",
               first ? "" : ",\n", bytes, k.name, mode == 0 ? "hipMemcpyAsync" : "kernel stores", gbs[gbs.size() / 2],
               gbs.back());
        first = false;
        fflush(stdout);
      }
    }
  }
  printf("\n]}\n");
  return 0;
}
