// Host wake-up latency on an idle MI355X: how soon after a query's last kernel the host can
// read its result.  (a) the engine's wait today: an event behind the last kernel, polled with
// hipEventQuery; (b) the last kernel stores a sequence number into mapped coherent host memory
// after a system-scope release, and the host polls that word.  Both for one small kernel and
// for a chain of four (the GO query's MARK, MARK, FINAL, q_out).  p50 / p90 of 2000 runs each.
// Build: hipcc --offload-arch=gfx950 -O2 tools/wake_probe.hip -o tools/wake_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_work(uint32_t* buf, int n) {   // a little dependent work, like a tiny step
  uint32_t v = buf[threadIdx.x];
  for (int k = 0; k < n; ++k) v = v * 2654435761u + k;
  buf[threadIdx.x] = v;
}

__global__ void k_tail(uint32_t* buf, unsigned long long* flag, unsigned long long seq) {
  buf[threadIdx.x] += 1;
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint32_t* buf;
  CK(hipMalloc((void**)&buf, 4096));
  CK(hipMemset(buf, 0, 4096));
  unsigned long long* h_flag;
  CK(hipHostMalloc((void**)&h_flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  unsigned long long* d_flag;
  CK(hipHostGetDevicePointer((void**)&d_flag, h_flag, 0));
  *h_flag = 0;
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  unsigned long long seq = 0;
  for (int chain : {1, 4}) {
    for (int mode = 0; mode < 2; ++mode) {
      std::vector<double> t;
      for (int it = 0; it < 2200; ++it) {
        ++seq;
        const double t0 = now_us();
        for (int k = 0; k + 1 < chain; ++k) hipLaunchKernelGGL(k_work, dim3(1), dim3(256), 0, s, buf, 64);
        hipLaunchKernelGGL(k_tail, dim3(1), dim3(256), 0, s, buf, d_flag, seq);
        if (mode == 0) {
          CK(hipEventRecord(ev, s));
          hipError_t e;
          while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
          }
          CK(e);
        } else {
          while (__atomic_load_n(h_flag, __ATOMIC_ACQUIRE) != seq) {
          }
        }
        const double t1 = now_us();
        CK(hipStreamSynchronize(s));
        if (it >= 200) t.push_back(t1 - t0);
      }
      std::sort(t.begin(), t.end());
      printf("chain %d  %-28s p50 %6.2f us  p90 %6.2f us\n", chain, mode ? "host polls the mapped flag" : "hipEventQuery spin",
             t[t.size() / 2], t[t.size() * 9 / 10]);
    }
  }
  return 0;
}
