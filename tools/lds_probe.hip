// LDS per workgroup on this device: the properties, and a launch with growing dynamic LDS
// (the interpreter's registers are [nregs][256] x 8 B of dynamic LDS; MAX_REGS follows from this).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_lds(long long* out, int n) {
  extern __shared__ long long buf[];
  for (int i = threadIdx.x; i < n; i += blockDim.x) buf[i] = i;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = buf[n - 1];
}

int main() {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
  printf("%s sharedMemPerBlock %zu maxSharedMemoryPerMultiProcessor %zu\n", p.gcnArchName, p.sharedMemPerBlock,
         p.maxSharedMemoryPerMultiProcessor);
  long long* d = nullptr;
  if (hipMalloc(&d, 64 * sizeof(long long)) != hipSuccess) return 1;
  for (int kb : {32, 48, 64, 80, 96, 128, 160}) {
    const size_t bytes = (size_t)kb * 1024;
    (void)hipFuncSetAttribute((const void*)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    hipLaunchKernelGGL(k_lds, dim3(8), dim3(256), bytes, 0, d, (int)(bytes / 8));
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    long long h = -1;
    if (e == hipSuccess) (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("dynamic LDS %3d KB: %s (last word %lld)\n", kb, hipGetErrorString(e), h);
    if (e != hipSuccess) (void)hipGetLastError();
  }
  return 0;
}
