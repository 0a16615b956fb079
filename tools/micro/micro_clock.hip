// Micro-benchmark (diagnostic only): shader clock vs wall clock. One wave per CU runs a dependent
// VALU loop; s_memtime (shader cycles) and s_memrealtime (fixed 100 MHz) are read around it, and
// the host times the launch with HIP events. Prints MHz = memtime ticks / realtime us.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(64) void k(float* out, unsigned long long* t, int n) {
  float a = threadIdx.x * 0.001f;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; ++i) a = __builtin_fmaf(a, 1.0000001f, 0.5f);
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 64 + threadIdx.x] = a;
  if (threadIdx.x == 0) { t[2 * blockIdx.x] = c1 - c0; t[2 * blockIdx.x + 1] = r1 - r0; }
}

int main() {
  float* out; unsigned long long* t;
  (void)hipMalloc(&out, 256 * 64 * 4); (void)hipMalloc(&t, 256 * 16);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (int n : {100000, 1000000}) {
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k, dim3(256), dim3(64), 0, 0, out, t, n);
      (void)hipEventRecord(e1);
      (void)hipDeviceSynchronize();
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      unsigned long long h[512]; (void)hipMemcpy(h, t, sizeof h, hipMemcpyDeviceToHost);
      printf("n=%d: memtime %llu ticks, realtime %llu (100MHz) -> %.0f MHz; wall %.3f ms -> %.0f MHz by wall; %.2f ticks/fma\n",
             n, h[0], h[1], h[0] / (h[1] / 100.0), ms, h[0] / (ms * 1e3), (double)h[0] / n);
    }
  }
  return 0;
}
