// Micro-probe (diagnostic only): which SIMD each wave of a 16-wave workgroup lands on
// (s_getreg HW_ID.SIMD_ID), for the role placement of the streaming fwd-bwd kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ __launch_bounds__(1024) void k(int* out) {
  __shared__ int pad[40 * 1024];  // ~160 KB LDS like the real kernel: one workgroup per CU
  const int wave = threadIdx.x >> 6;
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);  // HW_ID (all 32 bits)
  const unsigned simd = (hw >> 4) & 3;
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + wave] = simd;
  if (threadIdx.x == 0) pad[blockIdx.x & 1023] = (int)hw;
  __syncthreads();
  if (threadIdx.x == 1 && pad[0] == 12345) out[0] = 7;
}
int main() {
  int* d; (void)hipMalloc(&d, 256 * 16 * 4);
  hipLaunchKernelGGL(k, dim3(256), dim3(1024), 0, 0, d);
  (void)hipDeviceSynchronize();
  int h[256 * 16]; (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  int cnt[16][4] = {};
  for (int b = 0; b < 256; ++b) for (int w = 0; w < 16; ++w) cnt[w][h[b * 16 + w] & 3]++;
  for (int w = 0; w < 16; ++w) printf("wave %2d: simd0 %3d simd1 %3d simd2 %3d simd3 %3d\n", w, cnt[w][0], cnt[w][1], cnt[w][2], cnt[w][3]);
  return 0;
}
