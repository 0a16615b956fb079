// Micro-benchmark (diagnostic only): cycles per step of the split-exponent alpha recurrence
// on one wave, K=2, with optional LDS slot read / row write / release store per step.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "xf_math.h"
using namespace ssnt;

__device__ __forceinline__ float shr1f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ int shr1i(int x) { return __builtin_amdgcn_update_dpp(XF_EZERO, x, 0x138, 0xf, 0xf, false); }

template <int MODE>  // 0 regs only, 1 + LDS read, 2 + LDS write, 3 + release store
__global__ __launch_bounds__(64) void k(float* out, unsigned long long* cyc, int steps) {
  __shared__ __attribute__((aligned(16))) float ring[8][64 * 8];
  __shared__ __attribute__((aligned(16))) float rows[64 * 4];
  __shared__ int flag;
  const int lane = threadIdx.x;
  for (int i = lane; i < 8 * 64 * 8; i += 64) (&ring[0][0])[i] = 0.7f + 0.001f * (i & 31);
  __syncthreads();
  float am[2] = {0.6f, 0.7f}; int ae[2] = {-3, -4};
  float Em[2] = {0.8f, 0.9f}, Sm[2] = {0.75f, 0.85f}; int Ee[2] = {-1, -2}, Se[2] = {-1, -3};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < steps; ++s) {
    if (MODE >= 1) {
      const float4 v = *reinterpret_cast<const float4*>(&ring[s & 7][lane * 8]);
      const float4 w = *reinterpret_cast<const float4*>(&ring[s & 7][lane * 8 + 4]);
      Em[0] = v.x; Ee[0] = (int)v.y; Sm[0] = v.z; Se[0] = (int)v.w;
      Em[1] = w.x; Ee[1] = (int)w.y; Sm[1] = w.z; Se[1] = (int)w.w;
    }
    float stm[2], shm[2]; int ste[2], she[2];
    for (int j = 0; j < 2; ++j) { stm[j] = am[j] * Em[j]; ste[j] = ae[j] + Ee[j]; shm[j] = am[j] * Sm[j]; she[j] = ae[j] + Se[j]; }
    const float lm = shr1f(shm[1]); const int le = shr1i(she[1]);
    for (int j = 0; j < 2; ++j) {
      const float hm = j == 0 ? lm : shm[0]; const int he = j == 0 ? le : she[0];
      const int em = max(ste[j], he);
      const float sum = xldexp(stm[j], ste[j] - em) + xldexp(hm, he - em);
      const xf r = xf_norm(sum, em);
      am[j] = r.m; ae[j] = r.e;
    }
    if (MODE >= 2) *reinterpret_cast<float4*>(&rows[lane * 4]) = make_float4(am[0], (float)ae[0], am[1], (float)ae[1]);
    if (MODE >= 3) if (lane == 0) __hip_atomic_store(&flag, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = am[0] + am[1] + ae[0] + ae[1] + rows[lane];
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out; unsigned long long* cyc;
  hipMalloc(&out, 256 * 64 * 4); hipMalloc(&cyc, 256 * 8);
  unsigned long long h[256];
  const int steps = 2000;
  #define RUN(M) { hipLaunchKernelGGL(k<M>, dim3(256), dim3(64), 0, 0, out, cyc, steps); hipDeviceSynchronize(); \
    hipLaunchKernelGGL(k<M>, dim3(256), dim3(64), 0, 0, out, cyc, steps); hipDeviceSynchronize(); \
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost); printf("mode %d: %.1f cycles/step\n", M, (double)h[7] / steps); }
  RUN(0) RUN(1) RUN(2) RUN(3)
  return 0;
}
