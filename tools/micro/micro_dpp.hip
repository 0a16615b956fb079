// Micro-benchmark (diagnostic only): cycles per step of the lazy split-exponent alpha
// recurrence (K=2, normalized every 4th step, as alpha_chain in fwd_bwd_stream.hip) on one wave,
// registers only, by the cross-lane move used for the shifted term:
//   0 DPP wave_shr:1 (the kernel's)  1 DPP row_shr:1 (intra-row, timing only)  2 none (timing only)
//   3 wave_shr, ldexp replaced by a multiply (timing only)  4 wave_shr, 2 independent chains
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "xf_math.h"
using namespace ssnt;

template <int M>
__device__ __forceinline__ int shft(int x) {
  if constexpr (M == 1) return __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
  else if constexpr (M == 2) return x;
  else return __builtin_amdgcn_update_dpp(0, x, 0x138, 0xf, 0xf, true);
}
template <int M>
__device__ __forceinline__ float shft(float x) { return __builtin_bit_cast(float, shft<M>(__builtin_bit_cast(int, x))); }
template <int M>
__device__ __forceinline__ float scl(float m, int e) {
  if constexpr (M == 3) return m * (float)e;
  else return __builtin_ldexpf(m, e);
}

template <int M, bool NORM>
__device__ __forceinline__ void step(float* am, int* ae, const float* Em, const int* Ee, const float* Lm, const int* Le) {
  float hm[2], sm[2];
  int he[2], se[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    hm[j] = (j == 0 ? shft<M>(am[1]) : am[0]) * Lm[j];
    he[j] = (j == 0 ? shft<M>(ae[1]) : ae[0]) + Le[j];
    sm[j] = am[j] * Em[j];
    se[j] = ae[j] + Ee[j];
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int em = max(max(se[j], he[j]), XF_EZERO);
    const float s = scl<M>(sm[j], se[j] - em) + scl<M>(hm[j], he[j] - em);
    if (NORM) {
      const xf r = xf_norm(s, em);
      am[j] = r.m;
      ae[j] = r.e;
    } else {
      am[j] = s;
      ae[j] = em;
    }
  }
}

template <int M>
__global__ __launch_bounds__(64) void k(float* out, unsigned long long* cyc, int steps) {
  const int lane = threadIdx.x;
  float am[2] = {0.6f, 0.7f}, bm[2] = {0.5f, 0.55f};
  int ae[2] = {-3, -4}, be[2] = {-2, -5};
  const float Em[2] = {0.8f + 0.001f * lane, 0.9f}, Lm[2] = {0.75f, 0.85f};
  const int Ee[2] = {-1, -2}, Le[2] = {-1, -3};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < steps; s += 4) {
    step<M, false>(am, ae, Em, Ee, Lm, Le);
    if (M == 4) step<0, false>(bm, be, Em, Ee, Lm, Le);
    step<M, false>(am, ae, Em, Ee, Lm, Le);
    if (M == 4) step<0, false>(bm, be, Em, Ee, Lm, Le);
    step<M, false>(am, ae, Em, Ee, Lm, Le);
    if (M == 4) step<0, false>(bm, be, Em, Ee, Lm, Le);
    step<M, true>(am, ae, Em, Ee, Lm, Le);
    if (M == 4) step<0, true>(bm, be, Em, Ee, Lm, Le);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = am[0] + am[1] + ae[0] + ae[1] + bm[0] + be[1];
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out;
  unsigned long long* cyc;
  if (hipMalloc(&out, 256 * 64 * 4) != hipSuccess || hipMalloc(&cyc, 256 * 8) != hipSuccess) return 1;
  unsigned long long h[256];
  const int steps = 4000;
#define RUN(M)                                                                       \
  {                                                                                  \
    for (int rep = 0; rep < 2; ++rep) {                                              \
      hipLaunchKernelGGL(k<M>, dim3(256), dim3(64), 0, 0, out, cyc, steps);          \
      if (hipDeviceSynchronize() != hipSuccess) return 2;                            \
    }                                                                                \
    if (hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 3;  \
    printf("mode %d: %.1f cycles/step\n", M, (double)h[7] / steps);                  \
  }
  RUN(0) RUN(1) RUN(2) RUN(3) RUN(4)
  return 0;
}
