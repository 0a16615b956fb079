// Micro-benchmark (diagnostic only): cycles per alpha-chain step of the streaming fwd-bwd
// kernel, K=2, U=80, with the kernel's LDS traffic (prefetched slot reads, row store, counter
// store), optionally beside co-resident waves that (1) spin on an LDS counter with s_sleep,
// (2) run dense VALU, (3) stream LDS reads+writes.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "xf_math.h"
using namespace ssnt;
constexpr int K = 2, U = 80, S = 200, R = 8;

__device__ __forceinline__ float shr_z(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ int shr_z(int x) { return __builtin_amdgcn_update_dpp(0, x, 0x138, 0xf, 0xf, true); }

template <int MODE, int NOTHER>
__global__ __launch_bounds__(64 * (1 + NOTHER)) void k(float* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) float ring[R][U * 4];
  __shared__ __attribute__((aligned(16))) float rows[S][U * 2];
  __shared__ int ctr[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < R * U * 4; i += blockDim.x) (&ring[0][0])[i] = (i & 1) ? __builtin_bit_cast(float, -1 - (i & 3)) : 0.7f + 0.001f * (i & 31);
  if (threadIdx.x < 4) ctr[threadIdx.x] = 0;
  __syncthreads();
  const int p0 = K * lane;
  const int pr = p0 < U ? p0 : U - K;
  if (wave == 0) {
    __builtin_amdgcn_s_setprio(3);
    float am[K] = {0.6f, 0.7f}; int ae[K] = {-3, -4};
    float Em[K], Lm[K]; int Ee[K], Le[K];
    auto rd = [&](int j, float* em, int* ee, float* lm, int* le) {
      const float4 v = *reinterpret_cast<const float4*>(&ring[j][4 * pr]);
      const float4 w = *reinterpret_cast<const float4*>(&ring[j][4 * pr + 4]);
      em[0] = v.x; ee[0] = __builtin_bit_cast(int, v.y); lm[0] = v.z; le[0] = __builtin_bit_cast(int, v.w);
      em[1] = w.x; ee[1] = __builtin_bit_cast(int, w.y); lm[1] = w.z; le[1] = __builtin_bit_cast(int, w.w);
    };
    rd(0, Em, Ee, Lm, Le);
    float E2m[K], L2m[K]; int E2e[K], L2e[K];
    rd(1, E2m, E2e, L2m, L2e);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int base = 0; base < S; base += R) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        float En[K], Ln[K]; int Een[K], Len[K];
        if (MODE >= 1 && MODE != 10) rd((i + 1) % R, En, Een, Ln, Len);
        if (MODE == 10) { asm volatile("" ::: "memory"); rd((i + 2) % R, En, Een, Ln, Len); }
        float hm[K]; int he[K];
        for (int j = 0; j < K; ++j) {
          hm[j] = ((j == 0) ? shr_z(am[K - 1]) : am[j - 1]) * Lm[j];
          he[j] = ((j == 0) ? shr_z(ae[K - 1]) : ae[j - 1]) + Le[j];
        }
        for (int j = 0; j < K; ++j) {
          const float sm = am[j] * Em[j]; const int se = ae[j] + Ee[j];
          const int em = max(se, he[j]);
          const float s = __builtin_amdgcn_ldexpf(sm, se - em) + __builtin_amdgcn_ldexpf(hm[j], he[j] - em);
          am[j] = __builtin_amdgcn_frexp_mantf(s);
          ae[j] = max(em + __builtin_amdgcn_frexp_expf(s), XF_EZERO);
        }
        if (MODE >= 2 && MODE != 9) *reinterpret_cast<float4*>(&rows[base + i][2 * (p0 < U ? p0 : 0)]) = make_float4(am[0], __builtin_bit_cast(float, ae[0]), am[1], __builtin_bit_cast(float, ae[1]));
        if (MODE == 3 || MODE == 10 || (MODE >= 4 && MODE <= 6)) { asm volatile("" ::: "memory"); __hip_atomic_store(&ctr[0], base + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
        if (MODE == 7) { asm volatile("" ::: "memory"); if (lane == 0) __hip_atomic_store(&ctr[0], base + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
        if (MODE == 8 && (i & 1)) { asm volatile("" ::: "memory"); if (lane == 0) __hip_atomic_store(&ctr[0], base + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
        if (MODE >= 1 && MODE != 10) for (int j = 0; j < K; ++j) { Em[j] = En[j]; Ee[j] = Een[j]; Lm[j] = Ln[j]; Le[j] = Len[j]; }
        if (MODE == 10) for (int j = 0; j < K; ++j) { Em[j] = E2m[j]; Ee[j] = E2e[j]; Lm[j] = L2m[j]; Le[j] = L2e[j]; E2m[j] = En[j]; E2e[j] = Een[j]; L2m[j] = Ln[j]; L2e[j] = Len[j]; }
      }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __hip_atomic_store(&ctr[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    out[blockIdx.x * 64 + lane] = am[0] + am[1] + ae[0] + ae[1];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
  } else {
    // co-resident waves until the chain is done
    float a = lane * 0.001f, b = 1.0001f;
    int n = 0;
    while (__hip_atomic_load(&ctr[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0 && ++n < (1 << 20)) {
      if (NOTHER > 0 && MODE >= 4 && (MODE == 4)) {
        __builtin_amdgcn_s_sleep(1);
      } else if (MODE == 5) {
        for (int q = 0; q < 32; ++q) a = a * b + 0.5f;
      } else if (MODE == 6) {
        const float4 v = *reinterpret_cast<const float4*>(&ring[n & 7][4 * pr]);
        *reinterpret_cast<float4*>(&ring[(n + 4) & 7][4 * pr]) = v;
      } else {
        __builtin_amdgcn_s_sleep(1);
      }
    }
    out[(blockIdx.x + 256) * 64 + threadIdx.x] = a;
  }
}

int main() {
  float* out; unsigned long long* cyc;
  (void)hipMalloc(&out, 4096 * 64 * 4 * 4); (void)hipMalloc(&cyc, 256 * 8);
  unsigned long long h[256];
#define RUN(M, N, name) { for (int w = 0; w < 2; ++w) { hipLaunchKernelGGL((k<M, N>), dim3(256), dim3(64 * (1 + N)), 0, 0, out, cyc); (void)hipDeviceSynchronize(); } \
    (void)hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost); unsigned long long s = 0; for (int i = 0; i < 256; ++i) s += h[i]; \
    printf("%-58s %.1f cycles/step\n", name, (double)s / 256 / S); fflush(stdout); }
  RUN(0, 0, "regs only (stale factors)")
  RUN(1, 0, "+ prefetched slot reads")
  RUN(2, 0, "+ row store")
  RUN(3, 0, "+ counter store")
  RUN(4, 9, "+ 9 co-resident waves spinning with s_sleep")
  RUN(5, 9, "+ 9 co-resident waves dense VALU")
  RUN(6, 9, "+ 9 co-resident waves LDS read/write")
  RUN(5, 3, "+ 3 co-resident waves dense VALU")
  RUN(7, 0, "slot reads + row store + lane-0 counter store")
  RUN(8, 0, "slot reads + row store + lane-0 counter store every 2nd step")
  RUN(10, 0, "reads 2 rows ahead + row store + counter store")
  RUN(10, 9, "reads 2 ahead + row store + ctr + 9 waves spinning")
  RUN(10, 15, "reads 2 ahead + row store + ctr + 15 waves spinning")
  RUN(5, 15, "+ 15 co-resident waves dense VALU")
  RUN(6, 15, "+ 15 co-resident waves LDS read/write")
  return 0;
}
