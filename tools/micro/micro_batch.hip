// Micro-benchmark (diagnostic only): cycles per alpha-chain step (K=2, U=80, 200 steps) when the
// chain reads its factors from LDS in batches of NB rows one batch ahead (register double
// buffer: no LDS wait inside a batch), optionally storing each row (ds_write_b128), with
// NOTHER co-resident waves that run dense VALU (MODE 1) or sleep (MODE 0). Compare with
// micro_step.hip (one row ahead per step). Build: hipcc --offload-arch=gfx950 -O3 -I csrc.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "xf_math.h"
using namespace ssnt;
constexpr int K = 2, U = 80, S = 200, R = 16;

__device__ __forceinline__ float shr_z(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ int shr_z(int x) { return __builtin_amdgcn_update_dpp(0, x, 0x138, 0xf, 0xf, true); }

struct F {
  float em[K], lm[K];
  int ee[K], le[K];
};

template <int NB, bool STORE, int MODE, int NOTHER, bool LAZY>
__global__ __launch_bounds__(64 * (1 + NOTHER)) void k(float* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) float ring[R][U * 4];
  __shared__ __attribute__((aligned(16))) float rows[S][U * 2];
  __shared__ int ctr[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < R * U * 4; i += blockDim.x)
    (&ring[0][0])[i] = (i & 1) ? __builtin_bit_cast(float, -1 - (i & 3)) : 0.7f + 0.001f * (i & 31);
  if (threadIdx.x < 4) ctr[threadIdx.x] = 0;
  __syncthreads();
  const int p0 = K * lane;
  const int pr = p0 < U ? p0 : U - K;
  if (wave == 0) {
    __builtin_amdgcn_s_setprio(3);
    float am[K] = {0.6f, 0.7f};
    int ae[K] = {-3, -4};
    F buf[2][NB];
    auto rd = [&](int row, F& f) {
      const float4 v = *reinterpret_cast<const float4*>(&ring[row % R][4 * pr]);
      const float4 w = *reinterpret_cast<const float4*>(&ring[row % R][4 * pr + 4]);
      f.em[0] = v.x; f.ee[0] = __builtin_bit_cast(int, v.y); f.lm[0] = v.z; f.le[0] = __builtin_bit_cast(int, v.w);
      f.em[1] = w.x; f.ee[1] = __builtin_bit_cast(int, w.y); f.lm[1] = w.z; f.le[1] = __builtin_bit_cast(int, w.w);
    };
#pragma unroll
    for (int i = 0; i < NB; ++i) rd(i, buf[0][i]);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int base = 0; base < S; base += 2 * NB) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int b0 = base + h * NB;
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < NB; ++i) rd(b0 + NB + i, buf[h ^ 1][i]);  // next batch
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const F& f = buf[h][i];
          float hm[K];
          int he[K];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            hm[j] = ((j == 0) ? shr_z(am[K - 1]) : am[j - 1]) * f.lm[j];
            he[j] = ((j == 0) ? shr_z(ae[K - 1]) : ae[j - 1]) + f.le[j];
          }
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const float sm = am[j] * f.em[j];
            const int se = ae[j] + f.ee[j];
            const int em = max(max(se, he[j]), XF_EZERO);
            const float s = __builtin_amdgcn_ldexpf(sm, se - em) + __builtin_amdgcn_ldexpf(hm[j], he[j] - em);
            if (LAZY && (i % 4) != 3) {
              am[j] = s;
              ae[j] = em;
            } else {
              am[j] = __builtin_amdgcn_frexp_mantf(s);
              ae[j] = em + __builtin_amdgcn_frexp_expf(s);
            }
          }
          if (STORE)
            *reinterpret_cast<float4*>(&rows[(b0 + i) % S][2 * (p0 < U ? p0 : 0)]) =
                make_float4(am[0], __builtin_bit_cast(float, ae[0]), am[1], __builtin_bit_cast(float, ae[1]));
        }
      }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __hip_atomic_store(&ctr[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    out[blockIdx.x * 64 + lane] = am[0] + am[1] + ae[0] + ae[1];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
  } else {
    float a = lane * 0.001f, b = 1.0001f;
    int n = 0;
    while (__hip_atomic_load(&ctr[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0 && ++n < (1 << 20)) {
      if (MODE == 1) {
        for (int q = 0; q < 32; ++q) a = a * b + 0.5f;
      } else {
        __builtin_amdgcn_s_sleep(1);
      }
    }
    out[(blockIdx.x + 256) * 64 + threadIdx.x] = a;
  }
}

int main() {
  float* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 4096 * 64 * 4 * 4);
  (void)hipMalloc(&cyc, 256 * 8);
  unsigned long long h[256];
#define RUN(NB, ST, M, N, LZ, name)                                                              \
  {                                                                                          \
    for (int w = 0; w < 2; ++w) {                                                            \
      hipLaunchKernelGGL((k<NB, ST, M, N, LZ>), dim3(256), dim3(64 * (1 + N)), 0, 0, out, cyc); \
      (void)hipDeviceSynchronize();                                                          \
    }                                                                                        \
    (void)hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);                                \
    unsigned long long s = 0;                                                                \
    for (int i = 0; i < 256; ++i) s += h[i];                                                 \
    printf("NB=%d store=%d lazy=%d %-34s %.1f cycles/step\n", NB, (int)ST, (int)LZ, name, (double)s / 256 / S); \
    fflush(stdout);                                                                          \
  }
  RUN(4, false, 0, 0, false, "alone")
  RUN(4, true, 0, 0, false, "alone")
  RUN(8, false, 0, 0, false, "alone")
  RUN(8, true, 0, 0, false, "alone")
  RUN(8, true, 0, 0, true, "alone")
  RUN(8, true, 0, 15, true, "+15 sleeping")
  RUN(8, true, 1, 3, true, "+3 dense VALU (one per SIMD)")
  RUN(8, true, 1, 7, true, "+7 dense VALU")
  RUN(8, true, 1, 11, true, "+11 dense VALU")
  RUN(8, true, 1, 15, true, "+15 dense VALU")
  RUN(8, false, 1, 15, true, "+15 dense VALU")
  return 0;
}
