// Micro-benchmark (diagnostic only): issue cost of the VALU / DPP / LDS instructions the
// fwd-bwd recurrence is made of, on one wave64 per CU. Cycles per instruction (s_memtime).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int MODE>
__global__ __launch_bounds__(64) void k(float* out, unsigned long long* cyc, int iters) {
  float a = threadIdx.x * 0.001f + 1.0f, b = 1.0001f, c = 0.999f, d = 0.5f;
  int ia = threadIdx.x, ib = 3;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if constexpr (MODE == 0) {  // dependent v_mul_f32 chain
      asm volatile(REP64("v_mul_f32 %0, %0, %1\n") : "+v"(a) : "v"(b));
    } else if constexpr (MODE == 1) {  // 2 independent v_mul chains interleaved
      asm volatile(REP64("v_mul_f32 %0, %0, %2\nv_mul_f32 %1, %1, %2\n") : "+v"(a), "+v"(c) : "v"(b));
    } else if constexpr (MODE == 2) {  // dependent v_ldexp
      asm volatile(REP64("v_ldexp_f32 %0, %0, %1\n") : "+v"(a) : "v"(ib));
    } else if constexpr (MODE == 3) {  // dependent frexp_mant
      asm volatile(REP64("v_frexp_mant_f32 %0, %0\n") : "+v"(a));
    } else if constexpr (MODE == 4) {  // dependent DPP wave_shr:1 (+ s_nop)
      asm volatile(REP64("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\ns_nop 1\n") : "+v"(a));
    } else if constexpr (MODE == 5) {  // DPP row_shr:1 dependent
      asm volatile(REP64("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\ns_nop 1\n") : "+v"(a));
    } else if constexpr (MODE == 6) {  // v_pk_mul_f32 dependent
      asm volatile(REP64("v_pk_mul_f32 %0, %0, %1\n") : "+v"(*(double*)&a) : "v"(*(double*)&c));
    } else if constexpr (MODE == 7) {  // v_add_u32 dependent
      asm volatile(REP64("v_add_u32 %0, %0, %1\n") : "+v"(ia) : "v"(ib));
    } else if constexpr (MODE == 8) {  // 4 independent chains
      asm volatile(REP64("v_mul_f32 %0, %0, %4\nv_mul_f32 %1, %1, %4\nv_mul_f32 %2, %2, %4\nv_mul_f32 %3, %3, %4\n")
                   : "+v"(a), "+v"(c), "+v"(d), "+v"(*(float*)&ia) : "v"(b));
    } else if constexpr (MODE == 9) {  // s_nop 0 only (issue of a SALU-ish op)
      asm volatile(REP64("s_add_u32 %0, %0, 1\n") : "+s"(ib) : : "scc");
    } else if constexpr (MODE == 10) {  // v_cndmask dependent (vcc)
      asm volatile("v_cmp_gt_f32 vcc, %1, 0\n" REP64("v_cndmask_b32 %0, %1, %0, vcc\n") : "+v"(a) : "v"(b) : "vcc");
    } else if constexpr (MODE == 11) {  // dependent v_max_i32
      asm volatile(REP64("v_max_i32 %0, %0, %1\n") : "+v"(ia) : "v"(ib));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = a + c + d + ia + ib;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 64 * 4);
  hipMalloc(&cyc, 256 * 8);
  unsigned long long h[256];
  const int iters = 1000;
  const char* names[] = {"v_mul dep", "v_mul x2 indep (per instr)", "v_ldexp dep", "v_frexp_mant dep",
                         "dpp wave_shr dep (+s_nop1)", "dpp row_shr dep (+s_nop1)", "v_pk_mul dep",
                         "v_add_u32 dep", "v_mul x4 indep (per instr)", "s_add_u32 dep",
                         "v_cndmask dep", "v_max_i32 dep"};
  const int per[] = {64, 128, 64, 64, 64, 64, 64, 64, 256, 64, 64, 64};
#define RUN(M)                                                                            \
  {                                                                                       \
    for (int w = 0; w < 2; ++w) {                                                         \
      hipLaunchKernelGGL(k<M>, dim3(256), dim3(64), 0, 0, out, cyc, iters);               \
      hipDeviceSynchronize();                                                             \
    }                                                                                     \
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);                                   \
    printf("%-30s %.2f cycles/instr\n", names[M], (double)h[7] / iters / per[M]);        \
    fflush(stdout);                                                                       \
  }
  RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7) RUN(8) RUN(9) RUN(10) RUN(11)
  return 0;
}
