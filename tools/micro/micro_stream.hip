// Micro-benchmark (diagnostic only): the headline kernel's HBM read pattern without any
// compute -- one 1024-thread workgroup per CU (256), NL loader waves per workgroup each
// streaming its share of 2 x 200 rows of 640 B (40 lanes x 16 B) with D loads in flight
// (register ring), as the converters do. Reports the time and the achieved read bandwidth:
// whether per-CU memory-level parallelism bounds the converters.
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int B = 256, T = 200, U = 80;

template <int D, int NL, int LANES>
__global__ __launch_bounds__(1024) void k(const float4* lt, float* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= NL) return;
  const int b = blockIdx.x;
  const float4* base = lt + (size_t)b * T * U * 2 / 4;  // (T, U, 2) floats per utterance
  const int rowq = U * 2 / 4;                            // float4 per row (40)
  // loader w handles rows w, w+NL, ... of both directions (2T row reads)
  const int n = (2 * T - wave + NL - 1) / NL;
  auto row_of = [&](int k) { const int r = wave + NL * k; return r < T ? r : 2 * T - 1 - r; };
  float4 ring[D];
  const int l = lane < LANES ? lane : 0;
#pragma unroll
  for (int i = 0; i < D; ++i) ring[i] = base[(size_t)row_of(i < n ? i : 0) * rowq + (l % rowq)];
  float acc = 0.0f;
  for (int k0 = 0; k0 < n; k0 += D) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int k = k0 + i;
      if (k < n) acc += ring[i].x + ring[i].w;
      const int kn = k + D < n ? k + D : 0;
      ring[i] = base[(size_t)row_of(kn) * rowq + (l % rowq)];
    }
  }
  if (acc == 12345.0f) out[b] = acc;
}

template <int D, int NL, int LANES>
void run(const float4* lt, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k<D, NL, LANES>), dim3(B), dim3(1024), 0, 0, lt, out);
  hipEventRecord(e0);
  const int it = 20;
  for (int w = 0; w < it; ++w) hipLaunchKernelGGL((k<D, NL, LANES>), dim3(B), dim3(1024), 0, 0, lt, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / it;
  const double bytes = (double)B * 2 * T * 640;  // row reads (both directions)
  printf("D=%2d loaders=%2d lanes=%d: %7.2f us  %6.2f TB/s (row reads)\n", D, NL, LANES, us, bytes / us / 1e6);
}

int main() {
  float4* lt;
  float* out;
  hipMalloc(&lt, (size_t)B * T * U * 2 * 4);
  hipMalloc(&out, B * 4);
  hipMemset(lt, 0, (size_t)B * T * U * 2 * 4);
  run<8, 6, 40>(lt, out);
  run<16, 6, 40>(lt, out);
  run<4, 6, 40>(lt, out);
  run<8, 12, 40>(lt, out);
  run<8, 16, 40>(lt, out);
  run<8, 2, 40>(lt, out);
  run<8, 6, 64>(lt, out);
  return 0;
}
