// decode.hip -- beam-search decode steps and alignment utilities for gfx950.
//
// One wave (64 lanes) owns one batch element. A step generates every candidate of every beam
// into LDS, ranks them (stable descending sort on log_prob, generation index as tie-break,
// src/lib.rs:161), drops consecutive duplicates (src/lib.rs:162), optionally injects v2's
// on-diagonal candidate (src/v2.rs:283-308) and pads cyclically (src/lib.rs:163-167). All of it
// is integer / compare work plus one f32 add per candidate, so the result is bit-exact with the
// Rust step (and with oracle/ssnt_oracle.c) by construction.
#include <hip/hip_runtime.h>

#include <atomic>

#include "decode_dev.h"

namespace ssnt {
namespace {

using namespace dec;

__global__ __launch_bounds__(64) void k_decode_step(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int n = a.W * a.C;
  Cand* cand = reinterpret_cast<Cand*>(smem);
  int* order = reinterpret_cast<int*>(cand + n);
  int* kept = order + n;
  BatchView v;
  const size_t bw = (size_t)b * a.W;
  v.h = a.h + bw * a.C;
  v.hist = a.hist + bw;
  v.fin = a.fin + bw;
  v.t = a.t + bw;
  v.u = a.u + bw;
  v.total = a.total ? a.total + bw : nullptr;
  v.I = as_usize(a.input_length ? a.input_length[b] : a.scalar_input_length);
  v.O = as_usize(a.output_length ? a.output_length[b] : 0);
  const size_t o = (size_t)b * a.Wmax;
  const int nk = step_wave(a, v, cand, order, kept, a.Wmax, [&](int i, const Cand& r) {
    a.prediction[o + i] = r.pred;  // src/lib.rs:138-145
    a.log_prob[o + i] = r.lp;
    a.next_t[o + i] = (int)(unsigned)r.nt;
    a.next_u[o + i] = (int)(unsigned)r.nu;
    a.beam_branch[o + i] = r.parent;
    a.next_fin[o + i] = r.fin != 0;
    if (a.next_total) a.next_total[o + i] = r.tot;
  });
  if (nk == 0 && a.status && (threadIdx.x & 63) == 0) atomicOr(a.status, kStatusNoCandidate);
}

// Backtrace along beam_branch (B,T,W) for n_paths (<= 64) final branches per batch element
// (util.rs:20-33 with n_paths = 1 and t history; v2_util.rs:6-36 with n_paths = W). A null
// final_branch means branch 0 (the best slot after the final sort). Rows are staged into LDS
// in chunks (coalesced), then lane k walks path k back through the chunk.
__global__ __launch_bounds__(64) void k_backtrace(int B, int W, int T, int n_paths,
                                                  const int* __restrict__ final_branch,
                                                  const int* __restrict__ beam_branch,
                                                  const int* __restrict__ t_history,
                                                  int* __restrict__ out_branch,
                                                  int* __restrict__ out_t, int chunk, int* status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* sb = reinterpret_cast<int*>(smem);
  int* st = sb + (size_t)chunk * W;
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int* bb = beam_branch + (size_t)b * T * W;
  const int* th = t_history ? t_history + (size_t)b * T * W : nullptr;
  const bool active = lane < n_paths;
  int c = (active && final_branch) ? final_branch[(size_t)b * n_paths + lane] : 0;
  int* ob = out_branch + ((size_t)b * n_paths + lane) * T;
  int* ot = out_t ? out_t + ((size_t)b * n_paths + lane) * T : nullptr;
  bool bad = false;
  for (int hi = T; hi > 0; hi -= chunk) {
    const int lo = max(hi - chunk, 0);
    const int cnt = (hi - lo) * W;
    __syncthreads();
    for (int i = lane; i < cnt; i += 64) {
      sb[i] = bb[(size_t)lo * W + i];
      if (th) st[i] = th[(size_t)lo * W + i];
    }
    __syncthreads();
    if (active) {
      for (int s = hi - 1; s >= lo; --s) {
        if (c < 0 || c >= W) {  // Rust would panic on the out-of-bounds index
          bad = true;
          c = c < 0 ? 0 : W - 1;
        }
        ob[s] = c;
        const int r = (s - lo) * W + c;
        if (ot) ot[s] = st[r];
        c = sb[r];
      }
    }
  }
  if (bad && status) atomicOr(status, kStatusBadIndex);
}

__device__ __forceinline__ int wave_incl_scan_add(int x, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  return x;
}
__device__ __forceinline__ int wave_incl_scan_min(int x, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off);
    if (lane >= off) x = min(x, y);
  }
  return x;
}

// upsample_source_indexes (src/v2_util.rs:39-66): one wave per (b,w) row.
__global__ __launch_bounds__(64) void k_upsample(int rows, int T, int max_u,
                                                 const int* __restrict__ duration,
                                                 const int* __restrict__ output_length,
                                                 int* __restrict__ out, int* status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* cum = reinterpret_cast<int*>(smem);  // inclusive prefix sums (T)
  const int r = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int* d = duration + (size_t)r * T;
  long long carry = 0;
  bool neg = false;
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + lane;
    const int x = t < T ? d[t] : 0;
    neg |= x < 0;
    const int inc = wave_incl_scan_add(x, lane);
    if (t < T) cum[t] = (int)(carry + inc);
    carry += __shfl(inc, 63);
  }
  const bool anyneg = __any(neg);
  const int L = output_length[r];
  if (anyneg || carry != (long long)L) {
    if (lane == 0 && status) atomicOr(status, kStatusDurationMismatch);
    return;
  }
  __syncthreads();
  const int n = min(L, max_u);
  int* o = out + (size_t)r * max_u;
  for (int k = lane; k < n; k += 64) {
    int lo = 0, hi = T;  // first t with cum[t] > k
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cum[mid] > k) hi = mid;
      else lo = mid + 1;
    }
    o[k] = lo;
  }
}

// Levenshtein distance (src/edit_distance.rs:27-60, Kaldi): one wave per pair. Row m of the DP
// is new[n] = n + prefix_min_{n'<=n}(base[n'] - n'), base[n] = min(e[n-1]+delta, e[n]+1),
// base[0] = e[0]+1 -- the in-row dependency of the reference loop as a wave min-scan.
__global__ __launch_bounds__(64) void k_levenshtein(int B, int L, const int* __restrict__ a,
                                                    const int* __restrict__ bsq,
                                                    const int* __restrict__ a_len,
                                                    const int* __restrict__ b_len,
                                                    int* __restrict__ dist) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* e = reinterpret_cast<int*>(smem);  // (L+1)
  int* nb = e + (L + 1);                  // (L+1)
  const int i = blockIdx.x;
  const int lane = threadIdx.x & 63;
  // lengths outside [0, L] panic in the reference (slice bounds); the host layer rejects them,
  // the kernel clamps so a bad device-side length can never read out of bounds
  const int M = min(max(a_len[i], 0), L), N = min(max(b_len[i], 0), L);
  const int* A = a + (size_t)i * L;
  const int* Bv = bsq + (size_t)i * L;
  for (int n = lane; n <= N; n += 64) e[n] = n;
  __syncthreads();
  for (int m = 1; m <= M; ++m) {
    const int am = A[m - 1];
    int carry = 0x3fffffff;
    for (int n0 = 0; n0 <= N; n0 += 64) {
      const int n = n0 + lane;
      int base = 0x3fffffff;
      if (n == 0) base = e[0] + 1;
      else if (n <= N) base = min(e[n - 1] + (am == Bv[n - 1] ? 0 : 1), e[n] + 1);
      int v = (n <= N) ? base - n : 0x3fffffff;
      v = wave_incl_scan_min(v, lane);
      v = min(v, carry);
      if (n <= N) nb[n] = n + v;
      carry = __shfl(v, 63);
    }
    __syncthreads();
    for (int n = lane; n <= N; n += 64) e[n] = nb[n];
    __syncthreads();
  }
  if (lane == 0) dist[i] = e[N];
}

inline int last_error() { return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP; }

}  // namespace

int launch_decode_step(const StepArgs& a, hipStream_t st) {
  if (a.B < 0 || a.W <= 0 || a.Wmax <= 0 || a.C <= 0) return SSNT_ERR_INVALID_ARG;
  if (a.variant == Variant::V1 && a.C != 2) return SSNT_ERR_INVALID_ARG;
  if (a.variant == Variant::V2 && (!a.total || !a.table || !a.output_length || !a.next_total))
    return SSNT_ERR_INVALID_ARG;
  if (a.B == 0) return SSNT_OK;
  const size_t n = (size_t)a.W * a.C;
  const size_t lds = n * sizeof(Cand) + 2 * n * sizeof(int);
  if (lds > 150 * 1024) return SSNT_ERR_UNSUPPORTED;
  if (lds > 64 * 1024) {  // (the attribute is per device: set once per device, not per call)
    static std::atomic<unsigned long long> set_on{0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    const unsigned long long bit = 1ull << (dev & 63);
    if (!(set_on.load(std::memory_order_relaxed) & bit)) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_decode_step),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
      set_on.fetch_or(bit);
    }
  }
  hipLaunchKernelGGL(k_decode_step, dim3(a.B), dim3(64), lds, st, a);
  return last_error();
}

int launch_extract_best(int B, int W, int U, const int* best_final_branch, const int* beam_branch,
                        const int* t_history, int* best_beam_branch, int* best_t_history,
                        int* status, hipStream_t st) {
  if (B < 0 || W <= 0 || U < 0) return SSNT_ERR_INVALID_ARG;
  if (B == 0 || U == 0) return SSNT_OK;
  const int chunk = max(1, min(U, 8192 / W));
  const size_t lds = (size_t)chunk * W * 2 * sizeof(int);
  hipLaunchKernelGGL(k_backtrace, dim3(B), dim3(64), lds, st, B, W, U, 1, best_final_branch,
                     beam_branch, t_history, best_beam_branch, best_t_history, chunk, status);
  return last_error();
}

int launch_order_beam_branch(int B, int W, int T, const int* final_branch, const int* beam_branch,
                             int* ordered, int* status, hipStream_t st) {
  if (B < 0 || W <= 0 || T < 0) return SSNT_ERR_INVALID_ARG;
  if (W > 64) return SSNT_ERR_UNSUPPORTED;
  if (B == 0 || T == 0) return SSNT_OK;
  const int chunk = max(1, min(T, 8192 / W));
  const size_t lds = (size_t)chunk * W * 2 * sizeof(int);
  hipLaunchKernelGGL(k_backtrace, dim3(B), dim3(64), lds, st, B, W, T, W, final_branch,
                     beam_branch, nullptr, ordered, nullptr, chunk, status);
  return last_error();
}

int launch_upsample(int B, int W, int T, int max_u, const int* duration, const int* output_length,
                    int* out, int* status, hipStream_t st) {
  if (B < 0 || W <= 0 || T < 0 || max_u < 0) return SSNT_ERR_INVALID_ARG;
  if (B == 0) return SSNT_OK;
  const size_t lds = (size_t)(T + 1) * sizeof(int);
  if (lds > 150 * 1024) return SSNT_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(k_upsample, dim3(B * W), dim3(64), lds, st, B * W, T, max_u, duration,
                     output_length, out, status);
  return last_error();
}

int launch_levenshtein(int B, int max_length, const int* a, const int* b, const int* a_len,
                       const int* b_len, int* dist, hipStream_t st) {
  if (B < 0 || max_length < 0) return SSNT_ERR_INVALID_ARG;
  if (B == 0) return SSNT_OK;
  const size_t lds = (size_t)(max_length + 1) * 2 * sizeof(int);
  if (lds > 150 * 1024) return SSNT_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(k_levenshtein, dim3(B), dim3(64), lds, st, B, max_length, a, b, a_len,
                     b_len, dist);
  return last_error();
}

}  // namespace ssnt
