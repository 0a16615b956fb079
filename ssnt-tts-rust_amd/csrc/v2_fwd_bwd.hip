// v2_fwd_bwd.hip -- F4: the v2 duration-class (semi-Markov) forward-backward for gfx950.
//
// The training-side counterpart of the v2 decode (not in the reference). The
// lattice, its move rules (src/v2.rs:94-166) and the split-exponent arithmetic are defined in
// oracle/ssnt_oracle.c ("F4") and DESIGN.md "Duration lattice"; this kernel reproduces that
// definition bit for bit.
//
// Layout: one workgroup (256 threads, 4 waves) per utterance. State rows r = 0..I (input steps
// consumed) over totals x; only the window of row r (f4_window: the v2 band, or [0, r*dmax] in
// test mode) can hold mass, so rows are stored window-relative, Wcap xf wide:
//   LDS:  duration table | class weights w[t] (2 steps, double-buffered) | alpha rows (2) |
//         beta rows (2)                                    -- 32*Wcap + 20*D bytes
//   HBM:  alpha rows 0..I of every utterance (workspace, B*(Imax+1)*Wcap xf), written by the
//         forward sweep, read back one row per step by the backward sweep.
// Forward: per step, each thread owns cells x = lo + tid (+256 ...) and sums its D class terms
// (two passes: exponent max, then the ldexp-aligned f32 sum in class order); one barrier per
// step; the next step's class weights are converted in the same step by the first D threads.
// Backward: per step, beta of row t (as the forward), and the gradients of step t: class i on
// wave i % 4, its sum over destination totals in 64 lane partials (x mod 64) + an xor butterfly
// -- the oracle's summation order. HBM traffic per utterance: logits once per sweep, alpha rows
// once each way, the gradients once: a few hundred KB, so the sweeps are latency-bound
// (I dependent steps), not bandwidth-bound.
#include <hip/hip_runtime.h>

#include "ssnt_internal.h"
#include "xf_math.h"

namespace ssnt {
namespace {

constexpr int kF4Threads = 256;
constexpr int kF4Waves = kF4Threads / 64;

__device__ __forceinline__ int f4_f2i(float x) {  // Rust `f32 as i32` (saturating, NaN -> 0)
  if (x != x) return 0;
  if (x >= 2147483648.0f) return 2147483647;
  if (x <= -2147483648.0f) return (-2147483647 - 1);
  return (int)x;
}

struct F4Utt {
  int I, O, X, dmax;
  bool test;
};

// cells of row r that can hold mass: [lo, hi] (empty when lo > hi); = oracle f4_window
__device__ __forceinline__ void f4_window(const F4Utt& u, int r, int& lo, int& hi) {
  if (r == 0) {
    lo = 0;
    hi = 0;
    return;
  }
  if (u.test) {
    const long long h = (long long)r * u.dmax;
    lo = 0;
    hi = h < u.X - 1 ? (int)h : u.X - 1;
    return;
  }
  const int t = r - 1;
  if ((long long)(u.I - (t + 1)) * 3 > u.O) {  // will_overrun (src/v2.rs:106-111)
    lo = 1;
    hi = 0;
    return;
  }
  const float diagonal = (float)u.O / (float)u.I * (float)(t + 1);  // src/v2.rs:94-104
  const float upper_range = (float)u.O * 0.1f;
  const float lower_range = (float)u.O * 0.05f;
  int lb = f4_f2i(fmaxf(diagonal - lower_range, 0.0f));
  int ub = f4_f2i(fminf(diagonal + upper_range, (float)u.O));
  if (t == u.I - 1) {  // src/v2.rs:135-137
    lb = max(lb, u.O);
    ub = min(ub, u.O);
  }
  lo = max(lb, 0);
  hi = min(ub, u.X - 1);
}

// debug row: ln of the window cells, -inf elsewhere (row == nullptr: all -inf)
__device__ __forceinline__ void f4_log_row(float* dst, const xf* row, int lo, int hi, int X) {
  for (int x = threadIdx.x; x < X; x += kF4Threads)
    dst[x] = (row && x >= lo && x <= hi) ? xf_log(row[x - lo]) : -__builtin_inff();
}

// one cell: sum over classes of src[x -/+ d_i] (x) w[i], class order (oracle f4_cell_sum).
// FWD: alpha (source total x - d_i, product a.m * w.m); else beta (x + d_i, w.m * b.m).
template <bool FWD>
__device__ __forceinline__ xf f4_cell(int x, const int* dur, const xf* w, int D, const xf* src,
                                      int slo, int shi) {
  int em = XF_EZERO;
  for (int i = 0; i < D; ++i) {
    const int y = FWD ? x - dur[i] : x + dur[i];
    const bool in = y >= slo && y <= shi;
    const int e = in ? src[in ? y - slo : 0].e + w[i].e : XF_EZERO;
    em = max(em, e);
  }
  float s = 0.0f;
  for (int i = 0; i < D; ++i) {
    const int y = FWD ? x - dur[i] : x + dur[i];
    const bool in = y >= slo && y <= shi;
    const xf v = src[in ? y - slo : 0];
    const float m = in ? (FWD ? v.m * w[i].m : w[i].m * v.m) : 0.0f;
    const int e = in ? v.e + w[i].e : XF_EZERO;
    s = s + xldexp(m, e - em);
  }
  return xf_norm(s, em);
}

// xor butterfly over the 64 lane partials (xf_add is commutative: every lane ends equal)
__device__ __forceinline__ xf f4_butterfly(xf acc) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float om = __shfl_xor(acc.m, off);
    const int oe = __shfl_xor(acc.e, off);
    acc = xf_add(acc.m, acc.e, om, oe);
  }
  return acc;
}

__global__ __launch_bounds__(kF4Threads) void k_v2_fwd_bwd(V2FwdBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ xf z_sh;
  __shared__ int bad_sh;
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D = a.D, X = a.X, Imax = a.Imax, Wc = a.Wcap;
  int* dur = reinterpret_cast<int*>(smem);
  xf* wbuf = reinterpret_cast<xf*>(smem + ((D * 4 + 15) & ~15));  // [2][D]
  xf* rowA = wbuf + 2 * D;                                          // [2][Wc]
  xf* rowB = rowA + 2 * Wc;                                         // [2][Wc]
  const float* lg = a.logits + (size_t)b * Imax * D;
  float* g = a.grad ? a.grad + (size_t)b * Imax * D : nullptr;
  const size_t drow = (size_t)(Imax + 1) * X;
  float* la = a.log_alpha ? a.log_alpha + b * drow : nullptr;
  float* lb = a.log_beta ? a.log_beta + b * drow : nullptr;
  xf* ws = reinterpret_cast<xf*>(a.workspace) + (size_t)b * (Imax + 1) * Wc;
  const float inf_loss = (a.flags & SSNT_FLAG_ZERO_INFINITY) ? 0.0f : __builtin_inff();

  if (tid == 0) bad_sh = 0;
  for (int i = tid; i < D; i += kF4Threads) dur[i] = a.table[i];
  __syncthreads();
  F4Utt u;
  u.I = a.input_length[b];
  u.O = a.output_length[b];
  u.X = X;
  u.test = a.test_mode;
  u.dmax = 0;
  bool neg = false;
  for (int i = 0; i < D; ++i) {
    u.dmax = max(u.dmax, dur[i]);
    neg |= dur[i] < 0;
  }
  const bool bad_len = u.I < 0 || u.I > Imax || u.O < 0;
  if ((bad_len || neg) && tid == 0 && a.status) atomicOr(a.status, neg ? kStatusBadIndex : kStatusBadLength);
  // every gradient row starts at zero (rows t < I are overwritten by the backward sweep)
  if (g)
    for (int k = tid; k < Imax * D; k += kF4Threads) g[k] = 0.0f;
  auto finish_debug = [&](int r0, bool alpha_too) {  // rows r0..Imax of the debug outputs: -inf
    for (int r = r0; r <= Imax; ++r) {
      if (alpha_too && la) f4_log_row(la + (size_t)r * X, nullptr, 0, -1, X);
      if (lb) f4_log_row(lb + (size_t)r * X, nullptr, 0, -1, X);
    }
  };
  if (bad_len || neg || u.I == 0) {
    if (tid == 0) a.loss[b] = inf_loss;
    finish_debug(0, true);
    return;
  }
  const int I = u.I;
  auto cls_ok = [&](int i) { return a.allow_skip || i != a.zid; };

  // ================================ forward sweep ==========================================
  int plo = 0, phi = 0;
  if (tid == 0) {
    rowA[0] = xf{0.5f, 1};
    ws[0] = xf{0.5f, 1};
  }
  for (int i = tid; i < D; i += kF4Threads) wbuf[i] = xf_exp(lg[i], cls_ok(i));
  __syncthreads();
  if (la) f4_log_row(la, rowA, 0, 0, X);
  for (int r = 1; r <= I; ++r) {
    int lo, hi;
    f4_window(u, r, lo, hi);
    if (hi - lo + 1 > Wc) {  // host sizing bug: report, drop the utterance (uniform branch)
      if (tid == 0) {
        if (a.status) atomicOr(a.status, kStatusBadLength);
        a.loss[b] = __builtin_nanf("");
      }
      finish_debug(r, true);
      return;
    }
    const xf* w = wbuf + ((r - 1) & 1) * D;
    if (r < I)
      for (int i = tid; i < D; i += kF4Threads) wbuf[(r & 1) * D + i] = xf_exp(lg[(size_t)r * D + i], cls_ok(i));
    const xf* src = rowA + ((r - 1) & 1) * Wc;
    xf* dst = rowA + (r & 1) * Wc;
    xf* wrow = ws + (size_t)r * Wc;
    for (int x = lo + tid; x <= hi; x += kF4Threads) {
      const xf v = f4_cell<true>(x, dur, w, D, src, plo, phi);
      dst[x - lo] = v;
      wrow[x - lo] = v;
    }
    __syncthreads();
    if (la) f4_log_row(la + (size_t)r * X, dst, lo, hi, X);
    plo = lo;
    phi = hi;
  }
  if (la)
    for (int r = I + 1; r <= Imax; ++r) f4_log_row(la + (size_t)r * X, nullptr, 0, -1, X);

  // ================================ Z =======================================================
  const int zlo = plo, zhi = phi;  // window(I)
  if (wave == 0) {
    xf acc = xf_zero();
    const xf* rI = rowA + (I & 1) * Wc;
    for (int x = zlo + ((lane - zlo) & 63); x <= zhi; x += 64) {
      const xf v = rI[x - zlo];
      acc = xf_add(acc.m, acc.e, v.m, v.e);
    }
    acc = f4_butterfly(acc);
    if (lane == 0) {
      z_sh = acc;
      a.loss[b] = acc.m == 0.0f ? inf_loss : 0.0f - xf_log(acc);
    }
  }
  __syncthreads();
  const xf Z = z_sh;
  if (Z.m == 0.0f) {
    finish_debug(0, false);
    return;
  }
  const float izm = 1.0f / Z.m;
  const int ize = -Z.e;

  // ================================ backward sweep =========================================
  for (int x = zlo + tid; x <= zhi; x += kF4Threads) rowB[(I & 1) * Wc + x - zlo] = xf{0.5f, 1};
  __syncthreads();
  if (lb) {
    f4_log_row(lb + (size_t)I * X, rowB + (I & 1) * Wc, zlo, zhi, X);
    for (int r = I + 1; r <= Imax; ++r) f4_log_row(lb + (size_t)r * X, nullptr, 0, -1, X);
  }
  int nlo = zlo, nhi = zhi;  // window(t+1)
  int lo, hi;
  f4_window(u, I - 1, lo, hi);  // window(t)
  for (int t = I - 1; t >= 0; --t) {
    int plo2 = 0, phi2 = -1;  // window(t-1)
    if (t >= 1) f4_window(u, t - 1, plo2, phi2);
    // alpha row t-1 from HBM into the buffer that held row t+1; weights of step t-1
    if (t >= 1) {
      xf* pre = rowA + ((t - 1) & 1) * Wc;
      const xf* srow = ws + (size_t)(t - 1) * Wc;
      for (int k = tid; k <= phi2 - plo2; k += kF4Threads) pre[k] = srow[k];
      for (int i = tid; i < D; i += kF4Threads) wbuf[((t - 1) & 1) * D + i] = xf_exp(lg[(size_t)(t - 1) * D + i], cls_ok(i));
    }
    const xf* w = wbuf + (t & 1) * D;
    const xf* bn = rowB + ((t + 1) & 1) * Wc;  // beta row t+1
    const xf* at = rowA + (t & 1) * Wc;         // alpha row t
    xf* bt = rowB + (t & 1) * Wc;
    for (int y = lo + tid; y <= hi; y += kF4Threads) bt[y - lo] = f4_cell<false>(y, dur, w, D, bn, nlo, nhi);
    // gradients of step t: class i on wave i % 4, destination totals x in lane partials
    if (g) {
      for (int i = wave; i < D; i += kF4Waves) {
        xf acc = xf_zero();
        const int di = dur[i];
        for (int x = nlo + ((lane - nlo) & 63); x <= nhi; x += 64) {
          const int y = x - di;
          if (y < lo || y > hi) continue;
          const xf av = at[y - lo], bv = bn[x - nlo];
          acc = xf_add(acc.m, acc.e, av.m * bv.m, av.e + bv.e);
        }
        acc = f4_butterfly(acc);
        if (lane == 0) g[(size_t)t * D + i] = xf_neg_post((acc.m * w[i].m) * izm, acc.e + w[i].e + ize);
      }
    }
    __syncthreads();
    if (lb) f4_log_row(lb + (size_t)t * X, bt, lo, hi, X);
    nlo = lo;
    nhi = hi;
    lo = plo2;
    hi = phi2;
  }
}

}  // namespace

size_t v2_fwd_bwd_wcap(int max_total, bool test_mode) {
  const int X = max_total + 1;
  if (test_mode) return (size_t)X;
  const size_t band = (size_t)(0.15 * (double)max_total) + 8;  // ub - lb + 1 <= 0.15 O + 3
  return band < (size_t)X ? band : (size_t)X;
}

size_t v2_fwd_bwd_workspace_bytes(int B, int Imax, int max_total, bool test_mode) {
  if (B <= 0 || Imax <= 0 || max_total < 0) return 0;
  return (size_t)B * (Imax + 1) * v2_fwd_bwd_wcap(max_total, test_mode) * sizeof(xf);
}

int launch_v2_fwd_bwd(const V2FwdBwdArgs& in, hipStream_t st) {
  V2FwdBwdArgs a = in;
  if (a.B < 0 || a.Imax <= 0 || a.D <= 0 || a.X <= 0 || !a.logits || !a.table || !a.input_length ||
      !a.output_length || !a.loss)
    return SSNT_ERR_INVALID_ARG;
  if (a.B == 0) return SSNT_OK;
  a.Wcap = (int)v2_fwd_bwd_wcap(a.X - 1, a.test_mode);
  const size_t lds = (size_t)((a.D * 4 + 15) & ~15) + 2 * (size_t)a.D * sizeof(xf) + 4 * (size_t)a.Wcap * sizeof(xf);
  if (lds > 160 * 1024 - 1024) return SSNT_ERR_UNSUPPORTED;
  if (!a.workspace || a.workspace_bytes < v2_fwd_bwd_workspace_bytes(a.B, a.Imax, a.X - 1, a.test_mode))
    return SSNT_ERR_WORKSPACE;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_v2_fwd_bwd),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k_v2_fwd_bwd, dim3(a.B), dim3(kF4Threads), lds, st, a);
  return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
}

}  // namespace ssnt
