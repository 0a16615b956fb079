// xf_math.h -- split-exponent ("xf") f32 arithmetic for the lattice forward-backward on gfx950.
//
// A lattice probability is held as m * 2^e: an f32 mantissa m and an int32 exponent e. The
// recurrence then needs only IEEE mul/add plus v_frexp_mant_f32 / v_frexp_exp_i32_f32 /
// v_ldexp_f32 (one VALU instruction each on CDNA4) -- no transcendental on the serial chain,
// no underflow at any lattice size, and results that a CPU can reproduce bit for bit. The
// only transcendentals are exp() of each input log-prob (Cody-Waite + degree-6 polynomial,
// off the serial chain) and ln() of outputs (loss, optional log-alpha/log-beta).
//
// Canonical forms (DESIGN.md "Split-exponent arithmetic"):
//   normalized : m in [0.5, 1)  or  (m == 0 and e == XF_EZERO)
//   products   : unnormalized mantissas (m_a * m_b, e_a + e_b) are allowed as inputs to add.
// Every function below is specified operation by operation; compile with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ssnt {

constexpr int XF_EZERO = -(1 << 29);
constexpr float XF_LOG_MIN = -1.0e6f;  // log-probs below this (and NaN) are exact zeros
constexpr float XF_LOG_MAX = 1.0e6f;

constexpr float kL2E = 0x1.715476p+0f;
constexpr float kLN2HI = 0x1.62e400p-1f;
constexpr float kLN2LO = 0x1.7f7d1cp-20f;
constexpr float kSQRTH = 0x1.6a09e6p-1f;

struct xf {
  float m;
  int e;
};

__device__ __forceinline__ float xldexp(float x, int e) { return __builtin_amdgcn_ldexpf(x, e); }
__device__ __forceinline__ float xmant(float x) { return __builtin_amdgcn_frexp_mantf(x); }
__device__ __forceinline__ int xexpo(float x) { return __builtin_amdgcn_frexp_expf(x); }

__device__ __forceinline__ xf xf_zero() { return xf{0.0f, XF_EZERO}; }

// normalize (s, e): s == 0 -> canonical zero
__device__ __forceinline__ xf xf_norm(float s, int e) {
  const float m = xmant(s);
  const int k = xexpo(s);
  return xf{m, (s == 0.0f) ? XF_EZERO : e + k};
}

// (ma,ea) + (mb,eb), inputs possibly unnormalized; result normalized
__device__ __forceinline__ xf xf_add(float ma, int ea, float mb, int eb) {
  const int em = max(ea, eb);
  const float s = xldexp(ma, ea - em) + xldexp(mb, eb - em);
  return xf_norm(s, em);
}

// exp(x) as an unnormalized xf (mantissa in [~0.707, ~1.414]); !valid or x < XF_LOG_MIN -> 0
__device__ __forceinline__ xf xf_exp(float x, bool valid) {
  const bool live = valid && (x >= XF_LOG_MIN);
  x = fminf(x, XF_LOG_MAX);
  x = live ? x : 0.0f;
  const float n = __builtin_rintf(x * kL2E);
  float r = __builtin_fmaf(-n, kLN2HI, x);
  r = __builtin_fmaf(-n, kLN2LO, r);
  float p = 0x1.6b6ep-10f;
  p = __builtin_fmaf(p, r, 0x1.122f66p-7f);
  p = __builtin_fmaf(p, r, 0x1.555688p-5f);
  p = __builtin_fmaf(p, r, 0x1.5554a4p-3f);
  p = __builtin_fmaf(p, r, 0x1p-1f);
  p = __builtin_fmaf(p, r, 0x1p+0f);
  p = __builtin_fmaf(p, r, 0x1p+0f);
  return xf{live ? p : 0.0f, live ? (int)n : XF_EZERO};
}

// natural log of a normalized xf; zero -> -inf
__device__ __forceinline__ float xf_log(xf v) {
  float m = v.m;
  int e = v.e;
  const bool lo = m < kSQRTH;
  m = lo ? m * 2.0f : m;
  e = lo ? e - 1 : e;
  const float t = m - 1.0f;
  float q = 0x1.6626eap-4f;
  q = __builtin_fmaf(q, t, -0x1.26729ep-3f);
  q = __builtin_fmaf(q, t, 0x1.32285p-3f);
  q = __builtin_fmaf(q, t, -0x1.5329bep-3f);
  q = __builtin_fmaf(q, t, 0x1.98b80ap-3f);
  q = __builtin_fmaf(q, t, -0x1.0005a6p-2f);
  q = __builtin_fmaf(q, t, 0x1.55579p-2f);
  q = __builtin_fmaf(q, t, -0x1.fffff8p-2f);
  q = __builtin_fmaf(q, t, 0x1p+0f);
  const float lnm = t * q;
  const float ef = (float)e;
  const float r = __builtin_fmaf(ef, kLN2HI, __builtin_fmaf(ef, kLN2LO, lnm));
  return (v.m == 0.0f) ? -__builtin_inff() : r;
}

// -(m * 2^e) with +0 for zero
__device__ __forceinline__ float xf_neg_post(float m, int e) { return 0.0f - xldexp(m, e); }

}  // namespace ssnt
