// fwd_bwd.hip -- emit/shift lattice forward-backward (loss + gradients) for gfx950.
//
// Lattice semantics: DESIGN.md "Lattice semantics" (SURVEY.md 8(a) A11). The reference
// (nii-yamagishilab/ssnt-tts-rust) has no forward-backward; the transition rules come from its
// decode step: emit (s,p)->(s+1,p), shift (s,p)->(s+1,p+1), no shift out of the last input
// position, terminal emit at the last position (src/lib.rs:186-226).
//
// Kernel shape (one workgroup = one utterance, two waves):
//   wave 0 sweeps alpha rows upward, wave 1 sweeps beta rows downward, concurrently. Each row
//   is an anti-diagonal of the (position, emit-count) grid; a lane holds K consecutive
//   positions p = K*lane + j, and the only cross-lane dependency per step is one DPP
//   wave-shift (v_mov_dpp wave_shr:1 / wave_shl:1) of the boundary element.
//   Phase 1: alpha[0..M] and beta[S-1..M] (M = (S-1)>>1), rows kept in LDS (or a global
//   workspace when T*U*8 B does not fit), inputs streamed through a D-deep register ring.
//   Cut: Z = tree-sum over p of alpha[M][p]*beta[M][p] (canonical binary tree).
//   Phase 2: each wave keeps sweeping and, now that Z is known, emits the gradient row of every
//   transition it passes (wave 0: transitions M..S-1, wave 1: M-1..0) -- the gradient stores
//   stream out while the recurrence is still running.
// Arithmetic: split-exponent xf (xf_math.h); bit-exact with oracle/ssnt_oracle.c.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include "buffer_ops.h"
#include "ssnt_internal.h"
#include "xf_math.h"

namespace ssnt {
namespace {

constexpr size_t kLdsBudget = 160 * 1024 - 256;  // one workgroup per CU may use ~all 160 KiB
template <int K>
constexpr int ring_depth() { return K <= 2 ? 8 : 4; }  // input prefetch depth (rows)

typedef float f2 __attribute__((ext_vector_type(2)));

// DPP wave shifts; lanes without a source keep `old` (bound_ctrl off), which is set to the
// canonical xf zero, so lane 0 (shr) / lane 63 (shl) need no fix-up.
__device__ __forceinline__ float shr1(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ int shr1(int x) {
  return __builtin_amdgcn_update_dpp(XF_EZERO, x, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ float shl1(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x130, 0xf, 0xf, false));
}
__device__ __forceinline__ int shl1(int x) {
  return __builtin_amdgcn_update_dpp(XF_EZERO, x, 0x130, 0xf, 0xf, false);
}

template <int K, bool OBS>
struct Item {
  float lt[2 * K];
  float ob[OBS ? K : 1];
};

template <int K>
struct XRow {
  float m[K];
  int e[K];
};

// Lane slice of K consecutive positions, 4*N bytes, moved as one unit. VEC: U % K == 0 and
// 16-byte aligned bases, so a lane's slice is either whole or entirely beyond U: one predicate,
// widest loads. !VEC: per-element predicates (odd shapes only).
template <int N>
__device__ __forceinline__ void ld_vec(float* dst, const float* src) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
      const float4 v = reinterpret_cast<const float4*>(src)[q];
      dst[4 * q] = v.x; dst[4 * q + 1] = v.y; dst[4 * q + 2] = v.z; dst[4 * q + 3] = v.w;
    }
  } else if constexpr (N == 2) {
    const float2 v = *reinterpret_cast<const float2*>(src);
    dst[0] = v.x; dst[1] = v.y;
  } else {
    dst[0] = src[0];
  }
}
template <int N>
__device__ __forceinline__ void st_vec(float* dst, const float* v) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int q = 0; q < N / 4; ++q)
      reinterpret_cast<float4*>(dst)[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  } else if constexpr (N == 2) {
    *reinterpret_cast<float2*>(dst) = make_float2(v[0], v[1]);
  } else {
    dst[0] = v[0];
  }
}

template <int K, bool OBS, bool VEC>
__device__ __forceinline__ Item<K, OBS> load_item(const float* __restrict__ lt,
                                                  const float* __restrict__ lo, int row,
                                                  int orow, int T, int U, int lane) {
  Item<K, OBS> it;
  row = min(max(row, 0), T - 1);
  const int p0 = K * lane;
  const float* src = lt + ((size_t)row * U + p0) * 2;
  if constexpr (VEC) {
    if (p0 < U) {
      ld_vec<2 * K>(it.lt, src);
    } else {
#pragma unroll
      for (int j = 0; j < 2 * K; ++j) it.lt[j] = 0.0f;
    }
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      float2 v = make_float2(0.0f, 0.0f);
      if (p0 + j < U) v = reinterpret_cast<const float2*>(src)[j];
      it.lt[2 * j] = v.x;
      it.lt[2 * j + 1] = v.y;
    }
  }
  if constexpr (OBS) {
    orow = min(max(orow, 0), T - 1);
    const float* osrc = lo + (size_t)orow * U + p0;
    if constexpr (VEC) {
      if (p0 < U) {
        ld_vec<K>(it.ob, osrc);
      } else {
#pragma unroll
        for (int j = 0; j < K; ++j) it.ob[j] = 0.0f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) it.ob[j] = (p0 + j < U) ? osrc[j] : 0.0f;
    }
  }
  return it;
}

template <int K, bool VEC>
__device__ __forceinline__ void store_row(xf* __restrict__ dst, const XRow<K>& r, int U, int lane) {
  const int p0 = K * lane;
  if constexpr (VEC) {
    if (p0 < U) {
      float v[2 * K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        v[2 * j] = r.m[j];
        v[2 * j + 1] = __builtin_bit_cast(float, r.e[j]);
      }
      st_vec<2 * K>(reinterpret_cast<float*>(dst + p0), v);
    }
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (p0 + j < U) dst[p0 + j] = xf{r.m[j], r.e[j]};
  }
}

template <int K, bool VEC>
__device__ __forceinline__ XRow<K> load_row(const xf* __restrict__ src, int U, int lane) {
  XRow<K> r;
  const int p0 = K * lane;
  if constexpr (VEC) {
    float v[2 * K];
    if (p0 < U) {
      ld_vec<2 * K>(v, reinterpret_cast<const float*>(src + p0));
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        v[2 * j] = 0.0f;
        v[2 * j + 1] = __builtin_bit_cast(float, XF_EZERO);
      }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
      r.m[j] = v[2 * j];
      r.e[j] = __builtin_bit_cast(int, v[2 * j + 1]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      xf v = xf_zero();
      if (p0 + j < U) v = src[p0 + j];
      r.m[j] = v.m;
      r.e[j] = v.e;
    }
  }
  return r;
}

template <int K, bool VEC>
__device__ __forceinline__ void store_grad_row(float* __restrict__ g, const float* ge,
                                               const float* gs, int U, int lane) {
  const int p0 = K * lane;
  float v[2 * K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    v[2 * j] = ge[j];
    v[2 * j + 1] = gs[j];
  }
  if constexpr (VEC) {
    if (p0 < U) st_vec<2 * K>(g + (size_t)p0 * 2, v);
  } else {
    float2* dst = reinterpret_cast<float2*>(g + (size_t)p0 * 2);
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (p0 + j < U) dst[j] = make_float2(v[2 * j], v[2 * j + 1]);
  }
}

template <int K, bool VEC>
__device__ __forceinline__ void store_f_row(float* __restrict__ dst, const float* v, int U, int lane) {
  const int p0 = K * lane;
  if constexpr (VEC) {
    if (p0 < U) st_vec<K>(dst + p0, v);
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (p0 + j < U) dst[p0 + j] = v[j];
  }
}

template <int K, bool VEC>
__device__ __forceinline__ void store_log_row(float* __restrict__ dst, const XRow<K>& r, int U, int lane) {
  float v[K];
#pragma unroll
  for (int j = 0; j < K; ++j) v[j] = xf_log(xf{r.m[j], r.e[j]});
  store_f_row<K, VEC>(dst, v, U, lane);
}

// exp() of the (emit, shift) pair of one position as two unnormalized xf, with packed f32
// FMAs (v_pk_fma_f32): the same per-element IEEE operations as xf_exp (xf_math.h). Inputs are
// clamped into [XF_LOG_MIN, XF_LOG_MAX] for the arithmetic; dead elements are zeroed at the end.
__device__ __forceinline__ void xf_exp_pair(float xe, float xs, bool ve, bool vs, float& me,
                                            int& ee, float& ms, int& es) {
  const bool le = ve && (xe >= XF_LOG_MIN);
  const bool ls = vs && (xs >= XF_LOG_MIN);
  f2 x;
  x.x = __builtin_amdgcn_fmed3f(xe, XF_LOG_MIN, XF_LOG_MAX);
  x.y = __builtin_amdgcn_fmed3f(xs, XF_LOG_MIN, XF_LOG_MAX);
  const f2 t = x * (f2){kL2E, kL2E};
  f2 n;
  n.x = __builtin_rintf(t.x);
  n.y = __builtin_rintf(t.y);
  f2 r = __builtin_elementwise_fma(-n, (f2){kLN2HI, kLN2HI}, x);
  r = __builtin_elementwise_fma(-n, (f2){kLN2LO, kLN2LO}, r);
  f2 p = (f2){0x1.6da758p-10f, 0x1.6da758p-10f};
  p = __builtin_elementwise_fma(p, r, (f2){0x1.126facp-7f, 0x1.126facp-7f});
  p = __builtin_elementwise_fma(p, r, (f2){0x1.555464p-5f, 0x1.555464p-5f});
  p = __builtin_elementwise_fma(p, r, (f2){0x1.555404p-3f, 0x1.555404p-3f});
  p = __builtin_elementwise_fma(p, r, (f2){0x1p-1f, 0x1p-1f});
  p = __builtin_elementwise_fma(p, r, (f2){0x1p+0f, 0x1p+0f});
  p = __builtin_elementwise_fma(p, r, (f2){0x1p+0f, 0x1p+0f});
  me = le ? p.x : 0.0f;
  ee = le ? (int)n.x : XF_EZERO;
  ms = ls ? p.y : 0.0f;
  es = ls ? (int)n.y : XF_EZERO;
}

// Convert the lane's inputs of one row to xf: emit E, shift S (masked: p<P, shift p<P-1).
template <int K, bool OBS>
__device__ __forceinline__ void convert(const Item<K, OBS>& it, int P, int lane, XRow<K>& E,
                                        XRow<K>& Sh) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int p = K * lane + j;
    xf_exp_pair(it.lt[2 * j], it.lt[2 * j + 1], p < P, p < P - 1, E.m[j], E.e[j], Sh.m[j], Sh.e[j]);
  }
}

template <int K, bool OBS>
__device__ __forceinline__ void convert_obs(const Item<K, OBS>& it, int P, int lane, XRow<K>& O) {
  if constexpr (OBS) {
#pragma unroll
    for (int j = 0; j + 1 < K; j += 2) {  // pairs of positions through the packed path
      xf_exp_pair(it.ob[j], it.ob[j + 1], K * lane + j < P, K * lane + j + 1 < P, O.m[j], O.e[j],
                  O.m[j + 1], O.e[j + 1]);
    }
    if constexpr (K % 2 == 1) {
      const xf o = xf_exp(it.ob[K - 1], K * lane + K - 1 < P);
      O.m[K - 1] = o.m;
      O.e[K - 1] = o.e;
    }
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      O.m[j] = 1.0f;
      O.e[j] = 0;
    }
  }
}

// alpha[s+1] from alpha[s]: stay/shift products (returned for reuse by the gradients).
template <int K, bool OBS>
__device__ __forceinline__ void alpha_step(XRow<K>& A, const XRow<K>& E, const XRow<K>& Sh,
                                           const XRow<K>& O, XRow<K>& stay, XRow<K>& shft) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    stay.m[j] = A.m[j] * E.m[j];
    stay.e[j] = A.e[j] + E.e[j];
    shft.m[j] = A.m[j] * Sh.m[j];
    shft.e[j] = A.e[j] + Sh.e[j];
  }
  const float lm = shr1(shft.m[K - 1]);
  const int le = shr1(shft.e[K - 1]);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const float hm = (j == 0) ? lm : shft.m[j - 1];
    const int he = (j == 0) ? le : shft.e[j - 1];
    const int em = max(stay.e[j], he);
    float sum = xldexp(stay.m[j], stay.e[j] - em) + xldexp(hm, he - em);
    int ee = em;
    if constexpr (OBS) {
      sum = sum * O.m[j];
      ee = ee + O.e[j];
    }
    const xf r = xf_norm(sum, ee);
    A.m[j] = r.m;
    A.e[j] = r.e;
  }
}

// Q = beta[s+1] (x obs[s+1]) and its right neighbour R = Q[p+1].
template <int K, bool OBS>
__device__ __forceinline__ void entering(const XRow<K>& Bn, const XRow<K>& O, XRow<K>& Q,
                                         XRow<K>& R) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if constexpr (OBS) {
      Q.m[j] = Bn.m[j] * O.m[j];
      Q.e[j] = Bn.e[j] + O.e[j];
    } else {
      Q.m[j] = Bn.m[j];
      Q.e[j] = Bn.e[j];
    }
  }
  const float rm = shl1(Q.m[0]);
  const int re = shl1(Q.e[0]);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    R.m[j] = (j == K - 1) ? rm : Q.m[j + 1 < K ? j + 1 : 0];
    R.e[j] = (j == K - 1) ? re : Q.e[j + 1 < K ? j + 1 : 0];
  }
}

template <int K>
__device__ __forceinline__ void beta_step(XRow<K>& Bt, const XRow<K>& E, const XRow<K>& Sh,
                                          const XRow<K>& Q, const XRow<K>& R) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const xf r = xf_add(E.m[j] * Q.m[j], E.e[j] + Q.e[j], Sh.m[j] * R.m[j], Sh.e[j] + R.e[j]);
    Bt.m[j] = r.m;
    Bt.e[j] = r.e;
  }
}

template <int K, bool OBS, bool LDS, bool VEC>
__global__ __launch_bounds__(128) void k_fwd_bwd(FwdBwdArgs a) {
  constexpr int kRing = ring_depth<K>();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: SGPR rsrcs
  const int lane = threadIdx.x & 63;
  const int T = a.T, U = a.U;
  const int S = a.step_len[b];
  const int P = a.pos_len[b];
  const bool term = (a.flags & SSNT_FLAG_TERMINAL_EMIT) != 0;
  const size_t TU = (size_t)T * U;
  const float* __restrict__ lt = a.log_trans + (size_t)b * TU * 2;
  const float* __restrict__ lo = OBS ? a.log_obs + (size_t)b * TU : nullptr;
  float* __restrict__ g = a.grad ? a.grad + (size_t)b * TU * 2 : nullptr;
  float* __restrict__ go = (OBS && a.grad_obs) ? a.grad_obs + (size_t)b * TU : nullptr;
  float* __restrict__ la = a.log_alpha ? a.log_alpha + (size_t)b * TU : nullptr;
  float* __restrict__ lb = a.log_beta ? a.log_beta + (size_t)b * TU : nullptr;

  xf* cutb = reinterpret_cast<xf*>(smem);  // 64*K beta[M] slots
  xf* zsh = cutb + 64 * K;                 // Z broadcast (+ pad)
  xf* rows = LDS ? (zsh + 2) : reinterpret_cast<xf*>(a.workspace) + (size_t)b * TU;

  const bool feasible = S >= 1 && P >= 1 && S <= T && P <= U && S >= P;
  auto fill_rows = [&](int from) {  // zero grads / -inf debug for rows [from, T), split by wave
    for (int s = from + wave; s < T; s += 2) {
      float z[K], ninf[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        z[j] = 0.0f;
        ninf[j] = -__builtin_inff();
      }
      if (g) store_grad_row<K, VEC>(g + (size_t)s * U * 2, z, z, U, lane);
      if (go) store_f_row<K, VEC>(go + (size_t)s * U, z, U, lane);
      if (la) store_f_row<K, VEC>(la + (size_t)s * U, ninf, U, lane);
      if (lb) store_f_row<K, VEC>(lb + (size_t)s * U, ninf, U, lane);
    }
  };
  const float inf_loss = (a.flags & SSNT_FLAG_ZERO_INFINITY) ? 0.0f : __builtin_inff();
  if (!feasible) {
    if ((S > T || P > U || S < 0 || P < 0) && a.status && threadIdx.x == 0)
      atomicOr(a.status, kStatusBadLength);
    fill_rows(0);
    if (threadIdx.x == 0) a.loss[b] = inf_loss;
    return;
  }
  const int M = (S - 1) >> 1;
  const bool fwd = (wave == 0);
  // stream position r -> input row: fwd r, bwd S-1-r; obs row = row + 1 (fwd: alpha[row+1]
  // needs obs[row+1]; bwd: Q = beta[row+1]*obs[row+1]).
  auto srow = [&](int r) { return fwd ? r : S - 1 - r; };

  Item<K, OBS> ring[kRing];
#pragma unroll
  for (int i = 0; i < kRing; ++i) {
    const int row = srow(i);
    ring[i] = load_item<K, OBS, VEC>(lt, lo, row, row + 1, T, U, lane);
  }
  XRow<K> X;  // fwd: alpha row; bwd: beta row
  // ---------------- init ----------------
  if (fwd) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      X.m[j] = 0.0f;
      X.e[j] = XF_EZERO;
    }
    if (lane == 0) {
      if constexpr (OBS) {
        const xf o = xf_exp(lo[0], true);
        const xf n = xf_norm(o.m, o.e);
        X.m[0] = n.m;
        X.e[0] = n.e;
      } else {
        X.m[0] = 0.5f;
        X.e[0] = 1;
      }
    }
    store_row<K, VEC>(rows, X, U, lane);
    if (la) store_log_row<K, VEC>(la, X, U, lane);
  }
  const int r0 = fwd ? 0 : 1;               // bwd consumes stream slot 0 for its init
  const int r1 = fwd ? M : S - M;           // phase-1 end (exclusive)
  // bwd init uses ring slot 0 (row S-1)
  if (!fwd) {
    const Item<K, OBS> it = ring[0];
    ring[0] = load_item<K, OBS, VEC>(lt, lo, srow(kRing), srow(kRing) + 1, T, U, lane);
    XRow<K> E, Sh;
    convert<K, OBS>(it, P, lane, E, Sh);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const bool last = (K * lane + j) == P - 1;
      xf v = term ? xf_norm(E.m[j], E.e[j]) : xf{0.5f, 1};
      X.m[j] = last ? v.m : 0.0f;
      X.e[j] = last ? v.e : XF_EZERO;
    }
    const int s = S - 1;
    if (s > M) store_row<K, VEC>(rows + (size_t)s * U, X, U, lane);
    else store_row<K, VEC>(cutb, X, 64 * K, lane);
    if (lb) store_log_row<K, VEC>(lb + (size_t)s * U, X, U, lane);
  }
  // ---------------- phase 1 ----------------
  for (int base = (r0 / kRing) * kRing; base < r1; base += kRing) {
#pragma unroll
    for (int i = 0; i < kRing; ++i) {
      const int r = base + i;
      if (r >= r0 && r < r1) {
        const Item<K, OBS> it = ring[i];
        const int nr = srow(r + kRing);
        ring[i] = load_item<K, OBS, VEC>(lt, lo, nr, nr + 1, T, U, lane);
        XRow<K> E, Sh, O;
        convert<K, OBS>(it, P, lane, E, Sh);
        convert_obs<K, OBS>(it, P, lane, O);
        if (fwd) {  // alpha[r+1]
          XRow<K> stay, shft;
          alpha_step<K, OBS>(X, E, Sh, O, stay, shft);
          store_row<K, VEC>(rows + (size_t)(r + 1) * U, X, U, lane);
          if (la) store_log_row<K, VEC>(la + (size_t)(r + 1) * U, X, U, lane);
        } else {  // beta[s], s = S-1-r
          const int s = S - 1 - r;
          XRow<K> Q, R;
          entering<K, OBS>(X, O, Q, R);
          beta_step<K>(X, E, Sh, Q, R);
          if (s > M) store_row<K, VEC>(rows + (size_t)s * U, X, U, lane);
          else store_row<K, VEC>(cutb, X, 64 * K, lane);
          if (lb) store_log_row<K, VEC>(lb + (size_t)s * U, X, U, lane);
        }
      }
    }
  }
  __syncthreads();
  // ---------------- cut: Z = sum_p alpha[M][p] * beta[M][p] ----------------
  if (fwd) {
    float wm[K];
    int we[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const xf c = cutb[K * lane + j];
      wm[j] = X.m[j] * c.m;
      we[j] = X.e[j] + c.e;
    }
    // in-lane binary tree (pairs (2i,2i+1) first)
#pragma unroll
    for (int len = K; len > 1; len >>= 1) {
#pragma unroll
      for (int i = 0; i < len / 2; ++i) {
        const xf r = xf_add(wm[2 * i], we[2 * i], wm[2 * i + 1], we[2 * i + 1]);
        wm[i] = r.m;
        we[i] = r.e;
      }
    }
    xf z = (K == 1) ? xf_norm(wm[0], we[0]) : xf{wm[0], we[0]};
    if (K == 1) {  // level 1 of the tree happens across lanes: first combine leaves
      // (K == 1: the leaves are per-lane; the xor-1 butterfly below is level 1)
      z = xf{wm[0], we[0]};
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const float om = __shfl_xor(z.m, off);
      const int oe = __shfl_xor(z.e, off);
      z = xf_add(z.m, z.e, om, oe);
    }
    if (lane == 0) zsh[0] = z;
  }
  __syncthreads();
  const xf Z = zsh[0];
  if (Z.m == 0.0f) {
    fill_rows(0);
    if (threadIdx.x == 0) a.loss[b] = inf_loss;
    return;
  }
  if (fwd && lane == 0) a.loss[b] = 0.0f - xf_log(Z);
  const float izm = 1.0f / Z.m;
  const int ize = -Z.e;
  // ---------------- phase 2 ----------------
  const int q0 = fwd ? M : S - M;
  const int q1 = S;
  for (int base = (q0 / kRing) * kRing; base < q1; base += kRing) {
#pragma unroll
    for (int i = 0; i < kRing; ++i) {
      const int r = base + i;
      if (r >= q0 && r < q1) {
        const Item<K, OBS> it = ring[i];
        const int nr = srow(r + kRing);
        ring[i] = load_item<K, OBS, VEC>(lt, lo, nr, nr + 1, T, U, lane);
        XRow<K> E, Sh, O;
        convert<K, OBS>(it, P, lane, E, Sh);
        convert_obs<K, OBS>(it, P, lane, O);
        float ge[K], gs[K], gob[K];
        if (fwd) {
          const int s = r;  // transition s: alpha[s] (X) -> row s+1
          XRow<K> Q, R;
          if (s + 1 < S) {
            const XRow<K> Bn = load_row<K, VEC>(rows + (size_t)(s + 1) * U, U, lane);
            entering<K, OBS>(Bn, O, Q, R);
          } else {
#pragma unroll
            for (int j = 0; j < K; ++j) {
              const bool last = term && (K * lane + j) == P - 1;
              Q.m[j] = last ? 1.0f : 0.0f;
              Q.e[j] = last ? 0 : XF_EZERO;
              R.m[j] = 0.0f;
              R.e[j] = XF_EZERO;
            }
          }
          if constexpr (OBS) {
            const XRow<K> Bs = (s == M) ? load_row<K, VEC>(cutb, 64 * K, lane)
                                        : load_row<K, VEC>(rows + (size_t)s * U, U, lane);
#pragma unroll
            for (int j = 0; j < K; ++j)
              gob[j] = xf_neg_post((X.m[j] * Bs.m[j]) * izm, X.e[j] + Bs.e[j] + ize);
          }
          XRow<K> stay, shft;
          XRow<K> Xn = X;
          alpha_step<K, OBS>(Xn, E, Sh, O, stay, shft);  // (stay/shft of alpha[s])
#pragma unroll
          for (int j = 0; j < K; ++j) {
            ge[j] = xf_neg_post((stay.m[j] * Q.m[j]) * izm, stay.e[j] + Q.e[j] + ize);
            gs[j] = xf_neg_post((shft.m[j] * R.m[j]) * izm, shft.e[j] + R.e[j] + ize);
          }
          if (g) store_grad_row<K, VEC>(g + (size_t)s * U * 2, ge, gs, U, lane);
          if constexpr (OBS) {
            if (go) store_f_row<K, VEC>(go + (size_t)s * U, gob, U, lane);
          }
          if (s + 1 < S) {
            X = Xn;
            if (la) store_log_row<K, VEC>(la + (size_t)(s + 1) * U, X, U, lane);
          }
        } else {
          const int s = S - 1 - r;  // transition s: beta[s+1] (X) -> beta[s]
          XRow<K> Q, R;
          entering<K, OBS>(X, O, Q, R);
          const XRow<K> A = load_row<K, VEC>(rows + (size_t)s * U, U, lane);
#pragma unroll
          for (int j = 0; j < K; ++j) {
            ge[j] = xf_neg_post(((A.m[j] * E.m[j]) * Q.m[j]) * izm, A.e[j] + E.e[j] + Q.e[j] + ize);
            gs[j] = xf_neg_post(((A.m[j] * Sh.m[j]) * R.m[j]) * izm, A.e[j] + Sh.e[j] + R.e[j] + ize);
          }
          beta_step<K>(X, E, Sh, Q, R);
          if constexpr (OBS) {
#pragma unroll
            for (int j = 0; j < K; ++j)
              gob[j] = xf_neg_post((A.m[j] * X.m[j]) * izm, A.e[j] + X.e[j] + ize);
            if (go) store_f_row<K, VEC>(go + (size_t)s * U, gob, U, lane);
          }
          if (g) store_grad_row<K, VEC>(g + (size_t)s * U * 2, ge, gs, U, lane);
          if (lb) store_log_row<K, VEC>(lb + (size_t)s * U, X, U, lane);
        }
      }
    }
  }
  fill_rows(S);
}

// =============================================================================================
// Pipelined kernel (VEC shapes: U % K == 0, 16-byte aligned tensors):
//   2 chain waves + 2*NC converter waves per utterance (one workgroup).
//   Converter waves (NC per direction) stream log_trans / log_obs rows through a deep register
//   prefetch ring, convert them to split-exponent form (the exp of every input, the largest
//   block of VALU work) and hand them to their chain through an R-slot LDS ring. The chain
//   waves keep only the serial recurrence (+ the gradient rows in phase 2), at high priority.
// Every per-step memory access in the chain is unpredicated straight-line code, so the
// compiler can schedule the whole step as one block: global rows use buffer instructions whose
// hardware range check drops / zero-fills lanes past U; LDS accesses of lanes past U are
// redirected to a junk (stores) or canonical-zero (loads) area by an address select.
// Hand-off (all LDS, one workgroup): converter writes a slot, then release-stores its `done`
// counter; the chain acquire-loads `done` only when it runs out of known-ready rows. The chain
// returns a slot by storing `kprog` with a value that data-depends on the slot's contents
// (so the store cannot issue before the slot reads returned; LDS executes a wave's DS ops in
// order). Every spin is bounded (status bit on timeout).
// =============================================================================================
constexpr int kStatusTimeout = 1 << 4;
constexpr int kSpinLimit = 1 << 22;

// Diagnostic build only (-DSSNT_DIAG, `make lib-diag`): s_memtime stamps per role, read back with
// ssnt_diag_read(). Layout: g_diag[b*4 + role][8], role 0 fwd chain, 1 bwd chain, 2/3 first
// fwd/bwd converter. Slots: 0 total, 1 wait-for-rows (chain) / wait-for-slot (conv),
// 2 waits, 3 cut wait, 4 phase-1 end. Never present in the product build.
#ifdef SSNT_DIAG
__device__ unsigned long long g_diag[4096 * 4][8];
#define DIAG_T() __builtin_amdgcn_s_memtime()
#else
#define DIAG_T() 0ull
#endif

struct PipeCtl {
  int done[2][4];  // per direction, per converter: rows of its share completed
  int kprog[2];    // per direction: stream rows consumed by the chain
  int bm_ready;    // beta[M] is in the cut buffer
  int z_ready;     // Z is published
  int pad[20];
  xf z;
  xf pad2;
};

__device__ __forceinline__ int lds_acquire(const int* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// uniform counter stores: every lane stores the same value (one unpredicated ds_write)
__device__ __forceinline__ void lds_release(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_relaxed(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <bool SLEEP = true>
__device__ __forceinline__ int spin_geq(const int* p, int target, int* status) {
  int v = lds_acquire(p);
  int n = 0;
  while (v < target) {
    if constexpr (SLEEP) __builtin_amdgcn_s_sleep(1);
    v = lds_acquire(p);
    if (++n > kSpinLimit) {
      if (status && (threadIdx.x & 63) == 0) atomicOr(status, kStatusTimeout);
      return target;
    }
  }
  return v;
}

// raw buffer over [base, base+bytes): out-of-range lanes read 0 / drop their stores.
// `base` must be wave-uniform (the descriptor lives in SGPRs).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
// N floats at byte offset voff of a buffer range
template <int N>
__device__ __forceinline__ void buf_ld(float* dst, __amdgpu_buffer_rsrc_t r, int voff) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
      const f32x4 v = rbuf_ld4(r, voff + 16 * q, 0, 0);
      dst[4 * q] = v.x;
      dst[4 * q + 1] = v.y;
      dst[4 * q + 2] = v.z;
      dst[4 * q + 3] = v.w;
    }
  } else if constexpr (N == 2) {
    const f32x2 v = rbuf_ld2(r, voff, 0, 0);
    dst[0] = v.x;
    dst[1] = v.y;
  } else {
    dst[0] = rbuf_ld1(r, voff, 0, 0);
  }
}
// N floats to byte offset voff
template <int N>
__device__ __forceinline__ void buf_st(const float* v, __amdgpu_buffer_rsrc_t r, int voff) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int q = 0; q < N / 4; ++q)
      rbuf_st4(f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]}, r, voff + 16 * q, 0, 0);
  } else if constexpr (N == 2) {
    rbuf_st2(f32x2{v[0], v[1]}, r, voff, 0, 0);
  } else {
    rbuf_st1(v[0], r, voff, 0, 0);
  }
}

template <int K>
__device__ __forceinline__ void xrow_pack(const XRow<K>& r, float* v) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    v[2 * j] = r.m[j];
    v[2 * j + 1] = __builtin_bit_cast(float, r.e[j]);
  }
}
template <int K>
__device__ __forceinline__ XRow<K> xrow_unpack(const float* v) {
  XRow<K> r;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    r.m[j] = v[2 * j];
    r.e[j] = __builtin_bit_cast(int, v[2 * j + 1]);
  }
  return r;
}

// Lattice-row storage (alpha rows of phase 1, beta rows of phase 1): LDS with junk/zero
// redirection for lanes past U, or a global workspace through range-checked buffer ops.
template <int K, bool LDS>
struct RowStore {
  xf* rows;        // LDS rows (LDS) or this utterance's workspace rows (global)
  xf* junk;        // LDS: 64*K xf scratch for stores of lanes past U
  const xf* zero;  // LDS: 64*K canonical zeros for loads of lanes past U
  int U, lane;
  bool act;
  __device__ __forceinline__ void store(int s, const XRow<K>& r) const {
    float v[2 * K];
    xrow_pack<K>(r, v);
    if constexpr (LDS) {
      xf* p = act ? rows + (size_t)s * U + K * lane : junk + K * lane;
      st_vec<2 * K>(reinterpret_cast<float*>(p), v);
    } else {
      buf_st<2 * K>(v, brsrc(rows + (size_t)s * U, (unsigned)U * 8u), K * lane * 8);
    }
  }
  __device__ __forceinline__ XRow<K> load(int s) const {
    float v[2 * K];
    if constexpr (LDS) {
      const xf* p = act ? rows + (size_t)s * U + K * lane : zero + K * lane;
      ld_vec<2 * K>(v, reinterpret_cast<const float*>(p));
    } else {
      buf_ld<2 * K>(v, brsrc(rows + (size_t)s * U, (unsigned)U * 8u), K * lane * 8);
#pragma unroll
      for (int j = 0; j < K; ++j)  // out-of-range lanes read 0 bits: make them canonical zeros
        if (!act) v[2 * j + 1] = __builtin_bit_cast(float, XF_EZERO);
    }
    return xrow_unpack<K>(v);
  }
};

template <int K>
constexpr int conv_depth() { return K <= 2 ? 8 : (K <= 4 ? 4 : 2); }

// ISO: two extra idle waves at indices 4, 5 so that (with the usual round-robin wave -> SIMD
// placement) the chain waves 0, 1 own SIMD 0, 1 and the converters share SIMD 2, 3.
template <int K, bool OBS, bool LDS, int NC, int R, bool ISO>
__global__ __launch_bounds__(64 * (2 + 2 * NC + (ISO ? 2 : 0))) void k_fwd_bwd_pipe(FwdBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: SGPR rsrcs
  const int lane = threadIdx.x & 63;
  const int T = a.T, U = a.U;
  const int S = a.step_len[b];
  const int P = a.pos_len[b];
  const bool term = (a.flags & SSNT_FLAG_TERMINAL_EMIT) != 0;
  const size_t TU = (size_t)T * U;
  const float* lt = a.log_trans + (size_t)b * TU * 2;
  const float* lo = OBS ? a.log_obs + (size_t)b * TU : nullptr;
  float* g = a.grad ? a.grad + (size_t)b * TU * 2 : nullptr;
  float* go = (OBS && a.grad_obs) ? a.grad_obs + (size_t)b * TU : nullptr;
  float* la = a.log_alpha ? a.log_alpha + (size_t)b * TU : nullptr;
  float* lb = a.log_beta ? a.log_beta + (size_t)b * TU : nullptr;
  const int p0 = K * lane;
  const bool act = p0 < U;

  // LDS: control | cut buffer (64K xf) | zero area (64K xf) | junk area (64K xf) |
  //      rings [dir][R][E/S U*16 B + obs U*8 B] | storage rows (LDS mode)
  PipeCtl* ctl = reinterpret_cast<PipeCtl*>(smem);
  xf* cutb = reinterpret_cast<xf*>(smem + sizeof(PipeCtl));
  xf* zero = cutb + 64 * K;
  xf* junk = zero + 64 * K;
  const int es_words = U * 4;                // floats per E/S slot (U % K == 0 -> 16 B aligned)
  const int ob_words = OBS ? U * 2 : 0;      // floats per obs slot
  const int slot_words = es_words + ((ob_words + 3) & ~3);
  float* rings = reinterpret_cast<float*>(junk + 64 * K);
  xf* rows_base = LDS ? reinterpret_cast<xf*>(rings + 2 * R * slot_words)
                      : reinterpret_cast<xf*>(a.workspace) + (size_t)b * TU;
  const RowStore<K, LDS> store{rows_base, junk, zero, U, lane, act};

  const bool feasible = S >= 1 && P >= 1 && S <= T && P <= U && S >= P;
  const int nw = 2 + 2 * NC + (ISO ? 2 : 0);
  auto fill_rows = [&](int from, int w0, int wstep) {  // zero grads / -inf debug rows
    float z[2 * K], ninf[K];
#pragma unroll
    for (int j = 0; j < 2 * K; ++j) z[j] = 0.0f;
#pragma unroll
    for (int j = 0; j < K; ++j) ninf[j] = -__builtin_inff();
    for (int s = from + w0; s < T; s += wstep) {
      if (g) buf_st<2 * K>(z, brsrc(g + (size_t)s * U * 2, U * 8u), p0 * 8);
      if (go) buf_st<K>(z, brsrc(go + (size_t)s * U, U * 4u), p0 * 4);
      if (la) buf_st<K>(ninf, brsrc(la + (size_t)s * U, U * 4u), p0 * 4);
      if (lb) buf_st<K>(ninf, brsrc(lb + (size_t)s * U, U * 4u), p0 * 4);
    }
  };
  auto log_row = [&](float* dst, int s, const XRow<K>& r) {  // debug outputs (slow path)
    float v[K];
#pragma unroll
    for (int j = 0; j < K; ++j) v[j] = xf_log(xf{r.m[j], r.e[j]});
    buf_st<K>(v, brsrc(dst + (size_t)s * U, U * 4u), p0 * 4);
  };
  const float inf_loss = (a.flags & SSNT_FLAG_ZERO_INFINITY) ? 0.0f : __builtin_inff();
  if (!feasible) {
    if ((S > T || P > U || S < 0 || P < 0) && a.status && threadIdx.x == 0)
      atomicOr(a.status, kStatusBadLength);
    fill_rows(0, wave, nw);
    if (threadIdx.x == 0) a.loss[b] = inf_loss;
    return;
  }
  if (threadIdx.x < 32) reinterpret_cast<int*>(ctl)[threadIdx.x] = 0;
  for (int i = threadIdx.x; i < 64 * K; i += 64 * nw) zero[i] = xf_zero();
  __syncthreads();
  const int M = (S - 1) >> 1;

  if (ISO && (wave == 4 || wave == 5)) return;
  if (wave >= 2) {
    // ------------------------------ converter -----------------------------------------
    const int ci = (ISO && wave > 5) ? wave - 4 : wave - 2;
    const int d = ci / NC;  // 0 = forward stream, 1 = backward stream
    const int c = ci % NC;
    constexpr int D = conv_depth<K>();
    float* ring_d = rings + (size_t)d * R * slot_words;
    auto srow = [&](int r) { return min(max(d == 0 ? r : S - 1 - r, 0), T - 1); };
    auto load = [&](int r, Item<K, OBS>& it) {
      const int row = srow(r);
      buf_ld<2 * K>(it.lt, brsrc(lt + (size_t)row * U * 2, U * 8u), p0 * 8);
      if constexpr (OBS) {
        const int orow = min(row + 1, T - 1);
        buf_ld<K>(it.ob, brsrc(lo + (size_t)orow * U, U * 4u), p0 * 4);
      }
    };
    Item<K, OBS> pf[D];
#pragma unroll
    for (int i = 0; i < D; ++i) load(c + NC * i, pf[i]);
    int kseen = 0;
    unsigned long long cg_wait = 0, cg_n = 0;
    const unsigned long long cg_t0 = DIAG_T();
    const int nmine = (S - c + NC - 1) / NC;  // my stream rows: c, c+NC, ...
    for (int base = 0; base < nmine; base += D) {
#pragma unroll
      for (int i = 0; i < D; ++i) {
        const int k = base + i;
        if (k < nmine) {
          const int r = c + NC * k;
          const Item<K, OBS> it = pf[i];
          load(r + NC * D, pf[i]);
          XRow<K> E, Sh, O;
          convert<K, OBS>(it, P, lane, E, Sh);
          convert_obs<K, OBS>(it, P, lane, O);
          if (r - R >= kseen) {
            const unsigned long long t = DIAG_T();
            kseen = spin_geq(&ctl->kprog[d], r - R + 1, a.status);
            cg_wait += DIAG_T() - t;
            ++cg_n;
          }
          float* slot = ring_d + (size_t)(r % R) * slot_words;
          float v[4 * K];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            v[4 * j] = E.m[j];
            v[4 * j + 1] = __builtin_bit_cast(float, E.e[j]);
            v[4 * j + 2] = Sh.m[j];
            v[4 * j + 3] = __builtin_bit_cast(float, Sh.e[j]);
          }
          st_vec<4 * K>(act ? slot + 4 * p0 : reinterpret_cast<float*>(junk), v);
          if constexpr (OBS) {
            float o[2 * K];
            xrow_pack<K>(O, o);
            st_vec<2 * K>(act ? slot + es_words + 2 * p0 : reinterpret_cast<float*>(junk), o);
          }
          lds_release(&ctl->done[d][c], k + 1);
        }
      }
    }
#ifdef SSNT_DIAG
    if (c == 0 && lane == 0) {
      unsigned long long* dg = g_diag[b * 4 + 2 + d];
      dg[0] = DIAG_T() - cg_t0;
      dg[1] = cg_wait;
      dg[2] = cg_n;
      dg[5] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));  // HW_ID
    }
#else
    (void)cg_wait; (void)cg_n; (void)cg_t0;
#endif
    fill_rows(S, ci, 2 * NC);  // idle converters zero the rows beyond S
    return;
  }

  // ------------------------------ chains -------------------------------------------------
  __builtin_amdgcn_s_setprio(2);
  const bool fwd = (wave == 0);
  const int d = fwd ? 0 : 1;
  const float* ring_d = rings + (size_t)d * R * slot_words;
  unsigned long long dg_wait = 0, dg_n = 0, dg_cut = 0, dg_p1 = 0;
  const unsigned long long dg_t0 = DIAG_T();
  int ready = 0;  // stream rows known converted
  auto wait_row = [&](int r) {
    if (r < ready) return;
    int mn = 0x7fffffff;
    for (int c = 0; c < NC; ++c) {
      // converter c produced rows c, c+NC, ..., c+NC*(done-1): its first missing row c+NC*done
      const int need = (r - c + NC) / NC;
      int dn = lds_acquire(&ctl->done[d][c]);
      if (c + NC * dn <= r && need > 0) {
        const unsigned long long t = DIAG_T();
        dn = spin_geq<false>(&ctl->done[d][c], need, a.status);
        dg_wait += DIAG_T() - t;
        ++dg_n;
      }
      mn = min(mn, c + NC * dn);
    }
    ready = mn;
  };
  auto read_row = [&](int r, XRow<K>& E, XRow<K>& Sh, XRow<K>& O) {
    wait_row(r);
    const float* slot = ring_d + (size_t)(r % R) * slot_words;
    float v[4 * K];
    ld_vec<4 * K>(v, act ? slot + 4 * p0 : reinterpret_cast<const float*>(zero));
#pragma unroll
    for (int j = 0; j < K; ++j) {
      E.m[j] = v[4 * j];
      E.e[j] = act ? __builtin_bit_cast(int, v[4 * j + 1]) : XF_EZERO;
      Sh.m[j] = v[4 * j + 2];
      Sh.e[j] = act ? __builtin_bit_cast(int, v[4 * j + 3]) : XF_EZERO;
    }
    if constexpr (OBS) {
      float o[2 * K];
      ld_vec<2 * K>(o, act ? slot + es_words + 2 * p0 : reinterpret_cast<const float*>(zero));
      O = xrow_unpack<K>(o);
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        O.m[j] = 1.0f;
        O.e[j] = 0;
      }
    }
  };
  // slot of stream row r may be reused: the stored value data-depends on row r's slot contents
  // (x * 0.0f cannot be folded under IEEE), so the store issues only after those reads returned
  auto consumed = [&](int r, const XRow<K>& E) {
    lds_relaxed(&ctl->kprog[d], r + 1 + (int)(E.m[0] * 0.0f));
  };
  auto grad_row = [&](int s, const float* ge, const float* gs) {
    float v[2 * K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      v[2 * j] = ge[j];
      v[2 * j + 1] = gs[j];
    }
    buf_st<2 * K>(v, brsrc(g + (size_t)s * U * 2, U * 8u), p0 * 8);
  };
  auto bail = [&]() {  // Z == 0: release the converters, zero everything (chains only)
    lds_relaxed(&ctl->kprog[d], 0x3fffffff);
    fill_rows(0, wave, 2);
    if (threadIdx.x == 0) a.loss[b] = inf_loss;
  };

  XRow<K> X, E, Sh, O;
  if (fwd) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      X.m[j] = 0.0f;
      X.e[j] = XF_EZERO;
    }
    if (lane == 0) {
      if constexpr (OBS) {
        const xf o = xf_exp(lo[0], true);
        const xf n = xf_norm(o.m, o.e);
        X.m[0] = n.m;
        X.e[0] = n.e;
      } else {
        X.m[0] = 0.5f;
        X.e[0] = 1;
      }
    }
    store.store(0, X);
    if (la) log_row(la, 0, X);
    read_row(0, E, Sh, O);
    // ---- phase 1: alpha[1..M] ----
    for (int r = 0; r < M; ++r) {
      consumed(r, E);
      XRow<K> En, Shn, On, stay, shft;
      read_row(r + 1, En, Shn, On);  // one step ahead, off the serial chain
      alpha_step<K, OBS>(X, E, Sh, O, stay, shft);
      store.store(r + 1, X);
      if (la) log_row(la, r + 1, X);
      E = En;
      Sh = Shn;
      O = On;
    }
    dg_p1 = DIAG_T() - dg_t0;
    // ---- cut: Z = tree-sum over p of alpha[M][p] * beta[M][p] ----
    {
      const unsigned long long t = DIAG_T();
      spin_geq(&ctl->bm_ready, 1, a.status);
      dg_cut += DIAG_T() - t;
    }
    float wm[K];
    int we[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const xf cb = cutb[K * lane + j];
      wm[j] = X.m[j] * cb.m;
      we[j] = X.e[j] + cb.e;
    }
#pragma unroll
    for (int len = K; len > 1; len >>= 1) {
#pragma unroll
      for (int i = 0; i < len / 2; ++i) {
        const xf t = xf_add(wm[2 * i], we[2 * i], wm[2 * i + 1], we[2 * i + 1]);
        wm[i] = t.m;
        we[i] = t.e;
      }
    }
    xf z{wm[0], we[0]};
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const float om = __shfl_xor(z.m, off);
      const int oe = __shfl_xor(z.e, off);
      z = xf_add(z.m, z.e, om, oe);
    }
    if (lane == 0) ctl->z = z;
    lds_release(&ctl->z_ready, 1);
    if (z.m == 0.0f) {
      bail();
      return;
    }
    if (lane == 0) a.loss[b] = 0.0f - xf_log(z);
    const float izm = 1.0f / z.m;
    const int ize = -z.e;
    // ---- phase 2: transitions M..S-1 ----
    XRow<K> Bn = M + 1 < S ? store.load(M + 1) : XRow<K>{};
    for (int s = M; s < S; ++s) {
      consumed(s, E);
      const bool more = s + 1 < S;
      XRow<K> En, Shn, On, Bnn;
      if (more) read_row(s + 1, En, Shn, On);
      if (s + 2 < S) Bnn = store.load(s + 2);
      XRow<K> Q, R_;
      if (more) {
        entering<K, OBS>(Bn, O, Q, R_);
      } else {
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const bool last = term && (p0 + j) == P - 1;
          Q.m[j] = last ? 1.0f : 0.0f;
          Q.e[j] = last ? 0 : XF_EZERO;
          R_.m[j] = 0.0f;
          R_.e[j] = XF_EZERO;
        }
      }
      if constexpr (OBS) {
        const XRow<K> Bs = (s == M) ? xrow_unpack<K>(reinterpret_cast<const float*>(cutb + p0))
                                    : store.load(s);
        float gob[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
          gob[j] = xf_neg_post((X.m[j] * Bs.m[j]) * izm, X.e[j] + Bs.e[j] + ize);
        if (go) buf_st<K>(gob, brsrc(go + (size_t)s * U, U * 4u), p0 * 4);
      }
      XRow<K> stay, shft;
      XRow<K> Xn = X;
      alpha_step<K, OBS>(Xn, E, Sh, O, stay, shft);
      float ge[K], gs[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        ge[j] = xf_neg_post((stay.m[j] * Q.m[j]) * izm, stay.e[j] + Q.e[j] + ize);
        gs[j] = xf_neg_post((shft.m[j] * R_.m[j]) * izm, shft.e[j] + R_.e[j] + ize);
      }
      if (g) grad_row(s, ge, gs);
      if (more) {
        X = Xn;
        if (la) log_row(la, s + 1, X);
        E = En;
        Sh = Shn;
        O = On;
        Bn = Bnn;
      }
    }
  } else {
    // ---- backward chain: stream row r is lattice row S-1-r ----
    read_row(0, E, Sh, O);
#pragma unroll
    for (int j = 0; j < K; ++j) {  // terminal emit (src/lib.rs:187-195)
      const bool last = (p0 + j) == P - 1;
      xf v = term ? xf_norm(E.m[j], E.e[j]) : xf{0.5f, 1};
      X.m[j] = last ? v.m : 0.0f;
      X.e[j] = last ? v.e : XF_EZERO;
    }
    auto put_beta = [&](int s) {
      if (s > M) {
        store.store(s, X);
      } else {
        float v[2 * K];
        xrow_pack<K>(X, v);
        st_vec<2 * K>(reinterpret_cast<float*>(cutb + p0), v);
        lds_release(&ctl->bm_ready, 1);
      }
      if (lb) log_row(lb, s, X);
    };
    put_beta(S - 1);
    consumed(0, E);
    if (S > 1) read_row(1, E, Sh, O);
    // ---- phase 1: beta[S-2..M] ----
    for (int r = 1; r < S - M; ++r) {
      consumed(r, E);
      const int s = S - 1 - r;
      XRow<K> En, Shn, On, Q, R_;
      if (r + 1 < S) read_row(r + 1, En, Shn, On);
      entering<K, OBS>(X, O, Q, R_);
      beta_step<K>(X, E, Sh, Q, R_);
      put_beta(s);
      E = En;
      Sh = Shn;
      O = On;
    }
    dg_p1 = DIAG_T() - dg_t0;
    if (M > 0) {
      // ---- phase 2: transitions M-1..0 ----
      {
        const unsigned long long t = DIAG_T();
        spin_geq(&ctl->z_ready, 1, a.status);
        dg_cut += DIAG_T() - t;
      }
      const xf z = ctl->z;
      if (z.m == 0.0f) {
        bail();
        return;
      }
      const float izm = 1.0f / z.m;
      const int ize = -z.e;
      XRow<K> A = store.load(M - 1);
      for (int r = S - M; r < S; ++r) {  // transition s = S-1-r
        consumed(r, E);
        const int s = S - 1 - r;
        XRow<K> En, Shn, On, An;
        if (r + 1 < S) read_row(r + 1, En, Shn, On);
        if (s > 0) An = store.load(s - 1);
        XRow<K> Q, R_;
        entering<K, OBS>(X, O, Q, R_);
        float ge[K], gs[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
          ge[j] = xf_neg_post(((A.m[j] * E.m[j]) * Q.m[j]) * izm, A.e[j] + E.e[j] + Q.e[j] + ize);
          gs[j] = xf_neg_post(((A.m[j] * Sh.m[j]) * R_.m[j]) * izm, A.e[j] + Sh.e[j] + R_.e[j] + ize);
        }
        beta_step<K>(X, E, Sh, Q, R_);
        if constexpr (OBS) {
          float gob[K];
#pragma unroll
          for (int j = 0; j < K; ++j)
            gob[j] = xf_neg_post((A.m[j] * X.m[j]) * izm, A.e[j] + X.e[j] + ize);
          if (go) buf_st<K>(gob, brsrc(go + (size_t)s * U, U * 4u), p0 * 4);
        }
        if (g) grad_row(s, ge, gs);
        if (lb) log_row(lb, s, X);
        E = En;
        Sh = Shn;
        O = On;
        A = An;
      }
    }
  }
#ifdef SSNT_DIAG
  if (lane == 0) {
    unsigned long long* dg = g_diag[b * 4 + d];
    dg[0] = DIAG_T() - dg_t0;
    dg[1] = dg_wait;
    dg[2] = dg_n;
    dg[3] = dg_cut;
    dg[4] = dg_p1;
    dg[5] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));  // HW_ID
  }
#else
  (void)dg_wait; (void)dg_n; (void)dg_cut; (void)dg_p1; (void)dg_t0;
#endif
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <int K, bool OBS, bool LDS, bool VEC>
int launch_kernel(const FwdBwdArgs& a, size_t lds, hipStream_t st) {
  auto kern = k_fwd_bwd<K, OBS, LDS, VEC>;
  if (lds > 64 * 1024) {  // dynamic LDS above 64 KiB needs the attribute (idempotent)
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBudget);
      attr_set = true;
    }
  }
  hipLaunchKernelGGL(kern, dim3(a.B), dim3(128), lds, st, a);
  return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
}

template <int K, bool OBS>
int launch_k(const FwdBwdArgs& a, hipStream_t st) {
  const size_t head = (size_t)(64 * K + 2) * sizeof(xf);
  const size_t rows = (size_t)a.T * a.U * sizeof(xf);
  const bool lds = head + rows <= kLdsBudget;
  if (!lds && (a.workspace == nullptr || a.workspace_bytes < fwd_bwd_workspace_bytes(a.B, a.T, a.U)))
    return SSNT_ERR_WORKSPACE;
  // whole lane slices (U % K == 0) and 16-byte aligned tensors -> widest branch-free accesses
  const bool vec = (a.U % K == 0) && aligned16(a.log_trans) && aligned16(a.log_obs) &&
                   aligned16(a.grad) && aligned16(a.grad_obs) && aligned16(a.log_alpha) &&
                   aligned16(a.log_beta) && aligned16(a.workspace);
  const size_t shm = lds ? head + rows : head;
  if (lds)
    return vec ? launch_kernel<K, OBS, true, true>(a, shm, st) : launch_kernel<K, OBS, true, false>(a, shm, st);
  return vec ? launch_kernel<K, OBS, false, true>(a, shm, st) : launch_kernel<K, OBS, false, false>(a, shm, st);
}

constexpr int kPipeR = 8;   // ring slots per direction

inline size_t pipe_head_bytes(int K, int U, bool obs) {
  const size_t slot_words = (size_t)U * 4 + ((obs ? (size_t)U * 2 : 0) + 3) / 4 * 4;
  return sizeof(PipeCtl) + 3 * (size_t)64 * K * sizeof(xf) + 2 * (size_t)kPipeR * slot_words * 4;
}

template <int K, bool OBS, bool LDS, int NC, bool ISO>
int launch_pipe_kernel(const FwdBwdArgs& a, size_t lds, hipStream_t st) {
  auto kern = k_fwd_bwd_pipe<K, OBS, LDS, NC, kPipeR, ISO>;
  if (lds > 64 * 1024) {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBudget);
      attr_set = true;
    }
  }
  hipLaunchKernelGGL(kern, dim3(a.B), dim3(64 * (2 + 2 * NC + (ISO ? 2 : 0))), lds, st, a);
  return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
}

template <int K, bool OBS, int NC, bool ISO = false>
int launch_pipe(const FwdBwdArgs& a, hipStream_t st) {
  const bool vec = (a.U % K == 0) && aligned16(a.log_trans) && aligned16(a.log_obs) &&
                   aligned16(a.grad) && aligned16(a.grad_obs) && aligned16(a.log_alpha) &&
                   aligned16(a.log_beta) && aligned16(a.workspace);
  if (!vec) return launch_k<K, OBS>(a, st);  // odd shapes: the simple kernel
  const size_t head = pipe_head_bytes(K, a.U, OBS);
  const size_t rows = (size_t)a.T * a.U * sizeof(xf);
  if (head > kLdsBudget) return SSNT_ERR_UNSUPPORTED;
  const bool lds = head + rows <= kLdsBudget;
  if (!lds && (a.workspace == nullptr || a.workspace_bytes < (size_t)a.B * rows))
    return SSNT_ERR_WORKSPACE;
  return lds ? launch_pipe_kernel<K, OBS, true, NC, ISO>(a, head + rows, st)
             : launch_pipe_kernel<K, OBS, false, NC, ISO>(a, head, st);
}

// -1: not chosen yet (env SSNT_FWD_BWD_KERNEL), 0 pipelined (3 converters per direction),
// 1 simple two-wave kernel, 2 pipelined with 2 converters per direction
int g_variant = -1;

inline bool use_simple_kernel() {
  if (g_variant < 0) {
    const char* e = getenv("SSNT_FWD_BWD_KERNEL");
    g_variant = (e && strcmp(e, "simple") == 0) ? 1 : 0;
  }
  return g_variant == 1;
}

template <bool OBS>
int launch_obs(const FwdBwdArgs& a, hipStream_t st) {
  if (use_simple_kernel()) {
    if (a.U <= 64) return launch_k<1, OBS>(a, st);
    if (a.U <= 128) return launch_k<2, OBS>(a, st);
    if (a.U <= 256) return launch_k<4, OBS>(a, st);
    if (a.U <= 512) return launch_k<8, OBS>(a, st);
    return SSNT_ERR_UNSUPPORTED;
  }
  if (g_variant == 3) {
    if (a.U <= 64) return launch_pipe<1, OBS, 2, true>(a, st);
    if (a.U <= 128) return launch_pipe<2, OBS, 2, true>(a, st);
    if (a.U <= 256) return launch_pipe<4, OBS, 2, true>(a, st);
    if (a.U <= 512) return launch_pipe<8, OBS, 2, true>(a, st);
    return SSNT_ERR_UNSUPPORTED;
  }
  if (g_variant == 2) {
    if (a.U <= 64) return launch_pipe<1, OBS, 2>(a, st);
    if (a.U <= 128) return launch_pipe<2, OBS, 2>(a, st);
    if (a.U <= 256) return launch_pipe<4, OBS, 2>(a, st);
    if (a.U <= 512) return launch_pipe<8, OBS, 2>(a, st);
    return SSNT_ERR_UNSUPPORTED;
  }
  if (a.U <= 64) return launch_pipe<1, OBS, 3>(a, st);
  if (a.U <= 128) return launch_pipe<2, OBS, 3>(a, st);
  if (a.U <= 256) return launch_pipe<4, OBS, 3>(a, st);
  if (a.U <= 512) return launch_pipe<8, OBS, 3>(a, st);
  return SSNT_ERR_UNSUPPORTED;
}

}  // namespace

size_t fwd_bwd_workspace_bytes(int B, int T, int U) {
  // conservative over both kernels and with/without log_obs: rows go to global memory when
  // the largest LDS head plus T*U*8 bytes of rows does not fit
  const int K = U <= 64 ? 1 : U <= 128 ? 2 : U <= 256 ? 4 : 8;
  const size_t head = pipe_head_bytes(K, U, true);
  const size_t rows = (size_t)T * U * sizeof(xf);
  if (head + rows <= kLdsBudget) return 0;
  return (size_t)B * rows;
}

int diag_read(void* host, size_t bytes) {
#ifdef SSNT_DIAG
  if (bytes > sizeof(g_diag)) bytes = sizeof(g_diag);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? (int)bytes : -1;
#else
  (void)host;
  (void)bytes;
  return -1;
#endif
}

int set_fwd_bwd_variant(int v) {
  if (v < 0 || v > 3) return SSNT_ERR_INVALID_ARG;
  g_variant = v;
  return SSNT_OK;
}

int launch_fwd_bwd(const FwdBwdArgs& a, hipStream_t st) {
  if (a.B < 0 || a.T <= 0 || a.U <= 0 || !a.log_trans || !a.step_len || !a.pos_len || !a.loss)
    return SSNT_ERR_INVALID_ARG;
  if (a.grad_obs && !a.log_obs) return SSNT_ERR_INVALID_ARG;
  if (a.B == 0) return SSNT_OK;
  return a.log_obs ? launch_obs<true>(a, st) : launch_obs<false>(a, st);
}

}  // namespace ssnt
