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

#include "ssnt_internal.h"
#include "xf_math.h"

namespace ssnt {
namespace {

constexpr int kRing = 4;             // input prefetch depth (rows)
constexpr size_t kLdsBudget = 150 * 1024;

__device__ __forceinline__ float shr1(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ int shr1(int x) {
  return __builtin_amdgcn_update_dpp(0, x, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ float shl1(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x130, 0xf, 0xf, false));
}
__device__ __forceinline__ int shl1(int x) {
  return __builtin_amdgcn_update_dpp(0, x, 0x130, 0xf, 0xf, false);
}

template <int K, bool OBS>
struct Item {
  float lt[2 * K];
  float ob[OBS ? K : 1];
};

// Load lane's slice of lt row `row` (and obs row `orow`) with rows clamped into [0,T).
template <int K, bool OBS>
__device__ __forceinline__ Item<K, OBS> load_item(const float* __restrict__ lt,
                                                  const float* __restrict__ lo, int row,
                                                  int orow, int T, int U, int lane) {
  Item<K, OBS> it;
  row = min(max(row, 0), T - 1);
  const int p0 = K * lane;
  const float2* src = reinterpret_cast<const float2*>(lt + ((size_t)row * U + p0) * 2);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    float2 v = make_float2(0.0f, 0.0f);
    if (p0 + j < U) v = src[j];
    it.lt[2 * j] = v.x;
    it.lt[2 * j + 1] = v.y;
  }
  if constexpr (OBS) {
    orow = min(max(orow, 0), T - 1);
    const float* osrc = lo + (size_t)orow * U + p0;
#pragma unroll
    for (int j = 0; j < K; ++j) it.ob[j] = (p0 + j < U) ? osrc[j] : 0.0f;
  }
  return it;
}

template <int K>
struct XRow {
  float m[K];
  int e[K];
};

template <int K>
__device__ __forceinline__ void store_row(xf* __restrict__ dst, const XRow<K>& r, int U, int lane) {
  const int p0 = K * lane;
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (p0 + j < U) dst[p0 + j] = xf{r.m[j], r.e[j]};
}

template <int K>
__device__ __forceinline__ XRow<K> load_row(const xf* __restrict__ src, int U, int lane) {
  XRow<K> r;
  const int p0 = K * lane;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    xf v = xf_zero();
    if (p0 + j < U) v = src[p0 + j];
    r.m[j] = v.m;
    r.e[j] = v.e;
  }
  return r;
}

template <int K>
__device__ __forceinline__ void store_grad_row(float* __restrict__ g, const float* ge,
                                               const float* gs, int U, int lane) {
  const int p0 = K * lane;
  float2* dst = reinterpret_cast<float2*>(g + (size_t)p0 * 2);
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (p0 + j < U) dst[j] = make_float2(ge[j], gs[j]);
}

template <int K>
__device__ __forceinline__ void store_f_row(float* __restrict__ dst, const float* v, int U, int lane) {
  const int p0 = K * lane;
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (p0 + j < U) dst[p0 + j] = v[j];
}

template <int K>
__device__ __forceinline__ void store_log_row(float* __restrict__ dst, const XRow<K>& r, int U, int lane) {
  float v[K];
#pragma unroll
  for (int j = 0; j < K; ++j) v[j] = xf_log(xf{r.m[j], r.e[j]});
  store_f_row<K>(dst, v, U, lane);
}

// Convert the lane's inputs of one row to xf: emit E, shift S (masked: p<P, shift p<P-1).
template <int K, bool OBS>
__device__ __forceinline__ void convert(const Item<K, OBS>& it, int P, int lane, XRow<K>& E,
                                        XRow<K>& Sh) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int p = K * lane + j;
    const xf e = xf_exp(it.lt[2 * j], p < P);
    const xf s = xf_exp(it.lt[2 * j + 1], p < P - 1);
    E.m[j] = e.m;
    E.e[j] = e.e;
    Sh.m[j] = s.m;
    Sh.e[j] = s.e;
  }
}

template <int K, bool OBS>
__device__ __forceinline__ void convert_obs(const Item<K, OBS>& it, int P, int lane, XRow<K>& O) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if constexpr (OBS) {
      const xf o = xf_exp(it.ob[j], K * lane + j < P);
      O.m[j] = o.m;
      O.e[j] = o.e;
    } else {
      O.m[j] = 1.0f;
      O.e[j] = 0;
    }
  }
}

// alpha[s+1] from alpha[s]: stay/shift products (returned for reuse by the gradients).
template <int K, bool OBS>
__device__ __forceinline__ void alpha_step(XRow<K>& A, const XRow<K>& E, const XRow<K>& Sh,
                                           const XRow<K>& O, int lane, XRow<K>& stay,
                                           XRow<K>& shft) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    stay.m[j] = A.m[j] * E.m[j];
    stay.e[j] = A.e[j] + E.e[j];
    shft.m[j] = A.m[j] * Sh.m[j];
    shft.e[j] = A.e[j] + Sh.e[j];
  }
  float lm = shr1(shft.m[K - 1]);
  int le = shr1(shft.e[K - 1]);
  if (lane == 0) {
    lm = 0.0f;
    le = XF_EZERO;
  }
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
__device__ __forceinline__ void entering(const XRow<K>& Bn, const XRow<K>& O, int lane, XRow<K>& Q,
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
  float rm = shl1(Q.m[0]);
  int re = shl1(Q.e[0]);
  if (lane == 63) {
    rm = 0.0f;
    re = XF_EZERO;
  }
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

template <int K, bool OBS, bool LDS>
__global__ __launch_bounds__(128) void k_fwd_bwd(FwdBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int wave = threadIdx.x >> 6;
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
      if (g) store_grad_row<K>(g + (size_t)s * U * 2, z, z, U, lane);
      if (go) store_f_row<K>(go + (size_t)s * U, z, U, lane);
      if (la) store_f_row<K>(la + (size_t)s * U, ninf, U, lane);
      if (lb) store_f_row<K>(lb + (size_t)s * U, ninf, U, lane);
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
    ring[i] = load_item<K, OBS>(lt, lo, row, row + 1, T, U, lane);
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
    store_row<K>(rows, X, U, lane);
    if (la) store_log_row<K>(la, X, U, lane);
  }
  const int r0 = fwd ? 0 : 1;               // bwd consumes stream slot 0 for its init
  const int r1 = fwd ? M : S - M;           // phase-1 end (exclusive)
  // bwd init uses ring slot 0 (row S-1)
  if (!fwd) {
    const Item<K, OBS> it = ring[0];
    ring[0] = load_item<K, OBS>(lt, lo, srow(kRing), srow(kRing) + 1, T, U, lane);
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
    if (s > M) store_row<K>(rows + (size_t)s * U, X, U, lane);
    else store_row<K>(cutb, X, 64 * K, lane);
    if (lb) store_log_row<K>(lb + (size_t)s * U, X, U, lane);
  }
  // ---------------- phase 1 ----------------
  for (int base = (r0 / kRing) * kRing; base < r1; base += kRing) {
#pragma unroll
    for (int i = 0; i < kRing; ++i) {
      const int r = base + i;
      if (r >= r0 && r < r1) {
        const Item<K, OBS> it = ring[i];
        const int nr = srow(r + kRing);
        ring[i] = load_item<K, OBS>(lt, lo, nr, nr + 1, T, U, lane);
        XRow<K> E, Sh, O;
        convert<K, OBS>(it, P, lane, E, Sh);
        convert_obs<K, OBS>(it, P, lane, O);
        if (fwd) {  // alpha[r+1]
          XRow<K> stay, shft;
          alpha_step<K, OBS>(X, E, Sh, O, lane, stay, shft);
          store_row<K>(rows + (size_t)(r + 1) * U, X, U, lane);
          if (la) store_log_row<K>(la + (size_t)(r + 1) * U, X, U, lane);
        } else {  // beta[s], s = S-1-r
          const int s = S - 1 - r;
          XRow<K> Q, R;
          entering<K, OBS>(X, O, lane, Q, R);
          beta_step<K>(X, E, Sh, Q, R);
          if (s > M) store_row<K>(rows + (size_t)s * U, X, U, lane);
          else store_row<K>(cutb, X, 64 * K, lane);
          if (lb) store_log_row<K>(lb + (size_t)s * U, X, U, lane);
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
        ring[i] = load_item<K, OBS>(lt, lo, nr, nr + 1, T, U, lane);
        XRow<K> E, Sh, O;
        convert<K, OBS>(it, P, lane, E, Sh);
        convert_obs<K, OBS>(it, P, lane, O);
        float ge[K], gs[K], gob[K];
        if (fwd) {
          const int s = r;  // transition s: alpha[s] (X) -> row s+1
          XRow<K> Q, R;
          if (s + 1 < S) {
            const XRow<K> Bn = load_row<K>(rows + (size_t)(s + 1) * U, U, lane);
            entering<K, OBS>(Bn, O, lane, Q, R);
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
            const XRow<K> Bs = (s == M) ? load_row<K>(cutb, 64 * K, lane)
                                        : load_row<K>(rows + (size_t)s * U, U, lane);
#pragma unroll
            for (int j = 0; j < K; ++j)
              gob[j] = xf_neg_post((X.m[j] * Bs.m[j]) * izm, X.e[j] + Bs.e[j] + ize);
          }
          XRow<K> stay, shft;
          XRow<K> Xn = X;
          alpha_step<K, OBS>(Xn, E, Sh, O, lane, stay, shft);  // (stay/shft of alpha[s])
#pragma unroll
          for (int j = 0; j < K; ++j) {
            ge[j] = xf_neg_post((stay.m[j] * Q.m[j]) * izm, stay.e[j] + Q.e[j] + ize);
            gs[j] = xf_neg_post((shft.m[j] * R.m[j]) * izm, shft.e[j] + R.e[j] + ize);
          }
          if (g) store_grad_row<K>(g + (size_t)s * U * 2, ge, gs, U, lane);
          if constexpr (OBS) {
            if (go) store_f_row<K>(go + (size_t)s * U, gob, U, lane);
          }
          if (s + 1 < S) {
            X = Xn;
            if (la) store_log_row<K>(la + (size_t)(s + 1) * U, X, U, lane);
          }
        } else {
          const int s = S - 1 - r;  // transition s: beta[s+1] (X) -> beta[s]
          XRow<K> Q, R;
          entering<K, OBS>(X, O, lane, Q, R);
          const XRow<K> A = load_row<K>(rows + (size_t)s * U, U, lane);
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
            if (go) store_f_row<K>(go + (size_t)s * U, gob, U, lane);
          }
          if (g) store_grad_row<K>(g + (size_t)s * U * 2, ge, gs, U, lane);
          if (lb) store_log_row<K>(lb + (size_t)s * U, X, U, lane);
        }
      }
    }
  }
  fill_rows(S);
}

template <int K, bool OBS>
int launch_k(const FwdBwdArgs& a, hipStream_t st) {
  const size_t head = (size_t)(64 * K + 2) * sizeof(xf);
  const size_t rows = (size_t)a.T * a.U * sizeof(xf);
  if (head + rows <= kLdsBudget) {
    const size_t lds = head + rows;
    auto kern = k_fwd_bwd<K, OBS, true>;
    static bool attr_set = false;  // dynamic LDS above 64 KiB needs the attribute
    if (!attr_set) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBudget);
      attr_set = true;
    }
    hipLaunchKernelGGL(kern, dim3(a.B), dim3(128), lds, st, a);
  } else {
    if (a.workspace == nullptr || a.workspace_bytes < fwd_bwd_workspace_bytes(a.B, a.T, a.U))
      return SSNT_ERR_WORKSPACE;
    hipLaunchKernelGGL((k_fwd_bwd<K, OBS, false>), dim3(a.B), dim3(128), head, st, a);
  }
  return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
}

template <bool OBS>
int launch_obs(const FwdBwdArgs& a, hipStream_t st) {
  if (a.U <= 64) return launch_k<1, OBS>(a, st);
  if (a.U <= 128) return launch_k<2, OBS>(a, st);
  if (a.U <= 256) return launch_k<4, OBS>(a, st);
  if (a.U <= 512) return launch_k<8, OBS>(a, st);
  if (a.U <= 1024) return launch_k<16, OBS>(a, st);
  return SSNT_ERR_UNSUPPORTED;
}

}  // namespace

size_t fwd_bwd_workspace_bytes(int B, int T, int U) {
  const int K = U <= 64 ? 1 : U <= 128 ? 2 : U <= 256 ? 4 : U <= 512 ? 8 : 16;
  const size_t head = (size_t)(64 * K + 2) * sizeof(xf);
  const size_t rows = (size_t)T * U * sizeof(xf);
  if (head + rows <= kLdsBudget) return 0;
  return (size_t)B * rows;
}

int launch_fwd_bwd(const FwdBwdArgs& a, hipStream_t st) {
  if (a.B < 0 || a.T <= 0 || a.U <= 0 || !a.log_trans || !a.step_len || !a.pos_len || !a.loss)
    return SSNT_ERR_INVALID_ARG;
  if (a.grad_obs && !a.log_obs) return SSNT_ERR_INVALID_ARG;
  if (a.B == 0) return SSNT_OK;
  return a.log_obs ? launch_obs<true>(a, st) : launch_obs<false>(a, st);
}

}  // namespace ssnt
