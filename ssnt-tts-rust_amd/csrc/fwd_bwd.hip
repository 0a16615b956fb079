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
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>

#include "lattice_dev.h"

namespace ssnt {
namespace {

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
  int* __restrict__ lae = (la && a.log_alpha_e) ? a.log_alpha_e + (size_t)b * TU : nullptr;
  int* __restrict__ lbe = (lb && a.log_beta_e) ? a.log_beta_e + (size_t)b * TU : nullptr;
  const float dbg_zero = a.log_alpha_e ? 0.0f : -__builtin_inff();  // raw state: mantissa 0

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
        ninf[j] = dbg_zero;
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
    if (la) store_dbg_row<K, VEC>(la, lae, X, U, lane);
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
    if (lb) store_dbg_row<K, VEC>(lb + (size_t)s * U, lbe ? lbe + (size_t)s * U : nullptr, X, U, lane);
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
          if (la) store_dbg_row<K, VEC>(la + (size_t)(r + 1) * U, lae ? lae + (size_t)(r + 1) * U : nullptr, X, U, lane);
        } else {  // beta[s], s = S-1-r
          const int s = S - 1 - r;
          XRow<K> Q, R;
          entering<K, OBS>(X, O, Q, R);
          beta_step<K>(X, E, Sh, Q, R);
          if (s > M) store_row<K, VEC>(rows + (size_t)s * U, X, U, lane);
          else store_row<K, VEC>(cutb, X, 64 * K, lane);
          if (lb) store_dbg_row<K, VEC>(lb + (size_t)s * U, lbe ? lbe + (size_t)s * U : nullptr, X, U, lane);
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
  if (fwd && lane == 0) {
    a.loss[b] = 0.0f - xf_log(Z);
    if (a.z_state) {
      a.z_state[2 * b] = Z.m;
      a.z_state[2 * b + 1] = __builtin_bit_cast(float, Z.e);
    }
  }
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
            if (la) store_dbg_row<K, VEC>(la + (size_t)(s + 1) * U, lae ? lae + (size_t)(s + 1) * U : nullptr, X, U, lane);
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
          if (lb) store_dbg_row<K, VEC>(lb + (size_t)s * U, lbe ? lbe + (size_t)s * U : nullptr, X, U, lane);
        }
      }
    }
  }
  fill_rows(S);
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <int K, bool OBS, bool LDS, bool VEC>
int launch_kernel(const FwdBwdArgs& a, size_t lds, hipStream_t st) {
  auto kern = k_fwd_bwd<K, OBS, LDS, VEC>;
  note_fwd_bwd_dispatch("k_fwd_bwd<K=%d,OBS=%d,LDS=%d,VEC=%d>", K, (int)OBS, (int)LDS, (int)VEC);
  // dynamic LDS above 64 KiB needs the attribute; it is per device, so it is set on every such
  // launch (a host-side call, no device work) rather than cached in a process-wide flag
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBudget);
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
template <bool OBS>
int launch_simple(const FwdBwdArgs& a, hipStream_t st) {
  if (a.U <= 64) return launch_k<1, OBS>(a, st);
  if (a.U <= 128) return launch_k<2, OBS>(a, st);
  if (a.U <= 256) return launch_k<4, OBS>(a, st);
  if (a.U <= 512) return launch_k<8, OBS>(a, st);
  return SSNT_ERR_UNSUPPORTED;
}

// Kernel choice. The product dispatches by shape only (the streaming kernel, else the segmented
// kernel, else the two-wave kernel). The A/B build (-DSSNT_AB, `make lib-ab`; tests and tools
// only) adds a process-wide override: 1 two-wave kernel only, 2 segmented kernel;
// SSNT_FWD_BWD_KERNEL=simple selects 1 there. (The pair and rows kernels of rounds 2-4, both
// bit-exact and measured slower -- DESIGN.md 5.1a / 5.1c -- were retired to git history.)
#ifdef SSNT_AB
std::atomic<int> g_variant{0};
std::once_flag g_variant_env;
int variant() {
  std::call_once(g_variant_env, [] {
    const char* e = getenv("SSNT_FWD_BWD_KERNEL");
    if (e && strcmp(e, "simple") == 0) g_variant.store(1);
  });
  return g_variant.load(std::memory_order_relaxed);
}
#else
constexpr int variant() { return 0; }
#endif

thread_local char t_dispatch[160];

}  // namespace

void note_fwd_bwd_dispatch(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(t_dispatch, sizeof t_dispatch, fmt, ap);
  va_end(ap);
}
const char* last_fwd_bwd_dispatch() { return t_dispatch; }

size_t fwd_bwd_workspace_bytes(int B, int T, int U) {
  // 0 when the default dispatch keeps every row in LDS whatever the call brings: U <= 256, the
  // streaming kernel's rows fit beside its rings with or without log_obs and with the narrow
  // form's padded rows, and the two-wave kernel (what takes 4-byte-aligned tensors)
  // fits its rows too. (The A/B build's forced segmented kernel, pair kernel and deep rings
  // always get the workspace.)
  if (variant() == 0 && stream_ring() == 0 && U <= 256) {
    const int K = U <= 64 ? 1 : U <= 128 ? 2 : 4;
    const size_t Up = (size_t)K * ((U + K - 1) / K);
    const size_t rows = (size_t)T * Up * sizeof(xf);
    // (log_obs rings carry wider slots, the ones without more of them: take the larger head)
    const size_t h0 = stream_head_bytes(K, U, false), h1 = stream_head_bytes(K, U, true);
    const bool stream_lds = (h0 > h1 ? h0 : h1) + rows <= kLdsBudget;
    const bool simple_lds = (size_t)(64 * K + 2) * sizeof(xf) + (size_t)T * U * sizeof(xf) <= kLdsBudget;
    if (stream_lds && simple_lds) return 0;
  }
  // the segmented kernel keeps its rows (plus beta at the cut) in the workspace at every T; one
  // size serves every kernel (the two-wave kernel needs B*T*U xf at most; the streaming
  // kernel's narrow form pads rows to whole lane slices: U + 3 at most)
  const size_t wide = fwd_bwd_wide_workspace_bytes(B, T, U);
  const size_t stream = (size_t)B * T * ((size_t)U + 3) * sizeof(xf);
  return wide > stream ? wide : stream;
}

#ifdef SSNT_AB
int set_fwd_bwd_variant(int v) {
  // 0 default dispatch, 1 two-wave kernel, 2 segmented kernel at every U it takes
  if (v < 0 || v > 2) return SSNT_ERR_INVALID_ARG;
  variant();  // the environment is read once, before any explicit choice
  g_variant.store(v);
  return SSNT_OK;
}
#endif

namespace {
__global__ __launch_bounds__(64) void k_loss_sum(const float* loss, int B, float* out) {
  const float sum = wave_loss_sum(loss, B);
  if (threadIdx.x == 0) *out = sum;
}

int launch_variant(const FwdBwdArgs& a, hipStream_t st, bool& summed) {
  summed = false;
  if (variant() == 0) {
    FwdBwdArgs x = a;
    if (!a.sum_state) x.loss_sum = nullptr;
    int rc = launch_fwd_bwd_stream(x, st);
    summed = x.loss_sum != nullptr;
    if (rc != SSNT_ERR_UNSUPPORTED) return rc;
    summed = false;
    // long rows, and what the streaming kernel declines (4-byte-aligned log_trans / grad): the
    // segmented kernel takes any U <= 1024 at 8-byte alignment (loss sum: the separate pass)
    if (a.workspace && a.workspace_bytes >= fwd_bwd_wide_workspace_bytes(a.B, a.T, a.U)) {
      rc = launch_fwd_bwd_wide(a, st, true);
      if (rc != SSNT_ERR_UNSUPPORTED) return rc;
    }
  } else if (variant() == 2) {
    const int rc = launch_fwd_bwd_wide(a, st, true);
    if (rc != SSNT_ERR_UNSUPPORTED) return rc;
  }
  FwdBwdArgs x = a;
  x.loss_sum = nullptr;  // the two-wave kernel only writes loss[]
  return a.log_obs ? launch_simple<true>(x, st) : launch_simple<false>(x, st);
}
}  // namespace

// ---- float64 debug outputs (ssnt_fwd_bwd_debug64_device) -------------------------------------
// The kernels run in raw-state mode: mantissa / exponent planes of alpha and beta and Z per
// utterance land in the workspace; this pass forms e*ln2 + ln(m) in float64 (zero mantissa:
// -inf; loss: -ln Z, or the f32 kernel's +inf / 0 where Z was never formed or is 0).
__global__ __launch_bounds__(256) void k_debug64(const float* am, const int* ae, const float* bm,
                                                 const int* be, size_t n, double* la, double* lb,
                                                 const float* zs, const float* loss32, int B,
                                                 double* loss) {
  constexpr double kLn2 = 0x1.62e42fefa39efp-1;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (la) la[i] = am[i] == 0.0f ? -__builtin_inf() : (double)ae[i] * kLn2 + log((double)am[i]);
    if (lb) lb[i] = bm[i] == 0.0f ? -__builtin_inf() : (double)be[i] * kLn2 + log((double)bm[i]);
  }
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)B; i += stride) {
    const float zm = zs[2 * i];
    const int ze = __builtin_bit_cast(int, zs[2 * i + 1]);
    loss[i] = zm == 0.0f ? (double)loss32[i] : -((double)ze * kLn2 + log((double)zm));
  }
}

namespace {
inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

size_t fwd_bwd_debug64_workspace_bytes(int B, int T, int U) {
  const size_t cells = (size_t)B * T * U;
  return al256(fwd_bwd_workspace_bytes(B, T, U)) + 4 * al256(cells * 4) + al256((size_t)B * 8) +
         al256((size_t)B * 4);
}

int launch_fwd_bwd_debug64(const FwdBwdArgs& a0, double* loss64, double* la64, double* lb64,
                           hipStream_t st) {
  if (a0.B < 0 || a0.T <= 0 || a0.U <= 0 || !loss64 || a0.loss_sum) return SSNT_ERR_INVALID_ARG;
  if (a0.B == 0) return SSNT_OK;
  const size_t need = fwd_bwd_debug64_workspace_bytes(a0.B, a0.T, a0.U);
  if (!a0.workspace || a0.workspace_bytes < need) return SSNT_ERR_WORKSPACE;
  const size_t cells = (size_t)a0.B * a0.T * a0.U;
  const size_t base = fwd_bwd_workspace_bytes(a0.B, a0.T, a0.U);
  unsigned char* w = static_cast<unsigned char*>(a0.workspace);
  size_t off = al256(base);
  auto take = [&](size_t bytes) { unsigned char* p = w + off; off += al256(bytes); return p; };
  float* am = reinterpret_cast<float*>(take(cells * 4));
  int* ae = reinterpret_cast<int*>(take(cells * 4));
  float* bm = reinterpret_cast<float*>(take(cells * 4));
  int* be = reinterpret_cast<int*>(take(cells * 4));
  float* zs = reinterpret_cast<float*>(take((size_t)a0.B * 8));
  float* l32 = reinterpret_cast<float*>(take((size_t)a0.B * 4));
  FwdBwdArgs a = a0;
  a.workspace = base ? a0.workspace : nullptr;  // the product dispatch sees the plain call's workspace
  a.workspace_bytes = base;
  a.loss = l32;
  a.log_alpha = am;
  a.log_beta = bm;
  a.log_alpha_e = ae;
  a.log_beta_e = be;
  a.z_state = zs;
  if (hipMemsetAsync(zs, 0, (size_t)a.B * 8, st) != hipSuccess) return SSNT_ERR_HIP;
  int rc = launch_fwd_bwd(a, st);
  if (rc != SSNT_OK) return rc;
  const size_t n = la64 || lb64 ? cells : 0;
  const int blocks = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 + 1 : 4096);
  hipLaunchKernelGGL(k_debug64, dim3(blocks), dim3(256), 0, st, am, ae, bm, be, n, la64, lb64, zs,
                     l32, a.B, loss64);
  return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
}

size_t fwd_bwd_sum_state_bytes(int B) { return kSumGranuleOffset + 8 * (size_t)(B > 0 ? B : 0); }

int launch_fwd_bwd(const FwdBwdArgs& a, hipStream_t st) {
  t_dispatch[0] = 0;  // (an argument error or an empty batch dispatches nothing)
  if (a.B < 0 || a.T <= 0 || a.U <= 0 || !a.log_trans || !a.step_len || !a.pos_len || !a.loss)
    return SSNT_ERR_INVALID_ARG;
  if (a.grad_obs && !a.log_obs) return SSNT_ERR_INVALID_ARG;
  if (a.B == 0) {
    if (a.loss_sum) return hipMemsetAsync(a.loss_sum, 0, sizeof(float), st) == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
    return SSNT_OK;
  }
  // batch loss sum: inside the streaming kernel when the caller gives a sum state, else one
  // extra single-wave pass over loss[] (same fixed order, same bits)
  bool summed = false;
  const int rc = launch_variant(a, st, summed);
  if (rc != SSNT_OK || !a.loss_sum || summed) return rc;
  const size_t n = strlen(t_dispatch);
  snprintf(t_dispatch + n, sizeof t_dispatch - n, "+k_loss_sum");
  hipLaunchKernelGGL(k_loss_sum, dim3(1), dim3(64), 0, st, a.loss, a.B, a.loss_sum);
  return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
}

}  // namespace ssnt
