// fwd_bwd_wide.hip -- lattice forward-backward for long rows (256 < U <= 512: BASELINE
// configs[4], B=64 T=2000 U=400) on gfx950.
//
// Same lattice and the same split-exponent arithmetic as fwd_bwd.hip / fwd_bwd_stream.hip
// (DESIGN.md "Lattice semantics"); bit-exact with oracle/ssnt_oracle.c. What differs is the
// decomposition, shaped by two facts of the long form: a row of U=400 positions is too wide for
// one wave's chain step (K = 8 positions per lane made the two-wave kernel's step ~1.3 us), and
// 64 utterances leave three quarters of the 256 CUs idle with one workgroup per utterance.
//
//   * One workgroup per (utterance, direction): 2B workgroups (128 at configs[4]).
//   * A direction's chain is split over NW waves, wave w owning positions [128w, 128w+128)
//     (2 per lane). The recurrence's only cross-segment dependency -- alpha needs the left
//     neighbour's shift product, beta the right neighbour's entering product -- is handed over
//     through an LDS ring, one 8-byte xf per step, in blocks of kBS steps: the downstream wave
//     runs a block behind the upstream one (a pipeline, not a per-step round trip).
//   * Each wave loads its own log_trans rows (kDepth rows in flight), converts them, steps the
//     chain, and writes its rows / gradients: one wave per SIMD, nothing shared but the ring.
//   * Two launches, split at the cut M = (S-1)>>1 (so no workgroup ever waits for another):
//       phase 1: alpha[0..M] and beta[S-1..M] to the workspace (rows of xf; beta[M] in row T);
//       phase 2: both form Z = sum_p alpha[M][p] beta[M][p] (the oracle's binary tree); the
//       alpha workgroup continues M..S-1 emitting the gradient rows s >= M (beta[s+1] read
//       back), the beta workgroup continues M-1..0 emitting rows s < M (alpha[s] read back).
//     The kernel boundary between them is the only inter-workgroup synchronisation.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "lattice_dev.h"

namespace ssnt {
namespace {

constexpr int kSeg = 128;      // positions per wave (2 per lane)
constexpr int kBS = 8;         // steps per hand-off block (= prefetch depth: ring indices static)
constexpr int kRB = 32;        // hand-off ring slots (steps) per wave
constexpr int kDepth = kBS;    // rows in flight per wave
constexpr int kMaxNW = 4;      // waves per direction: U <= 512
constexpr int kSpinMax = 1 << 22;

struct WideCtl {
  int prod[kMaxNW];     // steps whose hand-off value wave w has written
  int cons[kMaxNW];     // steps of its upstream ring wave w has read
  xf zpart[kMaxNW];     // per-segment sums of alpha[M] * beta[M]
  xf z;
  xf bnd[kMaxNW][kRB];  // hand-off rings
};

// compile-time loop: f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>)
template <typename F, int... I>
__device__ __forceinline__ void wfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  wfor_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ int wctr_ld(const int* p) {
  return __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void wctr_st(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// compiler-only barrier: LDS data and counter accesses stay in program order (a wave's DS
// instructions execute in order, so "write data, then counter" publishes without a wait)
__device__ __forceinline__ void wbar() { asm volatile("" ::: "memory"); }

// spin until *p >= target (bounded; an expired bound sets kStatusTimeout and gives up)
__device__ __forceinline__ void wait_ge(const int* p, int target, int* status) {
  if (wctr_ld(p) >= target) return;
  for (int n = 0; wctr_ld(p) < target; ++n) {
    if (n > kSpinMax) {
      if (status && (threadIdx.x & 63) == 0) atomicOr(status, kStatusTimeout);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

struct WItem {  // one row's inputs for this lane's two positions
  float lt[4];  // emit/shift of p0, p0+1
  float ob[2];  // log_obs of the entering row (OBS)
};
struct WRows {  // phase-2 workspace rows for this lane
  float r0[4];  // alpha: beta[s+1]; beta: alpha[s]        (m, e, m, e)
  float r1[4];  // alpha: beta[s] (grad_obs)
  float nb[2];  // alpha: beta[s+1] at p0+2 (lane 63: next segment's first position)
  float nob;    // alpha: log_obs[s+1] at p0+2
};

template <bool OBS, int PHASE>
__global__ __launch_bounds__(64 * kMaxNW) void k_fwd_bwd_wide(FwdBwdArgs a) {
  __shared__ WideCtl ctl;
  const int b = blockIdx.x;
  const int dir = blockIdx.y;  // 0 alpha, 1 beta
  const int NW = blockDim.x >> 6;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int T = a.T, U = a.U;
  // lengths are wave-uniform: every buffer descriptor built from them must live in SGPRs (a
  // VGPR base turns each buffer access into a readfirstlane waterfall loop)
  const int S = __builtin_amdgcn_readfirstlane(a.step_len[b]);
  const int P = __builtin_amdgcn_readfirstlane(a.pos_len[b]);
  const bool term = (a.flags & SSNT_FLAG_TERMINAL_EMIT) != 0;
  const size_t TU = (size_t)T * U;
  const float* lt = a.log_trans + (size_t)b * TU * 2;
  const float* lo = OBS ? a.log_obs + (size_t)b * TU : nullptr;
  float* g = a.grad ? a.grad + (size_t)b * TU * 2 : nullptr;
  float* go = (OBS && a.grad_obs) ? a.grad_obs + (size_t)b * TU : nullptr;
  float* la = a.log_alpha ? a.log_alpha + (size_t)b * TU : nullptr;
  float* lb = a.log_beta ? a.log_beta + (size_t)b * TU : nullptr;
  xf* rows = reinterpret_cast<xf*>(a.workspace) + (size_t)b * (T + 1) * U;  // row T: beta[M]
  const int p0 = kSeg * w + 2 * lane;
  const unsigned rowb = (unsigned)U * 8u, rowf = (unsigned)U * 4u;

  if (threadIdx.x < 2 * kMaxNW) reinterpret_cast<int*>(&ctl)[threadIdx.x] = 0;
  __syncthreads();

  // ---- row helpers (8-byte granules: any U, rows only 8-byte aligned). Row indices are
  // wave-uniform; readfirstlane says so to the compiler, so the descriptors stay in SGPRs.
  auto uni = [](int x) __attribute__((always_inline)) { return __builtin_amdgcn_readfirstlane(x); };
  auto st_pair = [&](float* base, unsigned bytes, int off, float x0, float x1) __attribute__((always_inline)) {
    rbuf_st2(f32x2{x0, x1}, brsrc(base, bytes), off, 0, 0);
  };
  auto put_grad = [&](int s, const float* ge, const float* gs) __attribute__((always_inline)) {
    if (!g) return;
    float* row = g + (size_t)uni(s) * U * 2;
    st_pair(row, rowb, p0 * 8, ge[0], gs[0]);
    st_pair(row, rowb, p0 * 8 + 8, ge[1], gs[1]);
  };
  auto put_f = [&](float* base, int s, const float* v) __attribute__((always_inline)) {  // grad_obs / debug rows
    const __amdgpu_buffer_rsrc_t r = brsrc(base + (size_t)uni(s) * U, rowf);
    rbuf_st1(v[0], r, p0 * 4, 0, 0);
    rbuf_st1(v[1], r, p0 * 4 + 4, 0, 0);
  };
  auto put_log = [&](float* base, int s, const XRow<2>& x) __attribute__((always_inline)) {
    const float v[2] = {xf_log(xf{x.m[0], x.e[0]}), xf_log(xf{x.m[1], x.e[1]})};
    put_f(base, s, v);
  };
  // workspace row s (s == T: the cut row). The fields go through registers one by one: a vector
  // built straight from the adjacent fields of the row makes the compiler keep the row in memory
  auto put_row = [&](int s, const XRow<2>& x) __attribute__((always_inline)) {
    float m0 = x.m[0], m1 = x.m[1];
    int e0 = x.e[0], e1 = x.e[1];
    asm volatile("" : "+v"(m0), "+v"(m1), "+v"(e0), "+v"(e1));
    const __amdgpu_buffer_rsrc_t r = brsrc(rows + (size_t)uni(s) * U, rowb);
    rbuf_st2(f32x2{m0, __builtin_bit_cast(float, e0)}, r, p0 * 8, 0, 0);
    rbuf_st2(f32x2{m1, __builtin_bit_cast(float, e1)}, r, p0 * 8 + 8, 0, 0);
  };
  auto ld_row = [&](int s, float* v) __attribute__((always_inline)) {  // 4 floats; past U: zeros (exponent fixed by callers)
    const __amdgpu_buffer_rsrc_t r = brsrc(rows + (size_t)uni(s) * U, rowb);
    const f32x2 x = rbuf_ld2(r, p0 * 8, 0, 0), y = rbuf_ld2(r, p0 * 8 + 8, 0, 0);
    v[0] = x.x; v[1] = x.y; v[2] = y.x; v[3] = y.y;
  };
  auto unpack = [&](const float* v) __attribute__((always_inline)) {
    XRow<2> x;
    x.m[0] = v[0]; x.e[0] = __builtin_bit_cast(int, v[1]);
    x.m[1] = v[2]; x.e[1] = __builtin_bit_cast(int, v[3]);
    return x;
  };
  // zero gradients, -inf debug rows (rows [from, to)); each wave writes its own segment
  auto zero_rows = [&](int from, int to) __attribute__((always_inline)) {
    const float z[2] = {0.0f, 0.0f}, ninf[2] = {-__builtin_inff(), -__builtin_inff()};
    for (int s = from; s < to; ++s) {
      put_grad(s, z, z);
      if (go) put_f(go, s, z);
      if (la) put_f(la, s, ninf);
      if (lb) put_f(lb, s, ninf);
    }
  };
  const float inf_loss = (a.flags & SSNT_FLAG_ZERO_INFINITY) ? 0.0f : __builtin_inff();
  const bool feasible = S >= 1 && P >= 1 && S <= T && P <= U && S >= P;
  if (!feasible) {
    if (PHASE == 2 && dir == 0) {
      if ((S > T || P > U || S < 0 || P < 0) && a.status && threadIdx.x == 0)
        atomicOr(a.status, kStatusBadLength);
      zero_rows(0, T);
      if (threadIdx.x == 0) a.loss[b] = inf_loss;
    }
    return;
  }
  const int M = (S - 1) >> 1;

  auto load_item = [&](int row, WItem& it) __attribute__((always_inline)) {
    row = uni(min(max(row, 0), T - 1));
    const __amdgpu_buffer_rsrc_t r = brsrc(lt + (size_t)row * U * 2, rowb);
    const f32x2 x = rbuf_ld2(r, p0 * 8, 0, 0), y = rbuf_ld2(r, p0 * 8 + 8, 0, 0);
    it.lt[0] = x.x; it.lt[1] = x.y; it.lt[2] = y.x; it.lt[3] = y.y;
    if constexpr (OBS) {
      const __amdgpu_buffer_rsrc_t o = brsrc(lo + (size_t)uni(min(row + 1, T - 1)) * U, rowf);
      it.ob[0] = rbuf_ld1(o, p0 * 4, 0, 0);
      it.ob[1] = rbuf_ld1(o, p0 * 4 + 4, 0, 0);
    }
  };
  auto convert2 = [&](const WItem& it, XRow<2>& E, XRow<2>& Sh, XRow<2>& O) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      xf_exp_pair(it.lt[2 * j], it.lt[2 * j + 1], p0 + j < P, p0 + j < P - 1, E.m[j], E.e[j],
                  Sh.m[j], Sh.e[j]);
    if constexpr (OBS) {
      xf_exp_pair(it.ob[0], it.ob[1], p0 < P, p0 + 1 < P, O.m[0], O.e[0], O.m[1], O.e[1]);
    } else {
      O.m[0] = O.m[1] = 1.0f;
      O.e[0] = O.e[1] = 0;
    }
  };

  // ---- the hand-off pipeline: up = the wave whose boundary value this wave needs
  const int up = dir == 0 ? w - 1 : w + 1;
  const int dn = dir == 0 ? w + 1 : w - 1;
  const bool has_up = up >= 0 && up < NW;
  const bool has_dn = dn >= 0 && dn < NW;
  const int pub_lane = dir == 0 ? 63 : 0;
  // n iterations in blocks of kBS; step(i, K, bm, be, pm, pe) with K = i % kBS a compile-time
  // constant (register ring indices), (bm, be) the upstream value of iteration i and (pm, pe)
  // the value this wave hands on. The downstream wave runs at least one block behind.
  auto pipeline = [&](int n, auto&& step) __attribute__((always_inline)) {
    for (int i0 = 0; i0 < n; i0 += kBS) {
      const int i1 = min(i0 + kBS, n);
      float bm[kBS];
      int be[kBS];
      if (has_up) {
        wait_ge(&ctl.prod[up], i1, a.status);
        wbar();
#pragma unroll
        for (int k = 0; k < kBS; ++k) {
          const xf v = ctl.bnd[up][(i0 + k) % kRB];
          bm[k] = v.m;
          be[k] = v.e;
        }
      } else {
#pragma unroll
        for (int k = 0; k < kBS; ++k) {
          bm[k] = 0.0f;
          be[k] = XF_EZERO;
        }
      }
      if (has_dn) wait_ge(&ctl.cons[dn], i1 - kRB, a.status);
      wbar();
      sfor<kBS>([&](auto Kc) __attribute__((always_inline)) {
        constexpr int k = decltype(Kc)::value;
        if (i0 + k < i1) {
          float pm;
          int pe;
          step(i0 + k, Kc, bm[k], be[k], pm, pe);
          if (has_dn && lane == pub_lane) ctl.bnd[w][(i0 + k) % kRB] = xf{pm, pe};
        }
      });
      wbar();
      if (has_dn) wctr_st(&ctl.prod[w], i1);
      if (has_up) wctr_st(&ctl.cons[w], i1);
    }
  };

  // alpha[r+1] from alpha[r] (= A); (bm, be): the left segment's shift product of its last
  // position; hands on this segment's. The operations of lattice_dev.h alpha_step.
  auto alpha_next = [&](XRow<2>& A, const XRow<2>& E, const XRow<2>& Sh, const XRow<2>& O,
                        float bm, int be, float& pm, int& pe) __attribute__((always_inline)) {
    XRow<2> st, sh;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      st.m[j] = A.m[j] * E.m[j];
      st.e[j] = A.e[j] + E.e[j];
      sh.m[j] = A.m[j] * Sh.m[j];
      sh.e[j] = A.e[j] + Sh.e[j];
    }
    pm = sh.m[1];
    pe = sh.e[1];
    float lm = shr1(sh.m[1]);
    int le = shr1(sh.e[1]);
    lm = lane == 0 ? bm : lm;
    le = lane == 0 ? be : le;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float hm = j == 0 ? lm : sh.m[0];
      const int he = j == 0 ? le : sh.e[0];
      const int em = max(st.e[j], he);
      float sum = xldexp(st.m[j], st.e[j] - em) + xldexp(hm, he - em);
      int ee = em;
      if constexpr (OBS) {
        sum = sum * O.m[j];
        ee = ee + O.e[j];
      }
      const xf r = xf_norm(sum, ee);
      A.m[j] = r.m;
      A.e[j] = r.e;
    }
  };
  // Q = beta[s+1] (x obs[s+1]) and R = Q[p+1]; (bm, be): the right segment's Q of its first
  // position; hands on this segment's. The operations of lattice_dev.h entering.
  auto entering2 = [&](const XRow<2>& X, const XRow<2>& O, float bm, int be, XRow<2>& Q,
                       XRow<2>& R, float& pm, int& pe) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      Q.m[j] = OBS ? X.m[j] * O.m[j] : X.m[j];
      Q.e[j] = OBS ? X.e[j] + O.e[j] : X.e[j];
    }
    pm = Q.m[0];
    pe = Q.e[0];
    float rm = shl1(Q.m[0]);
    int re = shl1(Q.e[0]);
    rm = lane == 63 ? bm : rm;
    re = lane == 63 ? be : re;
    R.m[0] = Q.m[1];
    R.e[0] = Q.e[1];
    R.m[1] = rm;
    R.e[1] = re;
  };
  auto beta_next = [&](XRow<2>& X, const XRow<2>& E, const XRow<2>& Sh, const XRow<2>& Q,
                       const XRow<2>& R) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const xf r = xf_add(E.m[j] * Q.m[j], E.e[j] + Q.e[j], Sh.m[j] * R.m[j], Sh.e[j] + R.e[j]);
      X.m[j] = r.m;
      X.e[j] = r.e;
    }
  };

  WItem ring[kDepth];
  if constexpr (PHASE == 1) {
    if (dir == 0) {
      // ---------------- alpha[0..M]: rows 0..M of the workspace ----------------
      // alpha[0]: 1 at p = 0 (x obs[0][0]). Selects, not conditional stores: the row must stay
      // in registers (a partially written aggregate ends up in memory)
      xf a0{0.5f, 1};
      if constexpr (OBS) {
        const xf o = xf_exp(lo[0], true);
        a0 = xf_norm(o.m, o.e);
      }
      const bool first = w == 0 && lane == 0;
      XRow<2> X;  // alpha row of this lane's two positions
      X.m[0] = first ? a0.m : 0.0f;
      X.e[0] = first ? a0.e : XF_EZERO;
      X.m[1] = 0.0f;
      X.e[1] = XF_EZERO;
      put_row(0, X);
      if (la) put_log(la, 0, X);
#pragma unroll
      for (int k = 0; k < kDepth; ++k) load_item(k, ring[k]);
      pipeline(M, [&](int r, auto Kc, float bm, int be, float& pm, int& pe) __attribute__((always_inline)) {
        constexpr int k = decltype(Kc)::value;
        XRow<2> E, Sh, O;
        convert2(ring[k], E, Sh, O);
        load_item(r + kDepth, ring[k]);
        alpha_next(X, E, Sh, O, bm, be, pm, pe);
        put_row(r + 1, X);
        if (la) put_log(la, r + 1, X);
      });
    } else {
      // ---------------- beta[S-1..M]: rows S-1..M+1, beta[M] to row T ----------------
      XRow<2> X;  // beta row of this lane's two positions
      load_item(S - 1, ring[0]);
      {
        XRow<2> E, Sh, O;
        convert2(ring[0], E, Sh, O);
#pragma unroll
        for (int j = 0; j < 2; ++j) {  // terminal emit (src/lib.rs:187-195)
          const bool last = p0 + j == P - 1;
          const xf v = term ? xf_norm(E.m[j], E.e[j]) : xf{0.5f, 1};
          X.m[j] = last ? v.m : 0.0f;
          X.e[j] = last ? v.e : XF_EZERO;
        }
      }
      put_row(S - 1 > M ? S - 1 : T, X);
      if (lb) put_log(lb, S - 1, X);
#pragma unroll
      for (int k = 0; k < kDepth; ++k) load_item(S - 2 - k, ring[k]);
      pipeline(S - 1 - M, [&](int i, auto Kc, float bm, int be, float& pm, int& pe) __attribute__((always_inline)) {
        constexpr int k = decltype(Kc)::value;
        const int s = S - 2 - i;
        XRow<2> E, Sh, O, Q, R;
        convert2(ring[k], E, Sh, O);  // E, Sh of row s; O of row s+1
        load_item(s - kDepth, ring[k]);
        entering2(X, O, bm, be, Q, R, pm, pe);
        beta_next(X, E, Sh, Q, R);
        put_row(s > M ? s : T, X);
        if (lb) put_log(lb, s, X);
      });
    }
    return;
  } else {
    // ---------------- phase 2: Z at the cut (both workgroups, the oracle's tree) ----------------
    float v[4], u[4];
    ld_row(M, v);
    ld_row(T, u);
    float wm[2];
    int we[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool live = p0 + j < P;
      wm[j] = live ? v[2 * j] * u[2 * j] : 0.0f;
      we[j] = live ? __builtin_bit_cast(int, v[2 * j + 1]) + __builtin_bit_cast(int, u[2 * j + 1])
                   : XF_EZERO;
    }
    xf z = xf_add(wm[0], we[0], wm[1], we[1]);
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const float om = __shfl_xor(z.m, off);
      const int oe = __shfl_xor(z.e, off);
      z = xf_add(z.m, z.e, om, oe);
    }
    if (lane == 0) ctl.zpart[w] = z;
    __syncthreads();
    if (threadIdx.x == 0) {
      xf t[kMaxNW];
#pragma unroll
      for (int q = 0; q < kMaxNW; ++q) t[q] = q < NW ? ctl.zpart[q] : xf{0.0f, XF_EZERO};
#pragma unroll
      for (int len = kMaxNW; len > 1; len >>= 1) {
#pragma unroll
        for (int q = 0; q < len / 2; ++q) t[q] = xf_add(t[2 * q].m, t[2 * q].e, t[2 * q + 1].m, t[2 * q + 1].e);
      }
      ctl.z = t[0];
    }
    __syncthreads();
    const xf Z = ctl.z;
    if (Z.m == 0.0f) {  // no path: every output row is the infeasible one
      if (dir == 0) {
        zero_rows(0, T);
        if (threadIdx.x == 0) a.loss[b] = inf_loss;
      }
      return;
    }
    if (dir == 0 && threadIdx.x == 0) a.loss[b] = 0.0f - xf_log(Z);
    const float izm = 1.0f / Z.m;
    const int ize = -Z.e;
    WRows wr[kDepth];
    if (dir == 0) {
      // ---------------- alpha: rows M..S-1, gradient rows s >= M ----------------
      auto load_rows = [&](int s, WRows& r) __attribute__((always_inline)) {  // beta[s+1] (+ its position p0+2), beta[s]
        const int sn = uni(min(s + 1, S - 1));
        ld_row(sn, r.r0);
        const __amdgpu_buffer_rsrc_t rr = brsrc(rows + (size_t)sn * U, rowb);
        const f32x2 x = rbuf_ld2(rr, p0 * 8 + 16, 0, 0);
        r.nb[0] = x.x;
        r.nb[1] = x.y;
        if constexpr (OBS) {
          ld_row(s == M ? T : min(s, S - 1), r.r1);
          r.nob = rbuf_ld1(brsrc(lo + (size_t)uni(min(s + 1, T - 1)) * U, rowf), p0 * 4 + 8, 0, 0);
        }
      };
      ld_row(M, v);
      XRow<2> X = unpack(v);
#pragma unroll
      for (int k = 0; k < kDepth; ++k) {
        load_item(M + k, ring[k]);
        load_rows(M + k, wr[k]);
      }
      pipeline(S - M, [&](int i, auto Kc, float bm, int be, float& pm, int& pe) __attribute__((always_inline)) {
        constexpr int k = decltype(Kc)::value;
        const int s = M + i;
        XRow<2> E, Sh, O, Q, R;
        convert2(ring[k], E, Sh, O);
        const WRows rw = wr[k];
        load_item(s + kDepth, ring[k]);
        load_rows(s + kDepth, wr[k]);
        if (s + 1 < S) {
          XRow<2> Bn = unpack(rw.r0);
          // the right neighbour of position p0+1 (lane 63: the next segment's first position)
          float om = 1.0f;
          int oe = 0;
          if constexpr (OBS) {
            const xf o = xf_exp(rw.nob, p0 + 2 < P);
            om = o.m;
            oe = o.e;
          }
          const float nbm = OBS ? rw.nb[0] * om : rw.nb[0];
          const int nbe = OBS ? __builtin_bit_cast(int, rw.nb[1]) + oe : __builtin_bit_cast(int, rw.nb[1]);
          float qm;
          int qe;
          entering2(Bn, O, nbm, nbe, Q, R, qm, qe);
        } else {  // terminal transition: only the terminal emit at P-1 (src/lib.rs:187-195)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const bool last = term && p0 + j == P - 1;
            Q.m[j] = last ? 1.0f : 0.0f;
            Q.e[j] = last ? 0 : XF_EZERO;
            R.m[j] = 0.0f;
            R.e[j] = XF_EZERO;
          }
        }
        float ge[2], gs[2], gob[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          ge[j] = xf_neg_post(((X.m[j] * E.m[j]) * Q.m[j]) * izm, X.e[j] + E.e[j] + Q.e[j] + ize);
          gs[j] = xf_neg_post(((X.m[j] * Sh.m[j]) * R.m[j]) * izm, X.e[j] + Sh.e[j] + R.e[j] + ize);
        }
        put_grad(s, ge, gs);
        if constexpr (OBS) {
          const XRow<2> Bs = unpack(rw.r1);
#pragma unroll
          for (int j = 0; j < 2; ++j)
            gob[j] = xf_neg_post((X.m[j] * Bs.m[j]) * izm, X.e[j] + Bs.e[j] + ize);
          if (go) put_f(go, s, gob);
        }
        if (s + 1 < S) {
          alpha_next(X, E, Sh, O, bm, be, pm, pe);
          if (la) put_log(la, s + 1, X);
        } else {
          pm = 0.0f;
          pe = XF_EZERO;
        }
      });
      zero_rows(S, T);  // rows past the lattice
    } else {
      // ---------------- beta: rows M-1..0, gradient rows s < M ----------------
      ld_row(T, v);
      XRow<2> X = unpack(v);
      auto load_rows = [&](int s, WRows& r) __attribute__((always_inline)) { ld_row(max(s, 0), r.r0); };  // alpha[s]
#pragma unroll
      for (int k = 0; k < kDepth; ++k) {
        load_item(M - 1 - k, ring[k]);
        load_rows(M - 1 - k, wr[k]);
      }
      pipeline(M, [&](int i, auto Kc, float bm, int be, float& pm, int& pe) __attribute__((always_inline)) {
        constexpr int k = decltype(Kc)::value;
        const int s = M - 1 - i;
        XRow<2> E, Sh, O, Q, R;
        convert2(ring[k], E, Sh, O);  // E, Sh of row s; O of row s+1
        const XRow<2> A = unpack(wr[k].r0);
        load_item(s - kDepth, ring[k]);
        load_rows(s - kDepth, wr[k]);
        entering2(X, O, bm, be, Q, R, pm, pe);
        float ge[2], gs[2], gob[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          ge[j] = xf_neg_post(((A.m[j] * E.m[j]) * Q.m[j]) * izm, A.e[j] + E.e[j] + Q.e[j] + ize);
          gs[j] = xf_neg_post(((A.m[j] * Sh.m[j]) * R.m[j]) * izm, A.e[j] + Sh.e[j] + R.e[j] + ize);
        }
        beta_next(X, E, Sh, Q, R);
        put_grad(s, ge, gs);
        if constexpr (OBS) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
            gob[j] = xf_neg_post((A.m[j] * X.m[j]) * izm, A.e[j] + X.e[j] + ize);
          if (go) put_f(go, s, gob);
        }
        if (lb) put_log(lb, s, X);
      });
    }
  }
}

template <bool OBS>
int launch_wide(const FwdBwdArgs& a, hipStream_t st) {
  const int NW = (a.U + kSeg - 1) / kSeg;
  const dim3 grid(a.B, 2), block(64 * NW);
  hipLaunchKernelGGL((k_fwd_bwd_wide<OBS, 1>), grid, block, 0, st, a);
  if (hipGetLastError() != hipSuccess) return SSNT_ERR_HIP;
  hipLaunchKernelGGL((k_fwd_bwd_wide<OBS, 2>), grid, block, 0, st, a);
  return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
}

}  // namespace

size_t fwd_bwd_wide_workspace_bytes(int B, int T, int U) {
  return (size_t)B * ((size_t)T + 1) * U * sizeof(xf);  // rows 0..T-1 + the cut row T
}

int launch_fwd_bwd_wide(const FwdBwdArgs& a, hipStream_t st) {
  if (a.U <= 256 || a.U > kSeg * kMaxNW) return SSNT_ERR_UNSUPPORTED;
  if (!a.workspace || a.workspace_bytes < fwd_bwd_wide_workspace_bytes(a.B, a.T, a.U))
    return SSNT_ERR_WORKSPACE;
  return a.log_obs ? launch_wide<true>(a, st) : launch_wide<false>(a, st);
}

}  // namespace ssnt
