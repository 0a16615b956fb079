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
//     The kernel boundary between them is the only inter-workgroup synchronisation...
//   * ...except in the SPLIT form (small batches, 8B <= CUs, and the 8-wave K = 2 rows; the
//     rule and its measurements: launch_wide): a direction's segments over TWO
//     workgroups, so twice the CUs work. The upstream workgroup (the segments the
//     recurrence flows out of: the low positions for alpha, the high ones for beta) hands its
//     boundary values to the downstream one through global memory, one block of kBS steps at a
//     time, by two proxy waves that carry no arithmetic:
//       publisher (upstream workgroup): reads the last compute wave's LDS ring, stores the block
//         write-through (sc1), drains its own stores (vmcnt(0): it has no loads in flight) and
//         advances a global counter (relaxed agent-scope atomic store);
//       receiver (downstream workgroup): polls that counter (relaxed agent loads + s_sleep), loads
//         the block with sc1 loads (no L1 copy can be stale, so no acquire fence) and feeds it
//         into the first compute wave's LDS ring.
//     The global ring holds every step of the phase, so the upstream workgroup never waits for
//     the downstream one; the counters are zeroed by a memset node before phase 1 on every call.
//     Upstream workgroups have the lower block ids (dispatched first) and sit 2B ids before
//     their partner, so the pair shares an XCD (and its L2) whenever 2B % 8 == 0.
#include <hip/hip_runtime.h>

#include <atomic>
#include <type_traits>
#include <utility>

#include "lattice_dev.h"

namespace ssnt {
namespace {

// steps per hand-off block = rows in flight per wave (ring indices static). At K = 1, 16 rows of
// 512 B per wave keep ~2 us of HBM latency covered at a ~0.2 us step (Little's law: 8 rows held
// the kernel near 3 TB/s); K = 2 has twice the bytes per row and the registers for 8.
// SPLIT phase 1 at K = 1 keeps 32 rows in flight (at most 2 waves per SIMD leave it the
// registers; configs[4]: 660 -> 625 us), one workgroup per direction 16 (32 measured slower there).
template <int K, int PHASE, bool SPLIT>
constexpr int block_steps() {
  return K == 1 ? (PHASE == 1 ? (SPLIT ? 32 : 16) : 16) : 8;
}
// hand-off ring slots (steps) per wave: 64 in one workgroup; 128 when a direction is split, so
// that the global hand-off moves 64 steps per publication (kPub; 16-step publications made the
// split form slower than one workgroup, 64 made it faster: DESIGN.md 5.2 round 5)
template <bool SPLIT>
constexpr int ring_slots() { return SPLIT ? 128 : 64; }
constexpr int kPub = 64;       // steps per global publication (SPLIT)
constexpr int kMaxNW = 8;      // waves per direction: U <= 512 (K = 1) / 1024 (K = 2)
constexpr int kProxy = kMaxNW; // ring / counter index of the proxy wave (SPLIT)
constexpr int kSpinMax = 1 << 22;

template <int kRB>
struct WideCtl {
  int prod[kMaxNW + 1];     // steps whose hand-off value ring w holds (w = kProxy: the receiver's)
  int cons[kMaxNW + 1];     // steps of its upstream ring wave w has read (kProxy: the publisher)
  xf zpart[kMaxNW];         // per-segment sums of alpha[M] * beta[M]
  xf z;
  alignas(16) xf bnd[kMaxNW + 1][kRB];  // hand-off rings
  xf junk[kMaxNW][64];      // where the lanes that do not publish write (branch-free publication)
};

// Global side of the SPLIT hand-off, carved from the head of the workspace (wide_layout):
// ctr[phase][b][dir] counters (the memset block), then gring[b][dir][RL] boundary values.
struct WideGrid {
  int NW;     // segments (64K positions each) per direction
  int NWp;    // segments of the upstream workgroup (SPLIT)
  int* ctr;
  xf* gring;
  int RL;     // ring entries per (utterance, direction): T + 32
  xf* rows;   // rows base (after the sync block)
};

__device__ __forceinline__ int gctr_ld(const int* p) {
  return __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

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
// a plain LDS store (the address space spelled out: a volatile or atomic store through a generic
// pointer can become a flat store, whose completion the compiler then waits for with vmcnt(0))
typedef __attribute__((address_space(3))) int lds_int;
__device__ __forceinline__ void wctr_st(int* p, int v) {
  *reinterpret_cast<lds_int*>(reinterpret_cast<size_t>(p) & 0xffffffffu) = v;
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

// the same on a global counter written by another workgroup (relaxed agent-scope polls);
// -1 when the bound expired (the caller poisons what it forwards)
__device__ __forceinline__ int gwait_ge(const int* p, int target, int* status) {
  int v = gctr_ld(p);
  for (int n = 0; v < target; ++n) {
    if (n > kSpinMax) {
      if (status && (threadIdx.x & 63) == 0) atomicOr(status, kStatusTimeout);
      return -1;
    }
    __builtin_amdgcn_s_sleep(2);
    v = gctr_ld(p);
  }
  return v;
}
constexpr int kSC1 = 16;  // buffer-op cache policy: sc1 (write-through store / L1-bypassing load)

template <int K>
struct WItem {    // one row's inputs for this lane's K positions
  float lt[2 * K];  // emit/shift of p0 .. p0+K-1
  float ob[K];      // log_obs of the entering row (OBS)
};
template <int K>
struct WRows {    // phase-2 workspace rows for this lane
  float r0[2 * K];  // alpha: beta[s+1]; beta: alpha[s]        (m, e, m, e, ...)
  float r1[2 * K];  // alpha: beta[s] (grad_obs)
  float nb[2];      // alpha: beta[s+1] at p0+K (lane 63: next segment's first position)
  float nob;        // alpha: log_obs[s+1] at p0+K
};

// DBG: log-alpha / log-beta outputs requested (a separate instantiation, so the product path's
// step bodies carry no debug branches: straight-line blocks keep the compiler's memory wait
// counts exact, and a wait for row r+8's loads does not drain the stores issued since)
// K: positions per lane; a wave owns 64K consecutive positions.
// SPLIT: a direction's segments over two workgroups (header); 1-D grid of 4B workgroups, id =
// part * 2B + 2b + dir, part 0 = upstream. Waves in flow order (alpha: increasing positions,
// beta: decreasing): local wave w < ncomp computes flow segment f0 + w; wave ncomp is the proxy.
template <int K, bool OBS, int PHASE, bool DBG, bool SPLIT>
__global__ __launch_bounds__(SPLIT ? 64 * (kMaxNW / 2 + 1) : 64 * kMaxNW) void k_fwd_bwd_wide(FwdBwdArgs a, WideGrid gd) {
  constexpr int kSeg = 64 * K;
  constexpr int kBS = block_steps<K, PHASE, SPLIT>();
  constexpr int kRB = ring_slots<SPLIT>();
  static_assert(kRB % kBS == 0, "hand-off blocks must tile the ring");
  constexpr int kDepth = kBS;  // rows in flight per wave
  __shared__ WideCtl<kRB> ctl;
  int b, dir, part;  // dir 0 alpha, 1 beta; part 0 upstream, 1 downstream (SPLIT)
  if constexpr (SPLIT) {
    const int id = blockIdx.x;
    part = id >= 2 * a.B ? 1 : 0;
    const int r = id - part * 2 * a.B;
    b = r >> 1;
    dir = r & 1;
  } else {
    b = blockIdx.x;
    dir = blockIdx.y;
    part = 0;
  }
  const int NW = gd.NW;
  const int ncomp = SPLIT ? (part == 0 ? gd.NWp : NW - gd.NWp) : NW;  // compute waves here
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool comp = w < ncomp;
  const bool proxy = SPLIT && w == ncomp;
  const int f = (SPLIT && part == 1 ? gd.NWp : 0) + (comp ? w : 0);  // flow segment
  const int seg = dir == 0 ? f : NW - 1 - f;
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
  float* la = (DBG && a.log_alpha) ? a.log_alpha + (size_t)b * TU : nullptr;
  float* lb = (DBG && a.log_beta) ? a.log_beta + (size_t)b * TU : nullptr;
  // raw-state debug mode (ssnt_fwd_bwd_debug64_device): mantissas in la / lb, exponents here
  float* lae = (la && a.log_alpha_e) ? reinterpret_cast<float*>(a.log_alpha_e) + (size_t)b * TU : nullptr;
  float* lbe = (lb && a.log_beta_e) ? reinterpret_cast<float*>(a.log_beta_e) + (size_t)b * TU : nullptr;
  xf* rows = gd.rows + (size_t)b * (T + 1) * U;  // row T: beta[M]
  const int p0 = kSeg * seg + K * lane;
  const unsigned rowb = (unsigned)U * 8u, rowf = (unsigned)U * 4u;

  if (threadIdx.x < 2 * (kMaxNW + 1)) reinterpret_cast<int*>(&ctl)[threadIdx.x] = 0;
  __syncthreads();

  // ---- row helpers (8-byte granules: any U, rows only 8-byte aligned). One buffer descriptor
  // per tensor of this utterance, built once; a row is its scalar offset s * U * 8 (soffset, one
  // s_mul per access -- per-row descriptors cost ~10 SALU of 64-bit address arithmetic each, a
  // quarter of a step's instructions). Row indices are wave-uniform (readfirstlane), so the
  // offsets stay in SGPRs. A lane's position offsets are fixed per lane: positions past U get an
  // offset beyond every descriptor (loads return 0, stores are dropped: what a row-sized
  // descriptor did), and the host keeps every descriptor below 2 GB (launch_fwd_bwd_wide).
  auto uni = [](int x) __attribute__((always_inline)) { return __builtin_amdgcn_readfirstlane(x); };
  constexpr int kOOR = (int)0x80000000u;
  int vo8[K], vo4[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    vo8[j] = p0 + j < U ? (p0 + j) * 8 : kOOR;
    vo4[j] = p0 + j < U ? (p0 + j) * 4 : kOOR;
  }
  const int vnb8 = p0 + K < U ? (p0 + K) * 8 : kOOR;  // the next lane slice's first position
  const int vnb4 = p0 + K < U ? (p0 + K) * 4 : kOOR;
  const unsigned tub8 = (unsigned)((size_t)T * U * 8), tub4 = (unsigned)((size_t)T * U * 4);
  const unsigned wsb8 = (unsigned)((size_t)(T + 1) * U * 8);
  auto so8 = [&](int s) __attribute__((always_inline)) { return (int)((unsigned)uni(s) * rowb); };
  auto so4 = [&](int s) __attribute__((always_inline)) { return (int)((unsigned)uni(s) * rowf); };
  // Stores take a `live` flag: a dead step (past the end of the last, partial block) runs the
  // same straight-line code but its descriptors cover 0 bytes, so its stores are dropped.
  auto put_grad = [&](int s, const float* ge, const float* gs, bool live = true) __attribute__((always_inline)) {
    if (!g) return;
    const __amdgpu_buffer_rsrc_t r = brsrc(g, live ? tub8 : 0u);
    const int so = so8(s);
#pragma unroll
    for (int j = 0; j < K; ++j) rbuf_st2(f32x2{ge[j], gs[j]}, r, vo8[j], so, 0);
  };
  auto put_f = [&](float* base, int s, const float* v, bool live = true) __attribute__((always_inline)) {
    const bool on = live && base != nullptr;  // a null base (output not requested): 0 bytes
    const __amdgpu_buffer_rsrc_t r = brsrc(on ? base : nullptr, on ? tub4 : 0u);
    const int so = so4(s);
#pragma unroll
    for (int j = 0; j < K; ++j) rbuf_st1(v[j], r, vo4[j], so, 0);
  };
  auto put_log = [&](float* base, int s, const XRow<K>& x, bool live = true) __attribute__((always_inline)) {
    float v[K], ev[K];
    float* ebase = base == la ? lae : lbe;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const xf n = xf_norm(x.m[j], x.e[j]);  // (rows are normalized: an identity)
      v[j] = ebase ? n.m : xf_log(n);
      ev[j] = __builtin_bit_cast(float, n.e);
    }
    put_f(base, s, v, live);
    if (ebase) put_f(ebase, s, ev, live);
  };
  // workspace row s (s == T: the cut row). The fields go through registers one by one: a vector
  // built straight from the adjacent fields of the row makes the compiler keep the row in memory
  auto put_row = [&](int s, const XRow<K>& x, bool live = true) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t r = brsrc(rows, live ? wsb8 : 0u);
    const int so = so8(s);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      float mj = x.m[j];
      int ej = x.e[j];
      asm volatile("" : "+v"(mj), "+v"(ej));
      rbuf_st2(f32x2{mj, __builtin_bit_cast(float, ej)}, r, vo8[j], so, 0);
    }
  };
  const __amdgpu_buffer_rsrc_t rows_r = brsrc(rows, wsb8);
  auto ld_row = [&](int s, float* v) __attribute__((always_inline)) {  // 2K floats; past U: zeros
    const int so = so8(s);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const f32x2 x = rbuf_ld2(rows_r, vo8[j], so, 0);
      v[2 * j] = x.x;
      v[2 * j + 1] = x.y;
    }
  };
  auto unpack = [&](const float* v) __attribute__((always_inline)) {
    XRow<K> x;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      x.m[j] = v[2 * j];
      x.e[j] = __builtin_bit_cast(int, v[2 * j + 1]);
    }
    return x;
  };
  // zero gradients, -inf debug rows (rows [from, to)); each wave writes its own segment
  auto zero_rows = [&](int from, int to) __attribute__((always_inline)) {
    float z[K], ninf[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      z[j] = 0.0f;
      ninf[j] = a.log_alpha_e ? 0.0f : -__builtin_inff();  // raw state: mantissa 0
    }
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
      if ((S > T || P > U || S < 0 || P < 0) && a.status && part == 0 && threadIdx.x == 0)
        atomicOr(a.status, kStatusBadLength);
      if (comp) zero_rows(0, T);
      if (part == 0 && threadIdx.x == 0) a.loss[b] = inf_loss;
    }
    return;
  }
  const int M = (S - 1) >> 1;

  const __amdgpu_buffer_rsrc_t lt_r = brsrc(lt, tub8);
  const __amdgpu_buffer_rsrc_t lo_r = brsrc(lo, OBS ? tub4 : 0u);
  auto load_item = [&](int row, WItem<K>& it) __attribute__((always_inline)) {
    row = uni(min(max(row, 0), T - 1));
    const int so = so8(row);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const f32x2 x = rbuf_ld2(lt_r, vo8[j], so, 0);
      it.lt[2 * j] = x.x;
      it.lt[2 * j + 1] = x.y;
    }
    if constexpr (OBS) {
      const int oso = so4(min(row + 1, T - 1));
#pragma unroll
      for (int j = 0; j < K; ++j) it.ob[j] = rbuf_ld1(lo_r, vo4[j], oso, 0);
    }
  };
  auto convert2 = [&](const WItem<K>& it, XRow<K>& E, XRow<K>& Sh, XRow<K>& O) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < K; ++j)
      xf_exp_pair(it.lt[2 * j], it.lt[2 * j + 1], p0 + j < P, p0 + j < P - 1, E.m[j], E.e[j],
                  Sh.m[j], Sh.e[j]);
    if constexpr (OBS) {
      if constexpr (K == 1) {
        const xf o = xf_exp(it.ob[0], p0 < P);
        O.m[0] = o.m;
        O.e[0] = o.e;
      } else {
#pragma unroll
        for (int j = 0; j + 1 < K; j += 2)
          xf_exp_pair(it.ob[j], it.ob[j + 1], p0 + j < P, p0 + j + 1 < P, O.m[j], O.e[j],
                      O.m[j + 1], O.e[j + 1]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        O.m[j] = 1.0f;
        O.e[j] = 0;
      }
    }
  };

  // ---- the hand-off pipeline: up = the ring whose boundary values this wave needs (the
  // previous wave in flow order, or the receiver's), dn = the wave that reads this wave's ring
  // (the next one, or the publisher)
  const int up = w > 0 ? w - 1 : kProxy;
  const int dn = w + 1 < ncomp ? w + 1 : kProxy;
  const bool has_up = comp && (w > 0 || (SPLIT && part == 1));
  const bool has_dn = comp && (w + 1 < ncomp || (SPLIT && part == 0));
  const int pub_lane = dir == 0 ? 63 : 0;
  // n iterations in blocks of kBS; step(i, K, bm, be, pm, pe) with K = i % kBS a compile-time
  // constant (register ring indices), (bm, be) the upstream value of iteration i and (pm, pe)
  // the value this wave hands on. The downstream wave runs at least one block behind.
  auto pipeline = [&](int n, auto&& step) __attribute__((always_inline)) {
    // the lanes that do not publish write to their own junk slot: publication is branch-free
    const bool pub = has_dn && lane == pub_lane;
    for (int i0 = 0; i0 < n; i0 += kBS) {
      const int i1 = min(i0 + kBS, n);
      float bm[kBS];
      int be[kBS];
      if (has_up) wait_ge(&ctl.prod[up], i1, a.status);
      if (has_dn) wait_ge(&ctl.cons[dn], i1 - kRB, a.status);
      wbar();
      const xf* rd = &ctl.bnd[has_up ? up : 0][i0 % kRB];
#pragma unroll
      for (int k = 0; k < kBS; ++k) {  // (stale values when there is no upstream: unused)
        const xf v = rd[k];
        bm[k] = has_up ? v.m : 0.0f;
        be[k] = has_up ? v.e : XF_EZERO;
      }
      xf* wp = pub ? &ctl.bnd[w][i0 % kRB] : &ctl.junk[w][lane];
      const int ws = pub ? 1 : 0;
      // one straight-line path for every block (steps past n are dead: their stores are
      // dropped): no join of two paths, so no register copies of rows with loads in flight
      sfor<kBS>([&](auto Kc) __attribute__((always_inline)) {
        constexpr int k = decltype(Kc)::value;
        float pm;
        int pe;
        step(i0 + k, Kc, bm[k], be[k], pm, pe, i0 + k < i1);
        wp[k * ws] = xf{pm, pe};
      });
      wbar();
      if (has_dn) wctr_st(&ctl.prod[w], i1);
      if (has_up) wctr_st(&ctl.cons[w], i1);
    }
  };

  // SPLIT proxies (header): n steps of hand-off, kBS values per block, 16 B per lane
  auto run_proxy = [&](int n) __attribute__((always_inline)) {
    // hand-off granule: kPub steps (2 - 4 blocks) per global publication
    constexpr int kPB = kPub;
    static_assert(kRB % kPB == 0, "publication granules tile the ring");
    constexpr int kL = kPB / 4;  // lanes moving the granule, 32 B (4 xf) each
    const __amdgpu_buffer_rsrc_t gr = brsrc(gd.gring + (size_t)(b * 2 + dir) * gd.RL, gd.RL * 8u);
    int* ctr = gd.ctr + ((PHASE - 1) * a.B + b) * 2 + dir;
    if (part == 0) {  // publisher: the last compute wave's ring -> global
      const int src = ncomp - 1;
      for (int i0 = 0; i0 < n; i0 += kPB) {
        const int i1 = min(i0 + kPB, n);
        wait_ge(&ctl.prod[src], i1, a.status);
        wbar();
        f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f}, v2 = {0.0f, 0.0f, 0.0f, 0.0f};
        if (lane < kL) {
          v = *reinterpret_cast<const f32x4*>(&ctl.bnd[src][i0 % kRB + 4 * lane]);
          v2 = *reinterpret_cast<const f32x4*>(&ctl.bnd[src][i0 % kRB + 4 * lane + 2]);
        }
        wbar();
        wctr_st(&ctl.cons[kProxy], i1);  // (DS in order: the reads above are done first)
        if (lane < kL) {
          rbuf_st4(v, gr, (i0 + 4 * lane) * 8, 0, kSC1);
          rbuf_st4(v2, gr, (i0 + 4 * lane + 2) * 8, 0, kSC1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores only
        if (lane == 0) __hip_atomic_store(ctr, i1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {  // receiver: global -> the first compute wave's upstream ring
      int seen = 0;
      bool dead = false;  // the upstream workgroup never published: forward NaN from here on, so
                          // the utterance's loss and gradients are NaN, never plausible values
      for (int i0 = 0; i0 < n; i0 += kPB) {
        const int i1 = min(i0 + kPB, n);
        if (!dead && seen < i1) {
          seen = gwait_ge(ctr, i1, a.status);
          dead = seen < 0;
        }
        asm volatile("" ::: "memory");  // the payload loads stay behind the poll
        f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f}, v2 = {0.0f, 0.0f, 0.0f, 0.0f};
        if (lane < kL) {
          v = rbuf_ld4(gr, (i0 + 4 * lane) * 8, 0, kSC1);
          v2 = rbuf_ld4(gr, (i0 + 4 * lane + 2) * 8, 0, kSC1);
        }
        if (dead) {
          v = f32x4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
          v2 = v;
        }
        wait_ge(&ctl.cons[0], i1 - kRB, a.status);
        wbar();
        if (lane < kL) {
          *reinterpret_cast<f32x4*>(&ctl.bnd[kProxy][i0 % kRB + 4 * lane]) = v;
          *reinterpret_cast<f32x4*>(&ctl.bnd[kProxy][i0 % kRB + 4 * lane + 2]) = v2;
        }
        wbar();
        wctr_st(&ctl.prod[kProxy], i1);
      }
    }
  };

  // alpha[r+1] from alpha[r] (= A); (bm, be): the left segment's shift product of its last
  // position; hands on this segment's. The operations of lattice_dev.h alpha_step.
  auto alpha_next = [&](XRow<K>& A, const XRow<K>& E, const XRow<K>& Sh, const XRow<K>& O,
                        float bm, int be, float& pm, int& pe) __attribute__((always_inline)) {
    XRow<K> st, sh;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      st.m[j] = A.m[j] * E.m[j];
      st.e[j] = A.e[j] + E.e[j];
      sh.m[j] = A.m[j] * Sh.m[j];
      sh.e[j] = A.e[j] + Sh.e[j];
    }
    pm = sh.m[K - 1];
    pe = sh.e[K - 1];
    float lm = shr1(sh.m[K - 1]);
    int le = shr1(sh.e[K - 1]);
    lm = lane == 0 ? bm : lm;
    le = lane == 0 ? be : le;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const float hm = j == 0 ? lm : sh.m[j > 0 ? j - 1 : 0];
      const int he = j == 0 ? le : sh.e[j > 0 ? j - 1 : 0];
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
  auto entering2 = [&](const XRow<K>& X, const XRow<K>& O, float bm, int be, XRow<K>& Q,
                       XRow<K>& R, float& pm, int& pe) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      Q.m[j] = OBS ? X.m[j] * O.m[j] : X.m[j];
      Q.e[j] = OBS ? X.e[j] + O.e[j] : X.e[j];
    }
    pm = Q.m[0];
    pe = Q.e[0];
    float rm = shl1(Q.m[0]);
    int re = shl1(Q.e[0]);
    rm = lane == 63 ? bm : rm;
    re = lane == 63 ? be : re;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      R.m[j] = j == K - 1 ? rm : Q.m[j + 1 < K ? j + 1 : 0];
      R.e[j] = j == K - 1 ? re : Q.e[j + 1 < K ? j + 1 : 0];
    }
  };
  auto beta_next = [&](XRow<K>& X, const XRow<K>& E, const XRow<K>& Sh, const XRow<K>& Q,
                       const XRow<K>& R) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const xf r = xf_add(E.m[j] * Q.m[j], E.e[j] + Q.e[j], Sh.m[j] * R.m[j], Sh.e[j] + R.e[j]);
      X.m[j] = r.m;
      X.e[j] = r.e;
    }
  };

  // Dead stores (0-byte descriptor: dropped) that give the prefetch prologue the steady state's
  // load/store pattern. vmcnt counts loads and stores together, and at the block loop's header
  // the compiler's wait counts take the minimum over the prologue (loads only) and the back edge
  // (each step's loads + stores): without these, the first steps of every block waited for loads
  // issued ~8 rows back instead of kDepth.
  constexpr int kPad = PHASE == 1 ? K * (DBG ? 2 : 1) : K * (1 + (OBS ? 1 : 0) + (DBG ? 1 : 0));
  // (distinct offsets: identical stores to one address would be merged away)
  auto vm_pad = [&](int k) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t r = brsrc(rows, 0u);
#pragma unroll
    for (int q = 0; q < kPad; ++q) rbuf_st1(0.0f, r, (k * kPad + q) * 4, 0, 0);
  };
  WItem<K> ring[kDepth];
  if constexpr (PHASE == 1) {
    if (!comp) {
      if (proxy) run_proxy(dir == 0 ? M : S - 1 - M);
      return;
    }
    if (dir == 0) {
      // ---------------- alpha[0..M]: rows 0..M of the workspace ----------------
      // alpha[0]: 1 at p = 0 (x obs[0][0]). Selects, not conditional stores: the row must stay
      // in registers (a partially written aggregate ends up in memory)
      xf a0{0.5f, 1};
      if constexpr (OBS) {
        const xf o = xf_exp(lo[0], true);
        a0 = xf_norm(o.m, o.e);
      }
      const bool first = seg == 0 && lane == 0;
      XRow<K> X;  // alpha row of this lane's K positions
      X.m[0] = first ? a0.m : 0.0f;
      X.e[0] = first ? a0.e : XF_EZERO;
#pragma unroll
      for (int j = 1; j < K; ++j) {
        X.m[j] = 0.0f;
        X.e[j] = XF_EZERO;
      }
      put_row(0, X);
      if constexpr (DBG) { if (la) put_log(la, 0, X); }
#pragma unroll
      for (int k = 0; k < kDepth; ++k) {
        load_item(k, ring[k]);
        vm_pad(k);
      }
      pipeline(M, [&](int r, auto Kc, float bm, int be, float& pm, int& pe, bool live) __attribute__((always_inline)) {
        constexpr int k = decltype(Kc)::value;
        XRow<K> E, Sh, O;
        convert2(ring[k], E, Sh, O);
        load_item(r + kDepth, ring[k]);
        alpha_next(X, E, Sh, O, bm, be, pm, pe);
        put_row(r + 1, X, live);
        if constexpr (DBG) put_log(la, r + 1, X, live);
      });
    } else {
      // ---------------- beta[S-1..M]: rows S-1..M+1, beta[M] to row T ----------------
      XRow<K> X;  // beta row of this lane's K positions
      load_item(S - 1, ring[0]);
      {
        XRow<K> E, Sh, O;
        convert2(ring[0], E, Sh, O);
#pragma unroll
        for (int j = 0; j < K; ++j) {  // terminal emit (src/lib.rs:187-195)
          const bool last = p0 + j == P - 1;
          const xf v = term ? xf_norm(E.m[j], E.e[j]) : xf{0.5f, 1};
          X.m[j] = last ? v.m : 0.0f;
          X.e[j] = last ? v.e : XF_EZERO;
        }
      }
      put_row(S - 1 > M ? S - 1 : T, X);
      if constexpr (DBG) { if (lb) put_log(lb, S - 1, X); }
#pragma unroll
      for (int k = 0; k < kDepth; ++k) {
        load_item(S - 2 - k, ring[k]);
        vm_pad(k);
      }
      pipeline(S - 1 - M, [&](int i, auto Kc, float bm, int be, float& pm, int& pe, bool live) __attribute__((always_inline)) {
        constexpr int k = decltype(Kc)::value;
        const int s = S - 2 - i;
        XRow<K> E, Sh, O, Q, R;
        convert2(ring[k], E, Sh, O);  // E, Sh of row s; O of row s+1
        load_item(s - kDepth, ring[k]);
        entering2(X, O, bm, be, Q, R, pm, pe);
        beta_next(X, E, Sh, Q, R);
        put_row(s > M ? s : T, X, live);
        if constexpr (DBG) put_log(lb, s, X, live);
      });
    }
    return;
  } else {
    // ---------------- phase 2: Z at the cut (every workgroup, the oracle's tree) ----------------
    // segment sums (in-lane levels of the tree, pairs (2i, 2i+1) first, then across lanes), then
    // across segments; the waves of this workgroup cover all NW segments between them
    const int nwaves = __builtin_amdgcn_readfirstlane(blockDim.x >> 6);
    for (int sg = w; sg < NW; sg += nwaves) {
      float v[2 * K], u[2 * K];
      const int ps = kSeg * sg + K * lane;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const int vo = ps + j < U ? (ps + j) * 8 : kOOR;
        const f32x2 x = rbuf_ld2(rows_r, vo, so8(M), 0);
        const f32x2 y = rbuf_ld2(rows_r, vo, so8(T), 0);
        v[2 * j] = x.x;
        v[2 * j + 1] = x.y;
        u[2 * j] = y.x;
        u[2 * j + 1] = y.y;
      }
      float wm[K];
      int we[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const bool live = ps + j < P;
        wm[j] = live ? v[2 * j] * u[2 * j] : 0.0f;
        we[j] = live ? __builtin_bit_cast(int, v[2 * j + 1]) + __builtin_bit_cast(int, u[2 * j + 1])
                     : XF_EZERO;
      }
#pragma unroll
      for (int len = K; len > 1; len >>= 1) {
#pragma unroll
        for (int q = 0; q < len / 2; ++q) {
          const xf t2 = xf_add(wm[2 * q], we[2 * q], wm[2 * q + 1], we[2 * q + 1]);
          wm[q] = t2.m;
          we[q] = t2.e;
        }
      }
      xf z{wm[0], we[0]};
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const float om = __shfl_xor(z.m, off);
        const int oe = __shfl_xor(z.e, off);
        z = xf_add(z.m, z.e, om, oe);
      }
      if (lane == 0) ctl.zpart[sg] = z;
    }
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
      if (dir == 0 && comp) zero_rows(0, T);
      if (dir == 0 && part == 0 && threadIdx.x == 0) a.loss[b] = inf_loss;
      return;
    }
    if (dir == 0 && part == 0 && threadIdx.x == 0) {
      a.loss[b] = 0.0f - xf_log(Z);
      if (a.z_state) {
        a.z_state[2 * b] = Z.m;
        a.z_state[2 * b + 1] = __builtin_bit_cast(float, Z.e);
      }
    }
    if (!comp) {
      if (proxy) run_proxy(dir == 0 ? S - M : M);
      return;
    }
    const float izm = 1.0f / Z.m;
    const int ize = -Z.e;
    WRows<K> wr[kDepth];
    if (dir == 0) {
      // ---------------- alpha: rows M..S-1, gradient rows s >= M ----------------
      // (K = 1: beta[s+1] at p0 and p0+1 in ONE 16-byte load -- a vector-memory instruction
      // fewer per step; the step holds ~4 in flight per row and vmcnt counts at most 63)
      const bool nb_ok = p0 + K < U;
      auto load_rows = [&](int s, WRows<K>& r) __attribute__((always_inline)) {  // beta[s+1] (+ position p0+K), beta[s]
        const int sn = uni(min(s + 1, S - 1));
        if constexpr (K == 1) {
          const f32x4 x = rbuf_ld4(rows_r, vo8[0], so8(sn), 0);
          r.r0[0] = x.x;
          r.r0[1] = x.y;
          r.nb[0] = nb_ok ? x.z : 0.0f;  // (past U: what the out-of-range load returned)
          r.nb[1] = nb_ok ? x.w : 0.0f;
        } else {
          ld_row(sn, r.r0);
          const f32x2 x = rbuf_ld2(rows_r, vnb8, so8(sn), 0);
          r.nb[0] = x.x;
          r.nb[1] = x.y;
        }
        if constexpr (OBS) {
          ld_row(s == M ? T : min(s, S - 1), r.r1);
          r.nob = rbuf_ld1(lo_r, vnb4, so4(min(s + 1, T - 1)), 0);
        }
      };
      float v[2 * K];
      ld_row(M, v);
      XRow<K> X = unpack(v);
#pragma unroll
      for (int k = 0; k < kDepth; ++k) {
        load_item(M + k, ring[k]);
        load_rows(M + k, wr[k]);
        vm_pad(k);
      }
      pipeline(S - M, [&](int i, auto Kc, float bm, int be, float& pm, int& pe, bool live) __attribute__((always_inline)) {
        constexpr int k = decltype(Kc)::value;
        const int s = M + i;
        const bool fin = s + 1 >= S;  // the terminal transition (selects, not a branch)
        XRow<K> E, Sh, O, Q, R;
        convert2(ring[k], E, Sh, O);
        const WRows<K> rw = wr[k];
        load_item(s + kDepth, ring[k]);
        load_rows(s + kDepth, wr[k]);
        {
          const XRow<K> Bn = unpack(rw.r0);
          // the right neighbour of position p0+1 (lane 63: the next segment's first position)
          float om = 1.0f;
          int oe = 0;
          if constexpr (OBS) {
            const xf o = xf_exp(rw.nob, p0 + K < P);
            om = o.m;
            oe = o.e;
          }
          const float nbm = OBS ? rw.nb[0] * om : rw.nb[0];
          const int nbe = OBS ? __builtin_bit_cast(int, rw.nb[1]) + oe : __builtin_bit_cast(int, rw.nb[1]);
          float qm;
          int qe;
          entering2(Bn, O, nbm, nbe, Q, R, qm, qe);
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {  // terminal: only the terminal emit at P-1 (src/lib.rs:187-195)
          const bool last = term && p0 + j == P - 1;
          Q.m[j] = fin ? (last ? 1.0f : 0.0f) : Q.m[j];
          Q.e[j] = fin ? (last ? 0 : XF_EZERO) : Q.e[j];
          R.m[j] = fin ? 0.0f : R.m[j];
          R.e[j] = fin ? XF_EZERO : R.e[j];
        }
        float ge[K], gs[K], gob[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
          ge[j] = xf_neg_post(((X.m[j] * E.m[j]) * Q.m[j]) * izm, X.e[j] + E.e[j] + Q.e[j] + ize);
          gs[j] = xf_neg_post(((X.m[j] * Sh.m[j]) * R.m[j]) * izm, X.e[j] + Sh.e[j] + R.e[j] + ize);
        }
        put_grad(s, ge, gs, live);
        if constexpr (OBS) {
          const XRow<K> Bs = unpack(rw.r1);
#pragma unroll
          for (int j = 0; j < K; ++j)
            gob[j] = xf_neg_post((X.m[j] * Bs.m[j]) * izm, X.e[j] + Bs.e[j] + ize);
          put_f(go, s, gob, live);
        }
        // past the terminal transition X is dead (no live step follows)
        alpha_next(X, E, Sh, O, bm, be, pm, pe);
        if constexpr (DBG) put_log(la, s + 1, X, live && !fin);
      });
      zero_rows(S, T);  // rows past the lattice
    } else {
      // ---------------- beta: rows M-1..0, gradient rows s < M ----------------
      float v[2 * K];
      ld_row(T, v);
      XRow<K> X = unpack(v);
      auto load_rows = [&](int s, WRows<K>& r) __attribute__((always_inline)) { ld_row(max(s, 0), r.r0); };  // alpha[s]
#pragma unroll
      for (int k = 0; k < kDepth; ++k) {
        load_item(M - 1 - k, ring[k]);
        load_rows(M - 1 - k, wr[k]);
        vm_pad(k);
      }
      pipeline(M, [&](int i, auto Kc, float bm, int be, float& pm, int& pe, bool live) __attribute__((always_inline)) {
        constexpr int k = decltype(Kc)::value;
        const int s = M - 1 - i;
        XRow<K> E, Sh, O, Q, R;
        convert2(ring[k], E, Sh, O);  // E, Sh of row s; O of row s+1
        const XRow<K> A = unpack(wr[k].r0);
        load_item(s - kDepth, ring[k]);
        load_rows(s - kDepth, wr[k]);
        entering2(X, O, bm, be, Q, R, pm, pe);
        float ge[K], gs[K], gob[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
          ge[j] = xf_neg_post(((A.m[j] * E.m[j]) * Q.m[j]) * izm, A.e[j] + E.e[j] + Q.e[j] + ize);
          gs[j] = xf_neg_post(((A.m[j] * Sh.m[j]) * R.m[j]) * izm, A.e[j] + Sh.e[j] + R.e[j] + ize);
        }
        beta_next(X, E, Sh, Q, R);
        put_grad(s, ge, gs, live);
        if constexpr (OBS) {
#pragma unroll
          for (int j = 0; j < K; ++j)
            gob[j] = xf_neg_post((A.m[j] * X.m[j]) * izm, A.e[j] + X.e[j] + ize);
          put_f(go, s, gob, live);
        }
        if constexpr (DBG) put_log(lb, s, X, live);
      });
    }
  }
}

// workspace carve (WideGrid): the counter block first (the memset zeroes exactly it), then the
// global hand-off rings, then the rows; every piece a multiple of 256 B
struct WideLayout {
  size_t ctr, gring, rows;
};
inline WideLayout wide_layout(int B, int T, int U) {
  auto r256 = [](size_t x) { return (x + 255) & ~(size_t)255; };
  WideLayout l;
  l.ctr = r256((size_t)16 * B);  // ctr[2 phases][B][2 dirs]
  l.gring = r256((size_t)B * 2 * ((size_t)T + 32) * sizeof(xf));
  l.rows = (size_t)B * ((size_t)T + 1) * U * sizeof(xf);  // rows 0..T-1 + the cut row T
  return l;
}

// -1 auto (default): split when the unsplit grid would leave most CUs idle (8B <= CUs), or when
// the split grid fits the chip (4B <= CUs) and the lattice is long (T >= 640) -- measured per
// shape; 0 never; 1 whenever NW >= 2; 2 (A/B study) phase 2 only
#ifdef SSNT_AB
std::atomic<int> g_wide_split{-1};  // A/B build: ssnt_fwd_bwd_wide_split
int wide_split_mode() { return g_wide_split.load(std::memory_order_relaxed); }
#else
constexpr int wide_split_mode() { return -1; }
#endif

int device_cus() {
  static std::atomic<int> cus[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  int n = cus[dev].load(std::memory_order_relaxed);
  if (n == 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 0;
    cus[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

template <int K, bool OBS, bool DBG>
int launch_wide(const FwdBwdArgs& a, hipStream_t st) {
  const int NW = (a.U + 64 * K - 1) / (64 * K);
  const WideLayout l = wide_layout(a.B, a.T, a.U);
  unsigned char* ws = reinterpret_cast<unsigned char*>(a.workspace);
  WideGrid gd;
  gd.NW = NW;
  gd.NWp = (NW + 1) / 2;
  gd.ctr = reinterpret_cast<int*>(ws);
  gd.gring = reinterpret_cast<xf*>(ws + l.ctr);
  gd.RL = a.T + 32;  // whole blocks of up to 32 steps
  gd.rows = reinterpret_cast<xf*>(ws + l.ctr + l.gring);
  const int mode = wide_split_mode();
  bool split = false;
  if (NW >= 2 && mode == 1) {
    split = true;
  } else if (NW >= 2 && mode == -1) {
    const int cus = device_cus();
    // (round 5, 64-step publications: lattices of T >= 640 split whenever the split grid still
    // fits the chip -- configs[4] B=64 T=2000 U=400 539 vs 585 us, T=760 U=700 399 vs 496,
    // T=1100 U=1024 671 vs 867; at T=400 U=300 the one-workgroup form stays ahead, 132 vs 154;
    // profiles/r5i_split_shapes.jsonl)
    split = 8 * a.B <= cus || (4 * a.B <= cus && a.T >= 640);
  }
  if (NW >= 2 && mode == 2) {  // A/B study: phase 1 in one workgroup per direction, phase 2 split
    if (hipMemsetAsync(gd.ctr, 0, l.ctr, st) != hipSuccess) return SSNT_ERR_HIP;
    note_fwd_bwd_dispatch("k_fwd_bwd_wide<K=%d,OBS=%d,DBG=%d,NW=%d>+SPLIT2", K, (int)OBS, (int)DBG, NW);
    hipLaunchKernelGGL((k_fwd_bwd_wide<K, OBS, 1, DBG, false>), dim3(a.B, 2), dim3(64 * NW), 0, st, a, gd);
    if (hipGetLastError() != hipSuccess) return SSNT_ERR_HIP;
    hipLaunchKernelGGL((k_fwd_bwd_wide<K, OBS, 2, DBG, true>), dim3(4 * a.B), dim3(64 * (gd.NWp + 1)), 0, st, a, gd);
    return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
  }
  if (split) {
    if (hipMemsetAsync(gd.ctr, 0, l.ctr, st) != hipSuccess) return SSNT_ERR_HIP;
    const dim3 grid(4 * a.B), block(64 * (gd.NWp + 1));
    note_fwd_bwd_dispatch("k_fwd_bwd_wide<K=%d,OBS=%d,DBG=%d,NW=%d,SPLIT>x2", K, (int)OBS, (int)DBG, NW);
    hipLaunchKernelGGL((k_fwd_bwd_wide<K, OBS, 1, DBG, true>), grid, block, 0, st, a, gd);
    if (hipGetLastError() != hipSuccess) return SSNT_ERR_HIP;
    hipLaunchKernelGGL((k_fwd_bwd_wide<K, OBS, 2, DBG, true>), grid, block, 0, st, a, gd);
    return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
  }
  const dim3 grid(a.B, 2), block(64 * NW);
  note_fwd_bwd_dispatch("k_fwd_bwd_wide<K=%d,OBS=%d,DBG=%d,NW=%d>x2", K, (int)OBS, (int)DBG, NW);
  hipLaunchKernelGGL((k_fwd_bwd_wide<K, OBS, 1, DBG, false>), grid, block, 0, st, a, gd);
  if (hipGetLastError() != hipSuccess) return SSNT_ERR_HIP;
  hipLaunchKernelGGL((k_fwd_bwd_wide<K, OBS, 2, DBG, false>), grid, block, 0, st, a, gd);
  return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
}

template <int K>
int launch_wide_k(const FwdBwdArgs& a, hipStream_t st) {
  const bool dbg = a.log_alpha || a.log_beta;
  if (a.log_obs) return dbg ? launch_wide<K, true, true>(a, st) : launch_wide<K, true, false>(a, st);
  return dbg ? launch_wide<K, false, true>(a, st) : launch_wide<K, false, false>(a, st);
}

// positions per lane: 1 up to U = 512 (A/B build: ssnt_fwd_bwd_wide_lanes forces 2)
#ifdef SSNT_AB
std::atomic<int> g_wide_k{1};
int wide_lanes() { return g_wide_k.load(std::memory_order_relaxed); }
#else
constexpr int wide_lanes() { return 1; }
#endif

}  // namespace

size_t fwd_bwd_wide_workspace_bytes(int B, int T, int U) {
  const WideLayout l = wide_layout(B, T, U);
  return l.ctr + l.gring + l.rows;
}

int launch_fwd_bwd_wide(const FwdBwdArgs& a, hipStream_t st, bool any_u) {
  if ((!any_u && a.U <= 256) || a.U > 64 * 2 * kMaxNW) return SSNT_ERR_UNSUPPORTED;
  // 8-byte granules: every tensor base must be 8-byte aligned (4 for the f32-element ones)
  auto al = [](const void* p, uintptr_t m) { return (reinterpret_cast<uintptr_t>(p) & (m - 1)) == 0; };
  if (!al(a.log_trans, 8) || !al(a.grad, 8) || !al(a.workspace, 8) || !al(a.log_obs, 4) ||
      !al(a.grad_obs, 4) || !al(a.log_alpha, 4) || !al(a.log_beta, 4))
    return SSNT_ERR_UNSUPPORTED;
  if (!a.workspace || a.workspace_bytes < fwd_bwd_wide_workspace_bytes(a.B, a.T, a.U))
    return SSNT_ERR_WORKSPACE;
  // one descriptor per utterance tensor, position offsets up to 2^31 (row helpers)
  if ((size_t)(a.T + 1) * a.U * 8 >= ((size_t)1 << 31)) return SSNT_ERR_UNSUPPORTED;
  const bool k1 = wide_lanes() == 1 && a.U <= 64 * kMaxNW;
  return k1 ? launch_wide_k<1>(a, st) : launch_wide_k<2>(a, st);
}

#ifdef SSNT_AB
int set_fwd_bwd_wide_lanes(int k) {
  if (k != 1 && k != 2) return SSNT_ERR_INVALID_ARG;
  g_wide_k.store(k);
  return SSNT_OK;
}

int set_fwd_bwd_wide_split(int mode) {
  if (mode < -1 || mode > 2) return SSNT_ERR_INVALID_ARG;
  g_wide_split.store(mode);
  return SSNT_OK;
}
#endif

}  // namespace ssnt
