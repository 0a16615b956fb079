// stream_dev.h -- device building blocks of the role-pipelined streaming lattice kernel
// (fwd_bwd_stream.hip): LDS counters and bounded spins, wave roles, the one-step chain
// recurrences in split-exponent form, LDS row moves and the lane-slice global accesses. Included
// inside namespace ssnt::{anonymous}.
#pragma once
#include <hip/hip_runtime.h>
#include <limits.h>

#include <type_traits>
#include <utility>

#include "lattice_dev.h"

namespace ssnt {
namespace {
constexpr int kMaxW = 4;  // max converter / gradient waves per direction
constexpr int kSpinLimit = 1 << 22;
#ifdef SSNT_DIAG
constexpr size_t kCtlBytes = 512;  // + the ring tags below
#else
constexpr size_t kCtlBytes = 256;
#endif

struct Ctl {
  int conv[2][kMaxW];  // per direction / converter: rows of its share written to the ring
  int chain[2];        // per direction: stream rows the chain has finished (outputs written)
  int sread[2];        // per direction: stream rows whose ring slots the chain has read
  int help[2][kMaxW];  // per direction / gradient wave: rows of its share finished
  int a_ready;       // alpha[0..M] stored
  int bm_ready;      // beta[M+1..S-1] stored, beta[M] in the cut buffer
  int z_ready;       // Z published
  int pad;
  xf z;
#ifdef SSNT_DIAG
  // Diagnostic builds: the stream row each converter-ring slot holds (written after the slot's
  // data, before the publishing counter) and the lattice / stream row each chain-ring row holds;
  // every consumer reads the tag after its data and ORs kStatusRingTag into the status word when
  // it is not the row it expected (tests/test_gpu_fwd_bwd.py::test_ring_tags_diag_build)
  int ctag[2][32];
  int rtag[2][16];
#endif
};
static_assert(sizeof(Ctl) <= kCtlBytes, "control block");

#ifdef SSNT_DIAG
__device__ __forceinline__ void tag_put(int* t, int v) {
  if ((threadIdx.x & 63) == 0) *t = v;
}
__device__ __forceinline__ void tag_check(const int* t, int want, int* status) {
  if ((threadIdx.x & 63) == 0 && *t != want && status) atomicOr(status, kStatusRingTag);
}
// negative control (`make lib-diag-fault` only): converters label every slot with a wrong row
#ifndef SSNT_DIAG_TAG_FAULT
#define SSNT_DIAG_TAG_FAULT 0
#endif
constexpr int kTagFault = SSNT_DIAG_TAG_FAULT;
#endif

__device__ __forceinline__ int ctr_ld(const int* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ int ctr_acq(const int* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void ctr_st(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void ctr_rel(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// compiler-only barrier: keeps LDS data accesses and counter accesses in program order (the
// hardware then executes them in that order)
__device__ __forceinline__ void cbar() { asm volatile("" ::: "memory"); }

// Diagnostic build only (-DSSNT_DIAG, `make lib-diag`): per-wave s_memtime totals, read back
// with ssnt_diag_read() (tools/diag_fwd_bwd.py). g_diag[b][wave][8]: 0 total cycles, 1 cycles
// spent spinning, 2 spins that waited, 3 cycle of the cut (chains: alpha[M] / beta[M] stored;
// gradient waves: Z known), 4 cycles spent spinning before the cut. Never present in the product build.
// (s_memtime is a scalar-memory read: reading it waits lgkmcnt(0), i.e. drains the wave's LDS
// queue, so stamps inside a loop perturb what they time.)
#ifdef SSNT_DIAG
__device__ unsigned long long g_diag[1024][2 + 4 * kMaxW][8];
struct Diag {
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), wait = 0, cut = 0, cut_wait = 0;
  unsigned long long ph[3] = {0, 0, 0};  // converters: cycles in convert (incl. load wait), ring write
  unsigned long long n = 0;
  __device__ unsigned long long now() const { return __builtin_amdgcn_s_memtime(); }
  __device__ void mark_cut() {
    cut = now() - t0;
    cut_wait = wait;
  }
  __device__ void flush(int b, int w) {
    if ((threadIdx.x & 63) == 0 && b < 1024) {
      g_diag[b][w][0] = now() - t0;
      g_diag[b][w][1] = wait;
      g_diag[b][w][2] = n;
      g_diag[b][w][3] = cut;
      g_diag[b][w][4] = cut_wait;
      g_diag[b][w][5] = ph[0];
      g_diag[b][w][6] = ph[1];
      g_diag[b][w][7] = ph[2];
    }
  }
};
#else
struct Diag {
  unsigned long long ph[3] = {0, 0, 0};
  __device__ unsigned long long now() const { return 0; }
  __device__ void mark_cut() {}
  __device__ void flush(int, int) {}
  unsigned long long wait = 0, n = 0;
};
#endif

// spin until f() >= target (bounded); returns the last value seen
template <bool SLEEP, typename F>
__device__ __forceinline__ int spin_until(F f, int target, int* status, Diag& dg) {
  int v = f();
  if (v >= target) return v;
  const unsigned long long t = dg.now();
  ++dg.n;
  for (int n = 0; v < target; ++n) {
    if (n > kSpinLimit) {
      if (status && (threadIdx.x & 63) == 0) atomicOr(status, kStatusTimeout);
      return target;
    }
    if constexpr (SLEEP) __builtin_amdgcn_s_sleep(1);
    v = f();
  }
  dg.wait += dg.now() - t;
  return v;
}

// workers w = 0..NW-1 own rows begin + w + NW*i; counter w = rows done. First row not done.
template <int NW>
__device__ __forceinline__ int first_missing(const int* cnt, int begin) {
  int m = INT_MAX;
#pragma unroll
  for (int w = 0; w < NW; ++w) m = min(m, begin + w + NW * ctr_ld(cnt + w));
  return m;
}

// compile-time loop: f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>)
template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// Wave roles: chains, converters, gradient waves, in wave order. The hardware places wave w of
// a workgroup on SIMD (base + w) % 4 (measured, tools/micro/micro_simd.hip), so this order
// spreads each role over all four SIMDs. (Tried: giving each chain a SIMD shared only with
// gradient waves -- idle until the cut -- and packing the converters onto the other two SIMDs:
// the chains ran no faster and the packed converters starved them, 44 -> 48 us. kSimdRoles.)
constexpr bool kSimdRoles = false;
struct Role {
  int kind;  // 0 chain, 1 converter, 2 gradient wave
  int d;     // direction: 0 forward, 1 backward
  int idx;   // converter c / gradient wave h within the direction
  int slot;  // linear index (diagnostics): 0/1 chains, 2+2c+d converters, 2+2kNC+2h+d gradient
};
template <int kNC, int kNH>
__device__ __forceinline__ Role role_of(int w) {
  constexpr int kW = 2 + 2 * kNC + 2 * kNH;
  constexpr int n0 = (kW + 3) / 4, n1 = (kW + 2) / 4, n2 = (kW + 1) / 4, n3 = kW / 4;
  constexpr bool simd_aware = kSimdRoles && n2 >= kNC && n3 >= kNC &&
                              (n0 - 1) + (n2 - kNC) == kNH && (n1 - 1) + (n3 - kNC) == kNH;
  Role r;
  if constexpr (simd_aware) {
    const int g = w & 3, k = w >> 2;
    if (g <= 1) {
      r = k == 0 ? Role{0, g, 0, 0} : Role{2, g, k - 1, 0};
    } else if (k < kNC) {
      r = Role{1, g - 2, k, 0};
    } else {
      r = Role{2, g - 2, (g == 2 ? n0 - 1 : n1 - 1) + (k - kNC), 0};
    }
  } else {
    if (w < 2) r = Role{0, w, 0, 0};
    else if (w < 2 + 2 * kNC) r = Role{1, (w - 2) & 1, (w - 2) >> 1, 0};
    else r = Role{2, (w - 2 - 2 * kNC) & 1, (w - 2 - 2 * kNC) >> 1, 0};
  }
  r.slot = r.kind == 0 ? r.d : r.kind == 1 ? 2 + 2 * r.idx + r.d : 2 + 2 * kNC + 2 * r.idx + r.d;
  return r;
}

// neighbour moves with zero fill at the wave edge (bound_ctrl): foldable into the consumer
__device__ __forceinline__ float shr_z(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ int shr_z(int x) { return __builtin_amdgcn_update_dpp(0, x, 0x138, 0xf, 0xf, true); }
__device__ __forceinline__ float shl_z(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x130, 0xf, 0xf, true));
}
__device__ __forceinline__ int shl_z(int x) { return __builtin_amdgcn_update_dpp(0, x, 0x130, 0xf, 0xf, true); }

// (ma,ea) + (mb,eb) -> normalized; zero results keep a (very negative) exponent >= XF_EZERO
// instead of exactly XF_EZERO: the mantissa is the same as xf_add's and a zero's exponent stays
// below every live exponent, so every value downstream is bit-identical.
//
// Lazy normalization (!OBS, NORM false): the sum is left unnormalized, (s, em), and only every
// kChainNorm-th step pays frexp. Every operation a row then meets -- f32 products and sums of
// ldexp-aligned terms, in the chain, in the gradient products and in the Z tree -- is exact
// under a power-of-two rescaling of its operands, and the mantissas stay within [2^-8, 2^8]
// between normalizations (factor mantissas lie in [0.707, 1.414], all terms are >= 0), far from
// f32 overflow and from the subnormal range wherever a term can still affect a rounded sum. So
// the value represented is the oracle's to the bit, whatever the step's normalization; only
// xf_log needs a normalized input (the debug rows normalize first). The zero clamp moves into
// the exponent max (v_max3_i32) and is therefore applied on every step.
constexpr int kChainNorm = 4;
template <bool NORM>
__device__ __forceinline__ void chain_add(float ma, int ea, float mb, int eb, float om, int oe,
                                          bool obs, float& m, int& e) {
  if (obs) {
    const int em = max(ea, eb);
    float s = xldexp(ma, ea - em) + xldexp(mb, eb - em);
    s = s * om;
    const int ee = em + oe;
    m = xmant(s);
    e = max(ee + xexpo(s), XF_EZERO);
    return;
  }
  const int em = max(max(ea, eb), XF_EZERO);
  const float s = xldexp(ma, ea - em) + xldexp(mb, eb - em);
  if constexpr (NORM) {
    m = xmant(s);
    e = em + xexpo(s);
  } else {
    m = s;
    e = em;
  }
}

// alpha[s+1] = (alpha[s] * E + alpha[s][p-1] * Sh[p-1]) (* O); L = pre-shifted shift factors
template <int K, bool OBS, bool NORM>
__device__ __forceinline__ void alpha_chain(XRow<K>& A, const XRow<K>& E, const XRow<K>& L,
                                            const XRow<K>& O) {
  float hm[K];
  int he[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    hm[j] = ((j == 0) ? shr_z(A.m[K - 1]) : A.m[j - 1]) * L.m[j];
    he[j] = ((j == 0) ? shr_z(A.e[K - 1]) : A.e[j - 1]) + L.e[j];
  }
#pragma unroll
  for (int j = 0; j < K; ++j)
    chain_add<NORM>(A.m[j] * E.m[j], A.e[j] + E.e[j], hm[j], he[j], O.m[j], O.e[j], OBS, A.m[j], A.e[j]);
}

// beta[s] = E * Q[p] + Sh * Q[p+1], Q = beta[s+1] (* O[s+1])
template <int K, bool OBS, bool NORM>
__device__ __forceinline__ void beta_chain(XRow<K>& Bt, const XRow<K>& E, const XRow<K>& Sh,
                                           const XRow<K>& O) {
  float qm[K];
  int qe[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    qm[j] = OBS ? Bt.m[j] * O.m[j] : Bt.m[j];
    qe[j] = OBS ? Bt.e[j] + O.e[j] : Bt.e[j];
  }
  float rm[K];
  int re[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    rm[j] = ((j == K - 1) ? shl_z(qm[0]) : qm[j + 1 < K ? j + 1 : 0]) * Sh.m[j];
    re[j] = ((j == K - 1) ? shl_z(qe[0]) : qe[j + 1 < K ? j + 1 : 0]) + Sh.e[j];
  }
#pragma unroll
  for (int j = 0; j < K; ++j)
    chain_add<OBS || NORM>(E.m[j] * qm[j], E.e[j] + qe[j], rm[j], re[j], 0.0f, 0, false, Bt.m[j], Bt.e[j]);
}

template <int K>
__device__ __forceinline__ XRow<K> xrow_zero() {
  XRow<K> r;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    r.m[j] = 0.0f;
    r.e[j] = XF_EZERO;
  }
  return r;
}

template <int K>
__device__ __forceinline__ XRow<K> lds_xrow(const xf* p) {
  float v[2 * K];
  ld_vec<2 * K>(v, reinterpret_cast<const float*>(p));
  return xrow_unpack<K>(v);
}
template <int K>
__device__ __forceinline__ void lds_xrow_st(xf* p, const XRow<K>& r) {
  float v[2 * K];
  xrow_pack<K>(r, v);
  st_vec<2 * K>(reinterpret_cast<float*>(p), v);
}

// Global accesses of a lane's K positions, F floats per position. NV (narrow): one access per
// position -- U % K != 0 or tensors aligned to 8 or 4 bytes: a slice may straddle the row end, and each
// position is then entirely inside the row's buffer range or entirely outside it (reads 0,
// stores dropped). Otherwise one vector access per slice.
template <int K, int F, bool NV>
__device__ __forceinline__ void gld(float* dst, __amdgpu_buffer_rsrc_t r, int p0) {
  if constexpr (NV) {
#pragma unroll
    for (int j = 0; j < K; ++j) buf_ld<F>(dst + F * j, r, (p0 + j) * 4 * F);
  } else {
    buf_ld<F * K>(dst, r, p0 * 4 * F);
  }
}
template <int K, int F, bool NV>
__device__ __forceinline__ void gst(const float* v, __amdgpu_buffer_rsrc_t r, int p0) {
  if constexpr (NV) {
#pragma unroll
    for (int j = 0; j < K; ++j) buf_st<F>(v + F * j, r, (p0 + j) * 4 * F);
  } else {
    buf_st<F * K>(v, r, p0 * 4 * F);
  }
}


}  // namespace
}  // namespace ssnt
