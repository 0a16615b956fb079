// lattice_dev.h -- device building blocks shared by the lattice forward-backward kernels
// (fwd_bwd.hip: two-wave kernel; fwd_bwd_stream.hip: streaming kernel). Split-exponent
// arithmetic itself is in xf_math.h.
#pragma once
#include <hip/hip_runtime.h>

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

// A debug row: f32 log values, or -- raw-state mode (dst_e set, ssnt_fwd_bwd_debug64_device) --
// the normalized mantissas into dst and the exponents into dst_e, from which the host entry forms
// float64 logs. The same normalization xf_log starts from, so nothing is rounded on the way.
template <int K, bool VEC>
__device__ __forceinline__ void store_dbg_row(float* __restrict__ dst, int* __restrict__ dst_e,
                                              const XRow<K>& r, int U, int lane) {
  if (dst_e) {
    float m[K], e[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const xf n = xf_norm(r.m[j], r.e[j]);
      m[j] = n.m;
      e[j] = __builtin_bit_cast(float, n.e);
    }
    store_f_row<K, VEC>(dst, m, U, lane);
    store_f_row<K, VEC>(reinterpret_cast<float*>(dst_e), e, U, lane);
  } else {
    store_log_row<K, VEC>(dst, r, U, lane);
  }
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
  f2 p = (f2){0x1.6b6ep-10f, 0x1.6b6ep-10f};
  p = __builtin_elementwise_fma(p, r, (f2){0x1.122f66p-7f, 0x1.122f66p-7f});
  p = __builtin_elementwise_fma(p, r, (f2){0x1.555688p-5f, 0x1.555688p-5f});
  p = __builtin_elementwise_fma(p, r, (f2){0x1.5554a4p-3f, 0x1.5554a4p-3f});
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

// Batch loss sum inside the launch (ssnt_fwd_bwd_sum_device). Utterance b publishes
// {tag, loss bits} as ONE 8-byte write-through granule (MI355X hand-off form R2: the data is the
// flag -- no fence, no read-modify-write atomic, nothing for 256 workgroups to serialise on).
// Workgroup 0 re-reads the B granules until every tag is this launch's, sums them in a fixed
// order (64 lane-strided partial sums, then an xor butterfly: f32 addition is commutative, so
// every lane ends with the same bits) and advances the epoch word. State layout: u32 epoch at
// byte 0, granule b at byte 64 + 8b; all zero before the first call.
constexpr size_t kSumGranuleOffset = 64;
__device__ __forceinline__ unsigned long long* sum_granule(const FwdBwdArgs& a, int b) {
  return reinterpret_cast<unsigned long long*>(reinterpret_cast<unsigned char*>(a.sum_state) +
                                               kSumGranuleOffset) + b;
}
// this launch's tag: epoch + 1 (the epoch only advances after every workgroup has published)
__device__ __forceinline__ unsigned sum_tag(const FwdBwdArgs& a) {
  return __hip_atomic_load(reinterpret_cast<unsigned*>(a.sum_state), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT) + 1u;
}
// one lane: loss[b] = v, and the granule when a batch sum is requested
__device__ __forceinline__ void publish_loss(const FwdBwdArgs& a, int b, float v, unsigned tag) {
  a.loss[b] = v;
  if (a.loss_sum)
    __hip_atomic_store(sum_granule(a, b),
                       ((unsigned long long)tag << 32) | __builtin_bit_cast(unsigned, v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one wave of workgroup 0: wait for every granule of this launch, write the sum, advance epoch
__device__ __forceinline__ void finish_loss_sum(const FwdBwdArgs& a, unsigned tag) {
  const int lane = threadIdx.x & 63;
  for (int spins = 0;; ++spins) {
    bool ok = true;
    for (int i = lane; i < a.B; i += 64)
      ok &= (unsigned)(__hip_atomic_load(sum_granule(a, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) == tag;
    if (__all(ok)) break;
    if (spins > (1 << 24)) {  // bounded (~4 s): report, poison the sum, still advance the epoch
      // (a later launch must never accept this launch's granules: its tag is epoch + 1 again
      // only if the epoch moved on)
      if (lane == 0) {
        if (a.status) atomicOr(a.status, kStatusTimeout);
        *a.loss_sum = __builtin_nanf("");
        __hip_atomic_store(reinterpret_cast<unsigned*>(a.sum_state), tag, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  float acc = 0.0f;
  for (int i = lane; i < a.B; i += 64)
    acc += __builtin_bit_cast(float, (unsigned)__hip_atomic_load(sum_granule(a, i), __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
  if (lane == 0) {
    *a.loss_sum = acc;
    __hip_atomic_store(reinterpret_cast<unsigned*>(a.sum_state), tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// the same fixed order over a finished loss[] (the separate pass when no state is given)
__device__ __forceinline__ float wave_loss_sum(const float* loss, int B) {
  const int lane = threadIdx.x & 63;
  float acc = 0.0f;
  for (int i = lane; i < B; i += 64) acc += loss[i];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
  return acc;
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

}  // namespace
}  // namespace ssnt
