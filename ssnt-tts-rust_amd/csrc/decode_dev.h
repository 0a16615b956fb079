// decode_dev.h -- device-side pieces of the beam-search step shared by the per-step kernels
// (decode.hip) and the fused multi-step kernels (fused_decode.hip): the candidate record, the
// expansion rules of v1 / v2 / tone, and the one-wave LDS step (rank, dedup, diagonal, pad).
#pragma once
#include <hip/hip_runtime.h>

#include "ssnt_internal.h"

namespace ssnt {
namespace dec {

typedef unsigned long long u64;

struct Cand {
  u64 nt, nu;  // next_t / next_u as Rust usize
  float lp;
  int pred, parent, tot;
  int fin, valid;
};

__device__ __forceinline__ u64 as_usize(int v) { return (u64)(long long)v; }

// Rust `f32 as i32` (saturating, NaN -> 0)
__device__ __forceinline__ int f2i_sat(float x) {
  if (x != x) return 0;
  if (x >= 2147483648.0f) return 2147483647;
  if (x <= -2147483648.0f) return (-2147483647 - 1);
  return (int)x;
}

// the same as selects only (no exec-mask branch): below 2^31 the clamp is exact (the largest f32
// under 2^31 is 2^31 - 128), at or above it the saturated value is selected, NaN gives 0
__device__ __forceinline__ int f2i_sat_sel(float x) {
  const int r = (int)fminf(fmaxf(x, -2147483648.0f), 2147483520.0f);
  const int s = x >= 2147483648.0f ? 2147483647 : r;
  return x != x ? 0 : s;
}

// Sort key of a log-prob: the IEEE order of the reference's comparison (src/lib.rs:161), so -0
// and +0 share a key, extended to a total order by placing NaN below -inf. NaN inputs are
// outside the parity contract; the total order only guarantees that ranks are
// a permutation (every output stays in range). Never 0: 0 marks "no candidate".
__device__ __forceinline__ unsigned lp_key(float x) {  // selects only: no exec-mask branch
  // x + 0 maps -0 to +0 and is x otherwise (NaN aside); flipping every bit of a negative value
  // and the sign bit of a positive one orders the bit patterns like the floats
  const unsigned bits = __float_as_uint(x + 0.0f);
  const unsigned key = bits ^ ((unsigned)((int)bits >> 31) | 0x80000000u);
  return x != x ? 1u : key;
}

__device__ __forceinline__ bool cand_eq(const Cand& a, const Cand& b, bool with_tot) {
  return a.pred == b.pred && a.lp == b.lp && a.nt == b.nt && a.nu == b.nu && a.fin == b.fin &&
         (!with_tot || a.tot == b.tot);
}

struct BatchView {
  const float* h;
  const float* hist;
  const bool* fin;
  const int* t;
  const int* u;
  const int* total;
  u64 I, O;
};

// Candidate c = w*C + i (generation order of src/lib.rs:150-158's ordered flat_map).
__device__ Cand gen_candidate(const StepArgs& a, const BatchView& v, int c) {
  const int C = a.C;
  const int w = c / C, i = c - w * C;
  const u64 t = as_usize(v.t[w]);
  const u64 u = as_usize(v.u[w]);
  const float hist = v.hist[w];
  const bool defined = (t < v.I) && !v.fin[w];  // decode_beam_at (src/lib.rs:57-67 etc.)
  Cand r;
  r.parent = w;
  r.tot = 0;
  if (!defined) {  // "End of input. Return values to fill padding region."
    r.valid = (i == 0);
    r.pred = a.variant == Variant::V1 ? 0 : a.special_id;
    r.lp = hist;
    r.nt = t;
    r.nu = u;
    r.fin = 1;
    r.tot = a.variant == Variant::V2 ? v.total[w] : 0;
    return r;
  }
  const float hv = v.h[w * C + i];
  r.valid = 1;
  if (a.variant == Variant::V1) {  // src/lib.rs:186-227
    const u64 last = v.I - 1;
    if (i == 0 && t == last) {
      r.pred = 0; r.lp = hist + hv; r.nt = t; r.nu = u; r.fin = 1;
    } else if (i == 1 && t == last) {  // prohibited shift
      r.pred = 0; r.lp = hist; r.nt = t; r.nu = u; r.fin = 1;
    } else if (i == 1) {
      r.pred = 1; r.lp = hist + hv; r.nt = t + 1; r.nu = u + 1; r.fin = 0;
    } else {
      r.pred = 0; r.lp = hist + hv; r.nt = t; r.nu = u + 1; r.fin = 0;
    }
    return r;
  }
  if (a.variant == Variant::Tone) {  // src/tone_latent.rs:87-93, 220-231
    r.pred = i; r.lp = hist + hv; r.nt = t + 1; r.nu = u + 1; r.fin = 0;
    return r;
  }
  // v2: src/v2.rs:119-166, 326-336
  const int duration = a.table[i];
  const int tot = (int)((unsigned)v.total[w] + (unsigned)duration);
  const float diagonal = (float)v.O / (float)v.I * (float)(t + 1);
  const float upper_range = (float)v.O * 0.1f;
  const float lower_range = (float)v.O * 0.05f;
  const int lb = f2i_sat(fmaxf(diagonal - lower_range, 0.0f));
  const int ub = f2i_sat(fminf(diagonal + upper_range, (float)v.O));
  const u64 remaining = v.I - (t + 1);
  const bool overrun = remaining * 3 > v.O;
  bool fin = false;
  bool ok = true;
  if (!a.test_mode && (tot < lb || tot > ub)) ok = false;
  else if (!a.test_mode && overrun) ok = false;
  else if (t == v.I - 1) {
    if (!a.test_mode && tot != (int)v.O) ok = false;
    else if (!a.allow_skip && i == a.special_id) ok = false;
    else fin = true;
  } else if (!a.allow_skip && i == a.special_id) ok = false;
  r.valid = ok;
  r.pred = i;
  r.lp = hist + hv;
  r.nt = fin ? t : t + 1;
  r.nu = fin ? u : u + 1;
  r.fin = fin;
  r.tot = tot;
  return r;
}

__device__ __forceinline__ bool on_diagonal(const BatchView& v, const Cand& r) {
  const float diagonal = (float)v.O / (float)v.I * (float)r.nt;  // src/v2.rs:113-117
  const float diff = (float)r.tot - diagonal;
  return diff >= -20.0f && diff <= 0.0f;
}

__device__ __forceinline__ int wave_sum(int x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
  return x;
}
__device__ __forceinline__ int wave_min(int x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x = min(x, __shfl_xor(x, off));
  return x;
}

// One decode step for one batch element, executed by the whole wave. `cand` has n = W*C
// entries, `order` and `kept` n ints each (LDS). Writes the Wmax result slots through `emit`.
// Returns n_kept (0 = no candidate).
template <typename Emit>
__device__ int step_wave(const StepArgs& a, const BatchView& v, Cand* cand, int* order, int* kept,
                         int Wmax, Emit emit) {
  const int lane = threadIdx.x & 63;
  const int n = a.W * a.C;
  for (int c = lane; c < n; c += 64) cand[c] = gen_candidate(a, v, c);
  __syncthreads();
  // rank = position in the stable descending sort
  int nvalid_local = 0;
  for (int c = lane; c < n; c += 64) {
    const Cand me = cand[c];
    if (!me.valid) continue;
    ++nvalid_local;
    const unsigned km = lp_key(me.lp);
    int rank = 0;
    for (int j = 0; j < n; ++j) {
      const unsigned kj = lp_key(cand[j].lp);
      const int vj = cand[j].valid;
      rank += (vj && (kj > km || (kj == km && j < c))) ? 1 : 0;
    }
    order[rank] = c;
  }
  const int nvalid = wave_sum(nvalid_local);
  __syncthreads();
  // consecutive dedup (keep first of each run), stream-compacted into kept[]
  const bool with_tot = a.variant == Variant::V2;
  int base = 0;
  for (int r0 = 0; r0 < nvalid; r0 += 64) {
    const int r = r0 + lane;
    bool keep = false;
    if (r < nvalid) keep = (r == 0) || !cand_eq(cand[order[r]], cand[order[r - 1]], with_tot);
    const u64 mask = __ballot(keep);
    const int pos = base + __popcll(mask & ((1ull << lane) - 1ull));
    if (keep) kept[pos] = order[r];
    base += __popcll(mask);
  }
  const int nkept = base;
  __syncthreads();
  if (nkept == 0) return 0;
  int diag = nkept;  // first kept candidate on the diagonal (v2, not test_mode)
  if (a.variant == Variant::V2 && !a.test_mode) {
    int best = nkept;
    for (int k = lane; k < nkept; k += 64)
      if (on_diagonal(v, cand[kept[k]])) {
        best = k;
        break;
      }
    diag = wave_min(best);
  }
  for (int i = lane; i < Wmax; i += 64) {
    const int k = (diag < nkept && i == Wmax - 1) ? diag : (i % nkept);
    emit(i, cand[kept[k]]);
  }
  return nkept;
}


// lane helpers for one-candidate-per-lane steps
__device__ __forceinline__ int perm_i(int dst_lane, int v) {  // lane sends v to dst_lane
  return __builtin_amdgcn_ds_permute(dst_lane << 2, v);
}
__device__ __forceinline__ int bperm_i(int src_lane, int v) {  // lane reads v from src_lane
  return __builtin_amdgcn_ds_bpermute(src_lane << 2, v);
}
__device__ __forceinline__ int wave_shr1(int v) {  // lane l gets lane l-1's v (lane 0: 0)
  return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false);
}

// max of x over each aligned group of N lanes (N = 8, 16, 32, 64), every lane of the group ends
// with it: quad xor moves, the half-mirror / mirror (xor 4 / 8 once the smaller groups agree) by
// DPP, then 16- and 32-lane swaps by v_permlane16/32_swap -- VALU only, no LDS
template <int N>
__device__ __forceinline__ unsigned group_max_u32(unsigned x) {
  static_assert(N == 8 || N == 16 || N == 32 || N == 64, "group size");
  x = max(x, (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, false));   // xor 1
  x = max(x, (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, false));   // xor 2
  x = max(x, (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xf, 0xf, false));  // 8-group
  if constexpr (N >= 16) x = max(x, (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xf, 0xf, false));
  if constexpr (N >= 32) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    x = max((unsigned)r[0], (unsigned)r[1]);
  }
  if constexpr (N >= 64) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    x = max((unsigned)r[0], (unsigned)r[1]);
  }
  return x;
}
__device__ __forceinline__ int readlane_i(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }

}  // namespace dec
}  // namespace ssnt
