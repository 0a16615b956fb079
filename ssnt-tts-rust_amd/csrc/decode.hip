// decode.hip -- beam-search decode steps and alignment utilities for gfx950.
//
// One wave (64 lanes) owns one batch element. A step generates every candidate of every beam
// into LDS, ranks them (stable descending sort on log_prob, generation index as tie-break,
// src/lib.rs:161), drops consecutive duplicates (src/lib.rs:162), optionally injects v2's
// on-diagonal candidate (src/v2.rs:283-308) and pads cyclically (src/lib.rs:163-167). All of it
// is integer / compare work plus one f32 add per candidate, so the result is bit-exact with the
// Rust step (and with oracle/ssnt_oracle.c) by construction.
#include <hip/hip_runtime.h>

#include "decode_dev.h"

namespace ssnt {
namespace {

using namespace dec;

__global__ __launch_bounds__(64) void k_decode_step(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int n = a.W * a.C;
  Cand* cand = reinterpret_cast<Cand*>(smem);
  int* order = reinterpret_cast<int*>(cand + n);
  int* kept = order + n;
  BatchView v;
  const size_t bw = (size_t)b * a.W;
  v.h = a.h + bw * a.C;
  v.hist = a.hist + bw;
  v.fin = a.fin + bw;
  v.t = a.t + bw;
  v.u = a.u + bw;
  v.total = a.total ? a.total + bw : nullptr;
  v.I = as_usize(a.input_length ? a.input_length[b] : a.scalar_input_length);
  v.O = as_usize(a.output_length ? a.output_length[b] : 0);
  const size_t o = (size_t)b * a.Wmax;
  const int nk = step_wave(a, v, cand, order, kept, a.Wmax, [&](int i, const Cand& r) {
    a.prediction[o + i] = r.pred;  // src/lib.rs:138-145
    a.log_prob[o + i] = r.lp;
    a.next_t[o + i] = (int)(unsigned)r.nt;
    a.next_u[o + i] = (int)(unsigned)r.nu;
    a.beam_branch[o + i] = r.parent;
    a.next_fin[o + i] = r.fin != 0;
    if (a.next_total) a.next_total[o + i] = r.tot;
  });
  if (nk == 0 && a.status && (threadIdx.x & 63) == 0) atomicOr(a.status, kStatusNoCandidate);
}

// Fused multi-step v1 decode: the whole T-step loop of one utterance in one wave. Beam state
// lives in LDS (W entries); step s reads h[w] = lattice[b, u_w, t_w, :] where every live beam has
// u_w = s (each step advances u by one; finished beams read nothing, src/lib.rs:175-226). So
// row s of the lattice does not depend on the beam state: rows are prefetched kRowAhead steps
// ahead into registers and staged in LDS, and a step's only dependent read is an LDS read --
// not an HBM round trip per step (that was ~1 us of each ~2.5 us step before).
constexpr int kRowAhead = 4;    // lattice rows in flight
constexpr int kRowRegs = 4;     // floats per lane per row: staged while 2U <= 256
template <bool STAGED>
__global__ __launch_bounds__(64) void k_lattice_decode(LatticeDecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int W = a.W, T = a.T, U = a.U;
  const int n = 2 * W;
  Cand* cand = reinterpret_cast<Cand*>(smem);
  int* order = reinterpret_cast<int*>(cand + n);
  int* kept = order + n;
  float* hbuf = reinterpret_cast<float*>(kept + n);   // (W,2)
  float* hist = hbuf + 2 * W;                         // (W)
  int* tt = reinterpret_cast<int*>(hist + W);         // (W)
  int* uu = tt + W;                                   // (W)
  float* rowbuf = reinterpret_cast<float*>(uu + W);   // (U,2): lattice row s (STAGED)
  bool* ff = reinterpret_cast<bool*>(rowbuf + (STAGED ? 2 * U : 0));  // (W)
  StepArgs sa{};
  sa.variant = Variant::V1;
  sa.B = a.B;
  sa.W = W;
  sa.Wmax = W;
  sa.C = 2;
  BatchView v;
  v.h = hbuf;
  v.hist = hist;
  v.fin = ff;
  v.t = tt;
  v.u = uu;
  v.total = nullptr;
  v.I = as_usize(a.input_length[b]);
  v.O = 0;
  const float* lat = a.lattice + (size_t)b * T * U * 2;
  const int row_len = 2 * U;
  for (int w = lane; w < W; w += 64) {
    hist[w] = 0.0f;
    tt[w] = 0;
    uu[w] = 0;
    ff[w] = false;
  }
  float pre[kRowAhead][kRowRegs];
  // unconditional (clamped) loads: a conditional load becomes a branch whose join waits
  // vmcnt(0), i.e. for the load just issued -- which would undo the prefetch
  auto load_row = [&](int s, float* dst) {  // the row does not depend on the beam state
#pragma unroll
    for (int q = 0; q < kRowRegs; ++q)
      dst[q] = lat[(size_t)min(s, T - 1) * row_len + min(lane + 64 * q, row_len - 1)];
  };
  if constexpr (STAGED) {
#pragma unroll
    for (int k = 0; k < kRowAhead; ++k) load_row(k, pre[k]);
  }
  __syncthreads();
  auto step = [&](int s, float* staged_row) {
    if constexpr (STAGED) {  // row s to LDS, then row s + kRowAhead into the freed registers
#pragma unroll
      for (int q = 0; q < kRowRegs; ++q) {
        const int idx = lane + 64 * q;
        if (idx < row_len) rowbuf[idx] = staged_row[q];
      }
      load_row(s + kRowAhead, staged_row);
      __syncthreads();
    }
    for (int w = lane; w < W; w += 64) {
      const bool defined = !ff[w] && as_usize(tt[w]) < v.I && (unsigned)uu[w] < (unsigned)T &&
                           (unsigned)tt[w] < (unsigned)U;
      float2 x = make_float2(0.0f, 0.0f);
      if (defined) {
        if constexpr (STAGED) {
          x = make_float2(rowbuf[2 * tt[w]], rowbuf[2 * tt[w] + 1]);  // uu[w] == s
        } else {
          x = *reinterpret_cast<const float2*>(lat + ((size_t)uu[w] * U + tt[w]) * 2);
        }
      }
      hbuf[2 * w] = x.x;
      hbuf[2 * w + 1] = x.y;
    }
    __syncthreads();
    const size_t o = ((size_t)b * T + s) * W;
    // results are staged in registers, state is updated after every lane has read it
    int rnt = 0, rnu = 0;
    float rlp = 0.0f;
    bool rfin = false;
    step_wave(sa, v, cand, order, kept, W, [&](int i, const Cand& r) {
      a.prediction[o + i] = r.pred;
      a.log_prob[o + i] = r.lp;
      a.next_t[o + i] = (int)(unsigned)r.nt;
      a.next_u[o + i] = (int)(unsigned)r.nu;
      a.beam_branch[o + i] = r.parent;
      a.next_fin[o + i] = r.fin != 0;
      rlp = r.lp;
      rnt = (int)(unsigned)r.nt;
      rnu = (int)(unsigned)r.nu;
      rfin = r.fin != 0;
    });
    __syncthreads();
    if (lane < W) {
      hist[lane] = rlp;
      tt[lane] = rnt;
      uu[lane] = rnu;
      ff[lane] = rfin;
    }
    __syncthreads();
  };
  for (int s0 = 0; s0 < T; s0 += kRowAhead) {  // unrolled by the ring: register indices fixed
#pragma unroll
    for (int k = 0; k < kRowAhead; ++k)
      if (s0 + k < T) step(s0 + k, pre[k]);
  }
}

// Register-resident fused v1 decode for 2W <= 64 candidates (config 3: W = 4). Same step
// contract as step_wave (src/lib.rs:149-230; DESIGN.md / SURVEY.md Appendix A), but every
// candidate lives in one lane and never touches LDS: rank by v_readlane over the other
// candidates (stable: ties by generation index), ds_permute into sorted order, consecutive dedup
// against the DPP-shifted neighbour, ballot + ds_permute compaction, ds_bpermute cyclic pad.
// Beam w's state (hist, t, u, fin) is held by lane w between steps.
// Per-step outputs are staged in LDS and written out every kOutChunk steps: a global store
// inside the step makes the next row prefetch's vmcnt wait also wait for that store (~1 us).
constexpr int kOutChunk = 32;
template <bool STAGED>
__global__ __launch_bounds__(64) void k_lattice_decode_reg(LatticeDecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int W = a.W, T = a.T, U = a.U;
  int* o_pred = reinterpret_cast<int*>(smem);       // (kOutChunk, W) each
  float* o_lpb = reinterpret_cast<float*>(o_pred + kOutChunk * W);
  int* o_nt = reinterpret_cast<int*>(o_lpb + kOutChunk * W);
  int* o_nu = o_nt + kOutChunk * W;
  int* o_br = o_nu + kOutChunk * W;
  int* o_fin = o_br + kOutChunk * W;
  float* rowbuf = reinterpret_cast<float*>(o_fin + kOutChunk * W);  // (U,2): lattice row s
  const int n = 2 * W;
  const u64 I = as_usize(a.input_length[b]);
  const float* lat = a.lattice + (size_t)b * T * U * 2;
  const int row_len = 2 * U;
  // beam state, lane w < W
  float hist = 0.0f;
  int bt = 0, bu = 0, bfin = 0;
  float pre[kRowAhead][kRowRegs];
  // unconditional (clamped) loads: a conditional load becomes a branch whose join waits
  // vmcnt(0), i.e. for the load just issued -- which would undo the prefetch
  auto load_row = [&](int s, float* dst) {  // the row does not depend on the beam state
#pragma unroll
    for (int q = 0; q < kRowRegs; ++q)
      dst[q] = lat[(size_t)min(s, T - 1) * row_len + min(lane + 64 * q, row_len - 1)];
  };
  if constexpr (STAGED) {
#pragma unroll
    for (int k = 0; k < kRowAhead; ++k) load_row(k, pre[k]);
  }
  const int c = lane;          // candidate index = w*2 + i (generation order, src/lib.rs:150-158)
  const int w = c >> 1, i = c & 1;
  const bool is_cand = c < n;
  auto step = [&](int s, float* staged_row) {
    if constexpr (STAGED) {
#pragma unroll
      for (int q = 0; q < kRowRegs; ++q) {
        const int idx = lane + 64 * q;
        if (idx < row_len) rowbuf[idx] = staged_row[q];
      }
      load_row(s + kRowAhead, staged_row);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    // ---- candidates (gen_candidate, V1)
    const float ph = __shfl(hist, w);
    const int pt = __shfl(bt, w), pu = __shfl(bu, w), pf = __shfl(bfin, w);
    const bool defined = !pf && as_usize(pt) < I;
    const bool hdef = defined && (unsigned)pu < (unsigned)T && (unsigned)pt < (unsigned)U;
    float hv = 0.0f;
    if (is_cand && hdef) {
      if constexpr (STAGED) hv = rowbuf[2 * pt + i];  // pu == s for every live beam
      else hv = lat[((size_t)pu * U + pt) * 2 + i];
    }
    int valid, pred, nt, nu, fin;
    float lp;
    if (!defined) {  // "End of input": one finished candidate per beam (src/lib.rs:175-184)
      valid = (i == 0); pred = 0; lp = ph; nt = pt; nu = pu; fin = 1;
    } else {
      const bool last = as_usize(pt) == I - 1;
      valid = 1;
      if (i == 0 && last) { pred = 0; lp = ph + hv; nt = pt; nu = pu; fin = 1; }
      else if (i == 1 && last) { pred = 0; lp = ph; nt = pt; nu = pu; fin = 1; }  // prohibited shift
      else if (i == 1) { pred = 1; lp = ph + hv; nt = pt + 1; nu = pu + 1; fin = 0; }
      else { pred = 0; lp = ph + hv; nt = pt; nu = pu + 1; fin = 0; }
    }
    valid = valid && is_cand;
    // ---- stable descending rank among valid candidates (src/lib.rs:161)
    int rank = 0;
    for (int j = 0; j < n; ++j) {
      const float lj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lp), j));
      const int vj = __builtin_amdgcn_readlane(valid, j);
      rank += (vj && (lj > lp || (lj == lp && j < c))) ? 1 : 0;
    }
    const u64 vmask = __ballot(valid);
    const int nvalid = __popcll(vmask);
    // ---- into sorted order: lane r holds the candidate of rank r (r < nvalid)
    const int packed = pred | (fin << 1) | (w << 2);
    // a full permutation of the 64 lanes (ds_permute must not send two values to one lane):
    // valid candidates to their rank, the other lanes after them in lane order
    const u64 below = (1ull << lane) - 1ull;
    const int dst = valid ? rank : nvalid + __popcll(~vmask & below);
    const int s_lp = perm_i(dst, __builtin_bit_cast(int, lp));
    const int s_nt = perm_i(dst, nt);
    const int s_nu = perm_i(dst, nu);
    const int s_pk = perm_i(dst, packed);
    // ---- consecutive dedup, keep the first of each run (src/lib.rs:162, eq_ignore_parent :81-87)
    const float q_lp = __builtin_bit_cast(float, s_lp);
    const float p_lp = __builtin_bit_cast(float, wave_shr1(s_lp));
    const int p_nt = wave_shr1(s_nt), p_nu = wave_shr1(s_nu), p_pk = wave_shr1(s_pk);
    const bool same = (s_pk & 3) == (p_pk & 3) && q_lp == p_lp && s_nt == p_nt && s_nu == p_nu;
    const bool keep = lane < nvalid && (lane == 0 || !same);
    const u64 kmask = __ballot(keep);
    const int nkept = __popcll(kmask);
    // compact: kept candidate k to lane k (again a full permutation)
    const int cdst = keep ? __popcll(kmask & below) : nkept + __popcll(~kmask & below);
    const int k_lp = perm_i(cdst, s_lp);
    const int k_nt = perm_i(cdst, s_nt);
    const int k_nu = perm_i(cdst, s_nu);
    const int k_pk = perm_i(cdst, s_pk);
    // ---- cyclic pad to W slots (src/lib.rs:163-168): slot i <- kept[i % nkept]
    const int src = (lane < W ? lane : 0) % (nkept > 0 ? nkept : 1);
    const float o_lp = __builtin_bit_cast(float, bperm_i(src, k_lp));
    const int o_nt_r = bperm_i(src, k_nt), o_nu_r = bperm_i(src, k_nu), o_pk = bperm_i(src, k_pk);
    const int cs = s % kOutChunk;
    if (lane < W) {
      const int o = cs * W + lane;
      o_pred[o] = o_pk & 1;
      o_lpb[o] = o_lp;
      o_nt[o] = o_nt_r;
      o_nu[o] = o_nu_r;
      o_br[o] = o_pk >> 2;
      o_fin[o] = (o_pk >> 1) & 1;
      hist = o_lp;
      bt = o_nt_r;
      bu = o_nu_r;
      bfin = (o_pk >> 1) & 1;
    }
    if (cs == kOutChunk - 1 || s == T - 1) {  // flush the chunk, coalesced (one wave: in order)
      const int s_first = s - cs;
      const int cnt = (cs + 1) * W;
      const size_t g0 = ((size_t)b * T + s_first) * W;
      for (int k = lane; k < cnt; k += 64) {
        a.prediction[g0 + k] = o_pred[k];
        a.log_prob[g0 + k] = o_lpb[k];
        a.next_t[g0 + k] = o_nt[k];
        a.next_u[g0 + k] = o_nu[k];
        a.beam_branch[g0 + k] = o_br[k];
        a.next_fin[g0 + k] = o_fin[k] != 0;
      }
    }
    if constexpr (STAGED) __builtin_amdgcn_s_barrier();  // rowbuf is rewritten next step
  };
  for (int s0 = 0; s0 < T; s0 += kRowAhead) {
#pragma unroll
    for (int k = 0; k < kRowAhead; ++k)
      if (s0 + k < T) step(s0 + k, pre[k]);
  }
}

// Backtrace along beam_branch (B,T,W) for n_paths (<= 64) final branches per batch element
// (util.rs:20-33 with n_paths = 1 and t history; v2_util.rs:6-36 with n_paths = W). A null
// final_branch means branch 0 (the best slot after the final sort). Rows are staged into LDS
// in chunks (coalesced), then lane k walks path k back through the chunk.
__global__ __launch_bounds__(64) void k_backtrace(int B, int W, int T, int n_paths,
                                                  const int* __restrict__ final_branch,
                                                  const int* __restrict__ beam_branch,
                                                  const int* __restrict__ t_history,
                                                  int* __restrict__ out_branch,
                                                  int* __restrict__ out_t, int chunk, int* status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* sb = reinterpret_cast<int*>(smem);
  int* st = sb + (size_t)chunk * W;
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int* bb = beam_branch + (size_t)b * T * W;
  const int* th = t_history ? t_history + (size_t)b * T * W : nullptr;
  const bool active = lane < n_paths;
  int c = (active && final_branch) ? final_branch[(size_t)b * n_paths + lane] : 0;
  int* ob = out_branch + ((size_t)b * n_paths + lane) * T;
  int* ot = out_t ? out_t + ((size_t)b * n_paths + lane) * T : nullptr;
  bool bad = false;
  for (int hi = T; hi > 0; hi -= chunk) {
    const int lo = max(hi - chunk, 0);
    const int cnt = (hi - lo) * W;
    __syncthreads();
    for (int i = lane; i < cnt; i += 64) {
      sb[i] = bb[(size_t)lo * W + i];
      if (th) st[i] = th[(size_t)lo * W + i];
    }
    __syncthreads();
    if (active) {
      for (int s = hi - 1; s >= lo; --s) {
        if (c < 0 || c >= W) {  // Rust would panic on the out-of-bounds index
          bad = true;
          c = c < 0 ? 0 : W - 1;
        }
        ob[s] = c;
        const int r = (s - lo) * W + c;
        if (ot) ot[s] = st[r];
        c = sb[r];
      }
    }
  }
  if (bad && status) atomicOr(status, kStatusBadIndex);
}

__device__ __forceinline__ int wave_incl_scan_add(int x, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  return x;
}
__device__ __forceinline__ int wave_incl_scan_min(int x, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off);
    if (lane >= off) x = min(x, y);
  }
  return x;
}

// upsample_source_indexes (src/v2_util.rs:39-66): one wave per (b,w) row.
__global__ __launch_bounds__(64) void k_upsample(int rows, int T, int max_u,
                                                 const int* __restrict__ duration,
                                                 const int* __restrict__ output_length,
                                                 int* __restrict__ out, int* status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* cum = reinterpret_cast<int*>(smem);  // inclusive prefix sums (T)
  const int r = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int* d = duration + (size_t)r * T;
  long long carry = 0;
  bool neg = false;
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + lane;
    const int x = t < T ? d[t] : 0;
    neg |= x < 0;
    const int inc = wave_incl_scan_add(x, lane);
    if (t < T) cum[t] = (int)(carry + inc);
    carry += __shfl(inc, 63);
  }
  const bool anyneg = __any(neg);
  const int L = output_length[r];
  if (anyneg || carry != (long long)L) {
    if (lane == 0 && status) atomicOr(status, kStatusDurationMismatch);
    return;
  }
  __syncthreads();
  const int n = min(L, max_u);
  int* o = out + (size_t)r * max_u;
  for (int k = lane; k < n; k += 64) {
    int lo = 0, hi = T;  // first t with cum[t] > k
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cum[mid] > k) hi = mid;
      else lo = mid + 1;
    }
    o[k] = lo;
  }
}

// Levenshtein distance (src/edit_distance.rs:27-60, Kaldi): one wave per pair. Row m of the DP
// is new[n] = n + prefix_min_{n'<=n}(base[n'] - n'), base[n] = min(e[n-1]+delta, e[n]+1),
// base[0] = e[0]+1 -- the in-row dependency of the reference loop as a wave min-scan.
__global__ __launch_bounds__(64) void k_levenshtein(int B, int L, const int* __restrict__ a,
                                                    const int* __restrict__ bsq,
                                                    const int* __restrict__ a_len,
                                                    const int* __restrict__ b_len,
                                                    int* __restrict__ dist) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* e = reinterpret_cast<int*>(smem);  // (L+1)
  int* nb = e + (L + 1);                  // (L+1)
  const int i = blockIdx.x;
  const int lane = threadIdx.x & 63;
  // lengths outside [0, L] panic in the reference (slice bounds); the host layer rejects them,
  // the kernel clamps so a bad device-side length can never read out of bounds
  const int M = min(max(a_len[i], 0), L), N = min(max(b_len[i], 0), L);
  const int* A = a + (size_t)i * L;
  const int* Bv = bsq + (size_t)i * L;
  for (int n = lane; n <= N; n += 64) e[n] = n;
  __syncthreads();
  for (int m = 1; m <= M; ++m) {
    const int am = A[m - 1];
    int carry = 0x3fffffff;
    for (int n0 = 0; n0 <= N; n0 += 64) {
      const int n = n0 + lane;
      int base = 0x3fffffff;
      if (n == 0) base = e[0] + 1;
      else if (n <= N) base = min(e[n - 1] + (am == Bv[n - 1] ? 0 : 1), e[n] + 1);
      int v = (n <= N) ? base - n : 0x3fffffff;
      v = wave_incl_scan_min(v, lane);
      v = min(v, carry);
      if (n <= N) nb[n] = n + v;
      carry = __shfl(v, 63);
    }
    __syncthreads();
    for (int n = lane; n <= N; n += 64) e[n] = nb[n];
    __syncthreads();
  }
  if (lane == 0) dist[i] = e[N];
}

inline int last_error() { return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP; }

}  // namespace

int launch_decode_step(const StepArgs& a, hipStream_t st) {
  if (a.B < 0 || a.W <= 0 || a.Wmax <= 0 || a.C <= 0) return SSNT_ERR_INVALID_ARG;
  if (a.variant == Variant::V1 && a.C != 2) return SSNT_ERR_INVALID_ARG;
  if (a.variant == Variant::V2 && (!a.total || !a.table || !a.output_length || !a.next_total))
    return SSNT_ERR_INVALID_ARG;
  if (a.B == 0) return SSNT_OK;
  const size_t n = (size_t)a.W * a.C;
  const size_t lds = n * sizeof(Cand) + 2 * n * sizeof(int);
  if (lds > 150 * 1024) return SSNT_ERR_UNSUPPORTED;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_decode_step),
                      hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  hipLaunchKernelGGL(k_decode_step, dim3(a.B), dim3(64), lds, st, a);
  return last_error();
}

int launch_lattice_decode(const LatticeDecodeArgs& a, hipStream_t st) {
  if (a.B < 0 || a.W <= 0 || a.W > 64 || a.T <= 0 || a.U <= 0) return SSNT_ERR_INVALID_ARG;
  if (a.B == 0) return SSNT_OK;
  const size_t n = 2 * (size_t)a.W;
  const bool staged = 2 * (size_t)a.U <= 64 * (size_t)kRowRegs;
  const size_t lds = n * sizeof(Cand) + 2 * n * sizeof(int) + (size_t)a.W * (2 + 1 + 1 + 1) * 4 + a.W + 16 +
                     (staged ? (size_t)a.U * 2 * sizeof(float) : 0);
  if (2 * a.W <= 64) {  // one candidate per lane: the register-resident step
    const size_t lds_reg = (size_t)kOutChunk * a.W * 6 * sizeof(int) +
                           (staged ? (size_t)a.U * 2 * sizeof(float) : 16);
    if (staged) hipLaunchKernelGGL(k_lattice_decode_reg<true>, dim3(a.B), dim3(64), lds_reg, st, a);
    else hipLaunchKernelGGL(k_lattice_decode_reg<false>, dim3(a.B), dim3(64), lds_reg, st, a);
  } else if (staged) {
    hipLaunchKernelGGL(k_lattice_decode<true>, dim3(a.B), dim3(64), lds, st, a);
  } else {
    hipLaunchKernelGGL(k_lattice_decode<false>, dim3(a.B), dim3(64), lds, st, a);
  }
  int rc = last_error();
  if (rc != SSNT_OK) return rc;
  // alignment of the best final beam (slot 0), t history = next_t (util.rs:20-33)
  return launch_extract_best(a.B, a.W, a.T, nullptr, a.beam_branch, a.next_t, a.best_beam_branch,
                             a.best_t_history, a.status, st);
}

int launch_extract_best(int B, int W, int U, const int* best_final_branch, const int* beam_branch,
                        const int* t_history, int* best_beam_branch, int* best_t_history,
                        int* status, hipStream_t st) {
  if (B < 0 || W <= 0 || U < 0) return SSNT_ERR_INVALID_ARG;
  if (B == 0 || U == 0) return SSNT_OK;
  const int chunk = max(1, min(U, 8192 / W));
  const size_t lds = (size_t)chunk * W * 2 * sizeof(int);
  hipLaunchKernelGGL(k_backtrace, dim3(B), dim3(64), lds, st, B, W, U, 1, best_final_branch,
                     beam_branch, t_history, best_beam_branch, best_t_history, chunk, status);
  return last_error();
}

int launch_order_beam_branch(int B, int W, int T, const int* final_branch, const int* beam_branch,
                             int* ordered, int* status, hipStream_t st) {
  if (B < 0 || W <= 0 || T < 0) return SSNT_ERR_INVALID_ARG;
  if (W > 64) return SSNT_ERR_UNSUPPORTED;
  if (B == 0 || T == 0) return SSNT_OK;
  const int chunk = max(1, min(T, 8192 / W));
  const size_t lds = (size_t)chunk * W * 2 * sizeof(int);
  hipLaunchKernelGGL(k_backtrace, dim3(B), dim3(64), lds, st, B, W, T, W, final_branch,
                     beam_branch, nullptr, ordered, nullptr, chunk, status);
  return last_error();
}

int launch_upsample(int B, int W, int T, int max_u, const int* duration, const int* output_length,
                    int* out, int* status, hipStream_t st) {
  if (B < 0 || W <= 0 || T < 0 || max_u < 0) return SSNT_ERR_INVALID_ARG;
  if (B == 0) return SSNT_OK;
  const size_t lds = (size_t)(T + 1) * sizeof(int);
  if (lds > 150 * 1024) return SSNT_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(k_upsample, dim3(B * W), dim3(64), lds, st, B * W, T, max_u, duration,
                     output_length, out, status);
  return last_error();
}

int launch_levenshtein(int B, int max_length, const int* a, const int* b, const int* a_len,
                       const int* b_len, int* dist, hipStream_t st) {
  if (B < 0 || max_length < 0) return SSNT_ERR_INVALID_ARG;
  if (B == 0) return SSNT_OK;
  const size_t lds = (size_t)(max_length + 1) * 2 * sizeof(int);
  if (lds > 150 * 1024) return SSNT_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(k_levenshtein, dim3(B), dim3(64), lds, st, B, max_length, a, b, a_len,
                     b_len, dist);
  return last_error();
}

}  // namespace ssnt
