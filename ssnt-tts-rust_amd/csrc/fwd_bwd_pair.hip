// fwd_bwd_pair.hip -- pair lattice forward-backward for gfx950 (default for U <= 128 without
// log_obs).
//
// The lattice and the split-exponent arithmetic are those of the streaming kernel
// (fwd_bwd_stream.hip), with one change that halves the serial chain: the alpha and beta chains
// advance TWO rows per dependent step. For the row pair (s, s+1) with factors E, Sh (row s) and
// E', Sh' (row s+1) the two steps compose into
//   alpha[s+2][p] = c0 alpha[s][p] + c1 alpha[s][p-1] + c2 alpha[s][p-2]
//   beta[s][p]    = d0 beta[s+2][p] + d1 beta[s+2][p+1] + d2 beta[s+2][p+2]
// with c0 = d0 = E E', c1 = Sh[p-1] E'[p] (+) E[p-1] Sh'[p-1], c2 = Sh[p-2] Sh'[p-1],
// d1 = E Sh' (+) Sh E'[p+1], d2 = Sh Sh'[p+1]; the converter waves form these coefficients
// once per pair (off the chain). Even rows come off the chains; an odd row is one ordinary step
// from the even row before it (alpha) or after it (beta), recomputed by the gradient waves that
// need it. The cut M = ((S-1)>>1) & ~1 is even, so both chains produce it. oracle/ssnt_oracle.c
// (ORACLE_PAIR) restates exactly this; tests/test_oracle_fwd_bwd.py pins it to the f64 DP.
//
// Roles (16 waves, role_of in stream_dev.h): 1 alpha chain, 1 beta chain, 3 + 3 converters,
// 4 + 4 gradient waves. Per pair a converter loads two log_trans rows, exp()s them and writes one
// ring slot of seven blocks: c0 c1 c2 (the chain's) and E, X, E', X' (the gradient waves';
// X = the shift factor, pre-shifted by one position in the forward ring). Per pair a chain reads
// three blocks and writes one row, where the one-step chain read four blocks and wrote two rows:
// the chain's LDS operations, not its arithmetic, are what bounds a step.
//
// Rows kept for the gradients: even rows alpha[0..M] and beta[M+2..] (plus beta[S-1] when it is
// odd) in "storage" at index (s+1)>>1 (LDS, or the workspace when they do not fit), beta[M] in
// a cut buffer, and the chain rows past the cut in a 4-entry ring per direction.
//
// Gradient pair g of the forward direction covers rows (M+2g, M+2g+1); of the backward direction
// rows (M-2g-2, M-2g-1). A gradient wave rebuilds the odd rows it needs with one ordinary step
// (alpha from the even row before, beta from the even row after) and emits both rows.
#include <hip/hip_runtime.h>
#include <limits.h>

#include <type_traits>
#include <utility>

#include "lattice_dev.h"
#include "stream_dev.h"

namespace ssnt {
namespace {

// timing-experiment knobs (tools/build_fixed.sh builds only: one mask baked in; compiled out of
// the product): 0 gradient waves read and release but do no math, 1 converters skip exp() and
// the coefficients, 3 chains never poll converters, 11 chains never poll releases, 12 chains
// alone (other roles exit), 13 converters alone
#if defined(SSNT_EXP) && defined(SSNT_EXP_FIXED)
#define PEXP(bit) ((((SSNT_EXP_FIXED) >> (bit)) & 1) != 0)
#else
#define PEXP(bit) false
#endif

constexpr int kPairOut = 8;         // chain-row ring entries per direction (even rows past the cut)
constexpr int kPairConvDepth = 4;   // pairs in flight per converter (8 log_trans rows)
constexpr int kPairPF = 2;          // coefficient sets in flight per chain
enum PairBlk { kC0 = 0, kC1, kC2, kNBlk };  // ring slot blocks: the chain's coefficients

// ring slots (pairs) per direction: 16 (32 rows of slack) while the rings stay under ~64 KB
__host__ __device__ constexpr int pair_slots_for(int Up) { return Up <= 80 ? 16 : 8; }

// x[p - O] (FWD) or x[p + O] of this lane's K positions, O = 1 or 2: own positions, the
// neighbour lane's by one DPP, two lanes away (K = 1, O = 2) by two. Zero-filled at the wave
// edge (m = 0, e = 0): such a term always meets a canonical zero coefficient (e = XF_EZERO).
template <int K, bool FWD, int O>
__device__ __forceinline__ void nb(const XRow<K>& A, float* m, int* e) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int i = FWD ? j - O : j + O;
    if (i >= 0 && i < K) {
      m[j] = A.m[i];
      e[j] = A.e[i];
    } else if (FWD && i >= -K) {
      m[j] = shr_z(A.m[K + i]);
      e[j] = shr_z(A.e[K + i]);
    } else if (FWD) {
      m[j] = shr_z(shr_z(A.m[2 * K + i]));
      e[j] = shr_z(shr_z(A.e[2 * K + i]));
    } else if (i < 2 * K) {
      m[j] = shl_z(A.m[i - K]);
      e[j] = shl_z(A.e[i - K]);
    } else {
      m[j] = shl_z(shl_z(A.m[i - 2 * K]));
      e[j] = shl_z(shl_z(A.e[i - 2 * K]));
    }
  }
}

// the chain: x = t0 + t1 + t2 over the row two steps back (FWD: alpha) or ahead (beta).
// Lazy normalization as in the streaming kernel (stream_dev.h chain_add): unnormalized pairs
// (s, e_max) between NORM steps; every operation is exact under power-of-two rescaling and the
// mantissas stay within [2^-6, 2^6] over two pair steps (coefficient mantissas lie in [0.5, 2)).
template <int K, bool FWD, bool NORM>
__device__ __forceinline__ void pair_chain(XRow<K>& A, const XRow<K>& C0, const XRow<K>& C1,
                                           const XRow<K>& C2) {
  float m1[K], m2[K];
  int e1[K], e2[K];
  nb<K, FWD, 1>(A, m1, e1);
  nb<K, FWD, 2>(A, m2, e2);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const float t0 = A.m[j] * C0.m[j], t1 = m1[j] * C1.m[j], t2 = m2[j] * C2.m[j];
    const int f0 = A.e[j] + C0.e[j], f1 = e1[j] + C1.e[j], f2 = e2[j] + C2.e[j];
    const int em = max(max(f0, f1), max(f2, XF_EZERO));
    const float s = (xldexp(t0, f0 - em) + xldexp(t1, f1 - em)) + xldexp(t2, f2 - em);
    if constexpr (NORM) {
      A.m[j] = xmant(s);
      A.e[j] = em + xexpo(s);
    } else {
      A.m[j] = s;
      A.e[j] = em;
    }
  }
}

__device__ __forceinline__ void xmul(float am, int ae, float bm, int be, float& m, int& e) {
  m = am * bm;
  e = ae + be;
}

// the pair coefficients of one lane from the converted rows (X = L pre-shifted for FWD, Sh else)
template <int K, bool FWD>
__device__ __forceinline__ void pair_coefs(const XRow<K>& E0, const XRow<K>& X0, const XRow<K>& E1,
                                           const XRow<K>& X1, XRow<K>& C0, XRow<K>& C1, XRow<K>& C2) {
#pragma unroll
  for (int j = 0; j < K; ++j) xmul(E0.m[j], E0.e[j], E1.m[j], E1.e[j], C0.m[j], C0.e[j]);
  if constexpr (FWD) {
    // E[p-1], L[p-1]: canonical zero left of p = 0 (shr1 fills e with XF_EZERO)
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const float em1 = j ? E0.m[j - 1] : shr1(E0.m[K - 1]);
      const int ee1 = j ? E0.e[j - 1] : shr1(E0.e[K - 1]);
      const float lm1 = j ? X0.m[j - 1] : shr1(X0.m[K - 1]);
      const int le1 = j ? X0.e[j - 1] : shr1(X0.e[K - 1]);
      float am, bm;
      int ae, be;
      xmul(X0.m[j], X0.e[j], E1.m[j], E1.e[j], am, ae);  // Sh[p-1] E'[p]
      xmul(em1, ee1, X1.m[j], X1.e[j], bm, be);          // E[p-1] Sh'[p-1]
      const xf c1 = xf_add(am, ae, bm, be);
      C1.m[j] = c1.m;
      C1.e[j] = c1.e;
      xmul(lm1, le1, X1.m[j], X1.e[j], C2.m[j], C2.e[j]);  // Sh[p-2] Sh'[p-1]
    }
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const float ep1 = (j + 1 < K) ? E1.m[j + 1] : shl1(E1.m[0]);
      const int eep1 = (j + 1 < K) ? E1.e[j + 1] : shl1(E1.e[0]);
      const float sp1 = (j + 1 < K) ? X1.m[j + 1] : shl1(X1.m[0]);
      const int sep1 = (j + 1 < K) ? X1.e[j + 1] : shl1(X1.e[0]);
      float am, bm;
      int ae, be;
      xmul(E0.m[j], E0.e[j], X1.m[j], X1.e[j], am, ae);  // E[p] Sh'[p]
      xmul(X0.m[j], X0.e[j], ep1, eep1, bm, be);         // Sh[p] E'[p+1]
      const xf c1 = xf_add(am, ae, bm, be);
      C1.m[j] = c1.m;
      C1.e[j] = c1.e;
      xmul(X0.m[j], X0.e[j], sp1, sep1, C2.m[j], C2.e[j]);  // Sh[p] Sh'[p+1]
    }
  }
}

// Sh[p] = L[p+1] (undo the forward ring's pre-shift), exact zero for p >= P-1 (src/lib.rs:196-205)
template <int K>
__device__ __forceinline__ XRow<K> unshift(const XRow<K>& L, int p0, int P) {
  XRow<K> Sh;
#pragma unroll
  for (int q = 0; q < K; ++q) {
    const float lm = (q == K - 1) ? shl_z(L.m[0]) : L.m[q + 1 < K ? q + 1 : 0];
    const int le = (q == K - 1) ? shl_z(L.e[0]) : L.e[q + 1 < K ? q + 1 : 0];
    const bool live = p0 + q < P - 1;
    Sh.m[q] = live ? lm : 0.0f;
    Sh.e[q] = live ? le : XF_EZERO;
  }
  return Sh;
}
// L[p] = Sh[p-1] (the forward pre-shift), canonical zero at p = 0
template <int K>
__device__ __forceinline__ XRow<K> preshift(const XRow<K>& Sh) {
  XRow<K> L;
  L.m[0] = shr1(Sh.m[K - 1]);
  L.e[0] = shr1(Sh.e[K - 1]);
#pragma unroll
  for (int q = 1; q < K; ++q) {
    L.m[q] = Sh.m[q - 1];
    L.e[q] = Sh.e[q - 1];
  }
  return L;
}

template <int K, bool LDS, int kNC, int kNH, int R, bool NV>
__global__ __launch_bounds__(64 * (2 + 2 * kNC + 2 * kNH)) void k_fwd_bwd_pair(FwdBwdArgs a) {
  constexpr int kWaves = 2 + 2 * kNC + 2 * kNH;
  constexpr int kR2 = kPairOut;
  constexpr int PF = kPairPF;
  static_assert(R % PF == 0 && PF < R, "prefetch buffers tile the ring");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Role role = role_of<kNC, kNH>(wave);
  const int lane = threadIdx.x & 63;
  const int T = a.T, U = a.U;
  const int Up = NV ? K * ((U + K - 1) / K) : U;  // internal row stride: whole lane slices
  const int S = a.step_len[b];
  const int P = a.pos_len[b];
  const bool term = (a.flags & SSNT_FLAG_TERMINAL_EMIT) != 0;
  const size_t TU = (size_t)T * U;
  const float* lt = a.log_trans + (size_t)b * TU * 2;
  float* g = a.grad ? a.grad + (size_t)b * TU * 2 : nullptr;
  float* la = a.log_alpha ? a.log_alpha + (size_t)b * TU : nullptr;
  float* lb = a.log_beta ? a.log_beta + (size_t)b * TU : nullptr;
  const int p0 = K * lane;
  const bool act = p0 < U;
  const int pr = act ? p0 : Up - K;  // LDS read position (clamped for lanes past U)
  const int NS = (T >> 1) + 1;       // storage rows: index (s+1)>>1

  // ---- LDS: ctl | cut (64K xf) | junk (64 x 16K B) | rings [2][R][7 blocks][Up xf] |
  //      chain-row rings [2][kR2][Up xf] | storage [NS][Up xf] (LDS mode)
  Ctl* ctl = reinterpret_cast<Ctl*>(smem);
  xf* cutb = reinterpret_cast<xf*>(smem + kCtlBytes);
  unsigned char* junk = reinterpret_cast<unsigned char*>(cutb + 64 * K);
  xf* ring0 = reinterpret_cast<xf*>(junk + 64 * 16 * K);
  const int blk = Up;              // xf per block
  const int slot = kNBlk * Up;     // xf per slot
  xf* outr = ring0 + (size_t)2 * R * slot;
  xf* rows = LDS ? outr + 2 * kR2 * Up : reinterpret_cast<xf*>(a.workspace) + (size_t)b * NS * Up;
  xf* junk_lane = reinterpret_cast<xf*>(junk + 16 * K * lane);

  auto fill_rows = [&](int from, int w0, int wstep) {  // zero grads / -inf debug rows
    float z[2 * K], ninf[K];
#pragma unroll
    for (int j = 0; j < 2 * K; ++j) z[j] = 0.0f;
#pragma unroll
    for (int j = 0; j < K; ++j) ninf[j] = -__builtin_inff();
    for (int s = from + w0; s < T; s += wstep) {
      if (g) gst<K, 2, NV>(z, brsrc(g + (size_t)s * U * 2, U * 8u), p0);
      if (la) gst<K, 1, NV>(ninf, brsrc(la + (size_t)s * U, U * 4u), p0);
      if (lb) gst<K, 1, NV>(ninf, brsrc(lb + (size_t)s * U, U * 4u), p0);
    }
  };
  const float inf_loss = (a.flags & SSNT_FLAG_ZERO_INFINITY) ? 0.0f : __builtin_inff();
  const bool feasible = S >= 1 && P >= 1 && S <= T && P <= U && S >= P;
  if (!feasible) {
    if ((S > T || P > U || S < 0 || P < 0) && a.status && threadIdx.x == 0)
      atomicOr(a.status, kStatusBadLength);
    fill_rows(0, wave, kWaves);
    if (wave == 0) {
      const unsigned tag = a.loss_sum ? __builtin_amdgcn_readfirstlane(sum_tag(a)) : 0u;
      if (lane == 0) publish_loss(a, b, inf_loss, tag);
      if (a.loss_sum && b == 0) finish_loss_sum(a, tag);
    }
    return;
  }
  const int M = ((S - 1) >> 1) & ~1;  // the cut (even)
  const int qc = M >> 1;              // alpha pair steps before the cut
  const int kmax = (S - 1) >> 1;      // last lattice pair (rows 2 kmax, 2 kmax + 1)
  const int nstream = kmax + 1;       // converted pairs per direction
  const int nA = (S - 1) >> 1;        // alpha pair steps: alpha[2], ..., alpha[2 nA]
  // gradient pairs: forward (M+2g, M+2g+1) for g < ngf; backward (M-2g-2, M-2g-1) for g < qc;
  const int ngf = (S - M + 1) >> 1;

  auto row_st = [&](int idx, const XRow<K>& r) {  // storage row idx
    if constexpr (LDS) {
      lds_xrow_st<K>(act ? rows + (size_t)idx * Up + p0 : junk_lane, r);
    } else {
      float v[2 * K];
      xrow_pack<K>(r, v);
      buf_st<2 * K>(v, brsrc(rows + (size_t)idx * Up, Up * 8u), p0 * 8);
    }
  };
  auto row_ld = [&](int idx) {
    if constexpr (LDS) {
      return lds_xrow<K>(rows + (size_t)idx * Up + pr);
    } else {
      float v[2 * K];
      buf_ld<2 * K>(v, brsrc(rows + (size_t)idx * Up, Up * 8u), pr * 8);
      return xrow_unpack<K>(v);
    }
  };
  auto slot_of = [&](int d, int j) { return ring0 + (size_t)(d * R + j % R) * slot; };
  auto blk_ld = [&](const xf* sl, int k) { return lds_xrow<K>(sl + (size_t)k * blk + pr); };

  if (threadIdx.x < kCtlBytes / 4) reinterpret_cast<int*>(smem)[threadIdx.x] = 0;
  XRow<K> X = xrow_zero<K>();
  if (role.kind == 0 && role.d == 0) {  // alpha[0]: 1 at p = 0
    if (lane == 0) {
      X.m[0] = 0.5f;
      X.e[0] = 1;
    }
    row_st(0, X);
  }
  __syncthreads();
  Diag dg;
  if (PEXP(12) && role.kind != 0) return;
  if (PEXP(13) && role.kind != 1) return;

  if (role.kind == 2) {
    // =============================== gradient waves ======================================
    const int d = role.d;
    const int h = role.idx;
    const int npairs = d == 0 ? ngf : qc;
    // ---- Z at the cut: tree-sum over p of alpha[M][p] * beta[M][p] (fixed order, = oracle)
    if (d == 0 && h == 0) {
      const unsigned tag = a.loss_sum ? sum_tag(a) : 0u;
      spin_until<true>([&] { return ctr_acq(&ctl->a_ready); }, 1, a.status, dg);
      spin_until<true>([&] { return ctr_acq(&ctl->bm_ready); }, 1, a.status, dg);
      const XRow<K> Am = row_ld(qc);
      const XRow<K> Bm = lds_xrow<K>(cutb + pr);
      float wm[K];
      int we[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        wm[j] = act ? Am.m[j] * Bm.m[j] : 0.0f;
        we[j] = act ? Am.e[j] + Bm.e[j] : XF_EZERO;
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
      if (lane == 0) {
        ctl->z = z;
        publish_loss(a, b, (z.m == 0.0f) ? inf_loss : 0.0f - xf_log(z), tag);
      }
      ctr_rel(&ctl->z_ready, 1);
    } else {
      spin_until<true>([&] { return ctr_acq(&ctl->z_ready); }, 1, a.status, dg);
    }
    dg.mark_cut();
    const xf Z = ctl->z;
    const bool zero_z = (Z.m == 0.0f);
    const float izm = 1.0f / Z.m;
    const int ize = -Z.e;
    const XRow<K> ONE = [] {
      XRow<K> o;
#pragma unroll
      for (int q = 0; q < K; ++q) {
        o.m[q] = 1.0f;
        o.e[q] = 0;
      }
      return o;
    }();

    // one gradient row: A = alpha[s], E / Sh = factors of row s, Q = beta[s+1] (or the terminal)
    auto emit = [&](int s, const XRow<K>& A, const XRow<K>& E, const XRow<K>& Sh,
                    const XRow<K>& Bn, const XRow<K>& Bs) {
      float ge[2 * K];
      if (zero_z) {
#pragma unroll
        for (int q = 0; q < 2 * K; ++q) ge[q] = 0.0f;
      } else {
        XRow<K> Q, Rr;
        if (s + 1 < S) {
          Q = Bn;
#pragma unroll
          for (int q = 0; q < K; ++q) {
            Rr.m[q] = (q == K - 1) ? shl_z(Q.m[0]) : Q.m[q + 1 < K ? q + 1 : 0];
            Rr.e[q] = (q == K - 1) ? shl_z(Q.e[0]) : Q.e[q + 1 < K ? q + 1 : 0];
          }
        } else {  // terminal transition: only the terminal emit at P-1 (src/lib.rs:187-195)
#pragma unroll
          for (int q = 0; q < K; ++q) {
            const bool lastp = term && (p0 + q) == P - 1;
            Q.m[q] = lastp ? 1.0f : 0.0f;
            Q.e[q] = lastp ? 0 : XF_EZERO;
            Rr.m[q] = 0.0f;
            Rr.e[q] = XF_EZERO;
          }
        }
#pragma unroll
        for (int q = 0; q < K; ++q) {
          const int ae = A.e[q] + ize;  // (integer exponent sums are exact in any order)
          ge[2 * q] = xf_neg_post(((A.m[q] * E.m[q]) * Q.m[q]) * izm, ae + E.e[q] + Q.e[q]);
          ge[2 * q + 1] = xf_neg_post(((A.m[q] * Sh.m[q]) * Rr.m[q]) * izm, ae + Sh.e[q] + Rr.e[q]);
        }
      }
      if (g) gst<K, 2, NV>(ge, brsrc(g + (size_t)s * U * 2, U * 8u), p0);
      if (la || lb) {  // debug outputs (slow path)
        float va[K], vb[K];
#pragma unroll
        for (int q = 0; q < K; ++q) {
          va[q] = zero_z ? -__builtin_inff() : xf_log(xf_norm(A.m[q], A.e[q]));  // (lazy rows)
          vb[q] = zero_z ? -__builtin_inff() : xf_log(xf_norm(Bs.m[q], Bs.e[q]));
        }
        if (la) gst<K, 1, NV>(va, brsrc(la + (size_t)s * U, U * 4u), p0);
        if (lb) gst<K, 1, NV>(vb, brsrc(lb + (size_t)s * U, U * 4u), p0);
      }
    };

    int chain_seen = 0;
    auto wait_chain = [&](int need) {
      if (chain_seen < need)
        chain_seen = spin_until<true>([&] { return ctr_ld(&ctl->chain[d]); }, need, a.status, dg);
      cbar();
    };
    const bool dbg = la || lb;
    // The factors of the pair come from log_trans itself (loaded one pair ahead, converted here
    // with the converters' own exp): the ring carries only the chain's three coefficient blocks,
    // since LDS stores, not loads, bound the converters.
    const int nmine = (npairs - h + kNH - 1) / kNH;
    auto gload = [&](int i, Item<K, false>& r0, Item<K, false>& r1) {
      const int gp = h + kNH * i;
      const int k = d == 0 ? qc + gp : qc - 1 - gp;
      const int row0 = min(max(2 * k, 0), T - 1), row1 = min(max(2 * k + 1, 0), T - 1);
      gld<K, 2, NV>(r0.lt, brsrc(lt + (size_t)row0 * U * 2, U * 8u), p0);
      gld<K, 2, NV>(r1.lt, brsrc(lt + (size_t)row1 * U * 2, U * 8u), p0);
    };
    auto body = [&](int i, const Item<K, false>& r0, const Item<K, false>& r1) {
      const int gp = h + kNH * i;
      if (d == 0) {
        const int k = qc + gp;  // lattice pair (2k, 2k+1)
        const int s0 = 2 * k, s1 = s0 + 1;
        if (gp > 0) wait_chain(qc + gp);  // alpha[s0] written by pair step qc + gp - 1
        const XRow<K> A0 = (gp == 0) ? row_ld(qc) : lds_xrow<K>(outr + (size_t)(gp % kR2) * Up + pr);
        // beta[s1]: beta[S-1] itself when s1 = S-1 (odd, stored), else one step down from the
        // stored beta[2k+2]; beta[s0] only for the debug rows
        XRow<K> Bt, Bs0;
        if (s1 < S) Bt = row_ld((s1 == S - 1) ? (S >> 1) : k + 1);
        if (dbg) Bs0 = (s0 == M) ? lds_xrow<K>(cutb + pr) : row_ld(k);
        cbar();
        ctr_st(&ctl->help[0][h], i + 1);  // ring row read (in-order DS): reusable
        if (PEXP(0)) return;
        XRow<K> E0, Sh0, E1, Sh1;
        convert<K, false>(r0, P, lane, E0, Sh0);
        if (s1 < S) {
          convert<K, false>(r1, P, lane, E1, Sh1);
          XRow<K> B1 = Bt, B2 = Bt;
          if (s1 + 1 < S) beta_chain<K, false, true>(B1, E1, Sh1, ONE);  // beta[s1] from beta[2k+2]
          emit(s0, A0, E0, Sh0, B1, Bs0);
          XRow<K> A1 = A0;  // alpha[s1] = one step from alpha[s0]
          alpha_chain<K, false, true>(A1, E0, preshift<K>(Sh0), ONE);
          emit(s1, A1, E1, Sh1, B2, B1);  // (s1 = S-1: the terminal row; B2 unused)
        } else {
          emit(s0, A0, E0, Sh0, Bt, Bs0);  // s0 = S-1: the terminal row
        }
      } else {
        const int k = qc - 1 - gp;  // lattice pair (2k, 2k+1); beta stream entry kmax - k
        const int s0 = 2 * k, s1 = s0 + 1;
        const int j = kmax - k;
        if (gp > 0) wait_chain(j);  // beta[2k+2]: stream entry j - 1 done
        if (dbg) wait_chain(j + 1); // beta[2k]: stream entry j
        const XRow<K> B2 = (gp == 0) ? lds_xrow<K>(cutb + pr) : lds_xrow<K>(outr + (size_t)(kR2 + gp % kR2) * Up + pr);
        const XRow<K> A0 = row_ld(k);
        XRow<K> Bs0;
        if (dbg) Bs0 = lds_xrow<K>(outr + (size_t)(kR2 + (gp + 1) % kR2) * Up + pr);
        cbar();
        ctr_st(&ctl->help[1][h], i + 1);
        if (PEXP(0)) return;
        XRow<K> E0, Sh0, E1, Sh1;
        convert<K, false>(r0, P, lane, E0, Sh0);
        convert<K, false>(r1, P, lane, E1, Sh1);
        XRow<K> B1 = B2;  // beta[s1] = one step down from beta[2k+2]
        beta_chain<K, false, true>(B1, E1, Sh1, ONE);
        XRow<K> A1 = A0;  // alpha[s1] = one step from alpha[2k]
        alpha_chain<K, false, true>(A1, E0, preshift<K>(Sh0), ONE);
        emit(s0, A0, E0, Sh0, B1, Bs0);
        emit(s1, A1, E1, Sh1, B2, B1);
      }
    };
    Item<K, false> a0, a1, b0, b1;  // alternating buffers: pair i+1 loads while pair i computes
    if (nmine > 0) gload(0, a0, a1);
    for (int i = 0; i < nmine; i += 2) {
      if (i + 1 < nmine) gload(i + 1, b0, b1);
      body(i, a0, a1);
      if (i + 1 < nmine) {
        if (i + 2 < nmine) gload(i + 2, a0, a1);
        body(i + 1, b0, b1);
      }
    }
    dg.flush(b, role.slot);
    return;
  }

  if (role.kind == 1) {
    // =============================== converters ==========================================
    const int d = role.d;
    const int c = role.idx;
    constexpr int D = kPairConvDepth;
    const unsigned tag0 = (d == 0 && c == 0 && b == 0 && a.loss_sum) ? sum_tag(a) : 0u;
    const int chain_end = d == 0 ? nA : nstream;  // stream entries the chain reads
    // stream entry j -> lattice pair k: forward j, backward kmax - j
    auto load = [&](int j, Item<K, false>& r0, Item<K, false>& r1) {
      if (PEXP(15)) {  // (experiment 15: no loads)
#pragma unroll
        for (int q = 0; q < 2 * K; ++q) {
          r0.lt[q] = -0.5f - 0.01f * j;
          r1.lt[q] = -0.7f - 0.01f * j;
        }
        return;
      }
      const int k = d == 0 ? j : kmax - j;
      const int row0 = min(max(2 * k, 0), T - 1), row1 = min(max(2 * k + 1, 0), T - 1);
      gld<K, 2, NV>(r0.lt, brsrc(lt + (size_t)row0 * U * 2, U * 8u), p0);
      gld<K, 2, NV>(r1.lt, brsrc(lt + (size_t)row1 * U * 2, U * 8u), p0);
    };
    Item<K, false> pf0[D], pf1[D];
#pragma unroll
    for (int i = 0; i < D; ++i) load(c + kNC * i, pf0[i], pf1[i]);
    int seen_chain = 0;
    const int nmine = (nstream - c + kNC - 1) / kNC;  // my stream entries: c, c + kNC, ...
    // Two entries per group, their math interleaved (a converter's instruction stream is
    // latency-bound at ~5 cycles per dependent VALU; two independent streams fill the gaps), one
    // loop per direction so the group is branch-free.
    static_assert(D % 2 == 0, "entries are converted two at a time");
    auto conv_loop = [&](auto Fwd) {
      constexpr bool FWD = decltype(Fwd)::value;
      auto math = [&](int n, const Item<K, false>& r0, const Item<K, false>& r1, XRow<K>* o) {
        // o: C0 C1 C2 E0 E1 X0
        const int j = c + kNC * n;
        const int k = FWD ? j : kmax - j;
        const int P1 = (2 * k + 1 < S) ? P : 0;  // row 2k+1 beyond S: all factors zero
        XRow<K> S0, S1;
        if (PEXP(1)) {
#pragma unroll
          for (int q = 0; q < K; ++q) {
            o[3].m[q] = r0.lt[2 * q]; o[3].e[q] = 0; o[5].m[q] = r0.lt[2 * q + 1]; o[5].e[q] = -1;
            o[4].m[q] = r1.lt[2 * q]; o[4].e[q] = 0;
          }
          o[0] = o[3]; o[1] = o[5]; o[2] = o[4];
          return;
        }
        convert<K, false>(r0, P, lane, o[3], S0);
        convert<K, false>(r1, P1, lane, o[4], S1);
        o[5] = FWD ? preshift<K>(S0) : S0;
        const XRow<K> X1 = FWD ? preshift<K>(S1) : S1;
        pair_coefs<K, FWD>(o[3], o[5], o[4], X1, o[0], o[1], o[2]);
      };
      auto put_entry = [&](int n, const XRow<K>* o) {
        const int j = c + kNC * n;
        xf* sl = slot_of(d, j);
        auto put = [&](int k2, const XRow<K>& r) {
          if (!PEXP(14)) lds_xrow_st<K>(act ? sl + (size_t)k2 * blk + p0 : junk_lane, r);  // (14: no ring writes)
        };
        if (!FWD && j == 0) {
          // the backward chain's first entry: E of row S-1 (terminal emit) and, S-1 odd, the
          // factors of row S-2 for its one ordinary step (this pair's coefficients are unused)
          const bool odd = ((S - 1) & 1) != 0;
          put(kC0, odd ? o[4] : o[3]);
          put(kC1, o[3]);
          put(kC2, o[5]);
        } else {
          put(kC0, o[0]);
          put(kC1, o[1]);
          put(kC2, o[2]);
        }
      };
      for (int base = 0; base < nmine; base += D) {
#pragma unroll
        for (int i = 0; i < D; i += 2) {
          const int n0 = base + i, n1 = n0 + 1;
          if (n0 < nmine) {
            XRow<K> o0[6], o1[6];
            math(n0, pf0[i], pf1[i], o0);
            math(n1, pf0[i + 1], pf1[i + 1], o1);  // (past the end: garbage, never stored)
            // slots of entries n0, n1 last held entries j - R: the chain must have read them
            const int q = c + kNC * min(n1, nmine - 1) - R;
            if (q >= 0 && !PEXP(13)) {
              const int need_c = min(q + 1, chain_end);
              if (seen_chain < need_c)
                seen_chain = spin_until<true>([&] { return ctr_ld(&ctl->sread[d]); }, need_c, a.status, dg);
            }
            cbar();
            put_entry(n0, o0);
            if (n1 < nmine) put_entry(n1, o1);
            cbar();
            ctr_st(&ctl->conv[d][c], min(n1, nmine - 1) + 1);
          }
          // refill after the old items are consumed (same registers, no copy)
          load(c + kNC * (n0 + D), pf0[i], pf1[i]);
          load(c + kNC * (n1 + D), pf0[i + 1], pf1[i + 1]);
        }
      }
    };
    if (d == 0) conv_loop(std::true_type{});
    else conv_loop(std::false_type{});
    dg.flush(b, role.slot);
    fill_rows(S, d * kNC + c, 2 * kNC);  // zero the rows beyond S
    if (d == 0 && c == 0 && b == 0 && a.loss_sum) finish_loss_sum(a, tag0);
    return;
  }

  // ================================== chains =============================================
  // Unrolled blocks of R pair steps aligned to R (slot offsets compile-time), sub-blocks of H
  // steps between waits (converted slots, released ring rows) and progress publication.
  __builtin_amdgcn_s_setprio(3);
  const int d = role.d;
  int ready = 0;  // stream entries known converted
  auto wait_entry = [&](int j) {
    if (PEXP(3)) return;
    if (j >= ready)
      ready = spin_until<false>([&] { return first_missing<kNC>(ctl->conv[d], 0); }, j + 1, a.status, dg);
  };
  const xf* cptr[R];  // slot j, this lane's c0 (c1, c2 follow at + blk, + 2 blk)
#pragma unroll
  for (int j = 0; j < R; ++j) cptr[j] = ring0 + (size_t)(d * R + j) * slot + pr;
  xf* optr[kR2];  // chain-row ring entry e, this lane (junk past U)
#pragma unroll
  for (int j = 0; j < kR2; ++j) optr[j] = act ? outr + (size_t)(d * kR2 + j) * Up + p0 : junk_lane;
  XRow<K> C0b[PF], C1b[PF], C2b[PF];
  auto rd = [&](int j, int par) {
    C0b[par] = lds_xrow<K>(cptr[j]);
    C1b[par] = lds_xrow<K>(cptr[j] + blk);
    C2b[par] = lds_xrow<K>(cptr[j] + 2 * blk);
  };
  constexpr int H1 = 4;  // sub-block before the cut
  constexpr int H2 = 2;  // past the cut (chain-ring rows released right behind)
  // steps [lo, hi) of stream entries, blocks of R aligned to R
  auto run = [&](auto Hc, int lo, int hi, auto&& step, auto&& hwait) {
    constexpr int HS = decltype(Hc)::value;
    static_assert(R % HS == 0, "sub-blocks tile the ring");
    for (int base = lo & ~(R - 1); base < hi; base += R) {
      sfor<R / HS>([&](auto Q) {
        constexpr int h0 = decltype(Q)::value * HS;
        const int hb0 = base + h0;
        if (hb0 + HS <= lo || hb0 >= hi) return;
        hwait(max(hb0, lo), min(hb0 + HS, hi));
        if (hb0 >= lo && hb0 + HS <= hi) {
          sfor<HS>([&](auto J) { step(std::integral_constant<int, h0 + decltype(J)::value>{}, base, true); });
        } else {
          sfor<HS>([&](auto J) {
            constexpr int jj = decltype(J)::value;
            step(std::integral_constant<int, h0 + jj>{}, base, hb0 + jj >= lo && hb0 + jj < hi);
          });
        }
        cbar();
        ctr_st(&ctl->chain[d], min(hb0 + HS, hi));
        ctr_st(&ctl->sread[d], min(hb0 + HS, hi) + PF);  // slot reads run PF entries ahead
      });
    }
  };
  using HA = std::integral_constant<int, H1>;
  using HB = std::integral_constant<int, H2>;
  if (d == 0) {
    // ---------------- alpha chain: stream entry q = pair step alpha[2q] -> alpha[2q+2] ---------
    const int last = max(nA - 1, 0);
    if (nA > 0) {
      wait_entry(min(PF - 1, last));
      cbar();
      sfor<PF>([&](auto J) { rd(decltype(J)::value, decltype(J)::value); });
    }
    int help_seen = 0;  // forward gradient pairs known done
    xf* wp = act ? rows + (size_t)Up + p0 : junk_lane;  // storage row 1 = alpha[2] (LDS mode)
    const int wstep = act ? Up : 0;
    auto hwait = [&](int r0, int r1, bool phase2) {
      (void)r0;
      wait_entry(min(r1 - 1 + PF, last));
      if (phase2) {  // ring entries for steps up to r1-1: g = step + 1 - qc; previous occupant g - kR2
        const int gq = r1 - qc - kR2;
        if (gq >= 1 && help_seen <= gq && !PEXP(11))
          help_seen = spin_until<false>([&] { return first_missing<kNH>(ctl->help[0], 0); }, gq + 1, a.status, dg);
      }
      cbar();
    };
    auto step = [&](auto Ic, int base, bool live, auto Ph) {
      constexpr int i = decltype(Ic)::value;
      constexpr int par = i % PF;
      constexpr bool phase2 = decltype(Ph)::value;
      if (!live) return;
      const int q = base + i;
      pair_chain<K, true, (i % 2) == 1>(X, C0b[par], C1b[par], C2b[par]);
      if constexpr (!phase2) {
        if constexpr (LDS) {
          lds_xrow_st<K>(wp, X);
          wp += wstep;
        } else {
          row_st(q + 1, X);
        }
      } else {
        lds_xrow_st<K>(optr[(q + 1 - qc) % kR2], X);
      }
      rd((i + PF) % R, par);  // entry q+PF (a stale slot past the end is dropped)
    };
    if (qc == 0) ctr_rel(&ctl->a_ready, 1);
    ctr_st(&ctl->sread[0], PF);
    run(HA{}, 0, qc, [&](auto Ic, int base, bool live) { step(Ic, base, live, std::false_type{}); },
        [&](int r0, int r1) { hwait(r0, r1, false); });
    if (qc > 0) {
      cbar();
      ctr_rel(&ctl->a_ready, 1);
      dg.mark_cut();
    }
    run(HB{}, qc, nA, [&](auto Ic, int base, bool live) { step(Ic, base, live, std::true_type{}); },
        [&](int r0, int r1) { hwait(r0, r1, true); });
  } else {
    // ---------------- beta chain: stream entry j = lattice pair kmax - j -------------------
    // entry 0: beta[S-1] (terminal) and, S-1 odd, one step to beta[S-2]; entries j >= 1:
    // beta[2k] from beta[2k+2], k = kmax - j. Rows > M: storage (s+1)>>1; M: cut buffer;
    // < M: chain-row ring entry qc - k.
    const int jcut = kmax - qc;  // entry that produces beta[M]
    auto put_row = [&](int s, const XRow<K>& r) {
      if (s > M) {
        row_st((s + 1) >> 1, r);
      } else if (s == M) {
        lds_xrow_st<K>(act ? cutb + p0 : junk_lane, r);
        cbar();
        ctr_rel(&ctl->bm_ready, 1);
        dg.mark_cut();
      } else {
        lds_xrow_st<K>(optr[(qc - (s >> 1)) % kR2], r);
      }
    };
    wait_entry(min(PF, nstream - 1));
    cbar();
    {
      const xf* sl = ring0 + (size_t)R * slot;  // backward slot 0
      const XRow<K> Et = blk_ld(sl, kC0);  // E of row S-1 (converter entry 0)
#pragma unroll
      for (int j = 0; j < K; ++j) {  // beta[S-1]: terminal emit (src/lib.rs:187-195)
        const bool lastp = (p0 + j) == P - 1;
        const xf v = term ? xf_norm(Et.m[j], Et.e[j]) : xf{0.5f, 1};
        X.m[j] = lastp ? v.m : 0.0f;
        X.e[j] = lastp ? v.e : XF_EZERO;
      }
      put_row(S - 1, X);
      if ((S - 1) & 1) {  // beta[S-2] = one step down with the factors of row S-2
        const XRow<K> E0 = blk_ld(sl, kC1), Sh0 = blk_ld(sl, kC2);  // row S-2
        cbar();
        beta_chain<K, false, true>(X, E0, Sh0, X);
        put_row(S - 2, X);
      }
    }
    cbar();
    sfor<PF>([&](auto J) { rd(1 + decltype(J)::value, (1 + decltype(J)::value) % PF); });
    int help_seen = 0;  // backward gradient pairs known done
    xf* wp = act ? rows + (size_t)(kmax - 1) * Up + p0 : junk_lane;  // storage index of beta[2 kmax - 2]
    const int wstep = act ? Up : 0;
    auto hwait = [&](int r0, int r1, bool ring) {
      (void)r0;
      wait_entry(min(r1 - 1 + PF, nstream - 1));
      if (ring) {  // entries up to r1-1 write ring entries g = j - jcut; previous occupant g - kR2
        const int gq = r1 - 1 - jcut - kR2;
        if (gq >= 1 && help_seen <= gq && !PEXP(11))
          help_seen = spin_until<false>([&] { return first_missing<kNH>(ctl->help[1], 0); }, gq + 1, a.status, dg);
      }
      cbar();
    };
    // kind 0: storage (rows > M), 1: the cut row, 2: ring rows (< M)
    auto step = [&](auto Ic, int base, bool live, auto Kd) {
      constexpr int i = decltype(Ic)::value;
      constexpr int par = i % PF;
      constexpr int kind = decltype(Kd)::value;
      if (!live) return;
      const int j = base + i;
      pair_chain<K, false, (i % 2) == 1>(X, C0b[par], C1b[par], C2b[par]);
      if constexpr (kind == 0) {
        if constexpr (LDS) {
          lds_xrow_st<K>(wp, X);
        } else {
          row_st(kmax - j, X);
        }
        wp -= wstep;
      } else if constexpr (kind == 1) {
        lds_xrow_st<K>(act ? cutb + p0 : junk_lane, X);
        cbar();
        ctr_rel(&ctl->bm_ready, 1);
        dg.mark_cut();
      } else {
        lds_xrow_st<K>(optr[(j - jcut) % kR2], X);
      }
      rd((i + PF) % R, par);
    };
    cbar();
    ctr_st(&ctl->chain[1], 1);  // entry 0 (beta[S-1], beta[S-2]) done
    ctr_st(&ctl->sread[1], PF + 1);
    run(HA{}, 1, jcut, [&](auto Ic, int base, bool live) { step(Ic, base, live, std::integral_constant<int, 0>{}); },
        [&](int r0, int r1) { hwait(r0, r1, false); });
    if (jcut >= 1)
      run(HA{}, jcut, jcut + 1, [&](auto Ic, int base, bool live) { step(Ic, base, live, std::integral_constant<int, 1>{}); },
          [&](int r0, int r1) { hwait(r0, r1, false); });
    run(HB{}, jcut + 1, nstream, [&](auto Ic, int base, bool live) { step(Ic, base, live, std::integral_constant<int, 2>{}); },
        [&](int r0, int r1) { hwait(r0, r1, true); });
  }
  dg.flush(b, role.slot);
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
inline bool aligned_to(const void* p, uintptr_t m) { return (reinterpret_cast<uintptr_t>(p) & (m - 1)) == 0; }

template <int K, bool LDS, int NC, int NH, int R, bool NV>
int launch_pair_kernel(const FwdBwdArgs& a, size_t lds, hipStream_t st) {
  auto kern = k_fwd_bwd_pair<K, LDS, NC, NH, R, NV>;
  note_fwd_bwd_dispatch("k_fwd_bwd_pair<K=%d,LDS=%d,NC=%d,NH=%d,R=%d,NV=%d>", K, (int)LDS, NC, NH, R, (int)NV);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBudget);
  hipLaunchKernelGGL(kern, dim3(a.B), dim3(64 * (2 + 2 * NC + 2 * NH)), lds, st, a);
  return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
}

template <int K, int R>
int launch_pair_k(const FwdBwdArgs& a, hipStream_t st) {
  const bool vec = (a.U % K == 0) && aligned16(a.log_trans) && aligned16(a.grad) &&
                   aligned16(a.log_alpha) && aligned16(a.log_beta) && aligned16(a.workspace);
  const bool narrow_ok = aligned_to(a.log_trans, 4) && aligned_to(a.grad, 4) && aligned16(a.workspace) &&
                         aligned_to(a.log_alpha, 4) && aligned_to(a.log_beta, 4);
  if (!vec && !narrow_ok) return SSNT_ERR_UNSUPPORTED;
  const int Up = K * ((a.U + K - 1) / K);
  const size_t head = pair_head_bytes(K, a.U);
  if (head > kLdsBudget) return SSNT_ERR_UNSUPPORTED;
  const size_t rows = (size_t)((a.T >> 1) + 1) * Up * sizeof(xf);
  const bool lds = head + rows <= kLdsBudget;
  if (!lds && (a.workspace == nullptr || a.workspace_bytes < (size_t)a.B * rows))
    return SSNT_ERR_WORKSPACE;
  if (vec)
    return lds ? launch_pair_kernel<K, true, 3, 4, R, false>(a, head + rows, st)
               : launch_pair_kernel<K, false, 3, 4, R, false>(a, head, st);
  return lds ? launch_pair_kernel<K, true, 3, 4, R, true>(a, head + rows, st)
             : launch_pair_kernel<K, false, 3, 4, R, true>(a, head, st);
}

}  // namespace

size_t pair_head_bytes(int K, int U) {
  const size_t Up = (size_t)K * ((U + K - 1) / K);
  const size_t R = pair_slots_for((int)Up);
  return kCtlBytes + (size_t)64 * K * sizeof(xf) + (size_t)64 * 16 * K +
         2 * R * kNBlk * Up * sizeof(xf) + 2 * (size_t)kPairOut * Up * sizeof(xf);
}
size_t pair_storage_bytes(int K, int T, int U) {
  const size_t Up = (size_t)K * ((U + K - 1) / K);
  return (size_t)((T >> 1) + 1) * Up * sizeof(xf);
}

int launch_fwd_bwd_pair(const FwdBwdArgs& a, hipStream_t st) {
  if (a.log_obs || a.grad_obs || a.U > 128) return SSNT_ERR_UNSUPPORTED;
  if (a.U <= 64) return launch_pair_k<1, pair_slots_for(64)>(a, st);
  return pair_slots_for(2 * ((a.U + 1) / 2)) == 16 ? launch_pair_k<2, 16>(a, st) : launch_pair_k<2, 8>(a, st);
}

}  // namespace ssnt
