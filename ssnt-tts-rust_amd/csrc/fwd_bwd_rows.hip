// fwd_bwd_rows.hip -- an A/B lattice forward-backward for U <= 128 without log_obs (gfx950;
// `make lib-ab` variants 13 / 14 only: bit-exact, measured slower than the streaming kernel,
// DESIGN.md 5.1c): batch-fed chains, half the lattice rows kept, the other half rebuilt on demand.
//
// Same lattice and the same split-exponent arithmetic as every fwd-bwd kernel,
// bit-exact with oracle/ssnt_oracle.c. One workgroup = one utterance, 16 waves in the roles of
// the streaming kernel (fwd_bwd_stream.hip): an alpha and a beta chain, 3 + 3 converters (log_trans
// rows -> split-exponent factors in an LDS ring per direction), 4 + 4 gradient waves behind the
// chains once Z is known. What changes (each change from a measurement):
//
//  * A chain reads the factors of NB rows at once, one batch ahead, into registers, and polls
//    the converters / publishes its progress once per batch. A chain step then costs ~150
//    cycles beside 15 busy waves (tools/micro/micro_batch.hip) against ~500 in the streaming
//    kernel, whose chain polled and published every 2-4 steps and waited on each slot read.
//  * Only EVEN lattice rows are kept: alpha[s] for even s < M and beta[s] for even s > M, plus
//    alpha[M] / beta[M] in cut buffers. The gradient waves take transition rows in pairs
//    (2j, 2j+1): the pair's odd row rebuilds its missing alpha (backward pairs) or beta (forward
//    pairs) with one chain step from the even row beside it and the factors of the pair's other
//    row, which the pair reads anyway -- the chain's own operations on the chain's own operands,
//    so the same bits. That halves the stored rows (64 KB instead of 128 KB at configs[1]), and
//    the factor rings grow from 8 to 16-24 slots, so the converters run ahead of the chains and
//    the gradient waves hold slots without starving them.
//  * The chains store every second row before the cut.
//
// Synchronisation is LDS counters as in the streaming kernel (a wave's DS instructions execute
// in order: "write, then counter" publishes, "read, then counter" releases; every spin bounded).
// Slot and ring-row reuse: a converter overwrites the slot of stream row q only after the chain
// has read it and, for rows whose gradient this direction emits, after the gradient pair that
// reads it is done; a chain overwrites a chain-ring row only after the pairs that read the
// previous occupant are done (no cycle: DESIGN.md 5.1b).
#include <hip/hip_runtime.h>
#include <limits.h>

#include <type_traits>
#include <utility>

#include "lattice_dev.h"
#include "stream_dev.h"

namespace ssnt {
namespace {

constexpr int kRowsNC = 3, kRowsNH = 4;         // converters / gradient waves per direction
constexpr int kRowsWaves = 2 + 2 * kRowsNC + 2 * kRowsNH;  // 16
constexpr int kRowsR2 = 8;                     // chain-row ring rows per direction
constexpr int kRowsConvDepth = 8;              // converter prefetch (rows of log_trans in flight)
// rows per dense-converter chunk (DC). A converter overwrites a chunk's slots only when the
// chain has read the chunk R rows before it and the gradient pairs of those rows are done; the
// chain asks for rows 2 NB ahead of what it has written, so a chunk must fit in R - 2 NB + 1 rows
// or the converter would wait on alpha / beta rows the chain cannot produce yet (a deadlock).
template <int R, int NB>
constexpr int rows_chunk() { return R - 2 * NB + 1 >= 8 ? 8 : 4; }

// LDS: ctl | cutA, cutB (64K xf each) | junk (64 x 16K B) | factor rings |
//      chain-row rings [2][kR2][U xf] | kept rows [(T+1)/2][U xf] (lattice row s at s >> 1)
// Factor rings slot-minor: entry (direction d, element block q, lane l, slot j) -- the 16-byte
// (E.m, E.e, X.m, X.e) of position K*l + q -- at ((d*K + q) * (U/K) + l) * (R+1) * 16 + 16*j, so a
// slot is a compile-time offset from one per-lane base (the chains' batched reads), and the odd
// lane stride of R+1 entries keeps a wave's 16-byte accesses on distinct banks.
size_t rows_lds_bytes(int K, int T, int U, int R) {
  return kCtlBytes + 2 * (size_t)64 * K * sizeof(xf) + (size_t)64 * 16 * K +
         2 * (size_t)(R + 1) * U * 16 + 2 * (size_t)kRowsR2 * U * sizeof(xf) +
         (size_t)((T + 1) / 2) * U * sizeof(xf);
}

// Sh[p] = L[p+1] (undo the forward ring's pre-shift), masked (exact zero) for p >= P-1
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

// alpha[s+1] from alpha[s] with UNSHIFTED shift factors (the backward ring): the shift product
// is formed in the lane of p-1 and moved, the same f32 product alpha_chain forms in the lane of
// p from the pre-shifted factor; lane 0 receives the canonical zero (0, XF_EZERO) as there.
template <int K>
__device__ __forceinline__ void alpha_step_sh(XRow<K>& A, const XRow<K>& E, const XRow<K>& Sh) {
  float hm[K];
  int he[K];
  hm[0] = shr1(A.m[K - 1] * Sh.m[K - 1]);
  he[0] = shr1(A.e[K - 1] + Sh.e[K - 1]);
#pragma unroll
  for (int j = 1; j < K; ++j) {
    hm[j] = A.m[j - 1] * Sh.m[j - 1];
    he[j] = A.e[j - 1] + Sh.e[j - 1];
  }
#pragma unroll
  for (int j = 0; j < K; ++j)
    chain_add<true>(A.m[j] * E.m[j], A.e[j] + E.e[j], hm[j], he[j], 0.0f, 0, false, A.m[j], A.e[j]);
}

// beta[S-1]: the terminal emit at P-1 (src/lib.rs:187-195), as the beta chain starts
template <int K>
__device__ __forceinline__ XRow<K> terminal_row(const XRow<K>& E, int p0, int P, bool term) {
  XRow<K> X;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const bool lastp = (p0 + j) == P - 1;
    const xf v = term ? xf_norm(E.m[j], E.e[j]) : xf{0.5f, 1};
    X.m[j] = lastp ? v.m : 0.0f;
    X.e[j] = lastp ? v.e : XF_EZERO;
  }
  return X;
}

template <int K, int R, int NB, bool DC>
__global__ __launch_bounds__(64 * kRowsWaves) void k_fwd_bwd_rows(FwdBwdArgs a) {
  constexpr int kNC = kRowsNC, kNH = kRowsNH, kWaves = kRowsWaves, kR2 = kRowsR2;
  constexpr int kChunk = rows_chunk<R, NB>();
  static_assert(R >= 2 * NB + kChunk - 1, "a dense-converter chunk must fit behind the chain");
  static_assert(NB % 2 == 0 && R % NB == 0 && (R / NB) % 2 == 0 && R % kR2 == 0 && R % 4 == 0 &&
                R >= 2 * NB && kR2 > NB, "batch / ring sizes");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Role role = role_of<kNC, kNH>(wave);
  const int lane = threadIdx.x & 63;
  const int T = a.T, U = a.U;  // U % K == 0 (the launcher checks)
  const int S = a.step_len[b];
  const int P = a.pos_len[b];
  const bool term = (a.flags & SSNT_FLAG_TERMINAL_EMIT) != 0;
  const size_t TU = (size_t)T * U;
  const float* lt = a.log_trans + (size_t)b * TU * 2;
  float* g = a.grad ? a.grad + (size_t)b * TU * 2 : nullptr;
  float* la = a.log_alpha ? a.log_alpha + (size_t)b * TU : nullptr;
  float* lb = a.log_beta ? a.log_beta + (size_t)b * TU : nullptr;
  const bool dbg = la || lb;
  const int p0 = K * lane;
  const bool act = p0 < U;
  const int pr = act ? p0 : U - K;  // LDS read position (clamped for lanes past U)

  Ctl* ctl = reinterpret_cast<Ctl*>(smem);
  xf* cuta = reinterpret_cast<xf*>(smem + kCtlBytes);
  xf* cutb = cuta + 64 * K;
  unsigned char* junk = reinterpret_cast<unsigned char*>(cutb + 64 * K);
  unsigned char* junk_lane = junk + 16 * K * lane;
  constexpr int kEnt = (R + 1) * 16;  // bytes per (d, q, lane) run of slots
  const int nl = U / K;               // lanes with positions
  unsigned char* inr = junk + 64 * 16 * K;
  xf* outr = reinterpret_cast<xf*>(inr + 2 * (size_t)(R + 1) * U * 16);
  xf* rows = outr + 2 * kR2 * U;  // kept lattice row s (even) at rows + (s >> 1) * U

  auto fill_rows = [&](int from, int w0, int wstep) {  // zero grads / -inf debug rows
    float z[2 * K], ninf[K];
#pragma unroll
    for (int j = 0; j < 2 * K; ++j) z[j] = 0.0f;
#pragma unroll
    for (int j = 0; j < K; ++j) ninf[j] = -__builtin_inff();
    for (int s = from + w0; s < T; s += wstep) {
      if (g) gst<K, 2, false>(z, brsrc(g + (size_t)s * U * 2, U * 8u), p0);
      if (la) gst<K, 1, false>(ninf, brsrc(la + (size_t)s * U, U * 4u), p0);
      if (lb) gst<K, 1, false>(ninf, brsrc(lb + (size_t)s * U, U * 4u), p0);
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
  const int M = (S - 1) >> 1;  // the cut
  const int n = S - 1;         // alpha chain steps (stream rows 0..n-1)
  const int jf0 = M >> 1;      // first forward pair (contains row M)
  const int jb0 = (M - 1) >> 1;  // first backward pair (contains row M-1; -1 when M == 0)

  if (threadIdx.x < kCtlBytes / 4) reinterpret_cast<int*>(smem)[threadIdx.x] = 0;
  __syncthreads();
  Diag dg;

  // pair bookkeeping: gradient wave h finishes its pairs in order (forward j = jf0 + h + kNH i,
  // backward j = jb0 - h - kNH i); help[d][h] counts them
  auto fwd_not_done = [&]() {  // smallest forward pair not done
    int m = INT_MAX;
#pragma unroll
    for (int h = 0; h < kNH; ++h) m = min(m, jf0 + h + kNH * ctr_ld(&ctl->help[0][h]));
    return m;
  };
  auto bwd_not_done = [&]() {  // largest backward pair not done
    int m = INT_MIN;
#pragma unroll
    for (int h = 0; h < kNH; ++h) m = max(m, jb0 - h - kNH * ctr_ld(&ctl->help[1][h]));
    return m;
  };
  // rows converted (a prefix): converter c owns rows c, c + kNC, ... -- or, dense (DC), chunks
  // of kChunk rows c, c + kNC, ...; conv[d][c] counts its rows / chunks done
  auto conv_rows = [&](int d) {
    if constexpr (DC) {
      int m = INT_MAX;
#pragma unroll
      for (int c = 0; c < kNC; ++c) m = min(m, kChunk * (c + kNC * ctr_ld(&ctl->conv[d][c])));
      return m;
    } else {
      return first_missing<kNC>(ctl->conv[d], 0);
    }
  };
  // factor entry of stream row r, lane l, element block 0 (block q: + q * nl * kEnt)
  auto slot_l = [&](int d, int r, int l) { return inr + ((size_t)(d * K) * nl + l) * kEnt + 16 * (r % R); };
  auto slot = [&](int d, int r) { return slot_l(d, r, pr / K); };
  auto rd_slot = [&](const unsigned char* sp, XRow<K>& E, XRow<K>& X) {
    float v[4 * K];
#pragma unroll
    for (int q = 0; q < K; ++q) ld_vec<4>(v + 4 * q, reinterpret_cast<const float*>(sp + (size_t)q * nl * kEnt));
#pragma unroll
    for (int q = 0; q < K; ++q) {
      E.m[q] = v[4 * q];
      E.e[q] = __builtin_bit_cast(int, v[4 * q + 1]);
      X.m[q] = v[4 * q + 2];
      X.e[q] = __builtin_bit_cast(int, v[4 * q + 3]);
    }
  };

  if (role.kind == 2) {
    // =============================== gradient waves ======================================
    const int d = role.d;
    const int h = role.idx;
    if (d == 0 && h == 0) {  // Z at the cut: tree-sum over p of alpha[M][p] * beta[M][p] (= oracle)
      const unsigned tag = a.loss_sum ? sum_tag(a) : 0u;
      spin_until<true>([&] { return ctr_acq(&ctl->a_ready); }, 1, a.status, dg);
      spin_until<true>([&] { return ctr_acq(&ctl->bm_ready); }, 1, a.status, dg);
      const XRow<K> Am = lds_xrow<K>(cuta + pr);
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

    // gradient (and debug) row s: A = alpha[s], E / Sh = factors of row s (Sh unshifted),
    // Bn = beta[s+1] (unused on the terminal transition), Bs = beta[s] (debug rows only)
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
      if (g) gst<K, 2, false>(ge, brsrc(g + (size_t)s * U * 2, U * 8u), p0);
      if (dbg) {  // debug outputs (slow path)
        float va[K], vb[K];
#pragma unroll
        for (int q = 0; q < K; ++q) {
          va[q] = zero_z ? -__builtin_inff() : xf_log(xf_norm(A.m[q], A.e[q]));  // (lazy rows)
          vb[q] = zero_z ? -__builtin_inff() : xf_log(xf_norm(Bs.m[q], Bs.e[q]));
        }
        if (la) gst<K, 1, false>(va, brsrc(la + (size_t)s * U, U * 4u), p0);
        if (lb) gst<K, 1, false>(vb, brsrc(lb + (size_t)s * U, U * 4u), p0);
      }
    };
    const XRow<K> zr = xrow_zero<K>();
    int done = 0;
    if (d == 0) {
      // forward pairs: rows ra = 2j (if >= M), rb = 2j+1 (if <= S-1); alpha from the chain ring
      // (alpha[M]: cut A); beta[2j+2] kept, beta[2j+1] rebuilt (beta[M]: cut B)
      int seen_chain = 0, seen_conv = 0;
      for (int j = jf0 + h; 2 * j <= S - 1; j += kNH) {
        const int ra = 2 * j, rb = 2 * j + 1;
        const bool has_a = ra >= M, has_b = rb <= S - 1;
        const int last = has_b ? rb : ra;
        if (last > M && seen_chain < last)
          seen_chain = spin_until<true>([&] { return ctr_ld(&ctl->chain[0]); }, last, a.status, dg);
        if (seen_conv <= last)
          seen_conv = spin_until<true>([&] { return conv_rows(0); }, last + 1, a.status, dg);
        cbar();
        XRow<K> Aa = zr, Ab = zr, Ea = zr, La = zr, Eb = zr, Lb = zr, Bc = zr, Bdbg = zr, Bmb = zr;
        auto rdA = [&](int s) {
          return s == M ? lds_xrow<K>(cuta + pr) : lds_xrow<K>(outr + (size_t)(s % kR2) * U + pr);
        };
        if (has_a) {
          Aa = rdA(ra);
          rd_slot(slot(0, ra), Ea, La);
        }
        if (has_b) {
          Ab = rdA(rb);
          rd_slot(slot(0, rb), Eb, Lb);
        }
        if (rb + 1 <= S - 1) Bc = lds_xrow<K>(rows + (size_t)(j + 1) * U + pr);  // beta[2j+2]
        if (dbg && has_a) Bdbg = (ra == M) ? lds_xrow<K>(cutb + pr) : lds_xrow<K>(rows + (size_t)j * U + pr);
        if (has_b && rb == M) Bmb = lds_xrow<K>(cutb + pr);
        cbar();
        ctr_st(&ctl->help[0][h], ++done);  // every LDS read of the pair issued (in-order DS)
        // beta[2j+1] (odd): cut B when it is beta[M], the terminal row when rb = S-1, else one
        // beta step from beta[2j+2] with the factors of row 2j+1
        XRow<K> Shb = zr;
        XRow<K> Bodd = Bmb;
        if (has_b) {
          Shb = unshift<K>(Lb, p0, P);
          if (rb != M) {
            if (rb == S - 1) {
              Bodd = terminal_row<K>(Eb, p0, P, term);
            } else if (has_a || dbg) {
              Bodd = Bc;
              XRow<K> ones;
#pragma unroll
              for (int q = 0; q < K; ++q) {
                ones.m[q] = 1.0f;
                ones.e[q] = 0;
              }
              beta_chain<K, false, true>(Bodd, Eb, Shb, ones);
            }
          }
        }
        if (has_a) emit(ra, Aa, Ea, unshift<K>(La, p0, P), Bodd, Bdbg);
        if (has_b) emit(rb, Ab, Eb, Shb, Bc, Bodd);
      }
    } else if (M >= 1) {
      // backward pairs (descending): rows ra = 2j, rb = 2j+1 (if <= M-1); alpha[2j] kept,
      // alpha[2j+1] rebuilt; beta from the chain ring (beta[M]: cut B)
      int seen_chain = 0, seen_conv = 0;
      auto bring = [&](int x) {  // beta[x], x <= M: chain ring row of stream row S-1-x, or cut B
        return x == M ? lds_xrow<K>(cutb + pr) : lds_xrow<K>(outr + (size_t)(kR2 + (S - 1 - x) % kR2) * U + pr);
      };
      for (int j = jb0 - h; j >= 0; j -= kNH) {
        const int ra = 2 * j, rb = 2 * j + 1;
        const bool has_b = rb <= M - 1;
        const int xlow = dbg ? ra : ra + 1;  // lowest beta row read
        const int need = S - xlow;           // beta[x] is stream row S-1-x
        if (xlow < M && seen_chain < need)
          seen_chain = spin_until<true>([&] { return ctr_ld(&ctl->chain[1]); }, need, a.status, dg);
        if (seen_conv <= S - 1 - ra)
          seen_conv = spin_until<true>([&] { return conv_rows(1); }, S - ra, a.status, dg);
        cbar();
        XRow<K> Ea, Sa, Eb = zr, Sb = zr, Bdbg = zr, B2 = zr;
        const XRow<K> Aa = lds_xrow<K>(rows + (size_t)j * U + pr);  // alpha[2j]
        rd_slot(slot(1, S - 1 - ra), Ea, Sa);
        const XRow<K> B1 = bring(ra + 1);  // beta[2j+1]
        if (has_b) {
          rd_slot(slot(1, S - 1 - rb), Eb, Sb);
          B2 = bring(rb + 1);  // beta[2j+2]
        }
        if (dbg) Bdbg = bring(ra);
        cbar();
        ctr_st(&ctl->help[1][h], ++done);
        emit(ra, Aa, Ea, Sa, B1, Bdbg);
        if (has_b) {
          XRow<K> Ab = Aa;  // alpha[2j+1]: one alpha step from alpha[2j] with row 2j's factors
          alpha_step_sh<K>(Ab, Ea, Sa);
          emit(rb, Ab, Eb, Sb, B2, B1);
        }
      }
    }
    dg.flush(b, role.slot);
    return;
  }

  if (DC && role.kind == 1) {
    // ============================ dense converters (K = 2) ===============================
    // A chunk = kChunk consecutive stream rows, contiguous in log_trans; its nl = U/2 position
    // pairs per row are spread over all 64 lanes: item t of chunk k is granule g = 64 t + lane,
    // row rr = g / nl of the chunk, pair l = g % nl (NI = ceil(kChunk nl / 64) items; at U = 80
    // 5 items for 8 rows, where the row layout spends 8 wave-passes with 24 idle lanes each).
    // The loads are 1 KiB contiguous per wave-instruction; the forward ring's pre-shift
    // L[2l] = Sh[2l-1] comes from the lane before (DPP), lane 0 from the previous item's lane 63.
    const int d = role.d;
    const int c = role.idx;
    constexpr int D = kRowsConvDepth;  // items in flight
    const unsigned tag0 = (d == 0 && c == 0 && b == 0 && a.loss_sum) ? sum_tag(a) : 0u;
    const int NI = (kChunk * nl + 63) >> 6;
    const int nchunks = (S + kChunk - 1) / kChunk;
    const int mine = nchunks > c ? (nchunks - c + kNC - 1) / kNC : 0;  // chunks c, c + kNC, ...
    const int nitems = mine * NI;
    const unsigned mnl = ((1u << 20) + (unsigned)nl - 1) / (unsigned)nl;  // g / nl = g * mnl >> 20
    const __amdgpu_buffer_rsrc_t lt_r = brsrc(lt, (unsigned)(TU * 8));
    auto item_src = [&](int t) {  // byte offset of item t's granule (negative: before the tensor)
      const int k = t / NI, it = t - k * NI;
      const int cc = c + kNC * k;
      const int g = 64 * it + lane;
      const int row0 = d == 0 ? kChunk * cc : S - kChunk - kChunk * cc;  // lowest lattice row
      return (row0 * nl + g) * 16;
    };
    auto load = [&](int t, float* v) {
      const int off = item_src(t);
      buf_ld<4>(v, lt_r, off >= 0 ? off : INT_MIN);  // (out of range: zeros)
    };
    float pf[D][4];
#pragma unroll
    for (int i = 0; i < D; ++i) load(i, pf[i]);
    int seen_read = 0;
    int fwd_nd = d == 0 ? jf0 : 0, bwd_nd = d == 1 ? jb0 : 0;
    const int grow0 = d == 0 ? M : S - M;
    float carry_m = 0.0f;  // Sh[2l+1] of the previous item's lane 63 (forward pre-shift)
    int carry_e = XF_EZERO;
    for (int base = 0; base < nitems; base += D) {
#pragma unroll
      for (int i = 0; i < D; ++i) {
        const int t = base + i;
        if (t < nitems) {
          const int k = t / NI, it = t - k * NI;
          const int cc = c + kNC * k;  // chunk: stream rows kChunk cc .. + kChunk - 1
          if (it == 0) {
            // the chunk's slots last held stream rows up to kChunk (cc + 1) - 1 - R: read by the
            // chain, and (gradient rows of this direction) by a gradient pair
            const int qmax = kChunk * (cc + 1) - 1 - R;
            if (qmax >= 0) {
              if (seen_read <= qmax)
                seen_read = spin_until<true>([&] { return ctr_ld(&ctl->sread[d]); }, qmax + 1, a.status, dg);
              if (qmax >= grow0) {
                if (d == 0) {
                  const int pj = qmax >> 1;
                  if (fwd_nd <= pj)
                    fwd_nd = spin_until<true>([&] { return fwd_not_done(); }, pj + 1, a.status, dg);
                } else {
                  const int pj = (S - 1 - qmax) >> 1;
                  if (bwd_nd >= pj)
                    bwd_nd = -spin_until<true>([&] { return -bwd_not_done(); }, 1 - pj, a.status, dg);
                }
              }
            }
            carry_m = 0.0f;
            carry_e = XF_EZERO;
          }
          const int g = 64 * it + lane;
          const int rl = (int)(((unsigned)g * mnl) >> 20);  // row of the chunk, in lattice order
          const int l = g - rl * nl;
          const int rr = d == 0 ? rl : kChunk - 1 - rl;  // row of the chunk, in stream order
          const int r = kChunk * cc + rr;                // stream row
          const bool live = rl < kChunk && r < S;
          const int pp = 2 * l;
          float em0, ms0, em1, ms1;
          int ee0, es0, ee1, es1;
          xf_exp_pair(pf[i][0], pf[i][1], pp < P, pp < P - 1, em0, ee0, ms0, es0);
          xf_exp_pair(pf[i][2], pf[i][3], pp + 1 < P, pp + 1 < P - 1, em1, ee1, ms1, es1);
          float xm0 = ms0, xm1 = ms1;
          int xe0 = es0, xe1 = es1;
          if (d == 0) {  // L[2l] = Sh[2l-1] (lane before; zero at l = 0), L[2l+1] = Sh[2l]
            const float lm = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                 __builtin_bit_cast(int, carry_m), __builtin_bit_cast(int, ms1), 0x138, 0xf, 0xf, false));
            const int le = __builtin_amdgcn_update_dpp(carry_e, es1, 0x138, 0xf, 0xf, false);
            carry_m = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ms1), 63));
            carry_e = __builtin_amdgcn_readlane(es1, 63);
            xm1 = ms0;
            xe1 = es0;
            xm0 = l == 0 ? 0.0f : lm;
            xe0 = l == 0 ? XF_EZERO : le;
          }
          cbar();
          if (live) {
            unsigned char* e0 = slot_l(d, r, l);
            const float v0[4] = {em0, __builtin_bit_cast(float, ee0), xm0, __builtin_bit_cast(float, xe0)};
            const float v1[4] = {em1, __builtin_bit_cast(float, ee1), xm1, __builtin_bit_cast(float, xe1)};
            st_vec<4>(reinterpret_cast<float*>(e0), v0);
            st_vec<4>(reinterpret_cast<float*>(e0 + (size_t)nl * kEnt), v1);
          }
          cbar();
          if (it == NI - 1) ctr_st(&ctl->conv[d][c], k + 1);
        }
        load(t + D, pf[i]);  // refill in place
      }
    }
    dg.flush(b, role.slot);
    fill_rows(S, d * kNC + c, 2 * kNC);  // zero the rows beyond S
    if (d == 0 && c == 0 && b == 0 && a.loss_sum) finish_loss_sum(a, tag0);
    return;
  }

  if (role.kind == 1) {
    // =============================== converters ==========================================
    const int d = role.d;
    const int c = role.idx;
    constexpr int D = kRowsConvDepth;
    const unsigned tag0 = (d == 0 && c == 0 && b == 0 && a.loss_sum) ? sum_tag(a) : 0u;
    auto load = [&](int r, Item<K, false>& it) {
      const int row = min(max(d == 0 ? r : S - 1 - r, 0), T - 1);
      gld<K, 2, false>(it.lt, brsrc(lt + (size_t)row * U * 2, U * 8u), p0);
    };
    Item<K, false> pf[D];
#pragma unroll
    for (int i = 0; i < D; ++i) load(c + kNC * i, pf[i]);
    int seen_read = 0;
    int fwd_nd = d == 0 ? jf0 : 0, bwd_nd = d == 1 ? jb0 : 0;
    // the gradient rows of this direction: forward s >= M, backward s <= M-1 (stream >= S-M)
    const int grow0 = d == 0 ? M : S - M;
    const int nmine = (S - c + kNC - 1) / kNC;  // my stream rows: c, c + kNC, ...
    for (int base = 0; base < nmine; base += D) {
#pragma unroll
      for (int i = 0; i < D; ++i) {
        const int k = base + i;
        if (k < nmine) {
          const int r = c + kNC * k;
          XRow<K> E, Sh;
          convert<K, false>(pf[i], P, lane, E, Sh);
          XRow<K> Xs;
          if (d == 0) {  // L[p] = Sh[p-1]: canonical zero at p = 0
            Xs.m[0] = shr1(Sh.m[K - 1]);
            Xs.e[0] = shr1(Sh.e[K - 1]);
#pragma unroll
            for (int j = 1; j < K; ++j) {
              Xs.m[j] = Sh.m[j - 1];
              Xs.e[j] = Sh.e[j - 1];
            }
          } else {
            Xs = Sh;
          }
          // slot r % R last held stream row q = r - R: read by the chain, and by a gradient pair
          const int q = r - R;
          if (q >= 0) {
            if (seen_read <= q)
              seen_read = spin_until<true>([&] { return ctr_ld(&ctl->sread[d]); }, q + 1, a.status, dg);
            if (q >= grow0) {
              if (d == 0) {
                const int pj = q >> 1;  // forward pair of row q
                if (fwd_nd <= pj)
                  fwd_nd = spin_until<true>([&] { return fwd_not_done(); }, pj + 1, a.status, dg);
              } else {
                const int pj = (S - 1 - q) >> 1;  // backward pair of row S-1-q (done: j > not_done)
                if (bwd_nd >= pj)
                  bwd_nd = -spin_until<true>([&] { return -bwd_not_done(); }, 1 - pj, a.status, dg);
              }
            }
          }
          cbar();
          unsigned char* sl = slot_l(d, r, lane);
          float v[4 * K];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            v[4 * j] = E.m[j];
            v[4 * j + 1] = __builtin_bit_cast(float, E.e[j]);
            v[4 * j + 2] = Xs.m[j];
            v[4 * j + 3] = __builtin_bit_cast(float, Xs.e[j]);
          }
#pragma unroll
          for (int q2 = 0; q2 < K; ++q2)
            st_vec<4>(reinterpret_cast<float*>(act ? sl + (size_t)q2 * nl * kEnt : junk_lane + 16 * q2), v + 4 * q2);
          cbar();
          ctr_st(&ctl->conv[d][c], k + 1);
        }
        load(c + kNC * (k + D), pf[i]);  // refill in place (no register copy with a load in flight)
      }
    }
    dg.flush(b, role.slot);
    fill_rows(S, d * kNC + c, 2 * kNC);  // zero the rows beyond S
    if (d == 0 && c == 0 && b == 0 && a.loss_sum) finish_loss_sum(a, tag0);
    return;
  }

  // ================================== chains =============================================
  // Stream rows in unrolled blocks of R (so every slot index, ring-row index and normalisation
  // point is a compile-time constant); a block is R / NB batches. At the start of a batch the
  // chain waits until the NEXT batch is converted (and, past the cut, until the chain-ring rows
  // it will write are free), issues that batch's slot reads into the other register buffer and
  // publishes them, then steps through the current batch from registers.
  __builtin_amdgcn_s_setprio(3);
  const int d = role.d;
  const unsigned char* sbase = slot(d, 0);  // slot j of this lane: sbase + 16 j (+ q nl kEnt)
  XRow<K> Eb[2][NB], Xb[2][NB];
  XRow<K> ones;
#pragma unroll
  for (int q = 0; q < K; ++q) {
    ones.m[q] = 1.0f;
    ones.e[q] = 0;
  }
  const int nrows = d == 0 ? n : S;  // stream rows the chain consumes
  int ready = 0;
  auto wait_conv = [&](int need) {
    if (ready < need) ready = spin_until<false>([&] { return conv_rows(d); }, need, a.status, dg);
  };
  auto read_batch = [&](auto Hc, int base) {  // slots of batch Hc of the block at `base`
    constexpr int H = decltype(Hc)::value;
    (void)base;
    sfor<NB>([&](auto Ic) {
      constexpr int i = decltype(Ic)::value;
      rd_slot(sbase + 16 * ((H * NB + i) % R), Eb[H & 1][i], Xb[H & 1][i]);
    });
  };
  // Batch head: drain this wave's LDS queue (the current batch's slot reads, issued a batch ago,
  // and the previous batch's row stores -- long done in the steady state), then issue the next
  // batch's reads unconditionally (past the last row they read stale slots, harmlessly) and
  // publish them. With every path through a batch issuing the same LDS operations and nothing
  // outstanding from before, the compiler needs no LDS wait inside the batch: counted waits
  // merged across the batch kinds' paths had made steps wait for the NEXT batch's reads.
  auto batch_head = [&](auto Hn, int read_to) {
    cbar();
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) (vmcnt, expcnt: no wait)
    read_batch(Hn, 0);
    cbar();
    ctr_st(&ctl->sread[d], read_to);
  };
  const int wstep = act ? U : 0;
  if (d == 0) {
    // ---------------- alpha chain: stream row r = transition r -> alpha[r+1] --------------
    XRow<K> X = xrow_zero<K>();
    if (lane == 0) {
      X.m[0] = 0.5f;  // alpha[0] = 1 at p = 0
      X.e[0] = 1;
    }
    xf* wp = act ? rows + p0 : reinterpret_cast<xf*>(junk_lane);  // kept row 0 (then 2, 4, ...)
    if (M == 0) {
      lds_xrow_st<K>(act ? cuta + p0 : reinterpret_cast<xf*>(junk_lane), X);
      cbar();
      ctr_rel(&ctl->a_ready, 1);
    } else {
      lds_xrow_st<K>(wp, X);
      wp += wstep;
    }
    xf* optr[kR2];  // chain-ring row j, this lane
#pragma unroll
    for (int j = 0; j < kR2; ++j) optr[j] = act ? outr + (size_t)j * U + p0 : reinterpret_cast<xf*>(junk_lane);
    int fwd_nd = jf0;
    if (nrows > 0) {
      wait_conv(min(NB, nrows));
      cbar();
      read_batch(std::integral_constant<int, 0>{}, 0);
      cbar();
      ctr_st(&ctl->sread[0], min(NB, nrows));
    }
    for (int base = 0; base < nrows; base += R) {
      sfor<R / NB>([&](auto Hc) {
        constexpr int H = decltype(Hc)::value;
        const int b0 = base + H * NB, b1 = b0 + NB;
        if (b0 >= nrows) return;
        if (b1 < nrows) wait_conv(min(b1 + NB, nrows));
        const int xmax = min(b1, nrows);  // alpha rows written: (b0, xmax]
        if (xmax - kR2 > M) {  // previous occupant alpha[x - kR2] read by forward pair (x - kR2)/2
          const int pj = (xmax - kR2) >> 1;
          if (fwd_nd <= pj) fwd_nd = spin_until<false>([&] { return fwd_not_done(); }, pj + 1, a.status, dg);
        }
        batch_head(std::integral_constant<int, H + 1>{}, min(b1 + NB, nrows));
        auto step = [&](auto Ic, auto Mode) {
          constexpr int i = decltype(Ic)::value;
          constexpr int mode = decltype(Mode)::value;  // 0 before the cut, 1 past it, 2 guarded
          const int r = b0 + i;
          if constexpr (mode == 2) {
            if (r >= nrows) return;
          }
          alpha_chain<K, false, ((H * NB + i) % kChainNorm) == kChainNorm - 1>(X, Eb[H & 1][i], Xb[H & 1][i], ones);
          constexpr int xo = (H * NB + i + 1) % kR2;  // ring row of alpha[r+1]
          if constexpr (mode == 0) {
            if constexpr ((i & 1) == 1) {  // r + 1 even (b0 is even): kept
              lds_xrow_st<K>(wp, X);
              wp += wstep;
            }
          } else if constexpr (mode == 1) {
            lds_xrow_st<K>(optr[xo], X);
          } else {
            const int x = r + 1;
            if (x < M) {
              if ((x & 1) == 0) {
                lds_xrow_st<K>(wp, X);
                wp += wstep;
              }
            } else if (x == M) {
              lds_xrow_st<K>(act ? cuta + p0 : reinterpret_cast<xf*>(junk_lane), X);
              cbar();
              ctr_rel(&ctl->a_ready, 1);
              dg.mark_cut();
            } else {
              lds_xrow_st<K>(optr[xo], X);
            }
          }
        };
        if (b1 < M) {
          sfor<NB>([&](auto Ic) { step(Ic, std::integral_constant<int, 0>{}); });
        } else if (b0 + 1 > M && b1 <= nrows) {
          sfor<NB>([&](auto Ic) { step(Ic, std::integral_constant<int, 1>{}); });
        } else {
          sfor<NB>([&](auto Ic) { step(Ic, std::integral_constant<int, 2>{}); });
        }
        cbar();
        ctr_st(&ctl->chain[0], xmax);
      });
    }
  } else {
    // ---------------- beta chain: stream row r -> beta[S-1-r] (row 0: the terminal row) ----
    const int c = S - 1 - M;  // stream row of the cut (beta[M])
    XRow<K> X = xrow_zero<K>();
    // kept beta rows descend from the highest even row <= S-1
    xf* wp = act ? rows + (size_t)((S - 1) >> 1) * U + p0 : reinterpret_cast<xf*>(junk_lane);
    xf* optr[kR2];
#pragma unroll
    for (int j = 0; j < kR2; ++j) optr[j] = act ? outr + (size_t)(kR2 + j) * U + p0 : reinterpret_cast<xf*>(junk_lane);
    int bwd_nd = jb0;
    wait_conv(min(NB, nrows));
    cbar();
    read_batch(std::integral_constant<int, 0>{}, 0);
    cbar();
    ctr_st(&ctl->sread[1], min(NB, nrows));
    for (int base = 0; base < nrows; base += R) {
      sfor<R / NB>([&](auto Hc) {
        constexpr int H = decltype(Hc)::value;
        const int b0 = base + H * NB, b1 = b0 + NB;
        if (b0 >= nrows) return;
        if (b1 < nrows) wait_conv(min(b1 + NB, nrows));
        // beta rows written below the cut: x = S-1-r for r in [b0, min(b1, S)); the lowest is
        // xmin = S - min(b1, S); its ring row's previous occupant beta[xmin + kR2] is read by
        // backward pairs (xmin + kR2)/2 and (xmin + kR2 - 1)/2
        const int xmin = S - min(b1, nrows);
        if (xmin + kR2 < M) {
          const int pj = (xmin + kR2 - 1) >> 1;
          if (bwd_nd >= pj) bwd_nd = -spin_until<false>([&] { return -bwd_not_done(); }, 1 - pj, a.status, dg);
        }
        batch_head(std::integral_constant<int, H + 1>{}, min(b1 + NB, nrows));
        auto step = [&](auto Ic, auto Mode) {
          constexpr int i = decltype(Ic)::value;
          constexpr int mode = decltype(Mode)::value;  // 0 above the cut, 1 below it, 2 guarded
          const int r = b0 + i;
          if constexpr (mode == 2) {
            if (r >= nrows) return;
            if (r == 0) {
              X = terminal_row<K>(Eb[H & 1][i], p0, P, term);
            } else {
              beta_chain<K, false, ((H * NB + i) % kChainNorm) == kChainNorm - 1>(X, Eb[H & 1][i], Xb[H & 1][i], ones);
            }
          } else {
            beta_chain<K, false, ((H * NB + i) % kChainNorm) == kChainNorm - 1>(X, Eb[H & 1][i], Xb[H & 1][i], ones);
          }
          constexpr int ro = (H * NB + i) % kR2;  // ring row of stream row r
          const int x = S - 1 - r;
          if constexpr (mode == 0) {
            if ((x & 1) == 0) {
              lds_xrow_st<K>(wp, X);
              wp -= wstep;
            }
          } else if constexpr (mode == 1) {
            lds_xrow_st<K>(optr[ro], X);
          } else {
            if (x > M) {
              if ((x & 1) == 0) {
                lds_xrow_st<K>(wp, X);
                wp -= wstep;
              }
            } else if (x == M) {
              lds_xrow_st<K>(act ? cutb + p0 : reinterpret_cast<xf*>(junk_lane), X);
              cbar();
              ctr_rel(&ctl->bm_ready, 1);
              dg.mark_cut();
            } else {
              lds_xrow_st<K>(optr[ro], X);
            }
          }
        };
        if (b0 >= 1 && b1 <= c) {
          sfor<NB>([&](auto Ic) { step(Ic, std::integral_constant<int, 0>{}); });
        } else if (b0 > c && b1 <= nrows) {
          sfor<NB>([&](auto Ic) { step(Ic, std::integral_constant<int, 1>{}); });
        } else {
          sfor<NB>([&](auto Ic) { step(Ic, std::integral_constant<int, 2>{}); });
        }
        cbar();
        ctr_st(&ctl->chain[1], min(b1, nrows));
      });
    }
  }
  dg.flush(b, role.slot);
}

template <int K, int R, int NB, bool DC>
int launch_rows_kernel(const FwdBwdArgs& a, hipStream_t st) {
  auto kern = k_fwd_bwd_rows<K, R, NB, DC>;
  const size_t lds = rows_lds_bytes(K, a.T, a.U, R);
  note_fwd_bwd_dispatch("k_fwd_bwd_rows<K=%d,R=%d,NB=%d,DC=%d>", K, R, NB, (int)DC);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBudget);
  hipLaunchKernelGGL(kern, dim3(a.B), dim3(64 * kRowsWaves), lds, st, a);
  return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
}

template <int K, bool DC>
int launch_rows_k(const FwdBwdArgs& a, hipStream_t st) {
  if (rows_lds_bytes(K, a.T, a.U, 24) <= kLdsBudget) return launch_rows_kernel<K, 24, 4, DC>(a, st);
  if (rows_lds_bytes(K, a.T, a.U, 16) <= kLdsBudget) return launch_rows_kernel<K, 16, 4, DC>(a, st);
  if (rows_lds_bytes(K, a.T, a.U, 8) <= kLdsBudget) return launch_rows_kernel<K, 8, 2, DC>(a, st);
  return SSNT_ERR_UNSUPPORTED;
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

int launch_fwd_bwd_rows(const FwdBwdArgs& a, hipStream_t st, bool dense) {
  // U <= 128 without log_obs, whole lane slices and 16-byte aligned tensors; else the streaming
  // kernel (which takes log_obs, odd U and 4- / 8-byte alignment)
  if (a.log_obs || a.U > 128) return SSNT_ERR_UNSUPPORTED;
  const int K = a.U <= 64 ? 1 : 2;
  if (a.U % K != 0 || !al16(a.log_trans) || !al16(a.grad) || !al16(a.log_alpha) || !al16(a.log_beta))
    return SSNT_ERR_UNSUPPORTED;
  if (K == 1) return launch_rows_k<1, false>(a, st);
  return dense ? launch_rows_k<2, true>(a, st) : launch_rows_k<2, false>(a, st);
}

#ifdef SSNT_DIAG
// this file's copy of the per-wave cycle totals (stream_dev.h g_diag is per translation unit)
int rows_diag_read(void* host, size_t bytes) {
  if (bytes > sizeof(g_diag)) bytes = sizeof(g_diag);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? (int)bytes : -1;
}
#endif

size_t rows_kernel_lds(int T, int U) {  // 0 when the kernel does not take the shape
  if (U > 128 || U <= 0) return 0;
  const int K = U <= 64 ? 1 : 2;
  if (U % K != 0) return 0;
  for (int R : {24, 16, 8})
    if (rows_lds_bytes(K, T, U, R) <= kLdsBudget) return rows_lds_bytes(K, T, U, R);
  return 0;
}

}  // namespace ssnt
