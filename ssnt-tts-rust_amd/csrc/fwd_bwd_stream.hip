// fwd_bwd_stream.hip -- streaming lattice forward-backward for gfx950 (the default kernel).
//
// Same lattice and the same split-exponent arithmetic as the two-wave kernel in fwd_bwd.hip
// (DESIGN.md "Lattice semantics", "Split-exponent arithmetic"); bit-exact with
// oracle/ssnt_oracle.c. What differs is who does what. One workgroup = one utterance; roles
// (role_of) for the default K <= 2 mix, 16 waves:
//
//   1 wave      alpha chain: alpha[1..S-1], nothing else on its instruction stream
//   1 wave      beta chain:  beta[S-1..0]
//   3 + 3 waves converters (per direction): load log_trans / log_obs rows from HBM, exp() them
//               into split-exponent factors, write them to an R-slot LDS ring per direction.
//               The forward ring holds the shift factors pre-shifted by one position
//               (L[p] = Sh[p-1]), so the alpha chain's only cross-lane move is a DPP of its own
//               row that the compiler folds into the multiply (v_mul_f32_dpp / v_add_u32_dpp).
//   4 + 4 waves gradient waves (per direction): one of them forms Z at the cut M = (S-1)>>1,
//               then they emit d loss / d log_trans (and d loss / d log_obs) row by row behind
//               the chains, reading the chain rows, the stored rows and the converters' ring
//               (each cell is converted once per direction; these waves load nothing from HBM).
// K >= 4 runs 2 + 2 + 2 per direction (10 waves: 168 VGPRs per wave, no spills).
//
// The cost model that shapes this (measured, tools/micro/): a lone wave issues one VALU
// instruction per ~4.4 cycles whether or not the instructions depend on each other, so a chain
// step costs its instruction count. The chains therefore carry only the recurrence; every
// other instruction lives on another wave.
//
// Rows kept for the gradients: alpha[0..M] and beta[M+1..S-1] in "storage" (LDS when T*U*8 B
// fits beside the rings, else a global workspace), beta[M] in a cut buffer; the chain rows past
// the cut (alpha[M+1..], beta[..M-1]) go through a 4-row LDS ring to the gradient waves.
//
// Synchronisation is all LDS counters in one workgroup. A wave's DS instructions execute in
// order, so "write data, then store counter" publishes and "read slot, then store counter"
// releases without a wait; a compiler barrier keeps the program order. Every spin is bounded
// (status bit kStatusTimeout).
//
// Lanes past U (p0 = K*lane >= U) read a clamped valid position and write to a junk area; their
// values never reach a valid position except multiplied by a masked (exact zero) factor.
#include <hip/hip_runtime.h>
#include <string.h>
#include <limits.h>

#include <atomic>
#include <type_traits>
#include <utility>

#include "lattice_dev.h"
#include "stream_dev.h"

namespace ssnt {
namespace {


template <bool OBS>
constexpr int in_slots() { return OBS ? 4 : 8; }  // converted-row ring slots per direction
template <bool OBS>
constexpr int out_slots() { return OBS ? 4 : 8; }  // chain-row ring (rows past the cut) per direction
template <bool OBS>
constexpr int kChainPrefetch(int R) { return R >= 16 ? 4 : 2; }  // factor rows in flight per chain
template <int K>
constexpr int conv_depth() { return K <= 2 ? 8 : (K <= 4 ? 4 : 2); }  // converter prefetch rows

// DBG: debug rows requested (log_alpha / log_beta, f32 logs or the raw split-exponent state of
// ssnt_fwd_bwd_debug64_device) -- a separate instance, so the product's carries neither the
// debug path nor its pointers (their SGPRs spilled into VGPR lanes in the hot loops)
template <int K, bool OBS, bool LDS, int kNC, int kNH, int kRingSel, bool NV, bool DBG>
__global__ __launch_bounds__(64 * (2 + 2 * kNC + 2 * kNH)) void k_fwd_bwd_stream(FwdBwdArgs a) {
  constexpr int kWaves = 2 + 2 * kNC + 2 * kNH;
  // kRingSel: ring slots (0 = default; 16 / 32: the A/B build's deep rings)
  constexpr int R = kRingSel ? kRingSel : in_slots<OBS>();
  constexpr int kR2 = out_slots<OBS>() < R ? out_slots<OBS>() : R;
  static_assert(R % kR2 == 0, "ring sizes");
#ifdef SSNT_DIAG
  static_assert(R <= 32 && kR2 <= 16, "ring tags (Ctl)");
#endif
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
  const float* lo = OBS ? a.log_obs + (size_t)b * TU : nullptr;
  float* g = a.grad ? a.grad + (size_t)b * TU * 2 : nullptr;
  float* go = (OBS && a.grad_obs) ? a.grad_obs + (size_t)b * TU : nullptr;
  float* la = (DBG && a.log_alpha) ? a.log_alpha + (size_t)b * TU : nullptr;
  float* lb = (DBG && a.log_beta) ? a.log_beta + (size_t)b * TU : nullptr;
  int* lae = (DBG && la && a.log_alpha_e) ? a.log_alpha_e + (size_t)b * TU : nullptr;  // raw-state debug
  int* lbe = (DBG && lb && a.log_beta_e) ? a.log_beta_e + (size_t)b * TU : nullptr;
  const int p0 = K * lane;
  const bool act = p0 < U;
  const int pr = act ? p0 : Up - K;  // LDS read position (clamped for lanes past U)

  // ---- LDS: ctl | cut (64K xf) | junk (64 x 16K B) | input rings [2][R] | chain-row rings
  //      [2][kR2][U xf] | storage rows [T][U xf] (LDS mode)
  Ctl* ctl = reinterpret_cast<Ctl*>(smem);
  xf* cutb = reinterpret_cast<xf*>(smem + kCtlBytes);
  unsigned char* junk = reinterpret_cast<unsigned char*>(cutb + 64 * K);
  const int slot_bytes = (Up * 16 + (OBS ? Up * 8 : 0) + 15) & ~15;
  const int nl16 = (Up / K) * 16;  // bytes of one element block of a slot
  unsigned char* inr = junk + 64 * 16 * K;
  xf* outr = reinterpret_cast<xf*>(inr + 2 * R * slot_bytes);
  xf* rows = LDS ? outr + 2 * kR2 * Up : reinterpret_cast<xf*>(a.workspace) + (size_t)b * T * Up;
  unsigned char* junk_lane = junk + 16 * K * lane;
#define SSNT_GST2(v, tensor, s) gst<K, 2, NV>(v, brsrc(tensor + (size_t)(s) * U * 2, U * 8u), p0)
#define SSNT_GST1(v, tensor, s) gst<K, 1, NV>(v, brsrc(tensor + (size_t)(s) * U, U * 4u), p0)

  auto fill_rows = [&](int from, int w0, int wstep) {  // zero grads / -inf debug rows
    float z[2 * K], ninf[K];
#pragma unroll
    for (int j = 0; j < 2 * K; ++j) z[j] = 0.0f;
#pragma unroll
    for (int j = 0; j < K; ++j) ninf[j] = (DBG && a.log_alpha_e) ? 0.0f : -__builtin_inff();  // raw: mantissa 0
    for (int s = from + w0; s < T; s += wstep) {
      if (g) SSNT_GST2(z, g, s);
      if (go) SSNT_GST1(z, go, s);
      if (la) SSNT_GST1(ninf, la, s);
      if (lb) SSNT_GST1(ninf, lb, s);
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
  const int M = (S - 1) >> 1;

  // storage rows: LDS, or this utterance's workspace rows through range-checked buffer ops
  auto row_st = [&](int s, const XRow<K>& r) {
    if constexpr (LDS) {
      lds_xrow_st<K>(act ? rows + (size_t)s * Up + p0 : reinterpret_cast<xf*>(junk_lane), r);
    } else {
      float v[2 * K];
      xrow_pack<K>(r, v);
      buf_st<2 * K>(v, brsrc(rows + (size_t)s * Up, Up * 8u), p0 * 8);
    }
  };
  auto row_ld = [&](int s) {
    if constexpr (LDS) {
      return lds_xrow<K>(rows + (size_t)s * Up + pr);
    } else {
      float v[2 * K];
      buf_ld<2 * K>(v, brsrc(rows + (size_t)s * Up, Up * 8u), pr * 8);
      return xrow_unpack<K>(v);
    }
  };
  // converted-input slot j of direction d: per position (E.m, E.e, X.m, X.e); obs block after


  if (threadIdx.x < kCtlBytes / 4) reinterpret_cast<int*>(smem)[threadIdx.x] = 0;
  XRow<K> X = xrow_zero<K>();
  if (role.kind == 0 && role.d == 0) {  // alpha[0]: 1 at p = 0 (x obs[0][0])
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
    row_st(0, X);
  }
  __syncthreads();
  Diag dg;

  if (role.kind == 2) {
    // =============================== gradient waves ======================================
    const int d = role.d;
    const int h = role.idx;
    const int hb = d == 0 ? M : S - M;  // first stream row of this direction's gradient rows
    const int n_rows = d == 0 ? S - M : M;  // transitions M..S-1 / M-1..0
    const int nmine = (n_rows - h + kNH - 1) / kNH;
    // The gradient waves take their (E, Sh) factors from the converters' input ring: the slot
    // of stream row r holds exactly the factors of that row (the forward ring holds the
    // pre-shifted L[p] = Sh[p-1], undone here with one DPP). Each cell is therefore converted
    // once per direction, and these waves issue no global loads at all: their only vector
    // memory instructions are the gradient stores. The converters keep a slot until the
    // gradient waves of its row have read it (help counters).
    auto row_of = [&](int i) {
      const int r = hb + h + kNH * i;
      return d == 0 ? r : S - 1 - r;
    };
    // ---- Z at the cut: tree-sum over p of alpha[M][p] * beta[M][p] (fixed order, = oracle)
    if (d == 0 && h == 0) {
      const unsigned tag = a.loss_sum ? sum_tag(a) : 0u;  // (load in flight while waiting)
      spin_until<true>([&] { return ctr_acq(&ctl->a_ready); }, 1, a.status, dg);
      spin_until<true>([&] { return ctr_acq(&ctl->bm_ready); }, 1, a.status, dg);
      const XRow<K> Am = row_ld(M);
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
        if (DBG && a.z_state) {
          a.z_state[2 * b] = z.m;
          a.z_state[2 * b + 1] = __builtin_bit_cast(float, z.e);
        }
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

    // Rows are software-pipelined: row i+1's LDS reads are issued before row i's arithmetic
    // whenever the chain is already known to be past row i+1 (the steady state -- these waves
    // trail the chain), so a row costs its arithmetic, not an LDS round trip.
    struct GIn {
      XRow<K> A, Bn, Bs, E, Sh, O;
    };
    int chain_seen = 0;
    auto need_of = [&](int i) {  // fwd: alpha[s] is written after chain stream row s-1;
      const int r = hb + h + kNH * i;  // bwd: beta[s] at stream row r
      return d == 0 ? r : r + 1;
    };
    auto wait_chain = [&](int i) {
      const int need = need_of(i);
      if (chain_seen < need)
        chain_seen = spin_until<true>([&] { return ctr_ld(&ctl->chain[d]); }, need, a.status, dg);
      cbar();
    };
    auto fetch = [&](int i, GIn& in) {
      const int r = hb + h + kNH * i;  // stream row
      const int s = row_of(i);         // transition / lattice row
      const unsigned char* sl = inr + (size_t)(d * R + r % R) * slot_bytes;  // factors of row r
      float v[4 * K];
#pragma unroll
      for (int q = 0; q < K; ++q)
        ld_vec<4>(v + 4 * q, reinterpret_cast<const float*>(sl + (size_t)q * nl16 + 16 * (pr / K)));
#pragma unroll
      for (int q = 0; q < K; ++q) {
        in.E.m[q] = v[4 * q];
        in.E.e[q] = __builtin_bit_cast(int, v[4 * q + 1]);
        in.Sh.m[q] = v[4 * q + 2];
        in.Sh.e[q] = __builtin_bit_cast(int, v[4 * q + 3]);
      }
      if constexpr (OBS) in.O = lds_xrow<K>(reinterpret_cast<const xf*>(sl + 16 * Up) + pr);
      if (d == 0) {
        in.A = (s == M) ? row_ld(M) : lds_xrow<K>(outr + (size_t)(s % kR2) * Up + pr);
        in.Bn = row_ld(min(s + 1, S - 1));  // (terminal transition: unused)
        if (OBS || lb) in.Bs = (s == M) ? lds_xrow<K>(cutb + pr) : row_ld(s);
      } else {
        in.A = row_ld(s);  // beta[s] is ring row r % kR2 (r = S-1-s), beta[s+1] ring row (r-1)
        in.Bn = (s + 1 == M) ? lds_xrow<K>(cutb + pr) : lds_xrow<K>(outr + (size_t)(kR2 + (r - 1) % kR2) * Up + pr);
        if (OBS || lb) in.Bs = lds_xrow<K>(outr + (size_t)(kR2 + r % kR2) * Up + pr);
      }
#ifdef SSNT_DIAG
      tag_check(&ctl->ctag[d][r % R], r, a.status);
      if (d == 0) {
        if (s != M) tag_check(&ctl->rtag[0][s % kR2], s, a.status);
      } else {
        if (s + 1 != M) tag_check(&ctl->rtag[1][(r - 1) % kR2], r - 1, a.status);
        if ((OBS || lb) && s != M) tag_check(&ctl->rtag[1][r % kR2], r, a.status);
      }
#endif
      cbar();
      ctr_st(&ctl->help[d][h], i + 1);  // ring rows read (in-order DS): reusable
    };
    auto emit = [&](int i, const GIn& in) {
          const int s = row_of(i);
          const XRow<K>& A = in.A;
          const XRow<K>& Bn = in.Bn;
          const XRow<K>& Bs = in.Bs;
          const XRow<K>& E = in.E;
          const XRow<K>& O = in.O;
          XRow<K> Sh = in.Sh;
          float ge[2 * K], gob[K];
          if (zero_z) {
#pragma unroll
            for (int q = 0; q < K; ++q) {
              ge[2 * q] = 0.0f;
              ge[2 * q + 1] = 0.0f;
              gob[q] = 0.0f;
            }
          } else {
            if (d == 0) {  // Sh[p] = L[p+1]; masked (exact zero) for p >= P-1 (src/lib.rs:196-205)
              XRow<K> L = Sh;
#pragma unroll
              for (int q = 0; q < K; ++q) {
                const float lm = (q == K - 1) ? shl_z(L.m[0]) : L.m[q + 1 < K ? q + 1 : 0];
                const int le = (q == K - 1) ? shl_z(L.e[0]) : L.e[q + 1 < K ? q + 1 : 0];
                const bool live = p0 + q < P - 1;
                Sh.m[q] = live ? lm : 0.0f;
                Sh.e[q] = live ? le : XF_EZERO;
              }
            }
            XRow<K> Q, Rr;
            if (s + 1 < S) {
#pragma unroll
              for (int q = 0; q < K; ++q) {
                Q.m[q] = OBS ? Bn.m[q] * O.m[q] : Bn.m[q];
                Q.e[q] = OBS ? Bn.e[q] + O.e[q] : Bn.e[q];
              }
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
              if constexpr (OBS) gob[q] = xf_neg_post((A.m[q] * Bs.m[q]) * izm, ae + Bs.e[q]);
            }
          }
          if (g) SSNT_GST2(ge, g, s);
          if constexpr (OBS) {
            if (go) gst<K, 1, NV>(gob, brsrc(go + (size_t)s * U, U * 4u), p0);
          }
          if (DBG && (la || lb)) {  // debug outputs (the DBG instance only)
            float va[K], vb[K], ea[K], eb[K];
#pragma unroll
            for (int q = 0; q < K; ++q) {
              const xf na = xf_norm(A.m[q], A.e[q]);  // (lazy rows)
              const xf nb = xf_norm(Bs.m[q], Bs.e[q]);
              const bool raw = a.log_alpha_e != nullptr;  // raw state: mantissa + exponent plane
              va[q] = zero_z ? (raw ? 0.0f : -__builtin_inff()) : raw ? na.m : xf_log(na);
              vb[q] = zero_z ? (raw ? 0.0f : -__builtin_inff()) : raw ? nb.m : xf_log(nb);
              ea[q] = __builtin_bit_cast(float, na.e);
              eb[q] = __builtin_bit_cast(float, nb.e);
            }
            if (la) gst<K, 1, NV>(va, brsrc(la + (size_t)s * U, U * 4u), p0);
            if (lb) gst<K, 1, NV>(vb, brsrc(lb + (size_t)s * U, U * 4u), p0);
            if (lae) gst<K, 1, NV>(ea, brsrc(lae + (size_t)s * U, U * 4u), p0);
            if (lbe) gst<K, 1, NV>(eb, brsrc(lbe + (size_t)s * U, U * 4u), p0);
          }
    };
    auto row = [&](int i, GIn& cur, GIn& nxt) {
      const bool more = i + 1 < nmine;
      const bool early = more && chain_seen >= need_of(i + 1);
      if (early) fetch(i + 1, nxt);
      emit(i, cur);
      if (more && !early) {
        wait_chain(i + 1);
        fetch(i + 1, nxt);
      }
    };
    GIn gin0, gin1;  // alternating buffers (no register copies of rows with reads in flight)
    if (nmine > 0) {
      wait_chain(0);
      fetch(0, gin0);
    }
    for (int i = 0; i < nmine; i += 2) {
      row(i, gin0, gin1);
      if (i + 1 < nmine) row(i + 1, gin1, gin0);
    }
    dg.flush(b, role.slot);
    return;
  }

  if (role.kind == 1) {
    // =============================== converters ==========================================
    const int d = role.d;
    const int c = role.idx;
    constexpr int D = conv_depth<K>();
    const unsigned tag0 = (d == 0 && c == 0 && b == 0 && a.loss_sum) ? sum_tag(a) : 0u;
    const int chain_end = d == 0 ? S - 1 : S;
    unsigned char* ring = inr + (size_t)d * R * slot_bytes;
    auto load = [&](int r, Item<K, OBS>& it) {
      const int row = min(max(d == 0 ? r : S - 1 - r, 0), T - 1);
      gld<K, 2, NV>(it.lt, brsrc(lt + (size_t)row * U * 2, U * 8u), p0);
      if constexpr (OBS) {
        const int orow = min(row + 1, T - 1);
        gld<K, 1, NV>(it.ob, brsrc(lo + (size_t)orow * U, U * 4u), p0);
      }
    };
    Item<K, OBS> pf[D];
#pragma unroll
    for (int i = 0; i < D; ++i) load(c + kNC * i, pf[i]);
    int seen_chain = 0;
    const int hb = d == 0 ? M : S - M;  // first stream row the gradient waves read
    int seen_grad = hb;
    const int nmine = (S - c + kNC - 1) / kNC;  // my stream rows: c, c + kNC, ...
    for (int base = 0; base < nmine; base += D) {
#pragma unroll
      for (int i = 0; i < D; ++i) {
        const int k = base + i;
        if (k < nmine) {
          const int r = c + kNC * k;
          const Item<K, OBS>& it = pf[i];
          XRow<K> E, Sh, O;
#ifdef SSNT_DIAG
          const unsigned long long tl0 = dg.now();
          asm volatile("" :: "v"(it.lt[0]), "v"(it.lt[2 * K - 1]));  // wait for the row here
          const unsigned long long tc0 = dg.now();
          dg.ph[2] += tc0 - tl0;
#endif
          convert<K, OBS>(it, P, lane, E, Sh);
          convert_obs<K, OBS>(it, P, lane, O);
#ifdef SSNT_DIAG
          asm volatile("" :: "v"(E.m[0]), "v"(E.e[0]), "v"(Sh.m[K - 1]), "v"(Sh.e[K - 1]));
          dg.ph[0] += dg.now() - tc0;
#endif
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
          // slot r % R last held row q = r - R: the chain and the gradient waves must be done
          const int q = r - R;  // (read by the chain, and by the gradient waves from row hb on)
          if (q >= 0) {
            const int need_c = min(q + 1, chain_end);
            if (seen_chain < need_c)
              seen_chain = spin_until<true>([&] { return ctr_ld(&ctl->sread[d]); }, need_c, a.status, dg);
            if (q >= hb && seen_grad <= q)
              seen_grad = spin_until<true>([&] { return first_missing<kNH>(ctl->help[d], hb); }, q + 1, a.status, dg);
          }
          cbar();
#ifdef SSNT_DIAG
          const unsigned long long tw0 = dg.now();
#endif
          unsigned char* sl = ring + (size_t)(r % R) * slot_bytes;
          float v[4 * K];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            v[4 * j] = E.m[j];
            v[4 * j + 1] = __builtin_bit_cast(float, E.e[j]);
            v[4 * j + 2] = Xs.m[j];
            v[4 * j + 3] = __builtin_bit_cast(float, Xs.e[j]);
          }
          // planar by element: block q holds (E, X) of positions K*l + q at 16*l -- every
          // 16-byte lane access is contiguous across the wave (no bank conflicts)
#pragma unroll
          for (int q = 0; q < K; ++q)
            st_vec<4>(reinterpret_cast<float*>(act ? sl + (size_t)q * nl16 + 16 * lane : junk_lane + 16 * q), v + 4 * q);
          if constexpr (OBS) {
            float o[2 * K];
            xrow_pack<K>(O, o);
            st_vec<2 * K>(reinterpret_cast<float*>(act ? sl + 16 * Up + 8 * p0 : junk_lane), o);
          }
#ifdef SSNT_DIAG
          tag_put(&ctl->ctag[d][r % R], r + kTagFault);
#endif
          cbar();
          ctr_st(&ctl->conv[d][c], k + 1);
#ifdef SSNT_DIAG
          dg.ph[1] += dg.now() - tw0;
#endif
        }
        // refill after the old item is consumed: same registers, no copy (a copy of a register
        // with a load in flight would wait for the load)
        load(c + kNC * (k + D), pf[i]);
      }
    }
    dg.flush(b, role.slot);
    fill_rows(S, d * kNC + c, 2 * kNC);  // zero the rows beyond S
    // workgroup 0 forms the batch loss sum once every utterance has published its loss (all
    // did so at their cut, long before this converter runs out of rows)
    if (d == 0 && c == 0 && b == 0 && a.loss_sum) finish_loss_sum(a, tag0);
    return;
  }

  // ================================== chains =============================================
  // Unrolled blocks of R steps aligned to R (slot offsets are compile-time); blocks that lie
  // inside one phase run without per-step guards. Factors for row r+PF are read into row r's
  // register buffer as soon as row r is done, so PF-1 steps hide the LDS latency (PF = 4 was
  // tried: no faster before the cut, slower after it -- less ring slack; so was issuing the
  // read of row r+3 into a dead buffer before the step's arithmetic, which does keep three reads
  // in flight in the .s: before the cut a step still costs ~300 cycles, so the LDS latency is
  // not what bounds it; nor do the converter polls -- with them skipped (timing experiment) a
  // step before the cut also takes ~300 cycles). All LDS
  // addresses are per-lane pointers prepared before the loop (lanes past U: junk / clamped).
  __builtin_amdgcn_s_setprio(3);
  const int d = role.d;
  int ready = 0;  // stream rows known converted
  auto wait_row = [&](int r) {  // r: a row that exists
    if (r >= ready)
      ready = spin_until<false>([&] { return first_missing<kNC>(ctl->conv[d], 0); }, r + 1, a.status, dg);
  };
  const unsigned char* sptr[R];  // slot j, this lane's factors (element block 0)
#pragma unroll
  for (int j = 0; j < R; ++j) sptr[j] = inr + (size_t)(d * R + j) * slot_bytes + 16 * (pr / K);
  xf* optr[kR2];  // chain-row ring row j, this lane (junk past U)
#pragma unroll
  for (int j = 0; j < kR2; ++j)
    optr[j] = act ? outr + (size_t)(d * kR2 + j) * Up + p0 : reinterpret_cast<xf*>(junk_lane);
  // slot j's factors (row: the stream row it should hold; check: a row the chain uses)
  auto rd = [&](int j, XRow<K>& E, XRow<K>& Xx, XRow<K>& O, int row = 0, bool check = false) {
    (void)row;
    (void)check;
    float v[4 * K];
#pragma unroll
    for (int q = 0; q < K; ++q) ld_vec<4>(v + 4 * q, reinterpret_cast<const float*>(sptr[j] + (size_t)q * nl16));
#pragma unroll
    for (int q = 0; q < K; ++q) {
      E.m[q] = v[4 * q];
      E.e[q] = __builtin_bit_cast(int, v[4 * q + 1]);
      Xx.m[q] = v[4 * q + 2];
      Xx.e[q] = __builtin_bit_cast(int, v[4 * q + 3]);
    }
    if constexpr (OBS) {
      O = lds_xrow<K>(reinterpret_cast<const xf*>(sptr[j] - 16 * (pr / K) + 16 * Up) + pr);
    } else {
#pragma unroll
      for (int q = 0; q < K; ++q) {
        O.m[q] = 1.0f;
        O.e[q] = 0;
      }
    }
#ifdef SSNT_DIAG
    if (check) tag_check(&ctl->ctag[d][j], row, a.status);
#endif
  };
  constexpr int PF = kChainPrefetch<OBS>(R);  // rows of factors in flight per chain
  static_assert(R % PF == 0 && PF < R, "prefetch buffers tile the ring");
  XRow<K> Eb[PF], Xb[PF], Ob[PF];
  // Steps run in half-blocks of H = R/2 (unrolled by R: slot offsets compile-time). All waits
  // -- converted rows up to two past the half-block, ring rows released by the gradient waves --
  // happen at half-block boundaries, so the H steps in between are straight-line code and the
  // compiler's LDS wait counts stay exact. Progress is published at the end of each half-block
  // (the rings have the slack: a converter may run R rows ahead of the published progress).
  // Phase 2 (past the cut) publishes every H2 steps instead: there the gradient waves read each
  // factor slot right behind the chain and the converters need it back, so the hand-off
  // chain -> gradient waves -> converters -> chain has to close within the ring's slack.
  using H1 = std::integral_constant<int, (R >= 16 ? R / 4 : R / 2)>;
  using H2 = std::integral_constant<int, (R >= 16 ? R / 8 : (R / 4 > 2 ? R / 4 : 2))>;
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
            constexpr int j = decltype(J)::value;
            step(std::integral_constant<int, h0 + j>{}, base, hb0 + j >= lo && hb0 + j < hi);
          });
        }
        cbar();
        ctr_st(&ctl->chain[d], min(hb0 + HS, hi));
        ctr_st(&ctl->sread[d], min(hb0 + HS, hi) + PF);  // slot reads run PF rows ahead
      });
    }
  };
  if (d == 0) {
    // ---------------- alpha chain: stream row r = transition r -> alpha[r+1] --------------
    const int n = S - 1;
    const int last = max(n - 1, 0);  // last stream row the chain reads
    wait_row(min(PF - 1, last));
    cbar();
    sfor<PF>([&](auto J) {
      constexpr int j = decltype(J)::value;
      rd(j, Eb[j], Xb[j], Ob[j], j, j <= last && n > 0);
    });
    int help_seen = M + 1;  // first alpha ring row not yet released by the gradient waves
    // storage write pointer for alpha[r+1] (LDS mode)
    xf* wp = act ? rows + (size_t)Up + p0 : reinterpret_cast<xf*>(junk_lane);
    const int wstep = act ? Up : 0;
    // steps [r0, r1): rows up to r1+1 converted; phase 2: ring rows up to r1-kR2 released
    auto hwait = [&](int r0, int r1, bool phase2) {
      (void)r0;
      wait_row(min(r1 - 1 + PF, last));
      if (phase2) {
        const int q = r1 - kR2;  // newest previous occupant the half-block overwrites
        if (q > M && help_seen <= q)
          help_seen = spin_until<false>([&] { return first_missing<kNH>(ctl->help[0], M); }, q + 1, a.status, dg);
      }
      cbar();
    };
    auto step = [&](auto Ic, int base, bool live, auto Ph) {
      constexpr int i = decltype(Ic)::value;
      constexpr int par = i % PF;
      constexpr bool phase2 = decltype(Ph)::value;
      if (!live) return;
      const int r = base + i;
      alpha_chain<K, OBS, (i % kChainNorm) == kChainNorm - 1>(X, Eb[par], Xb[par], Ob[par]);
      if constexpr (!phase2) {
        if constexpr (LDS) {
          lds_xrow_st<K>(wp, X);
          wp += wstep;
        } else {
          row_st(r + 1, X);
        }
      } else {
        lds_xrow_st<K>(optr[(i + 1) % kR2], X);
#ifdef SSNT_DIAG
        tag_put(&ctl->rtag[0][(i + 1) % kR2], r + 1);
#endif
      }
      rd((i + PF) % R, Eb[par], Xb[par], Ob[par], r + PF, r + PF <= last);  // row r+PF (a stale slot past the end is dropped)
    };
    if (M == 0) ctr_rel(&ctl->a_ready, 1);
    ctr_st(&ctl->sread[0], PF);  // slots of rows 0..PF-1 have been read
    run(H1{}, 0, M, [&](auto Ic, int base, bool live) { step(Ic, base, live, std::false_type{}); },
        [&](int r0, int r1) { hwait(r0, r1, false); });
    if (M > 0) {
      cbar();
      ctr_rel(&ctl->a_ready, 1);
      dg.mark_cut();
    }
    run(H2{}, M, n, [&](auto Ic, int base, bool live) { step(Ic, base, live, std::true_type{}); },
        [&](int r0, int r1) { hwait(r0, r1, true); });
  } else {
    // ---------------- beta chain: stream row r = transition S-1-r -> beta[S-1-r] ----------
    // beta rows past the cut (s < M) go to ring row r % kR2 (r = S-1-s)
    const int c = S - 1 - M;  // stream row of the cut (beta[M])
    const int last = S - 1;
    wait_row(min(PF, last));
    cbar();
    sfor<PF>([&](auto J) {
      constexpr int j = decltype(J)::value;
      rd(j, Eb[j], Xb[j], Ob[j], j, j <= last);
    });
    int help_seen = S - M;  // first beta gradient row (stream rows) not finished
    xf* wp = act ? rows + (size_t)(S - 1) * Up + p0 : reinterpret_cast<xf*>(junk_lane);  // beta[S-1-r]
    const int wstep = act ? Up : 0;
    // stream row r -> kind 0: storage row S-1-r; 1: cut buffer; 2: ring row r % kR2
    auto put = [&](int r, int i, auto Kd) {
      constexpr int kind = decltype(Kd)::value;
      if constexpr (kind == 0) {
        if constexpr (LDS) {
          lds_xrow_st<K>(wp, X);
        } else {
          row_st(S - 1 - r, X);
        }
      } else if constexpr (kind == 1) {
        lds_xrow_st<K>(act ? cutb + p0 : reinterpret_cast<xf*>(junk_lane), X);
        cbar();
        ctr_rel(&ctl->bm_ready, 1);
        dg.mark_cut();
      } else {
        lds_xrow_st<K>(optr[i % kR2], X);
#ifdef SSNT_DIAG
        tag_put(&ctl->rtag[1][i % kR2], r);
#endif
      }
      wp -= wstep;
    };
    auto hwait = [&](int r0, int r1, bool ring) {
      (void)r0;
      wait_row(min(r1 - 1 + PF, last));
      if (ring) {
        // previous occupants: stream rows up to r1-1-kR2, read by gradient rows q and q+1
        const int q = r1 - 1 - kR2;
        if (q > c && help_seen <= q + 1)
          help_seen = spin_until<false>([&] { return first_missing<kNH>(ctl->help[1], S - M); }, q + 2, a.status, dg);
      }
      cbar();
    };
#pragma unroll
    for (int j = 0; j < K; ++j) {  // beta[S-1]: terminal emit (src/lib.rs:187-195)
      const bool lastp = (p0 + j) == P - 1;
      const xf v = term ? xf_norm(Eb[0].m[j], Eb[0].e[j]) : xf{0.5f, 1};
      X.m[j] = lastp ? v.m : 0.0f;
      X.e[j] = lastp ? v.e : XF_EZERO;
    }
    if (c == 0) put(0, 0, std::integral_constant<int, 1>{});
    else put(0, 0, std::integral_constant<int, 0>{});
    cbar();
    rd(PF % R, Eb[0], Xb[0], Ob[0], PF, PF <= last);
    auto step = [&](auto Ic, int base, bool live, auto Kd) {
      constexpr int i = decltype(Ic)::value;
      constexpr int par = i % PF;
      if (!live) return;
      const int r = base + i;
      beta_chain<K, OBS, (i % kChainNorm) == kChainNorm - 1>(X, Eb[par], Xb[par], Ob[par]);
      put(r, i, Kd);
      rd((i + PF) % R, Eb[par], Xb[par], Ob[par], r + PF, r + PF <= last);
    };
    cbar();
    ctr_st(&ctl->chain[1], 1);  // stream row 0 (the terminal row) is done
    ctr_st(&ctl->sread[1], PF + 1);  // slots of rows 0..PF have been read
    run(H1{}, 1, c, [&](auto Ic, int base, bool live) { step(Ic, base, live, std::integral_constant<int, 0>{}); },
        [&](int r0, int r1) { hwait(r0, r1, false); });
    if (c >= 1)
      run(H1{}, c, c + 1, [&](auto Ic, int base, bool live) { step(Ic, base, live, std::integral_constant<int, 1>{}); },
          [&](int r0, int r1) { hwait(r0, r1, false); });
    run(H2{}, c + 1, S, [&](auto Ic, int base, bool live) { step(Ic, base, live, std::integral_constant<int, 2>{}); },
        [&](int r0, int r1) { hwait(r0, r1, true); });
  }
  dg.flush(b, role.slot);
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
inline bool aligned_to(const void* p, uintptr_t m) { return (reinterpret_cast<uintptr_t>(p) & (m - 1)) == 0; }

template <int K, bool OBS, bool LDS, int NC, int NH, int RS, bool NV>
int launch_stream_kernel(const FwdBwdArgs& a, size_t lds, hipStream_t st) {
  const bool dbg = a.log_alpha || a.log_beta;
  auto kern = dbg ? k_fwd_bwd_stream<K, OBS, LDS, NC, NH, RS, NV, true>
                  : k_fwd_bwd_stream<K, OBS, LDS, NC, NH, RS, NV, false>;
  note_fwd_bwd_dispatch("k_fwd_bwd_stream<K=%d,OBS=%d,LDS=%d,NC=%d,NH=%d,RS=%d,NV=%d%s>", K, (int)OBS,
                        (int)LDS, NC, NH, RS, (int)NV, dbg ? ",DBG" : "");
  // dynamic LDS above 64 KiB needs the attribute; it is per device, so it is set on every such
  // launch (a host-side call, no device work) rather than cached in a process-wide flag
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBudget);
  hipLaunchKernelGGL(kern, dim3(a.B), dim3(64 * (2 + 2 * NC + 2 * NH)), lds, st, a);
  return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
}

template <int K, bool OBS, int NC, int NH, int RS = 0>
int launch_stream_k(const FwdBwdArgs& a, hipStream_t st, bool force_ws = false) {
  // whole lane slices and 16-byte aligned tensors: the vector form; else (U % K != 0, or
  // tensors at 4-byte alignment) the narrow form: one 8-byte access per (emit, shift) position,
  // which buffer loads and stores take at any dword alignment (a sliced log_trans / grad at an
  // odd float offset no longer drops to the two-wave kernel)
  const bool vec = (a.U % K == 0) && aligned16(a.log_trans) && aligned16(a.log_obs) &&
                   aligned16(a.grad) && aligned16(a.grad_obs) && aligned16(a.log_alpha) &&
                   aligned16(a.log_beta) && aligned16(a.workspace);
  const bool narrow_ok = aligned_to(a.log_trans, 4) && aligned_to(a.grad, 4) && aligned16(a.workspace) &&
                         aligned_to(a.log_obs, 4) && aligned_to(a.grad_obs, 4) &&
                         aligned_to(a.log_alpha, 4) && aligned_to(a.log_beta, 4);
  if (!vec && !narrow_ok) return SSNT_ERR_UNSUPPORTED;
  const int Up = K * ((a.U + K - 1) / K);
  const size_t head = stream_head_bytes(K, a.U, OBS, RS);
  if (head > kLdsBudget) return SSNT_ERR_UNSUPPORTED;
  const size_t rows = (size_t)a.T * (vec ? a.U : Up) * sizeof(xf);
  const bool lds = !force_ws && head + rows <= kLdsBudget;
  if (!lds && (a.workspace == nullptr || a.workspace_bytes < (size_t)a.B * rows))
    return SSNT_ERR_WORKSPACE;
  if (vec)
    return lds ? launch_stream_kernel<K, OBS, true, NC, NH, RS, false>(a, head + rows, st)
               : launch_stream_kernel<K, OBS, false, NC, NH, RS, false>(a, head, st);
  return lds ? launch_stream_kernel<K, OBS, true, NC, NH, RS, true>(a, head + rows, st)
             : launch_stream_kernel<K, OBS, false, NC, NH, RS, true>(a, head, st);
}

#ifdef SSNT_AB
std::atomic<int> g_ring{0};  // A/B build: 0 default rings; 16 / 32 ring slots with workspace rows (K = 2)
#endif

template <bool OBS>
int launch_stream_obs(const FwdBwdArgs& a, hipStream_t st) {
  // wave mix per lane width: 16 waves (3 converters + 4 gradient waves per direction) while a
  // wave fits 128 VGPRs (K <= 2); 10 waves for K >= 4 (168 VGPRs, no spills)
  if (a.U <= 64) return launch_stream_k<1, OBS, 3, 4>(a, st);
#ifdef SSNT_AB
  if constexpr (!OBS) {  // A/B build (ssnt_fwd_bwd_stream_ring): deeper rings, rows in the workspace
    const int ring = g_ring.load(std::memory_order_relaxed);
    if (a.U > 64 && a.U <= 128 && ring == 16) return launch_stream_k<2, false, 3, 4, 16>(a, st, true);
    if (a.U > 64 && a.U <= 128 && ring == 32) return launch_stream_k<2, false, 3, 4, 32>(a, st, true);
  }
#endif
  if (a.U <= 128) return launch_stream_k<2, OBS, 3, 4>(a, st);
  if (a.U <= 256) return launch_stream_k<4, OBS, 2, 2>(a, st);
  // K = 8 (U <= 512, configs[4]): the two-wave kernel. The streaming kernel needs 4-slot rings to
  // fit LDS there and then ran 2.2x slower (5.7 vs 2.6 ms at B=64 T=2000 U=400).
  return SSNT_ERR_UNSUPPORTED;
}

}  // namespace

int diag_read(void* host, size_t bytes) {
#ifdef SSNT_DIAG
  if (bytes > sizeof(g_diag)) bytes = sizeof(g_diag);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? (int)bytes : -1;
#else
  (void)host;
  (void)bytes;
  return -1;
#endif
}

size_t stream_head_bytes(int K, int U, bool obs, int ring) {
  const int R = ring ? ring : obs ? in_slots<true>() : in_slots<false>();
  const int R2o = obs ? out_slots<true>() : out_slots<false>();
  const int R2 = R2o < R ? R2o : R;
  const size_t Up = (size_t)K * ((U + K - 1) / K);  // (= U when U % K == 0)
  const size_t slot = (Up * 16 + (obs ? Up * 8 : 0) + 15) & ~(size_t)15;
  return kCtlBytes + (size_t)64 * K * sizeof(xf) + (size_t)64 * 16 * K + 2 * (size_t)R * slot +
         2 * (size_t)R2 * Up * sizeof(xf);
}

int launch_fwd_bwd_stream(const FwdBwdArgs& a, hipStream_t st) {
  return a.log_obs ? launch_stream_obs<true>(a, st) : launch_stream_obs<false>(a, st);
}

#ifdef SSNT_AB
int set_stream_ring(int r) {
  if (r != 0 && r != 16 && r != 32) return SSNT_ERR_INVALID_ARG;
  g_ring.store(r);
  return SSNT_OK;
}
int stream_ring() { return g_ring.load(std::memory_order_relaxed); }
#endif

}  // namespace ssnt
