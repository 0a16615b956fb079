// v2_fwd_bwd.hip -- F4: the v2 duration-class (semi-Markov) forward-backward for gfx950.
//
// The training-side counterpart of the v2 decode (not in the reference). The
// lattice, its move rules (src/v2.rs:94-166) and the split-exponent arithmetic are defined in
// oracle/ssnt_oracle.c ("F4") and DESIGN.md "Duration lattice"; this kernel reproduces that
// definition bit for bit.
//
// Layout. alpha does not depend on beta or the other way round, so the two sweeps run at the
// same time: launch 1 has one workgroup (512 threads, 8 waves) per (utterance, direction).
// State rows r = 0..I (input steps consumed) over totals x; only the window of row r
// (f4_window: the v2 band, or [0, r*dmax] in test mode) can hold mass, so rows are stored
// window-relative, Wcap xf wide:
//   LDS:  duration table | class weights (xf, chunks of 64 steps, double-buffered) | 2 row
//         buffers (ping-pong), each with kF4Pad zero cells on both sides of its window
//   HBM:  alpha and beta rows 0..I of every utterance (workspace), Z per utterance.
// A sweep step: each thread owns cells x = lo + tid (+512 ...) and sums its D class terms
// (exponent max, then the ldexp-aligned f32 sum in class order; the class loop is unrolled for
// D <= 64, the step's weights read into registers once); one barrier per step. With the zero
// cells around every window, a term's LDS address is one subtraction from its cell's (the
// clamp to the window happens once per cell, not per term). Class log-probs are loaded a
// chunk ahead and converted into LDS half a chunk later, so no global load and no exp sits on
// the I-step dependency chain. The forward workgroup also forms Z (lane partials x mod 64 +
// butterfly) and the loss.
// Launch 2 (one workgroup per (utterance, step)): the gradients of step t -- class i on wave
// i % 4, every class of a wave accumulated in one pass over the destination totals (lane
// partial x mod 64, the oracle's order), one butterfly per class (DPP quad/mirror moves, a
// swizzle, one bpermute) -- and the debug beta row. Fully parallel (B * I workgroups).
#include <hip/hip_runtime.h>
#include <limits.h>

#include "buffer_ops.h"
#include "ssnt_internal.h"
#include "xf_math.h"

namespace ssnt {
namespace {

constexpr int kF4Threads = 512;

__device__ __forceinline__ int f4_f2i(float x) {  // Rust `f32 as i32` (saturating, NaN -> 0)
  if (x != x) return 0;
  if (x >= 2147483648.0f) return 2147483647;
  if (x <= -2147483648.0f) return (-2147483647 - 1);
  return (int)x;
}

struct F4Utt {
  int I, O, X, dmax;
  bool test;
};

// cells of row r that can hold mass: [lo, hi] (empty when lo > hi); = oracle f4_window
__device__ __forceinline__ void f4_window(const F4Utt& u, int r, int& lo, int& hi) {
  if (r == 0) {
    lo = 0;
    hi = 0;
    return;
  }
  if (u.test) {
    const long long h = (long long)r * u.dmax;
    lo = 0;
    hi = h < u.X - 1 ? (int)h : u.X - 1;
    return;
  }
  const int t = r - 1;
  if ((long long)(u.I - (t + 1)) * 3 > u.O) {  // will_overrun (src/v2.rs:106-111)
    lo = 1;
    hi = 0;
    return;
  }
  const float diagonal = (float)u.O / (float)u.I * (float)(t + 1);  // src/v2.rs:94-104
  const float upper_range = (float)u.O * 0.1f;
  const float lower_range = (float)u.O * 0.05f;
  int lb = f4_f2i(fmaxf(diagonal - lower_range, 0.0f));
  int ub = f4_f2i(fminf(diagonal + upper_range, (float)u.O));
  if (t == u.I - 1) {  // src/v2.rs:135-137
    lb = max(lb, u.O);
    ub = min(ub, u.O);
  }
  lo = max(lb, 0);
  hi = min(ub, u.X - 1);
}

// debug row: ln of the window cells, -inf elsewhere (row == nullptr: all -inf)
__device__ __forceinline__ void f4_log_row(float* dst, const xf* row, int lo, int hi, int X) {
  for (int x = threadIdx.x; x < X; x += kF4Threads)
    dst[x] = (row && x >= lo && x <= hi) ? xf_log(row[x - lo]) : -__builtin_inff();
}

// one cell: sum over classes of src[x -/+ d_i] (x) w[i] (oracle f4_cell_sum). FWD: alpha
// (source total x - d_i, product a.m * w.m); else beta (x + d_i, w.m * b.m). Classes padded to
// DC = next power of two >= D with w = 0 and duration 0 (exact zero terms, as the oracle's
// padding), so the 2 DC LDS reads of a cell issue back to back and the sum is the oracle's
// pairwise tree (depth log2 DC instead of a DC-long add chain). srcw is the source row's window
// cell 0; every cell a term can reach outside the window holds the canonical zero (0, XF_EZERO):
// an exact zero term, as the oracle's skip.
//  PADDED (dmax <= kF4Pad): the row buffers carry kF4Pad zero cells on both sides of the window,
//   and the caller clamps xr = x - slo into the band from which every term stays inside them, so
//   a term's address is ONE subtraction from the cell's (8 d_i, hoisted out of the step loop).
//  else: offsets are taken +1, so anything left of the window wraps to a huge unsigned value,
//   and one unsigned min clamps an out-of-window term onto the zero cell just right of the window
//   (index span + 1); offset 0 is the zero cell left of it (index -1).
template <bool FWD, int DC, bool PADDED>
__device__ __forceinline__ xf f4_cell(int xr, const int (&dk)[DC], const xf* w, const xf* srcw, int span) {
  float m[DC];
  int e[DC];
  int em = XF_EZERO;
  // opaque: otherwise the compiler reassociates the cell offset with the uniform durations into
  // 2 DC uniform sums in SGPRs, which overflows the SGPR file into lane spills every step
  int xb = PADDED ? xr : xr + 1;
  asm volatile("" : "+v"(xb));
  const xf* px = srcw + xb;  // PADDED: the cell's own source cell
  const unsigned lim = (unsigned)(span + 2);
#pragma unroll
  for (int i = 0; i < DC; ++i) {
    xf v;
    if constexpr (PADDED) {
      v = px[FWD ? -dk[i] : dk[i]];
    } else {
      const unsigned yr1 = (unsigned)(FWD ? xb - dk[i] : xb + dk[i]);
      v = srcw[(int)min(yr1, lim) - 1];
    }
    const xf ww = w[i];
    m[i] = FWD ? v.m * ww.m : ww.m * v.m;
    e[i] = v.e + ww.e;
    em = max(em, e[i]);
  }
#pragma unroll
  for (int i = 0; i < DC; ++i) m[i] = xldexp(m[i], e[i] - em);
#pragma unroll
  for (int len = DC; len > 1; len >>= 1) {
#pragma unroll
    for (int i = 0; i < len / 2; ++i) m[i] = m[2 * i] + m[2 * i + 1];
  }
  return xf_norm(m[0], em);
}

// workgroup barrier ordering LDS only: __syncthreads() would also wait for every global store
// in flight (vmcnt(0)), i.e. one HBM write round trip per sweep step; nothing in these kernels
// reads back global memory written in the same launch
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int CTRL>
__device__ __forceinline__ xf dpp_xf(xf v) {
  return xf{__builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v.m), CTRL, 0xf, 0xf, false)),
            __builtin_amdgcn_update_dpp(0, v.e, CTRL, 0xf, 0xf, false)};
}
__device__ __forceinline__ xf f4_add(xf a, xf b) { return xf_add(a.m, a.e, b.m, b.e); }

// xor butterfly over the 64 lane partials, = the oracle's xor 1, 2, 4, ..., 32 (xf_add is
// commutative, so every lane ends equal). Once a quad (8-group) is uniform, the half-mirror
// (mirror) partner holds the xor-4 (xor-8) partner's value, so those two levels are DPP moves.
// Whole wave active (no divergent caller).
__device__ __forceinline__ xf f4_butterfly(xf acc) {
  acc = f4_add(acc, dpp_xf<0xB1>(acc));   // quad_perm [1,0,3,2]: xor 1
  acc = f4_add(acc, dpp_xf<0x4E>(acc));   // quad_perm [2,3,0,1]: xor 2
  acc = f4_add(acc, dpp_xf<0x141>(acc));  // row_half_mirror: xor 4
  acc = f4_add(acc, dpp_xf<0x140>(acc));  // row_mirror: xor 8
  acc = f4_add(acc, xf{__builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, acc.m), 0x401F)),
                       __builtin_amdgcn_ds_swizzle(acc.e, 0x401F)});  // xor 16
  acc = f4_add(acc, xf{__shfl_xor(acc.m, 32), __shfl_xor(acc.e, 32)});  // xor 32
  return acc;
}

// value of the lane at xor distance D (whole wave active): DPP quad permutes for 1 and 2, a
// ds_swizzle xor for 4..16, a bpermute for 32
template <int D>
__device__ __forceinline__ xf xor_xf(xf v) {
  if constexpr (D == 1) {
    return dpp_xf<0xB1>(v);
  } else if constexpr (D == 2) {
    return dpp_xf<0x4E>(v);
  } else if constexpr (D < 32) {
    return xf{__builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v.m), (D << 10) | 0x1F)),
              __builtin_amdgcn_ds_swizzle(v.e, (D << 10) | 0x1F)};
  } else {
    return xf{__shfl_xor(v.m, 32), __shfl_xor(v.e, 32)};
  }
}

// The xor butterfly of N classes' 64 lane partials at once, transposed: at distance 1, 2, ...,
// N/2 a lane keeps half of the classes it still holds (the lower half if its distance bit is 0)
// and adds its partner's partial of each, so N classes cost N/2 + N/4 + ... + 1 adds instead of
// N per level; past N/2 each lane holds one class and the plain butterfly finishes it. Every
// sum is the oracle's f4_butterfly tree node for that class (xf_add is commutative), so the
// result is bit-identical. Returns the class index (0..N-1) this lane's acc[0] holds; lanes
// 0..N-1 hold distinct classes.
template <int N, int Dist = 1>
__device__ __forceinline__ int f4_reduce_classes(xf (&acc)[N], int lane, int cls = 0) {
  if constexpr (Dist >= 64) {
    return cls;
  } else {
    constexpr int n = N / Dist;  // classes still in hand (1 once Dist >= N)
    if constexpr (n > 1) {
      const bool up = (lane & Dist) != 0;
#pragma unroll
      for (int i = 0; i < n / 2; ++i) {
        const xf keep = up ? acc[n / 2 + i] : acc[i];
        const xf give = up ? acc[i] : acc[n / 2 + i];
        acc[i] = f4_add(keep, xor_xf<Dist>(give));
      }
      cls += up ? n / 2 : 0;
    } else {
      acc[0] = f4_add(acc[0], xor_xf<Dist>(acc[0]));
    }
    return f4_reduce_classes<N, Dist * 2>(acc, lane, cls);
  }
}

// per-utterance state both kernels derive the same way; false: no lattice (loss written by
// the forward sweep, every output row zero / -inf)
__device__ __forceinline__ bool f4_setup(const V2FwdBwdArgs& a, int b, const int* dur, F4Utt& u,
                                         bool report) {
  u.I = a.input_length[b];
  u.O = a.output_length[b];
  u.X = a.X;
  u.test = a.test_mode;
  u.dmax = 0;
  bool neg = false;
  for (int i = 0; i < a.D; ++i) {
    u.dmax = max(u.dmax, dur[i]);
    neg |= dur[i] < 0;
  }
  const bool bad_len = u.I < 0 || u.I > a.Imax || u.O < 0;
  if (report && (bad_len || neg) && threadIdx.x == 0 && a.status)
    atomicOr(a.status, neg ? kStatusBadIndex : kStatusBadLength);
  // band mode with O > max_total: the final total can never equal O (src/v2.rs:135-137), so the
  // lattice is empty (= oracle f4_one); its windows could also exceed the band-sized Wcap
  const bool beyond = !u.test && u.O > u.X - 1;
  return !(bad_len || neg || u.I == 0 || beyond);
}

// workspace: alpha rows [B][Imax+1][Wc] | beta rows [B][Imax+1][Wc] | Z [B]
struct F4Ws {
  xf *alpha, *beta, *z;
};
__device__ __forceinline__ F4Ws f4_ws(const V2FwdBwdArgs& a) {
  xf* base = reinterpret_cast<xf*>(a.workspace);
  const size_t rows = (size_t)a.B * (a.Imax + 1) * a.Wcap;
  return F4Ws{base, base + rows, base + 2 * rows};
}

constexpr int kF4Pad = 64;  // zero cells either side of a row window (PADDED: dmax <= kF4Pad)
// sweep steps per staged chunk of class weights
template <int DC>
constexpr int f4_chunk() { return DC <= 32 ? 64 : 32; }

// One direction's sweep (FWD: alpha rows 0..I upward, and Z / the loss; else beta rows I..0).
// LDS: durations | class weights [2][CH][DC] xf (a chunk of CH sweep steps, converted when staged)
//      | row buffers [2][Wc + 2 kF4Pad + 2] xf (window cell j at kF4Pad + j; zeros around it)
// A step: each thread owns cells x = lo + tid (+512 ...) of the new row and sums its DC class
// terms from the previous row (f4_cell); one barrier per step. The class log-probs of chunk c + 1
// are loaded into registers when chunk c starts and converted into LDS half a chunk later, so
// no global load and no exp sits on the I-step dependency chain.
template <int DC, bool FWD, bool PADDED>
__device__ __forceinline__ void f4_sweep(const V2FwdBwdArgs& a, unsigned char* smem, const F4Utt& u,
                                         int dmax) {
  constexpr int CH = f4_chunk<DC>();
  constexpr int NPF = (CH * DC + kF4Threads - 1) / kF4Threads;  // staged values per thread
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D = a.D, X = a.X, Imax = a.Imax, Wc = a.Wcap;
  const int* dur = reinterpret_cast<const int*>(smem);
  xf* cw = reinterpret_cast<xf*>(smem + ((DC * 4 + 15) & ~15));  // [2][CH][DC]
  xf* row = cw + 2 * CH * DC;
  const int RS = Wc + 2 * kF4Pad + 2;
  auto rw = [&](int k) { return row + k * RS + kF4Pad; };  // buffer k's window cell 0
  const float* lg = a.logits + (size_t)b * Imax * D;
  const size_t drow = (size_t)(Imax + 1) * X;
  float* la = (FWD && a.log_alpha) ? a.log_alpha + b * drow : nullptr;
  const F4Ws W = f4_ws(a);
  xf* ws = (FWD ? W.alpha : W.beta) + (size_t)b * (Imax + 1) * Wc;
  const float inf_loss = (a.flags & SSNT_FLAG_ZERO_INFINITY) ? 0.0f : __builtin_inff();
  const int I = u.I;
  int dk[DC];  // term offsets (VGPRs: the SGPR file is full with addresses)
#pragma unroll
  for (int i = 0; i < DC; ++i) dk[i] = dur[i];
  auto st = [&](int k) { return FWD ? k : I - 1 - k; };  // input step of sweep step k
  float pre[NPF];
  // class log-probs through one descriptor: masked entries read past its end (zeros), so the
  // loads need no exec mask and no default writes into registers with loads in flight
  const __amdgpu_buffer_rsrc_t lg_r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(lg), (short)0, (int)((size_t)Imax * D * sizeof(float)), 0x00020000);
  auto load_chunk = [&](int c) {  // chunk c = sweep steps [c CH, (c + 1) CH): class log-probs
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      const int idx = tid + kF4Threads * j;
      const int k = c * CH + idx / DC, i = idx % DC;
      const bool live = idx < CH * DC && i < D && k < I;
      pre[j] = rbuf_ld1(lg_r, live ? (st(k) * D + i) * (int)sizeof(float) : (int)0x80000000, 0, 0);
    }
  };
  auto put_chunk = [&](int c) {  // ... converted into the chunk's LDS buffer
    xf* dst = cw + (c & 1) * CH * DC;
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      const int idx = tid + kF4Threads * j;
      const int i = idx % DC;
      if (idx < CH * DC) dst[idx] = i < D ? xf_exp(pre[j], a.allow_skip || i != a.zid) : xf_zero();
    }
  };
  // both row buffers zero (the cells around every window stay zero: see the step)
  for (int k = tid; k < 2 * RS; k += kF4Threads) row[k] = xf_zero();
  load_chunk(0);
  put_chunk(0);
  load_chunk(1);
  put_chunk(1);
  // first row: alpha[0] = 1 at total 0; beta[I] = 1 over window(I)
  int plo, phi;
  f4_window(u, FWD ? 0 : I, plo, phi);
  if (phi - plo + 1 > Wc) {
    if (tid == 0 && a.status) atomicOr(a.status, kStatusBadLength);
    return;
  }
  lds_sync();  // (zeros before the first row's cells)
  for (int k = tid; k <= phi - plo; k += kF4Threads) {
    rw(0)[k] = xf{0.5f, 1};
    ws[(size_t)(FWD ? 0 : I) * Wc + k] = xf{0.5f, 1};
  }
  lds_sync();
  if (la) f4_log_row(la, rw(0), 0, 0, X);
  // the utterance's workspace rows through one buffer descriptor (32-bit offsets: no 64-bit
  // address arithmetic per cell)
  const __amdgpu_buffer_rsrc_t ws_r = __builtin_amdgcn_make_buffer_rsrc(
      ws, (short)0, (int)((size_t)(Imax + 1) * Wc * sizeof(xf)), 0x00020000);
  // the windows of 64 consecutive steps, one per lane (lane l: the row of step 64 j + l), formed
  // once per block; a step reads the next step's window with two v_readlane instead of the
  // f32 band arithmetic and its branches (the same rule, f4_window, evaluated per lane)
  int wlo = 0, whi = 0;
  auto win_block = [&](int k0) {
    const int kk = k0 + lane;
    f4_window(u, FWD ? kk : I - kk, wlo, whi);
  };
  auto win_at = [&](int kk, int& l, int& h) {
    l = __builtin_amdgcn_readlane(wlo, kk & 63);
    h = __builtin_amdgcn_readlane(whi, kk & 63);
  };
  win_block(0);
  int lo, hi;  // window of the row the next step produces (formed before the barrier)
  win_at(1, lo, hi);
  // step k (1..I) produces row r = k (alpha) / I - k (beta) from the row of step k - 1 with the
  // class weights of sweep step k - 1; false: a window beyond the row capacity (reported)
  auto step = [&](int k) {
    const int r = FWD ? k : I - k;
    if (hi - lo + 1 > Wc) {  // host sizing bug: report, poison the loss (uniform branch)
      if (tid == 0) {
        if (a.status) atomicOr(a.status, kStatusBadLength);
        if (FWD) a.loss[b] = __builtin_nanf("");
      }
      return false;
    }
    const int ci = (k - 1) / CH, kk = (k - 1) - ci * CH;  // sweep step k - 1 in its chunk
    const xf* w = cw + (ci & 1) * CH * DC + kk * DC;
    const xf* srcw = rw((k - 1) & 1);
    xf* dst = rw(k & 1);
    const bool pe = phi >= plo;  // previous window non-empty
    const int slo = pe ? plo : 0;
    const int span = pe ? phi - plo : -1;
    // PADDED: cells whose every term lies outside the previous window are zero; the others have
    // xr = x - slo within [0, span + dmax] (alpha) / [-dmax, span] (beta), so every term's cell
    // lies within kF4Pad of the window
    const int xlo = PADDED ? (FWD ? 0 : -dmax) : INT_MIN, xhi = PADDED ? (FWD ? span + dmax : span) : INT_MAX;
    const int so = r * Wc * (int)sizeof(xf);
    // this step's weights into registers before the cell loop (read once, ahead of the cells'
    // row reads: measured 335 -> 323 us at configs[4] against reads inside the loop body)
    xf wh[DC];
#pragma unroll
    for (int i = 0; i < DC; ++i) wh[i] = w[i];
    for (int x = lo + tid; x <= hi; x += kF4Threads) {
      const int xr = x - slo;
      const int xc = min(max(xr, xlo), xhi);
      xf v = f4_cell<FWD, DC, PADDED>(xc, dk, wh, srcw, span);
      if (PADDED && (xr != xc || !pe)) v = xf_zero();
      dst[x - lo] = v;
      rbuf_st2(f32x2{v.m, __builtin_bit_cast(float, v.e)}, ws_r, (x - lo) * (int)sizeof(xf), so, 0);
    }
    // the cells right of the new window that the next step can reach: zero (a row two steps back
    // may have left values there). Wave 7's lanes: idle unless the window exceeds 448 cells.
    const int nz = PADDED ? dmax : 1;
    const int zi = tid - (kF4Threads - 64);
    if (zi >= 0 && zi < nz) dst[max(hi - lo + 1, 0) + zi] = xf_zero();
    plo = lo;
    phi = hi;
    if (k < I) {  // (before the barrier)
      if (((k + 1) & 63) == 0) win_block(k + 1);
      win_at(k + 1, lo, hi);
    }
    lds_sync();
    if (la) f4_log_row(la + (size_t)r * X, dst, plo, phi, X);
    return true;
  };
  // chunk c = sweep steps [c CH, (c + 1) CH) = steps k in [c CH + 1, (c + 1) CH]. The weights of
  // chunk c + 1 are loaded into registers as chunk c starts and put into LDS halfway through it
  // (their buffer's last reader, chunk c - 1, is done by then): one wait for global memory per
  // chunk, none inside a step (a load pending across steps would make every step wait for the
  // previous step's row stores, vmcnt counting both)
  for (int c = 0; c * CH < I; ++c) {
    const bool next = c >= 1 && (c + 1) * CH < I;  // (chunks 0 and 1 are in place)
    if (next) load_chunk(c + 1);
    const int kmid = min(c * CH + CH / 2, I), kend = min((c + 1) * CH, I);
    bool ok = true;
    for (int k = c * CH + 1; ok && k <= kmid; ++k) ok = step(k);
    if (!ok) return;
    if (next) put_chunk(c + 1);  // (the next step's barrier publishes it before its first reader)
    for (int k = kmid + 1; ok && k <= kend; ++k) ok = step(k);
    if (!ok) return;
  }
  if (!FWD) return;
  if (la)
    for (int r = I + 1; r <= Imax; ++r) f4_log_row(la + (size_t)r * X, nullptr, 0, -1, X);
  // Z over window(I): lane partials x mod 64, butterfly
  if (wave == 0) {
    xf acc = xf_zero();
    const xf* rI = rw(I & 1);
    for (int x = plo + ((lane - plo) & 63); x <= phi; x += 64) acc = f4_add(acc, rI[x - plo]);
    acc = f4_butterfly(acc);
    if (lane == 0) {
      W.z[b] = acc;
      a.loss[b] = acc.m == 0.0f ? inf_loss : 0.0f - xf_log(acc);
    }
  }
}

template <int DC>
__global__ __launch_bounds__(kF4Threads) void k_f4_sweep(V2FwdBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const bool fwd = blockIdx.y == 0;
  const int tid = threadIdx.x;
  int* dur = reinterpret_cast<int*>(smem);
  for (int i = tid; i < DC; i += kF4Threads) dur[i] = i < a.D ? a.table[i] : 0;
  lds_sync();
  F4Utt u;
  if (!f4_setup(a, b, dur, u, fwd)) {
    if (fwd) {
      const float inf_loss = (a.flags & SSNT_FLAG_ZERO_INFINITY) ? 0.0f : __builtin_inff();
      if (tid == 0) a.loss[b] = inf_loss;
      if (a.log_alpha)
        for (int r = 0; r <= a.Imax; ++r)
          f4_log_row(a.log_alpha + b * (size_t)(a.Imax + 1) * a.X + (size_t)r * a.X, nullptr, 0, -1, a.X);
    }
    return;
  }
  const bool padded = u.dmax <= kF4Pad;  // (uniform)
  if (fwd) {
    if (padded) f4_sweep<DC, true, true>(a, smem, u, u.dmax);
    else f4_sweep<DC, true, false>(a, smem, u, u.dmax);
  } else {
    if (padded) f4_sweep<DC, false, true>(a, smem, u, u.dmax);
    else f4_sweep<DC, false, false>(a, smem, u, u.dmax);
  }
}

// threads of a gradient workgroup: one wave up to 16 classes (a workgroup's time is its chain of
// dependent global loads, so more, smaller workgroups per CU overlap more of them: 64 threads
// 75 us, 128 87 us, 256 102 us at configs[4]), then more waves so a wave's class partials stay
// within its registers
template <int DC>
constexpr int f4_grad_threads() { return DC <= 16 ? 64 : DC <= 32 ? 128 : 256; }

// gradients of step t = blockIdx.y (and the debug beta row t); rows t >= I: zeros / -inf
template <int DC>
__global__ __launch_bounds__(f4_grad_threads<DC>()) void k_f4_grad(V2FwdBwdArgs a) {
  constexpr int kF4GradThreads = f4_grad_threads<DC>();
  constexpr int kF4GradWaves = kF4GradThreads / 64;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x, t = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D = a.D, X = a.X, Imax = a.Imax, Wc = a.Wcap;
  int* dur = reinterpret_cast<int*>(smem);
  xf* at = reinterpret_cast<xf*>(smem + ((D * 4 + 15) & ~15));  // alpha row t (+ zero cell Wc)
  xf* bn = at + Wc + 1;                                             // beta row t+1
  float* g = a.grad ? a.grad + ((size_t)b * Imax + (t < Imax ? t : 0)) * D : nullptr;
  float* lb = a.log_beta ? a.log_beta + ((size_t)b * (Imax + 1) + t) * X : nullptr;
  const F4Ws W = f4_ws(a);
  for (int i = tid; i < D; i += kF4GradThreads) dur[i] = a.table[i];
  lds_sync();
  F4Utt u;
  const bool ok = f4_setup(a, b, dur, u, false);
  const xf Z = ok ? W.z[b] : xf_zero();
  const bool live = ok && Z.m != 0.0f;
  if (lb) {
    int lo = 0, hi = -1;
    if (live && t <= u.I) f4_window(u, t, lo, hi);
    const xf* br = W.beta + ((size_t)b * (Imax + 1) + t) * Wc;
    for (int x = tid; x < X; x += kF4GradThreads)
      lb[x] = (x >= lo && x <= hi) ? xf_log(br[x - lo]) : -__builtin_inff();
  }
  if (t >= Imax || !g) return;
  if (!live || t >= u.I) {
    for (int i = tid; i < D; i += kF4GradThreads) g[i] = 0.0f;
    return;
  }
  int lo, hi, nlo, nhi;
  f4_window(u, t, lo, hi);
  f4_window(u, t + 1, nlo, nhi);
  const xf* ga = W.alpha + ((size_t)b * (Imax + 1) + t) * Wc;
  const xf* gb = W.beta + ((size_t)b * (Imax + 1) + t + 1) * Wc;
  for (int k = tid; k <= hi - lo; k += kF4GradThreads) at[k] = ga[k];
  if (tid == 0) at[Wc] = xf_zero();
  for (int k = tid; k <= nhi - nlo; k += kF4GradThreads) bn[k] = gb[k];
  lds_sync();
  const float izm = 1.0f / Z.m;
  const int ize = -Z.e;
  const unsigned span = hi >= lo ? (unsigned)(hi - lo) : 0u;
  if (hi < lo) lo = 1 << 29;  // empty alpha window: every offset out of range
  constexpr int NCW = (DC + kF4GradWaves - 1) / kF4GradWaves;  // classes per wave
  xf acc[NCW];
  int di[NCW];
#pragma unroll
  for (int j = 0; j < NCW; ++j) {
    acc[j] = xf_zero();
    const int i = wave + j * kF4GradWaves;
    di[j] = i < D ? dur[i] : 0;
  }
  for (int x = nlo + ((lane - nlo) & 63); x <= nhi; x += 64) {
    const xf bv = bn[x - nlo];
#pragma unroll
    for (int j = 0; j < NCW; ++j) {
      // a term outside the window is an exact zero: adding it leaves a normalized (or zero)
      // partial unchanged, so the select is the oracle's skip
      const unsigned yr = (unsigned)(x - di[j] - lo);
      const xf av = at[yr <= span ? (int)yr : Wc];  // (zero cell: the oracle's skip)
      acc[j] = xf_add(acc[j].m, acc[j].e, av.m * bv.m, av.e + bv.e);
    }
  }
  // every class of this wave reduced at once; lane l < NCW then holds class cls (distinct)
  const int cls = f4_reduce_classes<NCW>(acc, lane);
  const int i = wave + cls * kF4GradWaves;
  if (lane < NCW && i < D) {
    const xf w = xf_exp(a.logits[((size_t)b * Imax + t) * D + i], a.allow_skip || i != a.zid);
    g[i] = xf_neg_post((acc[0].m * w.m) * izm, acc[0].e + w.e + ize);
  }
}

}  // namespace

size_t v2_fwd_bwd_wcap(int max_total, bool test_mode) {
  const int X = max_total + 1;
  if (test_mode) return (size_t)X;
  const size_t band = (size_t)(0.15 * (double)max_total) + 8;  // ub - lb + 1 <= 0.15 O + 3
  return band < (size_t)X ? band : (size_t)X;
}

size_t v2_fwd_bwd_workspace_bytes(int B, int Imax, int max_total, bool test_mode) {
  if (B <= 0 || Imax <= 0 || max_total < 0) return 0;
  return (2 * (size_t)B * (Imax + 1) * v2_fwd_bwd_wcap(max_total, test_mode) + B) * sizeof(xf);
}

template <int DC>
int launch_f4(const V2FwdBwdArgs& a, size_t lds, size_t glds, hipStream_t st) {
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_f4_sweep<DC>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k_f4_sweep<DC>, dim3(a.B, 2), dim3(kF4Threads), lds, st, a);
  if (hipGetLastError() != hipSuccess) return SSNT_ERR_HIP;
  if (!a.grad && !a.log_beta) return SSNT_OK;
  if (glds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_f4_grad<DC>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)glds);
  hipLaunchKernelGGL(k_f4_grad<DC>, dim3(a.B, a.Imax + 1), dim3(f4_grad_threads<DC>()), glds, st, a);
  return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP;
}

int launch_v2_fwd_bwd(const V2FwdBwdArgs& in, hipStream_t st) {
  V2FwdBwdArgs a = in;
  if (a.B < 0 || a.Imax <= 0 || a.D <= 0 || a.X <= 0 || !a.logits || !a.table || !a.input_length ||
      !a.output_length || !a.loss)
    return SSNT_ERR_INVALID_ARG;
  if (a.B == 0) return SSNT_OK;
  if (a.D > 64) return SSNT_ERR_UNSUPPORTED;  // cell sums unrolled over <= 64 classes
  if ((size_t)a.B * (a.Imax + 1) > 0x7fffffffu / 2) return SSNT_ERR_UNSUPPORTED;
  a.Wcap = (int)v2_fwd_bwd_wcap(a.X - 1, a.test_mode);
  const int Dp = a.D <= 8 ? 8 : a.D <= 16 ? 16 : a.D <= 32 ? 32 : 64;  // = DC
  const size_t head = (size_t)((Dp * 4 + 15) & ~15);
  a.chunk = Dp <= 32 ? 64 : 32;  // = f4_chunk<DC>()
  const size_t lds = head + 2 * (size_t)a.chunk * Dp * sizeof(xf) +
                     2 * ((size_t)a.Wcap + 2 * kF4Pad + 2) * sizeof(xf);
  const size_t glds = head + (2 * (size_t)a.Wcap + 1) * sizeof(xf);
  if (lds > 160 * 1024 - 1024 || glds > 160 * 1024 - 1024) return SSNT_ERR_UNSUPPORTED;
  // (a sweep addresses one utterance's workspace rows with 32-bit offsets)
  if ((size_t)(a.Imax + 1) * a.Wcap * sizeof(xf) > 0x7fffffffu) return SSNT_ERR_UNSUPPORTED;
  // the gradient launch reads one utterance's class log-probs through a buffer descriptor of
  // Imax*D*4 bytes with 32-bit lane offsets: past 2 GB it would read zeros
  if ((size_t)a.Imax * a.D * sizeof(float) > 0x7fffffffu) return SSNT_ERR_UNSUPPORTED;
  if (!a.workspace || a.workspace_bytes < v2_fwd_bwd_workspace_bytes(a.B, a.Imax, a.X - 1, a.test_mode))
    return SSNT_ERR_WORKSPACE;
  if (a.D <= 8) return launch_f4<8>(a, lds, glds, st);
  if (a.D <= 16) return launch_f4<16>(a, lds, glds, st);
  if (a.D <= 32) return launch_f4<32>(a, lds, glds, st);
  return launch_f4<64>(a, lds, glds, st);
}

}  // namespace ssnt
