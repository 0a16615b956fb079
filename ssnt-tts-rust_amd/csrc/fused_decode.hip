// fused_decode.hip -- the whole T-step beam-search decode of one utterance in one wave, for the
// v1 emit/shift lattice (BASELINE configs[2]) and the v2 duration-class and tone-latent paths
// (configs[4]), plus the backtrace of the final slots in the same launch.
//
// Step contract: the reference's per-step kernels, bit-exact (src/lib.rs:149-230,
// src/v2.rs:269-339, src/tone_latent.rs:184-234). n = W*C candidates.
//
//   n <= 64  k_fused_reg: one candidate per lane; only the sort keys and the staged outputs touch
//            LDS.
//     rank     #{j : key_j > key_c} with key = (lp_key(lp), 63 - c): the stable descending sort
//              of src/lib.rs:161 (ties keep generation order), over broadcast LDS reads; for
//              n <= 8 the wave holds 8 replicas of the candidates and each lane does one of the
//              64 pairwise compares (one bpermute, one ballot, a byte popcount)
//     sort     ds_permute of the packed candidate fields to lane = rank
//     dedup    compare with the DPP-shifted left neighbour (src/lib.rs:162, eq_ignore_parent)
//     diagonal ballot of the kept on-diagonal lanes (src/v2.rs:283-308)
//     pad      each candidate lane fetches (ds_bpermute) the result slot its own beam index names
//              (cyclic pad src/lib.rs:163-167): the next step's beam state arrives in exactly the
//              lanes that expand that beam next.
//   n > 64   k_fused_lds: the one-wave LDS step of decode_dev.h in a loop.
//
// Step s's input row does not depend on the beam state (v2/tone: logits[b,s]; v1: every live
// beam has u == s, so its row is lattice[b,s]); rows are prefetched kAhead steps ahead.
#include <hip/hip_runtime.h>

#include <atomic>
#include <type_traits>

#include "buffer_ops.h"
#include "decode_dev.h"

namespace ssnt {
namespace {

using namespace dec;

constexpr int kAhead = 8;    // input rows in flight
// the rank counts by sign bits from this many compares per lane up
constexpr int kSignMin = 16;

// Diagnostic build only (-DSSNT_DIAG, `make lib-diag`): s_memtime cycle totals of the register
// kernel's step phases for utterance 0 (tools/diag_decode.py): 0 candidate generation, 1 rank /
// selection, 2 sort permute + dedup + keep ballot, 3 compaction + slot gather, 4 output staging
// and flush, 5 between steps (row refill, loop); [6] steps. Never present in the product build.
#ifdef SSNT_DIAG
__device__ unsigned long long g_dec_diag[8];
#define DSTAMP(k)                                                   \
  do {                                                              \
    const unsigned long long dnow_ = __builtin_amdgcn_s_memtime();  \
    dacc[k] += dnow_ - dlast;                                       \
    dlast = dnow_;                                                  \
  } while (0)
#else
#define DSTAMP(k) \
  do {            \
  } while (0)
#endif

// buffer resource over [base, base + bytes): loads past the end return 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
constexpr int kV1Regs = 4;   // v1 lattice row floats per lane: the row is staged while 2U <= 256
constexpr int kChunk = 32;   // per-step outputs staged in LDS and flushed every kChunk steps
constexpr int kRec = 4;      // ints per staged output record (one per step and slot)

// lane of the k-th set bit (k from 0) of a mask whose bits all lie below NMAX: a binary search
// on popcounts -- replaces the compaction permute and one bpermute (two LDS round trips)
template <int NMAX>
__device__ __forceinline__ int kth_set_bit(u64 m64, int k) {
  static_assert(NMAX <= 32, "32-bit search");
  unsigned m = (unsigned)m64;  // 32-bit shifts and popcounts (the 64-bit forms take two passes)
  int pos = 0;
#pragma unroll
  for (int half = NMAX / 2; half >= 1; half >>= 1) {
    const unsigned low = (1u << half) - 1u;
    const int c = __popc(m & low);
    const bool up = k >= c;
    k -= up ? c : 0;
    pos += up ? half : 0;
    m = up ? (m >> half) : m;
  }
  return pos;
}

// ballot of a bool (HIP's __ballot takes an int, and the int -> bool compare costs a select and a
// compare per call)
__device__ __forceinline__ u64 ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// per lane: bit `lane` of the wave-uniform mask m selects if_set, else if_clear (one v_cndmask with
// m as its lane mask; the compiler would shift and compare per lane)
__device__ __forceinline__ int mask_sel(u64 m, int if_set, int if_clear) {
  int r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(m));
  return r;
}

// One wave per workgroup: LDS operations of a wave complete in order, so a write followed by a
// read of the same location needs no barrier -- only the compiler must keep the order.
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

// LDS layout of k_fused_reg (bytes), shared with the host launcher.
// Staged outputs are records of kRec ints per (step, slot): the slot's packed state as the step
// gathered it, {log_prob, next_t << 16 | next_u, code | fin << 7 | parent << 8, next_total} --
// one 16-byte store per step with no repacking; the flush and the backtrace decode it.
// WHOLE: the records of all T steps fit, so they are flushed once after the loop -- no global
// store inside the step loop, whose wait-count merge would otherwise turn the row prefetch's
// wait into a vmcnt(0) once per unrolled group -- and the backtrace reads them directly (no
// separate history arrays).
// waves per utterance of the register kernel: 64 candidates of a v2 / tone step rank on 4 waves
// (each compares every candidate with 16 of the keys; the partial counts cross through LDS, one
// barrier per step), everything else runs identically in each wave, and wave 0 alone writes
// outputs. The 64 compares of one wave were a third of the step.
// Tone's 20 candidates (NMAX 32: two in-wave replicas) can split their rank over TW waves the
// same way (each wave counts JN / TW of its replica's keys): TW is a template parameter, chosen by
// the launcher (kToneWaves; the A/B build's ssnt_fused_decode_tone_waves overrides it).
constexpr int fused_waves(Variant v, int nmax, bool sel, int tw = 1) {
  return (nmax == 64 && v != Variant::V1 && !sel) ? 4 : (nmax == 32 && v == Variant::Tone && !sel) ? tw : 1;
}

struct RegLayout {
  size_t ring, hist, row, total;
  __host__ __device__ RegLayout(Variant v, int W, int T, int U, bool hist_lds, bool staged,
                                bool whole, int waves) {
    // per wave 64 sort keys (u64); with several waves the partial ranks, [2 steps][64][waves];
    // per wave 64 compacted kept records (int4) and 64 spare ones (the stores of lanes not kept),
    // then per wave the 128 v1 second row values
    ring = 512 * (size_t)waves + (waves > 1 ? (size_t)2 * 64 * waves * 4 : 0) + (size_t)2048 * waves +
           (size_t)512 * waves;
    hist = ring + (size_t)kRec * (whole ? T : kChunk) * W * 4;
    const int nh = v == Variant::V2 ? 3 : 2;
    row = hist + ((hist_lds && !whole) ? (size_t)nh * T * W * 4 : 0);
    // the staged v1 rows, double-buffered: 64 * kV1Regs floats each, so every lane stores all its
    // registers without a branch (a branch around the store merges the wait counts into a vmcnt(0))
    total = row + ((v == Variant::V1 && staged) ? (size_t)2 * 64 * kV1Regs * 4 : 0);
  }
};

// NMAX: a compile-time bound on n (8, 16, 32 or 64): the rank loop is unrolled to NMAX so its
// broadcast key reads are issued back to back instead of one LDS round trip per pair.
// SEL: the step's ordering by selection instead of a full rank (select_step below); the two
// forms give identical outputs.
// One wave per workgroup and (staged rows, history) LDS enough that one workgroup fills a CU: the
// compiler is told one wave per SIMD, so it may spend registers on keeping loads in flight (its
// default occupancy target of 8 waves caps a wave at 64 VGPRs, which serialised the rank's
// broadcast key reads into one LDS round trip per two keys).
template <Variant V, bool STAGED, int NMAX, bool WHOLE, bool SEL, int TW = 1>
__global__ __launch_bounds__(64 * fused_waves(V, NMAX, SEL, TW)) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_fused_reg(FusedDecodeArgs a, int hist_lds) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool kV1 = V == Variant::V1, kV2 = V == Variant::V2;
  constexpr int kNW = fused_waves(V, NMAX, SEL, TW);
  // sort and compaction through LDS records (v2 / tone beyond 16 candidates, staged v1); the
  // other forms permute the fields across lanes
  constexpr bool kRecs = (NMAX > 16 && !kV1) || (kV1 && STAGED);
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wv = kNW > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
  const int W = a.W, T = a.T, U = a.U;
  const int C = kV1 ? 2 : a.C;
  const int n = W * C;
  const RegLayout L(V, W, T, U, hist_lds != 0, STAGED, WHOLE, kNW);
  u64* keys = reinterpret_cast<u64*>(smem) + 64 * wv;  // this wave's copy
  int* xrank = reinterpret_cast<int*>(smem + 512 * kNW);  // [2][64][kNW] partial ranks
  // this wave's compacted kept records (lp, ntu, pk, total) of the current step
  int4* crec = reinterpret_cast<int4*>(smem + 512 * kNW + (kNW > 1 ? 2 * 64 * kNW * 4 : 0)) + 128 * wv;
  // v1: the second staged row value of each record, 128 per wave after the waves' records
  int* crec2 = reinterpret_cast<int*>(smem + 512 * kNW + (kNW > 1 ? 2 * 64 * kNW * 4 : 0) + 2048 * kNW) + 128 * wv;
  int4* rec = reinterpret_cast<int4*>(smem + L.ring);  // 2 x int4 per (step, slot)
  int* h_br = reinterpret_cast<int*>(smem + L.hist);  // (T,W) parent slot (!WHOLE)
  int* h_aux = h_br + (size_t)T * W;                   // (T,W) v1: next_t; v2/tone: prediction
  int* h_tot = h_aux + (size_t)T * W;                  // (T,W) v2: next_total_duration
  float* rowbuf = reinterpret_cast<float*>(smem + L.row);

  const u64 I = as_usize(a.input_length[b]);
  const u64 O = kV2 ? as_usize(a.output_length[b]) : 0;
  // NMAX < 64: the wave holds 64 / NMAX replicas of the candidate set (lane = NMAX * replica +
  // candidate); each replica does its share of the rank compares, and every later stage runs
  // identically in each replica. NMAX == 8: the rank is one pairwise compare per lane and a byte
  // popcount of its ballot; 16 / 32: partial counts summed across replicas by lane swaps.
  constexpr bool kRep8 = NMAX == 8;
  constexpr bool kRep = NMAX < 64;
  constexpr int kReps = 64 / NMAX;
  constexpr u64 kGrp = NMAX == 64 ? ~0ull : ((1ull << NMAX) - 1ull);  // ballot bits of replica 0
  const int c = lane & (NMAX - 1);      // candidate index of this lane
  const int gbase = lane & ~(NMAX - 1);  // first lane of this lane's replica
  const bool is_cand = c < n;
  const int w = is_cand ? c / C : 0;  // the beam this lane expands (generation order w*C + i)
  const int i = is_cand ? c - w * C : 0;
  const bool writer = wv == 0 && gbase == 0 && is_cand && i == 0;  // stages slot w's outputs
  const int sid = a.special_id;
  // prediction code: class index, or C for the "not defined" padding candidate whose prediction
  // is the special id (equal to class sid when sid names a class: eq_ignore_parent compares it)
  const int scode = kV1 ? 0 : ((sid >= 0 && sid < C) ? sid : C);
  const int dur = (kV2 && is_cand) ? a.table[i] : 0;
  // v2 band constants, f32 as in total_duration_bounds (src/v2.rs:94-104)
  const float o_over_i = (float)O / (float)I;
  const float upper_range = (float)O * 0.1f;
  const float lower_range = (float)O * 0.05f;

  // v2 band of step s (src/v2.rs:94-111; uniform per step: every defined beam has t == s). The
  // usize t + 1 converts to f32 like the int s + 1 for any s < 2^31 (the same integer, correctly
  // rounded).
  // test_mode is folded in: the band then spans every int, nothing overruns and the last step
  // needs no exact total (`exact`), so a candidate's check is one conjunction without branches.
  struct Band {
    int lb, ub;
    bool overrun, last, exact;
  };
  const bool tmode = a.test_mode;
  const int o_int = (int)O;  // the final total is compared as `next_total == output_length as i32`
  auto band_of = [&](int s) {
    Band r;
    const float diagonal = o_over_i * (float)(s + 1);
    r.lb = f2i_sat_sel(fmaxf(diagonal - lower_range, 0.0f));
    r.ub = f2i_sat_sel(fminf(diagonal + upper_range, (float)O));
    r.lb = tmode ? (-2147483647 - 1) : r.lb;
    r.ub = tmode ? 2147483647 : r.ub;
    const u64 t = (u64)s;
    r.overrun = !tmode && (I - (t + 1)) * 3 > O;
    r.last = t == I - 1;
    r.exact = !tmode && r.last;
    return r;
  };
  Band band{0, 0, false, false, false};
  // the bands of 64 consecutive steps, one per lane (lane l: step 64 j + l), formed once per 64
  // steps; step s reads its own with three v_readlane instead of ~22 instructions of f32 band
  // arithmetic per step
  int bl_lb = 0, bl_ub = 0, bl_fl = 0;
  // The overrun and exact-length rules are folded into the range as well: an overrunning step
  // admits no total (an empty range), and an exact last step admits only O within the band.
  auto band_block = [&](int s0) {
    const Band r = band_of(s0 + lane);
    int lb = r.exact ? max(r.lb, o_int) : r.lb;
    int ub = r.exact ? min(r.ub, o_int) : r.ub;
    lb = r.overrun ? 2147483647 : lb;
    ub = r.overrun ? (-2147483647 - 1) : ub;
    bl_lb = lb;
    bl_ub = ub;
    bl_fl = r.last ? 2 : 0;
  };
  auto band_at = [&](int s) {
    const int l = s & 63;
    Band r;
    r.lb = readlane_i(bl_lb, l);
    r.ub = readlane_i(bl_ub, l);
    const int fl = readlane_i(bl_fl, l);
    r.overrun = false;  // (folded into the range)
    r.last = (fl & 2) != 0;
    r.exact = false;
    return r;
  };
  // the class rule of decode_beam_at (src/v2.rs:127-133), a per-lane constant
  const bool class_ok = a.allow_skip || i != sid;

  // state of beam w, replicated in its C candidate lanes
  float hist = 0.0f;
  int bt = 0, bu = 0, bfin = 0, btot = 0;
  // v1 staged: the two lattice values of beam w's next row at t = bt, read one step ahead by the
  // candidate that became the beam and carried through the sort and the gather, so a step starts
  // without an LDS round trip
  float cv0 = 0.0f, cv1 = 0.0f;

  const int row_len = kV1 ? 2 * U : n;
  const float* src = a.src + (size_t)b * T * row_len;
  constexpr int R = kV1 ? kV1Regs : 1;
  float pre[kAhead][R];
  // unconditional loads (a conditional load becomes a branch whose join waits for it) through a
  // buffer resource over this utterance's rows: one lane offset, the row as the scalar offset,
  // the register index as the immediate; entries past the row end are never read, and past the
  // utterance the hardware returns 0
  const __amdgpu_buffer_rsrc_t rows_rs = brsrc(src, (unsigned)((size_t)T * row_len * 4));
  auto load_row = [&](int s, float* dst) {
    const int soff = min(s, T - 1) * row_len * 4;
#pragma unroll
    for (int q = 0; q < R; ++q) dst[q] = rbuf_ld1(rows_rs, 4 * (kV1 ? lane : c) + 256 * q, soff, 0);
  };
  if constexpr (!kV1 || STAGED) {
#pragma unroll
    for (int k = 0; k < kAhead; ++k) load_row(k, pre[k]);
  }
  if constexpr (kV1 && STAGED) {  // row 0 -> buffer 0; every beam starts at t = 0
#pragma unroll
    for (int q = 0; q < R; ++q) rowbuf[lane + 64 * q] = pre[0][q];
    lds_order();
    cv0 = rowbuf[0];
    cv1 = rowbuf[1];
    lds_order();
  }

  // prediction of a packed code: class index, or the special id for the padding candidate
  auto rec_pred = [&](int pk) {
    const int pc = pk & 0x7f;
    return pc == C ? sid : pc;
  };
  auto flush = [&](int s0, int steps) {  // staged outputs of steps [s0, s0+steps), coalesced
    lds_order();
    const int cnt = steps * W;
    const size_t g0 = ((size_t)b * T + s0) * W;
    for (int k = lane; k < cnt; k += 64) {
      const int4 r = rec[k];
      a.prediction[g0 + k] = rec_pred(r.z);
      a.log_prob[g0 + k] = __int_as_float(r.x);
      a.next_t[g0 + k] = (int)((unsigned)r.y >> 16);
      a.next_u[g0 + k] = r.y & 0xffff;
      a.next_fin[g0 + k] = ((r.z >> 7) & 1) != 0;
      a.beam_branch[g0 + k] = (r.z >> 8) & 63;
      if constexpr (kV2) a.next_total[g0 + k] = r.w;
    }
    lds_order();
  };

  // one step; false when v2 finds no candidate (src/v2.rs:292)
#ifdef SSNT_DIAG
  unsigned long long dacc[7] = {0, 0, 0, 0, 0, 0, 0};
  unsigned long long dlast = __builtin_amdgcn_s_memtime();
#endif
  auto step = [&](int s, float* row, const float* nrow) -> bool {
    DSTAMP(5);
    float* nbuf = rowbuf + ((s + 1) & 1) * 64 * R;  // row s+1 (buffer last read by step s-1)
    if constexpr (kV1 && STAGED) {
#pragma unroll
      for (int q = 0; q < R; ++q) nbuf[lane + 64 * q] = nrow[q];  // (entries past 2U: never read)
      lds_order();
    }
    (void)row;
    if constexpr (kV2) band = band_at(s);
    // ---- candidate of this lane (decode_dev.h gen_candidate, one lane per candidate)
    // straight-line selects, no exec-mask branches (each branch costs exec save/restore and
    // splits the wait counts)
    // v2 / tone: every unfinished beam has t == s (each starts at t = 0 and an unfinished
    // candidate moves to t + 1), so the test of t < I is the uniform s < I
    const bool defined = kV1 ? (!bfin && as_usize(bt) < I) : (!bfin & ((u64)s < I));
    int valid, code, nt, nu, fin, tot = btot;
    float lp;
    if constexpr (kV1) {  // src/lib.rs:186-227
      const bool hdef = ((is_cand ? 1 : 0) & ((unsigned)bu < (unsigned)T ? 1 : 0) &
                         ((unsigned)bt < (unsigned)U ? 1 : 0)) != 0;  // bitwise: no branch
      float hv;
      if constexpr (STAGED) hv = i == 0 ? cv0 : cv1;  // row s at t = bt (bu == s for every live beam)
      else hv = src[hdef ? ((size_t)bu * U + bt) * 2 + i : 0];
      hv = hdef ? hv : 0.0f;
      const bool last = as_usize(bt) == I - 1;
      const bool shift = i == 1;
      valid = 1;
      code = (shift && !last) ? 1 : 0;
      lp = (shift && last) ? hist : hist + hv;  // the prohibited last shift keeps the history
      nt = (shift && !last) ? bt + 1 : bt;
      nu = last ? bu : bu + 1;
      fin = last ? 1 : 0;
    } else if constexpr (V == Variant::Tone) {  // src/tone_latent.rs:87-93, 220-231
      valid = 1; code = i; lp = hist + row[0]; nt = bt + 1; nu = bu + 1; fin = 0;
    } else {  // v2: src/v2.rs:119-166, 326-336
      tot = (int)((unsigned)btot + (unsigned)dur);
      // a defined beam (the only kind whose candidate is used) has t == s: every beam starts at
      // t = 0, an unfinished candidate of a defined beam moves to t + 1, and every other
      // candidate is finished (never defined again) -- so the band of src/v2.rs:94-111 is
      // uniform per step
      // the else-if chain of decode_beam_at as one conjunction (test_mode folded into the band),
      // bitwise so that no term becomes an exec-mask branch
      const bool ok = (tot >= band.lb) & (tot <= band.ub) & class_ok;  // (rules folded into the range)
      const bool f = ok & band.last;
      valid = ok; code = i; lp = hist + row[0];
      nt = f ? bt : bt + 1; nu = f ? bu : bu + 1; fin = f;
    }
    // "End of input. Return values to fill padding region." (src/lib.rs:57-67 etc.)
    valid = defined ? valid : (i == 0);
    code = defined ? code : scode;
    lp = defined ? lp : hist;
    nt = defined ? nt : bt;
    nu = defined ? nu : bu;
    fin = defined ? fin : 1;
    tot = defined ? tot : btot;
    valid = valid && is_cand;
    // v2: whether this candidate lies on the diagonal (src/v2.rs:283-289) -- a property of its own
    // (total, next_t), so it is formed here and rides through the sort as bit 14 of the packed
    // fields instead of being computed from the sorted fields on the step's critical path
    int on_diag = 0;
    if constexpr (kV2) {
      const float diff = (float)tot - o_over_i * (float)(u64)(unsigned)nt;
      on_diag = (!tmode & (valid != 0) & (diff >= -20.0f) & (diff <= 0.0f)) ? 1 : 0;
    }
    // v1 staged: this candidate's row s+1 values at t = nt (read now, used by the next step)
    float nv0 = 0.0f, nv1 = 0.0f;
    if constexpr (kV1 && STAGED) {
      const float2 v = *reinterpret_cast<const float2*>(nbuf + ((unsigned)nt < (unsigned)U ? 2 * nt : 0));
      nv0 = v.x;
      nv1 = v.y;
    }
    int g_lp, g_ntu, g_pk, g_tot;
    DSTAMP(0);
    if constexpr (SEL) {
      // ---- selection (src/lib.rs:161-168, src/v2.rs:280-308): only the first W kept candidates
      // of the sorted, deduplicated list (and the v2 diagonal one) are ever used, so they are
      // extracted one by one instead of ranking all n. A round takes the largest key among the
      // candidates not yet extracted (group max, ties to the lowest generation index: the stable
      // descending order), reads its fields into scalars and keeps it unless it equals the
      // previous extracted candidate (consecutive dedup: equal to the previous extracted is equal
      // to the last kept, eq_ignore_parent being an equivalence). Kept record k goes to lane k.
      const unsigned key = valid ? lp_key(lp) : 0u;  // valid keys are >= 1
      const int lpb = __float_as_int(lp);
      const int pk = code | (fin << 7) | (w << 8);
      const int ntu = (nt << 16) | (nu & 0xffff);
      const int v0b = __float_as_int(nv0), v1b = __float_as_int(nv1);
      u64 rem = ballot(valid != 0) & kGrp;  // (replicas mirror replica 0)
      int nk = 0;
      int r_lp = 0, r_ntu = 0, r_pk = 0, r_tot = 0, r_v0 = 0, r_v1 = 0;
      int q_lp = 0, q_ntu = 0, q_pk = 0, q_tot = 0;
      bool have_q = false;
      while (rem != 0 && nk < W) {
        const bool in = ((rem >> c) & 1ull) != 0;
        const unsigned m = group_max_u32<NMAX>(in ? key : 0u);
        const int sel = (int)__builtin_ctzll(ballot(in && key == m) & kGrp);
        rem &= ~(1ull << sel);
        const int f_lp = readlane_i(lpb, sel), f_ntu = readlane_i(ntu, sel), f_pk = readlane_i(pk, sel);
        const int f_tot = kV2 ? readlane_i(tot, sel) : 0;
        const bool dup = have_q && ((f_pk ^ q_pk) & 0xff) == 0 &&
                         __int_as_float(f_lp) == __int_as_float(q_lp) && f_ntu == q_ntu && f_tot == q_tot;
        if (!dup) {
          const bool mine = lane == nk;
          r_lp = mine ? f_lp : r_lp;
          r_ntu = mine ? f_ntu : r_ntu;
          r_pk = mine ? f_pk : r_pk;
          if constexpr (kV2) r_tot = mine ? f_tot : r_tot;
          if constexpr (kV1 && STAGED) {
            r_v0 = mine ? readlane_i(v0b, sel) : r_v0;
            r_v1 = mine ? readlane_i(v1b, sel) : r_v1;
          }
          ++nk;
        }
        q_lp = f_lp; q_ntu = f_ntu; q_pk = f_pk; q_tot = f_tot;
        have_q = true;
      }
      if constexpr (kV2) {  // assert_ne!(n_results, 0) (src/v2.rs:292); v1/tone always keep one
        if (nk == 0) return false;
      }
      // v2 diagonal candidate (src/v2.rs:283-289): the first kept one on the diagonal is the
      // largest-key valid one on it -- a dedup-dropped candidate equals its kept predecessor in
      // total and next_t, so that predecessor is on the diagonal too and comes first
      bool have_d = false;
      int d_lp = 0, d_ntu = 0, d_pk = 0, d_tot = 0;
      if constexpr (kV2) {
        if (!a.test_mode) {
          const float diff = (float)tot - o_over_i * (float)(u64)(unsigned)nt;
          const bool on = valid && diff >= -20.0f && diff <= 0.0f;
          const u64 dm = ballot(on) & kGrp;
          if (dm) {
            const unsigned m = group_max_u32<NMAX>(on ? key : 0u);
            const int ds = (int)__builtin_ctzll(ballot(on && key == m) & kGrp);
            d_lp = readlane_i(lpb, ds); d_ntu = readlane_i(ntu, ds); d_pk = readlane_i(pk, ds);
            d_tot = readlane_i(tot, ds);
            have_d = true;
          }
        }
      }
      // slot w: kept[w % nk] (cyclic pad, src/v2.rs:293-297 / src/lib.rs:163-167), the last slot
      // the diagonal candidate when there is one (src/v2.rs:298-308)
      int j = w;
      while (j >= nk) j -= nk;
      g_lp = bperm_i(j, r_lp);
      g_ntu = bperm_i(j, r_ntu);
      g_pk = bperm_i(j, r_pk);
      g_tot = kV2 ? bperm_i(j, r_tot) : 0;
      if constexpr (kV1 && STAGED) {
        cv0 = __int_as_float(bperm_i(j, r_v0));
        cv1 = __int_as_float(bperm_i(j, r_v1));
      }
      if (have_d && w == W - 1) {
        g_lp = d_lp; g_ntu = d_ntu; g_pk = d_pk; g_tot = d_tot;
      }
    } else {
    // ---- stable descending rank (src/lib.rs:161): keys are unique, so ranks are a permutation
    const unsigned khi = lp_key(lp);
    // kSign (>= 32 compares per lane): a 63-bit key (high word shifted by 31), so a difference of
    // two keys never overflows and its sign bit is the comparison; else (khi, 63 - c) as a pair
    constexpr int kJN = kRep8 ? 1 : NMAX / kReps;
    constexpr bool kSign = kJN >= kSignMin;
    const u64 key = ((u64)(valid ? khi : 0u) << (kSign ? 31 : 32)) | (unsigned)(63 - c);
    int rank = 0;
    int rank16 = -1;  // 16 * rank when the partial counts arrive premultiplied (four waves)
    // count the keys in kr[0, JN) (stored negated) that beat this lane's: key + (-key_j) has its
    // sign bit set iff key_j > key; the signs are shifted into a bit mask by v_alignbit and
    // counted per 32 -- no compare into an SGPR mask, so no VALU -> SGPR -> VALU hazard waits
    auto count_beats = [&](const u64* kr, auto jn) {
      constexpr int JN = decltype(jn)::value;
      int r = 0;
      if constexpr (!kSign) {  // keys stored as they are
        ulonglong2 kk[JN / 2];  // (JN <= 16: every broadcast read issued before the compares)
#pragma unroll
        for (int q = 0; q < JN / 2; ++q) kk[q] = reinterpret_cast<const ulonglong2*>(kr)[q];
#pragma unroll
        for (int q = 0; q < JN / 2; ++q) r += (kk[q].x > key ? 1 : 0) + (kk[q].y > key ? 1 : 0);
        return r;
      }
      unsigned bits = 0;
      // groups of 16 keys: 8 broadcast reads issued back to back, then their compares (one LDS
      // round trip per group instead of one per read)
      constexpr int G = JN < 16 ? JN : 16;
#pragma unroll
      for (int j0 = 0; j0 < JN; j0 += G) {
        ulonglong2 kk[G / 2];
#pragma unroll
        for (int q = 0; q < G / 2; ++q) kk[q] = reinterpret_cast<const ulonglong2*>(kr + j0)[q];
#pragma unroll
        for (int q = 0; q < G / 2; ++q) {
          const int j = j0 + 2 * q;
          bits = __builtin_amdgcn_alignbit(bits, (unsigned)((key + kk[q].x) >> 32), 31);
          bits = __builtin_amdgcn_alignbit(bits, (unsigned)((key + kk[q].y) >> 32), 31);
          if ((j + 2) % 32 == 0 || j + 2 >= JN) {
            r += __popc(bits);
            bits = 0;
          }
        }
      }
      return r;
    };
    // several waves: each wave's partial counts meet in LDS (double-buffered by step parity: a
    // wave a step ahead writes the other buffer) across one barrier that orders LDS only (no
    // wait for the row prefetch's global loads); the sum comes back premultiplied by 16
    auto wave_sum16 = [&](int part) {
      int* xr = xrank + (s & 1) * 64 * kNW;
      xr[lane * kNW + wv] = part << 4;  // (premultiplied: the sum is a record's byte offset)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
      int r16;
      if constexpr (kNW == 4) {
        const int4 pr = *reinterpret_cast<const int4*>(xr + lane * kNW);
        r16 = (pr.x + pr.y) + (pr.z + pr.w);
      } else if constexpr (kNW == 2) {
        const int2 pr = *reinterpret_cast<const int2*>(xr + lane * kNW);
        r16 = pr.x + pr.y;
      } else {
        r16 = part << 4;  // (one wave: never called)
      }
      lds_order();
      return r16;
    };
    if constexpr (kRep8) {
      // lane 8x + y compares its candidate y with candidate x (read from lane x): bit 8x + y of
      // the ballot says y sorts before x, so candidate x's rank is the popcount of byte x
      const int xl = lane >> 3;
      const unsigned klo = (unsigned)bperm_i(xl, (int)(unsigned)key);
      const unsigned khx = (unsigned)bperm_i(xl, (int)(unsigned)(key >> 32));
      const u64 beats = ballot(key > (((u64)khx << 32) | klo));  // (63-bit keys compare as u64)
      rank = __popc((unsigned)(beats >> (8 * c)) & 0xffu);
    } else if constexpr (kRep) {
      // replica r counts the keys [r JN, (r + 1) JN) of replica 0 that beat its candidate (reads
      // broadcast within the replica); the partial counts are summed across replicas by swapping
      // 16-lane rows and 32-lane halves
      // (several waves: each wave counts JN / kNW of those keys, and the waves' partial counts
      // are summed like the four-wave rank below)
      constexpr int JN = NMAX / kReps;
      constexpr int JW = JN / kNW;
      keys[lane] = kSign ? 0ull - key : key;
      lds_order();
      rank = count_beats(keys + (lane / NMAX) * JN + JW * wv, std::integral_constant<int, JW>{});
      lds_order();
      if constexpr (kReps == 4) {
        const auto r16 = __builtin_amdgcn_permlane16_swap(rank, rank, false, false);
        rank = (int)(r16[0] + r16[1]);
      }
      const auto r32 = __builtin_amdgcn_permlane32_swap(rank, rank, false, false);
      rank = (int)(r32[0] + r32[1]);
      if constexpr (kNW > 1) {
        rank = wave_sum16(rank) >> 4;
        rank16 = (gbase | rank) << 4;
      }
    } else if constexpr (kNW > 1) {
      // wave wv counts the keys [16 wv, 16 wv + 16) of its own copy; the partial counts meet in
      // LDS (double-buffered by step parity: a wave a step ahead writes the other buffer) across
      // one barrier that orders LDS only (no wait for the row prefetch's global loads)
      keys[lane] = kSign ? 0ull - key : key;
      lds_order();
      const int part = count_beats(keys + (64 / kNW) * wv, std::integral_constant<int, 64 / kNW>{});
      rank16 = wave_sum16(part);
      rank = rank16 >> 4;
    } else {
      keys[lane] = kSign ? 0ull - key : key;
      lds_order();
      // keys of lanes >= n are below every valid key (their high bits are 0): reading them is harmless
      rank = count_beats(keys, std::integral_constant<int, NMAX>{});
      lds_order();
    }
    DSTAMP(1);
    const u64 vmask = ballot(valid != 0) & kGrp;
    const int nvalid = __popcll(vmask);
    const u64 below = (1ull << c) - 1ull;  // candidates of this replica before this lane
    // a full permutation of the 64 lanes: every key is distinct and the invalid ones (high word
    // 0) lie below the valid ones, so the lanes < NMAX rank to [0, NMAX) -- valid candidates to
    // [0, nvalid) -- and the lanes past the bound keep their place (replicas: within the replica)
    const int dst = kRep ? (gbase | rank) : (lane < NMAX ? rank : lane);
    const int sp = c;  // sorted position of this lane within its replica
    const int pk = code | (fin << 7) | (w << 8) | (on_diag << 14);
    const int ntu = (nt << 16) | (nu & 0xffff);
    int s_lp, s_ntu, s_pk, s_tot, s_v0 = 0, s_v1 = 0, p_lp, p_ntu, p_pk, p_tot;
    if constexpr (kRecs) {
      // sort through LDS records: each candidate stores its (lp, ntu, pk, total) at record
      // `rank`, and sorted lane l reads records l and l - 1 (its predecessor, for the dedup) --
      // one LDS round trip, in place of four permutes and four DPP shifts. v1 carries its two
      // staged row values instead of the total: the first in the record, the second beside it.
      int4* const crd = kNW > 1 ? reinterpret_cast<int4*>(reinterpret_cast<char*>(crec) + rank16) : crec + dst;
      *crd = make_int4(__float_as_int(lp), ntu, pk, kV1 ? __float_as_int(nv0) : tot);
      if constexpr (kV1) crec2[dst] = __float_as_int(nv1);
      lds_order();
      const int4 cr = crec[lane];
      const int4 pr = crec[lane > 0 ? lane - 1 : 0];
      if constexpr (kV1) s_v1 = crec2[lane];
      lds_order();
      s_lp = cr.x; s_ntu = cr.y; s_pk = cr.z; s_tot = kV2 ? cr.w : 0;
      p_lp = pr.x; p_ntu = pr.y; p_pk = pr.z; p_tot = kV2 ? pr.w : 0;
      if constexpr (kV1) s_v0 = cr.w;
    } else {
      s_lp = perm_i(dst, __float_as_int(lp));
      s_ntu = perm_i(dst, ntu);
      s_pk = perm_i(dst, pk);
      s_tot = kV2 ? perm_i(dst, tot) : 0;
      if constexpr (kV1 && STAGED) {
        s_v0 = perm_i(dst, __float_as_int(nv0));
        s_v1 = perm_i(dst, __float_as_int(nv1));
      }
      // ---- consecutive dedup, keep the first of each run (src/lib.rs:162; v2 adds the total)
      // every cross-lane read happens with the whole wave active: a DPP read of a lane that is
      // off in the exec mask returns the old value, so no shift may sit behind a short circuit
      p_lp = wave_shr1(s_lp); p_ntu = wave_shr1(s_ntu); p_pk = wave_shr1(s_pk);
      p_tot = kV2 ? wave_shr1(s_tot) : 0;
    }
    const bool same = (((s_pk ^ p_pk) & 0xff) == 0) & (__int_as_float(s_lp) == __int_as_float(p_lp)) &
                      (s_ntu == p_ntu) & (s_tot == p_tot);
    // bitwise, not short-circuit: the && form compiles to an exec-mask branch around the compare
    const bool keep = (sp < nvalid) & ((sp == 0) | !same);
    u64 kmask;
    if constexpr (kRecs || NMAX <= 16) {  // (the v1 permute form beyond 16 uses `keep` itself)
      // the same mask from direct compare ballots: sorted positions [0, nvalid) (a scalar mask),
      // kept at position 0 or where the fields differ from the predecessor's -- no per-lane bool
      // materialised and ballotted again
      // (one ballot per compare: a ballot of a combined bool is materialised and compared again)
      const u64 differ = ballot(((s_pk ^ p_pk) & 0xff) != 0) |
                         ballot(__int_as_float(s_lp) != __int_as_float(p_lp)) | ballot(s_ntu != p_ntu) |
                         ballot(s_tot != p_tot);
      const u64 lowv = nvalid >= 64 ? ~0ull : ((1ull << nvalid) - 1ull);
      kmask = lowv & (differ | 1ull) & kGrp;
    } else {
      kmask = ballot(keep) & kGrp;
    }
    const int nkept = __popcll(kmask);
    if constexpr (kV2) {  // assert_ne!(n_results, 0) (src/v2.rs:292); v1/tone always keep one
      if (nkept == 0) return false;
    }
    // ---- v2 diagonal injection (src/v2.rs:283-308): first kept candidate on the diagonal
    int dk = -1;
    if constexpr (kV2) {
      // (the on-diagonal bit is 0 in test mode)
      const u64 dmask = ballot((s_pk & (1 << 14)) != 0) & kmask;
      if (dmask) dk = __popcll(kmask & ((1ull << (__ffsll((long long)dmask) - 1)) - 1ull));
    }
    // ---- compaction (kept element k -> its sorted lane) and the cyclic pad
    int k;
    if constexpr (kV1 && kRep8) {  // w < W <= 4: w % nkept by three wrapping subtractions
      unsigned kk = (unsigned)w;
#pragma unroll
      for (int r = 0; r < 3; ++r) kk = min(kk, kk - (unsigned)nkept);
      k = (int)kk;
    } else {
      // nkept, W and dk are wave-uniform: both tests are scalar branches, and the modulo runs
      // only when the kept list is shorter than the beam
      k = w;
      if (nkept < W) k = w % nkept;
      if (dk >= 0) k = w == W - 1 ? dk : k;
    }
    DSTAMP(2);
    if constexpr (kRecs) {
      // compaction and slot fetch in one LDS round trip: kept element ck (its sorted lane's
      // fields) is stored at record ck, and each lane reads record k (in-order DS within the
      // wave: no barrier, and the sort's reads of these records are done; replica 0 writes,
      // every replica reads the same records)
      // kept lane of replica 0 -> record mbcnt(kmask) (the kept lanes before it); every other lane
      // (dropped, or a later replica's: kmask's bits lie below NMAX) stores to its own spare
      // record 64 + lane, so the store needs no exec mask
      const int cidx = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(kmask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)kmask, 0u));
      const int widx = mask_sel(kmask, cidx, 64 + lane);
      crec[widx] = make_int4(s_lp, s_ntu, s_pk, kV1 ? s_v0 : s_tot);
      if constexpr (kV1) crec2[widx] = s_v1;
      lds_order();
      const int4 kr = crec[k];
      if constexpr (kV1) cv1 = __int_as_float(crec2[k]);
      lds_order();
      g_lp = kr.x; g_ntu = kr.y; g_pk = kr.z; g_tot = kV2 ? kr.w : 0;
      if constexpr (kV1) cv0 = __int_as_float(kr.w);
    } else {
    int srcl;  // sorted lane of kept element k
    if constexpr (NMAX <= 16) {
      srcl = gbase | kth_set_bit<NMAX>(kmask, k);
    } else {  // (wider masks: the search costs more than the permute round trip it saves)
      const int cdst = keep ? __popcll(kmask & below) : nkept + __popcll(~kmask & below);
      srcl = bperm_i(gbase | k, perm_i(gbase | cdst, lane));
    }
    g_lp = bperm_i(srcl, s_lp); g_ntu = bperm_i(srcl, s_ntu); g_pk = bperm_i(srcl, s_pk);
    g_tot = kV2 ? bperm_i(srcl, s_tot) : 0;
    if constexpr (kV1 && STAGED) {
      cv0 = __int_as_float(bperm_i(srcl, s_v0));
      cv1 = __int_as_float(bperm_i(srcl, s_v1));
    }
    }
    }
    hist = __int_as_float(g_lp);
    bt = (int)((unsigned)g_ntu >> 16);
    bu = g_ntu & 0xffff;
    bfin = (g_pk >> 7) & 1;
    btot = g_tot;
    DSTAMP(3);
    // ---- outputs of slot w (src/lib.rs:138-145), staged
    const int cs = WHOLE ? s : s % kChunk;
    if (writer) {
      // (.w is read back for v2 only: v1 stores its carried row value there as gathered)
      rec[cs * W + w] = make_int4(g_lp, g_ntu, g_pk, kV2 ? g_tot : (kV1 && kRecs) ? __float_as_int(cv0) : 0);
      if (!WHOLE && hist_lds) {
        const int hs = s * W + w;
        h_br[hs] = (g_pk >> 8) & 63;
        h_aux[hs] = kV1 ? bt : rec_pred(g_pk);
        if constexpr (kV2) h_tot[hs] = btot;
      }
    }
    if constexpr (!WHOLE) {
      if (wv == 0 && (cs == kChunk - 1 || s == T - 1)) flush(s - cs, cs + 1);
    }
    DSTAMP(4);
#ifdef SSNT_DIAG
    ++dacc[6];
#endif
    return true;
  };

  bool ok = true;
  for (int s0 = 0; s0 < T && ok; s0 += kAhead) {  // unrolled by the ring: register indices fixed
    if constexpr (kV2) {
      static_assert(64 % kAhead == 0, "a band block starts at a loop iteration");
      if ((s0 & 63) == 0) band_block(s0);
    }
#pragma unroll
    for (int k = 0; k < kAhead; ++k) {
      // the refill is unconditional (clamped rows past T): a load skipped on some path would
      // make the wait for the next row a vmcnt(0). v1 staged: step s reads only row s+1 (row s
      // was staged by step s-1), so row s's registers are refilled before the step, ahead of
      // its LDS traffic; the other variants read row s in the step and refill after it.
      if constexpr (kV1 && STAGED) load_row(s0 + k + kAhead, pre[k]);
      if (ok && s0 + k < T) ok = step(s0 + k, pre[k], pre[(k + 1) % kAhead]);
      if constexpr (!kV1) load_row(s0 + k + kAhead, pre[k]);
    }
  }
  if (!ok) {
    if (wv == 0 && lane == 0 && a.status) atomicOr(a.status, kStatusNoCandidate);
    return;
  }
  if (wv != 0) return;  // (the other waves' copies of the state are identical)
  if constexpr (WHOLE) flush(0, T);
#ifdef SSNT_DIAG
  if (b == 0 && lane == 0)
    for (int k = 0; k < 7; ++k) g_dec_diag[k] = dacc[k];
#endif
  if (!hist_lds) return;  // the host runs k_fused_paths over the global outputs
  // ---- backtrace of final slot `lane` (v2_util.rs:6-36 with final_branch = [0..W); util.rs:20-33
  // for slot 0 with t history = next_t)
  lds_order();
  if (lane < W) {
    int cur = lane;
    int* ord = a.ordered ? a.ordered + ((size_t)b * W + lane) * T : nullptr;
    int* pp = a.path_pred ? a.path_pred + ((size_t)b * W + lane) * T : nullptr;
    int* du = a.duration ? a.duration + ((size_t)b * W + lane) * T : nullptr;
    const bool best = lane == 0 && a.best_beam_branch;
    // history of (s, slot): parent, aux (v1: next_t; v2/tone: prediction), next_total
    auto hist_at = [&](int hs, int& parent, int& aux, int& tot) {
      if constexpr (WHOLE) {
        const int4 r = rec[hs];
        parent = (r.z >> 8) & 63;
        aux = kV1 ? (int)((unsigned)r.y >> 16) : rec_pred(r.z);
        tot = r.w;
      } else {
        parent = h_br[hs];
        aux = h_aux[hs];
        tot = kV2 ? h_tot[hs] : 0;
      }
    };
    for (int s = T - 1; s >= 0; --s) {
      const int hs = s * W + cur;
      int parent, aux, tot;
      hist_at(hs, parent, aux, tot);
      if (ord) ord[s] = cur;
      if constexpr (!kV1) {
        if (pp) pp[s] = aux;
      }
      if constexpr (kV2) {
        if (du) {
          int pp_, pa_, ptot = 0;
          if (s > 0) hist_at(hs - W - cur + parent, pp_, pa_, ptot);
          du[s] = tot - ptot;
        }
      }
      if (best) {
        a.best_beam_branch[(size_t)b * T + s] = cur;
        a.best_t_history[(size_t)b * T + s] = aux;
      }
      cur = parent;
    }
  }
}

// Any n: the one-wave LDS step (decode_dev.h step_wave) in a loop; beam state in LDS.
template <Variant V>
__global__ __launch_bounds__(64) void k_fused_lds(FusedDecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool kV1 = V == Variant::V1;
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int W = a.W, T = a.T, U = a.U;
  const int C = kV1 ? 2 : a.C;
  const int n = W * C;
  Cand* cand = reinterpret_cast<Cand*>(smem);
  int* order = reinterpret_cast<int*>(cand + n);
  int* kept = order + n;
  float* st_hist = reinterpret_cast<float*>(kept + n);  // (W) state, then (W) next state
  int* st_t = reinterpret_cast<int*>(st_hist + 2 * W);
  int* st_u = st_t + 2 * W;
  int* st_tot = st_u + 2 * W;
  float* hbuf = reinterpret_cast<float*>(st_tot + 2 * W);  // (W,2) v1 inputs
  bool* st_fin = reinterpret_cast<bool*>(hbuf + (kV1 ? 2 * W : 0));  // (2W)
  StepArgs sa{};
  sa.variant = V;
  sa.B = a.B; sa.W = W; sa.Wmax = W; sa.C = C;
  sa.table = a.table; sa.special_id = kV1 ? 0 : a.special_id;
  sa.allow_skip = a.allow_skip; sa.test_mode = a.test_mode;
  BatchView v;
  v.hist = st_hist; v.fin = st_fin; v.t = st_t; v.u = st_u; v.total = st_tot;
  v.I = as_usize(a.input_length[b]);
  v.O = V == Variant::V2 ? as_usize(a.output_length[b]) : 0;
  const int row_len = kV1 ? 2 * U : n;
  const float* src = a.src + (size_t)b * T * row_len;
  for (int x = lane; x < W; x += 64) {
    st_hist[x] = 0.0f; st_t[x] = 0; st_u[x] = 0; st_tot[x] = 0; st_fin[x] = false;
  }
  __syncthreads();
  for (int s = 0; s < T; ++s) {
    if constexpr (kV1) {
      for (int x = lane; x < W; x += 64) {
        const bool hdef = !st_fin[x] && as_usize(st_t[x]) < v.I && (unsigned)st_u[x] < (unsigned)T &&
                          (unsigned)st_t[x] < (unsigned)U;
        float2 h = make_float2(0.0f, 0.0f);
        if (hdef) h = *reinterpret_cast<const float2*>(src + ((size_t)st_u[x] * U + st_t[x]) * 2);
        hbuf[2 * x] = h.x;
        hbuf[2 * x + 1] = h.y;
      }
      v.h = hbuf;
      __syncthreads();
    } else {
      v.h = src + (size_t)s * row_len;
    }
    const size_t o = ((size_t)b * T + s) * W;
    const int nk = step_wave(sa, v, cand, order, kept, W, [&](int x, const Cand& r) {
      a.prediction[o + x] = r.pred;
      a.log_prob[o + x] = r.lp;
      a.next_t[o + x] = (int)(unsigned)r.nt;
      a.next_u[o + x] = (int)(unsigned)r.nu;
      a.next_fin[o + x] = r.fin != 0;
      a.beam_branch[o + x] = r.parent;
      if (V == Variant::V2) a.next_total[o + x] = r.tot;
      st_hist[W + x] = r.lp;
      st_t[W + x] = (int)(unsigned)r.nt;
      st_u[W + x] = (int)(unsigned)r.nu;
      st_tot[W + x] = r.tot;
      st_fin[W + x] = r.fin != 0;
    });
    if (nk == 0) {
      if (lane == 0 && a.status) atomicOr(a.status, kStatusNoCandidate);
      return;
    }
    __syncthreads();
    for (int x = lane; x < W; x += 64) {
      st_hist[x] = st_hist[W + x]; st_t[x] = st_t[W + x]; st_u[x] = st_u[W + x];
      st_tot[x] = st_tot[W + x]; st_fin[x] = st_fin[W + x];
    }
    __syncthreads();
  }
}

// Backtrace over the global per-step outputs, one thread per (utterance, final slot): the path
// outputs of k_fused_lds, and of k_fused_reg when its history does not fit LDS.
__global__ __launch_bounds__(64) void k_fused_paths(FusedDecodeArgs a) {
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  const int W = a.W, T = a.T;
  if (id >= a.B * W) return;
  const int b = id / W, w = id - b * W;
  int* ord = a.ordered ? a.ordered + ((size_t)b * W + w) * T : nullptr;
  int* pp = a.path_pred ? a.path_pred + ((size_t)b * W + w) * T : nullptr;
  int* du = a.duration ? a.duration + ((size_t)b * W + w) * T : nullptr;
  const bool best = w == 0 && a.best_beam_branch;
  bool bad = false;
  int cur = w;
  for (int s = T - 1; s >= 0; --s) {
    const size_t o = ((size_t)b * T + s) * W;
    int parent = a.beam_branch[o + cur];
    if (parent < 0 || parent >= W) {  // only after "no candidate" left this utterance unwritten
      bad = true;
      parent = 0;
    }
    if (ord) ord[s] = cur;
    if (pp) pp[s] = a.prediction[o + cur];
    if (du) du[s] = a.next_total[o + cur] - (s > 0 ? a.next_total[o - W + parent] : 0);
    if (best) {
      a.best_beam_branch[(size_t)b * T + s] = cur;
      a.best_t_history[(size_t)b * T + s] = a.next_t[o + cur];
    }
    cur = parent;
  }
  if (bad && a.status) atomicOr(a.status, kStatusBadIndex);
}

inline int last_error() { return hipGetLastError() == hipSuccess ? SSNT_OK : SSNT_ERR_HIP; }

constexpr size_t kMaxLds = 150 * 1024;

// ordering of the register kernel's step: the full rank. The selection ordering (SEL) is
// bit-identical and measured slower at every BASELINE shape; it is compiled
// only into the A/B build (-DSSNT_AB: ssnt_fused_decode_select 0 full rank, 1 selection).
// waves of tone's replicated rank (1, 2 or 4); the A/B build can override it per process. One:
// at configs[4] two waves measured 202 us and four 215 us against 189 us for one
// (profiles/r5b_tone_waves.json) -- the step's LDS round trips, not its 16 compares, set it
constexpr int kToneWaves = 1;
#ifdef SSNT_AB
std::atomic<int> g_select{-1};
bool use_select() { return g_select.load(std::memory_order_relaxed) == 1; }
std::atomic<int> g_tone_waves{-1};
int tone_waves() {
  const int t = g_tone_waves.load(std::memory_order_relaxed);
  return t > 0 ? t : kToneWaves;
}
#define SSNT_SEL_OR_RANK(sel, RANK, SELK) ((sel) ? (SELK) : (RANK))
#else
constexpr bool use_select() { return false; }
constexpr int tone_waves() { return kToneWaves; }
#define SSNT_SEL_OR_RANK(sel, RANK, SELK) (RANK)
#endif

template <typename K>
int launch_with_lds(K kernel, size_t lds, int B, hipStream_t st, const FusedDecodeArgs& a,
                    int extra, int waves = 1) {
  if (lds > 64 * 1024)  // per launch: the attribute is per device, and cheap to set
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds);
  hipLaunchKernelGGL(kernel, dim3(B), dim3(64 * waves), lds, st, a, extra);
  return last_error();
}

template <Variant V>
int launch_variant(const FusedDecodeArgs& a, hipStream_t st) {
  const int C = V == Variant::V1 ? 2 : a.C;
  const int n = a.W * C;
  const bool want_paths = a.ordered || a.path_pred || a.duration || a.best_beam_branch;
  bool paths_kernel = want_paths;
  int rc = SSNT_OK;
  if (n <= 64) {
    const bool staged = V != Variant::V1 || 2 * (size_t)a.U <= 64 * (size_t)kV1Regs;
    const bool sel = use_select();
    const int nmax = n <= 8 ? 8 : n <= 16 ? 16 : n <= 32 ? 32 : 64;
    const int tw = V == Variant::Tone ? tone_waves() : 1;
    const int nw = staged ? fused_waves(V, nmax, sel, tw) : 1;
    const bool whole = RegLayout(V, a.W, a.T, a.U, true, staged, true, nw).total <= kMaxLds;
    const bool hist_lds = whole || RegLayout(V, a.W, a.T, a.U, true, staged, false, nw).total <= kMaxLds;
    const size_t lds = RegLayout(V, a.W, a.T, a.U, hist_lds, staged, whole, nw).total;
    if (lds > kMaxLds) return SSNT_ERR_UNSUPPORTED;
    const int h = hist_lds ? 1 : 0;
    auto go = [&](auto kw, auto kc) {  // (NMAX, WHOLE) instance
      constexpr int NM = decltype(kw)::value;
      constexpr bool WH = decltype(kc)::value;
      if (!staged) {  // only v1 rows can be too long to stage
        if constexpr (V == Variant::V1) {
          return SSNT_SEL_OR_RANK(sel, launch_with_lds(k_fused_reg<V, false, 64, WH, false>, lds, a.B, st, a, h),
                                  launch_with_lds(k_fused_reg<V, false, 64, WH, true>, lds, a.B, st, a, h));
        }
        return (int)SSNT_ERR_UNSUPPORTED;
      }
#ifdef SSNT_AB
      if constexpr (V == Variant::Tone && NM == 32) {  // (A/B study forms; measured slower)
        if (!sel && tw == 2)
          return launch_with_lds(k_fused_reg<V, true, NM, WH, false, 2>, lds, a.B, st, a, h, 2);
        if (!sel && tw == 4)
          return launch_with_lds(k_fused_reg<V, true, NM, WH, false, 4>, lds, a.B, st, a, h, 4);
      }
#endif
      return SSNT_SEL_OR_RANK(sel, launch_with_lds(k_fused_reg<V, true, NM, WH, false>, lds, a.B, st, a, h,
                                                   fused_waves(V, NM, false)),
                              launch_with_lds(k_fused_reg<V, true, NM, WH, true>, lds, a.B, st, a, h,
                                              fused_waves(V, NM, true)));
    };
    auto pick = [&](auto kc) {
      if (n <= 8) return go(std::integral_constant<int, 8>{}, kc);
      if (n <= 16) return go(std::integral_constant<int, 16>{}, kc);
      if (n <= 32) return go(std::integral_constant<int, 32>{}, kc);
      return go(std::integral_constant<int, 64>{}, kc);
    };
    rc = whole ? pick(std::true_type{}) : pick(std::false_type{});
    paths_kernel = want_paths && !hist_lds;
  } else {
    const size_t lds = (size_t)n * sizeof(Cand) + 2 * (size_t)n * 4 + (size_t)a.W * 2 * 16 +
                       (V == Variant::V1 ? (size_t)a.W * 8 : 0) + 2 * (size_t)a.W + 16;
    if (lds > kMaxLds) return SSNT_ERR_UNSUPPORTED;
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_fused_lds<V>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds);
    hipLaunchKernelGGL(k_fused_lds<V>, dim3(a.B), dim3(64), lds, st, a);
    rc = last_error();
  }
  if (rc != SSNT_OK || !paths_kernel) return rc;
  const int threads = a.B * a.W;
  hipLaunchKernelGGL(k_fused_paths, dim3((threads + 63) / 64), dim3(64), 0, st, a);
  return last_error();
}

}  // namespace

int diag_decode_read(void* host, size_t bytes) {
#ifdef SSNT_DIAG
  if (bytes > sizeof(g_dec_diag)) bytes = sizeof(g_dec_diag);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dec_diag), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? (int)bytes : -1;
#else
  (void)host;
  (void)bytes;
  return -1;
#endif
}

#ifdef SSNT_AB
int set_fused_decode_select(int mode) {
  if (mode < -1 || mode > 1) return SSNT_ERR_INVALID_ARG;
  g_select.store(mode);
  return SSNT_OK;
}
int set_fused_decode_tone_waves(int n) {
  if (n != -1 && n != 1 && n != 2 && n != 4) return SSNT_ERR_INVALID_ARG;
  g_tone_waves.store(n);
  return SSNT_OK;
}
#endif

int launch_fused_decode(const FusedDecodeArgs& a, hipStream_t st) {
  if (a.B < 0 || a.W <= 0 || a.T <= 0 || !a.src || !a.input_length || !a.prediction ||
      !a.log_prob || !a.next_t || !a.next_u || !a.next_fin || !a.beam_branch)
    return SSNT_ERR_INVALID_ARG;
  // packed (next_t, next_u) in 16 bits each: every value stays <= T in a fused decode
  if (a.T > 32767) return SSNT_ERR_UNSUPPORTED;
  if ((a.best_beam_branch == nullptr) != (a.best_t_history == nullptr)) return SSNT_ERR_INVALID_ARG;
  switch (a.variant) {
    case Variant::V1:
      if (a.U <= 0 || a.C != 2 || a.path_pred || a.duration) return SSNT_ERR_INVALID_ARG;
      if (a.W > 64) return SSNT_ERR_UNSUPPORTED;
      break;
    case Variant::V2:
      if (a.C <= 0 || !a.table || !a.output_length || !a.next_total) return SSNT_ERR_INVALID_ARG;
      if (a.best_beam_branch) return SSNT_ERR_INVALID_ARG;
      break;
    case Variant::Tone:
      if (a.C <= 0 || a.duration || a.best_beam_branch) return SSNT_ERR_INVALID_ARG;
      break;
  }
  if (a.B == 0) return SSNT_OK;
  switch (a.variant) {
    case Variant::V1: return launch_variant<Variant::V1>(a, st);
    case Variant::V2: return launch_variant<Variant::V2>(a, st);
    default: return launch_variant<Variant::Tone>(a, st);
  }
}

}  // namespace ssnt
