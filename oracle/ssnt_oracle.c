/*
 * ssnt_oracle.c -- CPU ORACLE. TEST INFRASTRUCTURE ONLY.
 *
 * This file is the checker, never the product. Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it (through oracle/oracle.py). The product path
 * (ssnt-tts-rust_amd/, libssnt_tts_c.so) never links, loads or calls anything in oracle/.
 *
 * What it is: a plain-C restatement of the reference hot path of nii-yamagishilab/ssnt-tts-rust
 * (Rust; cargo/rustc are absent in this image so the reference itself cannot be built -- see
 * DESIGN.md "Oracle"). Every function cites the reference file:line it restates.
 *
 *   decode (bit-exact integer/f32-add work)    -> src/lib.rs, src/v2.rs, src/tone_latent.rs
 *   backtraces                                 -> src/util.rs, src/v2_util.rs
 *   upsample / edit distance ("next" rows)     -> src/v2_util.rs, src/edit_distance.rs
 *   forward-backward lattice (A11)             -> NOT in the reference;
 *       semantics derived from the emit/shift transition rules of src/lib.rs:186-226 and
 *       defined in DESIGN.md. Two forms:
 *         oracle_fwd_bwd_xf  : the exact split-exponent f32 arithmetic the GPU kernel must
 *                              reproduce bit for bit;
 *         oracle_fwd_bwd_f64 : an independent log-domain float64 DP (the mathematical truth)
 *                              used to pin the f32 arithmetic (tolerance in tests/).
 *
 * Parity pins: tests/test_oracle_golden.py checks this file against every known answer the
 * reference's own tests hold (tests/test_decoding.rs:120-130, tests/test_edit_distance.rs,
 * ssnt-tts-tensorflow/tests/test_upsample_source_indexes.py:40-53) and the derived answers of
 * SURVEY.md Appendix B. v2 / tone_latent / fwd-bwd have no reference fixtures ("parity
 * unpinned" by the reference; fwd-bwd pinned by f64 DP + brute-force path enumeration).
 *
 * Build: gcc -O3 -fopenmp -ffp-contract=off -fPIC -shared (see Makefile). -ffp-contract=off is
 * REQUIRED: a contracted a*b+c would break bit-exactness with the device code.
 */
#include <math.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_OK 0
#define ORC_ERR_NO_CANDIDATE 3
#define ORC_ERR_DURATION_MISMATCH 4
#define ORC_ERR_INVALID 1

/* ------------------------------------------------------------------------------------------
 * Decode: candidate record (src/lib.rs:70-88, src/v2.rs:169-189, src/tone_latent.rs:98-101,208-234).
 * next_t / next_u are Rust `usize`: the i32 inputs are converted with `as usize` (sign
 * extension, src/lib.rs:135-136) and written back `as i32` (src/lib.rs:141-142).
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    int32_t pred;
    float lp;
    uint64_t next_t, next_u;
    bool fin;
    int32_t parent;
    int32_t tot; /* v2 only */
} cand_t;

static inline uint64_t as_usize(int32_t v) { return (uint64_t)(int64_t)v; }

/* Rust `f32 as i32`: saturating, NaN -> 0 (used by src/v2.rs:101-102). */
static inline int32_t f2i_sat(float x) {
    if (x != x) return 0;
    if (x >= 2147483648.0f) return INT32_MAX;
    if (x <= -2147483648.0f) return INT32_MIN;
    return (int32_t)x;
}

/* Sort key: the IEEE order of `partial_cmp` (src/lib.rs:161) -- -0 and +0 share a key --
 * extended to a total order with NaN below -inf (the GPU kernels use the same key). NaN keys are
 * outside the parity contract: Rust's result for them depends on its sort implementation. */
static inline uint32_t lp_key(float x) {
    if (x != x) return 1u;
    uint32_t bits;
    if (x == 0.0f) bits = 0u;
    else memcpy(&bits, &x, 4);
    return (bits & 0x80000000u) ? ~bits : (bits | 0x80000000u);
}

/* Stable sort by log_prob descending; `partial_cmp(..).unwrap_or(Equal).reverse()`
 * (src/lib.rs:161). Insertion sort = stable; element moves before its predecessor only when
 * its key is strictly greater. */
static void sort_desc_stable(cand_t *c, int n) {
    for (int i = 1; i < n; ++i) {
        cand_t x = c[i];
        const uint32_t kx = lp_key(x.lp);
        int j = i - 1;
        while (j >= 0 && lp_key(c[j].lp) < kx) {
            c[j + 1] = c[j];
            --j;
        }
        c[j + 1] = x;
    }
}

/* `eq_ignore_parent` (src/lib.rs:81-87; v2 adds total_duration, src/v2.rs:181-188). */
static inline bool eq_ignore_parent(const cand_t *a, const cand_t *b, bool with_tot) {
    return a->pred == b->pred && a->lp == b->lp && a->next_t == b->next_t &&
           a->next_u == b->next_u && a->fin == b->fin && (!with_tot || a->tot == b->tot);
}

/* Vec::dedup_by keeps the first of each run of consecutive equal elements (src/lib.rs:162). */
static int dedup(cand_t *c, int n, bool with_tot) {
    if (n == 0) return 0;
    int k = 1;
    for (int i = 1; i < n; ++i)
        if (!eq_ignore_parent(&c[i], &c[k - 1], with_tot)) c[k++] = c[i];
    return k;
}

/* ---------------------------- v1 (src/lib.rs:121-230) ---------------------------------- */
/* beam_search_kernel_internal, src/lib.rs:172-230. */
static int v1_internal(const float *h, const float *hist, const bool *fin, uint64_t input_length,
                       int w, uint64_t t, uint64_t u, cand_t *out) {
    /* decode_beam_at (src/lib.rs:57-67): defined iff t < input_length and not finished. */
    if (!(t < input_length) || fin[w]) {
        out[0] = (cand_t){0, hist[w], t, u, true, w, 0};
        return 1;
    }
    const uint64_t last = input_length - 1; /* usize arithmetic, src/lib.rs:187 */
    for (int k = 0; k < 2; ++k) {
        const float v = h[w * 2 + k];
        if (k == 0 && t == last)
            out[k] = (cand_t){0, hist[w] + v, t, u, true, w, 0};
        else if (k == 1 && t == last) /* prohibited shift, src/lib.rs:196-205 */
            out[k] = (cand_t){0, hist[w], t, u, true, w, 0};
        else if (k == 1)
            out[k] = (cand_t){1, hist[w] + v, t + 1, u + 1, false, w, 0};
        else
            out[k] = (cand_t){0, hist[w] + v, t, u + 1, false, w, 0};
    }
    return 2;
}

/* beam_search_kernel (src/lib.rs:149-170) for one batch element. */
static void v1_kernel(const float *h, const float *hist, const bool *fin, const int32_t *t,
                      const int32_t *u, uint64_t input_length, int W, int Wmax, cand_t *buf,
                      cand_t *res) {
    int n = 0;
    for (int w = 0; w < W; ++w)
        n += v1_internal(h, hist, fin, input_length, w, as_usize(t[w]), as_usize(u[w]), buf + n);
    sort_desc_stable(buf, n);
    n = dedup(buf, n, false);
    /* pad: results.push(results[i]) while growing == cyclic copy (src/lib.rs:163-167) */
    for (int i = 0; i < Wmax; ++i) res[i] = buf[i % n];
}

static void write_results(const cand_t *res, int Wmax, int32_t *prediction, float *log_probs,
                          int32_t *next_t, int32_t *next_u, bool *next_fin, int32_t *next_tot,
                          int32_t *beam_branch) {
    for (int i = 0; i < Wmax; ++i) { /* src/lib.rs:138-145 */
        prediction[i] = res[i].pred;
        log_probs[i] = res[i].lp;
        next_t[i] = (int32_t)(uint32_t)res[i].next_t;
        next_u[i] = (int32_t)(uint32_t)res[i].next_u;
        beam_branch[i] = res[i].parent;
        next_fin[i] = res[i].fin;
        if (next_tot) next_tot[i] = res[i].tot;
    }
}

/* Batched v1 step: SsntTtsCpu::beam_search_decode (src/lib.rs:121-147). The reference takes one
 * input_length for the batch (src/lib.rs:99,134); here it is per batch element (all equal
 * reproduces the reference exactly). Inputs: h (B,W,2), state (B,W); outputs (B,Wmax). */
int oracle_v1_step(int B, int W, int Wmax, const float *h, const float *hist, const bool *fin,
                   const int32_t *t, const int32_t *u, const int32_t *input_length,
                   int32_t *prediction, float *log_probs, int32_t *next_t, int32_t *next_u,
                   bool *next_fin, int32_t *beam_branch) {
    if (W <= 0 || Wmax <= 0) return ORC_ERR_INVALID;
    cand_t *buf = (cand_t *)malloc(sizeof(cand_t) * (2 * W + Wmax));
    cand_t *res = buf + 2 * W;
    for (int b = 0; b < B; ++b) {
        v1_kernel(h + (size_t)b * W * 2, hist + (size_t)b * W, fin + (size_t)b * W,
                  t + (size_t)b * W, u + (size_t)b * W, as_usize(input_length[b]), W, Wmax, buf,
                  res);
        const size_t o = (size_t)b * Wmax;
        write_results(res, Wmax, prediction + o, log_probs + o, next_t + o, next_u + o,
                      next_fin + o, NULL, beam_branch + o);
    }
    free(buf);
    return ORC_OK;
}

/* ---------------------------- v2 (src/v2.rs:94-339) ------------------------------------ */
typedef struct {
    uint64_t I, O; /* input_length, output_length as usize (src/v2.rs:249-250) */
    const int32_t *total, *table;
    int D, zid;
    bool allow_skip, test_mode;
} v2_ctx;

/* total_duration_bounds, src/v2.rs:94-104 (f32 arithmetic, 0.1 / 0.05 are f32 literals). */
static void v2_bounds(const v2_ctx *c, uint64_t t, int32_t *lb, int32_t *ub) {
    const float diagonal = (float)c->O / (float)c->I * (float)(t + 1);
    const float upper_range = (float)c->O * 0.1f;
    const float lower_range = (float)c->O * 0.05f;
    *lb = f2i_sat(fmaxf(diagonal - lower_range, 0.0f));
    *ub = f2i_sat(fminf(diagonal + upper_range, (float)c->O));
}

/* will_overrun, src/v2.rs:106-111. */
static bool v2_will_overrun(const v2_ctx *c, uint64_t t) {
    const uint64_t remaining = c->I - (t + 1);
    return remaining * 3 > c->O;
}

/* on_diagonal, src/v2.rs:113-117. */
static bool v2_on_diagonal(const v2_ctx *c, const cand_t *r) {
    const float diagonal = (float)c->O / (float)c->I * (float)r->next_t;
    const float diff = (float)r->tot - diagonal;
    return diff >= -20.0f && diff <= 0.0f;
}

/* decode_beam_at (src/v2.rs:119-166) + beam_search_kernel_internal (src/v2.rs:311-339). */
static int v2_internal(const v2_ctx *c, const float *h, const float *hist, const bool *fin, int w,
                       uint64_t t, uint64_t u, cand_t *out) {
    if (!(t < c->I) || fin[w]) {
        out[0] = (cand_t){c->zid, hist[w], t, u, true, w, c->total[w]};
        return 1;
    }
    int n = 0;
    int32_t lb, ub;
    v2_bounds(c, t, &lb, &ub);
    const bool overrun = v2_will_overrun(c, t);
    for (int i = 0; i < c->D; ++i) {
        const float v = h[w * c->D + i];
        const int32_t duration = c->table[i];
        const int32_t tot = (int32_t)((uint32_t)c->total[w] + (uint32_t)duration);
        bool is_fin;
        if (!c->test_mode && (tot < lb || tot > ub)) continue;
        if (!c->test_mode && overrun) continue;
        if (t == c->I - 1) {
            if (!c->test_mode && tot != (int32_t)c->O) continue;
            if (!c->allow_skip && i == c->zid) continue;
            is_fin = true;
        } else {
            if (!c->allow_skip && i == c->zid) continue;
            is_fin = false;
        }
        out[n++] = (cand_t){i,        hist[w] + v, is_fin ? t : t + 1, is_fin ? u : u + 1,
                            is_fin, w,           tot};
    }
    return n;
}

/* One batch element of the v2 step: beam_search_kernel (src/v2.rs:269-309) over the W beams.
 * buf holds W*D + W candidates, res Wmax. Returns 0, or ORC_ERR_NO_CANDIDATE where the reference
 * panics (assert_ne!(n_results, 0), src/v2.rs:292). */
static int v2_step_one(const v2_ctx *c, int W, int Wmax, const float *hb, const float *hist,
                       const bool *fin, const int32_t *t, const int32_t *u, cand_t *buf,
                       cand_t *res) {
    int n = 0;
    for (int w = 0; w < W; ++w)
        n += v2_internal(c, hb, hist, fin, w, as_usize(t[w]), as_usize(u[w]), buf + n);
    sort_desc_stable(buf, n);
    n = dedup(buf, n, true);
    int diag = -1; /* src/v2.rs:283-289: first sorted+deduped candidate on the diagonal */
    if (!c->test_mode)
        for (int i = 0; i < n; ++i)
            if (v2_on_diagonal(c, &buf[i])) {
                diag = i;
                break;
            }
    if (n == 0) return ORC_ERR_NO_CANDIDATE;
    for (int i = 0; i < Wmax; ++i) res[i] = buf[i % n]; /* src/v2.rs:293-297 */
    if (diag >= 0) res[Wmax - 1] = buf[diag];             /* src/v2.rs:298-303 */
    return ORC_OK;
}

/* Batched v2 step: SsntTtsV2Cpu::beam_search_decode (src/v2.rs:221-309). */
int oracle_v2_step(int B, int W, int Wmax, int D, const float *h, const float *hist,
                   const bool *fin, const int32_t *total, const int32_t *table, const int32_t *t,
                   const int32_t *u, const int32_t *input_length, const int32_t *output_length,
                   int zero_duration_id, bool allow_skip, bool test_mode, int32_t *prediction,
                   float *log_probs, int32_t *next_t, int32_t *next_u, bool *next_fin,
                   int32_t *next_tot, int32_t *beam_branch) {
    if (W <= 0 || Wmax <= 0 || D <= 0) return ORC_ERR_INVALID;
    cand_t *buf = (cand_t *)malloc(sizeof(cand_t) * ((size_t)W * D + W + Wmax));
    cand_t *res = buf + (size_t)W * D + W;
    int status = ORC_OK;
    for (int b = 0; b < B; ++b) {
        v2_ctx c = {as_usize(input_length[b]), as_usize(output_length[b]), total + (size_t)b * W,
                    table, D, zero_duration_id, allow_skip, test_mode};
        const size_t o = (size_t)b * W;
        if (v2_step_one(&c, W, Wmax, h + o * D, hist + o, fin + o, t + o, u + o, buf, res) != ORC_OK) {
            status = ORC_ERR_NO_CANDIDATE;
            continue;
        }
        const size_t ow = (size_t)b * Wmax;
        write_results(res, Wmax, prediction + ow, log_probs + ow, next_t + ow, next_u + ow,
                      next_fin + ow, next_tot + ow, beam_branch + ow);
    }
    free(buf);
    return status;
}

/* ---------------------------- tone latent (src/tone_latent.rs:144-234) ------------------ */
/* One batch element: beam_search_kernel (src/tone_latent.rs:184-206). */
static void tone_step_one(uint64_t I, int W, int Wmax, int C, const float *hb, const float *hi,
                          const bool *fb, const int32_t *t, const int32_t *u, int empty_tone_id,
                          cand_t *buf, cand_t *res) {
    int n = 0;
    for (int w = 0; w < W; ++w) {
        const uint64_t tw = as_usize(t[w]), uw = as_usize(u[w]);
        /* decode_beam_at (src/tone_latent.rs:79-96): undefined past the input or finished ->
         * one finished "padding" candidate (src/tone_latent.rs:212-219) */
        if (!(tw < I) || fb[w]) {
            buf[n++] = (cand_t){empty_tone_id, hi[w], tw, uw, true, w, 0};
            continue;
        }
        /* every class, never finished (src/tone_latent.rs:87-93, 220-231) */
        for (int i = 0; i < C; ++i)
            buf[n++] = (cand_t){i, hi[w] + hb[w * C + i], tw + 1, uw + 1, false, w, 0};
    }
    sort_desc_stable(buf, n);
    n = dedup(buf, n, false);
    for (int i = 0; i < Wmax; ++i) res[i] = buf[i % n];
}

int oracle_tone_step(int B, int W, int Wmax, int C, const float *h, const float *hist,
                     const bool *fin, const int32_t *t, const int32_t *u,
                     const int32_t *input_length, int empty_tone_id, int32_t *prediction,
                     float *log_probs, int32_t *next_t, int32_t *next_u, bool *next_fin,
                     int32_t *beam_branch) {
    if (W <= 0 || Wmax <= 0 || C <= 0) return ORC_ERR_INVALID;
    cand_t *buf = (cand_t *)malloc(sizeof(cand_t) * ((size_t)W * C + W + Wmax));
    cand_t *res = buf + (size_t)W * C + W;
    for (int b = 0; b < B; ++b) {
        const size_t o = (size_t)b * W;
        tone_step_one(as_usize(input_length[b]), W, Wmax, C, h + o * C, hist + o, fin + o, t + o,
                      u + o, empty_tone_id, buf, res);
        const size_t ow = (size_t)b * Wmax;
        write_results(res, Wmax, prediction + ow, log_probs + ow, next_t + ow, next_u + ow,
                      next_fin + ow, NULL, beam_branch + ow);
    }
    free(buf);
    return ORC_OK;
}

/* ---------------------------- backtraces ------------------------------------------------ */
/* util::extract_best_beam_branch_kernel, src/util.rs:20-33 (rfold over (U,W) rows). */
void oracle_extract_best_beam_branch(int best_final_branch, const int32_t *beam_branch,
                                     const int32_t *t_history, int W, int max_u,
                                     int32_t *best_beam_branch, int32_t *best_t_history) {
    int32_t cur = best_final_branch;
    for (int uu = max_u - 1; uu >= 0; --uu) {
        best_beam_branch[uu] = cur;
        best_t_history[uu] = t_history[(size_t)uu * W + cur];
        cur = beam_branch[(size_t)uu * W + cur];
    }
}

/* v2_util::order_beam_branch, src/v2_util.rs:6-36: final_branch (B,W), beam_branch (B,T,W)
 * -> ordered (B,W,T). */
void oracle_order_beam_branch(int B, int W, int T, const int32_t *final_branch,
                              const int32_t *beam_branch, int32_t *ordered) {
    for (int b = 0; b < B; ++b)
        for (int w = 0; w < W; ++w) {
            int32_t cur = final_branch[(size_t)b * W + w];
            int32_t *o = ordered + ((size_t)b * W + w) * T;
            const int32_t *bb = beam_branch + (size_t)b * T * W;
            for (int s = T - 1; s >= 0; --s) {
                o[s] = cur;
                cur = bb[(size_t)s * W + cur];
            }
        }
}

/* v2_util::upsample_source_indexes, src/v2_util.rs:39-66: durations (B,W,T) -> (B,W,max_u);
 * only the first output_length[b,w] entries of each row are written (the TF op prefills the
 * rest, upsample_source_indexes_op.cc:75,90-92). Sum mismatch -> assert panic (:58). */
int oracle_upsample_source_indexes(int B, int W, int T, int max_u, const int32_t *duration,
                                   const int32_t *output_length, int32_t *out) {
    int status = ORC_OK;
    for (int r = 0; r < B * W; ++r) {
        const int32_t *d = duration + (size_t)r * T;
        int64_t total = 0;
        for (int t = 0; t < T; ++t) {
            if (d[t] < 0) return ORC_ERR_DURATION_MISMATCH;
            total += d[t];
        }
        if (total != (int64_t)output_length[r]) {
            status = ORC_ERR_DURATION_MISMATCH;
            continue;
        }
        int32_t *o = out + (size_t)r * max_u;
        int64_t k = 0;
        for (int t = 0; t < T; ++t)
            for (int j = 0; j < d[t]; ++j, ++k)
                if (k < max_u) o[k] = t;
    }
    return status;
}

/* edit_distance::levenshtein_edit_distance(_kernel), src/edit_distance.rs:6-60 (Kaldi). */
void oracle_levenshtein(int B, int max_length, const int32_t *a, const int32_t *b,
                        const int32_t *a_len, const int32_t *b_len, int32_t *dist) {
    int32_t *e = (int32_t *)malloc(sizeof(int32_t) * (max_length + 1) * 2);
    for (int i = 0; i < B; ++i) {
        const int32_t *A = a + (size_t)i * max_length, *Bv = b + (size_t)i * max_length;
        const int M = a_len[i], N = b_len[i];
        int32_t *cur = e, *nxt = e + max_length + 1;
        for (int n = 0; n <= N; ++n) cur[n] = n;
        for (int m = 1; m <= M; ++m) {
            nxt[0] = cur[0] + 1;
            for (int n = 1; n <= N; ++n) {
                int32_t t1 = cur[n - 1] + (A[m - 1] == Bv[n - 1] ? 0 : 1);
                int32_t t2 = cur[n] + 1, t3 = nxt[n - 1] + 1;
                int32_t mn = t2 < t3 ? t2 : t3;
                nxt[n] = t1 < mn ? t1 : mn;
            }
            int32_t *tmp = cur; cur = nxt; nxt = tmp;
        }
        dist[i] = cur[N];
    }
    free(e);
}

/* Fused multi-step v1 lattice decode (the config-3 workload): all beams start
 * at (t=0,u=0, hist=0); step s reads h[b,w] = lattice[b, u_w, t_w, :] for beams that are
 * defined, runs the exact v1 step (Wmax = W), records every per-step output, then backtraces
 * the best final beam (slot 0 after the final sort) with util::extract_best_beam_branch
 * semantics, t_history = next_t history. lattice (B,T,U,2); outputs (B,T,W) and (B,T). */
int oracle_v1_lattice_decode(int B, int T, int U, int W, const float *lattice,
                             const int32_t *input_length, int32_t *pred, float *lp,
                             int32_t *next_t, int32_t *next_u, bool *fin, int32_t *branch,
                             int32_t *best_branch, int32_t *best_t, int n_threads) {
    if (W <= 0 || T <= 0) return ORC_ERR_INVALID;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic)
#endif
    for (int b = 0; b < B; ++b) {
        float *h = (float *)malloc(sizeof(float) * 2 * W);
        float *hist = (float *)calloc(W, sizeof(float));
        bool *f = (bool *)calloc(W, sizeof(bool));
        int32_t *tt = (int32_t *)calloc(W, sizeof(int32_t));
        int32_t *uu = (int32_t *)calloc(W, sizeof(int32_t));
        cand_t *buf = (cand_t *)malloc(sizeof(cand_t) * 3 * W);
        const uint64_t I = as_usize(input_length[b]);
        const float *lat = lattice + (size_t)b * T * U * 2;
        for (int s = 0; s < T; ++s) {
            for (int w = 0; w < W; ++w) {
                const bool defined = !f[w] && as_usize(tt[w]) < I && (uint32_t)uu[w] < (uint32_t)T &&
                                     (uint32_t)tt[w] < (uint32_t)U;
                const float *src = lat + ((size_t)(defined ? uu[w] : 0) * U + (defined ? tt[w] : 0)) * 2;
                h[2 * w] = defined ? src[0] : 0.0f;
                h[2 * w + 1] = defined ? src[1] : 0.0f;
            }
            cand_t *res = buf + 2 * W;
            v1_kernel(h, hist, f, tt, uu, I, W, W, buf, res);
            const size_t o = ((size_t)b * T + s) * W;
            write_results(res, W, pred + o, lp + o, next_t + o, next_u + o, fin + o, NULL,
                          branch + o);
            for (int w = 0; w < W; ++w) {
                hist[w] = lp[o + w];
                f[w] = fin[o + w];
                tt[w] = next_t[o + w];
                uu[w] = next_u[o + w];
            }
        }
        oracle_extract_best_beam_branch(0, branch + (size_t)b * T * W, next_t + (size_t)b * T * W,
                                        W, T, best_branch + (size_t)b * T, best_t + (size_t)b * T);
        free(h); free(hist); free(f); free(tt); free(uu); free(buf);
    }
    return ORC_OK;
}

/* Backtrace of every final slot w (v2_util::order_beam_branch, src/v2_util.rs:6-36, with
 * final_branch = [0..W)) plus the per-path class sequence and, when tot is given, the duration
 * each step added along the path (next_total_duration of the slot minus that of its parent;
 * initial totals are 0). Outputs (W,T) rows of one batch element. */
static void fused_paths(int T, int W, const int32_t *pred, const int32_t *branch,
                        const int32_t *tot, int32_t *ordered, int32_t *path_pred,
                        int32_t *duration) {
    for (int w = 0; w < W; ++w) {
        int32_t cur = w;
        for (int s = T - 1; s >= 0; --s) {
            const int32_t parent = branch[(size_t)s * W + cur];
            if (ordered) ordered[(size_t)w * T + s] = cur;
            if (path_pred) path_pred[(size_t)w * T + s] = pred[(size_t)s * W + cur];
            if (duration)
                duration[(size_t)w * T + s] =
                    tot[(size_t)s * W + cur] - (s > 0 ? tot[(size_t)(s - 1) * W + parent] : 0);
            cur = parent;
        }
    }
}

/* Fused multi-step v2 decode (BASELINE configs[4] "v2 path"): every beam starts at t=u=0,
 * log-prob 0, total_duration 0, not finished; step s runs the exact v2 step
 * (src/v2.rs:221-339, Wmax = W) with h = logits[b, s] (W,D) -- the per-step op's input, replayed
 * from a precomputed (B,T,W,D) tensor -- and feeds its outputs back as the next state (the TF
 * decode loop's role). Then fused_paths. An utterance that hits "no candidate" (the reference
 * panics, src/v2.rs:292) stops there; the call returns ORC_ERR_NO_CANDIDATE and that
 * utterance's remaining outputs are unspecified. */
int oracle_v2_lattice_decode(int B, int T, int W, int D, const float *logits,
                             const int32_t *table, const int32_t *input_length,
                             const int32_t *output_length, int zero_duration_id, bool allow_skip,
                             bool test_mode, int32_t *pred, float *lp, int32_t *next_t,
                             int32_t *next_u, bool *fin, int32_t *tot, int32_t *branch,
                             int32_t *ordered, int32_t *path_pred, int32_t *duration,
                             int n_threads) {
    if (W <= 0 || D <= 0 || T <= 0) return ORC_ERR_INVALID;
    int status = ORC_OK;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic)
#endif
    for (int b = 0; b < B; ++b) {
        float *hist = (float *)calloc(W, sizeof(float));
        bool *f = (bool *)calloc(W, sizeof(bool));
        int32_t *tt = (int32_t *)calloc(W, sizeof(int32_t));
        int32_t *uu = (int32_t *)calloc(W, sizeof(int32_t));
        int32_t *total = (int32_t *)calloc(W, sizeof(int32_t));
        cand_t *buf = (cand_t *)malloc(sizeof(cand_t) * ((size_t)W * D + 2 * W));
        const v2_ctx c0 = {as_usize(input_length[b]), as_usize(output_length[b]), NULL, table, D,
                           zero_duration_id, allow_skip, test_mode};
        bool ok = true;
        for (int s = 0; s < T; ++s) {
            v2_ctx c = c0;
            c.total = total;
            cand_t *res = buf + (size_t)W * D + W;
            if (v2_step_one(&c, W, W, logits + ((size_t)b * T + s) * W * D, hist, f, tt, uu, buf,
                            res) != ORC_OK) {
                ok = false;
                break;
            }
            const size_t o = ((size_t)b * T + s) * W;
            write_results(res, W, pred + o, lp + o, next_t + o, next_u + o, fin + o, tot + o,
                          branch + o);
            for (int w = 0; w < W; ++w) {
                hist[w] = lp[o + w];
                f[w] = fin[o + w];
                tt[w] = next_t[o + w];
                uu[w] = next_u[o + w];
                total[w] = tot[o + w];
            }
        }
        if (ok) {
            const size_t o = (size_t)b * T * W;
            fused_paths(T, W, pred + o, branch + o, tot + o, ordered ? ordered + o : NULL,
                        path_pred ? path_pred + o : NULL, duration ? duration + o : NULL);
        } else {
#ifdef _OPENMP
#pragma omp atomic write
#endif
            status = ORC_ERR_NO_CANDIDATE;
        }
        free(hist); free(f); free(tt); free(uu); free(total); free(buf);
    }
    return status;
}

/* Fused multi-step tone-latent decode (BASELINE configs[4] "tone_latent path"): as
 * oracle_v2_lattice_decode with the tone step (src/tone_latent.rs:144-234), h = logits[b, s]
 * (W,C); then fused_paths (no durations). */
int oracle_tone_lattice_decode(int B, int T, int W, int C, const float *logits,
                               const int32_t *input_length, int empty_tone_id, int32_t *pred,
                               float *lp, int32_t *next_t, int32_t *next_u, bool *fin,
                               int32_t *branch, int32_t *ordered, int32_t *path_pred,
                               int n_threads) {
    if (W <= 0 || C <= 0 || T <= 0) return ORC_ERR_INVALID;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic)
#endif
    for (int b = 0; b < B; ++b) {
        float *hist = (float *)calloc(W, sizeof(float));
        bool *f = (bool *)calloc(W, sizeof(bool));
        int32_t *tt = (int32_t *)calloc(W, sizeof(int32_t));
        int32_t *uu = (int32_t *)calloc(W, sizeof(int32_t));
        cand_t *buf = (cand_t *)malloc(sizeof(cand_t) * ((size_t)W * C + 2 * W));
        const uint64_t I = as_usize(input_length[b]);
        for (int s = 0; s < T; ++s) {
            cand_t *res = buf + (size_t)W * C + W;
            tone_step_one(I, W, W, C, logits + ((size_t)b * T + s) * W * C, hist, f, tt, uu,
                          empty_tone_id, buf, res);
            const size_t o = ((size_t)b * T + s) * W;
            write_results(res, W, pred + o, lp + o, next_t + o, next_u + o, fin + o, NULL,
                          branch + o);
            for (int w = 0; w < W; ++w) {
                hist[w] = lp[o + w];
                f[w] = fin[o + w];
                tt[w] = next_t[o + w];
                uu[w] = next_u[o + w];
            }
        }
        const size_t o = (size_t)b * T * W;
        fused_paths(T, W, pred + o, branch + o, NULL, ordered ? ordered + o : NULL,
                    path_pred ? path_pred + o : NULL, NULL);
        free(hist); free(f); free(tt); free(uu); free(buf);
    }
    return ORC_OK;
}

/* ==========================================================================================
 * Forward-backward emit/shift lattice (DESIGN.md "Lattice semantics").
 *
 * Lattice: utterance b has S steps (rows s = 0..S-1, the reference's decoder step u) and P
 * input positions (p = 0..P-1, the reference's t). log_trans[b,s,p,0] = log p(emit),
 * [..,1] = log p(shift) (src/lib.rs:14-15,65). Emit (s,p)->(s+1,p); shift (s,p)->(s+1,p+1)
 * (src/lib.rs:206-225); no shift out of the last position (src/lib.rs:196-205). alpha[0][0]=1.
 * Z = sum over monotone paths that reach p=P-1 at row S-1, times the terminal emit
 * exp(log_trans[S-1,P-1,0]) when FLAG_TERMINAL_EMIT (src/lib.rs:187-195). Optional log_obs[s,p]
 * multiplies every path entering cell (s,p). loss = -ln Z; grad = d loss / d log_trans (and
 * d loss / d log_obs). S < P (or Z == 0) is infeasible: loss = +inf (0 with
 * FLAG_ZERO_INFINITY), grads 0.
 * ========================================================================================== */
#define FLAG_TERMINAL_EMIT 1
#define FLAG_ZERO_INFINITY 2
/* --- split-exponent ("xf") f32 arithmetic: value = m * 2^e ------------------------------- */
typedef struct { float m; int32_t e; } xf;
#define XF_EZERO (-(1 << 29))
#define XF_LOG_MIN (-1.0e6f) /* log-probs below this (and NaN) are exact zeros */
#define XF_LOG_MAX (1.0e6f)

static const float L2E = 0x1.715476p+0f;
static const float LN2HI = 0x1.62e400p-1f;  /* 0x3f317200 */
static const float LN2LO = 0x1.7f7d1cp-20f; /* 0x35bfbe8e */
static const float SQRTH = 0x1.6a09e6p-1f;
/* e^r on [-ln2/2, ln2/2], deg 6, c0 = c1 = 1 and c2 = 1/2 exact, c3..c6 a relative-error minimax
 * fit (0.06 ulp of approximation error; tools/fit_exp_poly.py). The coefficients are fixed
 * constants of the arithmetic definition, shared with csrc/xf_math.h and csrc/lattice_dev.h.
 * Round 5 replaced a fit whose error curve had a one-sided bias (0.33 ulp at r = -0.3): over a
 * 2000-step lattice that bias accumulated to 1.1e-5 in log-alpha, past the north_star's 1e-5
 * (DESIGN.md 6.1). */
static const float EC[7] = {0x1p+0f, 0x1p+0f, 0x1p-1f, 0x1.5554a4p-3f, 0x1.555688p-5f,
                            0x1.122f66p-7f, 0x1.6b6ep-10f};
/* ln(1+t)/t on [sqrt(.5)-1, sqrt(2)-1], deg 8 */
static const float LC[9] = {0x1p+0f,         -0x1.fffff8p-2f, 0x1.55579p-2f,
                            -0x1.0005a6p-2f, 0x1.98b80ap-3f,  -0x1.5329bep-3f,
                            0x1.32285p-3f,   -0x1.26729ep-3f, 0x1.6626eap-4f};

static inline xf xf_norm(float s, int32_t e) {
    if (s == 0.0f) return (xf){0.0f, XF_EZERO};
    int k;
    const float m = frexpf(s, &k);
    return (xf){m, e + k};
}

/* exp(x) as an unnormalized xf: mantissa in [~0.707, ~1.414], Cody-Waite reduction. */
static inline xf xf_exp(float x, bool valid) {
    if (!valid || !(x >= XF_LOG_MIN)) return (xf){0.0f, XF_EZERO};
    if (x > XF_LOG_MAX) x = XF_LOG_MAX;
    const float n = rintf(x * L2E);
    float r = fmaf(-n, LN2HI, x);
    r = fmaf(-n, LN2LO, r);
    float p = EC[6];
    for (int i = 5; i >= 0; --i) p = fmaf(p, r, EC[i]);
    return (xf){p, (int32_t)n};
}

/* natural log of a normalized xf (xf_norm output). */
static inline float xf_log(xf v) {
    if (v.m == 0.0f) return -INFINITY;
    float m = v.m;
    int32_t e = v.e;
    if (m < SQRTH) { m = m * 2.0f; e -= 1; }
    const float t = m - 1.0f;
    float q = LC[8];
    for (int i = 7; i >= 0; --i) q = fmaf(q, t, LC[i]);
    const float lnm = t * q;
    const float ef = (float)e;
    return fmaf(ef, LN2HI, fmaf(ef, LN2LO, lnm));
}

/* a + b for (possibly unnormalized) a, b -> normalized */
static inline xf xf_add(float ma, int32_t ea, float mb, int32_t eb) {
    const int32_t em = ea > eb ? ea : eb;
    const float s = ldexpf(ma, ea - em) + ldexpf(mb, eb - em);
    return xf_norm(s, em);
}

static inline float xf_neg_post(float m, int32_t e) { return 0.0f - ldexpf(m, e); }


static void xf_fwd_bwd_one(const float *lt, const float *lo, int T, int U, int S, int P,
                           int flags, float *loss, float *g, float *go, float *la, float *lb,
                           xf *A, xf *Bt, xf *E, xf *Sh, xf *O, xf *st_a, xf *st_b, xf *st_z) {
    const bool term = (flags & FLAG_TERMINAL_EMIT) != 0;
    const size_t TU = (size_t)T * U;
    /* zero / -inf fill of every output cell (cells outside (S,P) keep these). */
    if (g) memset(g, 0, sizeof(float) * TU * 2);
    if (go) memset(go, 0, sizeof(float) * TU);
    for (size_t i = 0; la && i < TU; ++i) la[i] = -INFINITY;
    for (size_t i = 0; lb && i < TU; ++i) lb[i] = -INFINITY;
    for (size_t i = 0; st_a && i < TU; ++i) st_a[i] = (xf){0.0f, XF_EZERO};
    for (size_t i = 0; st_b && i < TU; ++i) st_b[i] = (xf){0.0f, XF_EZERO};
    if (st_z) *st_z = (xf){0.0f, XF_EZERO};
    const bool feasible = S >= 1 && P >= 1 && S <= T && P <= U && S >= P;
    if (!feasible) {
        *loss = (flags & FLAG_ZERO_INFINITY) ? 0.0f : INFINITY;
        return;
    }
    /* converted inputs; masks: p >= P zero, shift out of P-1 zero (src/lib.rs:196-205) */
    for (int s = 0; s < S; ++s)
        for (int p = 0; p < U; ++p) {
            const size_t c = (size_t)s * U + p;
            E[c] = xf_exp(lt[c * 2 + 0], p < P);
            Sh[c] = xf_exp(lt[c * 2 + 1], p < P - 1);
            O[c] = lo ? xf_exp(lo[c], p < P) : (xf){1.0f, 0};
        }
    /* alpha */
    for (int p = 0; p < U; ++p) A[p] = (xf){0.0f, XF_EZERO};
    A[0] = lo ? xf_norm(O[0].m, O[0].e) : (xf){0.5f, 1};
    for (int s = 1; s < S; ++s)
        for (int p = 0; p < U; ++p) {
            const xf a = A[(size_t)(s - 1) * U + p];
            const xf e = E[(size_t)(s - 1) * U + p];
            const float sm = a.m * e.m;
            const int32_t se = a.e + e.e;
            float hm = 0.0f;
            int32_t he = XF_EZERO;
            if (p > 0) {
                const xf al = A[(size_t)(s - 1) * U + p - 1];
                const xf sl = Sh[(size_t)(s - 1) * U + p - 1];
                hm = al.m * sl.m;
                he = al.e + sl.e;
            }
            const int32_t em = se > he ? se : he;
            float sum = ldexpf(sm, se - em) + ldexpf(hm, he - em);
            int32_t ee = em;
            if (lo) {
                const xf o = O[(size_t)s * U + p];
                sum = sum * o.m;
                ee = ee + o.e;
            }
            A[(size_t)s * U + p] = xf_norm(sum, ee);
        }
    /* beta */
    for (int p = 0; p < U; ++p) Bt[(size_t)(S - 1) * U + p] = (xf){0.0f, XF_EZERO};
    {
        const xf e = E[(size_t)(S - 1) * U + P - 1];
        Bt[(size_t)(S - 1) * U + P - 1] = term ? xf_norm(e.m, e.e) : (xf){0.5f, 1};
    }
    for (int s = S - 2; s >= 0; --s)
        for (int p = 0; p < U; ++p) {
            xf q = Bt[(size_t)(s + 1) * U + p], r = {0.0f, XF_EZERO};
            if (p + 1 < U) r = Bt[(size_t)(s + 1) * U + p + 1];
            if (lo) {
                const xf oq = O[(size_t)(s + 1) * U + p];
                q = (xf){q.m * oq.m, q.e + oq.e};
                if (p + 1 < U) {
                    const xf orr = O[(size_t)(s + 1) * U + p + 1];
                    r = (xf){r.m * orr.m, r.e + orr.e};
                }
            }
            const xf e = E[(size_t)s * U + p], sh = Sh[(size_t)s * U + p];
            Bt[(size_t)s * U + p] = xf_add(e.m * q.m, e.e + q.e, sh.m * r.m, sh.e + r.e);
        }
    /* Z at the cut M = (S-1)>>1: binary tree (pairs (2i,2i+1) first) over p in [0, 2^n). */
    const int M = (S - 1) >> 1;
    int n2 = 1;
    while (n2 < P) n2 <<= 1;
    xf *w = (xf *)malloc(sizeof(xf) * n2);
    for (int p = 0; p < n2; ++p) {
        if (p < P) {
            const xf a = A[(size_t)M * U + p], bb = Bt[(size_t)M * U + p];
            w[p] = (xf){a.m * bb.m, a.e + bb.e};
        } else
            w[p] = (xf){0.0f, XF_EZERO};
    }
    for (int len = n2; len > 1; len >>= 1)
        for (int i = 0; i < len / 2; ++i) w[i] = xf_add(w[2 * i].m, w[2 * i].e, w[2 * i + 1].m, w[2 * i + 1].e);
    xf Z = (n2 == 1) ? xf_norm(w[0].m, w[0].e) : w[0];
    free(w);
    if (st_z) *st_z = Z;
    if (Z.m == 0.0f) {
        *loss = (flags & FLAG_ZERO_INFINITY) ? 0.0f : INFINITY;
        return;
    }
    *loss = 0.0f - xf_log(Z);
    const float izm = 1.0f / Z.m;
    const int32_t ize = -Z.e;
    /* debug outputs */
    for (int s = 0; s < S; ++s)
        for (int p = 0; p < P; ++p) {
            if (la) la[(size_t)s * U + p] = xf_log(A[(size_t)s * U + p]);
            if (lb) lb[(size_t)s * U + p] = xf_log(Bt[(size_t)s * U + p]);
            if (st_a) st_a[(size_t)s * U + p] = A[(size_t)s * U + p];
            if (st_b) st_b[(size_t)s * U + p] = Bt[(size_t)s * U + p];
        }
    /* gradients */
    for (int s = 0; s < S; ++s)
        for (int p = 0; p < P; ++p) {
            const size_t c = (size_t)s * U + p;
            const xf a = A[c];
            xf q, r;
            if (s + 1 < S) {
                q = Bt[c + U];
                r = (p + 1 < U) ? Bt[c + U + 1] : (xf){0.0f, XF_EZERO};
                if (lo) {
                    const xf oq = O[c + U];
                    q = (xf){q.m * oq.m, q.e + oq.e};
                    if (p + 1 < U) {
                        const xf orr = O[c + U + 1];
                        r = (xf){r.m * orr.m, r.e + orr.e};
                    }
                }
            } else { /* terminal row: only the terminal emit at P-1 */
                q = (term && p == P - 1) ? (xf){1.0f, 0} : (xf){0.0f, XF_EZERO};
                r = (xf){0.0f, XF_EZERO};
            }
            const xf e = E[c], sh = Sh[c];
            g[c * 2 + 0] = xf_neg_post(((a.m * e.m) * q.m) * izm, a.e + e.e + q.e + ize);
            g[c * 2 + 1] = xf_neg_post(((a.m * sh.m) * r.m) * izm, a.e + sh.e + r.e + ize);
            if (go) {
                const xf bb = Bt[c];
                go[c] = xf_neg_post((a.m * bb.m) * izm, a.e + bb.e + ize);
            }
        }
}

/* Exact split-exponent fwd-bwd. log_trans (B,T,U,2); log_obs (B,T,U) or NULL; step_len /
 * pos_len (B). Outputs: loss (B); grad (B,T,U,2); grad_obs (B,T,U) or NULL; log_alpha /
 * log_beta (B,T,U) or NULL. n_threads <= 0: OpenMP default. */
int oracle_fwd_bwd_xf(int B, int T, int U, const float *log_trans, const float *log_obs,
                      const int32_t *step_len, const int32_t *pos_len, int flags, float *loss,
                      float *grad, float *grad_obs, float *log_alpha, float *log_beta,
                      int n_threads) {
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel
#endif
    {
        const size_t TU = (size_t)T * U;
        xf *buf = (xf *)malloc(sizeof(xf) * TU * 5);
#ifdef _OPENMP
#pragma omp for schedule(dynamic)
#endif
        for (int b = 0; b < B; ++b) {
            const size_t off = (size_t)b * TU;
            xf_fwd_bwd_one(log_trans + off * 2, log_obs ? log_obs + off : NULL, T, U, step_len[b],
                           pos_len[b], flags, loss + b, grad + off * 2,
                           grad_obs ? grad_obs + off : NULL, log_alpha ? log_alpha + off : NULL,
                           log_beta ? log_beta + off : NULL, buf, buf + TU, buf + 2 * TU,
                           buf + 3 * TU, buf + 4 * TU, NULL, NULL, NULL);
        }
        free(buf);
    }
    return ORC_OK;
}

/* The same computation, returning the normalized split-exponent state itself: alpha / beta
 * (B,T,U) and Z (B) as {m, e} pairs (m in [0.5, 1) or the zero {0, XF_EZERO}; cells outside
 * (S,P) and rows of infeasible utterances are zeros). This is what the device debug64 entry
 * (ssnt_fwd_bwd_debug64_device) turns into float64 logs, e*ln2 + ln(m): tests compare the GPU's
 * state with this bit for bit and its float64 logs with oracle_fwd_bwd_f64. */
int oracle_fwd_bwd_xf_state(int B, int T, int U, const float *log_trans, const float *log_obs,
                            const int32_t *step_len, const int32_t *pos_len, int flags,
                            float *loss, float *grad, void *alpha, void *beta, void *z,
                            int n_threads) {
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel
#endif
    {
        const size_t TU = (size_t)T * U;
        xf *buf = (xf *)malloc(sizeof(xf) * TU * 5);
#ifdef _OPENMP
#pragma omp for schedule(dynamic)
#endif
        for (int b = 0; b < B; ++b) {
            const size_t off = (size_t)b * TU;
            xf_fwd_bwd_one(log_trans + off * 2, log_obs ? log_obs + off : NULL, T, U, step_len[b],
                           pos_len[b], flags, loss + b, grad + off * 2, NULL, NULL, NULL, buf,
                           buf + TU, buf + 2 * TU, buf + 3 * TU, buf + 4 * TU,
                           (xf *)alpha + off, (xf *)beta + off, (xf *)z + b);
        }
        free(buf);
    }
    return ORC_OK;
}

/* ---- independent float64 log-domain DP (the mathematical definition, same semantics) ---- */
static inline double lse2(double a, double b) {
    if (a == -INFINITY) return b;
    if (b == -INFINITY) return a;
    const double m = a > b ? a : b;
    return m + log1p(exp(-fabs(a - b)));
}

int oracle_fwd_bwd_f64(int B, int T, int U, const float *log_trans, const float *log_obs,
                       const int32_t *step_len, const int32_t *pos_len, int flags, double *loss,
                       double *grad, double *grad_obs, double *log_alpha, double *log_beta) {
    const bool term = (flags & FLAG_TERMINAL_EMIT) != 0;
    const size_t TU = (size_t)T * U;
    double *A = (double *)malloc(sizeof(double) * TU), *Bt = (double *)malloc(sizeof(double) * TU);
    for (int b = 0; b < B; ++b) {
        const float *lt = log_trans + (size_t)b * TU * 2;
        const float *lo = log_obs ? log_obs + (size_t)b * TU : NULL;
        double *g = grad + (size_t)b * TU * 2, *go = grad_obs ? grad_obs + (size_t)b * TU : NULL;
        double *la = log_alpha ? log_alpha + (size_t)b * TU : NULL;
        double *lb = log_beta ? log_beta + (size_t)b * TU : NULL;
        const int S = step_len[b], P = pos_len[b];
        for (size_t i = 0; i < TU; ++i) {
            g[2 * i] = g[2 * i + 1] = 0.0;
            if (go) go[i] = 0.0;
            if (la) la[i] = -INFINITY;
            if (lb) lb[i] = -INFINITY;
            A[i] = Bt[i] = -INFINITY;
        }
        if (!(S >= 1 && P >= 1 && S <= T && P <= U && S >= P)) {
            loss[b] = (flags & FLAG_ZERO_INFINITY) ? 0.0 : INFINITY;
            continue;
        }
#define LT(s, p, k) ((double)lt[(((size_t)(s)) * U + (p)) * 2 + (k)])
#define LO(s, p) (lo ? (double)lo[((size_t)(s)) * U + (p)] : 0.0)
        A[0] = LO(0, 0);
        for (int s = 1; s < S; ++s)
            for (int p = 0; p < P; ++p) {
                double v = A[(size_t)(s - 1) * U + p] + LT(s - 1, p, 0);
                if (p > 0) v = lse2(v, A[(size_t)(s - 1) * U + p - 1] + LT(s - 1, p - 1, 1));
                A[(size_t)s * U + p] = v + LO(s, p);
            }
        Bt[(size_t)(S - 1) * U + P - 1] = term ? LT(S - 1, P - 1, 0) : 0.0;
        for (int s = S - 2; s >= 0; --s)
            for (int p = 0; p < P; ++p) {
                double v = LT(s, p, 0) + LO(s + 1, p) + Bt[(size_t)(s + 1) * U + p];
                if (p + 1 < P) v = lse2(v, LT(s, p, 1) + LO(s + 1, p + 1) + Bt[(size_t)(s + 1) * U + p + 1]);
                Bt[(size_t)s * U + p] = v;
            }
        const double logZ = A[(size_t)(S - 1) * U + P - 1] + (term ? LT(S - 1, P - 1, 0) : 0.0);
        if (logZ == -INFINITY) {
            loss[b] = (flags & FLAG_ZERO_INFINITY) ? 0.0 : INFINITY;
            continue;
        }
        loss[b] = -logZ;
        for (int s = 0; s < S; ++s)
            for (int p = 0; p < P; ++p) {
                const size_t c = (size_t)s * U + p;
                if (la) la[c] = A[c];
                if (lb) lb[c] = Bt[c];
                if (s + 1 < S) {
                    g[2 * c] = -exp(A[c] + LT(s, p, 0) + LO(s + 1, p) + Bt[c + U] - logZ);
                    if (p + 1 < P)
                        g[2 * c + 1] = -exp(A[c] + LT(s, p, 1) + LO(s + 1, p + 1) + Bt[c + U + 1] - logZ);
                } else if (term && p == P - 1) {
                    g[2 * c] = -exp(A[c] + LT(s, p, 0) - logZ);
                }
                if (go) go[c] = -exp(A[c] + Bt[c] - logZ);
            }
#undef LT
#undef LO
    }
    free(A);
    free(Bt);
    return ORC_OK;
}

int oracle_omp_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ==========================================================================================
 * F4: v2 duration-class forward-backward (DESIGN.md "Duration lattice").
 *
 * Not in the reference: the training-side counterpart of the v2 decode's expansion rules
 * (src/v2.rs:94-166). State (r, x): r = input steps consumed (0..I), x = total duration so far
 * (0..X-1, X = max_total + 1). Step t (row t -> t+1) picks one class i with weight
 * exp(logits[t][i]) and adds duration_table[i]; the move exists iff decode_beam_at would keep
 * that candidate (src/v2.rs:127-164):
 *   class rule, always:  !allow_skip && i == zero_duration_id is dropped (src/v2.rs:139,152);
 *   unless test_mode:    the new total inside total_duration_bounds(t) (src/v2.rs:94-104,131),
 *                        !will_overrun(t) (src/v2.rs:106-111,133),
 *                        at t = I-1 the new total == O (src/v2.rs:135-137).
 * Totals above max_total are outside the state space (reachable in test mode only); in band
 * mode O > max_total makes the lattice empty (loss +inf, every row -inf, grads 0).
 * Z = sum_x alpha[I][x]; loss = -ln Z (Z == 0: +inf, 0 with FLAG_ZERO_INFINITY, grads 0);
 * grad[t][i] = d loss / d logits[t][i] = -(posterior of class i at step t).
 *
 * Arithmetic (what csrc/v2_fwd_bwd.hip reproduces bit for bit): split-exponent xf as in the
 * lattice above; w[t][i] = xf_exp(logits[t][i], class rule);
 *   cell sums over classes (alpha, beta), D <= 64: em = max_i e_i (at least XF_EZERO),
 *     s = pairwise-tree sum of ldexp(m_i, e_i - em) over the classes zero-padded to a power of
 *     two, then xf_norm(s, em);
 *   sums over totals (Z, gradients): 64 partial sums -- total x goes to partial x mod 64, each
 *     accumulated with xf_add in increasing x -- then an xor butterfly over offsets 1..32 with
 *     xf_add (commutative: every partial ends equal).
 * Rows are only evaluated inside their window (f4_window): cells outside are exact zeros, and
 * neither sum depends on which zero cells it skips.
 * ========================================================================================== */
typedef struct {
    int I, O, X, D, dmax, zid;
    bool allow_skip, test_mode;
    const int32_t *dur;
} f4_ctx;

/* cells of row r that can be nonzero: [*lo, *hi] (empty when *lo > *hi) */
static void f4_window(const f4_ctx *c, int r, int *lo, int *hi) {
    if (r == 0) { *lo = 0; *hi = 0; return; }
    if (c->test_mode) {
        const long long h = (long long)r * c->dmax;
        *lo = 0;
        *hi = h < c->X - 1 ? (int)h : c->X - 1;
        return;
    }
    const int t = r - 1;
    if ((long long)(c->I - (t + 1)) * 3 > c->O) { *lo = 1; *hi = 0; return; } /* src/v2.rs:106-111 */
    const float diagonal = (float)c->O / (float)c->I * (float)(t + 1);      /* src/v2.rs:94-104 */
    const float upper_range = (float)c->O * 0.1f;
    const float lower_range = (float)c->O * 0.05f;
    int lb = f2i_sat(fmaxf(diagonal - lower_range, 0.0f));
    int ub = f2i_sat(fminf(diagonal + upper_range, (float)c->O));
    if (t == c->I - 1) { /* src/v2.rs:135-137 */
        lb = lb > c->O ? lb : c->O;
        ub = ub < c->O ? ub : c->O;
    }
    *lo = lb > 0 ? lb : 0;
    *hi = ub < c->X - 1 ? ub : c->X - 1;
}

static inline bool f4_in(int x, int lo, int hi) { return x >= lo && x <= hi; }

/* cell sum of D <= 64 class terms: em = max exponent (padding terms count as exact zeros
 * (0, EZERO)), then the ldexp-aligned f32 terms summed by a pairwise tree over the next power
 * of two (pairs (2i, 2i+1) first, zero padding) */
static xf f4_cell_sum(const xf *term, int D) {
    int P2 = 1;
    while (P2 < D) P2 <<= 1;
    int32_t em = XF_EZERO;
    for (int i = 0; i < D; ++i) em = term[i].e > em ? term[i].e : em;
    float v[64];
    for (int i = 0; i < P2; ++i) v[i] = i < D ? ldexpf(term[i].m, term[i].e - em) : 0.0f;
    for (int len = P2; len > 1; len >>= 1)
        for (int i = 0; i < len / 2; ++i) v[i] = v[2 * i] + v[2 * i + 1];
    return xf_norm(v[0], em);
}

/* 64 partials (x mod 64, increasing x) + xor butterfly: acc[64] in, result out */
static xf f4_butterfly(xf *acc) {
    xf nxt[64];
    for (int off = 1; off < 64; off <<= 1) {
        for (int l = 0; l < 64; ++l) nxt[l] = xf_add(acc[l].m, acc[l].e, acc[l ^ off].m, acc[l ^ off].e);
        memcpy(acc, nxt, sizeof(nxt));
    }
    return acc[0];
}

static void f4_one(const f4_ctx *c, int Imax, const float *lg, float *loss, float *g,
                   float *la, float *lb, int flags, xf *A, xf *Bt, xf *w, xf *term) {
    const int X = c->X, D = c->D, I = c->I;
    const float inf_loss = (flags & FLAG_ZERO_INFINITY) ? 0.0f : INFINITY;
    if (g) memset(g, 0, sizeof(float) * (size_t)Imax * D);
    for (size_t k = 0; la && k < (size_t)(Imax + 1) * X; ++k) la[k] = -INFINITY;
    for (size_t k = 0; lb && k < (size_t)(Imax + 1) * X; ++k) lb[k] = -INFINITY;
    /* no lattice: bad lengths, or (band mode) a final total O beyond max_total -- the exact
     * final-length rule (src/v2.rs:135-137) can then never hold, so Z = 0 whatever the rows */
    if (I <= 0 || I > Imax || c->O < 0 || (!c->test_mode && c->O > X - 1)) { *loss = inf_loss; return; }
    for (int t = 0; t < I; ++t)
        for (int i = 0; i < D; ++i)
            w[(size_t)t * D + i] = xf_exp(lg[(size_t)t * D + i], c->allow_skip || i != c->zid);
    const xf zero = {0.0f, XF_EZERO};
    /* alpha */
    for (size_t k = 0; k < (size_t)(I + 1) * X; ++k) A[k] = zero;
    A[0] = (xf){0.5f, 1};
    for (int r = 1; r <= I; ++r) {
        int plo, phi, lo, hi;
        f4_window(c, r - 1, &plo, &phi);
        f4_window(c, r, &lo, &hi);
        for (int x = lo; x <= hi; ++x) {
            for (int i = 0; i < D; ++i) {
                const int y = x - c->dur[i];
                if (f4_in(y, plo, phi)) {
                    const xf a = A[(size_t)(r - 1) * X + y], ww = w[(size_t)(r - 1) * D + i];
                    term[i] = (xf){a.m * ww.m, a.e + ww.e};
                } else {
                    term[i] = zero;
                }
            }
            A[(size_t)r * X + x] = f4_cell_sum(term, D);
        }
    }
    for (int r = 0; la && r <= I; ++r) {
        int lo, hi;
        f4_window(c, r, &lo, &hi);
        for (int x = lo; x <= hi; ++x) la[(size_t)r * X + x] = xf_log(A[(size_t)r * X + x]);
    }
    /* Z */
    xf acc[64];
    for (int l = 0; l < 64; ++l) acc[l] = zero;
    {
        int lo, hi;
        f4_window(c, I, &lo, &hi);
        for (int x = lo; x <= hi; ++x) {
            const xf a = A[(size_t)I * X + x];
            acc[x & 63] = xf_add(acc[x & 63].m, acc[x & 63].e, a.m, a.e);
        }
    }
    const xf Z = f4_butterfly(acc);
    if (Z.m == 0.0f) { *loss = inf_loss; return; }
    *loss = 0.0f - xf_log(Z);
    const float izm = 1.0f / Z.m;
    const int32_t ize = -Z.e;
    /* beta */
    for (size_t k = 0; k < (size_t)(I + 1) * X; ++k) Bt[k] = zero;
    {
        int lo, hi;
        f4_window(c, I, &lo, &hi);
        for (int x = lo; x <= hi; ++x) Bt[(size_t)I * X + x] = (xf){0.5f, 1};
    }
    for (int r = I - 1; r >= 0; --r) {
        int lo, hi, nlo, nhi;
        f4_window(c, r, &lo, &hi);
        f4_window(c, r + 1, &nlo, &nhi);
        for (int y = lo; y <= hi; ++y) {
            for (int i = 0; i < D; ++i) {
                const int x = y + c->dur[i];
                if (f4_in(x, nlo, nhi)) {
                    const xf bb = Bt[(size_t)(r + 1) * X + x], ww = w[(size_t)r * D + i];
                    term[i] = (xf){ww.m * bb.m, ww.e + bb.e};
                } else {
                    term[i] = zero;
                }
            }
            Bt[(size_t)r * X + y] = f4_cell_sum(term, D);
        }
    }
    for (int r = 0; lb && r <= I; ++r) {
        int lo, hi;
        f4_window(c, r, &lo, &hi);
        for (int x = lo; x <= hi; ++x) lb[(size_t)r * X + x] = xf_log(Bt[(size_t)r * X + x]);
    }
    /* gradients: posterior of class i at step t over the moves into row t+1 */
    for (int t = 0; g && t < I; ++t) {
        int plo, phi, lo, hi;
        f4_window(c, t, &plo, &phi);
        f4_window(c, t + 1, &lo, &hi);
        for (int i = 0; i < D; ++i) {
            for (int l = 0; l < 64; ++l) acc[l] = zero;
            for (int x = lo; x <= hi; ++x) {
                const int y = x - c->dur[i];
                if (!f4_in(y, plo, phi)) continue;
                const xf a = A[(size_t)t * X + y], bb = Bt[(size_t)(t + 1) * X + x];
                acc[x & 63] = xf_add(acc[x & 63].m, acc[x & 63].e, a.m * bb.m, a.e + bb.e);
            }
            const xf S = f4_butterfly(acc);
            const xf ww = w[(size_t)t * D + i];
            g[(size_t)t * D + i] = xf_neg_post((S.m * ww.m) * izm, S.e + ww.e + ize);
        }
    }
}

/* logits (B, Imax, D); duration_table (D) >= 0; input_length / output_length (B); X = max_total+1.
 * Outputs: loss (B); grad (B, Imax, D) or NULL; log_alpha / log_beta (B, Imax+1, X) or NULL. */
int oracle_v2_fwd_bwd(int B, int Imax, int D, int max_total, const float *logits,
                      const int32_t *duration_table, const int32_t *input_length,
                      const int32_t *output_length, int zero_duration_id, bool allow_skip,
                      bool test_mode, int flags, float *loss, float *grad, float *log_alpha,
                      float *log_beta, int n_threads) {
    if (B < 0 || Imax <= 0 || D <= 0 || D > 64 || max_total < 0) return ORC_ERR_INVALID;
    int dmax = 0;
    for (int i = 0; i < D; ++i) {
        if (duration_table[i] < 0) return ORC_ERR_INVALID;
        dmax = duration_table[i] > dmax ? duration_table[i] : dmax;
    }
    const int X = max_total + 1;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel
#endif
    {
        xf *A = (xf *)malloc(sizeof(xf) * (size_t)(Imax + 1) * X);
        xf *Bt = (xf *)malloc(sizeof(xf) * (size_t)(Imax + 1) * X);
        xf *w = (xf *)malloc(sizeof(xf) * (size_t)Imax * D);
        xf *term = (xf *)malloc(sizeof(xf) * (size_t)D);
#ifdef _OPENMP
#pragma omp for schedule(dynamic)
#endif
        for (int b = 0; b < B; ++b) {
            f4_ctx c = {input_length[b], output_length[b], X, D, dmax, zero_duration_id,
                        allow_skip, test_mode, duration_table};
            const size_t rows = (size_t)(Imax + 1) * X;
            f4_one(&c, Imax, logits + (size_t)b * Imax * D, loss + b,
                   grad ? grad + (size_t)b * Imax * D : NULL, log_alpha ? log_alpha + b * rows : NULL,
                   log_beta ? log_beta + b * rows : NULL, flags, A, Bt, w, term);
        }
        free(A);
        free(Bt);
        free(w);
        free(term);
    }
    return ORC_OK;
}

/* Independent float64 log-domain definition of the same lattice (no windows: every state,
 * the rules applied per move), for pinning the xf arithmetic. loss (B), grad (B, Imax, D). */
int oracle_v2_fwd_bwd_f64(int B, int Imax, int D, int max_total, const float *logits,
                          const int32_t *duration_table, const int32_t *input_length,
                          const int32_t *output_length, int zero_duration_id, bool allow_skip,
                          bool test_mode, double *loss, double *grad) {
    const int X = max_total + 1;
    double *A = (double *)malloc(sizeof(double) * (size_t)(Imax + 1) * X);
    double *Bt = (double *)malloc(sizeof(double) * (size_t)(Imax + 1) * X);
    for (int b = 0; b < B; ++b) {
        const int I = input_length[b], O = output_length[b];
        const float *lg = logits + (size_t)b * Imax * D;
        double *g = grad + (size_t)b * Imax * D;
        for (int k = 0; k < Imax * D; ++k) g[k] = 0.0;
        if (I <= 0 || I > Imax) { loss[b] = INFINITY; continue; }
        v2_ctx vc = {(uint64_t)I, (uint64_t)O, NULL, duration_table, D, zero_duration_id, allow_skip, test_mode};
        /* move (t, x -> x + d_i) allowed? */
#define F4_OK(t, nx, i)                                                                          \
    ((allow_skip || (i) != zero_duration_id) && (nx) >= 0 && (nx) < X &&                         \
     (test_mode || (({ int32_t lb_, ub_; v2_bounds(&vc, (uint64_t)(t), &lb_, &ub_);               \
                       (nx) >= lb_ && (nx) <= ub_; }) && !v2_will_overrun(&vc, (uint64_t)(t)) &&  \
                    ((t) != I - 1 || (nx) == O))))
        for (size_t k = 0; k < (size_t)(I + 1) * X; ++k) A[k] = Bt[k] = -INFINITY;
        A[0] = 0.0;
        for (int t = 0; t < I; ++t)
            for (int x = 0; x < X; ++x) {
                if (A[(size_t)t * X + x] == -INFINITY) continue;
                for (int i = 0; i < D; ++i) {
                    const int nx = x + duration_table[i];
                    if (!F4_OK(t, nx, i) || !(lg[(size_t)t * D + i] >= XF_LOG_MIN)) continue;
                    double *dst = &A[(size_t)(t + 1) * X + nx];
                    *dst = lse2(*dst, A[(size_t)t * X + x] + (double)lg[(size_t)t * D + i]);
                }
            }
        double Z = -INFINITY;
        for (int x = 0; x < X; ++x) Z = lse2(Z, A[(size_t)I * X + x]);
        if (Z == -INFINITY) { loss[b] = INFINITY; continue; }
        loss[b] = -Z;
        for (int x = 0; x < X; ++x) Bt[(size_t)I * X + x] = 0.0;
        for (int t = I - 1; t >= 0; --t)
            for (int x = 0; x < X; ++x)
                for (int i = 0; i < D; ++i) {
                    const int nx = x + duration_table[i];
                    if (!F4_OK(t, nx, i) || !(lg[(size_t)t * D + i] >= XF_LOG_MIN)) continue;
                    const double v = (double)lg[(size_t)t * D + i] + Bt[(size_t)(t + 1) * X + nx];
                    Bt[(size_t)t * X + x] = lse2(Bt[(size_t)t * X + x], v);
                    const double post = A[(size_t)t * X + x] + v - Z;
                    g[(size_t)t * D + i] -= exp(post);
                }
#undef F4_OK
    }
    free(A);
    free(Bt);
    return ORC_OK;
}
