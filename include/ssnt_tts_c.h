/*
 * ssnt_tts_c.h -- drop-in C ABI of libssnt_tts_c, MI355X (gfx950) implementation.
 *
 * Part 1 re-exports, with identical names, argument order, types and meaning, the seven
 * unmangled symbols of the reference's Rust `staticlib` ssnt_tts_c
 * (nii-yamagishilab/ssnt-tts-rust, ssnt_tts_c/src/lib.rs), which the TensorFlow custom ops in
 * ssnt-tts-tensorflow/src/ (*_op.cc) declare `extern "C"` and link with -lssnt_tts_c
 * (ssnt-tts-tensorflow/setup.py:15,40-42). Arguments are HOST pointers; each call is
 * synchronous; contract violations print to stderr and abort(), as the Rust assert!/panic in
 * an extern fn does. The work runs on the GPU (per-thread stream and scratch; reentrant).
 *
 * Part 2 adds entry points the reference does not have: the lattice forward-backward
 * (SURVEY.md 8(a) A11), batched and fused decode, and device-pointer + hipStream_t variants of
 * every kernel. They return an ssnt_status code instead of aborting.
 *
 * `bool` is the 1-byte C99/C++ bool, identical to Rust's `bool` in extern fns.
 */
#ifndef SSNT_TTS_C_H
#define SSNT_TTS_C_H

#include <stddef.h>
#include <stdint.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ===================== Part 1: reference symbols (host pointers) ===================== */

/* One v1 emit/shift beam-search step, batch fixed to 1.
 * Replaces ssnt_tts_c/src/lib.rs:11-83 (-> src/lib.rs:121-230); caller
 * ssnt-tts-tensorflow/src/ssnt_tts_beam_search_decode_op.cc:5-8,116-128.
 * h (W,2) [emit, shift] log-probs; log_prob_history, is_finished, t, u (W); outputs (W). */
void ssnt_tts_beam_search_decode(const float *h, const float *log_prob_history,
                                 const bool *is_finished, const int *t, const int *u, int max_t,
                                 int beam_width, int *prediction, float *log_probs, int *next_t,
                                 int *next_u, bool *next_is_finished, int *beam_branch);

/* Backtrace of the best final beam. Replaces ssnt_tts_c/src/lib.rs:87-116
 * (-> src/util.rs:20-33); caller ssnt_extract_best_beam_branch_op.cc:6-8 (declared `bool`
 * there, return value ignored). beam_branch, t_history (max_u, W); outputs (max_u). */
void ssnt_extract_best_beam_branch(int best_final_branch, const int *beam_branch,
                                   const int *t_history, int beam_width, int max_u,
                                   int *best_beam_branch, int *best_t_history);

/* One v2 duration-class beam-search step. Replaces ssnt_tts_c/src/lib.rs:119-218
 * (-> src/v2.rs:221-339); caller ssnt_tts_v2_beam_search_decode_op.cc:5-26,179-200.
 * h (B,W,D); state (B,W); duration_table (D); input/output_length (B); outputs (B,W). */
void ssnt_tts_v2_beam_search_decode(const float *h, const float *log_prob_history,
                                    const bool *is_finished, const int *total_duration,
                                    const int *duration_table, const int *t, const int *u,
                                    const int *input_length, const int *output_length,
                                    int batch_size, int beam_width, int duration_class_size,
                                    int zero_duration_id, bool allow_skip, bool test_mode,
                                    int *prediction, float *log_probs, int *next_t, int *next_u,
                                    bool *next_is_finished, int *next_total_duration,
                                    int *beam_branch);

/* Backtrace of every final beam. Replaces ssnt_tts_c/src/lib.rs:221-241
 * (-> src/v2_util.rs:6-36); caller ssnt_order_beam_branch_op.cc:6-11.
 * final_branch (B,W); beam_branch (B,max_t,W); ordered_beam_branch (B,W,max_t). */
void ssnt_order_beam_branch(const int *final_branch, const int *beam_branch, int batch_size,
                            int beam_width, int max_t, int *ordered_beam_branch);

/* Durations -> frame-to-input index map. Replaces ssnt_tts_c/src/lib.rs:245-265
 * (-> src/v2_util.rs:39-66); caller upsample_source_indexes_op.cc:6-12. Writes only the first
 * min(output_length[b,w], max_u) entries of each (b,w) row (the op prefills the rest). */
void ssnt_upsample_source_indexes(const int *duration, const int *output_length, int batch_size,
                                  int beam_width, int max_t, int max_u,
                                  int *upsampled_source_indexes);

/* One tone-latent beam-search step. Replaces ssnt_tts_c/src/lib.rs:268-343
 * (-> src/tone_latent.rs:144-234); caller tone_latent_beam_search_decode_op.cc. */
void tone_latent_beam_search_decode(const float *h, const float *log_prob_history,
                                    const bool *is_finished, const int *t, const int *u,
                                    const int *input_length, int batch_size, int beam_width,
                                    int tone_class_size, int empty_tone_id, int *prediction,
                                    float *log_probs, int *next_t, int *next_u,
                                    bool *next_is_finished, int *beam_branch);

/* Batched Levenshtein distance. Replaces ssnt_tts_c/src/lib.rs:347-381
 * (-> src/edit_distance.rs:6-60); caller ssnt_tts_edit_distance.cc. */
void tone_latent_levenshtein_edit_distance(const int *a, const int *b, const int *a_lengths,
                                           const int *b_lengths, int batch_size,
                                           int max_length, int *distance);

/* ===================== Part 2: extensions ===================== */

typedef enum {
  SSNT_OK = 0,
  SSNT_ERR_INVALID_ARG = 1,
  SSNT_ERR_HIP = 2,
  SSNT_ERR_NO_CANDIDATE = 3,      /* v2: src/v2.rs:292 assert */
  SSNT_ERR_DURATION_MISMATCH = 4, /* upsample: src/v2_util.rs:58 assert */
  SSNT_ERR_UNSUPPORTED = 5,       /* size outside what the kernels handle */
  SSNT_ERR_WORKSPACE = 6,         /* workspace missing / too small */
  SSNT_ERR_BAD_LENGTH = 7,        /* a length exceeds the tensor extent */
  SSNT_ERR_BAD_INDEX = 8,         /* backtrace branch index outside [0, W) */
  SSNT_ERR_INTERNAL = 9           /* fwd-bwd: a bounded intra-kernel wait expired (a bug) */
} ssnt_status;

const char *ssnt_status_string(int status);
/* translate the bits a kernel OR-ed into a device status word into an ssnt_status */
int ssnt_status_from_bits(int bits);
/* library / device info: fills a short human-readable string, returns SSNT_OK */
int ssnt_version(char *buf, size_t len);

/* lattice flags */
#define SSNT_FLAG_TERMINAL_EMIT 1 /* Z includes the terminal emit at (S-1,P-1) (src/lib.rs:187-195) */
#define SSNT_FLAG_ZERO_INFINITY 2 /* infeasible utterances report loss 0 instead of +inf */

/* ---- emit/shift lattice forward-backward ----
 * log_trans (B,T,U,2) f32 natural-log [emit, shift] probabilities, row-major;
 * log_obs (B,T,U) optional per-cell log-likelihood (NULL = none);
 * step_len, pos_len (B): lattice extent S_b <= T steps, P_b <= U positions.
 * Outputs: loss (B) = -ln Z; grad_trans (B,T,U,2) = d loss / d log_trans (NULL = skip);
 * grad_obs (B,T,U) = d loss / d log_obs (NULL = skip); log_alpha / log_beta (B,T,U) debug
 * outputs (NULL = skip). Cells outside (S_b,P_b) get grad 0 and log-alpha/beta -inf.
 * Device variant: all pointers are device pointers; `stream` is a hipStream_t (NULL = legacy
 * default); `workspace` must hold ssnt_fwd_bwd_workspace_size() bytes -- always take the size
 * from that query, never compute it: it is 0 (NULL workspace) when every row of the dispatched
 * kernel stays in LDS (U <= 256 and T*U small enough), else the segmented kernel's rows
 * ((T+1)*U xf per utterance) plus its hand-off counter block and hand-off rings, each padded to
 * 256 B; `status` (device int, may be NULL) receives error bits. Asynchronous. The kernel is
 * chosen from the shape and alignment alone (no process-wide state). */
size_t ssnt_fwd_bwd_workspace_size(int batch, int max_steps, int max_pos);
/* Name of the forward-backward kernel instance the calling thread's last ssnt_fwd_bwd* call
 * dispatched (e.g. "k_fwd_bwd_stream<K=2,OBS=0,LDS=1,NC=3,NH=4,RS=0,NV=0>"; launches of one call
 * joined by '+'), copied into buf (truncated to len); returns its full length. Lets a profile be
 * matched to the kernel a benchmark actually ran. */
int ssnt_fwd_bwd_last_kernel(char *buf, size_t len);
int ssnt_fwd_bwd_device(const float *log_trans, const float *log_obs, const int *step_len,
                        const int *pos_len, int batch, int max_steps, int max_pos, int flags,
                        float *loss, float *grad_trans, float *grad_obs, float *log_alpha,
                        float *log_beta, void *workspace, size_t workspace_bytes, int *status,
                        void *stream);
/* As ssnt_fwd_bwd_device, plus the batch loss sum *loss_sum = sum_b loss[b] (device float) in a
 * fixed summation order (deterministic; independent of the kernel variant). `sum_state` is a
 * device buffer of ssnt_fwd_bwd_sum_state_size(batch) bytes, zeroed once before its first use
 * and then left to the library: with it, workgroup 0 forms the sum inside the same launch from
 * per-utterance 8-byte {tag, loss} granules; NULL costs one extra single-wave launch. One state
 * per stream of concurrent calls. New: the reference has no forward-backward (SURVEY.md 8(a)
 * A11). */
size_t ssnt_fwd_bwd_sum_state_size(int batch);
int ssnt_fwd_bwd_sum_device(const float *log_trans, const float *log_obs, const int *step_len,
                            const int *pos_len, int batch, int max_steps, int max_pos, int flags,
                            float *loss, float *grad_trans, float *grad_obs, float *log_alpha,
                            float *log_beta, void *workspace, size_t workspace_bytes, int *status,
                            float *loss_sum, void *sum_state, void *stream);
/* Float64 outputs of the same computation (the north_star bar is 1e-5 abs on
 * log-alpha / log-beta, which an f32 value cannot hold once |log alpha| > ~84 -- half an f32
 * ulp at configs[4]'s |log alpha| ~ 2231 is 1.2e-4). The dispatched kernel writes its
 * split-exponent state m * 2^e (m in [0.5, 1)) instead of f32 logs, and a second pass forms
 * e*ln2 + ln(m) in float64 on the GPU: loss (B) = -ln Z, log_alpha / log_beta (B,T,U) (NULL =
 * skip; -inf outside the lattice). grad_trans / grad_obs and every rule as
 * ssnt_fwd_bwd_device (the same launch, the same kernel the shape dispatches; gradients
 * bit-identical). `workspace`: ssnt_fwd_bwd_debug64_workspace_size() bytes (the plain
 * workspace plus the state planes, 16 B per cell). Device pointers, asynchronous. New: the
 * reference has no forward-backward. */
size_t ssnt_fwd_bwd_debug64_workspace_size(int batch, int max_steps, int max_pos);
int ssnt_fwd_bwd_debug64_device(const float *log_trans, const float *log_obs, const int *step_len,
                                const int *pos_len, int batch, int max_steps, int max_pos,
                                int flags, double *loss, float *grad_trans, float *grad_obs,
                                double *log_alpha, double *log_beta, void *workspace,
                                size_t workspace_bytes, int *status, void *stream);
/* Host-pointer variant (synchronous; copies through the calling thread's GPU context). */
int ssnt_fwd_bwd(const float *log_trans, const float *log_obs, const int *step_len,
                 const int *pos_len, int batch, int max_steps, int max_pos, int flags,
                 float *loss, float *grad_trans, float *grad_obs, float *log_alpha,
                 float *log_beta);

/* ---- F4: v2 duration-class (semi-Markov) forward-backward (DESIGN.md
 * "Duration lattice"). New: the reference only decodes this lattice; the move rules are the v2
 * decode's (src/v2.rs:94-166 -- band, overrun, exact final total, zero-duration class; test_mode
 * keeps only the class rule). logits (B,T,D) per-step class log-probs (teacher-forced, one row
 * per input step); duration_table (D) >= 0; input_length I_b <= T, output_length O_b (B).
 * State totals run 0..max_total (totals above it -- test mode only -- are outside the lattice).
 * Outputs: loss (B) = -ln Z, Z = sum over every admissible class sequence of its probability
 * (+inf when none, 0 with SSNT_FLAG_ZERO_INFINITY); grad (B,T,D) = d loss / d logits = minus
 * the class posteriors (NULL = skip); log_alpha / log_beta (B,T+1,max_total+1) debug rows
 * (NULL = skip). `workspace` holds ssnt_v2_fwd_bwd_workspace_size() bytes. Device pointers,
 * asynchronous on `stream`; a negative duration sets SSNT_ERR_BAD_INDEX in `status`. */
size_t ssnt_v2_fwd_bwd_workspace_size(int batch, int max_steps, int max_total, bool test_mode);
int ssnt_v2_fwd_bwd_device(const float *logits, const int *duration_table, const int *input_length,
                           const int *output_length, int batch, int max_steps,
                           int duration_class_size, int max_total, int zero_duration_id,
                           bool allow_skip, bool test_mode, int flags, float *loss, float *grad,
                           float *log_alpha, float *log_beta, void *workspace,
                           size_t workspace_bytes, int *status, void *stream);

/* ---- batched decode steps, device pointers (the reference FFI fixes v1 to B=1,
 * ssnt_tts_c/src/lib.rs:13; its Rust API takes B, src/lib.rs:121). max_beam_width = beam_width
 * as in every reference call site (ssnt_tts_c/src/lib.rs:82,217,342). ---- */
int ssnt_beam_search_decode_device(const float *h, const float *log_prob_history,
                                   const bool *is_finished, const int *t, const int *u,
                                   const int *input_length, int batch_size, int beam_width,
                                   int *prediction, float *log_probs, int *next_t, int *next_u,
                                   bool *next_is_finished, int *beam_branch, int *status,
                                   void *stream);
int ssnt_v2_beam_search_decode_device(const float *h, const float *log_prob_history,
                                      const bool *is_finished, const int *total_duration,
                                      const int *duration_table, const int *t, const int *u,
                                      const int *input_length, const int *output_length,
                                      int batch_size, int beam_width, int duration_class_size,
                                      int zero_duration_id, bool allow_skip, bool test_mode,
                                      int *prediction, float *log_probs, int *next_t,
                                      int *next_u, bool *next_is_finished,
                                      int *next_total_duration, int *beam_branch, int *status,
                                      void *stream);
int ssnt_tone_latent_beam_search_decode_device(const float *h, const float *log_prob_history,
                                               const bool *is_finished, const int *t,
                                               const int *u, const int *input_length,
                                               int batch_size, int beam_width,
                                               int tone_class_size, int empty_tone_id,
                                               int *prediction, float *log_probs, int *next_t,
                                               int *next_u, bool *next_is_finished,
                                               int *beam_branch, int *status, void *stream);

/* Fused multi-step decodes (the three entries below) pack next_t / next_u into 16 bits each:
 * max_steps > 32767 returns SSNT_ERR_UNSUPPORTED, and so does beam_width > 64 for v1 (v2 / tone
 * take any W*C through the LDS step kernel).
 * Fused T-step v1 decode over a (B,T,U,2) log-prob lattice: step s feeds each beam
 * h = lattice[b, u, t, :]; all beams start at t=u=0, log-prob 0. Per-step outputs (B,T,W);
 * best_beam_branch / best_t_history (B,T) = backtrace of slot 0 after the last step with
 * t_history = next_t (src/util.rs:20-33). */
int ssnt_lattice_beam_search_decode_device(const float *lattice, const int *input_length,
                                           int batch_size, int max_steps, int max_pos,
                                           int beam_width, int *prediction, float *log_probs,
                                           int *next_t, int *next_u, bool *next_is_finished,
                                           int *beam_branch, int *best_beam_branch,
                                           int *best_t_history, int *status, void *stream);

/* Fused multi-step v2 duration-class decode (BASELINE configs[4] "v2 path"). Every beam starts
 * at t = u = 0, log-prob 0, total_duration 0, not finished; step s runs the exact
 * ssnt_tts_v2_beam_search_decode step (src/v2.rs:221-339, max_beam_width = beam_width) on
 * h = logits[b, s] (W,D) and feeds its outputs back as the next state -- what the TF decode loop
 * does around the per-step op, one launch instead of max_steps. logits (B,T,W,D); per-step
 * outputs (B,T,W). Then, in the same launch, every final slot w is backtraced
 * (src/v2_util.rs:6-36 with final_branch = [0..W)): ordered_beam_branch (B,W,T), the class
 * chosen at each step of each path (path_prediction, B,W,T) and the duration it added
 * (duration, B,W,T; sums to the path's final total, the input of
 * ssnt_upsample_source_indexes). The three path outputs may be NULL. An utterance where no
 * candidate survives (the reference panics, src/v2.rs:292) sets SSNT_ERR_NO_CANDIDATE in
 * `status` and its outputs are unspecified. New: the reference steps once per call. */
int ssnt_v2_lattice_beam_search_decode_device(
    const float *logits, const int *duration_table, const int *input_length,
    const int *output_length, int batch_size, int max_steps, int beam_width,
    int duration_class_size, int zero_duration_id, bool allow_skip, bool test_mode,
    int *prediction, float *log_probs, int *next_t, int *next_u, bool *next_is_finished,
    int *next_total_duration, int *beam_branch, int *ordered_beam_branch, int *path_prediction,
    int *duration, int *status, void *stream);

/* Fused multi-step tone-latent decode (BASELINE configs[4] "tone_latent path"): as
 * ssnt_v2_lattice_beam_search_decode_device with the tone step (src/tone_latent.rs:144-234),
 * logits (B,T,W,C); path outputs ordered_beam_branch and path_prediction (the tone sequence of
 * each final slot, the input of the edit-distance evaluation) may be NULL. */
int ssnt_tone_latent_lattice_beam_search_decode_device(
    const float *logits, const int *input_length, int batch_size, int max_steps, int beam_width,
    int tone_class_size, int empty_tone_id, int *prediction, float *log_probs, int *next_t,
    int *next_u, bool *next_is_finished, int *beam_branch, int *ordered_beam_branch,
    int *path_prediction, int *status, void *stream);

/* Batched backtraces / utilities, device pointers. */
int ssnt_extract_best_beam_branch_device(const int *best_final_branch, const int *beam_branch,
                                         const int *t_history, int batch_size, int beam_width,
                                         int max_u, int *best_beam_branch, int *best_t_history,
                                         int *status, void *stream);
int ssnt_order_beam_branch_device(const int *final_branch, const int *beam_branch,
                                  int batch_size, int beam_width, int max_t,
                                  int *ordered_beam_branch, int *status, void *stream);
int ssnt_upsample_source_indexes_device(const int *duration, const int *output_length,
                                        int batch_size, int beam_width, int max_t, int max_u,
                                        int *upsampled_source_indexes, int *status,
                                        void *stream);
int ssnt_levenshtein_edit_distance_device(const int *a, const int *b, const int *a_lengths,
                                          const int *b_lengths, int batch_size, int max_length,
                                          int *distance, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* SSNT_TTS_C_H */
