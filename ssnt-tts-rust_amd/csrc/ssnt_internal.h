// ssnt_internal.h -- launchers shared between the kernels (fwd_bwd.hip, decode.hip) and the
// C-ABI host layer (capi.hip). Not part of the public interface (that is include/ssnt_tts_c.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ssnt_tts_c.h"

namespace ssnt {

// device status word bits (OR-ed by kernels, read by the host layer)
constexpr int kStatusNoCandidate = 1 << 0;       // v2: no duration sequence fits (src/v2.rs:292)
constexpr int kStatusDurationMismatch = 1 << 1;  // upsample: sum(d) != output_length (src/v2_util.rs:58)
constexpr int kStatusBadLength = 1 << 2;         // fwd-bwd: step/pos length outside the tensor
constexpr int kStatusBadIndex = 1 << 3;          // backtrace: branch index outside [0, W)
constexpr int kStatusTimeout = 1 << 4;           // fwd-bwd: an intra-workgroup wait hit its bound
constexpr int kStatusRingTag = 1 << 5;           // diagnostic builds only: a ring slot / row held another row

int status_bits_to_code(int bits);

// ---- lattice forward-backward (fwd_bwd.hip) ----
struct FwdBwdArgs {
  const float* log_trans;  // (B,T,U,2)
  const float* log_obs;    // (B,T,U) or null
  const int* step_len;     // (B)
  const int* pos_len;      // (B)
  int B, T, U, flags;
  float* loss;       // (B)
  float* grad;       // (B,T,U,2) or null
  float* grad_obs;   // (B,T,U) or null (requires log_obs)
  float* log_alpha;  // (B,T,U) or null
  float* log_beta;   // (B,T,U) or null
  void* workspace;   // row storage when the rows do not fit LDS
  size_t workspace_bytes;
  int* status;  // device status word or null
  float* loss_sum;   // fixed-order sum of loss[0..B) or null
  void* sum_state;   // in-launch sum state (lattice_dev.h; zero before the first call) or null
  // raw-state debug mode (ssnt_fwd_bwd_debug64_device): with log_alpha_e / log_beta_e set, the
  // debug rows log_alpha / log_beta receive the normalized split-exponent mantissas (0 outside
  // the lattice) and these planes the exponents, (B,T,U); z_state (B x {m, e bits}) receives Z
  int* log_alpha_e;
  int* log_beta_e;
  float* z_state;
};
size_t fwd_bwd_workspace_bytes(int B, int T, int U);
// float64 debug outputs (ssnt_fwd_bwd_debug64_device): workspace bytes and the launch, which runs
// the product dispatch in raw-state mode and then forms e*ln2 + ln(m) in float64 on the GPU
size_t fwd_bwd_debug64_workspace_bytes(int B, int T, int U);
int launch_fwd_bwd_debug64(const FwdBwdArgs& a, double* loss64, double* log_alpha64,
                           double* log_beta64, hipStream_t stream);
size_t fwd_bwd_sum_state_bytes(int B);  // 64 + 8 B
int launch_fwd_bwd(const FwdBwdArgs& a, hipStream_t stream);
// streaming kernel (fwd_bwd_stream.hip): SSNT_ERR_UNSUPPORTED for shapes it does not take
int launch_fwd_bwd_stream(const FwdBwdArgs& a, hipStream_t stream);
// segmented kernel (fwd_bwd_wide.hip): long rows (256 < U <= 1024), or any U <= 1024 when
// any_u; SSNT_ERR_UNSUPPORTED for other shapes
int launch_fwd_bwd_wide(const FwdBwdArgs& a, hipStream_t stream, bool any_u);
size_t fwd_bwd_wide_workspace_bytes(int B, int T, int U);
size_t stream_head_bytes(int K, int U, bool obs, int ring = 0);  // LDS bytes besides the lattice rows
// Process-wide A/B knobs and the kernels only they reach: the A/B build (-DSSNT_AB, `make
// lib-ab`, lib/ab/libssnt_tts_c_ab.so; tests and tools) only. The product dispatches by shape.
#ifdef SSNT_AB
int set_fwd_bwd_variant(int v);
int set_stream_ring(int r);  // 0 default, 16 / 32 ring slots with workspace rows
int stream_ring();
int set_fwd_bwd_wide_lanes(int k);  // positions per lane of the long-row kernel (1 or 2)
int set_fwd_bwd_wide_split(int mode);  // two workgroups per direction (-1 auto, 0 off, 1 on)
int set_fused_decode_select(int mode);  // -1 default, 0 full rank, 1 selection
int set_fused_decode_tone_waves(int n);  // -1 default, 1 / 2 / 4 waves for tone's rank
#else
constexpr int stream_ring() { return 0; }
#endif
int diag_read(void* host, size_t bytes);  // -DSSNT_DIAG builds only (tools/diag_fwd_bwd.py)
// the fwd-bwd kernel instance this thread dispatched last ("k_fwd_bwd_stream<K=2,...>"; one
// name per launch of a multi-launch kernel, joined by '+'); for bench.py's profile check
void note_fwd_bwd_dispatch(const char* fmt, ...);
const char* last_fwd_bwd_dispatch();

// ---- F4: v2 duration-class forward-backward (v2_fwd_bwd.hip) ----
struct V2FwdBwdArgs {
  const float* logits;       // (B, Imax, D) per-step class log-probs
  const int* table;          // (D) duration_table, >= 0
  const int* input_length;   // (B) I_b <= Imax
  const int* output_length;  // (B) O_b
  int B, Imax, D, X;         // X = max_total + 1 totals per row
  int zid;                   // zero_duration_id
  bool allow_skip, test_mode;
  int flags;                 // SSNT_FLAG_ZERO_INFINITY
  float* loss;               // (B)
  float* grad;               // (B, Imax, D) or null
  float* log_alpha;          // (B, Imax+1, X) or null
  float* log_beta;           // (B, Imax+1, X) or null
  void* workspace;
  size_t workspace_bytes;
  int Wcap;                  // set by the launcher
  int chunk;                 // set by the launcher
  int* status;
};
size_t v2_fwd_bwd_wcap(int max_total, bool test_mode);
size_t v2_fwd_bwd_workspace_bytes(int B, int Imax, int max_total, bool test_mode);
int launch_v2_fwd_bwd(const V2FwdBwdArgs& a, hipStream_t stream);

// ---- beam-search decode (decode.hip) ----
enum class Variant : int { V1 = 0, V2 = 1, Tone = 2 };

struct StepArgs {
  Variant variant;
  int B, W, Wmax, C;  // C: classes per beam (2 for v1, D for v2, tone classes)
  const float* h;     // (B,W,C)
  const float* hist;  // (B,W)
  const bool* fin;    // (B,W)
  const int* t;       // (B,W)
  const int* u;       // (B,W)
  const int* input_length;   // (B) (v1: may be null -> scalar_input_length)
  int scalar_input_length;   // v1 reference symbol: one max_t for the batch (src/lib.rs:99)
  const int* output_length;  // (B) v2
  const int* total;          // (B,W) v2
  const int* table;          // (D) v2
  int special_id;            // v2 zero_duration_id / tone empty_tone_id
  bool allow_skip, test_mode;
  int* prediction;
  float* log_prob;
  int* next_t;
  int* next_u;
  bool* next_fin;
  int* next_total;  // v2
  int* beam_branch;
  int* status;
};
int launch_decode_step(const StepArgs& a, hipStream_t stream);

// Fused multi-step decode (fused_decode.hip): all beams start at t = u = 0, log-prob 0,
// total 0, not finished; step s feeds the exact per-step contract with
//   V1:        h[w] = src[b, s, t_w, :]  (src = (B,T,U,2) lattice; live beams have u_w == s)
//   V2 / Tone: h    = src[b, s]          (src = (B,T,W,C) per-step logits)
// and the step's outputs become the next state (the role of the TF decode loop). After the
// last step the final slots are backtraced in the same launch.
struct FusedDecodeArgs {
  Variant variant;
  int B, T, U, W, C;         // U: lattice positions (V1 only); C: classes (2 for V1)
  const float* src;
  const int* table;          // (C) v2 duration_table
  const int* input_length;   // (B)
  const int* output_length;  // (B) v2
  int special_id;            // v2 zero_duration_id / tone empty_tone_id (v1: 0)
  bool allow_skip, test_mode;
  // per-step outputs (B,T,W)
  int* prediction;
  float* log_prob;
  int* next_t;
  int* next_u;
  bool* next_fin;
  int* next_total;           // v2 (required)
  int* beam_branch;
  // path outputs, each optional
  int* ordered;              // (B,W,T): order_beam_branch with final_branch = [0..W)
  int* path_pred;            // (B,W,T): prediction along each path
  int* duration;             // (B,W,T): v2 duration added at each step of each path
  int* best_beam_branch;     // (B,T): path of slot 0 (util.rs:20-33)
  int* best_t_history;       // (B,T): next_t along that path
  int* status;
};
int launch_fused_decode(const FusedDecodeArgs& a, hipStream_t stream);
int diag_decode_read(void* host, size_t bytes);  // -DSSNT_DIAG builds only

int launch_extract_best(int B, int W, int U, const int* best_final_branch, const int* beam_branch,
                        const int* t_history, int* best_beam_branch, int* best_t_history,
                        int* status, hipStream_t stream);
int launch_order_beam_branch(int B, int W, int T, const int* final_branch,
                             const int* beam_branch, int* ordered, int* status,
                             hipStream_t stream);
int launch_upsample(int B, int W, int T, int max_u, const int* duration,
                    const int* output_length, int* out, int* status, hipStream_t stream);
int launch_levenshtein(int B, int max_length, const int* a, const int* b, const int* a_len,
                       const int* b_len, int* dist, hipStream_t stream);

}  // namespace ssnt
