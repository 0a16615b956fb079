/*
 * ssnt_tts_c_ab.h -- extra symbols of the A/B build of libssnt_tts_c (`make lib-ab`:
 * ssnt-tts-rust_amd/lib/ab/libssnt_tts_c_ab.so, compiled -DSSNT_AB). Tests and tuning tools only.
 *
 * The product library (include/ssnt_tts_c.h) dispatches every call by its shape alone and holds
 * no process-wide mutable state. The A/B build adds the knobs below, each PROCESS-WIDE: one
 * caller flipping one changes the kernel every other thread's next call runs. They exist to
 * force a kernel the default dispatch would not pick for a shape (parity of every kernel on
 * the same inputs) and to time alternatives. Every form they select is bit-identical to the
 * default.
 * The workspace size ssnt_fwd_bwd_workspace_size() returns holds for the knobs' values at the
 * time of the query.
 */
#ifndef SSNT_TTS_C_AB_H
#define SSNT_TTS_C_AB_H

#include <stddef.h>

#include "ssnt_tts_c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* forward-backward kernel: 0 default dispatch, 1 two-wave kernel, 2 segmented kernel at every U
 * it takes; env SSNT_FWD_BWD_KERNEL=simple selects 1 at first use */
int ssnt_fwd_bwd_set_variant(int variant);
/* segmented kernel: positions per lane (1 or 2) and the workgroup split (-1 auto, 0, 1; 2: phase 2
 * only, a study form) */
int ssnt_fwd_bwd_wide_lanes(int k);
int ssnt_fwd_bwd_wide_split(int mode);
/* streaming kernel: 0 default rings; 16 / 32 converter ring slots with the rows in the workspace */
int ssnt_fwd_bwd_stream_ring(int r);
/* fused decodes: -1 default, 0 full rank, 1 selection ordering */
int ssnt_fused_decode_select(int mode);
/* tone fused decode: waves its 20-candidate rank is split over (1, 2, 4; -1 the product's choice) */
int ssnt_fused_decode_tone_waves(int n);
/* per-step reference symbols: host staging 0 copies / 1 zero-copy; completion 0 stream
 * synchronise / 1 hipStreamWriteValue32 word / 2 flag kernel; both return the previous mode */
int ssnt_set_host_staging(int mode);
int ssnt_set_host_sync(int mode);
/* diagnostics: per-phase clock of the per-step symbols, empty-kernel launch + sync floor, and the
 * in-kernel stamps of the diagnostic build (make lib-diag; -1 elsewhere) */
int ssnt_diag_step_clock(int enable, double *out);
int ssnt_diag_null_launch(int reps, double *out);
int ssnt_diag_read(void *host, size_t bytes);
int ssnt_diag_decode_read(void *host, size_t bytes);

#ifdef __cplusplus
}
#endif

#endif /* SSNT_TTS_C_AB_H */
