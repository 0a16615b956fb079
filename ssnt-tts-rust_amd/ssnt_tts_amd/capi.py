"""Host-pointer access to the seven reference symbols of libssnt_tts_c (numpy in, numpy out).

This is exactly the binding the reference's TF ops use (extern "C", host arrays, synchronous;
ssnt-tts-tensorflow/src/*_op.cc), exposed for tests and for callers without torch. Each call
runs on the GPU through the library's per-thread stream and staging buffers.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import load


def _a(x, dt):
    return np.ascontiguousarray(x, dtype=dt)


def _p(a):
    # data_as keeps a reference to the array, so temporaries built in the argument list stay
    # alive for the duration of the call
    return a.ctypes.data_as(ctypes.c_void_p)


def ssnt_tts_beam_search_decode(h, log_prob_history, is_finished, t, u, max_t, beam_width):
    """ssnt_tts_c/src/lib.rs:11-83 (batch fixed to 1). Returns 6 arrays of length W."""
    W = int(beam_width)
    h, hist = _a(h, np.float32).reshape(W, 2), _a(log_prob_history, np.float32)
    fin, tt, uu = _a(is_finished, np.bool_), _a(t, np.int32), _a(u, np.int32)
    outs = [np.empty(W, dt) for dt in (np.int32, np.float32, np.int32, np.int32, np.bool_, np.int32)]
    load().ssnt_tts_beam_search_decode(_p(h), _p(hist), _p(fin), _p(tt), _p(uu), int(max_t), W,
                                       *[_p(o) for o in outs])
    return tuple(outs)


def ssnt_extract_best_beam_branch(best_final_branch, beam_branch, t_history, beam_width, max_u):
    """ssnt_tts_c/src/lib.rs:87-116. beam_branch, t_history (max_u, W)."""
    bb, th = _a(beam_branch, np.int32), _a(t_history, np.int32)
    ob, ot = np.empty(max_u, np.int32), np.empty(max_u, np.int32)
    load().ssnt_extract_best_beam_branch(int(best_final_branch), _p(bb), _p(th), int(beam_width),
                                         int(max_u), _p(ob), _p(ot))
    return ob, ot


def ssnt_tts_v2_beam_search_decode(h, log_prob_history, is_finished, total_duration,
                                   duration_table, t, u, input_length, output_length, batch_size,
                                   beam_width, duration_class_size, zero_duration_id, allow_skip,
                                   test_mode):
    """ssnt_tts_c/src/lib.rs:119-218. Returns 7 (B,W) arrays."""
    B, W, D = int(batch_size), int(beam_width), int(duration_class_size)
    ins = [_a(h, np.float32), _a(log_prob_history, np.float32), _a(is_finished, np.bool_),
           _a(total_duration, np.int32), _a(duration_table, np.int32), _a(t, np.int32),
           _a(u, np.int32), _a(input_length, np.int32), _a(output_length, np.int32)]
    outs = [np.empty((B, W), dt) for dt in
            (np.int32, np.float32, np.int32, np.int32, np.bool_, np.int32, np.int32)]
    load().ssnt_tts_v2_beam_search_decode(*[_p(x) for x in ins], B, W, D, int(zero_duration_id),
                                          bool(allow_skip), bool(test_mode), *[_p(o) for o in outs])
    return tuple(outs)


def ssnt_order_beam_branch(final_branch, beam_branch, batch_size, beam_width, max_t):
    """ssnt_tts_c/src/lib.rs:221-241 -> (B,W,T)."""
    fb, bb = _a(final_branch, np.int32), _a(beam_branch, np.int32)
    out = np.empty((batch_size, beam_width, max_t), np.int32)
    load().ssnt_order_beam_branch(_p(fb), _p(bb), int(batch_size), int(beam_width), int(max_t),
                                  _p(out))
    return out


def ssnt_upsample_source_indexes(duration, output_length, batch_size, beam_width, max_t, max_u,
                                 fill=-1):
    """ssnt_tts_c/src/lib.rs:245-265; `fill` plays the TF op's prefill."""
    d, ol = _a(duration, np.int32), _a(output_length, np.int32)
    out = np.full((batch_size, beam_width, max_u), fill, np.int32)
    load().ssnt_upsample_source_indexes(_p(d), _p(ol), int(batch_size), int(beam_width),
                                        int(max_t), int(max_u), _p(out))
    return out


def tone_latent_beam_search_decode(h, log_prob_history, is_finished, t, u, input_length,
                                   batch_size, beam_width, tone_class_size, empty_tone_id):
    """ssnt_tts_c/src/lib.rs:268-343. Returns 6 (B,W) arrays."""
    B, W = int(batch_size), int(beam_width)
    ins = [_a(h, np.float32), _a(log_prob_history, np.float32), _a(is_finished, np.bool_),
           _a(t, np.int32), _a(u, np.int32), _a(input_length, np.int32)]
    outs = [np.empty((B, W), dt) for dt in (np.int32, np.float32, np.int32, np.int32, np.bool_, np.int32)]
    load().tone_latent_beam_search_decode(*[_p(x) for x in ins], B, W, int(tone_class_size),
                                          int(empty_tone_id), *[_p(o) for o in outs])
    return tuple(outs)


def tone_latent_levenshtein_edit_distance(a, b, a_lengths, b_lengths, batch_size, max_length):
    """ssnt_tts_c/src/lib.rs:347-381."""
    ins = [_a(a, np.int32), _a(b, np.int32), _a(a_lengths, np.int32), _a(b_lengths, np.int32)]
    out = np.empty(batch_size, np.int32)
    load().tone_latent_levenshtein_edit_distance(*[_p(x) for x in ins], int(batch_size),
                                                 int(max_length), _p(out))
    return out


def ssnt_fwd_bwd(log_trans, step_len, pos_len, log_obs=None, flags=1, debug=False):
    """Host-pointer lattice forward-backward (synchronous)."""
    lt = _a(log_trans, np.float32)
    B, T, U, _ = lt.shape
    lo = None if log_obs is None else _a(log_obs, np.float32)
    loss = np.empty(B, np.float32)
    grad = np.empty((B, T, U, 2), np.float32)
    gobs = None if lo is None else np.empty((B, T, U), np.float32)
    la = np.empty((B, T, U), np.float32) if debug else None
    lb = np.empty((B, T, U), np.float32) if debug else None
    nul = ctypes.c_void_p(None)
    rc = load().ssnt_fwd_bwd(_p(lt), nul if lo is None else _p(lo), _p(_a(step_len, np.int32)),
                             _p(_a(pos_len, np.int32)), B, T, U, int(flags), _p(loss), _p(grad),
                             nul if gobs is None else _p(gobs), nul if la is None else _p(la),
                             nul if lb is None else _p(lb))
    if rc != 0:
        from ._lib import SsntError
        raise SsntError("ssnt_fwd_bwd", rc)
    out = {"loss": loss, "grad": grad}
    if gobs is not None:
        out["grad_obs"] = gobs
    if debug:
        out["log_alpha"], out["log_beta"] = la, lb
    return out
