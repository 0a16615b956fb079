"""CPU oracle loader -- TEST INFRASTRUCTURE ONLY.

Loads ``oracle/build/libssnt_oracle.so`` (built from ``oracle/ssnt_oracle.c`` by ``make oracle``)
and exposes numpy-in / numpy-out wrappers. Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module; the product package
(``ssnt-tts-rust_amd/``) never does. See ``oracle/ssnt_oracle.c`` for the reference citations.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "build" / "libssnt_oracle.so"
_lib = None

FLAG_TERMINAL_EMIT = 1
FLAG_ZERO_INFINITY = 2

_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_i32p = ctypes.POINTER(ctypes.c_int32)
_boolp = ctypes.POINTER(ctypes.c_bool)


def lib():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            raise RuntimeError(f"oracle not built: {_LIB_PATH} (run `make oracle`)")
        _lib = ctypes.CDLL(str(_LIB_PATH))
    return _lib


def _p(a, kind):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "oracle inputs must be C-contiguous"
    return a.ctypes.data_as(kind)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _b(a):
    return np.ascontiguousarray(a, dtype=np.bool_)


def v1_step(h, hist, fin, t, u, input_length, max_beam_width=None):
    """Batched v1 step (src/lib.rs:121-230). h (B,W,2); state (B,W); input_length (B,)."""
    h = _f32(h)
    B, W, _ = h.shape
    Wm = W if max_beam_width is None else max_beam_width
    outs = dict(
        prediction=np.zeros((B, Wm), np.int32), log_prob=np.zeros((B, Wm), np.float32),
        next_t=np.zeros((B, Wm), np.int32), next_u=np.zeros((B, Wm), np.int32),
        next_is_finished=np.zeros((B, Wm), np.bool_), beam_branch=np.zeros((B, Wm), np.int32))
    L = lib()
    rc = L.oracle_v1_step(
        B, W, Wm, _p(h, _f32p), _p(_f32(hist), _f32p), _p(_b(fin), _boolp), _p(_i32(t), _i32p),
        _p(_i32(u), _i32p), _p(_i32(input_length), _i32p), _p(outs["prediction"], _i32p),
        _p(outs["log_prob"], _f32p), _p(outs["next_t"], _i32p), _p(outs["next_u"], _i32p),
        _p(outs["next_is_finished"], _boolp), _p(outs["beam_branch"], _i32p))
    if rc != 0:
        raise RuntimeError(f"oracle_v1_step status {rc}")
    return outs


def v2_step(h, hist, fin, total, table, t, u, input_length, output_length, zero_duration_id,
            allow_skip, test_mode, max_beam_width=None):
    """Batched v2 step (src/v2.rs:221-339). Returns (outs, status)."""
    h = _f32(h)
    B, W, D = h.shape
    Wm = W if max_beam_width is None else max_beam_width
    outs = dict(
        prediction=np.zeros((B, Wm), np.int32), log_prob=np.zeros((B, Wm), np.float32),
        next_t=np.zeros((B, Wm), np.int32), next_u=np.zeros((B, Wm), np.int32),
        next_is_finished=np.zeros((B, Wm), np.bool_),
        next_total_duration=np.zeros((B, Wm), np.int32), beam_branch=np.zeros((B, Wm), np.int32))
    rc = lib().oracle_v2_step(
        B, W, Wm, D, _p(h, _f32p), _p(_f32(hist), _f32p), _p(_b(fin), _boolp),
        _p(_i32(total), _i32p), _p(_i32(table), _i32p), _p(_i32(t), _i32p), _p(_i32(u), _i32p),
        _p(_i32(input_length), _i32p), _p(_i32(output_length), _i32p), int(zero_duration_id),
        ctypes.c_bool(allow_skip), ctypes.c_bool(test_mode), _p(outs["prediction"], _i32p),
        _p(outs["log_prob"], _f32p), _p(outs["next_t"], _i32p), _p(outs["next_u"], _i32p),
        _p(outs["next_is_finished"], _boolp), _p(outs["next_total_duration"], _i32p),
        _p(outs["beam_branch"], _i32p))
    return outs, rc


def tone_step(h, hist, fin, t, u, input_length, empty_tone_id, max_beam_width=None):
    """Batched tone-latent step (src/tone_latent.rs:144-234)."""
    h = _f32(h)
    B, W, C = h.shape
    Wm = W if max_beam_width is None else max_beam_width
    outs = dict(
        prediction=np.zeros((B, Wm), np.int32), log_prob=np.zeros((B, Wm), np.float32),
        next_t=np.zeros((B, Wm), np.int32), next_u=np.zeros((B, Wm), np.int32),
        next_is_finished=np.zeros((B, Wm), np.bool_), beam_branch=np.zeros((B, Wm), np.int32))
    rc = lib().oracle_tone_step(
        B, W, Wm, C, _p(h, _f32p), _p(_f32(hist), _f32p), _p(_b(fin), _boolp),
        _p(_i32(t), _i32p), _p(_i32(u), _i32p), _p(_i32(input_length), _i32p),
        int(empty_tone_id), _p(outs["prediction"], _i32p), _p(outs["log_prob"], _f32p),
        _p(outs["next_t"], _i32p), _p(outs["next_u"], _i32p),
        _p(outs["next_is_finished"], _boolp), _p(outs["beam_branch"], _i32p))
    if rc != 0:
        raise RuntimeError(f"oracle_tone_step status {rc}")
    return outs


def extract_best_beam_branch(best_final_branch, beam_branch, t_history):
    """util::extract_best_beam_branch_kernel (src/util.rs:20-33); beam_branch (U,W)."""
    bb = _i32(beam_branch)
    th = _i32(t_history)
    U, W = bb.shape
    out = np.zeros(U, np.int32)
    out_t = np.zeros(U, np.int32)
    lib().oracle_extract_best_beam_branch(int(best_final_branch), _p(bb, _i32p), _p(th, _i32p),
                                          W, U, _p(out, _i32p), _p(out_t, _i32p))
    return out, out_t


def order_beam_branch(final_branch, beam_branch):
    """v2_util::order_beam_branch (src/v2_util.rs:6-36): (B,W),(B,T,W) -> (B,W,T)."""
    fb = _i32(final_branch)
    bb = _i32(beam_branch)
    B, T, W = bb.shape
    out = np.zeros((B, W, T), np.int32)
    lib().oracle_order_beam_branch(B, W, T, _p(fb, _i32p), _p(bb, _i32p), _p(out, _i32p))
    return out


def upsample_source_indexes(duration, output_length, max_u, fill=-1):
    """v2_util::upsample_source_indexes (src/v2_util.rs:39-66) + the TF op prefill."""
    d = _i32(duration)
    B, W, T = d.shape
    out = np.full((B, W, max_u), fill, np.int32)
    rc = lib().oracle_upsample_source_indexes(B, W, T, int(max_u), _p(d, _i32p),
                                              _p(_i32(output_length), _i32p), _p(out, _i32p))
    return out, rc


def levenshtein(a, b, a_len, b_len):
    """edit_distance::levenshtein_edit_distance (src/edit_distance.rs:6-31)."""
    a = _i32(a)
    b = _i32(b)
    B, L = a.shape
    out = np.zeros(B, np.int32)
    lib().oracle_levenshtein(B, L, _p(a, _i32p), _p(b, _i32p), _p(_i32(a_len), _i32p),
                             _p(_i32(b_len), _i32p), _p(out, _i32p))
    return out


def v1_lattice_decode(lattice, input_length, beam_width, n_threads=0):
    """Fused multi-step v1 decode over a (B,T,U,2) lattice (config 3 workload)."""
    lat = _f32(lattice)
    B, T, U, _ = lat.shape
    W = beam_width
    o = dict(prediction=np.zeros((B, T, W), np.int32), log_prob=np.zeros((B, T, W), np.float32),
             next_t=np.zeros((B, T, W), np.int32), next_u=np.zeros((B, T, W), np.int32),
             next_is_finished=np.zeros((B, T, W), np.bool_),
             beam_branch=np.zeros((B, T, W), np.int32),
             best_beam_branch=np.zeros((B, T), np.int32),
             best_t_history=np.zeros((B, T), np.int32))
    rc = lib().oracle_v1_lattice_decode(
        B, T, U, W, _p(lat, _f32p), _p(_i32(input_length), _i32p), _p(o["prediction"], _i32p),
        _p(o["log_prob"], _f32p), _p(o["next_t"], _i32p), _p(o["next_u"], _i32p),
        _p(o["next_is_finished"], _boolp), _p(o["beam_branch"], _i32p),
        _p(o["best_beam_branch"], _i32p), _p(o["best_t_history"], _i32p), int(n_threads))
    if rc != 0:
        raise RuntimeError(f"oracle_v1_lattice_decode status {rc}")
    return o


def _fused_outs(B, T, W, v2):
    o = dict(prediction=np.zeros((B, T, W), np.int32), log_prob=np.zeros((B, T, W), np.float32),
             next_t=np.zeros((B, T, W), np.int32), next_u=np.zeros((B, T, W), np.int32),
             next_is_finished=np.zeros((B, T, W), np.bool_))
    if v2:
        o["next_total_duration"] = np.zeros((B, T, W), np.int32)
    o["beam_branch"] = np.zeros((B, T, W), np.int32)
    o["ordered_beam_branch"] = np.zeros((B, W, T), np.int32)
    o["path_prediction"] = np.zeros((B, W, T), np.int32)
    if v2:
        o["duration"] = np.zeros((B, W, T), np.int32)
    return o


def v2_lattice_decode(logits, duration_table, input_length, output_length, zero_duration_id,
                      allow_skip, test_mode, n_threads=0):
    """Fused multi-step v2 decode over per-step logits (B,T,W,D) (configs[4] v2 path): the
    v2 step (src/v2.rs:221-339) T times from the all-zero state, then the backtrace of every
    final slot (src/v2_util.rs:6-36). Returns (outs, status); test_mode zeroes output_length
    like the reference wrapper (__init__.py:47)."""
    lg = _f32(logits)
    B, T, W, D = lg.shape
    ol = np.zeros(B, np.int32) if test_mode else _i32(output_length)
    o = _fused_outs(B, T, W, True)
    rc = lib().oracle_v2_lattice_decode(
        B, T, W, D, _p(lg, _f32p), _p(_i32(duration_table), _i32p), _p(_i32(input_length), _i32p),
        _p(ol, _i32p), int(zero_duration_id), ctypes.c_bool(allow_skip), ctypes.c_bool(test_mode),
        _p(o["prediction"], _i32p), _p(o["log_prob"], _f32p), _p(o["next_t"], _i32p),
        _p(o["next_u"], _i32p), _p(o["next_is_finished"], _boolp),
        _p(o["next_total_duration"], _i32p), _p(o["beam_branch"], _i32p),
        _p(o["ordered_beam_branch"], _i32p), _p(o["path_prediction"], _i32p),
        _p(o["duration"], _i32p), int(n_threads))
    return o, rc


def tone_lattice_decode(logits, input_length, empty_tone_id, n_threads=0):
    """Fused multi-step tone-latent decode over per-step logits (B,T,W,C) (configs[4] tone
    path): the tone step (src/tone_latent.rs:144-234) T times, then every final slot's path."""
    lg = _f32(logits)
    B, T, W, C = lg.shape
    o = _fused_outs(B, T, W, False)
    rc = lib().oracle_tone_lattice_decode(
        B, T, W, C, _p(lg, _f32p), _p(_i32(input_length), _i32p), int(empty_tone_id),
        _p(o["prediction"], _i32p), _p(o["log_prob"], _f32p), _p(o["next_t"], _i32p),
        _p(o["next_u"], _i32p), _p(o["next_is_finished"], _boolp), _p(o["beam_branch"], _i32p),
        _p(o["ordered_beam_branch"], _i32p), _p(o["path_prediction"], _i32p), int(n_threads))
    if rc != 0:
        raise RuntimeError(f"oracle_tone_lattice_decode status {rc}")
    return o


def fwd_bwd_xf(log_trans, step_len, pos_len, log_obs=None, flags=FLAG_TERMINAL_EMIT,
               debug=False, n_threads=0):
    """Exact split-exponent f32 fwd-bwd (the arithmetic the HIP kernel reproduces bit-exactly)."""
    lt = _f32(log_trans)
    B, T, U, _ = lt.shape
    lo = None if log_obs is None else _f32(log_obs)
    loss = np.zeros(B, np.float32)
    grad = np.zeros((B, T, U, 2), np.float32)
    gobs = None if lo is None else np.zeros((B, T, U), np.float32)
    la = np.zeros((B, T, U), np.float32) if debug else None
    lb = np.zeros((B, T, U), np.float32) if debug else None
    lib().oracle_fwd_bwd_xf(B, T, U, _p(lt, _f32p), _p(lo, _f32p), _p(_i32(step_len), _i32p),
                            _p(_i32(pos_len), _i32p), int(flags), _p(loss, _f32p),
                            _p(grad, _f32p), _p(gobs, _f32p), _p(la, _f32p), _p(lb, _f32p),
                            int(n_threads))
    out = dict(loss=loss, grad=grad)
    if gobs is not None:
        out["grad_obs"] = gobs
    if debug:
        out["log_alpha"] = la
        out["log_beta"] = lb
    return out


XF_DTYPE = np.dtype([("m", np.float32), ("e", np.int32)])
LN2_F64 = 0.6931471805599453


def xf_log64(state):
    """float64 natural log of split-exponent values {m, e}: e*ln2 + ln(m) (zeros -> -inf)."""
    m = state["m"].astype(np.float64)
    out = np.full(m.shape, -np.inf)
    nz = m != 0.0
    out[nz] = state["e"][nz].astype(np.float64) * LN2_F64 + np.log(m[nz])
    return out


def fwd_bwd_xf_state(log_trans, step_len, pos_len, log_obs=None, flags=FLAG_TERMINAL_EMIT,
                     n_threads=0):
    """The split-exponent fwd-bwd's own normalized state: alpha / beta (B,T,U) and Z (B) as
    XF_DTYPE records (what ssnt_fwd_bwd_debug64_device forms its float64 logs from)."""
    lt = _f32(log_trans)
    B, T, U, _ = lt.shape
    lo = None if log_obs is None else _f32(log_obs)
    loss = np.zeros(B, np.float32)
    grad = np.zeros((B, T, U, 2), np.float32)
    al = np.zeros((B, T, U), XF_DTYPE)
    be = np.zeros((B, T, U), XF_DTYPE)
    z = np.zeros(B, XF_DTYPE)
    vp = ctypes.c_void_p
    lib().oracle_fwd_bwd_xf_state(B, T, U, _p(lt, _f32p), _p(lo, _f32p),
                                  _p(_i32(step_len), _i32p), _p(_i32(pos_len), _i32p), int(flags),
                                  _p(loss, _f32p), _p(grad, _f32p), vp(al.ctypes.data),
                                  vp(be.ctypes.data), vp(z.ctypes.data), int(n_threads))
    return dict(loss=loss, grad=grad, alpha=al, beta=be, z=z)


def fwd_bwd_f64(log_trans, step_len, pos_len, log_obs=None, flags=FLAG_TERMINAL_EMIT):
    """Independent float64 log-domain DP: the mathematical definition of the lattice."""
    lt = _f32(log_trans)
    B, T, U, _ = lt.shape
    lo = None if log_obs is None else _f32(log_obs)
    loss = np.zeros(B, np.float64)
    grad = np.zeros((B, T, U, 2), np.float64)
    gobs = None if lo is None else np.zeros((B, T, U), np.float64)
    la = np.zeros((B, T, U), np.float64)
    lb = np.zeros((B, T, U), np.float64)
    lib().oracle_fwd_bwd_f64(B, T, U, _p(lt, _f32p), _p(lo, _f32p), _p(_i32(step_len), _i32p),
                             _p(_i32(pos_len), _i32p), int(flags), _p(loss, _f64p),
                             _p(grad, _f64p), _p(gobs, _f64p), _p(la, _f64p), _p(lb, _f64p))
    out = dict(loss=loss, grad=grad, log_alpha=la, log_beta=lb)
    if gobs is not None:
        out["grad_obs"] = gobs
    return out


def max_threads():
    return int(lib().oracle_omp_max_threads())


# ---- synthetic inputs shared by tests and bench (counter-based, reproducible) ----------------
def synth_log_trans(B, T, U, seed=0, scale=1.5):
    """log_softmax over k of z ~ N(0, scale^2), f32, shape (B,T,U,2)."""
    rng = np.random.default_rng(seed)
    z = rng.standard_normal((B, T, U, 2), dtype=np.float32) * np.float32(scale)
    m = z.max(axis=-1, keepdims=True)
    lse = m + np.log(np.exp(z - m).sum(axis=-1, keepdims=True))
    return (z - lse).astype(np.float32)


def synth_tie_rich_log_trans(B, T, U, seed=0):
    """Tie-rich lattice: p in {0.1,...,0.9}, ln in f32, like the reference tests
    (tests/test_decoding.rs:8, ssnt-tts-tensorflow/tests/test_beam_search_op.py:37-38)."""
    rng = np.random.default_rng(seed)
    p = (rng.integers(1, 10, size=(B, T, U, 1)) / 10.0).astype(np.float32)
    pe = p
    ps = (np.float32(1.0) - p).astype(np.float32)
    return np.log(np.concatenate([pe, ps], axis=-1).astype(np.float32)).astype(np.float32)


def synth_durations(B, I, O, D, seed=0):
    """Per-utterance duration sequences d (B,I) in [1, D-1] with sum == O[b] over the first
    I[b] positions (0 after), each prefix inside v2's band around the diagonal
    (src/v2.rs:94-104): the path the v2 decode must find."""
    rng = np.random.default_rng(seed)
    I = np.broadcast_to(np.asarray(I, np.int64), (B,))
    O = np.broadcast_to(np.asarray(O, np.int64), (B,))
    d = np.zeros((B, int(I.max())), np.int32)
    for b in range(B):
        n, tot = int(I[b]), int(O[b])
        base = tot / n
        x = np.clip(np.round(base + rng.normal(0, 1.0, n)), 1, D - 1).astype(np.int64)
        # fix the sum one step at a time, on random positions with room
        while x.sum() != tot:
            j = rng.integers(n)
            if x.sum() < tot and x[j] < D - 1:
                x[j] += 1
            elif x.sum() > tot and x[j] > 1:
                x[j] -= 1
        d[b, :n] = x
    return d


def synth_v2_logits(durations, W, D, seed=0, margin=8.0, tie_rich=False):
    """Per-step logits (B,T,W,D) peaked at the sampled duration class of each step (class index
    == duration with duration_table = [0..D-1]). tie_rich: ln of probabilities in {0.1..0.3}
    with 0.9 at the peak (f32), so equal log-probs are everywhere."""
    rng = np.random.default_rng(seed)
    B, T = durations.shape
    if tie_rich:
        p = rng.integers(1, 4, size=(B, T, W, D)).astype(np.float32) / np.float32(10.0)
        onehot = np.eye(D, dtype=bool)[durations][:, :, None, :]
        p = np.where(onehot, np.float32(0.9), p).astype(np.float32)
        return np.log(p).astype(np.float32)
    z = rng.standard_normal((B, T, W, D)).astype(np.float32)
    z += np.float32(margin) * np.eye(D, dtype=np.float32)[durations][:, :, None, :]
    m = z.max(axis=-1, keepdims=True)
    return (z - (m + np.log(np.exp(z - m).sum(axis=-1, keepdims=True)))).astype(np.float32)


def synth_tone_logits(B, T, W, C, seed=0, tie_rich=False):
    """Per-step tone logits (B,T,W,C): log_softmax of N(0,1.5^2), or tie-rich ln(p) with p in
    {0.1..0.9}."""
    rng = np.random.default_rng(seed)
    if tie_rich:
        return np.log((rng.integers(1, 10, size=(B, T, W, C)) / 10.0).astype(np.float32)).astype(np.float32)
    z = rng.standard_normal((B, T, W, C)).astype(np.float32) * np.float32(1.5)
    m = z.max(axis=-1, keepdims=True)
    return (z - (m + np.log(np.exp(z - m).sum(axis=-1, keepdims=True)))).astype(np.float32)


def v2_fwd_bwd(logits, duration_table, input_length, output_length, max_total, zero_duration_id,
               allow_skip, test_mode, flags=0, debug=False, n_threads=0):
    """F4: v2 duration-class fwd-bwd, exact split-exponent arithmetic (the bits the HIP kernel
    reproduces). logits (B,I,D). Returns dict(loss, grad[, log_alpha, log_beta])."""
    lg = _f32(logits)
    B, I, D = lg.shape
    X = int(max_total) + 1
    loss = np.zeros(B, np.float32)
    grad = np.zeros((B, I, D), np.float32)
    la = np.zeros((B, I + 1, X), np.float32) if debug else None
    lb = np.zeros((B, I + 1, X), np.float32) if debug else None
    rc = lib().oracle_v2_fwd_bwd(
        B, I, D, int(max_total), _p(lg, _f32p), _p(_i32(duration_table), _i32p),
        _p(_i32(input_length), _i32p), _p(_i32(output_length), _i32p), int(zero_duration_id),
        ctypes.c_bool(allow_skip), ctypes.c_bool(test_mode), int(flags), _p(loss, _f32p),
        _p(grad, _f32p), _p(la, _f32p), _p(lb, _f32p), int(n_threads))
    if rc != 0:
        raise RuntimeError(f"oracle_v2_fwd_bwd status {rc}")
    out = dict(loss=loss, grad=grad)
    if debug:
        out["log_alpha"] = la
        out["log_beta"] = lb
    return out


def v2_fwd_bwd_f64(logits, duration_table, input_length, output_length, max_total,
                   zero_duration_id, allow_skip, test_mode):
    """F4 float64 log-domain definition (rules applied per move, no windows)."""
    lg = _f32(logits)
    B, I, D = lg.shape
    loss = np.zeros(B, np.float64)
    grad = np.zeros((B, I, D), np.float64)
    lib().oracle_v2_fwd_bwd_f64(
        B, I, D, int(max_total), _p(lg, _f32p), _p(_i32(duration_table), _i32p),
        _p(_i32(input_length), _i32p), _p(_i32(output_length), _i32p), int(zero_duration_id),
        ctypes.c_bool(allow_skip), ctypes.c_bool(test_mode), _p(loss, _f64p), _p(grad, _f64p))
    return dict(loss=loss, grad=grad)


def synth_v2_step_logits(durations, D, seed=0, margin=3.0):
    """Teacher-forced per-step class logits (B,I,D) for the F4 fwd-bwd: log_softmax of N(0,1)
    plus `margin` at each step's sampled duration class (duration_table = [0..D-1])."""
    rng = np.random.default_rng(seed)
    B, T = durations.shape
    z = rng.standard_normal((B, T, D)).astype(np.float32)
    z += np.float32(margin) * np.eye(D, dtype=np.float32)[durations]
    m = z.max(axis=-1, keepdims=True)
    return (z - (m + np.log(np.exp(z - m).sum(axis=-1, keepdims=True)))).astype(np.float32)
