"""ssnt_tts_amd -- MI355X-native SSNT alignment engine, Python host mirror.

The function names, argument order and meaning mirror the reference's Python op wrappers
``ssnt_tts_tensorflow`` (ssnt-tts-tensorflow/ssnt_tts_tensorflow/__init__.py:8,24,33,76,85,99,
130), over torch device tensors instead of TF graph tensors. Every call goes through the C ABI
of ``lib/libssnt_tts_c.so`` (include/ssnt_tts_c.h) on torch's current HIP stream; there is no CPU
fallback. Added beside them: the lattice forward-backward (``ssnt_fwd_bwd``,
``SSNTLatticeLoss``) and a fused multi-step decode (``lattice_beam_search_decode``).

Errors the reference raises by panicking (v2 "no candidate", upsample duration mismatch,
out-of-range branch) are raised here as ``SsntError`` when ``check=True`` (the default), which
synchronises the stream; pass ``check=False`` to stay asynchronous.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import SsntError, last_fwd_bwd_kernel, load, load_ab, status_string, use_ab  # noqa: F401

FLAG_TERMINAL_EMIT = 1
FLAG_ZERO_INFINITY = 2

__all__ = [
    "beam_search_decode", "extract_best_beam_branch", "ssnt_tts_v2_beam_search_decode",
    "order_beam_branch", "upsample_source_indexes", "tone_latent_beam_search_decode",
    "levenshtein_edit_distance", "ssnt_fwd_bwd", "SSNTLatticeLoss", "ssnt_lattice_loss",
    "lattice_beam_search_decode", "v2_lattice_beam_search_decode",
    "tone_latent_lattice_beam_search_decode", "v2_fwd_bwd", "V2DurationLoss", "v2_duration_loss",
    "SsntError", "FLAG_TERMINAL_EMIT", "FLAG_ZERO_INFINITY",
]


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _dev(t, dtype, name):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a GPU tensor (libssnt_tts_c has no CPU fallback)")
    if t.dtype != dtype:
        t = t.to(dtype)
    return t.contiguous()


def _status(dev):
    return torch.zeros(1, dtype=torch.int32, device=dev)


def _finish(where, rc, status, check):
    if rc != 0:
        raise SsntError(where, rc)
    if check:
        bits = int(status.item())  # synchronises
        code = load().ssnt_status_from_bits(bits)
        if code != 0:
            raise SsntError(where, code)


# ----------------------------------------------------------------------------------------------
# Reference API mirror (ssnt_tts_tensorflow/__init__.py)
# ----------------------------------------------------------------------------------------------
def beam_search_decode(h, log_prob_history, is_finished, t, u, max_t, beam_width, *, check=True):
    """One v1 emit/shift beam-search step (ssnt_tts_tensorflow/__init__.py:8-21 ->
    src/lib.rs:121-230). h (W,2) as in the reference op, or batched (B,W,2). max_t: int or
    0-d tensor (one input length for the batch, src/lib.rs:99) or a (B,) tensor.
    Returns (prediction, log_prob, next_t, next_u, next_is_finished, beam_branch)."""
    lib = load(require_gpu=True)
    squeeze = h.dim() == 2
    h = _dev(h if not squeeze else h.unsqueeze(0), torch.float32, "h")
    dev = h.device
    B, W, C = h.shape
    if W != beam_width or C != 2:
        raise ValueError("h must be (W,2) / (B,W,2) with W == beam_width")
    hist = _dev(log_prob_history.reshape(B, W), torch.float32, "log_prob_history")
    fin = _dev(is_finished.reshape(B, W), torch.bool, "is_finished")
    tt = _dev(t.reshape(B, W), torch.int32, "t")
    uu = _dev(u.reshape(B, W), torch.int32, "u")
    if isinstance(max_t, torch.Tensor) and max_t.numel() == B and max_t.dim() == 1:
        il = _dev(max_t, torch.int32, "max_t")
    else:
        il = torch.full((B,), int(max_t), dtype=torch.int32, device=dev)
    outs = [torch.empty((B, W), dtype=dt, device=dev) for dt in
            (torch.int32, torch.float32, torch.int32, torch.int32, torch.bool, torch.int32)]
    st = _status(dev)
    rc = lib.ssnt_beam_search_decode_device(_p(h), _p(hist), _p(fin), _p(tt), _p(uu), _p(il), B,
                                            W, *[_p(o) for o in outs], _p(st), _stream(dev))
    _finish("beam_search_decode", rc, st, check)
    return tuple(o[0] for o in outs) if squeeze else tuple(outs)


def extract_best_beam_branch(best_final_branch, beam_branch, t_history, beam_width, *,
                             check=True):
    """Backtrace of the best final beam (ssnt_tts_tensorflow/__init__.py:24-30 ->
    src/util.rs:20-33). beam_branch, t_history (U,W) -> (U,), (U,); batched (B,U,W) with
    best_final_branch (B,) also accepted."""
    lib = load(require_gpu=True)
    squeeze = beam_branch.dim() == 2
    bb = _dev(beam_branch if not squeeze else beam_branch.unsqueeze(0), torch.int32, "beam_branch")
    dev = bb.device
    B, U, W = bb.shape
    if W != beam_width:
        raise ValueError("beam_branch last dim must equal beam_width")
    th = _dev(t_history.reshape(B, U, W), torch.int32, "t_history")
    fb = torch.as_tensor(best_final_branch, dtype=torch.int32, device=dev).reshape(B).contiguous()
    ob = torch.empty((B, U), dtype=torch.int32, device=dev)
    ot = torch.empty((B, U), dtype=torch.int32, device=dev)
    st = _status(dev)
    rc = lib.ssnt_extract_best_beam_branch_device(_p(fb), _p(bb), _p(th), B, W, U, _p(ob), _p(ot),
                                                  _p(st), _stream(dev))
    _finish("extract_best_beam_branch", rc, st, check)
    return (ob[0], ot[0]) if squeeze else (ob, ot)


def ssnt_tts_v2_beam_search_decode(h, log_prob_history, is_finished, total_duration,
                                   duration_table, t, u, input_length, output_length, beam_width,
                                   duration_class_size, zero_duration_id, allow_skip, test_mode,
                                   *, check=True):
    """One v2 duration-class step (ssnt_tts_tensorflow/__init__.py:33-73 -> src/v2.rs:221-339).
    h (B,W,D). Returns (prediction, log_prob, next_t, next_u, next_is_finished,
    next_total_duration, beam_branch), each (B,W)."""
    lib = load(require_gpu=True)
    h = _dev(h, torch.float32, "h")
    dev = h.device
    B, W, D = h.shape
    if W != beam_width or D != duration_class_size:
        raise ValueError("h must be (B, beam_width, duration_class_size)")
    il = _dev(input_length, torch.int32, "input_length").reshape(B)
    # the reference wrapper zeroes output_length in test mode (__init__.py:47)
    ol = torch.zeros_like(il) if test_mode else _dev(output_length, torch.int32,
                                                     "output_length").reshape(B)
    args = [_dev(x.reshape(B, W), dt, n) for x, dt, n in (
        (log_prob_history, torch.float32, "log_prob_history"), (is_finished, torch.bool, "is_finished"),
        (total_duration, torch.int32, "total_duration"))]
    table = _dev(duration_table, torch.int32, "duration_table").reshape(D)
    tt = _dev(t.reshape(B, W), torch.int32, "t")
    uu = _dev(u.reshape(B, W), torch.int32, "u")
    outs = [torch.empty((B, W), dtype=dt, device=dev) for dt in
            (torch.int32, torch.float32, torch.int32, torch.int32, torch.bool, torch.int32,
             torch.int32)]
    st = _status(dev)
    rc = lib.ssnt_v2_beam_search_decode_device(
        _p(h), _p(args[0]), _p(args[1]), _p(args[2]), _p(table), _p(tt), _p(uu), _p(il), _p(ol),
        B, W, D, int(zero_duration_id), bool(allow_skip), bool(test_mode),
        *[_p(o) for o in outs], _p(st), _stream(dev))
    _finish("ssnt_tts_v2_beam_search_decode", rc, st, check)
    return tuple(outs)


def order_beam_branch(final_branch, beam_branch, beam_width, *, check=True):
    """Backtrace of every final beam (ssnt_tts_tensorflow/__init__.py:76-82 ->
    src/v2_util.rs:6-36). final_branch (B,W), beam_branch (B,T,W) -> (B,W,T)."""
    lib = load(require_gpu=True)
    bb = _dev(beam_branch, torch.int32, "beam_branch")
    dev = bb.device
    B, T, W = bb.shape
    fb = _dev(final_branch, torch.int32, "final_branch").reshape(B, W)
    out = torch.empty((B, W, T), dtype=torch.int32, device=dev)
    st = _status(dev)
    rc = lib.ssnt_order_beam_branch_device(_p(fb), _p(bb), B, W, T, _p(out), _p(st), _stream(dev))
    _finish("order_beam_branch", rc, st, check)
    return out


def upsample_source_indexes(duration, output_length, out_of_range_source_index, beam_width, *,
                            check=True):
    """Durations -> frame-to-input index map (ssnt_tts_tensorflow/__init__.py:85-96 ->
    src/v2_util.rs:39-66). duration (B,W,T), output_length (B,W); the output is
    (B,W,max(output_length)) prefilled with out_of_range_source_index like the TF op
    (upsample_source_indexes_op.cc:75,90-92)."""
    lib = load(require_gpu=True)
    d = _dev(duration, torch.int32, "duration")
    dev = d.device
    B, W, T = d.shape
    ol = _dev(output_length, torch.int32, "output_length").reshape(B, W)
    max_u = int(ol.max().item()) if ol.numel() else 0
    out = torch.full((B, W, max_u), int(out_of_range_source_index), dtype=torch.int32, device=dev)
    if max_u == 0:
        return out
    st = _status(dev)
    rc = lib.ssnt_upsample_source_indexes_device(_p(d), _p(ol), B, W, T, max_u, _p(out), _p(st),
                                                 _stream(dev))
    _finish("upsample_source_indexes", rc, st, check)
    return out


def tone_latent_beam_search_decode(h, log_prob_history, is_finished, t, u, input_length,
                                   beam_width, tone_class_size, empty_tone_id, *, check=True):
    """One tone-latent step (ssnt_tts_tensorflow/__init__.py:99-127 ->
    src/tone_latent.rs:144-234). h (B,W,C). Returns 6 (B,W) tensors."""
    lib = load(require_gpu=True)
    h = _dev(h, torch.float32, "h")
    dev = h.device
    B, W, C = h.shape
    if W != beam_width or C != tone_class_size:
        raise ValueError("h must be (B, beam_width, tone_class_size)")
    hist = _dev(log_prob_history.reshape(B, W), torch.float32, "log_prob_history")
    fin = _dev(is_finished.reshape(B, W), torch.bool, "is_finished")
    tt = _dev(t.reshape(B, W), torch.int32, "t")
    uu = _dev(u.reshape(B, W), torch.int32, "u")
    il = _dev(input_length, torch.int32, "input_length").reshape(B)
    outs = [torch.empty((B, W), dtype=dt, device=dev) for dt in
            (torch.int32, torch.float32, torch.int32, torch.int32, torch.bool, torch.int32)]
    st = _status(dev)
    rc = lib.ssnt_tone_latent_beam_search_decode_device(
        _p(h), _p(hist), _p(fin), _p(tt), _p(uu), _p(il), B, W, C, int(empty_tone_id),
        *[_p(o) for o in outs], _p(st), _stream(dev))
    _finish("tone_latent_beam_search_decode", rc, st, check)
    return tuple(outs)


def levenshtein_edit_distance(a, b, a_lengths, b_lengths, *, check=True):
    """Batched Levenshtein distance (ssnt_tts_tensorflow/__init__.py:130-134 ->
    src/edit_distance.rs:6-60). a, b (B,L); lengths (B,) -> (B,)."""
    lib = load(require_gpu=True)
    a = _dev(a, torch.int32, "a")
    dev = a.device
    B, L = a.shape
    b = _dev(b, torch.int32, "b").reshape(B, L)
    al = _dev(a_lengths, torch.int32, "a_lengths").reshape(B)
    bl = _dev(b_lengths, torch.int32, "b_lengths").reshape(B)
    if check and B and (bool((al < 0).any()) or bool((al > L).any()) or bool((bl < 0).any())
                        or bool((bl > L).any())):
        raise ValueError("lengths must be within [0, max_length] (src/edit_distance.rs:17-18)")
    out = torch.empty((B,), dtype=torch.int32, device=dev)
    if B == 0:
        return out
    if L == 0:
        return out.zero_()
    rc = lib.ssnt_levenshtein_edit_distance_device(_p(a), _p(b), _p(al), _p(bl), B, L, _p(out),
                                                   _stream(dev))
    if rc != 0:
        raise SsntError("levenshtein_edit_distance", rc)
    return out


# ----------------------------------------------------------------------------------------------
# Lattice forward-backward (DESIGN.md "Lattice semantics")
# ----------------------------------------------------------------------------------------------
def _workspace(dev, nbytes):
    """Row workspace for one call, from torch's caching allocator on the current stream: reuse
    is free after the first call, and a buffer is never shared by launches on different streams
    (the allocator tracks the stream each block was allocated on)."""
    if nbytes == 0:
        return None
    return torch.empty(nbytes, dtype=torch.uint8, device=dev)


_sum_states = {}


def _sum_state(dev, B):
    """Zeroed in-launch loss-sum state (ssnt_fwd_bwd_sum_state_size), one per (device, stream)."""
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    nbytes = int(load().ssnt_fwd_bwd_sum_state_size(B))
    t = _sum_states.get(key)
    if t is None or t.numel() < nbytes:
        t = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
        _sum_states[key] = t
    return t


def ssnt_fwd_bwd(log_trans, step_len, pos_len, log_obs=None, *, terminal_emit=True,
                 zero_infinity=False, need_grad=True, debug=False, check=False, out=None,
                 loss_sum=False, debug64=False):
    """Forward-backward over the emit/shift lattice.

    log_trans (B,T,U,2) f32 [emit, shift] natural-log probabilities; step_len / pos_len (B,)
    lattice extents S_b <= T, P_b <= U; log_obs (B,T,U) optional. Returns a dict with
    ``loss`` (B,) = -ln Z, ``grad`` (B,T,U,2) = d loss / d log_trans (if need_grad),
    ``grad_obs`` (if log_obs given and need_grad), ``log_alpha`` / ``log_beta`` (if debug).
    ``out`` may pass preallocated tensors under the same keys (reused, for benchmarking).
    ``loss_sum=True`` adds ``loss_sum`` (1,) = sum_b loss[b], formed inside the same launch in a
    fixed order (ssnt_fwd_bwd_sum_device).
    ``debug64=True`` (ssnt_fwd_bwd_debug64_device) returns ``loss``, ``log_alpha`` and
    ``log_beta`` as float64, formed on the GPU from the kernel's split-exponent state (the
    north_star's 1e-5 bar on log-alpha / log-beta is below an f32 ulp at BASELINE magnitudes).
    """
    if debug64:
        return _fwd_bwd_debug64(log_trans, step_len, pos_len, log_obs, terminal_emit,
                                zero_infinity, need_grad, check)
    lib = load(require_gpu=True)
    lt = _dev(log_trans, torch.float32, "log_trans")
    dev = lt.device
    B, T, U, two = lt.shape
    if two != 2:
        raise ValueError("log_trans must be (B,T,U,2)")
    sl = _dev(step_len, torch.int32, "step_len").reshape(B)
    pl = _dev(pos_len, torch.int32, "pos_len").reshape(B)
    lo = None if log_obs is None else _dev(log_obs, torch.float32, "log_obs").reshape(B, T, U)
    flags = (FLAG_TERMINAL_EMIT if terminal_emit else 0) | (FLAG_ZERO_INFINITY if zero_infinity else 0)
    out = dict(out or {})

    def _buf(key, shape, want):
        if not want:
            return None
        t = out.get(key)
        if t is None:
            t = torch.empty(shape, dtype=torch.float32, device=dev)
        elif tuple(t.shape) != tuple(shape) or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"out[{key!r}] must be a contiguous float32 tensor of shape {shape}")
        return t

    loss = _buf("loss", (B,), True)
    grad = _buf("grad", (B, T, U, 2), need_grad)
    gobs = _buf("grad_obs", (B, T, U), need_grad and lo is not None)
    la = _buf("log_alpha", (B, T, U), debug)
    lb = _buf("log_beta", (B, T, U), debug)
    wsb = int(lib.ssnt_fwd_bwd_workspace_size(B, T, U))
    ws = _workspace(dev, wsb)
    st = out.get("status")
    if st is None:
        st = _status(dev)
    else:
        st.zero_()
    if loss_sum:
        lsum = _buf("loss_sum", (1,), True)
        rc = lib.ssnt_fwd_bwd_sum_device(_p(lt), _p(lo), _p(sl), _p(pl), B, T, U, flags, _p(loss),
                                         _p(grad), _p(gobs), _p(la), _p(lb), _p(ws), wsb, _p(st),
                                         _p(lsum), _p(_sum_state(dev, B)), _stream(dev))
    else:
        rc = lib.ssnt_fwd_bwd_device(_p(lt), _p(lo), _p(sl), _p(pl), B, T, U, flags, _p(loss),
                                     _p(grad), _p(gobs), _p(la), _p(lb), _p(ws), wsb, _p(st),
                                     _stream(dev))
    _finish("ssnt_fwd_bwd", rc, st, check)
    res = {"loss": loss, "status": st}
    if loss_sum:
        res["loss_sum"] = lsum
    if grad is not None:
        res["grad"] = grad
    if gobs is not None:
        res["grad_obs"] = gobs
    if debug:
        res["log_alpha"] = la
        res["log_beta"] = lb
    return res


def _fwd_bwd_debug64(log_trans, step_len, pos_len, log_obs, terminal_emit, zero_infinity,
                     need_grad, check):
    lib = load(require_gpu=True)
    lt = _dev(log_trans, torch.float32, "log_trans")
    dev = lt.device
    B, T, U, two = lt.shape
    if two != 2:
        raise ValueError("log_trans must be (B,T,U,2)")
    sl = _dev(step_len, torch.int32, "step_len").reshape(B)
    pl = _dev(pos_len, torch.int32, "pos_len").reshape(B)
    lo = None if log_obs is None else _dev(log_obs, torch.float32, "log_obs").reshape(B, T, U)
    flags = (FLAG_TERMINAL_EMIT if terminal_emit else 0) | (FLAG_ZERO_INFINITY if zero_infinity else 0)
    loss = torch.empty((B,), dtype=torch.float64, device=dev)
    la = torch.empty((B, T, U), dtype=torch.float64, device=dev)
    lb = torch.empty((B, T, U), dtype=torch.float64, device=dev)
    grad = torch.empty((B, T, U, 2), dtype=torch.float32, device=dev) if need_grad else None
    gobs = torch.empty((B, T, U), dtype=torch.float32, device=dev) if need_grad and lo is not None else None
    wsb = int(lib.ssnt_fwd_bwd_debug64_workspace_size(B, T, U))
    ws = _workspace(dev, wsb)
    st = _status(dev)
    rc = lib.ssnt_fwd_bwd_debug64_device(_p(lt), _p(lo), _p(sl), _p(pl), B, T, U, flags, _p(loss),
                                         _p(grad), _p(gobs), _p(la), _p(lb), _p(ws), wsb, _p(st),
                                         _stream(dev))
    _finish("ssnt_fwd_bwd_debug64", rc, st, check)
    res = {"loss": loss, "log_alpha": la, "log_beta": lb, "status": st}
    if grad is not None:
        res["grad"] = grad
    if gobs is not None:
        res["grad_obs"] = gobs
    return res


class SSNTLatticeLoss(torch.autograd.Function):
    """Autograd wrapper: per-utterance loss (B,), gradients computed in the same kernel launch.
    The launch's status word (bad lengths, a bounded intra-kernel wait that expired) is checked
    in backward, where the step synchronises anyway (check=False skips it)."""

    @staticmethod
    def forward(ctx, log_trans, step_len, pos_len, log_obs=None, terminal_emit=True,
                zero_infinity=False, check=True):
        need = log_trans.requires_grad or (log_obs is not None and log_obs.requires_grad)
        r = ssnt_fwd_bwd(log_trans.detach(), step_len, pos_len,
                         None if log_obs is None else log_obs.detach(),
                         terminal_emit=terminal_emit, zero_infinity=zero_infinity, need_grad=need)
        ctx.save_for_backward(r.get("grad"), r.get("grad_obs"), r["status"])
        ctx.check = check
        return r["loss"]

    @staticmethod
    def backward(ctx, grad_loss):
        g, go, st = ctx.saved_tensors
        if ctx.check:
            _finish("ssnt_lattice_loss", 0, st, True)
        gl = grad_loss.to(torch.float32)
        gt = None if g is None else g * gl[:, None, None, None]
        gobs = None if go is None else go * gl[:, None, None]
        return gt, None, None, gobs, None, None, None


def ssnt_lattice_loss(log_trans, step_len, pos_len, log_obs=None, terminal_emit=True,
                      zero_infinity=False, check=True):
    return SSNTLatticeLoss.apply(log_trans, step_len, pos_len, log_obs, terminal_emit,
                                 zero_infinity, check)


# ----------------------------------------------------------------------------------------------
# F4: v2 duration-class forward-backward (DESIGN.md "Duration lattice")
# ----------------------------------------------------------------------------------------------
def v2_fwd_bwd(logits, duration_table, input_length, output_length, zero_duration_id, *,
               allow_skip=False, test_mode=False, max_total=None, zero_infinity=False,
               need_grad=True, debug=False, check=False):
    """Forward-backward over the v2 duration-class lattice: the sum over every class sequence the
    v2 decode could keep (src/v2.rs:94-166 move rules) of its probability.

    logits (B,T,D) per-step class log-probs (teacher-forced); duration_table (D,) >= 0;
    input_length / output_length (B,). ``max_total`` bounds the state totals (default
    max(output_length), read back from the device). Returns ``loss`` (B,) = -ln Z, ``grad``
    (B,T,D) = d loss / d logits (= minus the class posteriors), and with ``debug`` the rows
    ``log_alpha`` / ``log_beta`` (B,T+1,max_total+1)."""
    lib = load(require_gpu=True)
    lg = _dev(logits, torch.float32, "logits")
    dev = lg.device
    B, T, D = lg.shape
    table = _dev(duration_table, torch.int32, "duration_table").reshape(D)
    il = _dev(input_length, torch.int32, "input_length").reshape(B)
    ol = _dev(output_length, torch.int32, "output_length").reshape(B)
    if max_total is None:
        max_total = int(ol.max().item()) if B > 0 else 0
    X = int(max_total) + 1
    loss = torch.empty(B, dtype=torch.float32, device=dev)
    grad = torch.empty((B, T, D), dtype=torch.float32, device=dev) if need_grad else None
    la = torch.empty((B, T + 1, X), dtype=torch.float32, device=dev) if debug else None
    lb = torch.empty((B, T + 1, X), dtype=torch.float32, device=dev) if debug else None
    wsb = int(lib.ssnt_v2_fwd_bwd_workspace_size(B, T, int(max_total), bool(test_mode)))
    ws = _workspace(dev, wsb)
    st = _status(dev)
    rc = lib.ssnt_v2_fwd_bwd_device(_p(lg), _p(table), _p(il), _p(ol), B, T, D, int(max_total),
                                    int(zero_duration_id), bool(allow_skip), bool(test_mode),
                                    FLAG_ZERO_INFINITY if zero_infinity else 0, _p(loss),
                                    _p(grad), _p(la), _p(lb), _p(ws), wsb, _p(st), _stream(dev))
    _finish("v2_fwd_bwd", rc, st, check)
    res = {"loss": loss, "status": st}
    if grad is not None:
        res["grad"] = grad
    if debug:
        res["log_alpha"] = la
        res["log_beta"] = lb
    return res


class V2DurationLoss(torch.autograd.Function):
    """Autograd wrapper of v2_fwd_bwd: per-utterance loss (B,), gradients from the same launch."""

    @staticmethod
    def forward(ctx, logits, duration_table, input_length, output_length, zero_duration_id,
                allow_skip=False, test_mode=False, max_total=None, zero_infinity=False, check=True):
        r = v2_fwd_bwd(logits.detach(), duration_table, input_length, output_length,
                       zero_duration_id, allow_skip=allow_skip, test_mode=test_mode,
                       max_total=max_total, zero_infinity=zero_infinity,
                       need_grad=logits.requires_grad)
        ctx.save_for_backward(r.get("grad"), r["status"])
        ctx.check = check
        return r["loss"]

    @staticmethod
    def backward(ctx, grad_loss):
        g, st = ctx.saved_tensors
        if ctx.check:
            _finish("v2_duration_loss", 0, st, True)
        gl = None if g is None else g * grad_loss.to(torch.float32)[:, None, None]
        return gl, None, None, None, None, None, None, None, None, None


def v2_duration_loss(logits, duration_table, input_length, output_length, zero_duration_id,
                     allow_skip=False, test_mode=False, max_total=None, zero_infinity=False,
                     check=True):
    return V2DurationLoss.apply(logits, duration_table, input_length, output_length,
                                zero_duration_id, allow_skip, test_mode, max_total, zero_infinity,
                                check)


def lattice_beam_search_decode(lattice, input_length, beam_width, *, check=True):
    """Fused T-step v1 beam search over a (B,T,U,2) log-prob lattice: step s feeds every beam
    h = lattice[b, u, t, :] and runs the exact src/lib.rs:121-230 step; then the best final
    beam is backtraced (src/util.rs:20-33, t_history = next_t). Returns a dict of (B,T,W)
    per-step outputs plus best_beam_branch / best_t_history (B,T)."""
    lib = load(require_gpu=True)
    lat = _dev(lattice, torch.float32, "lattice")
    dev = lat.device
    B, T, U, two = lat.shape
    il = _dev(input_length, torch.int32, "input_length").reshape(B)
    W = int(beam_width)
    o = {k: torch.empty((B, T, W), dtype=dt, device=dev) for k, dt in (
        ("prediction", torch.int32), ("log_prob", torch.float32), ("next_t", torch.int32),
        ("next_u", torch.int32), ("next_is_finished", torch.bool), ("beam_branch", torch.int32))}
    o["best_beam_branch"] = torch.empty((B, T), dtype=torch.int32, device=dev)
    o["best_t_history"] = torch.empty((B, T), dtype=torch.int32, device=dev)
    st = _status(dev)
    rc = lib.ssnt_lattice_beam_search_decode_device(
        _p(lat), _p(il), B, T, U, W, _p(o["prediction"]), _p(o["log_prob"]), _p(o["next_t"]),
        _p(o["next_u"]), _p(o["next_is_finished"]), _p(o["beam_branch"]),
        _p(o["best_beam_branch"]), _p(o["best_t_history"]), _p(st), _stream(dev))
    _finish("lattice_beam_search_decode", rc, st, check)
    return o


_STEP_OUTS = (("prediction", torch.int32), ("log_prob", torch.float32), ("next_t", torch.int32),
              ("next_u", torch.int32), ("next_is_finished", torch.bool))


def v2_lattice_beam_search_decode(logits, duration_table, input_length, output_length,
                                  beam_width, zero_duration_id, allow_skip, test_mode, *,
                                  upsample=False, out_of_range_source_index=-1, check=True):
    """Fused multi-step v2 decode over per-step logits (B,T,W,D): every beam starts at
    t = u = 0, log-prob 0, total 0; step s runs the ssnt_tts_v2_beam_search_decode step
    (src/v2.rs:221-339) on h = logits[:, s] and feeds its outputs back as the next state, all in
    one launch. Returns the per-step outputs (B,T,W) under the reference op's output names,
    plus ordered_beam_branch / path_prediction / duration (B,W,T) of every final slot
    (src/v2_util.rs:6-36). upsample=True adds upsampled_source_indexes (B,W,max total) from the
    durations and each slot's final total (src/v2_util.rs:39-66)."""
    lib = load(require_gpu=True)
    lg = _dev(logits, torch.float32, "logits")
    dev = lg.device
    B, T, W, D = lg.shape
    if W != beam_width:
        raise ValueError("logits must be (B, T, beam_width, duration_class_size)")
    table = _dev(duration_table, torch.int32, "duration_table").reshape(D)
    il = _dev(input_length, torch.int32, "input_length").reshape(B)
    # the reference wrapper zeroes output_length in test mode (__init__.py:47)
    ol = torch.zeros_like(il) if test_mode else _dev(output_length, torch.int32,
                                                     "output_length").reshape(B)
    o = {k: torch.empty((B, T, W), dtype=dt, device=dev) for k, dt in _STEP_OUTS}
    o["next_total_duration"] = torch.empty((B, T, W), dtype=torch.int32, device=dev)
    o["beam_branch"] = torch.empty((B, T, W), dtype=torch.int32, device=dev)
    for k in ("ordered_beam_branch", "path_prediction", "duration"):
        o[k] = torch.empty((B, W, T), dtype=torch.int32, device=dev)
    st = _status(dev)
    rc = lib.ssnt_v2_lattice_beam_search_decode_device(
        _p(lg), _p(table), _p(il), _p(ol), B, T, W, D, int(zero_duration_id), bool(allow_skip),
        bool(test_mode), _p(o["prediction"]), _p(o["log_prob"]), _p(o["next_t"]), _p(o["next_u"]),
        _p(o["next_is_finished"]), _p(o["next_total_duration"]), _p(o["beam_branch"]),
        _p(o["ordered_beam_branch"]), _p(o["path_prediction"]), _p(o["duration"]), _p(st),
        _stream(dev))
    _finish("v2_lattice_beam_search_decode", rc, st, check)
    if upsample:
        o["upsampled_source_indexes"] = upsample_source_indexes(
            o["duration"], o["next_total_duration"][:, -1, :], out_of_range_source_index, W,
            check=check)
    return o


def tone_latent_lattice_beam_search_decode(logits, input_length, beam_width, empty_tone_id, *,
                                           check=True):
    """Fused multi-step tone-latent decode over per-step logits (B,T,W,C): the
    tone_latent_beam_search_decode step (src/tone_latent.rs:144-234) T times in one launch.
    Returns the per-step outputs (B,T,W) plus ordered_beam_branch / path_prediction (B,W,T)."""
    lib = load(require_gpu=True)
    lg = _dev(logits, torch.float32, "logits")
    dev = lg.device
    B, T, W, C = lg.shape
    if W != beam_width:
        raise ValueError("logits must be (B, T, beam_width, tone_class_size)")
    il = _dev(input_length, torch.int32, "input_length").reshape(B)
    o = {k: torch.empty((B, T, W), dtype=dt, device=dev) for k, dt in _STEP_OUTS}
    o["beam_branch"] = torch.empty((B, T, W), dtype=torch.int32, device=dev)
    for k in ("ordered_beam_branch", "path_prediction"):
        o[k] = torch.empty((B, W, T), dtype=torch.int32, device=dev)
    st = _status(dev)
    rc = lib.ssnt_tone_latent_lattice_beam_search_decode_device(
        _p(lg), _p(il), B, T, W, C, int(empty_tone_id), _p(o["prediction"]), _p(o["log_prob"]),
        _p(o["next_t"]), _p(o["next_u"]), _p(o["next_is_finished"]), _p(o["beam_branch"]),
        _p(o["ordered_beam_branch"]), _p(o["path_prediction"]), _p(st), _stream(dev))
    _finish("tone_latent_lattice_beam_search_decode", rc, st, check)
    return o
