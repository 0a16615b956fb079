"""ctypes binding of libssnt_tts_c.so (include/ssnt_tts_c.h).

The library is the product: HIP kernels for gfx950 behind a C ABI. There is no CPU fallback --
if the shared library is missing or no GPU is visible, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_PKG_ROOT = Path(__file__).resolve().parent.parent
LIB_PATH = Path(os.environ.get("SSNT_TTS_C_LIB", _PKG_ROOT / "lib" / "libssnt_tts_c.so"))
# the A/B build (make lib-ab; include/ssnt_tts_c_ab.h): the product plus process-wide kernel /
# staging / sync knobs -- tests and tools only, never the product path
AB_LIB_PATH = _PKG_ROOT / "lib" / "ab" / "libssnt_tts_c_ab.so"

c_int, c_float, c_bool, c_size_t, c_void_p = (ctypes.c_int, ctypes.c_float, ctypes.c_bool,
                                             ctypes.c_size_t, ctypes.c_void_p)
c_char_p = ctypes.c_char_p
P = c_void_p  # every array argument is passed as a raw address

# name -> (restype, [argtypes]) ; mirrors include/ssnt_tts_c.h exactly
SIGNATURES = {
    # ---- reference symbols (ssnt_tts_c/src/lib.rs) ----
    "ssnt_tts_beam_search_decode": (None, [P, P, P, P, P, c_int, c_int, P, P, P, P, P, P]),
    "ssnt_extract_best_beam_branch": (None, [c_int, P, P, c_int, c_int, P, P]),
    "ssnt_tts_v2_beam_search_decode": (None, [P, P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int,
                                              c_bool, c_bool, P, P, P, P, P, P, P]),
    "ssnt_order_beam_branch": (None, [P, P, c_int, c_int, c_int, P]),
    "ssnt_upsample_source_indexes": (None, [P, P, c_int, c_int, c_int, c_int, P]),
    "tone_latent_beam_search_decode": (None, [P, P, P, P, P, P, c_int, c_int, c_int, c_int,
                                              P, P, P, P, P, P]),
    "tone_latent_levenshtein_edit_distance": (None, [P, P, P, P, c_int, c_int, P]),
    # ---- extensions ----
    "ssnt_status_string": (c_char_p, [c_int]),
    "ssnt_status_from_bits": (c_int, [c_int]),
    "ssnt_version": (c_int, [ctypes.c_char_p, c_size_t]),
    "ssnt_fwd_bwd_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "ssnt_fwd_bwd_sum_state_size": (c_size_t, [c_int]),
    "ssnt_fwd_bwd_last_kernel": (c_int, [ctypes.c_char_p, c_size_t]),
    "ssnt_fwd_bwd_device": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, P, P, P, P, P, P,
                                    c_size_t, P, P]),
    "ssnt_fwd_bwd_sum_device": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, P, P, P, P, P, P,
                                        c_size_t, P, P, P, P]),
    "ssnt_fwd_bwd_debug64_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "ssnt_fwd_bwd_debug64_device": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, P, P, P, P,
                                            P, P, c_size_t, P, P]),
    "ssnt_fwd_bwd": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, P, P, P, P, P]),
    "ssnt_v2_fwd_bwd_workspace_size": (c_size_t, [c_int, c_int, c_int, c_bool]),
    "ssnt_v2_fwd_bwd_device": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_bool,
                                       c_bool, c_int, P, P, P, P, P, c_size_t, P, P]),
    "ssnt_beam_search_decode_device": (c_int, [P, P, P, P, P, P, c_int, c_int, P, P, P, P, P, P,
                                               P, P]),
    "ssnt_v2_beam_search_decode_device": (c_int, [P, P, P, P, P, P, P, P, P, c_int, c_int, c_int,
                                                  c_int, c_bool, c_bool, P, P, P, P, P, P, P, P,
                                                  P]),
    "ssnt_tone_latent_beam_search_decode_device": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int,
                                                           c_int, P, P, P, P, P, P, P, P]),
    "ssnt_lattice_beam_search_decode_device": (c_int, [P, P, c_int, c_int, c_int, c_int, P, P, P,
                                                       P, P, P, P, P, P, P]),
    "ssnt_v2_lattice_beam_search_decode_device": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int,
                                                          c_int, c_bool, c_bool, P, P, P, P, P, P,
                                                          P, P, P, P, P, P]),
    "ssnt_tone_latent_lattice_beam_search_decode_device": (c_int, [P, P, c_int, c_int, c_int,
                                                                   c_int, c_int, P, P, P, P, P, P,
                                                                   P, P, P, P]),
    "ssnt_extract_best_beam_branch_device": (c_int, [P, P, P, c_int, c_int, c_int, P, P, P, P]),
    "ssnt_order_beam_branch_device": (c_int, [P, P, c_int, c_int, c_int, P, P, P]),
    "ssnt_upsample_source_indexes_device": (c_int, [P, P, c_int, c_int, c_int, c_int, P, P, P]),
    "ssnt_levenshtein_edit_distance_device": (c_int, [P, P, P, P, c_int, c_int, P, P]),
}

# include/ssnt_tts_c_ab.h: the A/B build's extra symbols
AB_SIGNATURES = {
    "ssnt_fwd_bwd_set_variant": (c_int, [c_int]),
    "ssnt_fwd_bwd_wide_lanes": (c_int, [c_int]),
    "ssnt_fwd_bwd_wide_split": (c_int, [c_int]),
    "ssnt_fwd_bwd_stream_ring": (c_int, [c_int]),
    "ssnt_fused_decode_select": (c_int, [c_int]),
    "ssnt_fused_decode_tone_waves": (c_int, [c_int]),
    "ssnt_set_host_staging": (c_int, [c_int]),
    "ssnt_set_host_sync": (c_int, [c_int]),
    "ssnt_diag_step_clock": (c_int, [c_int, c_void_p]),
    "ssnt_diag_null_launch": (c_int, [c_int, c_void_p]),
    "ssnt_diag_read": (c_int, [c_void_p, c_size_t]),
    "ssnt_diag_decode_read": (c_int, [c_void_p, c_size_t]),
}

_lib = None      # the product library
_ab = None       # the A/B build, loaded on demand
_active = None   # what the mirror calls (the product unless inside use_ab())


def _bind(path: Path, sigs) -> ctypes.CDLL:
    try:
        import torch  # noqa: F401  (shares the HIP runtime)
    except ImportError:
        pass
    if not path.exists():
        raise RuntimeError(f"{path.name} not found at {path}: build it with `make` "
                           "(there is no CPU fallback)")
    lib = ctypes.CDLL(str(path))
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def load(require_gpu: bool = False):
    """Load and bind libssnt_tts_c.so (`import torch` first so the library binds to the same
    libamdhip64 instance torch uses). Inside use_ab() this returns the A/B build instead."""
    global _lib
    if _lib is None:
        _lib = _bind(LIB_PATH, SIGNATURES)
    if require_gpu:
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("libssnt_tts_c: no GPU visible (there is no CPU fallback)")
    return _active if _active is not None else _lib


def load_ab():
    """The A/B build (lib/ab/libssnt_tts_c_ab.so): every product symbol plus the knobs of
    include/ssnt_tts_c_ab.h. Own soname, so it loads beside the product library."""
    global _ab
    if _ab is None:
        _ab = _bind(AB_LIB_PATH, {**SIGNATURES, **AB_SIGNATURES})
    return _ab


class use_ab:
    """Context manager: the mirror functions call the A/B build while inside (tests that force a
    kernel or a host mode). Nestable; the outermost exit resets every knob to its default."""
    _depth = 0

    def __enter__(self):
        global _active
        load()
        _active = load_ab()
        use_ab._depth += 1
        return _active

    def __exit__(self, *exc):
        global _active
        use_ab._depth -= 1
        if use_ab._depth == 0:
            ab = load_ab()
            ab.ssnt_fwd_bwd_set_variant(0)
            ab.ssnt_fwd_bwd_wide_lanes(1)
            ab.ssnt_fwd_bwd_wide_split(-1)
            ab.ssnt_fwd_bwd_stream_ring(0)
            ab.ssnt_fused_decode_select(-1)
            ab.ssnt_fused_decode_tone_waves(-1)
            ab.ssnt_set_host_staging(1)
            ab.ssnt_set_host_sync(2)
            _active = None
        return False


def last_fwd_bwd_kernel() -> str:
    """The fwd-bwd kernel instance this thread's last ssnt_fwd_bwd* call dispatched."""
    buf = ctypes.create_string_buffer(256)
    load().ssnt_fwd_bwd_last_kernel(buf, 256)
    return buf.value.decode()


def status_string(code: int) -> str:
    return load().ssnt_status_string(int(code)).decode()


class SsntError(RuntimeError):
    def __init__(self, where: str, code: int):
        super().__init__(f"{where}: {status_string(code)} (status {code})")
        self.code = code
