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
    "ssnt_fwd_bwd_set_variant": (c_int, [c_int]),
    "ssnt_fwd_bwd_last_kernel": (c_int, [ctypes.c_char_p, c_size_t]),
    "ssnt_fwd_bwd_device": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, P, P, P, P, P, P,
                                    c_size_t, P, P]),
    "ssnt_fwd_bwd_sum_device": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, P, P, P, P, P, P,
                                        c_size_t, P, P, P, P]),
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

_lib = None


def load(require_gpu: bool = False):
    """Load and bind libssnt_tts_c.so. `import torch` first so the library binds to the same
    libamdhip64 instance torch uses (same soname)."""
    global _lib
    if _lib is None:
        try:
            import torch  # noqa: F401  (shares the HIP runtime)
        except ImportError:
            pass
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"libssnt_tts_c.so not found at {LIB_PATH}: build it with `make lib` "
                "(there is no CPU fallback)")
        lib = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    if require_gpu:
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("libssnt_tts_c: no GPU visible (there is no CPU fallback)")
    return _lib


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
