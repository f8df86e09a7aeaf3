"""ctypes binding of libmmf_hip.so (include/mmf_hip.h).

The product path has no CPU fallback: if the library is missing or fails to load, `load()`
raises.  Build it with `make -C <pkg>/csrc` (or `__graft_entry__.build()`).
"""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libmmf_hip.so")

# exported symbols and their C signatures (kept in sync with include/mmf_hip.h)
_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
SIGNATURES = {
    "mmf_create": (_I, [_I, ctypes.POINTER(_P)]),
    "mmf_destroy": (None, [_P]),
    "mmf_last_error": (ctypes.c_char_p, []),
    "mmf_version": (ctypes.c_char_p, []),
    "mmf_load_tensor": (_I, [_P, ctypes.c_char_p, _I, _I, ctypes.POINTER(ctypes.c_int64), _P]),
    "mmf_finalize": (_I, [_P, _I]),
    "mmf_ready": (_I, [_P]),
    "mmf_reserve": (_I, [_P, _I, _I, _I]),
    "mmf_text_forward": (_I, [_P, _P, _P, _I, _I, _P, _P, _P, _P]),
    "mmf_effnet_forward": (_I, [_P, _P, _I, _P, _P, _P]),
    "mmf_effnet_forward_f32": (_I, [_P, _P, _I, _P, _P, _P]),
    "mmf_clip_image": (_I, [_P, _P, _I, _P, _P]),
    "mmf_clip_text": (_I, [_P, _P, _P, _I, _I, _P, _P]),
    "mmf_clip_consistency": (_I, [_P, _P, _P, _P, _I, _I, _P, _P, _P, _P]),
    "mmf_resize_pil": (_I, [_P, _P, _P, _P, _I, _I, _P, _P, _P]),
    "mmf_resize_supported": (_I, [_I, _I]),
    "mmf_jpeg_header": (_I, [_P, ctypes.c_int64, _P]),
    "mmf_jpeg_entropy": (_I, [_P, ctypes.c_int64, _P, _P]),
    "mmf_jpeg_packed_bound": (ctypes.c_int64, [ctypes.c_int32]),
    "mmf_jpeg_entropy_packed": (_I, [_P, ctypes.c_int64, _P, ctypes.c_int64, _P, _P, _P]),
    "mmf_jpeg_stage_packed": (_I, [_P, ctypes.c_int64, _P, ctypes.c_int64, _P, _P, _P, _P]),
    "mmf_jpeg_header_batch": (_I, [_P, _P, _I, _P, _P, _I]),
    "mmf_jpeg_stage_packed_batch": (_I, [_P, _P, _I, _P, ctypes.c_int64, _P, _P, _P, _P, _P, _I, _P]),
    "mmf_jpeg_reconstruct": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P]),
    "mmf_set_vault": (_I, [_P, _P, _I, _I]),
    "mmf_set_vault_normalized": (_I, [_P, _P, _I, _I]),
    "mmf_set_vault_titles": (_I, [_P, _P, _P, _I, _I, _P]),
    "mmf_vault_topk": (_I, [_P, _P, _I, _I, _F, _P, _P, _P, _P, _P, _P]),
    "mmf_fusion": (_I, [_P, _P, _I, _P, _P, _P, _P, _P]),
    "mmf_analyze_batch": (_I, [_P, _P, _P, _I, _P, _P, _I, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "mmf_profile_begin": (_I, [_P]),
    "mmf_profile_end": (_I, [_P, _I, _P, _P, _P, _P]),
    "mmf_profile_kind_name": (ctypes.c_char_p, [_I]),
    "mmf_set_option": (_I, [_P, ctypes.c_char_p, _I]),
    "mmf_get_option": (_I, [_P, ctypes.c_char_p, ctypes.POINTER(_I)]),
    "mmf_option_name": (ctypes.c_char_p, [_I]),
    "mmf_device_bytes": (ctypes.c_int64, [_P]),
    "mmf_gemm_f16": (_I, [_P, _I, _P, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "mmf_gemm_f16_ex": (_I, [_P, _I, _P, _I, _P, _P, _P, _I, _P, _I, _I, _I, _I, _I, _P]),
    "mmf_gemm_f16_split": (_I, [_P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "mmf_attention_f16": (_I, [_P, _P, _P, _I, _I, _I, _I, _P]),
}

_lib = None


class MMFError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load libmmf_hip.so and declare the ABI.  Raises MMFError (never falls back)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("MMF_HIP_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise MMFError(f"libmmf_hip.so not found at {p}; build it with `make -C {PKG_DIR}/csrc`")
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:
        raise MMFError(f"failed to load {p}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().mmf_last_error().decode(errors="replace")
        raise MMFError(f"{what or 'mmf call'} failed ({rc}): {msg}")


def set_process_option(name: str, value: int) -> None:
    """Process-wide default of a library option (mmf_set_option with a NULL handle): used by the
    handle-less ops and by handles created afterwards."""
    check(load().mmf_set_option(None, name.encode(), int(value)), f"mmf_set_option({name})")


def get_process_option(name: str) -> int:
    v = ctypes.c_int()
    check(load().mmf_get_option(None, name.encode(), ctypes.byref(v)), f"mmf_get_option({name})")
    return v.value


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None passes NULL)."""
    return None if t is None else t.data_ptr()


def stream_ptr(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
