"""ctypes binding of libaudiolcm_hip.so (the C-ABI declared in include/audiolcm_hip.h).

The library is built in-tree (``audiolcm_amd/libaudiolcm_hip.so``) by
``__graft_entry__.build()`` / ``make -C audiolcm_amd/csrc``.  There is no
fallback: if the library is missing or the device is not gfx950 every call
raises, so a GPU run can never silently take a CPU or eager-PyTorch path.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ALCM_LIB", os.path.join(HERE, "libaudiolcm_hip.so"))

ALCM_OPND_ACT, ALCM_OPND_ACT_T, ALCM_OPND_WEIGHT = 0, 1, 2
ALCM_MODEL_DIT, ALCM_MODEL_VAE, ALCM_MODEL_BIGVGAN, ALCM_MODEL_TEXT, ALCM_MODEL_MEL = 0, 1, 2, 3, 4
ACT_NONE, ACT_SILU, ACT_GELU_ERF, ACT_GELU_TANH, ACT_TANH = 0, 1, 2, 3, 4
PREC_BF16, PREC_SPLIT, PREC_F16, PREC_F16W2 = 0, 1, 2, 3   # per-launch MFMA operand precision
POLICY_BF16, POLICY_SPLIT, POLICY_MIXED = 0, 1, 2      # per-model precision policy
POLICIES = {"bf16": POLICY_BF16, "split": POLICY_SPLIT, "mixed": POLICY_MIXED}

i64 = C.c_int64
vp = C.c_void_p
fp = C.c_void_p  # float* passed as raw device address


class Operand(C.Structure):
    _fields_ = [("kind", C.c_int), ("ptr", vp), ("sb", i64), ("st", i64), ("sc", i64),
                ("T_in", C.c_int), ("C_in", C.c_int), ("Cpad", C.c_int), ("ksize", C.c_int), ("dil", C.c_int),
                ("pad", C.c_int), ("up", C.c_int), ("rows_per_batch", C.c_int), ("rows", C.c_int),
                ("zs1", i64), ("zs2", i64), ("pro_scale", fp), ("pro_shift", fp), ("pro_sb", i64),
                ("pro_mean", fp), ("pro_rstd", fp), ("pro_act", C.c_int), ("w_lo_off", i64)]


class GemmArgs(C.Structure):
    _fields_ = [("M", C.c_int), ("N", C.c_int), ("Kpad", C.c_int), ("batch", C.c_int), ("zdiv", C.c_int),
                ("a", Operand), ("b", Operand), ("bias", fp), ("acc_scale", C.c_float), ("out_scale", C.c_float),
                ("act", C.c_int), ("accumulate", C.c_int), ("geglu", C.c_int), ("res", fp),
                ("r_sb", i64), ("r_st", i64), ("r_sc", i64), ("r_zs1", i64), ("r_zs2", i64), ("out", fp),
                ("o_sb", i64), ("o_st", i64), ("o_sc", i64), ("o_zs1", i64), ("o_zs2", i64),
                ("out_rows_per_batch", C.c_int), ("out_step", C.c_int), ("out_off", C.c_int), ("prec", C.c_int),
                ("disable_window", C.c_int), ("tile_n", C.c_int)]


class OpConvArgs(C.Structure):
    _fields_ = [("a", vp), ("a_lo_off", i64), ("B", C.c_int), ("T", C.c_int), ("C", C.c_int), ("Cp", C.c_int),
                ("ksize", C.c_int), ("dil", C.c_int), ("pad", C.c_int), ("w", vp), ("w_lo_off", i64),
                ("kpad", C.c_int), ("N", C.c_int), ("bias", fp), ("res", fp), ("out", fp), ("out_act", C.c_int),
                ("accumulate", C.c_int), ("out_scale", C.c_float), ("prec", C.c_int),
                ("act_plane", vp), ("act_plane_lo_off", i64), ("act_alpha_exp", fp), ("act_inv_beta", fp),
                ("act_up_filter", fp), ("act_down_filter", fp), ("geglu_plane", vp),
                ("out_stride", C.c_int), ("out_offset", C.c_int), ("out_rows", C.c_int), ("out_plane", vp),
                ("ksplit_ws", fp), ("ksplit_ws_floats", i64)]


class NamedTensor(C.Structure):
    _fields_ = [("name", C.c_char_p), ("data", vp), ("ndim", C.c_int), ("shape", i64 * 4)]


class ProfEntry(C.Structure):
    _fields_ = [("name", C.c_char * 128), ("launches", i64), ("total_ms", C.c_double), ("flops", C.c_double),
                ("bytes", C.c_double), ("roof_ms", C.c_double), ("hbm_launches", i64), ("hbm_ms", C.c_double),
                ("hbm_bytes", C.c_double)]


# (name, restype, argtypes) — every symbol include/audiolcm_hip.h declares
_SIGS = [
    ("alcm_last_error", C.c_char_p, []),
    ("alcm_version", C.c_int, []),
    ("alcm_check_device", C.c_int, [C.c_int]),
    ("alcm_gemm", C.c_int, [C.POINTER(GemmArgs), vp]),
    ("alcm_pack_conv_weight", C.c_int, [fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                        vp, vp]),
    ("alcm_group_norm_affine", C.c_int, [fp, C.c_int, C.c_int, C.c_int, i64, i64, C.c_int, C.c_float, fp, fp, fp,
                                         fp, vp]),
    ("alcm_row_stats", C.c_int, [fp, C.c_int, C.c_int, i64, C.c_float, fp, fp, vp]),
    ("alcm_layer_norm", C.c_int, [fp, C.c_int, C.c_int, i64, C.c_float, fp, fp, fp, i64, fp, i64, vp]),
    ("alcm_softmax_rows", C.c_int, [fp, C.c_int, C.c_int, i64, vp]),
    ("alcm_activation1d", C.c_int, [fp, fp, C.c_int, C.c_int, C.c_int, i64, i64, fp, fp, fp, fp, vp]),
    ("alcm_activation1d_op", C.c_int, [fp, vp, C.c_int, C.c_int, C.c_int, C.c_int, fp, fp, fp, fp, C.c_int, vp]),
    ("alcm_activation1d_op_f16in", C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, fp, fp, fp, fp, C.c_int, vp]),
    ("alcm_opconv", C.c_int, [C.POINTER(OpConvArgs), vp]),
    ("alcm_opconv_sum", C.c_int, [C.POINTER(OpConvArgs), C.c_int, vp]),
    ("alcm_opconv_dense", C.c_int, [C.POINTER(OpConvArgs), vp]),
    ("alcm_flash_attention", C.c_int, [fp, fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp]),
    ("alcm_layer_norm_plane", C.c_int, [fp, C.c_int, C.c_int, i64, C.c_float, fp, fp, vp, C.c_int, vp]),
    ("alcm_lcm_step", C.c_int, [fp, fp, fp, C.POINTER(C.c_float), fp, fp, i64, vp]),
    ("alcm_lcm_step_cfg", C.c_int, [fp, fp, fp, C.c_float, fp, C.POINTER(C.c_float), fp, fp, i64, vp]),
    ("alcm_sincos_embedding", C.c_int, [fp, C.c_float, fp, C.c_int, C.c_int, C.c_int, fp, vp]),
    ("alcm_model_create", C.c_int, [C.c_int, C.POINTER(C.c_int), C.c_int, C.POINTER(NamedTensor), C.c_int, C.c_int,
                                    C.POINTER(vp)]),
    ("alcm_model_destroy", C.c_int, [vp]),
    ("alcm_model_weight_bytes", C.c_size_t, [vp]),
    ("alcm_model_set_split", C.c_int, [vp, C.c_int]),
    ("alcm_model_set_precision", C.c_int, [vp, C.c_int]),
    ("alcm_model_set_resblock_streams", C.c_int, [vp, C.c_int]),
    ("alcm_reload_knobs", C.c_int, []),
    ("alcm_debug_tconv_trace", C.c_int, [C.POINTER(C.c_ulonglong), C.c_int]),
    ("alcm_debug_tconv_wg_times", C.c_int, [C.POINTER(C.c_ulonglong), C.c_int]),
    ("alcm_dit_workspace_bytes", C.c_size_t, [vp, C.c_int, C.c_int]),
    ("alcm_dit_embed_context", C.c_int, [vp, fp, C.c_int, fp, vp, C.c_size_t, vp]),
    ("alcm_dit_forward", C.c_int, [vp, fp, vp, fp, fp, fp, C.c_int, C.c_int, vp, C.c_size_t, vp]),
    ("alcm_vae_workspace_bytes", C.c_size_t, [vp, C.c_int, C.c_int]),
    ("alcm_vae_decode", C.c_int, [vp, fp, C.c_float, fp, C.c_int, C.c_int, vp, C.c_size_t, vp]),
    ("alcm_bigvgan_workspace_bytes", C.c_size_t, [vp, C.c_int, C.c_int]),
    ("alcm_bigvgan_forward", C.c_int, [vp, fp, fp, C.c_int, C.c_int, vp, C.c_size_t, vp]),
    ("alcm_vae_encode_workspace_bytes", C.c_size_t, [vp, C.c_int, C.c_int]),
    ("alcm_vae_encode", C.c_int, [vp, fp, fp, C.c_int, C.c_int, vp, C.c_size_t, vp]),
    ("alcm_vae_encode_len", C.c_int, [vp, C.c_int]),
    ("alcm_mel_workspace_bytes", C.c_size_t, [vp, C.c_int, C.c_int]),
    ("alcm_mel_spectrogram", C.c_int, [vp, fp, fp, C.c_int, C.c_int, vp, C.c_size_t, vp]),
    ("alcm_text_workspace_bytes", C.c_size_t, [vp, C.c_int, C.c_int]),
    ("alcm_text_encode", C.c_int, [vp, vp, vp, fp, C.c_int, C.c_int, vp, C.c_size_t, vp]),
    ("alcm_profile_begin", C.c_int, [C.c_double, C.c_double]),
    ("alcm_profile_end", C.c_int, [C.POINTER(ProfEntry), C.c_int, C.POINTER(C.c_int)]),
]
EXPORTED = [s[0] for s in _SIGS]

_lib: Optional[C.CDLL] = None


def lib() -> C.CDLL:
    """Load the HIP library (raises if it was not built: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libaudiolcm_hip.so not found at {LIB_PATH}; run __graft_entry__.build() "
                              "(make -C audiolcm_amd/csrc). The MI355X path has no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        for name, res, args in _SIGS:
            if name.startswith("alcm_debug_") and "ALCM_LIB" in os.environ and not hasattr(L, name):
                continue  # an older library loaded for an A/B (ALCM_LIB) may predate a diagnostics entry
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class HipError(RuntimeError):
    pass


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().alcm_last_error().decode(errors="replace")
        raise HipError(f"{what or 'alcm call'} failed ({rc}): {msg}")


_checked_devices = set()


def require_device(dev: int = 0) -> None:
    if dev in _checked_devices:
        return
    check(lib().alcm_check_device(dev), "alcm_check_device")
    _checked_devices.add(dev)


def stream_handle(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t) -> Optional[int]:
    """Device address of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return int(t.data_ptr())


def reload_knobs() -> None:
    """Re-read the ALCM_* diagnostic switches (the library reads them once at load)."""
    check(lib().alcm_reload_knobs(), "alcm_reload_knobs")


def debug_tconv_trace(reset: bool = True) -> list:
    """Diagnostics: the tail-conv phase trace (ALCM_TCONV_TRACE=1; the first call allocates the buffer) since the last reset — 7 phase cycle sums and the wave-tile
    count (alcm_debug_tconv_trace)."""
    out = (C.c_ulonglong * 8)()
    check(lib().alcm_debug_tconv_trace(out, 1 if reset else 0), "alcm_debug_tconv_trace")
    return list(out)


def debug_tconv_wg_times(n_wg: int) -> list:
    """Diagnostics: per-workgroup [entry, exit (s_memrealtime, 100 MHz), HW_ID, XCC_ID] of the last traced
    resident-weight tail conv (alcm_debug_tconv_wg_times)."""
    out = (C.c_ulonglong * (4 * n_wg))()
    n = lib().alcm_debug_tconv_wg_times(out, n_wg)
    if n < 0:
        check(n, "alcm_debug_tconv_wg_times")
    return [tuple(out[4 * i: 4 * i + 4]) for i in range(n)]


PEAK_BF16_FLOPS = 2.5e15   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, spec)
PEAK_HBM_BYTES = 8.0e12    # MI355X HBM3E (spec)


def profile_begin(peak_flops: float = PEAK_BF16_FLOPS, peak_bytes: float = PEAK_HBM_BYTES) -> None:
    check(lib().alcm_profile_begin(peak_flops, peak_bytes), "alcm_profile_begin")


def profile_end(max_entries: int = 256):
    """-> list of dicts {name, launches, total_ms, flops, bytes, roof_ms, hbm_launches, hbm_ms, hbm_bytes}
    (synchronises the recorded events; hbm_* aggregate the launches whose algorithmic intensity is HBM-bound)."""
    arr = (ProfEntry * max_entries)()
    n = C.c_int(0)
    check(lib().alcm_profile_end(arr, max_entries, C.byref(n)), "alcm_profile_end")
    return [dict(name=arr[i].name.decode(), launches=int(arr[i].launches), total_ms=float(arr[i].total_ms),
                 flops=float(arr[i].flops), bytes=float(arr[i].bytes), roof_ms=float(arr[i].roof_ms),
                 hbm_launches=int(arr[i].hbm_launches), hbm_ms=float(arr[i].hbm_ms), hbm_bytes=float(arr[i].hbm_bytes))
            for i in range(min(n.value, max_entries))]
