"""ctypes binding of librecformer_hip.so (the C ABI declared in include/recformer_hip.h).

The product path has no CPU fallback: if the library is missing or a tensor is not on a
ROCm device, calls raise immediately.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_void_p
from typing import Optional

LIB_PATH = os.environ.get("RF_HIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                        "librecformer_hip.so")  # env: diagnostic builds

RF_F32, RF_BF16, RF_F16 = 0, 1, 2
RF_IO_C_F32, RF_IO_R_F32 = 1, 2
RF_EPI_NONE, RF_EPI_BIAS, RF_EPI_BIAS_GELU, RF_EPI_BIAS_RESID, RF_EPI_COS = 0, 1, 2, 3, 4
RF_EPI_BIAS_GELU_AUX = 6
RF_EPI_DGELU = 7
# rf_abi_version() of the library this binding's SIGNATURES describe; bumped whenever an entry point's
# arguments change (2: rf_prepare_inputs gained gstat, rf_drop_add_ln_*_t mask_row_mul)
ABI_VERSION = 2

# symbol -> (restype, argtypes); must match include/recformer_hip.h exactly
P = c_void_p
SIGNATURES = {
    "rf_last_error": (ctypes.c_char_p, []),
    "rf_abi_version": (c_int, []),
    "rf_debug_set_knob": (c_int, [ctypes.c_char_p, c_int]),
    "rf_debug_get_knob": (c_int, [ctypes.c_char_p]),
    "rf_prepare_inputs": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int,
                                  P, P, P, P, P, P, P, P]),
    "rf_embed_ln_fwd": (c_int, [c_int, c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, c_float,
                                P, P, P]),
    "rf_gemm": (c_int, [c_int, c_int, c_int, c_int, P, c_int, P, c_int, P, P, c_int, P, c_int,
                        c_int, c_int, c_int, c_float, P, P, P]),
    "rf_gemm_resid_ln": (c_int, [c_int, c_int, c_int, c_int, P, c_int, P, c_int, P, P, c_int, P, P,
                                 P, P, P, c_int, P]),
    "rf_layernorm_fwd":(c_int, [c_int, c_int, c_int, c_int, P, c_int, P, P, c_float, P, c_int, P,
                                 P, P, P]),
    "rf_add_layernorm_fwd": (c_int, [c_int, c_int, c_int, c_int, P, c_int, P, P, P, c_float, P, c_int, P,
                                     P, P, P]),
    "rf_embed_ln_split_fwd": (c_int, [c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, c_float, P, P, P]),
    "rf_add_layernorm_split_fwd": (c_int, [c_int, c_int, P, c_int, P, P, P, P, c_float, P, P, P, P]),
    "rf_layernorm_bwd_workspace": (ctypes.c_size_t, [c_int, c_int]),
    "rf_drop_add_ln_fwd": (c_int, [c_int, c_int, P, c_int, P, c_float, ctypes.c_uint64, P, P, c_float, P, P, P, P,
                                   P]),
    "rf_drop_add_ln_bwd": (c_int, [c_int, c_int, P, P, P, P, P, c_float, ctypes.c_uint64, P, P, P, P, P, P]),
    "rf_drop_add_ln_fwd_dual": (c_int, [c_int, c_int, P, c_int, P, c_float, ctypes.c_uint64, P, P, c_float, P, P, P,
                                        P, P, P]),
    "rf_drop_add_ln_bwd_dual": (c_int, [c_int, c_int, P, P, P, P, P, P, c_float, ctypes.c_uint64, P, P, P, P, P,
                                        P]),
    "rf_drop_add_ln_fwd_t": (c_int, [c_int, c_int, c_int, P, c_int, P, c_float, ctypes.c_uint64, P, P, c_float, P, P,
                                     P, P, P, c_int, P]),
    "rf_drop_add_ln_bwd_t": (c_int, [c_int, c_int, c_int, P, P, P, P, P, P, c_float, ctypes.c_uint64, P, P, P, P, P,
                                     c_int, P]),
    "rf_drop_add_ln_bwd_tb": (c_int, [c_int, c_int, c_int, P, P, P, P, P, P, c_float, ctypes.c_uint64, P, P, P, P, P,
                                      P, c_int, P]),
    "rf_colsum_workspace": (ctypes.c_size_t, [c_int, c_int]),
    "rf_embed_ln_bwd_workspace": (ctypes.c_size_t, [c_int, c_int]),
    "rf_embed_ln_bwd": (c_int, [c_int, c_int, P, P, P, P, P, P, P, P, P, c_float, P, P, P, P, P, P]),
    "rf_segment_rows_sum_workspace": (ctypes.c_size_t, [c_int, c_int]),
    "rf_segment_rows_sum": (c_int, [c_int, c_int, P, P, P, c_int, P, c_int, P, P]),
    "rf_pack_weights": (c_int, [c_int, P, c_int, P, c_int, P]),
    "rf_global_fold_bwd_workspace": (ctypes.c_size_t, [c_int, c_int, c_int, c_int]),
    "rf_global_fold_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_int, P, P, c_int, P, P, P, c_float,
                                   ctypes.c_uint64, P, c_int, P, P, P, P, P]),
    "rf_global_fold_bwd_full_workspace": (ctypes.c_size_t, [c_int, c_int, c_int, c_int]),
    "rf_global_fold_bwd_full": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_int, P, P, c_int, P, P, c_int, P,
                                        c_int, P, P, P, c_float, ctypes.c_uint64, P, c_int, P, P, P, P, P, P, P]),
    "rf_global_kv_grad": (c_int, [c_int, c_int, c_int, c_int, c_int, P, P, P, c_int, P, c_int, P, P, c_int, P, c_int,
                                  P]),
    "rf_global_query_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, P, c_float, P, c_int, P, P, P, P, c_int,
                                    P]),
    "rf_adamw_chunk": (c_int, []),
    "rf_set_seed_source": (P, [P]),
    "rf_adamw_step": (c_int, [P, c_int, P, c_int, P]),
    "rf_adamw_step_amp": (c_int, [P, c_int, P, c_int, P, P, P]),
    "rf_weight_grad_workspace": (ctypes.c_size_t, [c_int, c_int, c_int]),
    "rf_weight_grad": (c_int, [c_int, c_int, c_int, c_int, P, c_int, P, c_int, P, c_int, c_int, c_int, c_float, P,
                               ctypes.c_size_t, P]),
    "rf_scatter_add_rows": (c_int, [c_int, c_int, c_int, P, P, P, c_int, P, P, c_int, P]),
    "rf_colsum": (c_int, [c_int, c_int, c_int, P, ctypes.c_int64, P, c_int, c_float, P, P]),
    "rf_layernorm_bwd": (c_int, [c_int, c_int, P, P, c_int, P, P, P, P, P, P, P, P]),
    "rf_band_attn_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, c_int, P, P,
                                 c_int, P, c_int, P]),
    "rf_band_attn_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, P, P, c_int, P, c_int, P, c_int,
                                 P, P, c_int, P, P, P, c_int, P, P, P, P, P]),
    "rf_band_attn_bwd_dt": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, c_int, P, c_int, P, c_int,
                                    P, P, c_int, P, P, P, c_int, P, P, P, P, P]),
    "rf_band_attn_fwd_drop": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, c_int, P, P,
                                      c_int, P, c_int, c_float, ctypes.c_uint64, P]),
    "rf_band_attn_bwd_drop": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, c_int, P, c_int, P,
                                      c_int, P, P, c_int, P, P, P, c_int, P, P, P, P, c_float, ctypes.c_uint64, P]),
    "rf_global_attn_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_int, P, P, c_int, P,
                                   P, c_int, P, c_int, P]),
    "rf_global_fold_workspace": (ctypes.c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "rf_global_attn_fold_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_int, P, c_int, P, P,
                                        P, P, P, P, c_int, P, P, c_int, P]),
    "rf_global_attn_fold_fwd_drop": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_int, P, c_int, P, P,
                                             P, P, P, P, c_int, P, P, c_int, c_float, ctypes.c_uint64, P]),
    "rf_global_attn_fold_fwd_stage": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, c_int, P, c_int, P, P,
                                              P, P, P, P, c_int, P, P, c_int, c_float, ctypes.c_uint64, P]),
    "rf_attn_global_keep": (c_int, [c_int, c_int, c_int, P, c_int, c_float, ctypes.c_uint64, P, P]),
    "rf_global_attn_fold_h_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_int, P, P, c_float, P, P, P,
                                          P, P, P, c_int, P, P, c_int, P]),
    "rf_global_attn_fold_h_stage": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, c_int, P, P, c_float, P,
                                            P, P, P, P, P, c_int, P, P, c_int, P]),
    "rf_gather_global_rows":(c_int, [c_int, c_int, c_int, c_int, c_int, P, c_int, P, P, P]),
    "rf_row_inv_norm": (c_int, [c_int, c_int, c_int, P, c_int, c_float, P, P]),
    "rf_cos_score_cand": (c_int, [c_int, c_int, c_int, c_int, P, c_int, P, P, c_int, P, P,
                                  c_float, P, P]),
    "rf_cos_score_bwd_workspace": (ctypes.c_size_t, [c_int, c_int, c_int]),
    "rf_cos_score_bwd": (c_int, [c_int, c_int, c_int, c_int, P, c_int, P, P, c_int, P, P, c_float, P,
                                 ctypes.c_int64, P, ctypes.c_int64, P, P, ctypes.c_int64, P]),
    "rf_rank_accum": (c_int, [c_int, c_int, P, ctypes.c_int64, P, c_float, c_float, P, P, P, P]),
    "rf_label_scores": (c_int, [c_int, c_int, c_int, P, c_int, P, P, c_int, P, c_int, P, ctypes.c_int64, c_float, P,
                                P]),
    "rf_score_rank": (c_int, [c_int, c_int, c_int, c_int, P, c_int, P, P, c_int, P, c_int, c_int, c_float, P,
                              c_float, c_float, P, P, ctypes.c_int64, P, P, P, c_int, ctypes.c_int32, P, P, c_int, P]),
    "rf_score_rank_tiles": (c_int, [c_int]),
    "rf_rank_reduce": (c_int, [c_int, c_int, P, P, P, P, P, P]),
    "rf_topk_dense": (c_int, [c_int, c_int, P, ctypes.c_int64, P, ctypes.c_int64, ctypes.c_int32, c_int, P, P, P]),
    "rf_topk_merge": (c_int, [c_int, c_int, P, P, P, P, P, c_int, c_int, P, P, P, P]),
    "rf_cross_entropy_fwd": (c_int, [c_int, c_int, c_int, P, ctypes.c_int64, P, ctypes.c_int64, P, P, P]),
    "rf_cross_entropy_bwd": (c_int, [c_int, c_int, c_int, P, ctypes.c_int64, P, ctypes.c_int64, P, P,
                                     ctypes.c_int64, P]),
}

_LIB: Optional[ctypes.CDLL] = None


class RecformerHipError(RuntimeError):
    pass


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and type the library. Raises if it has not been built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.isfile(path):
        raise RecformerHipError(
            f"librecformer_hip.so not found at {path}: build it with "
            f"`python -c 'import __graft_entry__ as g; g.build()'` (make -C recformer_amd/csrc)")
    lib = ctypes.CDLL(path)
    lib.rf_abi_version.restype = c_int
    lib.rf_abi_version.argtypes = []
    ver = lib.rf_abi_version()
    if ver != ABI_VERSION:
        # an older / newer build (e.g. RF_HIP_LIB at a variant library) would read shifted arguments
        # (an int as the stream handle): refuse it instead of launching on garbage
        raise RecformerHipError(f"{path}: ABI version {ver}, this binding needs {ABI_VERSION}: rebuild the library")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def set_knob(name: str, value: int) -> int:
    """Diagnostics (tools/ A/B scripts): set a launch-path tuning knob, return its old value."""
    old = load().rf_debug_set_knob(name.encode(), int(value))
    if old == -2 ** 31:
        raise RecformerHipError(load().rf_last_error().decode(errors="replace"))
    return old


def get_knob(name: str) -> int:
    """A launch-path knob's current value (the dispatch choices the Python side must mirror)."""
    v = load().rf_debug_get_knob(name.encode())
    if v == -2 ** 31:
        raise RecformerHipError(load().rf_last_error().decode(errors="replace"))
    return v


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().rf_last_error().decode(errors="replace")
        raise RecformerHipError(f"{what} failed (rc={rc}): {msg}")
