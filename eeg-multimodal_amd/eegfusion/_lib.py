"""ctypes binding of the C-ABI library ``libeegfusion.so`` (declared in ``include/eegfusion.h``).

The library is the product: there is no CPU fallback.  ``lib()`` raises if the in-tree build is
missing, and every wrapper raises ``RuntimeError`` on a non-zero status.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_LIB = None
# EEGF_LIB: an alternative build of the same library for A/B timing (tools/); default the in-tree one
LIB_PATH = Path(os.environ.get("EEGF_LIB") or Path(__file__).resolve().parent / "libeegfusion.so").resolve()

F32, BF16 = 0, 1
ERR_ARG = -1

EPI_NONE, EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RELU, EPI_BIAS_TANH, EPI_DGELU, EPI_DRELU, EPI_DTANH = range(8)
EPI_BIAS_GELU_D, EPI_MUL_AUX = 8, 9
FUSE_CONCAT, FUSE_PRICONCAT, FUSE_PRICONCAT_LAP, FUSE_PRIGUMBEL = range(4)

i32, i64, f32, u64, vp = C.c_int, C.c_long, C.c_float, C.c_uint64, C.c_void_p

# name -> argtypes (restype is always c_int status)
SIGNATURES: dict[str, list] = {
    "eegf_gemm": [i32, i32, i32, i32, i32, i32, i32, i32, i32,
                  vp, i64, i64, vp, i64, i64, vp, i64, i64,
                  vp, i64, vp, i64, i64, f32, f32, f32, vp, i64, vp],
    "eegf_seq_lengths": [i32, i32, vp, vp, vp, vp],
    "eegf_varlen_embed": [i32, i32, i32, i32, vp, i64, i64, vp, vp, vp, vp, vp, vp],
    "eegf_varlen_rows": [i32, i32, i32, i32, vp, i64, i64, vp, i64, vp, i64, i32, vp],
    "eegf_attn_varlen_fwd": [i32, i32, i32, i32, vp, i64, i64, vp, i64, vp, f32, f32, u64, u64, vp, i64, vp, vp],
    "eegf_attn_varlen_bwd_workspace": [i64, i32],
    "eegf_attn_varlen_bwd": [i32, i32, i32, i32, vp, i64, i64, vp, i64, vp, f32, f32, u64, u64, vp, vp, i64, vp, vp,
                             vp, vp],
    "eegf_attn_small_fwd": [i32, i32, i32, vp, i64, f32, f32, u64, u64, vp, i64, vp, vp],
    "eegf_attn_small_bwd": [i32, i32, i32, vp, i64, vp, vp, i64, f32, f32, u64, u64, vp, i64, vp],
    "eegf_seq_mean": [i32, i32, i32, i32, vp, i64, vp, i64, vp],
    "eegf_seq_mean_bwd": [i32, i32, i32, i32, vp, i64, vp, i64, f32, vp],
    "eegf_gemm_wgrad_bias": [i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, f32, vp, vp, i64, vp],
    "eegf_tune": [i32, i32],
    "eegf_gemm_big_timestamps": [vp],
    "eegf_ring_proxy": [i64, i32, i32, vp, vp],
    "eegf_launch_log_reset": [],
    "eegf_launch_log_read": [vp, i64],
    "eegf_ln_fwd": [i32, i64, i32, vp, vp, vp, i32, vp, vp, vp, f32, f32, i32, u64, u64, vp, vp, vp, vp, vp],
    "eegf_ln_bwd_partial_rows": [i64],
    "eegf_ln_bwd": [i32, i64, i32, vp, vp, vp, vp, vp, f32, i32, u64, u64, vp, vp, vp, vp, vp],
    "eegf_colsum": [i32, vp, i64, i64, i32, i32, vp, i64, vp, f32, vp],
    "eegf_colsum_batch": [i32, vp, i32, vp],
    "eegf_attn_fwd": [i32, i32, i32, i32, vp, i64, vp, f32, f32, u64, u64, vp, i64, vp, vp, vp],
    "eegf_attn_bwd_workspace": [i32, i32],
    "eegf_attn_bwd": [i32, i32, i32, i32, vp, i64, vp, f32, f32, u64, u64, vp, vp, i64, vp, vp, vp, vp, vp],
    "eegf_xattn_fwd": [i32, i32, i32, i32, vp, vp, vp, f32, u64, u64, vp, vp, vp, vp, vp],
    "eegf_xattn_bwd": [i32, i32, i32, i32, vp, vp, vp, vp, vp, f32, u64, u64, vp, vp, f32, vp, vp],
    "eegf_head_bias_fwd": [i32, i32, i32, vp, vp, vp, vp],
    "eegf_head_bias_bwd": [i32, i32, i32, vp, vp, vp, vp, vp, f32, vp],
    "eegf_dropout": [i32, i64, i32, f32, u64, u64, vp, vp],
    "eegf_fusion_fwd": [i32, i32, i32, vp, i64, vp, i64, vp, i64, vp, vp, vp, vp, i32, i32, f32, f32, u64, u64,
                        vp, vp, vp, vp, vp, vp],
    "eegf_fusion_bwd": [i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, f32, u64, u64,
                        vp, i64, vp, i64, vp, i64, vp, vp],
    "eegf_cross_entropy": [i32, i32, i32, vp, vp, i32, f32, vp, vp, vp, vp],
    "eegf_feawei_init": [i32, vp, i64, f32, i32, vp, vp, vp],
    "eegf_adam": [i64, vp, vp, vp, vp, vp, f32, f32, f32, f32, f32, f32, i32, vp],
    "eegf_adam_consume": [i64, vp, vp, vp, vp, vp, f32, f32, f32, f32, f32, f32, i32, vp],
    "eegf_cast_f32_bf16": [i64, vp, vp, vp],
    "eegf_axpby": [i32, i64, f32, vp, f32, vp, vp],
    "eegf_tanh_bwd": [i32, i64, vp, vp, vp, vp],
    "eegf_key_bias": [i64, vp, vp, vp],
    "eegf_window_tokens": [i32, i32, i32, i32, vp, vp, vp],
    "eegf_embed_gather": [i32, i64, i32, vp, vp, vp, vp],
    "eegf_embed_scatter_add": [i32, i64, i32, vp, vp, vp, vp],
    "eegf_v1_gate_fwd": [i32, vp, i64, vp, vp, vp, f32, i32, f32, u64, u64, vp, vp, vp, vp, vp, vp],
    "eegf_v1_gate_bwd": [i32, vp, vp, i64, vp, vp, vp, vp, vp, vp, f32, i32, u64, u64, vp, vp, vp],
    "eegf_v1_wloss": [i32, vp, f32, f32, vp, vp, vp],
    # DP-SGD (dpsgd.hip)
    "eegf_ghost_norm_workspace": [i32, i32],
    "eegf_ghost_norm": [i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, f32, vp, vp],
    "eegf_seg_sqnorm": [i32, i32, i32, i32, vp, i64, vp, i64, vp, vp, i32, f32, vp, vp],
    "eegf_row_sqnorm": [i32, i32, i32, vp, i64, i32, vp, i64, vp, vp],
    "eegf_dp_clip_rows": [i32, i32, vp, f32, vp, vp, vp],
    "eegf_dp_noise": [i64, vp, f32, f32, u64, u64, vp],
}
RESTYPE_LONG = {"eegf_ln_bwd_partial_rows", "eegf_attn_bwd_workspace", "eegf_ghost_norm_workspace",
                "eegf_attn_varlen_bwd_workspace", "eegf_launch_log_read"}


def register(name: str, argtypes: list) -> None:
    SIGNATURES[name] = argtypes


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"libeegfusion.so not found at {LIB_PATH}; build it with "
                "`python -m eegfusion.build` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
        _LIB = C.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | os.RTLD_GLOBAL)
        for name, argtypes in SIGNATURES.items():
            if os.environ.get("EEGF_LIB") and not hasattr(_LIB, name):
                continue        # an older build under A/B (tools/ab_round.sh) may lack newer entry points
            fn = getattr(_LIB, name)
            fn.argtypes = argtypes
            fn.restype = C.c_long if name in RESTYPE_LONG else C.c_int
    return _LIB


def call(name: str, *args) -> None:
    st = getattr(lib(), name)(*args)
    if st != 0:
        raise RuntimeError(f"{name} failed with status {st}"
                           + (" (argument error)" if st == ERR_ARG else " (hipError)"))


def launch_counts() -> dict[str, int]:
    """kernel name -> launches since load or the last eegf_launch_log_reset (the library's own counters)"""
    n = lib().eegf_launch_log_read(None, 0)
    buf = C.create_string_buffer(int(n))
    lib().eegf_launch_log_read(buf, n)
    out = {}
    for line in buf.value.decode().splitlines():
        cnt, name = line.split("\t", 1)
        out[name] = out.get(name, 0) + int(cnt)
    return out


def has(name: str) -> bool:
    return hasattr(lib(), name)


def exported_symbols() -> list[str]:
    return list(SIGNATURES)
