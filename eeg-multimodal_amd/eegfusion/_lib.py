"""ctypes binding of the C-ABI library ``libeegfusion.so`` (declared in ``include/eegfusion.h``).

The library is the product: there is no CPU fallback.  ``lib()`` raises if the in-tree build is
missing, and every wrapper raises ``RuntimeError`` on a non-zero status.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_LIB = None
LIB_PATH = Path(__file__).resolve().parent / "libeegfusion.so"

F32, BF16 = 0, 1
ERR_ARG = -1

EPI_NONE, EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RELU, EPI_BIAS_TANH, EPI_DGELU, EPI_DRELU, EPI_DTANH = range(8)

i32, i64, f32, u64, vp = C.c_int, C.c_long, C.c_float, C.c_uint64, C.c_void_p

# name -> argtypes (restype is always c_int status)
SIGNATURES: dict[str, list] = {
    "eegf_gemm": [i32, i32, i32, i32, i32, i32, i32, i32, i32,
                  vp, i64, i64, vp, i64, i64, vp, i64, i64,
                  vp, vp, i64, i64, f32, f32, f32, vp],
}


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
            fn = getattr(_LIB, name)
            fn.argtypes = argtypes
            fn.restype = C.c_int
    return _LIB


def call(name: str, *args) -> None:
    st = getattr(lib(), name)(*args)
    if st != 0:
        raise RuntimeError(f"{name} failed with status {st}"
                           + (" (argument error)" if st == ERR_ARG else " (hipError)"))


def exported_symbols() -> list[str]:
    return list(SIGNATURES)
