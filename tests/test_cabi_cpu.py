"""The C-ABI library loads without a GPU and exports every entry point include/eegfusion.h declares."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _declared():
    txt = (ROOT / "include" / "eegfusion.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|long)\s+(eegf_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_entry_points():
    names = _declared()
    assert len(names) >= 20, names
    for must in ("eegf_gemm", "eegf_attn_fwd", "eegf_attn_bwd", "eegf_fusion_fwd", "eegf_fusion_bwd", "eegf_adam"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from eegfusion import _lib
    lib = _lib.lib()
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_signatures_cover_header():
    from eegfusion import _lib
    assert set(_declared()) == set(_lib.SIGNATURES), set(_declared()) ^ set(_lib.SIGNATURES)


def test_argument_errors_return_status_without_gpu():
    """Argument validation happens before any launch: returns EEGF_ERR_ARG, never throws."""
    from eegfusion import _lib
    lib = _lib.lib()
    assert lib.eegf_gemm(0, 0, 1, 1, 0, 0, 4, 4, 1, None, 4, 0, None, 4, 0, None, 4, 0, None, 0, None, 0, 0,
                         1.0, 0.0, 1.0, None, 0, None) == _lib.ERR_ARG
    assert lib.eegf_attn_fwd(1, 2, 11, 256, None, 2304, None, 0.125, 0.0, 0, 0, None, 768, None, None, None) == _lib.ERR_ARG
    assert lib.eegf_adam(0, None, None, None, None, None, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1.0, 1, None) == _lib.ERR_ARG


def test_tune_routing_keys_validate_and_restore_without_gpu():
    """eegf_tune is host state only: the GEMM routing keys report the production defaults (key 11 = 1
    persistent GEMMs, key 14 = 1 gemm4r, key 19 = 1 the MFMA cross-attention backward), refuse
    out-of-range values and retired keys (1, 8, 12, 15, 16, 18) with EEGF_ERR_ARG, and return the previous
    value when set."""
    from eegfusion import _lib
    lib = _lib.lib()
    lib.eegf_tune.argtypes = [_lib.i32, _lib.i32]
    for key, default, hi in ((11, 1, 1), (14, 1, 1), (19, 1, 1)):
        old = lib.eegf_tune(key, default)
        assert old == default, (key, old)
        assert lib.eegf_tune(key, hi + 1) == _lib.ERR_ARG
        assert lib.eegf_tune(key, -1) == _lib.ERR_ARG
        assert lib.eegf_tune(key, 0) == default
        assert lib.eegf_tune(key, old) == 0
    for key in (1, 8, 9, 12, 15, 16, 18):
        assert lib.eegf_tune(key, 0) == _lib.ERR_ARG, key


def test_launch_log_reads_empty_without_gpu():
    """The launch counters (eegf_launch_log_*) are host state: after a reset, with nothing launched, the
    log is the empty string (1 byte with the NUL) and _lib.launch_counts() an empty dict."""
    from eegfusion import _lib
    lib = _lib.lib()
    assert lib.eegf_launch_log_reset() == 0
    assert lib.eegf_launch_log_read(None, 0) == 1
    assert _lib.launch_counts() == {}
