"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/otamd.h declares,
and the ctypes struct layouts match the library's own sizeof.  No compute calls (no GPU here)."""
import re
from pathlib import Path

import pytest
import torch

from onetrainer_amd import _lib

ROOT = Path(__file__).resolve().parents[1]


def header_symbols():
    txt = (ROOT / "include" / "otamd.h").read_text()
    return set(re.findall(r"(?:int|long long)\s+(otamd_\w+)\s*\(", txt))


def test_header_declares_every_binding():
    assert header_symbols() == set(_lib.SIGNATURES), header_symbols() ^ set(_lib.SIGNATURES)


def test_library_exports_every_header_symbol():
    if not _lib.LIB_PATH.exists():
        pytest.fail(f"{_lib.LIB_PATH} not built (python -m onetrainer_amd.build)")
    L = _lib.lib()
    for s in header_symbols():
        assert hasattr(L, s), s


def test_struct_layouts_match_library():
    _lib.check_layouts()


def test_no_fallback_when_library_missing(tmp_path, monkeypatch):
    monkeypatch.setattr(_lib, "LIB_PATH", tmp_path / "missing.so")
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.lib()


def test_native_host_layer_loads():
    """the C++ host layer (_lib/_otamd_host.so) loads over libotamd.so, agrees on the struct layouts and maps
    a violated contract to ValueError, like the ctypes path (no compute: CPU tensors are rejected)."""
    from onetrainer_amd import kernels as K
    h = K._host()
    assert h is not None, "native host layer missing: run onetrainer_amd.build"
    assert h.gemm_args_size() == _lib.lib().otamd_gemm_args_size()
    assert h.attn_args_size() == _lib.lib().otamd_attn_args_size()
    assert h.plan_table_size() == len(K._plan_table())
    x = torch.zeros(4, 8, dtype=torch.bfloat16)
    with pytest.raises(ValueError, match="bf16 cuda"):
        h.linear(x, x, None, None, None, 0, None, False, 1.0, False, None, None, 0)
    with pytest.raises(ValueError, match="NHWC"):
        h.conv2d(x, x, None, 1, 1, False, None, None, None, None, None, 0, 0, 0)
    with K.python_host():
        assert K._host() is None
    assert K.host_layer() == "native"
