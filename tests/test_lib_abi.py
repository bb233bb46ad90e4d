"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/otamd.h declares,
and the ctypes struct layouts match the library's own sizeof.  No compute calls (no GPU here)."""
import re
from pathlib import Path

import pytest

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
