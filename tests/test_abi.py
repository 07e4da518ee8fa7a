"""C-ABI boundary checks that need no GPU: the library loads and exports every symbol the
header declares (no compute calls)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "fish-speech_amd", "fishmi", "libfishmi.so")


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "fishmi.h")).read()
    return sorted(set(re.findall(r"\b(fm_[a-z_0-9]+)\s*\(", src)))


def test_header_matches_python_binding_list():
    from fishmi import native

    assert sorted(native.ABI_SYMBOLS) == _header_symbols()


@pytest.mark.skipif(not os.path.exists(LIB), reason="libfishmi.so not built (run __graft_entry__.build())")
def test_library_exports_every_header_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(re.findall(r" T (fm_[a-z_0-9]+)", out))
    missing = [s for s in _header_symbols() if s not in exported]
    assert not missing, missing


@pytest.mark.skipif(not os.path.exists(LIB), reason="libfishmi.so not built")
def test_library_loads_without_gpu():
    from fishmi import native

    L = native.lib()
    assert L.fm_device_count() >= 0
    for s in _header_symbols():
        assert hasattr(L, s)
