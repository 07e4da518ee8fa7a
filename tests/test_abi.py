"""C-ABI boundary checks that need no GPU: the library loads and exports every symbol the
header declares (no compute calls)."""
import ast
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
def test_library_built_from_this_tree():
    """Build provenance: the loaded libfishmi.so carries the hash of the sources it was compiled
    from (Makefile HASHED), and it equals the hash of the sources in this tree -- a stale prebuilt
    library cannot pass (native.lib() refuses it)."""
    import ctypes

    from fishmi import native

    L = ctypes.CDLL(native.LIB_PATH)
    L.fm_source_hash.restype = ctypes.c_char_p
    built = L.fm_source_hash().decode()
    assert len(built) == 16 and built == native.tree_source_hash()


def test_library_loads_without_gpu():
    from fishmi import native

    L = native.lib()
    assert L.fm_device_count() >= 0
    for s in _header_symbols():
        assert hasattr(L, s)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libfishmi.so not built")
def test_library_maps_torch_hip_runtime_first():
    """A fresh process that loads fishmi first must end up on torch's libamdhip64 (one HIP runtime
    per process; the other order leaves torch with "No HIP GPUs are available" on the box)."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from fishmi import native; native.lib()\n"
            "maps = [l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l]\n"
            "print(sorted(set(maps)))\n") % os.path.join(ROOT, "fish-speech_amd")
    out = subprocess.check_output(["python3", "-c", code], text=True, timeout=300)
    paths = ast.literal_eval(out.strip().splitlines()[-1])
    assert len(paths) == 1 and "/torch/lib/" in paths[0], paths


@pytest.mark.skipif(not os.path.exists(LIB), reason="libfishmi.so not built")
def test_host_rope_table_matches_reference(golden):
    """The bf16 cos/sin table the library builds on the host (fm_rope_table, no device) equals the
    reference's precompute_freqs_cis (llama.py:1003-1022) bit for bit, both goldens of ops.npz."""
    import numpy as np

    from fishmi import ops

    g = golden("ops.npz")
    t = ops.rope_table(64, 32, 10000)
    np.testing.assert_array_equal(t, g["rope_table"].reshape(t.shape))
    t2 = ops.rope_table(4096, 128, 1000000)[::97]
    np.testing.assert_array_equal(t2, g["rope_table_big"].reshape(t2.shape))
