"""CPU: the C-ABI library builds for gfx950, loads, and exports exactly what include/zsaac.h
declares (no compute calls — there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "zsaac.h")


def _header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\bint\s+(zs_\w+)\s*\(", src))


@pytest.fixture(scope="module")
def libpath():
    from zsaac import _lib
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.LIB_PATH


def test_header_matches_binding_table():
    from zsaac._lib import SIGNATURES
    assert _header_symbols() == set(SIGNATURES)


def test_library_exports_every_header_symbol(libpath):
    out = subprocess.run(["nm", "-D", "--defined-only", libpath], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT\s+(zs_\w+)", out))
    missing = _header_symbols() - exported
    assert not missing, missing
    assert exported <= _header_symbols(), exported - _header_symbols()


def test_code_object_targets_gfx950(libpath):
    # the .hip_fatbin section bundles one code object per offload target
    data = open(libpath, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"gfx942" not in data and b"gfx90a" not in data


def test_load_and_error_path(libpath):
    from zsaac import _lib
    lib = _lib.lib()
    assert lib.zs_version() == 1
    # argument validation runs on the host before any launch: a bad shape fails cleanly
    rc = lib.zs_gemm(4, 8, 30, 0, None, 32, None, 32, None, None, 0, None, 8, 0, 0, 1, None, None)
    assert rc == -1
    assert "multiple of 32" in _lib.last_error()
    with pytest.raises(_lib.ZsError):
        _lib.call("zs_tune_set", b"no_such_knob", 1)
    assert lib.zs_gemm_workspace_floats(64, 768, 3072) > 0
    # 4 row blocks of 64: a 256-row launch needs 4x the slabs of a 64-row one (same counters)
    w64, w256 = lib.zs_gemm_workspace_floats(64, 768, 3072), lib.zs_gemm_workspace_floats(256, 768, 3072)
    assert w256 - 4096 == 4 * (w64 - 4096)
    assert lib.zs_gemm_workspace_floats(257, 768, 3072) == 0
    assert lib.zs_lmhead_nblk(50257) == 393


def test_ops_refuse_cpu_tensors():
    import torch
    from zsaac import ops
    from zsaac._lib import ZsError
    a = torch.zeros(4, 32)
    with pytest.raises(ZsError):
        ops.gemm(a, torch.zeros(8, 32), torch.zeros(4, 8), split_k=1)
