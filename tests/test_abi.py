"""CPU-side checks of the drop-in boundary: the C-ABI library builds, loads and exports
exactly what include/bchk.h declares; without a GPU it fails loudly (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import pytest

from bchk_pkg import REPO, load


def header_symbols():
    src = open(os.path.join(REPO, "include", "bchk.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(bchk_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_binding_exports():
    assert header_symbols() == sorted(load().EXPORTS)


def test_library_exports_every_declared_symbol():
    bchk = load()
    path = bchk.build()
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (bchk_[a-z0-9_]+)$", out, flags=re.M))
    missing = set(header_symbols()) - exported
    assert not missing, missing
    lib = ctypes.CDLL(path)
    for s in header_symbols():
        assert hasattr(lib, s)


def test_library_has_gfx950_code_object():
    data = open(load().build(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_create_fails_loudly_without_gpu():
    bchk = load()
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(bchk.BchkError, match="device|HIP"):
        bchk.KanekoKernelProcessor(6, 6)


def test_invalid_code_parameters_rejected():
    bchk = load()
    for m, t in ((1, 1), (9, 2), (4, 8), (6, 0)):
        with pytest.raises(bchk.BchkError):
            bchk.KanekoKernelProcessor(m, t)
