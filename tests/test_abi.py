"""CPU: the C-ABI library loads, exports every symbol include/nwcrypto.h declares, and refuses to
run without a GPU (no silent CPU fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nwcrypto.h")
LIB = os.path.join(ROOT, "narwhal_amd", "libnwcrypto.so")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nw_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ["nw_ctx_create", "nw_committee_load", "nw_verify_strict", "nw_verify_batch", "nw_verify_certs",
                 "nw_verify_certs_dev", "nw_sha512", "nw_sha512_many"]:
        assert must in names


@pytest.mark.skipif(not os.path.exists(LIB), reason="libnwcrypto.so not built")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


@pytest.mark.skipif(not os.path.exists(LIB), reason="libnwcrypto.so not built")
def test_no_gpu_fails_loudly():
    from narwhal_amd import _lib
    if _has_gpu():
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.DeviceError):
        _lib.Engine()


def _has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def test_product_never_imports_oracle():
    """The product package must not reference the oracle (tests/bench-only checker)."""
    pkg = os.path.join(ROOT, "narwhal_amd")
    py_import = re.compile(r"^\s*(import|from)\s+[\w.]*(oracle)", re.M)
    c_include = re.compile(r"#\s*include\s*[<\"][^>\"]*oracle|liboracle|oracle/_ref")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            txt = open(os.path.join(dirpath, f), errors="ignore").read() if f.endswith(
                (".py", ".cpp", ".hip", ".h", "Makefile")) else ""
            assert not py_import.search(txt), f
            assert not c_include.search(txt), f
            assert "sys.path" not in txt or "oracle" not in txt, f
