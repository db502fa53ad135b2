"""The C-ABI library loads and exports every symbol include/rdfind_hip.h declares (no compute calls
without a GPU), and the product path fails loudly instead of falling back to the CPU."""
import os
import re

import pytest

from rdfind_amd import _lib
from tests.conftest import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "rdfind_hip.h")).read()
    return sorted(set(re.findall(r"^(?:rdf_status|void\s*\*|void|const char\s*\*)\s*(rdf_[a-z_0-9]+)\s*\(", src, re.M)))


def test_library_exports_header_symbols():
    lib = _lib.load()
    names = declared_symbols()
    assert names, "no declarations found"
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) == set(_lib.EXPORTED_SYMBOLS)
    assert lib.rdf_version().startswith(b"rdfind_amd")


def test_no_silent_cpu_fallback():
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(_lib.RdfError):
        _lib.Context(0)


def test_missing_library_raises(monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/librdfind_hip.so")
    with pytest.raises(_lib.RdfError):
        _lib.load()
