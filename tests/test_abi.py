"""The C-ABI boundary (include/ksim_engine.h) without a GPU: the library loads,
exports every function the header declares, and the binding's struct layouts
match the C ones (ksim_abi_sizeof needs no device)."""
import ctypes
import os
import re

import pytest

from ksim import abi, engine

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def header_functions():
    src = open(os.path.join(ROOT, "include", "ksim_engine.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ksim_[a-z0-9_]+)\s*\(", src)))


def test_header_parses():
    names = header_functions()
    assert "ksim_create" in names and "ksim_schedule_loaded" in names
    assert len(names) >= 20


def test_library_exports_every_header_symbol():
    L = engine.lib()
    missing = [n for n in header_functions() if not hasattr(L, n)]
    assert not missing, f"declared in ksim_engine.h but not exported: {missing}"


def test_binding_lists_every_export():
    assert sorted(engine.EXPORTS) == header_functions()


def test_abi_version():
    assert engine.lib().ksim_abi_version() == abi.ABI_VERSION


@pytest.mark.parametrize("which", range(len(abi.STRUCT_ORDER)))
def test_struct_sizes_match(which):
    assert engine.lib().ksim_abi_sizeof(which) == abi.struct_size(abi.STRUCT_ORDER[which])


def test_batch_geometry():
    g = engine.batch_geometry()
    assert g["pods_per_batch"] % 64 == 0 and 0 < g["top_t"] <= 64
    assert g["top_threads"] % 64 == 0 and g["lane_cand"] > 0


def test_create_without_gpu_fails_loudly():
    """No CPU fallback: with no device, ksim_create returns an error code."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(engine.KsimError):
        engine.Engine(0)
