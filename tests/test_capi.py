"""The C-ABI boundary (no compute): libivfpq.so loads, exports every symbol
include/ivfpq.h declares, and the Python bindings cover exactly that set."""
import ctypes
import os
import re

import pytest

import faiss_amd as faiss
from faiss_amd import _lib

INCLUDE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
HEADER = os.path.join(INCLUDE, "ivfpq.h")
TEST_HEADER = os.path.join(INCLUDE, "ivfpq_test.h")


def declared_functions(path=HEADER):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ivfpq_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_functions()
    hooks = declared_functions(TEST_HEADER)
    assert len(names) >= 30
    for n in names + hooks:
        assert hasattr(lib, n), n
    assert sorted(_lib.SIGNATURES) == sorted(names + hooks)


def test_test_hooks_are_not_in_the_drop_in_header():
    """Fault injection, seeded bounds and workspace dumps are test hooks (ivfpq_test.h),
    not part of the Faiss-replacing boundary."""
    hooks = declared_functions(TEST_HEADER)
    assert sorted(hooks) == ["ivfpq_debug_seed_tau", "ivfpq_debug_workspace", "ivfpq_set_fault_injection"]
    assert not set(hooks) & set(declared_functions())


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_errors_without_device():
    lib = _lib.load()
    if lib.ivfpq_device_count() > 0:
        pytest.skip("a GPU is visible")
    h = ctypes.c_void_p()
    rc = lib.ivfpq_create(128, 1024, 16, 8, 1, 0, ctypes.byref(h))
    assert rc != 0
    assert len(lib.ivfpq_last_error()) > 0
    with pytest.raises(RuntimeError):
        faiss.IndexIVFPQ(None, 128, 1024, 16, 8, device=0)


def test_invalid_arguments_rejected_before_device():
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.ivfpq_create(100, 1024, 16, 8, 1, 0, ctypes.byref(h)) != 0
    assert b"multiple" in lib.ivfpq_last_error()
    assert lib.ivfpq_create(128, 1024, 16, 4, 1, 0, ctypes.byref(h)) != 0
    assert b"nbits" in lib.ivfpq_last_error()
    assert lib.ivfpq_create(120, 1024, 12, 8, 1, 0, ctypes.byref(h)) != 0
    assert lib.ivfpq_set_nprobe(None, 4) != 0
    assert lib.ivfpq_ntotal(None) == -1


def test_factory_and_parameter_parsing():
    assert faiss.index.parse_factory("IVF1024,PQ16") == (1024, 16, 8)
    assert faiss.index.parse_factory("IVF65536,PQ48x8") == (65536, 48, 8)
    assert faiss.index.parse_factory("OPQ16,IVF1024,PQ16") == (1024, 16, 8, 16, -1)
    with pytest.raises(RuntimeError):
        faiss.index.parse_factory("IVF1024,Flat")

    class Fake:
        nprobe = 1

    f = Fake()
    faiss.ParameterSpace().set_index_parameters(f, "nprobe=32")
    assert f.nprobe == 32
    with pytest.raises(RuntimeError):
        faiss.ParameterSpace().set_index_parameter(f, "efSearch", 3)


def test_swig_ptr_passthrough():
    import numpy as np

    a = np.zeros(3, np.float32)
    assert faiss.swig_ptr(a) is a
