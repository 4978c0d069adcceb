"""CPU-only checks of the C-ABI library: it loads, exports every symbol include/sirconv.h
declares, and argument validation rejects bad calls synchronously (no GPU work issued)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

import sirgcn
from sirgcn import _native

HEADER = os.path.join(ROOT, "include", "sirconv.h")


def declared_symbols():
    with open(HEADER) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(sir_\w+)\s*\(", text, re.M)))


def test_header_and_binding_agree():
    assert set(declared_symbols()) == set(_native.SIGNATURES), declared_symbols()


def test_library_loads_and_exports_all_symbols():
    lib = _native.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.sir_abi_version() == _native.ABI_VERSION


def _null():
    return ctypes.c_void_p(None)


def test_argument_checks_are_synchronous_and_reported():
    lib = _native.load()
    # unsupported dtype
    rc = lib.sir_edge_agg_fwd(_null(), _null(), _null(), 0, _null(), 0, 256, 7, _null(), 256, _null(), 256,
                              _null(), _null(), 0, 2, 0.2, _null(), 256, _null(), _null())
    assert rc == 2 and b"F32" in lib.sir_last_error()
    # bad agg
    rc = lib.sir_edge_agg_fwd(_null(), _null(), _null(), 0, _null(), 0, 256, 0, _null(), 256, _null(), 256,
                              _null(), _null(), 9, 2, 0.2, _null(), 256, _null(), _null())
    assert rc == 1 and b"agg" in lib.sir_last_error()
    # H out of range
    rc = lib.sir_edge_agg_bwd_dst(_null(), _null(), _null(), 0, _null(), 0, 4096, 0, _null(), 4096, _null(), 4096,
                                  _null(), 4096, _null(), _null(), 0, 2, 0.2, _null(), 4096, _null(), 4096,
                                  _null(), _null())
    assert rc == 1 and b"H must be" in lib.sir_last_error()
    # non-NULL requirements when there is work
    rc = lib.sir_edge_agg_bwd_src(_null(), _null(), _null(), 5, _null(), 0, 64, 0, _null(), 64, _null(), 64,
                                  _null(), 64, _null(), _null(), 0, 2, 0.2, _null(), 64, _null(), _null())
    assert rc == 1
    # SYM requires norms
    buf = ctypes.create_string_buffer(64)
    p = ctypes.cast(buf, ctypes.c_void_p)
    rc = lib.sir_edge_agg_fwd(p, p, p, 1, _null(), 0, 16, 0, p, 16, p, 16, _null(), _null(), 2, 2, 0.2,
                              p, 16, _null(), _null())
    assert rc == 1 and b"SYM" in lib.sir_last_error()
    # leading dimension smaller than H
    rc = lib.sir_edge_agg_fwd(p, p, p, 1, _null(), 0, 16, 0, p, 8, p, 16, _null(), _null(), 0, 2, 0.2,
                              p, 16, _null(), _null())
    assert rc == 1 and b"leading" in lib.sir_last_error()


def test_empty_work_is_a_no_op():
    lib = _native.load()
    rc = lib.sir_edge_agg_fwd(_null(), _null(), _null(), 0, _null(), 0, 256, 0, _null(), 256, _null(), 256,
                              _null(), _null(), 0, 2, 0.2, _null(), 256, _null(), _null())
    assert rc == 0


def test_package_surface():
    for name in ("SIRConv", "Graph", "get_plan", "EdgeAggregate"):
        assert hasattr(sirgcn, name)
