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
    return sorted(set(re.findall(r"^\s*(?:int64_t|int|const char\*)\s+(sir_\w+)\s*\(", text, re.M)))


def test_header_and_binding_agree():
    assert set(declared_symbols()) == set(_native.SIGNATURES), declared_symbols()


def test_library_loads_and_exports_all_symbols():
    lib = _native.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.sir_abi_version() == _native.ABI_VERSION


def _null():
    return ctypes.c_void_p(None)


def _fwd(lib, rowptr, col, items, n_items, H, dtype, Q, ldq, K, ldk, nr, nc, agg, act, S, lds, mask=None):
    return lib.sir_edge_agg_fwd(rowptr, col, items, n_items, _null(), 0, H, dtype, Q, ldq, K, ldk, nr, nc,
                                agg, act, 0.2, S, lds, mask if mask is not None else _null(), _null(), _null())


def test_argument_checks_are_synchronous_and_reported():
    lib = _native.load()
    n = _null()
    # unknown dtype (F32 = 0, BF16 = 1, F16 = 2 are the storage dtypes)
    assert _fwd(lib, n, n, n, 0, 256, 7, n, 256, n, 256, n, n, 0, 2, n, 256) == 1
    assert b"F32" in lib.sir_last_error()
    for dt in (1, 2):       # 16-bit storage: empty work is a no-op like fp32
        assert _fwd(lib, n, n, n, 0, 256, dt, n, 256, n, 256, n, n, 0, 2, n, 256) == 0
    # bad agg
    assert _fwd(lib, n, n, n, 0, 256, 0, n, 256, n, 256, n, n, 9, 2, n, 256) == 1
    assert b"agg" in lib.sir_last_error()
    # H out of range
    rc = lib.sir_edge_agg_bwd_dst(n, n, n, 0, n, 0, 4096, 0, n, 4096, n, 4096, n, n, 4096, n, n, 0, 2, 0.2,
                                  n, 4096, n, 4096, n, n, n)
    assert rc == 1 and b"H must be" in lib.sir_last_error()
    # non-NULL requirements when there is work
    rc = lib.sir_edge_agg_bwd_src(n, n, n, n, 5, n, 0, 64, 0, n, 64, n, 64, n, n, 64, n, n, 0, 2, 0.2,
                                  n, 64, n, n, n)
    assert rc == 1
    buf = ctypes.create_string_buffer(64)
    p = ctypes.cast(buf, ctypes.c_void_p)
    # SYM requires norms
    assert _fwd(lib, p, p, p, 1, 16, 0, p, 16, p, 16, n, n, 2, 2, p, 16) == 1
    assert b"SYM" in lib.sir_last_error()
    # leading dimension smaller than H
    assert _fwd(lib, p, p, p, 1, 16, 0, p, 8, p, 16, n, n, 0, 2, p, 16) == 1
    assert b"leading" in lib.sir_last_error()
    # sign mask is only defined for the ReLU family, H % 4 == 0 and H <= 1024
    assert _fwd(lib, p, p, p, 1, 66, 0, p, 66, p, 66, n, n, 0, 2, p, 66, mask=p) == 2
    assert _fwd(lib, p, p, p, 1, 256, 0, p, 256, p, 256, n, n, 0, 3, p, 256, mask=p) == 2
    assert b"sign mask" in lib.sir_last_error()
    # mask-mode src pass needs the permutation
    rc = lib.sir_edge_agg_bwd_src(p, p, n, p, 1, n, 0, 256, 0, n, 256, n, 256, p, p, 256, n, n, 0, 2, 0.2,
                                  p, 256, n, n, n)
    assert rc == 1 and b"perm" in lib.sir_last_error()


def test_resid_act_argument_checks():
    """sir_resid_act_bwd (ABI 16): the second gradient D2 needs 16-B rows, and in order 1 the dR buffer that
    receives the sum D + D2."""
    lib = _native.load()
    n = _null()
    buf = ctypes.create_string_buffer(256)
    p = ctypes.c_void_p((ctypes.addressof(buf) + 15) & ~15)
    # order 1 with D2 but no dR
    rc = lib.sir_resid_act_bwd(p, 4, p, 4, p, 4, 0, n, 0, p, 4, n, 0, 1, 4, 1, 0.0, 1, n)
    assert rc == 1 and b"D2" in lib.sir_last_error()
    # order 0 with a D2 leading dimension below N
    rc = lib.sir_resid_act_bwd(p, 4, p, 2, p, 4, 0, p, 4, p, 4, p, 4, 1, 4, 1, 0.0, 0, n)
    assert rc == 1 and b"D2" in lib.sir_last_error()
    # empty work with D2 is a no-op
    assert lib.sir_resid_act_bwd(p, 4, p, 4, p, 4, 0, p, 4, p, 4, p, 4, 0, 4, 1, 0.0, 0, n) == 0


def test_gemm16_argument_checks():
    """sir_gemm_pack16 / sir_gemm_nt16 (the autocast projections): bad dtypes, shapes and
    alignments are rejected synchronously with a message; sizing returns 0 for bad shapes."""
    lib = _native.load()
    n = _null()
    assert lib.sir_gemm_pack16_bytes(256, 256) == 256 * 256 * 2
    assert lib.sir_gemm_pack16_bytes(100, 256) == 256 * 256 * 2          # N padded to 256 rows
    assert lib.sir_gemm_pack16_bytes(256, 100) == 0                      # K % 16 != 0
    assert lib.sir_gemm_pack16(n, 256, 256, 256, 0, 0, n, n) == 1 and b"BF16 or F16" in lib.sir_last_error()
    BF, F32 = 1, 0
    # K must be 128 / 256 / 512, N <= 512
    assert lib.sir_gemm_nt16(n, 300, BF, 10, 300, n, 256, BF, n, n, 256, BF, n, 0, n, n) == 1
    assert b"bad shape" in lib.sir_last_error()
    assert lib.sir_gemm_nt16(n, 256, BF, 10, 256, n, 1024, BF, n, n, 1024, BF, n, 0, n, n) == 1
    # a_dtype / c_dtype must be the MFMA type or F32
    assert lib.sir_gemm_nt16(n, 256, 2, 10, 256, n, 256, BF, n, n, 256, BF, n, 0, n, n) == 1
    assert b"a_dtype" in lib.sir_last_error()
    # 16-bit C: N a multiple of 8
    assert lib.sir_gemm_nt16(n, 256, BF, 10, 256, n, 12, BF, n, n, 12, BF, n, 0, n, n) == 1
    assert b"multiples of 16 B" in lib.sir_last_error()
    # the rounded copy of A needs an fp32 A
    assert lib.sir_gemm_nt16(n, 256, BF, 10, 256, n, 256, BF, n, n, 256, BF, ctypes.c_void_p(16), 256, n, n) == 1
    assert b"Acopy" in lib.sir_last_error()
    # NULL buffers with work; an empty M is a no-op
    assert lib.sir_gemm_nt16(n, 256, F32, 10, 256, n, 256, BF, n, n, 256, F32, n, 0, n, n) == 1
    assert b"NULL" in lib.sir_last_error()
    assert lib.sir_gemm_nt16(n, 256, F32, 0, 256, n, 256, BF, n, n, 256, F32, n, 0, n, n) == 0


def test_mask_words_contract():
    lib = _native.load()
    assert lib.sir_mask_words(256, 2) == 4 and lib.sir_mask_words(256, 1) == 4
    assert lib.sir_mask_words(300, 2) == 8 and lib.sir_mask_words(1024, 2) == 16
    assert lib.sir_mask_words(256, 3) == 0 and lib.sir_mask_words(2048, 2) == 0
    assert lib.sir_mask_words(258, 2) == 0 and lib.sir_mask_words(75, 2) == 0
    # sub-wave rows: an H-bit record of >= 8 bytes (32 lanes: 16 B)
    assert lib.sir_mask_words(128, 2) == 2 and lib.sir_mask_words(68, 1) == 2 and lib.sir_mask_words(64, 2) == 1
    assert lib.sir_mask_words(60, 2) == 1 and lib.sir_mask_words(4, 2) == 1 and lib.sir_mask_words(32, 1) == 1


def test_empty_work_is_a_no_op():
    lib = _native.load()
    n = _null()
    assert _fwd(lib, n, n, n, 0, 256, 0, n, 256, n, 256, n, n, 0, 2, n, 256) == 0
    assert lib.sir_degree_norms(n, n, n, n, 0, n) == 0


def test_package_surface():
    for name in ("SIRConv", "Graph", "get_plan", "EdgeAggregate"):
        assert hasattr(sirgcn, name)


def test_abi_argument_checks_under_asan_ubsan(tmp_path):
    """the C ABI's validation built with host AddressSanitizer + UBSan
    (tools/build_abi_asan.sh, tools/abi_sanitize.cpp): every bad call rejected, no sanitizer report."""
    import shutil
    import subprocess
    if shutil.which("/opt/rocm/bin/hipcc") is None:
        import pytest
        pytest.skip("hipcc not available")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "build_abi_asan.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ok: 0 failure(s)" in r.stdout


def test_library_built_from_these_sources():
    """The library embeds a fingerprint of its sources (sir_source_hash); load() refuses a stale
    build whose fingerprint differs from the tree's."""
    lib = _native.load()
    assert lib.sir_source_hash().decode() == _native.source_hash()
