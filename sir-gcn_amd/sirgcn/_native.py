"""ctypes binding of ``libsirconv.so`` (the C ABI in ``include/sirconv.h``).

The product path has NO fallback: if the library is missing or a call fails, a
``RuntimeError`` is raised.  Build it with ``make -C sir-gcn_amd/csrc`` or
``python -c "import __graft_entry__ as g; g.build()"``.
"""
import ctypes
import os
import threading

import torch

# SIRGCN_LIB: an A/B build of the same sources (tools/build_variant.sh), for measurement runs only
LIB_PATH = os.environ.get("SIRGCN_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                        "lib", "libsirconv.so")

AGG = {"sum": 0, "mean": 1, "sym": 2}
ACT_IDENTITY, ACT_RELU, ACT_LEAKY, ACT_GELU, ACT_GELU_TANH = range(5)
DTYPE_F32, DTYPE_BF16, DTYPE_F16 = 0, 1, 2
ABI_VERSION = 16
STORAGE = {torch.float32: DTYPE_F32, torch.bfloat16: DTYPE_BF16, torch.float16: DTYPE_F16}

# exported symbol -> (restype, argtypes); mirrors include/sirconv.h
_P, _I64, _I, _F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
SIGNATURES = {
    "sir_abi_version": (ctypes.c_int, []),
    "sir_source_hash": (ctypes.c_char_p, []),
    "sir_last_error": (ctypes.c_char_p, []),
    "sir_mask_words": (ctypes.c_int64, [_I64, _I]),
    "sir_degree_norms": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P]),
    "sir_col_sum": (ctypes.c_int, [_P, _I64, _I64, _I64, _P, _P, _P]),
    "sir_graph_norm_fwd": (ctypes.c_int, [_P, _I64, _I64, _P, _I64, _P, _P, _P, _F, _P, _I64, _P, _P, _P]),
    "sir_graph_norm_bwd": (ctypes.c_int, [_P, _I64, _I64, _P, _I64, _P, _I64, _P, _P, _P, _P, _P, _I64,
                                          _P, _P, _P, _P]),
    "sir_resid_act_fwd": (ctypes.c_int, [_P, _I64, _I, _P, _I64, _P, _I64, _I64, _I64, _I, _F, _I, _P]),
    "sir_resid_act_bwd": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _I64, _I, _P, _I64, _P, _I64, _P, _I64, _I64, _I64, _I,
                                         _F, _I, _P]),
    "sir_graph_norm_act_fwd": (ctypes.c_int, [_P, _I64, _I64, _P, _I64, _P, _P, _P, _F, _I, _F, _P, _I64, _P, _I64,
                                              _P, _P, _P]),
    "sir_graph_norm_act_bwd": (ctypes.c_int, [_P, _I64, _I64, _P, _I64, _P, _I64, _P, _P, _P, _P, _P, _I, _F, _P,
                                              _I64, _P, _P, _P, _P]),
    "sir_edge_gather_add": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _P, _I64, _P, _I64, _P, _I64, _P]),
    "sir_edge_gather_act": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _P, _I64, _P, _I64, _I, _F, _P, _I64, _P, _P]),
    "sir_segment_sum": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _I64, _I64, _P, _I64, _P, _P, _I, _P, _I64,
                                       _P, _P]),
    "sir_edge_broadcast": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _P, _I64, _P, _P, _I, _P, _I64, _P]),
    "sir_segment_max": (ctypes.c_int, [_P, _I64, _P, _I64, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _P, _P]),
    "sir_segment_max_bwd": (ctypes.c_int, [_P, _I64, _I64, _P, _I64, _P, _I64, _P, _I64, _P]),
    "sir_csr_build_workspace": (ctypes.c_int64, [_I64, _I64]),
    "sir_csr_build": (ctypes.c_int, [_P, _P, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "sir_csr_perm": (ctypes.c_int, [_P, _P, _I64, _P, _P, _P]),
    "sir_gemm_pack_bytes": (ctypes.c_int64, [_I64, _I64]),
    "sir_gemm_pack": (ctypes.c_int, [_P, _I64, _I64, _I64, _I, _P, _P]),
    "sir_gemm_nt": (ctypes.c_int, [_P, _I64, _I64, _I64, _P, _I64, _P, _P, _I64, _P, _P]),
    "sir_gemm_nt_dact": (ctypes.c_int, [_P, _I64, _I64, _I64, _P, _I64, _P, _P, _I, _F, _P, _I64, _P]),
    "sir_gemm_nt_direct": (ctypes.c_int, [_P, _I64, _I64, _I64, _P, _I64, ctypes.c_int, _I64, _P, _P, _I64, _P, _P]),
    "sir_gemm_nt_direct2": (ctypes.c_int, [_P, _I64, _I64, _I64, _P, _I64, _P, _I64, _I64, ctypes.c_int, _I64, _P,
                                           _I64, _P, _I64, _P, _P]),
    "sir_gemm_tn_workspace": (ctypes.c_int64, [_I64, _I64, _I64]),
    "sir_gemm_tn": (ctypes.c_int, [_P, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _P, _P, _I64, _P]),
    "sir_gemm_tn16": (ctypes.c_int, [_P, _I64, _P, _I64, _I64, _I64, _I64, _I, _P, _I64, _P, _P, _I64, _P]),
    "sir_gemm_pack16_bytes": (ctypes.c_int64, [_I64, _I64]),
    "sir_gemm_pack16": (ctypes.c_int, [_P, _I64, _I64, _I64, _I, _I, _P, _P]),
    "sir_gemm_nt16": (ctypes.c_int, [_P, _I64, _I, _I64, _I64, _P, _I64, _I, _P, _P, _I64, _I, _P, _I64, _P, _P]),
    "sir_dropout_apply": (ctypes.c_int, [_P, _I64, _I64, _I64, _I, _I64, _P, _P]),
    "sir_edge_agg_fwd": (ctypes.c_int, [_P, _P, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _P, _I64,
                                        _P, _P, _I, _I, _F, _P, _I64, _P, _P, _P]),
    "sir_edge_agg_bwd_dst": (ctypes.c_int, [_P, _P, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _P, _I64, _P,
                                            _P, _I64, _P, _P, _I, _I, _F, _P, _I64, _P, _I64, _P, _P, _P]),
    "sir_edge_agg_bwd_src": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _I64, _I64, _I, _P, _I64, _P, _I64, _P,
                                            _P, _I64, _P, _P, _I, _I, _F, _P, _I64, _P, _P, _P]),
    "sir_edge_mlp_pack_bytes": (ctypes.c_int64, [_I64, _I64]),
    "sir_edge_mlp_pack": (ctypes.c_int, [_P, _I64, _I64, _P, _P]),
    "sir_edge_mlp_fwd": (ctypes.c_int, [_P, _P, _P, _I64, _P, _I64, _I64, _I64, _P, _I64, _P, _I64, _P, _P, _I, _I,
                                        _F, _I, _P, _P, _P, _I64, _P, _I64, _P, _P, _P]),
    "sir_edge_mlp_bwd_parts": (ctypes.c_int64, [_I64, _I64, _I64]),
    "sir_edge_mlp_stream_work_bytes": (ctypes.c_int64, [_I64]),
    "sir_edge_mlp_fwd_stream": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, _P, _I64, _P, _I64, _P, _P, _I, _I,
                                               _F, _I, _P, _P, _P, _I64, _P, _I64, _P, _P]),
    "sir_edge_mlp_pack_st": (ctypes.c_int, [_P, _I64, _I64, _I, _P, _P]),
    "sir_edge_mlp_fwd_st": (ctypes.c_int, [_P, _P, _P, _I64, _P, _I64, _I64, _I64, _P, _I64, _P, _I64, _I, _I, _I, _F,
                                           _I, _P, _P, _P, _I64, _P, _I64, _P, _P, _P]),
    "sir_edge_mlp_fwd_stream_st": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, _P, _I64, _P, _I64, _I, _I, _I,
                                                  _F, _I, _P, _P, _P, _I64, _P, _I64, _P, _P]),
    "sir_edge_max_bwd_dst": (ctypes.c_int, [_P, _P, _P, _I64, _P, _I64, _I64, _I64, _P, _I64, _P, _I64, _P, _I64,
                                            _P, _I64, _I, _F, _P, _P, _I64, _P, _P, _P]),
    "sir_edge_max_bwd_src": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _I64, _I64, _I64, _P, _I64, _P, _I64, _P,
                                            _I64, _P, _I64, _I, _F, _P, _P, _I64, _P, _P]),
    "sir_edge_max_bwd_sparse_parts": (ctypes.c_int, [_I64, _I64, _P, _P]),
    "sir_edge_max_bwd_sparse": (ctypes.c_int, [_P, _P, _P, _I64, _P, _I64, _P, _P, _I64, _P, _I64, _P, _I64, _I64,
                                               _I64, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _I, _F, _P,
                                               _P, _I64, _P, _I64, _P, _P, _P, _P, _P, _P, _P]),
    "sir_max_dw_rows_parts": (ctypes.c_int64, [_I64, _I64]),
    "sir_max_dw_rows": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _I64, _P, _I64, _I64, _I64, _P, _I64, _P]),
    "sir_max_dw_qk": (ctypes.c_int, [_P, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _I64, _I64, _I, _F, _P,
                                     _I64, _P]),
    "sir_edge_mlp_bwd_dst": (ctypes.c_int, [_P, _P, _P, _I64, _P, _I64, _I64, _I64, _P, _I64, _P, _I64, _P, _I64,
                                            _P, _P, _I, _I, _F, _I, _P, _P, _P, _P, _I64, _P, _P, _P, _P]),
    "sir_edge_mlp_bwd_src": (ctypes.c_int, [_P, _P, _P, _I64, _P, _I64, _I64, _I64, _P, _I64, _P, _I64, _P, _I64,
                                            _P, _P, _I, _I, _F, _I, _P, _P, _P, _P, _I64, _P, _P]),
    "sir_edge_agg_bwd": (ctypes.c_int, [_P, _P, _P, _I64, _P, _I64, _P, _P, _P, _P, _I64, _P, _I64, _I64, _I, _P,
                                        _P, _I64, _P, _P, _I, _I, _F, _P, _I64, _P, _I64, _P, _P, _P, _P]),
}

class Dropout(ctypes.Structure):
    """``sir_dropout_t`` (include/sirconv.h): the hashed feature-dropout mask of QK (seed, p), the
    seed given by value or as a device pointer (``seed_ptr``, read by the kernels)."""
    _fields_ = [("seed", ctypes.c_uint64), ("p", ctypes.c_double), ("seed_ptr", ctypes.c_void_p)]


def _drop(drop):
    """ctypes pointer argument for an optional (seed, p) pair; ``seed`` is an int or a one-element
    int64 device tensor (the graph-safe form: its value is read on the device by every kernel)."""
    if drop is None:
        return None
    seed, p = drop
    if isinstance(seed, torch.Tensor):
        if not (seed.is_cuda and seed.dtype == torch.int64 and seed.numel() >= 1):
            raise ValueError("dropout seed tensor must be a CUDA int64 tensor")
        return ctypes.byref(Dropout(0, float(p), seed.data_ptr()))
    return ctypes.byref(Dropout(int(seed) & (2 ** 64 - 1), float(p), None))


_lib = None
_lock = threading.Lock()

# Optional live per-call timing (bench.py): HIP events recorded on the launching stream.
_timing = None


def enable_timing(on=True):
    """Start (or stop) recording HIP events around every native call; returns the record dict
    {entry-point name: [(start_event, end_event), ...]}."""
    global _timing
    _timing = {} if on else None
    return _timing


class _Timed:
    """Records (start, end, work) on the launching stream; ``work`` = (flops, algorithmic HBM bytes)
    for the GEMMs (A, B read once, C written once; the packed weights are L2-resident)."""
    __slots__ = ("name", "dev", "ev", "work")

    def __init__(self, name, dev, work=0):
        self.name, self.dev, self.ev, self.work = name, dev, None, work

    def __enter__(self):
        if _timing is not None:
            s = torch.cuda.current_stream(self.dev)
            self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self.ev[0].record(s)

    def __exit__(self, *exc):
        if self.ev is not None:
            self.ev[1].record(torch.cuda.current_stream(self.dev))
            _timing.setdefault(self.name, []).append((self.ev[0], self.ev[1], self.work))


CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
INCLUDE = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "include")


def source_hash():
    """The fingerprint the Makefile embeds (sha256 of csrc/*.hip, *.h, *.cpp and include/*.h in path
    order, first 16 hex digits), or None when the sources are not in the tree."""
    import glob
    import hashlib
    files = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h"))
                   + glob.glob(os.path.join(CSRC, "*.cpp")) + glob.glob(os.path.join(INCLUDE, "*.h")))
    if not files:
        return None
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


EDGE_SOURCES = ("sirconv_edge_impl.h", "sirconv_dropout.h", "sirconv_internal.h", "sirconv_dispatch.hip",
                "sirconv_fwd_f32.hip", "sirconv_fwd_bf16.hip", "sirconv_fwd_f16.hip",
                "sirconv_bwd_dual_f32.hip", "sirconv_bwd_dual_bf16.hip", "sirconv_bwd_dual_f16.hip")


def edge_source_hash():
    """Fingerprint of the sources the edge-aggregation kernels are compiled from (the kernels the
    PMC traffic files of profiles/ describe): a counter file stays valid while this is unchanged."""
    import hashlib
    h = hashlib.sha256()
    for name in EDGE_SOURCES:
        p = os.path.join(CSRC, name)
        if not os.path.exists(p):
            return None
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_id():
    """{library source hash, edge-kernel source hash} of this tree."""
    return {"source_hash": source_hash(), "edge_source_hash": edge_source_hash()}


def load():
    """Load (once) and return the ctypes handle; raise loudly if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"sirgcn: native library not found at {LIB_PATH}; "
                                   "build it with `make -C sir-gcn_amd/csrc` (no CPU fallback exists)")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            if lib.sir_abi_version() != ABI_VERSION:
                raise RuntimeError(f"sirgcn: ABI mismatch (library {lib.sir_abi_version()}, host {ABI_VERSION})")
            want = source_hash()
            got = lib.sir_source_hash().decode()
            if want is not None and got != want:
                raise RuntimeError(f"sirgcn: {LIB_PATH} was built from other sources (library {got}, tree {want}); "
                                   "rebuild it with `make -C sir-gcn_amd/csrc`")
            _lib = lib
    return _lib


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _check(rc, lib):
    if rc != 0:
        raise RuntimeError(f"sirgcn native error {rc}: {lib.sir_last_error().decode()}")


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ld(t, H):
    assert t.dim() == 2 and t.stride(1) == 1 and t.shape[1] >= H, "rows must be unit-stride"
    return t.stride(0)


def mask_words(H, act):
    """64-bit words of sign mask per edge, or 0 if the sign-mask backward is unavailable."""
    return int(load().sir_mask_words(H, act))


def degree_norms(rowptr_dst, rowptr_src, in_norm, out_norm):
    lib = load()
    n = in_norm.numel()
    rc = lib.sir_degree_norms(_ptr(rowptr_dst), _ptr(in_norm), _ptr(rowptr_src), _ptr(out_norm), n,
                              _stream(in_norm.device))
    _check(rc, lib)


COLSUM_BLOCKS = 1024


def col_sum(X):
    """Deterministic column sums of a tall fp32 [n, m] view (bias gradients)."""
    lib = load()
    n, m = X.shape
    out = torch.empty(m, device=X.device, dtype=torch.float32)
    ws = torch.empty(COLSUM_BLOCKS * m, device=X.device, dtype=torch.float32)
    rc = lib.sir_col_sum(_ptr(X), X.stride(0), n, m, _ptr(out), _ptr(ws), _stream(X.device))
    _check(rc, lib)
    return out


def _ldx(t, H):
    return H if t is None else _ld(t, H)


def _storage(*ts):
    """SIR_DTYPE_* of the feature matrices of one edge-pass call (all must share one dtype)."""
    dts = {t.dtype for t in ts if t is not None}
    if len(dts) != 1 or next(iter(dts)) not in STORAGE:
        raise RuntimeError(f"edge pass: feature tensors must share one of fp32/bf16/fp16, got {dts}")
    return STORAGE[dts.pop()]


AGG_ACCUMULATE = 16       # SIR_AGG_ACCUMULATE


def edge_agg_fwd(csr, Q, K, norm_row, norm_col, agg, act, slope, S, partial, mask_out=None, accumulate=False):
    """``accumulate``: S[v] += the sum over ``csr.items``' edges (rows without items untouched; SUM / SYM)."""
    lib = load()
    H = S.shape[1]
    with _Timed("sir_edge_agg_fwd", S.device):
        rc = lib.sir_edge_agg_fwd(
            _ptr(csr.rowptr), _ptr(csr.col), _ptr(csr.items), csr.n_items, _ptr(csr.splits), csr.n_splits,
            H, _storage(Q, K, S), _ptr(Q), _ld(Q, H), _ptr(K), _ld(K, H), _ptr(norm_row), _ptr(norm_col),
            AGG[agg] | (AGG_ACCUMULATE if accumulate else 0), act, float(slope), _ptr(S), _ld(S, H),
            _ptr(mask_out), _ptr(partial), _stream(S.device))
    _check(rc, lib)


def edge_agg_bwd_dst(csr, Q, K, G, norm_row, norm_col, agg, act, slope, dQ, Gm, partial, mask=None, drop=None):
    lib = load()
    H = dQ.shape[1]
    with _Timed("sir_edge_agg_bwd_dst", dQ.device):
        rc = lib.sir_edge_agg_bwd_dst(
            _ptr(csr.rowptr), _ptr(csr.col), _ptr(csr.items), csr.n_items, _ptr(csr.splits), csr.n_splits,
            H, _storage(Q, K, G, dQ, Gm), _ptr(Q), _ldx(Q, H), _ptr(K), _ldx(K, H), _ptr(mask), _ptr(G), _ld(G, H),
            _ptr(norm_row), _ptr(norm_col), AGG[agg], act, float(slope),
            _ptr(dQ), _ld(dQ, H), _ptr(Gm), _ldx(Gm, H), _ptr(partial), _drop(drop), _stream(dQ.device))
    _check(rc, lib)


def edge_agg_bwd_src(csr_s, K, Q, Gd, norm_row, norm_col, agg, act, slope, dK, partial, mask=None, drop=None):
    lib = load()
    H = dK.shape[1]
    with _Timed("sir_edge_agg_bwd_src", dK.device):
        rc = lib.sir_edge_agg_bwd_src(
            _ptr(csr_s.rowptr), _ptr(csr_s.col), _ptr(csr_s.perm if mask is not None else None),
            _ptr(csr_s.items), csr_s.n_items, _ptr(csr_s.splits), csr_s.n_splits, H, _storage(K, Q, Gd, dK),
            _ptr(K), _ldx(K, H), _ptr(Q), _ldx(Q, H), _ptr(mask), _ptr(Gd), _ld(Gd, H),
            _ptr(norm_row), _ptr(norm_col), AGG[agg], act, float(slope),
            _ptr(dK), _ld(dK, H), _ptr(partial), _drop(drop), _stream(dK.device))
    _check(rc, lib)


def edge_agg_bwd(csr, csr_s, G, mask, in_norm, out_norm, agg, act, slope, dQ, dK, partial, partial_s, drop=None):
    """Both sign-mask backward passes in one launch (SUM / SYM); bit-identical to
    edge_agg_bwd_dst + edge_agg_bwd_src."""
    lib = load()
    H = dQ.shape[1]
    with _Timed("sir_edge_agg_bwd", dQ.device):
        rc = lib.sir_edge_agg_bwd(
            _ptr(csr.rowptr), _ptr(csr.col), _ptr(csr.items), csr.n_items, _ptr(csr.splits), csr.n_splits,
            _ptr(csr_s.rowptr), _ptr(csr_s.col), _ptr(csr_s.perm), _ptr(csr_s.items), csr_s.n_items,
            _ptr(csr_s.splits), csr_s.n_splits, H, _storage(G, dQ, dK), _ptr(mask), _ptr(G), _ld(G, H),
            _ptr(in_norm), _ptr(out_norm), AGG[agg], act, float(slope), _ptr(dQ), _ld(dQ, H), _ptr(dK), _ld(dK, H),
            _ptr(partial), _ptr(partial_s), _drop(drop), _stream(dQ.device))
    _check(rc, lib)


# ------------------------------------------------------------------------------ generic path
def edge_gather_add(csr, Q, K, Z):
    lib = load()
    F = Z.shape[1]
    with _Timed("sir_edge_gather_add", Z.device):
        rc = lib.sir_edge_gather_add(_ptr(csr.rowptr), _ptr(csr.col), _ptr(csr.items), csr.n_items, F,
                                     _ptr(Q), _ld(Q, F), _ptr(K), _ld(K, F), _ptr(Z), _ld(Z, F), _stream(Z.device))
    _check(rc, lib)


def edge_gather_act(csr, Q, K, act, slope, A, sign_mask=None):
    """A[e] = act(Q[row(e)] + K[col[e]]) for act in {identity, ReLU, LeakyReLU} (dst-CSR edge order);
    ``sign_mask`` (int64 [E, 4], F = 256): bit l of word x = A[e][4 l + x] > 0."""
    lib = load()
    F = A.shape[1]
    with _Timed("sir_edge_gather_act", A.device):
        rc = lib.sir_edge_gather_act(_ptr(csr.rowptr), _ptr(csr.col), _ptr(csr.items), csr.n_items, F,
                                     _ptr(Q), _ld(Q, F), _ptr(K), _ld(K, F), int(act), float(slope), _ptr(A),
                                     _ld(A, F), _ptr(sign_mask), _stream(A.device))
    _check(rc, lib)


def segment_sum(csr, X, out, norm_row=None, norm_col=None, mean=False, perm=None, partial=None):
    lib = load()
    F = out.shape[1]
    with _Timed("sir_segment_sum", out.device):
        rc = lib.sir_segment_sum(_ptr(csr.rowptr), _ptr(csr.col), _ptr(perm), _ptr(csr.items), csr.n_items,
                                 _ptr(csr.splits), csr.n_splits, F, _ptr(X), _ld(X, F), _ptr(norm_row),
                                 _ptr(norm_col), int(bool(mean)), _ptr(out), _ld(out, F), _ptr(partial),
                                 _stream(out.device))
    _check(rc, lib)


def edge_broadcast(csr, dS, dM, norm_row=None, norm_col=None, mean=False):
    lib = load()
    F = dM.shape[1]
    with _Timed("sir_edge_broadcast", dM.device):
        rc = lib.sir_edge_broadcast(_ptr(csr.rowptr), _ptr(csr.col), _ptr(csr.items), csr.n_items, F,
                                    _ptr(dS), _ld(dS, F), _ptr(norm_row), _ptr(norm_col), int(bool(mean)),
                                    _ptr(dM), _ld(dM, F), _stream(dM.device))
    _check(rc, lib)


def segment_max(csr, M, Y, arg, pval=None, parg=None):
    lib = load()
    F = Y.shape[1]
    with _Timed("sir_segment_max", Y.device):
        rc = lib.sir_segment_max(_ptr(csr.items), csr.n_items, _ptr(csr.splits), csr.n_splits, F,
                                 _ptr(M), _ld(M, F), _ptr(Y), _ld(Y, F), _ptr(arg), _ld(arg, F),
                                 _ptr(pval), _ptr(parg), _stream(Y.device))
    _check(rc, lib)


def segment_max_bwd(csr, arg, dY, dM):
    lib = load()
    F = dM.shape[1]
    with _Timed("sir_segment_max_bwd", dM.device):
        rc = lib.sir_segment_max_bwd(_ptr(csr.items), csr.n_items, F, _ptr(arg), _ld(arg, F),
                                     _ptr(dY), _ld(dY, F), _ptr(dM), _ld(dM, F), _stream(dM.device))
    _check(rc, lib)


# ------------------------------------------------------------------------------ plan build
def csr_build(rows, cols, n_rows, n_cols, chunk):
    """Device COO -> row CSR + work plan (async).  Returns (rowptr, col, eid, items_cap, splits_cap,
    counts); ``counts`` = int64 [5] {n_items, n_splits, n_slots, max_degree, n_bad_ids} on the device."""
    lib = load()
    dev = rows.device
    E = rows.numel()
    rows = rows.to(torch.int64).contiguous()
    cols = cols.to(torch.int64).contiguous()
    ws_bytes = lib.sir_csr_build_workspace(n_rows, E)
    if ws_bytes < 0:
        raise RuntimeError("sir_csr_build_workspace failed (sizes out of range or no device)")
    ws = torch.empty((ws_bytes,), dtype=torch.uint8, device=dev)
    rowptr = torch.empty((n_rows + 1,), dtype=torch.int32, device=dev)
    col = torch.empty((E,), dtype=torch.int32, device=dev)
    eid = torch.empty((E,), dtype=torch.int64, device=dev)
    items = torch.empty((n_rows + E // chunk + 1, 4), dtype=torch.int32, device=dev)
    splits = torch.empty((min(n_rows, E // (chunk + 1)) + 1, 4), dtype=torch.int32, device=dev)
    counts = torch.empty((5,), dtype=torch.int64, device=dev)
    with _Timed("sir_csr_build", dev):
        rc = lib.sir_csr_build(_ptr(rows), _ptr(cols), E, n_rows, n_cols, chunk, _ptr(rowptr), _ptr(col),
                               _ptr(eid), _ptr(items), _ptr(splits), _ptr(counts), _ptr(ws), ws_bytes,
                               _stream(dev))
    _check(rc, lib)
    return rowptr, col, eid, items, splits, counts


def csr_perm(eid_a, eid_b):
    """perm[j] = position in CSR A of the edge at position j of CSR B (int32, async)."""
    lib = load()
    E = eid_a.numel()
    pos = torch.empty((E,), dtype=torch.int32, device=eid_a.device)
    perm = torch.empty((E,), dtype=torch.int32, device=eid_a.device)
    rc = lib.sir_csr_perm(_ptr(eid_a), _ptr(eid_b), E, _ptr(pos), _ptr(perm), _stream(eid_a.device))
    _check(rc, lib)
    return perm


# ------------------------------------------------------------------------------ GraphNorm
def graph_norm_fwd(off, X, weight, bias, mean_scale, eps, Y, mean, std):
    lib = load()
    B, F = mean.shape
    with _Timed("sir_graph_norm_fwd", Y.device):
        rc = lib.sir_graph_norm_fwd(_ptr(off), B, F, _ptr(X), _ld(X, F), _ptr(weight), _ptr(bias),
                                    _ptr(mean_scale), float(eps), _ptr(Y), _ld(Y, F), _ptr(mean), _ptr(std),
                                    _stream(Y.device))
    _check(rc, lib)


_DT_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}     # SIR_DTYPE_F32 / BF16 / F16


def resid_act_fwd(Y, R, act, slope, order, out):
    """out = act(Y + R) (order 0) or act(Y) + R (order 1) in one pass (``sir_resid_act_fwd``)."""
    lib = load()
    M, N = Y.shape
    with _Timed("sir_resid_act_fwd", out.device):
        rc = lib.sir_resid_act_fwd(_ptr(Y), Y.stride(0), _DT_CODE[Y.dtype], _ptr(R), R.stride(0), _ptr(out),
                                   out.stride(0), M, N, int(act), float(slope), int(order), _stream(out.device))
    _check(rc, lib)


def resid_act_bwd(D, Y, R, act, slope, order, dY, dR=None, D2=None):
    """Backward of :func:`resid_act_fwd` (``sir_resid_act_bwd``): dY in Y's type; order 0 also dR.  D2
    (order 0): a second fp32 gradient of the output, added to D as it is read."""
    lib = load()
    M, N = Y.shape
    with _Timed("sir_resid_act_bwd", dY.device):
        rc = lib.sir_resid_act_bwd(_ptr(D), D.stride(0), _ptr(D2), D2.stride(0) if D2 is not None else 0,
                                   _ptr(Y), Y.stride(0), _DT_CODE[Y.dtype], _ptr(R),
                                   R.stride(0) if R is not None else 0, _ptr(dY), dY.stride(0), _ptr(dR),
                                   dR.stride(0) if dR is not None else 0, M, N, int(act), float(slope), int(order),
                                   _stream(dY.device))
    _check(rc, lib)


def graph_norm_act_fwd(off, X, weight, bias, mean_scale, eps, act, slope, R, Y, mean, std):
    """GraphNorm -> act -> + R in one kernel (``sir_graph_norm_act_fwd``; R may be None)."""
    lib = load()
    B, F = mean.shape
    with _Timed("sir_graph_norm_fwd", Y.device):
        rc = lib.sir_graph_norm_act_fwd(_ptr(off), B, F, _ptr(X), _ld(X, F), _ptr(weight), _ptr(bias),
                                        _ptr(mean_scale), float(eps), int(act), float(slope), _ptr(R),
                                        _ld(R, F) if R is not None else 0, _ptr(Y), _ld(Y, F), _ptr(mean), _ptr(std),
                                        _stream(Y.device))
    _check(rc, lib)


def graph_norm_act_bwd(off, X, dY, weight, bias, mean_scale, mean, std, act, slope, dX, dw_part, dms_part, db_part):
    """Backward of :func:`graph_norm_act_fwd` (dY: the gradient of its output)."""
    lib = load()
    B, F = mean.shape
    with _Timed("sir_graph_norm_bwd", dX.device):
        rc = lib.sir_graph_norm_act_bwd(_ptr(off), B, F, _ptr(X), _ld(X, F), _ptr(dY), _ld(dY, F), _ptr(weight),
                                        _ptr(bias), _ptr(mean_scale), _ptr(mean), _ptr(std), int(act), float(slope),
                                        _ptr(dX), _ld(dX, F), _ptr(dw_part), _ptr(dms_part), _ptr(db_part),
                                        _stream(dX.device))
    _check(rc, lib)


def graph_norm_bwd(off, X, dY, weight, mean_scale, mean, std, dX, dw_part, dms_part, db_part):
    lib = load()
    B, F = mean.shape
    with _Timed("sir_graph_norm_bwd", dX.device):
        rc = lib.sir_graph_norm_bwd(_ptr(off), B, F, _ptr(X), _ld(X, F), _ptr(dY), _ld(dY, F), _ptr(weight),
                                    _ptr(mean_scale), _ptr(mean), _ptr(std), _ptr(dX), _ld(dX, F),
                                    _ptr(dw_part), _ptr(dms_part), _ptr(db_part), _stream(dX.device))
    _check(rc, lib)


# ------------------------------------------------------------------------------ projection GEMMs
def gemm_pack(W, trans=False):
    """Pack the weight operand of ``gemm_nt``: B = W ([N, K], an nn.Linear weight used as x W^T)
    or, with trans=True, B = W^T (W [K, N], used as x W).  Returns (packed uint8 tensor, N, K)."""
    lib = load()
    assert W.dtype == torch.float32 and W.dim() == 2 and W.stride(1) == 1
    N, K = (W.shape[1], W.shape[0]) if trans else (W.shape[0], W.shape[1])
    nbytes = lib.sir_gemm_pack_bytes(N, K)
    if nbytes <= 0:
        raise RuntimeError(f"sir_gemm_pack_bytes({N}, {K}) failed")
    packed = torch.empty((nbytes,), dtype=torch.uint8, device=W.device)
    with _Timed("sir_gemm_pack", W.device):
        rc = lib.sir_gemm_pack(_ptr(W), W.stride(0), N, K, int(bool(trans)), _ptr(packed), _stream(W.device))
    _check(rc, lib)
    return packed, N, K


def gemm_nt(A, packed, bias=None, out=None, drop=None):
    """C = A B^T (+ bias) on the split-fp16 MFMA kernel; ``packed`` from gemm_pack.  ``drop``:
    optional (seed, p) feature dropout of the output (C columns = QK columns)."""
    lib = load()
    pk, N, K = packed
    M = A.shape[0]
    assert A.dim() == 2 and A.shape[1] == K and A.stride(1) == 1
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=A.device)
    with _Timed(f"sir_gemm_nt K={K} N={N}", A.device, (2 * M * N * K, 4 * M * (K + N))):
        rc = lib.sir_gemm_nt(_ptr(A), A.stride(0), M, K, _ptr(pk), N, _ptr(bias), _ptr(out), out.stride(0),
                             _drop(drop), _stream(A.device))
    _check(rc, lib)
    return out


def gemm_nt_dact(A, packed, gate, act, slope, out=None, gate_mask=None):
    """C = sigma'(gate) * (A B^T) (``sir_gemm_nt_dact``: the ReLU family's backward in the GEMM epilogue;
    ``gate`` = the activation's input or output, C's shape and leading dimension, or ``gate_mask`` =
    its sign words from ``edge_gather_act``, N = 256)."""
    lib = load()
    pk, N, K = packed
    M = A.shape[0]
    assert A.dim() == 2 and A.shape[1] == K and A.stride(1) == 1
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=A.device)
    if gate_mask is None:
        assert gate.shape == out.shape and gate.stride() == out.stride()
    else:
        assert N == 256 and gate_mask.numel() == 4 * M
    with _Timed(f"sir_gemm_nt_dact K={K} N={N}", A.device, (2 * M * N * K, 4 * M * (K + N))):
        rc = lib.sir_gemm_nt_dact(_ptr(A), A.stride(0), M, K, _ptr(pk), N, _ptr(gate) if gate_mask is None else None,
                                  _ptr(gate_mask), int(act), float(slope), _ptr(out), out.stride(0), _stream(A.device))
    _check(rc, lib)
    return out


def gemm_nt_direct(A, W, trans=False, bias=None, out=None, drop=None):
    """C = A W^T (+ bias) (trans=False, W [N, K]) or A W (trans=True, W [K, N]) with the fp32 weight
    read directly — no packing pass (``sir_gemm_nt_direct``: the small-batch route)."""
    lib = load()
    M, K = A.shape
    N = W.shape[1] if trans else W.shape[0]
    assert A.stride(1) == 1 and W.stride(1) == 1 and W.shape[0 if trans else 1] == K
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=A.device)
    with _Timed(f"sir_gemm_nt_direct K={K} N={N}", A.device, (2 * M * N * K, 4 * M * (K + N))):
        rc = lib.sir_gemm_nt_direct(_ptr(A), A.stride(0), M, K, _ptr(W), W.stride(0), int(trans), N, _ptr(bias),
                                    _ptr(out), out.stride(0), _drop(drop), _stream(A.device))
    _check(rc, lib)
    return out


def gemm_nt_direct2(A, W, W2, trans=False, bias=None, bias_cols=None, out=None, drop=None):
    """:func:`gemm_nt_direct` on the weight [W; W2] stacked along its row index (trans=False: W
    [N1, K], W2 [N2, K] -> N = N1 + N2 outputs; trans=True: W [K1, N], W2 [K2, N] -> K = K1 + K2),
    read in place (``sir_gemm_nt_direct2``), the bias on the first ``bias_cols`` outputs."""
    lib = load()
    M, K = A.shape
    if trans:
        N = W.shape[1]
        assert W2.shape[1] == N and W.shape[0] + W2.shape[0] == K
    else:
        N = W.shape[0] + W2.shape[0]
        assert W.shape[1] == K and W2.shape[1] == K
    assert A.stride(1) == 1 and W.stride(1) == 1 and W2.stride(1) == 1
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=A.device)
    bc = (bias.numel() if bias is not None else 0) if bias_cols is None else bias_cols
    with _Timed(f"sir_gemm_nt_direct K={K} N={N}", A.device, (2 * M * N * K, 4 * M * (K + N))):
        rc = lib.sir_gemm_nt_direct2(_ptr(A), A.stride(0), M, K, _ptr(W), W.stride(0), _ptr(W2), W2.stride(0),
                                     W.shape[0], int(trans), N, _ptr(bias), bc, _ptr(out), out.stride(0), _drop(drop),
                                     _stream(A.device))
    _check(rc, lib)
    return out


def gemm_tn(A, B, out=None, colsum=False):
    """C = A^T B (A [R, M], B [R, N]) on the split-fp16 MFMA kernel (split over row ranges).
    With ``colsum=True`` returns ``(C, A.sum(0))``: the column sums (a linear's bias gradient)
    come out of the same pass over A."""
    lib = load()
    R, M = A.shape
    N = B.shape[1]
    assert B.shape[0] == R and A.stride(1) == 1 and B.stride(1) == 1
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=A.device)
    cs = torch.empty((M,), dtype=torch.float32, device=A.device) if colsum else None
    ws_bytes = lib.sir_gemm_tn_workspace(R, M, N)
    ws = torch.empty((max(ws_bytes, 4),), dtype=torch.uint8, device=A.device)
    with _Timed(f"sir_gemm_tn M={M} N={N}", A.device, (2 * R * M * N, 4 * R * (M + N))):
        rc = lib.sir_gemm_tn(_ptr(A), A.stride(0), _ptr(B), B.stride(0), R, M, N, _ptr(out), out.stride(0),
                             _ptr(cs), _ptr(ws), ws.numel(), _stream(A.device))
    _check(rc, lib)
    return (out, cs) if colsum else out


_DT16 = {torch.bfloat16: 1, torch.float16: 2}      # SIR_DTYPE_BF16 / SIR_DTYPE_F16


def gemm_tn16(A, B, out=None, colsum=False):
    """C = A^T B for bf16 / fp16 A [R, M], B [R, N] (same dtype), fp32 result, on the 16-bit MFMA
    kernel (each 16-bit product exact in fp32; no operand split).  ``colsum=True`` also returns
    A.sum(0) in fp32 from the same pass."""
    lib = load()
    R, M = A.shape
    N = B.shape[1]
    assert B.shape[0] == R and A.stride(1) == 1 and B.stride(1) == 1 and A.dtype == B.dtype and A.dtype in _DT16
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=A.device)
    cs = torch.empty((M,), dtype=torch.float32, device=A.device) if colsum else None
    ws_bytes = lib.sir_gemm_tn_workspace(R, M, N)
    ws = torch.empty((max(ws_bytes, 4),), dtype=torch.uint8, device=A.device)
    with _Timed("sir_gemm_tn16", A.device, (2 * R * M * N, A.element_size() * R * (M + N))):
        rc = lib.sir_gemm_tn16(_ptr(A), A.stride(0), _ptr(B), B.stride(0), R, M, N, _DT16[A.dtype], _ptr(out),
                               out.stride(0), _ptr(cs), _ptr(ws), ws.numel(), _stream(A.device))
    _check(rc, lib)
    return (out, cs) if colsum else out


def gemm_pack16(W, dtype, trans=False):
    """Pack the weight operand of ``gemm_nt16``: B = W ([N, K]) or W^T (trans), rounded to the
    16-bit ``dtype`` (what autocast's ``W.to(dtype)`` holds).  Returns (packed, N, K, dtype)."""
    lib = load()
    assert W.dtype == torch.float32 and W.dim() == 2 and W.stride(1) == 1 and dtype in _DT16
    N, K = (W.shape[1], W.shape[0]) if trans else (W.shape[0], W.shape[1])
    nbytes = lib.sir_gemm_pack16_bytes(N, K)
    if nbytes <= 0:
        raise RuntimeError(f"sir_gemm_pack16_bytes({N}, {K}) failed")
    packed = torch.empty((nbytes,), dtype=torch.uint8, device=W.device)
    with _Timed("sir_gemm_pack16", W.device):
        rc = lib.sir_gemm_pack16(_ptr(W), W.stride(0), N, K, int(bool(trans)), _DT16[dtype], _ptr(packed),
                                 _stream(W.device))
    _check(rc, lib)
    return packed, N, K, dtype


def gemm_nt16(A, packed, bias=None, out_dtype=None, acopy=None, drop=None, out=None):
    """C = A B^T (+ bias) on the 16-bit MFMA kernel (``packed`` from gemm_pack16).  A in the
    packed dtype or fp32 (rounded on load; ``acopy`` [M, K] of that dtype receives the rounded A);
    C in ``out_dtype`` (the packed dtype by default, or fp32).  ``bias`` fp32 [N] (pass autocast's
    dtype-rounded bias to match its nn.Linear)."""
    lib = load()
    pk, N, K, dt = packed
    M = A.shape[0]
    assert A.dim() == 2 and A.shape[1] == K and A.stride(1) == 1 and A.dtype in (dt, torch.float32)
    od = out_dtype or dt
    if out is None:
        out = torch.empty((M, N), dtype=od, device=A.device)
    assert out.dtype == od and out.shape == (M, N) and out.stride(1) == 1
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous()
    with _Timed("sir_gemm_nt16", A.device, (2 * M * N * K, A.element_size() * M * K + out.element_size() * M * N
                                            + (acopy.element_size() * M * K if acopy is not None else 0))):
        rc = lib.sir_gemm_nt16(_ptr(A), A.stride(0), STORAGE[A.dtype], M, K, _ptr(pk), N, _DT16[dt], _ptr(bias),
                               _ptr(out), out.stride(0), STORAGE[od], _ptr(acopy),
                               acopy.stride(0) if acopy is not None else 0, _drop(drop), _stream(A.device))
    _check(rc, lib)
    return out


def dropout_apply(X, drop, col0=0):
    """In place: the hashed feature dropout (seed, p) of QK on the [M, N] block X (columns col0 ..)."""
    lib = load()
    M, N = X.shape
    assert X.stride(1) == 1 and X.dtype in STORAGE
    with _Timed("sir_dropout_apply", X.device):
        rc = lib.sir_dropout_apply(_ptr(X), X.stride(0), M, N, STORAGE[X.dtype], col0, _drop(drop), _stream(X.device))
    _check(rc, lib)
    return X


def max_dw_rows(dcsr, arg, dY, A, O):
    """dW_R [O, H], db_R [O] of the materialised max backward from A [E, H] (dst-CSR order) and the
    arg edges, without dM (``sir_max_dw_rows``)."""
    lib = load()
    H = A.shape[1]
    V = dcsr.n_rows
    R = max(int(lib.sir_max_dw_rows_parts(V, H)), 1)
    ldw = O * H + (O + 3) // 4 * 4
    wpart = torch.empty((R, ldw), device=A.device, dtype=torch.float32)
    with _Timed("sir_max_dw_rows", A.device):
        rc = lib.sir_max_dw_rows(_ptr(dcsr.rowptr), V, _ptr(arg), arg.stride(0), _ptr(dY), dY.stride(0), _ptr(A),
                                 A.stride(0), O, H, _ptr(wpart), ldw, _stream(A.device))
    _check(rc, lib)
    tot = col_sum(wpart)
    return tot[:O * H].view(O, H), tot[O * H:O * H + O]


def max_dw_qk(dcsr, arg, dY, Q, K, O, act1, slope):
    """dW_R [O, H], db_R [O] of the max backward with a = act1(Q[v] + K[u]) recomputed per row batch
    (``sir_max_dw_qk``): no A buffer."""
    lib = load()
    H = Q.shape[1]
    V = dcsr.n_rows
    R = max(int(lib.sir_max_dw_rows_parts(V, H)), 1)
    ldw = O * H + (O + 3) // 4 * 4
    wpart = torch.empty((R, ldw), device=Q.device, dtype=torch.float32)
    # a graph without edges has no col storage; the kernel reads no column id then (every row is empty)
    col = dcsr.col if dcsr.col.numel() else torch.zeros(1, dtype=torch.int32, device=Q.device)
    with _Timed("sir_max_dw_qk", Q.device):
        rc = lib.sir_max_dw_qk(_ptr(dcsr.rowptr), _ptr(col), V, _ptr(arg), arg.stride(0), _ptr(dY), dY.stride(0),
                               _ptr(Q), Q.stride(0), _ptr(K), K.stride(0), O, H, int(act1), float(slope), _ptr(wpart),
                               ldw, _stream(Q.device))
    _check(rc, lib)
    tot = col_sum(wpart)
    return tot[:O * H].view(O, H), tot[O * H:O * H + O]
