"""Debug: persistent vs classic NT GEMM element by element (one small shape)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "sir-gcn_amd"))
import torch
from sirgcn import _native


def open_lib(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _native.SIGNATURES.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    return lib


P = _native._ptr
dev = "cuda"
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
libs = {n: open_lib(os.path.join(ROOT, "sir-gcn_amd/lib", f)) for n, f in (("old", "libsirconv_ntclassic.so"), ("new", "libsirconv.so"))}
for (M, K, N, kind) in [(255, 256, 256, "ones"), (255, 256, 256, "randn"), (600, 256, 512, "randn")]:
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.ones(M, K, device=dev) if kind == "ones" else torch.randn(M, K, device=dev, generator=g)
    W = torch.ones(N, K, device=dev) if kind == "ones" else torch.randn(N, K, device=dev, generator=g)
    outs = {}
    for n, lib in libs.items():
        pk = torch.empty(lib.sir_gemm_pack_bytes(N, K), dtype=torch.uint8, device=dev)
        assert lib.sir_gemm_pack(P(W), W.stride(0), N, K, 0, P(pk), st) == 0
        C = torch.full((M, N), float("nan"), device=dev)
        assert lib.sir_gemm_nt(P(A), A.stride(0), M, K, P(pk), N, None, P(C), C.stride(0), None, st) == 0, lib.sir_last_error()
        torch.cuda.synchronize()
        outs[n] = C.cpu()
    ref = (A @ W.t()).cpu()
    o, nw = outs["old"], outs["new"]
    print(f"M={M} K={K} N={N} {kind}: old relerr {((o-ref).norm()/ref.norm()).item():.2e} new nan {torch.isnan(nw).sum().item()}")
    bad = ~torch.isclose(nw, o, rtol=1e-4, atol=1e-3)
    print("  bad elements", bad.sum().item(), "of", bad.numel())
    if bad.any():
        rows = bad.any(1).nonzero().flatten()
        cols = bad.any(0).nonzero().flatten()
        print("  bad rows", rows[:20].tolist(), "... n", rows.numel(), " bad cols", cols[:40].tolist(), "... n", cols.numel())
        r, c = bad.nonzero()[0].tolist()
        print("  first bad", r, c, "new", nw[r, c].item(), "old", o[r, c].item(), "ref", ref[r, c].item())
        print("  new row r[:16]", nw[r, :16].tolist())
        print("  old row r[:16]", o[r, :16].tolist())
        ratio = (nw / o)[bad]
        print("  ratio stats", ratio.min().item(), ratio.max().item(), ratio.median().item())
