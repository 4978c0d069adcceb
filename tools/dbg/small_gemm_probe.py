"""Per-launch time of the small-batch GEMMs at config 5's shapes (1582 node rows, hidden 300), timed
over back-to-back launches with HIP events, eager and inside a HIP graph, beside torch's fp32 GEMM
and a trivial elementwise launch of the same size (the fixed per-launch floor)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "sir-gcn_amd"))
from sirgcn import _native  # noqa: E402


def timeit(fn, n=200, graph=False):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        if graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(n):
                    fn()
            run = g.replay
        else:
            def run():
                for _ in range(n):
                    fn()
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        run()
        e1.record(s)
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / n


def main():
    torch.manual_seed(0)
    M = int(os.environ.get("M", 1582))
    H = 300
    X = torch.randn(M, H, device="cuda")
    X2 = torch.randn(M, 2 * H, device="cuda")
    Wqk = torch.randn(2 * H, H, device="cuda") * 0.05
    Wr = torch.randn(H, H, device="cuda") * 0.05
    Wcat = torch.randn(2 * H, H, device="cuda") * 0.05
    b = torch.randn(2 * H, device="cuda")
    dY = torch.randn(M, H, device="cuda")
    o600 = torch.empty(M, 2 * H, device="cuda")
    o300 = torch.empty(M, H, device="cuda")
    cases = {
        "nt_direct K=300 N=600 (QK fwd)": lambda: _native.gemm_nt_direct(X, Wqk, False, b, o600),
        "nt_direct K=300 N=300 (R fwd)": lambda: _native.gemm_nt_direct(X, Wr, False, None, o300),
        "nt_direct trans K=300 N=300 (dY W_R)": lambda: _native.gemm_nt_direct(dY, Wr, True, None, o300),
        "nt_direct trans K=600 N=300 (dX)": lambda: _native.gemm_nt_direct(X2, Wcat, True, None, o300),
        "gemm_tn 300x300 colsum (dW_R)": lambda: _native.gemm_tn(dY, X, colsum=True),
        "gemm_tn 600x300 colsum (dW_QK)": lambda: _native.gemm_tn(X2, X, colsum=True),
        "torch.mm K=300 N=600": lambda: torch.mm(X, Wqk.t(), out=o600),
        "torch.mm K=300 N=300": lambda: torch.mm(X, Wr.t(), out=o300),
        "torch.add M x 300": lambda: torch.add(X, dY, out=o300),
        "torch.zero_ M x 300": lambda: o300.zero_(),
    }
    lt = os.environ.get("LT_CFGS", "0,1,2,3,4,5").split(",")
    for name, fn in cases.items():
        var = "SIR_LT_NT" if "nt_direct" in name else ("SIR_LT_TN" if "gemm_tn" in name else None)
        for c in (lt if var else ["-"]):
            if var:
                if var == "SIR_LT_TN" and int(c) > 5:
                    continue
                os.environ[var] = c
            te = timeit(fn)
            tg = timeit(fn, graph=True)
            print(f"{name:40s} lt={c} eager {te:7.2f} us   graph {tg:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
