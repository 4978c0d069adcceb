"""Probe fp32 GEMM formulations of the SIRConv projections on MI355X (timing only)."""
import time
import torch

dev = "cuda"
V, H = 2_000_000, 256
torch.manual_seed(0)
X = torch.randn(V, H, device=dev)
dY = torch.randn(V, H, device=dev)
S = torch.randn(V, H, device=dev)
dQK = torch.randn(V, 2 * H, device=dev)
W = torch.randn(2 * H, H, device=dev)


def t(fn, n=10):
    fn(); torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def tf(ms, flops):
    return f"{ms:7.3f} ms {flops / ms / 1e9:7.1f} TF/s"


f1 = 2 * V * H * H
f2 = 2 * V * 2 * H * H
print("dW_R = dY^T S        ", tf(t(lambda: torch.mm(dY.t(), S)), f1))
print("dW_R = (S^T dY)^T    ", tf(t(lambda: torch.mm(S.t(), dY).t()), f1))
for k in (4, 8, 16, 32):
    print(f"dW_R bmm split{k:3d}     ", tf(t(lambda: torch.bmm(dY.view(k, V // k, H).transpose(1, 2), S.view(k, V // k, H)).sum(0)), f1))
print("dW_cat = dQK^T X     ", tf(t(lambda: torch.mm(dQK.t(), X)), f2))
print("dW_cat = (X^T dQK)^T ", tf(t(lambda: torch.mm(X.t(), dQK).t()), f2))
for k in (8, 16, 32):
    print(f"dW_cat bmm split{k:3d}   ", tf(t(lambda: torch.bmm(dQK.view(k, V // k, 2 * H).transpose(1, 2), X.view(k, V // k, H)).sum(0)), f2))
print("QK = X W^T           ", tf(t(lambda: torch.mm(X, W.t())), f2))
print("QK = addmm           ", tf(t(lambda: torch.addmm(torch.zeros(2 * H, device=dev), X, W.t())), f2))
print("dX = dQK W           ", tf(t(lambda: torch.mm(dQK, W)), f2))
print("Y = S W_R^T          ", tf(t(lambda: torch.mm(S, W[:H].t())), f1))
print("G = dY W_R           ", tf(t(lambda: torch.mm(dY, W[:H])), f1))
print("db = dY.sum(0)       ", f"{t(lambda: dY.sum(0)):7.3f} ms")
ones = torch.ones(V, device=dev)
print("db = ones@dY (gemv)  ", f"{t(lambda: torch.mv(dY.t(), ones)):7.3f} ms")
print("db = dQK.sum(0)      ", f"{t(lambda: dQK.sum(0)):7.3f} ms")
# precision check: is the library fp32 GEMM exact-fp32 class?
a = torch.randn(4096, 4096, device=dev); b = torch.randn(4096, 4096, device=dev)
r = (a.double() @ b.double())
e = ((a @ b).double() - r).norm() / r.norm()
print("fp32 GEMM rel err vs fp64:", e.item())
# concurrency: edge-like memory stream kernel + GEMM on two streams
s1 = torch.cuda.Stream()
idx = torch.randint(0, V, (20_000_000,), device=dev)
def gather(): return X.index_select(0, idx[:4_000_000])
tg = t(gather); tm = t(lambda: torch.mm(dY.t(), S))
def both():
    with torch.cuda.stream(s1):
        torch.mm(dY.t(), S)
    gather()
    torch.cuda.current_stream().wait_stream(s1)
print(f"gather {tg:.3f} ms, gemm {tm:.3f} ms, concurrent {t(both):.3f} ms")
