"""Feature dropout on Q and K (``conv.py:35,60-61``), fused into the layer (``sirconv_dropout.h``).

The reference trains most published configs with ``feat_dropout`` 0.1-0.2 (``ogbn-arxiv/train.py:303``,
``ogbg-molhiv/train.py:249``).  The fused layer applies a hashed mask in the QK GEMM's epilogue and
the same mask (recomputed from (seed, row, column)) in the backward edge passes — no mask tensor.
Checked here (through the C ABI):

* the mask itself: keep rate 1 - p per half, Q and K bits independent, survivors scaled by
  1 / (1 - p), different seeds give different masks;
* every QK GEMM the layer can route to (split-fp16 persistent / tiled / weight-resident kernels,
  16-bit kernel with fp32 or 16-bit A) applies EXACTLY the mask of ``sir_dropout_apply``;
* train mode: Y and every gradient equal the reference dataflow evaluated with that explicit mask
  (fp64 oracle; fp32 and bf16 autocast), i.e. the backward uses the forward's mask;
* eval mode: bit-identical to a dropout=0 layer, and equal to the golden fixtures of the
  reference's own ``conv.py``.
"""
import numpy as np
import pytest
import torch
from torch import nn

import oracle
from conftest import assert_parity, golden_manifest, load_case, rel_err

from sirgcn import SIRConv, _native
from sirgcn.graph import Graph

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need the MI355X box"
    _native.load()


def _mask(V, H2, seed, p, dtype=torch.float32):
    """The hashed keep mask x scale of QK [V, 2H] (sir_dropout_apply on ones)."""
    return _native.dropout_apply(torch.ones(V, H2, device=DEV, dtype=dtype), (seed, p))


@pytest.mark.parametrize("p", [0.1, 0.2, 0.5])
def test_mask_statistics(p):
    V, H = 20000, 256
    m = _mask(V, 2 * H, 12345, p)
    kept = m != 0
    scale = torch.tensor(1.0 / (1.0 - p), dtype=torch.float32).item()
    assert torch.all(m[kept] == scale), "survivors scaled by 1 / (1 - p) (fp32)"
    for half in (kept[:, :H], kept[:, H:]):
        assert abs(1 - half.float().mean().item() - p) < 0.003
    both = (kept[:, :H] & kept[:, H:]).float().mean().item()
    assert abs(both - (1 - p) ** 2) < 0.004, "Q and K bits independent"
    # rows and columns are not correlated with each other (a shifted row has its own bits)
    assert abs((kept[1:] & kept[:-1]).float().mean().item() - (1 - p) ** 2) < 0.004
    m2 = _mask(V, 2 * H, 12346, p)
    assert not torch.equal(m, m2)
    assert torch.equal(m, _mask(V, 2 * H, 12345, p)), "deterministic in (seed, p)"
    assert torch.all(_mask(64, 64, 1, 1.0) == 0) and torch.all(_mask(64, 64, 1, 0.0) == 1)


@pytest.mark.parametrize("M,K,N", [(70001, 256, 512), (3001, 128, 256), (5000, 256, 256), (2000, 300, 200),
                                   (4099, 512, 256), (300, 64, 96), (70001, 256, 200)])
def test_gemm_epilogue_applies_the_mask(M, K, N):
    """C = drop(A W^T + b) in the GEMM epilogue == sir_dropout_apply on the plain GEMM, bit for bit
    (the shapes route to the persistent, tiled and small-batch split-fp16 kernels)."""
    g = torch.Generator(device=DEV).manual_seed(M + N)
    A = torch.randn(M, K, device=DEV, generator=g)
    W = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
    b = torch.randn(N, device=DEV, generator=g)
    pk = _native.gemm_pack(W)
    d = (987654321, 0.2)
    C = _native.gemm_nt(A, pk, b, drop=d)
    ref = _native.dropout_apply(_native.gemm_nt(A, pk, b), d)
    assert torch.equal(C, ref)
    assert abs((C == 0).float().mean().item() - 0.2) < 0.02


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("a32", [True, False])
def test_gemm16_epilogue_applies_the_mask(dt, a32):
    """The autocast QK GEMM (16-bit output): drop(round(x)) rounded again == sir_dropout_apply on
    the 16-bit result, bit for bit."""
    g = torch.Generator(device=DEV).manual_seed(7)
    M, K, N = 33000, 256, 512
    A = torch.randn(M, K, device=DEV, generator=g)
    if not a32:
        A = A.to(dt)
    W = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
    b = torch.randn(N, device=DEV, generator=g).to(dt).float()
    pk = _native.gemm_pack16(W, dt)
    d = (42, 0.2)
    C = _native.gemm_nt16(A, pk, b, drop=d)
    ref = _native.dropout_apply(_native.gemm_nt16(A, pk, b), d)
    assert C.dtype == dt and torch.equal(C, ref)


def _explicit_mask_reference(src, dst, V, X, W_Q, b_Q, W_K, W_R, b_R, dY, Mk, agg, dtype=torch.float64):
    """The reference dataflow (conv.py:49-67 through the oracle) with the dropout replaced by the
    explicit keep-mask x scale ``Mk`` [V, 2H]: returns Y and the gradients (autograd)."""
    H = W_Q.shape[0]
    t = lambda x: x.detach().cpu().to(dtype).requires_grad_(True)
    X64, WQ, bQ, WK, WR, bR = (t(x) for x in (X, W_Q, b_Q, W_K, W_R, b_R))
    Mk = Mk.detach().cpu().to(dtype)
    Q = (X64 @ WQ.t() + bQ) * Mk[:, :H]
    K = (X64 @ WK.t()) * Mk[:, H:]
    S = oracle.edge_agg_fwd(src, dst, V, Q, K, agg, "leaky", 0.2)
    Y = S @ WR.t() + bR
    Y.backward(dY.detach().cpu().to(dtype))
    return {"Y": Y.detach(), "dX": X64.grad, "dW_Q": WQ.grad, "db_Q": bQ.grad, "dW_K": WK.grad, "dW_R": WR.grad,
            "db_R": bR.grad}


@pytest.mark.parametrize("agg", ["sum", "mean", "sym"])
@pytest.mark.parametrize("H", [256, 128])
def test_fused_layer_train_mode_vs_explicit_mask(agg, H):
    """Train mode, p = 0.2: the fused layer (SIRConvFunction) equals the reference dataflow with the
    same mask applied explicitly — forward and every gradient (so the backward edge passes apply
    the forward's mask to dQ and dK)."""
    gen = torch.Generator().manual_seed(11)
    V, E, d, O, p = 700, 12000, 48, 32, 0.2
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V, (E,), generator=gen)
    X, dY = torch.randn(V, d, generator=gen), torch.randn(V, O, generator=gen)
    torch.manual_seed(3)
    m = SIRConv(d, H, O, nn.LeakyReLU(0.2), p, agg_type=agg).to(DEV).train()
    seeds = []
    draw = m._drop
    m._drop = lambda dev: seeds.append(draw(dev)) or seeds[-1]
    g = Graph(src, dst, V)
    Xd = X.to(DEV).requires_grad_(True)
    Y = m(g, Xd)
    Y.backward(dY.to(DEV))
    assert len(seeds) == 1 and seeds[0][1] == p
    Mk = _mask(V, 2 * H, *seeds[0])
    w = lambda mod: getattr(m, mod)
    args = (X, w("linear_query").weight, w("linear_query").bias, w("linear_key").weight, w("linear_relation").weight,
            w("linear_relation").bias, dY, Mk, agg)
    truth = _explicit_mask_reference(src, dst, V, *args)
    ref32 = _explicit_mask_reference(src, dst, V, *args, dtype=torch.float32)
    assert_parity(Y.detach().cpu(), ref32["Y"], truth["Y"], 1e-5, f"dropout {agg} H={H} Y", strict=True)
    got = {"dX": Xd.grad, "dW_Q": m.linear_query.weight.grad, "db_Q": m.linear_query.bias.grad,
           "dW_K": m.linear_key.weight.grad, "dW_R": m.linear_relation.weight.grad, "db_R": m.linear_relation.bias.grad}
    for k, v in got.items():
        assert_parity(v.cpu(), ref32[k], truth[k], 1e-5, f"dropout {agg} H={H} {k}")


class _FixedMask(nn.Module):
    """nn.Dropout replaced by a given keep-mask x scale, in the reference's call order (conv.py:60
    then :61: K first, then Q); a 16-bit input is scaled in fp32 and rounded back, as torch's
    Dropout of a half-precision tensor does."""

    def __init__(self, Mk, H):
        super().__init__()
        self.parts = [Mk[:, H:], Mk[:, :H]]
        self.i = 0

    def forward(self, x):
        m = self.parts[self.i % 2]
        self.i += 1
        return (x.float() * m).to(x.dtype)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_fused_autocast_layer_train_mode_vs_explicit_mask(dt):
    """Under autocast (SIRConvFunction16): the same mask on the 16-bit QK.  Y and gradients against
    the fp64 explicit-mask truth: within the AMP bar (2e-2 bf16 / 1e-2 fp16), or no worse than 1.25x
    the reference's own AMP dataflow with the same mask (oracle.SIRConvRef under autocast) — the
    criterion of tests/test_amp_gpu.py."""
    gen = torch.Generator().manual_seed(12)
    V, E, d, H, O, p = 40000, 300000, 64, 256, 64, 0.2     # >= MIN_ROWS_16: the native 16-bit GEMMs
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V, (E,), generator=gen)
    X, dY = torch.randn(V, d, generator=gen), torch.randn(V, O, generator=gen)
    torch.manual_seed(5)
    m = SIRConv(d, H, O, nn.LeakyReLU(0.2), p, agg_type="sum").to(DEV).train()
    seeds = []
    draw = m._drop
    m._drop = lambda dev: seeds.append(draw(dev)) or seeds[-1]
    g = Graph(src, dst, V)
    Xd = X.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=dt):
        Y = m(g, Xd)
    Y.backward(dY.to(DEV).to(Y.dtype))
    assert len(seeds) == 1
    Mk = _mask(V, 2 * H, *seeds[0])
    w = lambda mod: getattr(m, mod)
    truth = _explicit_mask_reference(src, dst, V, X, w("linear_query").weight, w("linear_query").bias,
                                     w("linear_key").weight, w("linear_relation").weight,
                                     w("linear_relation").bias, dY, Mk, "sum")
    mr = oracle.SIRConvRef(d, H, O, nn.LeakyReLU(0.2), 0, agg_type="sum").to(DEV)
    mr.load_state_dict(m.state_dict())
    mr.dropout = _FixedMask(Mk, H)
    xr = X.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=dt):
        Yr = mr(g, xr)
    Yr.backward(dY.to(DEV).to(Yr.dtype))
    got = {"Y": Y, "dX": Xd.grad, "dW_Q": m.linear_query.weight.grad, "db_Q": m.linear_query.bias.grad,
           "dW_K": m.linear_key.weight.grad, "dW_R": m.linear_relation.weight.grad,
           "db_R": m.linear_relation.bias.grad}
    amp = {"Y": Yr, "dX": xr.grad, "dW_Q": mr.linear_query.weight.grad, "db_Q": mr.linear_query.bias.grad,
           "dW_K": mr.linear_key.weight.grad, "dW_R": mr.linear_relation.weight.grad,
           "db_R": mr.linear_relation.bias.grad}
    tol = 2e-2 if dt == torch.bfloat16 else 1e-2
    for k, v in got.items():
        e = rel_err(v.detach().double().cpu(), truth[k])
        e_amp = rel_err(amp[k].detach().double().cpu(), truth[k])
        assert e <= max(tol, 1.25 * e_amp), f"{k}: relL2 {e:.3e} vs fp64 (reference AMP {e_amp:.3e})"


def _weights(m, z):
    t = lambda k: torch.from_numpy(np.ascontiguousarray(z[k])).to(DEV)
    with torch.no_grad():
        m.linear_query.weight.copy_(t("W_Q")); m.linear_query.bias.copy_(t("b_Q"))
        m.linear_key.weight.copy_(t("W_K"))
        m.linear_relation.weight.copy_(t("W_R")); m.linear_relation.bias.copy_(t("b_R"))


@pytest.mark.parametrize("name", ["small_sum_leaky_f32", "wide_sym_leaky_h256_f32", "long_mean_leaky_h256_f32"])
def test_eval_mode_is_identity_and_matches_golden(name):
    """eval(): dropout is the identity — bit-identical to a dropout=0 layer, and the reference's
    own conv.py outputs (golden fixture) within the layer bar."""
    z = load_case(name)
    V = next(c["V"] for c in golden_manifest() if c["name"] == name)
    agg = name.split("_")[1]
    d, H, O = z["X"].shape[1], z["W_Q"].shape[0], z["W_R"].shape[0]
    g = Graph(z["src"], z["dst"], V)
    m = SIRConv(d, H, O, nn.LeakyReLU(0.2), 0.2, agg_type=agg).to(DEV).eval()
    m0 = SIRConv(d, H, O, nn.LeakyReLU(0.2), 0, agg_type=agg).to(DEV).eval()
    _weights(m, z)
    _weights(m0, z)
    X = torch.from_numpy(z["X"]).to(DEV).requires_grad_(True)
    X0 = X.detach().clone().requires_grad_(True)
    Y, Y0 = m(g, X), m0(g, X0)
    dY = torch.from_numpy(z["dY"]).to(DEV)
    Y.backward(dY)
    Y0.backward(dY)
    assert torch.equal(Y, Y0) and torch.equal(X.grad, X0.grad)
    assert torch.equal(m.linear_key.weight.grad, m0.linear_key.weight.grad)
    d64 = lambda k: torch.from_numpy(z[k]).double()
    truth = oracle.layer_fwd_bwd(z["src"], z["dst"], V, *[d64(k) for k in ("X", "W_Q", "b_Q", "W_K", "W_R", "b_R", "dY")],
                                 agg, "leaky", 0.2)
    assert_parity(Y.detach().cpu(), z["Y"], truth["Y"], 1e-5, f"{name} eval Y", strict=True)
    assert_parity(X.grad.cpu(), z["dX"], truth["dX"], 1e-5, f"{name} eval dX")


def test_modular_path_keeps_nn_dropout():
    """The paths that do not fuse the layer (e.g. tuple features) keep the module's own nn.Dropout:
    train-mode output differs from eval, gradients are finite."""
    gen = torch.Generator().manual_seed(9)
    V, E, d, H, O = 300, 4000, 16, 256, 8
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V, (E,), generator=gen)
    X = torch.randn(V, d, generator=gen).to(DEV)
    m = SIRConv(d, H, O, nn.LeakyReLU(0.2), 0.3, agg_type="sum").to(DEV).train()
    g = Graph(src, dst, V)
    Xs = X.clone().requires_grad_(True)
    Y = m(g, (Xs, X))
    Y.sum().backward()
    assert torch.isfinite(Xs.grad).all()
    m.eval()
    with torch.no_grad():
        assert not torch.equal(m(g, (X, X)), Y.detach())


def test_device_seed_equals_host_seed():
    """A seed given as a device tensor (the graph-safe form, sir_dropout_t.seed_ptr) draws exactly the
    mask of the same value given by value — in sir_dropout_apply, the GEMM epilogue and the edge passes."""
    seed = 0x1234_5678_9ABC_DEF0
    st = torch.tensor([seed], dtype=torch.int64, device=DEV)
    V, H2 = 1000, 512
    assert torch.equal(_mask(V, H2, st, 0.3), _mask(V, H2, seed, 0.3))
    g = torch.Generator(device=DEV).manual_seed(3)
    A = torch.randn(20000, 256, device=DEV, generator=g)
    W = torch.randn(512, 256, device=DEV, generator=g) / 16
    pk = _native.gemm_pack(W)
    assert torch.equal(_native.gemm_nt(A, pk, drop=(st, 0.2)), _native.gemm_nt(A, pk, drop=(seed, 0.2)))
    assert torch.equal(_native.gemm_nt_direct(A[:3000], W, False, drop=(st, 0.2)),
                       _native.gemm_nt_direct(A[:3000], W, False, drop=(seed, 0.2)))


def test_captured_training_step_draws_a_fresh_mask_per_replay():
    """a training forward captured in a HIP graph must not replay the capture-time mask.
    The seed is drawn on the device (torch.randint, graph-safe) and read by the kernels, so two replays
    give two different masks — each one consistent between the forward and the backward (the
    gradients equal an eager step run on the replay's own mask)."""
    gen = torch.Generator().manual_seed(21)
    V, E, d, H, O, p = 600, 9000, 32, 256, 16, 0.3
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V, (E,), generator=gen)
    X, dY = torch.randn(V, d, generator=gen).to(DEV), torch.randn(V, O, generator=gen).to(DEV)
    torch.manual_seed(4)
    m = SIRConv(d, H, O, nn.LeakyReLU(0.2), p, agg_type="sum").to(DEV).train()
    g = Graph(src, dst, V)
    seeds = []
    draw = m._drop
    m._drop = lambda dev: seeds.append(draw(dev)) or seeds[-1]
    x = X.clone().requires_grad_(True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):                       # warm-up (plans, packs) outside the capture
        for _ in range(2):
            m.zero_grad(set_to_none=False)
            x.grad = None
            m(g, x).backward(dY)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    x.grad = torch.zeros_like(x)
    with torch.cuda.graph(graph):
        Y = m(g, x)
        Y.backward(dY)
    seed_t = seeds[-1][0]
    outs = []
    for _ in range(2):
        x.grad.zero_()
        graph.replay()
        torch.cuda.synchronize()
        outs.append((seed_t.clone(), Y.detach().clone(), x.grad.clone()))
    assert not torch.equal(outs[0][0], outs[1][0]), "the captured seed draw must run again on replay"
    assert not torch.equal(outs[0][1], outs[1][1]), "two replays must use two different masks"
    m._drop = lambda dev: (outs[1][0].clone(), p)   # eager step on the second replay's mask
    x2 = X.clone().requires_grad_(True)
    Y2 = m(g, x2)
    Y2.backward(dY)
    assert torch.equal(Y2, outs[1][1]) and torch.equal(x2.grad, outs[1][2])
