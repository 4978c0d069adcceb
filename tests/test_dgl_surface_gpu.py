"""The rest of the reference's forward surface:

* a real ``DGLGraph`` is consumed through ``adj_tensors('csc')`` (``graph.py`` GraphPlan ``csc=``
  branch) — here a duck-typed stand-in with DGL 2.1.0's return convention (indptr, indices = source
  ids in CSC order, eids), ``in_degrees`` / ``out_degrees`` / ``num_nodes`` / ``edges``;
* ``forward(graph, (feat_src, feat_dst))`` — the tuple that ``expand_as_pair`` passes through
  (``conv.py:59``): keys from the source features, queries from the destination features;
* ``dropout > 0`` (``conv.py:35,60-61``) on the modular path: independent masks on Q and K in train
  mode, identity in eval mode (the fused layer's own dropout: ``tests/test_dropout_gpu.py``).
"""
import numpy as np
import pytest
import torch
from torch import nn

import oracle
from conftest import assert_close, assert_parity, golden_manifest, load_case

from sirgcn import SIRConv, _native
from sirgcn.graph import Graph, get_plan

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need the MI355X box"
    _native.load()


class DuckDGLGraph:
    """The DGLGraph methods SIRConv touches, with DGL 2.1.0 conventions."""

    def __init__(self, src, dst, n):
        self._src = torch.as_tensor(src, dtype=torch.int64)
        self._dst = torch.as_tensor(dst, dtype=torch.int64)
        self._n = n
        self.csc_calls = 0

    def num_nodes(self):
        return self._n

    def edges(self):
        return self._src, self._dst

    def in_degrees(self):
        return torch.bincount(self._dst, minlength=self._n)

    def out_degrees(self):
        return torch.bincount(self._src, minlength=self._n)

    def adj_tensors(self, fmt):
        assert fmt == "csc"
        self.csc_calls += 1
        eids = torch.sort(self._dst, stable=True)[1]           # DGL: stable counting sort by dst
        indptr = torch.zeros(self._n + 1, dtype=torch.int64)
        torch.cumsum(self.in_degrees(), 0, out=indptr[1:])
        return indptr, self._src[eids], eids


def _weights(m, z):
    t = lambda k: torch.from_numpy(np.ascontiguousarray(z[k])).to(DEV)
    with torch.no_grad():
        m.linear_query.weight.copy_(t("W_Q")); m.linear_query.bias.copy_(t("b_Q"))
        m.linear_key.weight.copy_(t("W_K"))
        m.linear_relation.weight.copy_(t("W_R")); m.linear_relation.bias.copy_(t("b_R"))


@pytest.mark.parametrize("name", ["small_sym_leaky_f32", "long_mean_leaky_h256_f32", "wide_sum_leaky_h256_f32"])
def test_dgl_csc_adapter_vs_reference_golden(name):
    z = load_case(name)
    V = next(c["V"] for c in golden_manifest() if c["name"] == name)
    act = nn.LeakyReLU(0.2)
    agg = name.split("_")[1]
    d, H, O = z["X"].shape[1], z["W_Q"].shape[0], z["W_R"].shape[0]
    g = DuckDGLGraph(z["src"], z["dst"], V)
    m = SIRConv(d, H, O, act, 0, agg_type=agg).to(DEV)
    _weights(m, z)
    X = torch.from_numpy(z["X"]).to(DEV).requires_grad_(True)
    Y = m(g, X)
    Y.backward(torch.from_numpy(z["dY"]).to(DEV))
    assert g.csc_calls == 1
    plan = get_plan(g, DEV)
    ref = get_plan(Graph(z["src"], z["dst"], V), DEV)     # the native device CSR build
    for a, b in ((plan.dst.rowptr, ref.dst.rowptr), (plan.dst.col, ref.dst.col), (plan.dst.eid, ref.dst.eid),
                 (plan.dst.items, ref.dst.items)):
        assert torch.equal(a.cpu().long(), b.cpu().long())     # DGL's CSC order, bit-exact indexing
    d64 = lambda k: torch.from_numpy(z[k]).double()
    truth = oracle.layer_fwd_bwd(z["src"], z["dst"], V, *[d64(k) for k in ("X", "W_Q", "b_Q", "W_K", "W_R", "b_R", "dY")],
                                 agg, "leaky", 0.2)
    assert_parity(Y.detach().cpu(), z["Y"], truth["Y"], 1e-5, f"{name} Y (DGL csc)", strict=True)
    assert_parity(X.grad.cpu(), z["dX"], truth["dX"], 1e-5, f"{name} dX (DGL csc)")
    assert_parity(m.linear_key.weight.grad.cpu(), z["dW_K"], truth["dW_K"], 1e-5, f"{name} dW_K (DGL csc)")


@pytest.mark.parametrize("agg", ["sum", "mean", "sym"])
def test_tuple_features_src_keys_dst_queries(agg):
    """expand_as_pair((feat_src, feat_dst)): K = W_K feat_src, Q = W_Q feat_dst + b_Q (conv.py:59-61)."""
    gen = torch.Generator().manual_seed(5)
    V, E, d, H, O = 200, 3000, 24, 256, 16
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V, (E,), generator=gen)
    Xs, Xd, dY = torch.randn(V, d, generator=gen), torch.randn(V, d, generator=gen), torch.randn(V, O, generator=gen)
    torch.manual_seed(2)
    m = SIRConv(d, H, O, nn.LeakyReLU(0.2), 0, agg_type=agg).to(DEV)
    g = Graph(src, dst, V)
    xs, xd = Xs.to(DEV).requires_grad_(True), Xd.to(DEV).requires_grad_(True)
    Y = m(g, (xs, xd))
    Y.backward(dY.to(DEV))
    W = {k: getattr(m, mod).weight.detach().cpu().double() for k, mod in
         (("Q", "linear_query"), ("K", "linear_key"), ("R", "linear_relation"))}
    bq, br = m.linear_query.bias.detach().cpu().double(), m.linear_relation.bias.detach().cpu().double()
    xs64, xd64 = Xs.double().requires_grad_(True), Xd.double().requires_grad_(True)
    Q, K = xd64 @ W["Q"].t() + bq, xs64 @ W["K"].t()
    S = oracle.edge_agg_fwd(src, dst, V, Q, K, agg, "leaky", 0.2)
    Y64 = S @ W["R"].t() + br
    Y64.backward(dY.double())
    xs32, xd32 = Xs.clone().requires_grad_(True), Xd.clone().requires_grad_(True)
    w32 = lambda k: W[k].float()
    S32 = oracle.edge_agg_fwd(src, dst, V, xd32 @ w32("Q").t() + bq.float(), xs32 @ w32("K").t(), agg, "leaky", 0.2)
    Y32 = S32 @ w32("R").t() + br.float()
    Y32.backward(dY)
    assert_parity(Y.detach().cpu(), Y32.detach(), Y64.detach(), 1e-5, f"tuple {agg} Y", strict=True)
    assert_parity(xs.grad.cpu(), xs32.grad, xs64.grad, 1e-5, f"tuple {agg} dX_src")
    assert_parity(xd.grad.cpu(), xd32.grad, xd64.grad, 1e-5, f"tuple {agg} dX_dst")
    # a tuple of two equal tensors is the plain call (tuple branch vs the fused single-feature path)
    with torch.no_grad():
        assert_close(m(g, (xd.detach(), xd.detach().clone())).cpu(), m(g, xd.detach()).cpu(), 1e-5, "tuple (X, X) == X")


class _RecordingDropout(nn.Dropout):
    def forward(self, x):
        y = super().forward(x)
        self.last_in, self.last_out = x.detach(), y.detach()
        return y


def test_dropout_train_masks_and_eval_identity():
    gen = torch.Generator().manual_seed(8)
    V, E, d, H, O, p = 600, 9000, 32, 256, 32, 0.3
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V, (E,), generator=gen)
    X, dY = torch.randn(V, d, generator=gen), torch.randn(V, O, generator=gen)
    torch.manual_seed(1)
    m = SIRConv(d, H, O, nn.LeakyReLU(0.2), p, agg_type="sum").to(DEV)
    m.dropout = _RecordingDropout(p)
    m0 = SIRConv(d, H, O, nn.LeakyReLU(0.2), 0, agg_type="sum").to(DEV)
    m0.load_state_dict(m.state_dict())
    # the modular path (nn.Dropout on [Q | K]); the fused layer's hashed dropout: tests/test_dropout_gpu.py
    m.use_fused = m0.use_fused = False
    g = Graph(src, dst, V)
    Xd = X.to(DEV)
    # train mode: the dropout sees [Q | K] (V x 2H): independent Bernoulli(1-p) masks, survivors / (1-p)
    m.train()
    Y = m(g, Xd)
    qk_in, qk_out = m.dropout.last_in, m.dropout.last_out
    assert qk_in.shape == (V, 2 * H)
    kept = qk_out != 0
    frac = 1 - kept.float().mean().item()
    assert abs(frac - p) < 0.01, frac
    assert abs((1 - kept[:, :H].float().mean()).item() - p) < 0.015       # Q mask
    assert abs((1 - kept[:, H:].float().mean()).item() - p) < 0.015       # K mask
    assert torch.allclose(qk_out[kept], qk_in[kept] / (1 - p), rtol=1e-6, atol=0)
    assert not torch.equal(kept[:, :H], kept[:, H:])                      # independent masks
    # the layer output is the message passing over exactly those dropped Q, K
    S = oracle.edge_agg_fwd(src, dst, V, qk_out[:, :H].cpu().double(), qk_out[:, H:].cpu().double(), "sum", "leaky", 0.2)
    Y64 = S @ m.linear_relation.weight.detach().cpu().double().t() + m.linear_relation.bias.detach().cpu().double()
    from conftest import rel_err
    assert rel_err(Y.detach().cpu(), Y64) < 1e-5
    Y.backward(dY.to(DEV))                  # gradients flow through the dropout
    assert torch.isfinite(m.linear_key.weight.grad).all()
    # eval mode: dropout is the identity, bit-identical to a dropout=0 layer
    m.eval()
    m0.eval()
    with torch.no_grad():
        assert torch.equal(m(g, Xd), m0(g, Xd))
