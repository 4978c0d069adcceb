"""Fused per-edge dense layer (sirgcn.edgemlp, csrc/sirconv_edgemlp.hip) against the oracle (fp32 and
fp64 evaluations of the reference dataflow, conv.py:43-47 + DGL update_all) and against the
edge-materialised native path it replaces — on random multigraphs with hub rows split into chunks
(chunk 4 / 64 / 256), isolated destinations, duplicate edges (exact max ties: first arg-max wins).
The golden-fixture cases of both forms run through the same code in test_gpu_parity.py
(test_generic_path_vs_reference_golden: small_*_seq, *_max_*)."""
import copy

import pytest
import torch
from torch import nn

import oracle
from conftest import assert_parity, tie_conditioned

from sirgcn import SIRConv, _native
from sirgcn.graph import Graph

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need the MI355X box"
    _native.load()


def _graph(seed, V=300, E=3000, dup=200):
    gen = torch.Generator().manual_seed(seed)
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V - 25, (E,), generator=gen)        # 25 isolated destinations
    dst[:500] = 7                                               # a hub row (split at every chunk tried)
    idx = torch.randint(0, E, (dup,), generator=gen)            # duplicate edges (exact max ties)
    return torch.cat([src, src[idx]]), torch.cat([dst, dst[idx]]), V, gen


def _run(m, g, X, dY, capture=None):
    """One fwd + bwd; ``capture`` (a dict) receives the layer's own QK (the projection the edge
    kernels read) and, for max, its arg edges as edge ids."""
    x = X.to(DEV).requires_grad_(True)
    m.zero_grad(set_to_none=True)
    restore = []
    if capture is not None:
        from sirgcn import edgemlp
        from sirgcn.graph import get_plan
        orig_proj, orig_fwd = m._project, edgemlp._fwd

        def proj(fk, fq):
            QK = orig_proj(fk, fq)
            capture["qk"] = QK.detach().double().cpu()
            return QK

        def fwd(*a, **k):
            out = orig_fwd(*a, **k)
            if a[-1] is not None and a[-1].dtype == torch.int32:
                pos = a[-1].long().cpu()
                eid = get_plan(g, torch.device(DEV), m.chunk).dst.eid.cpu()
                capture["arg"] = torch.where(pos >= 0, eid[pos.clamp_min(0)], torch.full_like(pos, -1))
            return out
        m._project = proj
        edgemlp._fwd = fwd
        restore = [lambda: delattr(m, "_project"), lambda: setattr(edgemlp, "_fwd", orig_fwd)]
    try:
        Y = m(g, x)
        Y.backward(dY.to(DEV))
    finally:
        for r in restore:
            r()
    torch.cuda.synchronize()
    out = {"Y": Y.detach().cpu(), "dX": x.grad.cpu()}
    out.update({n: p.grad.detach().cpu() for n, p in m.named_parameters() if p.grad is not None})
    return out


def _tie_condition(m, src, dst, V, X, act, cap, what):
    """oracle kwargs for scoring a layer whose sigma' signs or max arg edges differ from the fp64
    oracle's ONLY on near-ties (|z| or the gap within a few fp32 ulps of the values' magnitude;
    the assertion fails otherwise): the oracle is then evaluated on the kernel's own Q, K and arg
    edges (oracle.reference_cpu_step qk= / max_arg=).  {} when nothing flipped."""
    Wq, bq, Wk, Wr, br = (t.detach().cpu() for t in (m.linear_query.weight, m.linear_query.bias,
                                                     m.linear_key.weight, m.linear_relation.weight,
                                                     m.linear_relation.bias))
    n_s, w_s, bad_s = oracle.sigma_tie_flips(cap["qk"], src, dst, X, Wq, bq, Wk)
    assert bad_s == 0, f"{what}: {bad_s} sigma' sign flips beyond the fp32 rounding of z (worst {w_s:.1f} ulp-mag)"
    n_a = w_a = 0
    if "arg" in cap:
        M64, mag = oracle.max_edge_values(src, dst, X, Wq, bq, Wk, Wr, br, act, 0.2)
        n_a, w_a, bad_a = oracle.max_tie_flips(M64, mag, dst, V, cap["arg"])
        assert bad_a == 0, f"{what}: {bad_a} arg-max flips beyond fp32 rounding (worst {w_a:.1f} ulp-mag)"
    if n_s == 0 and n_a == 0:
        return {}
    tie_conditioned(what, n_s, w_s, n_a, w_a)
    kw = {"qk": cap["qk"]} if n_s else {}
    if n_a:
        kw["max_arg"] = cap["arg"]
    return kw


def _oracle(m, src, dst, V, X, dY, agg, act, dtype, **cond):
    """reference_cpu_step with m's weights, in dtype; act: kernel-activation name or a module;
    ``cond``: qk= / max_arg= (see :func:`_tie_condition`)."""
    w = [t.detach().cpu().to(dtype) for t in (m.linear_query.weight, m.linear_query.bias, m.linear_key.weight,
                                              m.linear_relation.weight, m.linear_relation.bias)]
    a = act
    if isinstance(act, nn.Module):
        a = copy.deepcopy(act).cpu().to(dtype)
        for p in a.parameters():
            p.requires_grad_(True)
    r = oracle.reference_cpu_step(src, dst, V, X.to(dtype), *w, dY.to(dtype), agg, a, 0.2, **cond)
    if isinstance(act, nn.Module):
        r["act.1.weight"] = a[1].weight.grad
        r["act.1.bias"] = a[1].bias.grad
    return r


def _no_generic(monkeypatch):
    """Make the edge-materialised path (sirgcn.generic) fail if the layer reaches it."""
    import sirgcn.generic

    def boom(*a, **k):
        raise AssertionError("generic_forward reached: the fused edge-MLP kernels should serve this shape")
    monkeypatch.setattr(sirgcn.generic, "generic_forward", boom)


@pytest.mark.parametrize("chunk", [256, 4])
@pytest.mark.parametrize("agg", ["sum", "mean", "sym"])
@pytest.mark.parametrize("H,Fo", [(64, 64), (32, 48), (16, 16), (200, 200), (128, 96), (100, 140), (256, 256)])
def test_seq_sigma_fused_vs_oracle(agg, H, Fo, chunk, monkeypatch):
    """H, F up to 256 (the DictionaryLookup sweep's nhidden = 4n reaches 200 at n = 50,
    dictionary-lookup/README.md:8) on the fused kernels — one to eight waves per block."""
    _no_generic(monkeypatch)
    src, dst, V, gen = _graph(H + Fo + len(agg))
    d, O = 24, 20
    X, dY = torch.randn(V, d, generator=gen), torch.randn(V, O, generator=gen)
    torch.manual_seed(H)
    sigma = nn.Sequential(nn.ReLU(inplace=True), nn.Linear(H, Fo), nn.ReLU(inplace=True))
    m = SIRConv(d, H, O, sigma, 0, agg_type=agg)
    m.linear_relation = nn.Linear(Fo, O)          # sigma changes the width: W_R takes Fo inputs
    m = m.to(DEV)
    m.chunk = chunk
    g = Graph(src, dst, V)
    cap = {}
    got = _run(m, g, X, dY, capture=cap)
    assert "activation.1.weight" in got
    cond = _tie_condition(m, src, dst, V, X, None, cap, f"seq {agg} H{H} F{Fo} c{chunk}")
    r32 = _oracle(m, src, dst, V, X, dY, agg, m.activation, torch.float32, **cond)
    r64 = _oracle(m, src, dst, V, X, dY, agg, m.activation, torch.float64, **cond)
    for k, kr in (("Y", "Y"), ("dX", "dX"), ("linear_query.weight", "dW_Q"), ("linear_query.bias", "db_Q"),
                  ("linear_key.weight", "dW_K"), ("linear_relation.weight", "dW_R"),
                  ("linear_relation.bias", "db_R"), ("activation.1.weight", "act.1.weight"),
                  ("activation.1.bias", "act.1.bias")):
        assert_parity(got[k], r32[kr], r64[kr], 1e-5, f"seq {agg} H{H} F{Fo} c{chunk} {k}", strict=(k == "Y"))


@pytest.mark.parametrize("chunk", [256, 64, 4])
@pytest.mark.parametrize("act", ["leaky", "relu", "gelu"])
@pytest.mark.parametrize("H,O", [(256, 40), (64, 64), (300, 24), (128, 256), (100, 200), (512, 512)])
def test_max_fused_vs_oracle_first_wins(act, H, O, chunk, monkeypatch):
    """Fused forward for H, O <= 512 (roman-empire: H = O = 512, heterophilous-datasets/README.md:8)
    and, for H, O <= 256, the fused backward (forced: the memory budget picks the edge-materialised
    one at these sizes): no [E, H] gather of edge activations is allowed."""
    from sirgcn.edgemlp import EdgeMaxLinear, max_bwd_fused
    _no_generic(monkeypatch)
    if max_bwd_fused(H, O):
        monkeypatch.setattr(EdgeMaxLinear, "fused_bwd", True)   # the budget would pick the materialised one here
        def boom(*a, **k):
            raise AssertionError("edge-materialised max backward reached")
        monkeypatch.setattr(_native, "edge_gather_add", boom)
    src, dst, V, gen = _graph(H + O + chunk)
    d = 32
    X, dY = torch.randn(V, d, generator=gen), torch.randn(V, O, generator=gen)
    torch.manual_seed(O)
    mod = {"leaky": nn.LeakyReLU(0.2), "relu": nn.ReLU(), "gelu": nn.GELU()}[act]
    m = SIRConv(d, H, O, mod, 0, agg_type="max").to(DEV)
    m.chunk = chunk
    g = Graph(src, dst, V)
    cap = {}
    got = _run(m, g, X, dY, capture=cap)
    assert torch.all(got["Y"][V - 25:] == 0)                   # isolated destinations: 0 (no bias)
    cond = _tie_condition(m, src, dst, V, X, act, cap, f"max {act} H{H} O{O} c{chunk}")
    r32 = _oracle(m, src, dst, V, X, dY, "max", act, torch.float32, **cond)
    r64 = _oracle(m, src, dst, V, X, dY, "max", act, torch.float64, **cond)
    for k, kr in (("Y", "Y"), ("dX", "dX"), ("linear_query.weight", "dW_Q"), ("linear_query.bias", "db_Q"),
                  ("linear_key.weight", "dW_K"), ("linear_relation.weight", "dW_R"),
                  ("linear_relation.bias", "db_R")):
        assert_parity(got[k], r32[kr], r64[kr], 1e-5, f"max {act} H{H} O{O} c{chunk} {k}", strict=(k == "Y"))


def test_fused_matches_edge_materialised_path():
    """Same layer, fused vs the edge-materialised native path (sirgcn.generic): max picks the same
    first arg-max edges (identical gradients routing) and both agree to fp32 rounding."""
    src, dst, V, gen = _graph(77)
    X, dY = torch.randn(V, 32, generator=gen), torch.randn(V, 48, generator=gen)
    for agg, sigma in (("max", nn.LeakyReLU(0.2)),
                       ("sum", nn.Sequential(nn.ReLU(), nn.Linear(64, 64), nn.ReLU()))):
        torch.manual_seed(5)
        m = SIRConv(32, 64, 48, sigma, 0, agg_type=agg).to(DEV)
        g = Graph(src, dst, V)
        a = _run(m, g, X, dY)
        SIRConv.fuse_edge_mlp = False
        try:
            b = _run(m, g, X, dY)
        finally:
            SIRConv.fuse_edge_mlp = True
        for k in a:
            e = (a[k] - b[k]).norm() / b[k].norm().clamp_min(1e-30)
            assert e < 1e-5, (agg, k, float(e))


def test_fused_max_s1_scale_fits_and_is_deterministic():
    """S1-scale max layer (V=500k, E=10M, H=O=256): runs without any [E, *] tensor in the forward,
    twice bit-identically."""
    from sirgcn.synth import powerlaw_graph
    g = powerlaw_graph(500_000, 10_000_000, 0.8, seed=0)
    torch.manual_seed(0)
    m = SIRConv(256, 256, 256, nn.LeakyReLU(0.2), 0, agg_type="max").to(DEV)
    X = torch.randn(500_000, 256, device=DEV)
    outs = []
    for _ in range(2):
        with torch.no_grad():
            outs.append(m(g, X))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert torch.isfinite(outs[0]).all()


@pytest.mark.parametrize("n", [10, 17, 50])
def test_dictionary_lookup_sweep_shapes_fused(n, monkeypatch):
    """The DictionaryLookup model at nhidden = 4n (dictionary-lookup/README.md:8, model.py:17,20:
    SIRConv(H, H, H) with sigma = Sequential(ReLU, Linear(H, H), ReLU), sum) on its own bipartite
    batch graph: fused forward and backward (no generic path) against the fp32 / fp64 oracle."""
    from sirgcn.synth import dictionary_lookup_batch
    _no_generic(monkeypatch)
    H = 4 * n
    g = dictionary_lookup_batch(n, 4)
    V = g.num_nodes()
    src, dst = g.edges()
    gen = torch.Generator().manual_seed(n)
    X, dY = torch.randn(V, H, generator=gen), torch.randn(V, H, generator=gen)
    torch.manual_seed(n)
    sigma = nn.Sequential(nn.ReLU(inplace=True), nn.Linear(H, H), nn.ReLU(inplace=True))
    m = SIRConv(H, H, H, sigma, 0, agg_type="sum").to(DEV)
    cap = {}
    got = _run(m, g, X, dY, capture=cap)
    cond = _tie_condition(m, src, dst, V, X, None, cap, f"dictionary n={n}")
    r32 = _oracle(m, src, dst, V, X, dY, "sum", m.activation, torch.float32, **cond)
    r64 = _oracle(m, src, dst, V, X, dY, "sum", m.activation, torch.float64, **cond)
    for k, kr in (("Y", "Y"), ("dX", "dX"), ("linear_query.weight", "dW_Q"), ("linear_key.weight", "dW_K"),
                  ("linear_relation.weight", "dW_R"), ("activation.1.weight", "act.1.weight"),
                  ("activation.1.bias", "act.1.bias")):
        assert_parity(got[k], r32[kr], r64[kr], 1e-5, f"dictionary n={n} {k}", strict=(k == "Y"))


@pytest.mark.parametrize("fused", [True, False])
def test_max_backward_routes_agree(fused, monkeypatch):
    """The two max backwards (fused, no [E, *] buffer / edge-materialised on the split-fp16 GEMMs)
    route dY to the same first arg-max edges: gradients agree to fp32 rounding."""
    from sirgcn.edgemlp import EdgeMaxLinear
    src, dst, V, gen = _graph(91)
    X, dY = torch.randn(V, 32, generator=gen), torch.randn(V, 96, generator=gen)
    torch.manual_seed(9)
    m = SIRConv(32, 128, 96, nn.LeakyReLU(0.2), 0, agg_type="max").to(DEV)
    g = Graph(src, dst, V)
    monkeypatch.setattr(EdgeMaxLinear, "fused_bwd", fused)
    a = _run(m, g, X, dY)
    monkeypatch.setattr(EdgeMaxLinear, "fused_bwd", not fused)
    b = _run(m, g, X, dY)
    for k in a:
        e = (a[k] - b[k]).norm() / b[k].norm().clamp_min(1e-30)
        assert e < 1e-5, (k, float(e))


@pytest.mark.parametrize("act,slope", [(_native.ACT_RELU, 0.0), (_native.ACT_LEAKY, 0.2), (_native.ACT_IDENTITY, 0.0)])
@pytest.mark.parametrize("H", [256, 37])
def test_edge_gather_act_bit_exact(act, slope, H):
    """sir_edge_gather_act: A[e] = act(Q[v] + K[u]) in dst-CSR edge order equals torch's own ops on the
    gathered sum bit for bit (the materialised max backward reads sigma' off A)."""
    from sirgcn.graph import get_plan
    src, dst, V, gen = _graph(11)
    plan = get_plan(Graph(src, dst, V), torch.device(DEV))
    QK = torch.randn(V, 2 * H, generator=gen).to(DEV)
    E = plan.dst.col.numel()
    A = torch.empty(E, H, device=DEV)
    smask = torch.empty(E, 4, device=DEV, dtype=torch.int64) if H == 256 else None
    _native.edge_gather_act(plan.dst, QK[:, :H], QK[:, H:], act, slope, A, sign_mask=smask)
    rows = torch.repeat_interleave(torch.arange(V, device=DEV), (plan.dst.rowptr[1:] - plan.dst.rowptr[:-1]).long())
    z = QK[rows, :H] + QK[plan.dst.col.long(), H:]
    ref = {_native.ACT_RELU: torch.relu, _native.ACT_LEAKY: lambda t: torch.nn.functional.leaky_relu(t, slope),
           _native.ACT_IDENTITY: lambda t: t}[act](z)
    assert torch.equal(A, ref)
    if smask is not None:                   # bit l of word x = A[e][4 l + x] > 0
        assert torch.equal(smask, sign_words(ref))


def sign_words(A):
    """int64 [E, 4]: bit l of word x = A[:, 4 l + x] > 0 (sir_edge_gather_act's sign mask, H = 256)."""
    bits = (A > 0).reshape(A.shape[0], 64, 4).permute(0, 2, 1).long()
    return (bits << torch.arange(64, device=A.device)).sum(-1)


@pytest.mark.parametrize("fused", [True, False])
def test_max_negative_slope_leaky_both_backwards(fused, monkeypatch):
    """a LeakyReLU with a negative slope flips the sign (z < 0 gives sigma(z) = slope z > 0),
    so sigma' must come from z, not from the activation: both max backwards against the oracle."""
    from sirgcn.edgemlp import EdgeMaxLinear
    src, dst, V, gen = _graph(101)
    X, dY = torch.randn(V, 32, generator=gen), torch.randn(V, 96, generator=gen)
    torch.manual_seed(11)
    m = SIRConv(32, 128, 96, nn.LeakyReLU(-0.2), 0, agg_type="max").to(DEV)
    monkeypatch.setattr(EdgeMaxLinear, "fused_bwd", fused)
    got = _run(m, Graph(src, dst, V), X, dY)
    w = [t.detach().cpu() for t in (m.linear_query.weight, m.linear_query.bias, m.linear_key.weight,
                                    m.linear_relation.weight, m.linear_relation.bias)]
    r32 = oracle.reference_cpu_step(src, dst, V, X, *w, dY, "max", "leaky", -0.2)
    r64 = oracle.reference_cpu_step(src, dst, V, X.double(), *[t.double() for t in w], dY.double(), "max", "leaky",
                                    -0.2)
    for k, kr in (("Y", "Y"), ("dX", "dX"), ("linear_query.weight", "dW_Q"), ("linear_key.weight", "dW_K"),
                  ("linear_relation.weight", "dW_R"), ("linear_relation.bias", "db_R")):
        assert_parity(got[k], r32[kr], r64[kr], 1e-5, f"max leaky(-0.2) fused={fused} {k}", strict=(k == "Y"))


def test_max_backward_row_ranges_match_whole_graph(monkeypatch):
    """Over budget, the edge-materialised max backward runs over destination-row ranges (the S2 shape):
    each range a rebased sub-graph, dW_R / db_R / dK summed over the ranges in order.  dQ rows are
    summed inside one range in the whole graph's order (bit-identical); the rest within fp32 rounding."""
    from sirgcn import edgemlp
    from sirgcn.edgemlp import EdgeMaxLinear
    src, dst, V, gen = _graph(131)
    X, dY = torch.randn(V, 32, generator=gen), torch.randn(V, 256, generator=gen)
    torch.manual_seed(13)
    m = SIRConv(32, 256, 256, nn.LeakyReLU(0.2), 0, agg_type="max").to(DEV)
    g = Graph(src, dst, V)
    monkeypatch.setattr(EdgeMaxLinear, "fused_bwd", None)
    monkeypatch.setattr(EdgeMaxLinear, "sparse_bwd", False)
    monkeypatch.setattr(EdgeMaxLinear, "hybrid_bwd", False)     # the edge-materialised route under test
    whole = _run(m, g, X, dY)
    calls = []
    orig = edgemlp._max_bwd_ranges
    monkeypatch.setattr(edgemlp, "_max_bwd_ranges", lambda *a: calls.append(a[-1]) or orig(*a[:-1], 3000))
    monkeypatch.setattr(EdgeMaxLinear, "materialised_budget", 1 << 20)     # 1 MiB: forces the ranges
    ranged = _run(m, g, X, dY)
    assert calls, "the row-range route was not taken"
    assert torch.equal(ranged["Y"], whole["Y"])
    for k in whole:
        e = float((ranged[k].double() - whole[k].double()).norm() / whole[k].double().norm().clamp_min(1e-30))
        assert e < 1e-6, (k, e)


def _no_edge_buffers(monkeypatch):
    """Make every edge-materialised / fused max backward fail if the layer reaches it."""
    from sirgcn import edgemlp

    def boom(*a, **k):
        raise AssertionError("a max backward other than the routed one was reached")
    for name in ("_max_bwd_materialised", "_max_bwd_fused", "_max_bwd_ranges"):
        monkeypatch.setattr(edgemlp, name, boom)


@pytest.mark.parametrize("chunk", [256, 64, 4])
@pytest.mark.parametrize("act", ["leaky", "relu", "gelu"])
@pytest.mark.parametrize("H,O", [(256, 256), (256, 40), (64, 64), (300, 24), (128, 256), (100, 200), (512, 256),
                                 (4, 1)])
def test_max_routed_backward_vs_oracle_first_wins(act, H, O, chunk, monkeypatch):
    """The routed max backward (sir_edge_max_bwd_sparse, opt-in for H % 4 == 0, H <= 512, O <= 256):
    dY reaches each (v, o)'s first arg-max edge only, dA from the routed W_R rows, no [E, *] buffer —
    against the fp32 / fp64 oracle on hub rows split at every chunk, isolated rows, exact ties."""
    from sirgcn.edgemlp import EdgeMaxLinear
    _no_generic(monkeypatch)
    _no_edge_buffers(monkeypatch)
    monkeypatch.setattr(EdgeMaxLinear, "fused_bwd", None)
    monkeypatch.setattr(EdgeMaxLinear, "sparse_bwd", True)
    src, dst, V, gen = _graph(3 * H + O + chunk)
    d = 32
    X, dY = torch.randn(V, d, generator=gen), torch.randn(V, O, generator=gen)
    torch.manual_seed(O + 1)
    mod = {"leaky": nn.LeakyReLU(0.2), "relu": nn.ReLU(), "gelu": nn.GELU()}[act]
    m = SIRConv(d, H, O, mod, 0, agg_type="max").to(DEV)
    m.chunk = chunk
    g = Graph(src, dst, V)
    cap = {}
    got = _run(m, g, X, dY, capture=cap)
    cond = _tie_condition(m, src, dst, V, X, act, cap, f"max routed {act} H{H} O{O} c{chunk}")
    r32 = _oracle(m, src, dst, V, X, dY, "max", act, torch.float32, **cond)
    r64 = _oracle(m, src, dst, V, X, dY, "max", act, torch.float64, **cond)
    for k, kr in (("Y", "Y"), ("dX", "dX"), ("linear_query.weight", "dW_Q"), ("linear_query.bias", "db_Q"),
                  ("linear_key.weight", "dW_K"), ("linear_relation.weight", "dW_R"),
                  ("linear_relation.bias", "db_R")):
        assert_parity(got[k], r32[kr], r64[kr], 1e-5, f"max routed {act} H{H} O{O} c{chunk} {k}", strict=(k == "Y"))


@pytest.mark.parametrize("other", [True, False])
def test_max_routed_backward_agrees_with_other_routes(other, monkeypatch):
    """Routed vs fused (True) / edge-materialised (False) max backward: the same first arg-max routing,
    gradients agree to fp32 rounding; the routed one is bit-identical run to run."""
    from sirgcn.edgemlp import EdgeMaxLinear
    src, dst, V, gen = _graph(97)
    X, dY = torch.randn(V, 32, generator=gen), torch.randn(V, 96, generator=gen)
    torch.manual_seed(19)
    m = SIRConv(32, 128, 96, nn.LeakyReLU(0.2), 0, agg_type="max").to(DEV)
    g = Graph(src, dst, V)
    monkeypatch.setattr(EdgeMaxLinear, "fused_bwd", None)
    monkeypatch.setattr(EdgeMaxLinear, "sparse_bwd", True)
    a = _run(m, g, X, dY)
    a2 = _run(m, g, X, dY)
    for k in a:
        assert torch.equal(a[k], a2[k]), k
    monkeypatch.setattr(EdgeMaxLinear, "fused_bwd", other)
    b = _run(m, g, X, dY)
    for k in a:
        e = (a[k] - b[k]).norm() / b[k].norm().clamp_min(1e-30)
        assert e < 1e-5, (k, float(e))


def test_max_routed_backward_s1_scale_deterministic_without_edge_buffers(monkeypatch):
    """S1-scale max layer (V=500k, E=10M, H=O=256) through the routed backward: twice bit-identically,
    with the backward's peak memory far below one [E, H] fp32 buffer (10 GB): no edge-sized tensor."""
    from sirgcn.edgemlp import EdgeMaxLinear
    from sirgcn.synth import powerlaw_graph
    _no_edge_buffers(monkeypatch)
    monkeypatch.setattr(EdgeMaxLinear, "fused_bwd", None)
    monkeypatch.setattr(EdgeMaxLinear, "sparse_bwd", True)
    V, E, H = 500_000, 10_000_000, 256
    g = powerlaw_graph(V, E, 0.8, seed=1)
    torch.manual_seed(2)
    m = SIRConv(H, H, H, nn.LeakyReLU(0.2), 0, agg_type="max").to(DEV)
    gen = torch.Generator(device=DEV).manual_seed(3)
    X = torch.randn(V, H, device=DEV, generator=gen).requires_grad_(True)
    dY = torch.randn(V, H, device=DEV, generator=gen)
    grads = []
    for _ in range(2):
        X.grad = None
        m.zero_grad(set_to_none=True)
        Y = m(g, X)
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        Y.backward(dY)
        torch.cuda.synchronize()
        peak = torch.cuda.max_memory_allocated() - base
        assert peak < E * H * 4 // 2, f"backward peak {peak / 2**30:.2f} GiB: an edge-sized buffer?"
        grads.append([X.grad.clone()] + [p.grad.clone() for p in m.parameters()])
        del Y
    for a, b in zip(*grads):
        assert torch.equal(a, b)
        assert torch.isfinite(a).all()


@pytest.mark.parametrize("chunk", [256, 4])
@pytest.mark.parametrize("H,O", [(256, 256), (128, 96), (300, 24), (64, 1), (512, 256)])
def test_max_dw_rows_matches_tn_gemm(H, O, chunk, monkeypatch):
    """The materialised max backward's dW_R / db_R from A and the arg edges (sir_max_dw_rows: row batches
    staged in LDS, hub rows read from global) against the same backward on dM^T A (the TN GEMM): fp32
    rounding apart; dQ / dK untouched (bit-identical); run to run bit-identical."""
    from sirgcn.edgemlp import EdgeMaxLinear
    monkeypatch.setattr(EdgeMaxLinear, "fused_bwd", False)
    src, dst, V, gen = _graph(5 * H + O + chunk, V=700, E=9000)
    X, dY = torch.randn(V, 32, generator=gen), torch.randn(V, O, generator=gen)
    torch.manual_seed(H + O)
    m = SIRConv(32, H, O, nn.LeakyReLU(0.2), 0, agg_type="max").to(DEV)
    m.chunk = chunk
    g = Graph(src, dst, V)
    monkeypatch.setattr(EdgeMaxLinear, "dw_rows", True)
    a = _run(m, g, X, dY)
    a2 = _run(m, g, X, dY)
    monkeypatch.setattr(EdgeMaxLinear, "dw_rows", False)
    b = _run(m, g, X, dY)
    for k in a:
        assert torch.equal(a[k], a2[k]), k
        if k in ("linear_relation.weight", "linear_relation.bias"):
            e = float((a[k].double() - b[k].double()).norm() / b[k].double().norm().clamp_min(1e-30))
            assert e < 2e-6, (k, e)
        else:
            assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("dw_qk", [True, False])
@pytest.mark.parametrize("act", [nn.LeakyReLU(0.2), nn.ReLU(), nn.GELU(), nn.LeakyReLU(-0.3)])
@pytest.mark.parametrize("chunk", [256, 4])
def test_max_hybrid_backward_matches_materialised(act, chunk, dw_qk, monkeypatch):
    """The default max backward when it fits (A materialised for dW_R via sir_max_dw_rows, dQ / dK from the
    routed passes: no dM, no dZ buffer) against the edge-materialised one: fp32 rounding apart, and
    bit-identical run to run."""
    from sirgcn import edgemlp
    from sirgcn.edgemlp import EdgeMaxLinear
    calls = []
    orig = edgemlp._max_bwd_hybrid
    monkeypatch.setattr(edgemlp, "_max_bwd_hybrid", lambda *a: calls.append(1) or orig(*a))
    monkeypatch.setattr(EdgeMaxLinear, "dw_qk", dw_qk)
    src, dst, V, gen = _graph(211 + chunk, V=700, E=9000)
    X, dY = torch.randn(V, 32, generator=gen), torch.randn(V, 96, generator=gen)
    torch.manual_seed(23)
    m = SIRConv(32, 128, 96, act, 0, agg_type="max").to(DEV)
    m.chunk = chunk
    g = Graph(src, dst, V)
    monkeypatch.setattr(EdgeMaxLinear, "fused_bwd", None)
    a = _run(m, g, X, dY)
    a2 = _run(m, g, X, dY)
    assert calls, "the hybrid route was not taken"
    monkeypatch.setattr(EdgeMaxLinear, "fused_bwd", False)
    b = _run(m, g, X, dY)
    for k in a:
        assert torch.equal(a[k], a2[k]), k
        e = float((a[k].double() - b[k].double()).norm() / b[k].double().norm().clamp_min(1e-30))
        assert e < 2e-6, (k, e)


@pytest.mark.parametrize("V", [0, 37])
def test_max_default_backward_empty_graph_zero_weight_grads(V):
    """A graph without edges (an empty batch, an edge-cut rank with no rows) through the DEFAULT max
    backward (the hybrid route, dW_R with Q / K recomputed): every partial the weight gradients are
    summed from is written as zeros (advisor r05: the V == 0 partial was left unset), so dW_R / db_R and
    every other gradient are exactly 0 — checked on a caching allocator primed with NaN blocks."""
    from sirgcn.edgemlp import EdgeMaxLinear
    assert EdgeMaxLinear.fused_bwd is None and EdgeMaxLinear.hybrid_bwd and EdgeMaxLinear.dw_qk
    junk = [torch.full((1 << 16,) if i % 2 else (1 << 18,), float("nan"), device=DEV) for i in range(64)]
    del junk
    src = dst = torch.zeros(0, dtype=torch.int64)
    torch.manual_seed(3)
    m = SIRConv(32, 256, 256, nn.LeakyReLU(0.2), 0, agg_type="max").to(DEV)
    X = torch.randn(V, 32, device=DEV).requires_grad_(True)
    Y = m(Graph(src, dst, V), X)
    Y.backward(torch.randn(V, 256, device=DEV))
    assert Y.shape == (V, 256) and torch.equal(Y, torch.zeros_like(Y))
    assert torch.equal(X.grad, torch.zeros_like(X))
    for n, p in m.named_parameters():
        assert p.grad is not None and torch.equal(p.grad, torch.zeros_like(p)), n
