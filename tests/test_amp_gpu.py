"""16-bit storage (SIR_DTYPE_BF16 / SIR_DTYPE_F16) edge kernels and the autocast path.

Kernel level: Q, K, dS are rounded to the storage dtype, the oracle evaluates the same rounded
values in fp64, and the kernels (fp32 math inside, one RNE rounding per output) must land within
two units of the storage dtype's roundoff u (bf16 2^-8, fp16 2^-11) of that truth, elementwise.
Layer level: SIRConv under ``torch.autocast`` (the reference's AMP path,
``heterophilous-datasets/train.py:75,92,106``) against the fp32 golden fixtures of the reference:
relative L2 within 2e-2 (bf16) / 1e-2 (fp16), or no worse than the reference's own AMP
dataflow (``oracle.SIRConvRef`` under the same autocast; ratio <= 1.25 — both are dominated by the
same half-precision GEMMs, the edge part here is fp32 inside).
"""
import copy
import numpy as np
import pytest
import torch
from torch import nn

import oracle
from conftest import golden_manifest, load_case, rel_err

from sirgcn import _native, linalg
from sirgcn.conv import EdgeAggregate, SIRConv, activation_code
from sirgcn.graph import Graph, GraphPlan

pytestmark = pytest.mark.gpu
DEV = "cuda"
DT = {"bf16": torch.bfloat16, "f16": torch.float16}
U = {"bf16": 2.0 ** -8, "f16": 2.0 ** -11}
ACTS = {"relu": nn.ReLU(), "leaky": nn.LeakyReLU(0.2), "gelu": nn.GELU()}
AMP_SLACK = 1.25     # allowed ratio to the reference AMP path's own error (both dominated by the same GEMMs)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need the MI355X box"
    _native.load()


def _within(got, truth, u, what):
    g = got.double().cpu()
    t = truth.double().cpu()
    bound = 2 * u * t.abs() + 1e-5 * t.abs().max()
    bad = (g - t).abs() > bound
    assert not bad.any(), f"{what}: {int(bad.sum())} elements off by more than 2u (max {(g - t).abs().max():.3e})"
    assert rel_err(g, t) <= 2 * u, (what, rel_err(g, t))


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("agg", ["sum", "mean", "sym"])
@pytest.mark.parametrize("H,act", [(256, "leaky"), (128, "relu"), (64, "gelu"), (300, "leaky"), (16, "leaky")])
def test_16bit_storage_kernels_vs_fp64(dt, agg, H, act):
    gen = torch.Generator().manual_seed(H + 3 * len(agg) + len(dt))
    V, E = 300, 2500
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V - 20, (E,), generator=gen)
    dst[:400] = 5                                            # a split row at chunk 256
    Q, K, dS = (torch.randn(V, H, generator=gen).to(DT[dt]) for _ in range(3))
    slope = 0.2 if act == "leaky" else 0.01
    S64 = oracle.edge_agg_fwd(src, dst, V, Q.double(), K.double(), agg, act, slope)
    if agg == "mean":
        # kernel contract (include/sirconv.h): in 16-bit storage the mean's g = G / deg is rounded to the
        # storage dtype (the Gm rows the src pass gathers; the reference likewise casts dm to half for
        # sigma's backward), so the truth is the plain sum over those rounded rows
        deg = torch.bincount(dst, minlength=V).clamp(min=1).float().unsqueeze(1)
        g = (dS.float() / deg).to(DT[dt]).double()
        dQ64, dK64 = oracle.edge_agg_bwd(src, dst, V, Q.double(), K.double(), g, "sum", act, slope)
    else:
        dQ64, dK64 = oracle.edge_agg_bwd(src, dst, V, Q.double(), K.double(), dS.double(), agg, act, slope)
    plan = GraphPlan(src, dst, V, DEV)
    code, sl = activation_code(ACTS[act])
    QK = torch.cat([Q, K], 1).to(DEV).requires_grad_(True)
    S = EdgeAggregate.apply(QK, plan, H, agg, code, sl)
    assert S.dtype == DT[dt]
    S.backward(dS.to(DEV))
    assert QK.grad.dtype == DT[dt]
    _within(S, S64, U[dt], "S")
    _within(QK.grad[:, :H], dQ64, U[dt], "dQ")
    _within(QK.grad[:, H:], dK64, U[dt], "dK")


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("agg", ["sum", "sym", "mean"])
def test_16bit_sign_mask_backward_bit_identical_to_recompute(dt, agg):
    gen = torch.Generator().manual_seed(7)
    V, E, H = 400, 6000, 256
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V, (E,), generator=gen)
    dst[:700] = 11
    QK = torch.randn(V, 2 * H, generator=gen).to(DEV, DT[dt])
    dS = torch.randn(V, H, generator=gen).to(DEV, DT[dt])
    plan = GraphPlan(src, dst, V, DEV)
    outs = []
    for use_mask in (True, False):
        EdgeAggregate.use_mask = use_mask
        try:
            x = QK.clone().requires_grad_(True)
            S = EdgeAggregate.apply(x, plan, H, agg, _native.ACT_LEAKY, 0.2)
            S.backward(dS)
            outs.append((S.detach(), x.grad))
        finally:
            EdgeAggregate.use_mask = True
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


CASES = [c for c in golden_manifest() if c["agg"] in ("sum", "mean", "sym") and c["dtype"] == "float32"
         and c["act"] in ("relu", "leaky", "gelu") and c["H"] % 4 == 0 and c["E"] > 0]


@pytest.mark.parametrize("native16", [False, True], ids=["route-default", "native16-every-size"])
@pytest.mark.parametrize("dt,tol", [("bf16", 2e-2), ("f16", 1e-2)])
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_sirconv_autocast_vs_reference_fp32_golden(case, dt, tol, native16, monkeypatch):
    """native16: linalg.MIN_ROWS_16 = 0, so the golden cases' small graphs run the native 16-bit NT / TN
    GEMMs (sir_gemm_nt16 for K in {128, 256, 512}, sir_gemm_tn16 for every shape) across aggs and
    dtypes, not only the large dedicated test."""
    if native16:
        from sirgcn import linalg
        monkeypatch.setattr(linalg, "MIN_ROWS_16", 0)
    z = load_case(case["name"])
    m = SIRConv(case["d"], case["H"], case["O"], ACTS[case["act"]], 0, agg_type=case["agg"]).to(DEV)
    t = lambda k: torch.from_numpy(np.ascontiguousarray(z[k])).to(DEV)
    with torch.no_grad():
        m.linear_query.weight.copy_(t("W_Q")); m.linear_query.bias.copy_(t("b_Q"))
        m.linear_key.weight.copy_(t("W_K"))
        m.linear_relation.weight.copy_(t("W_R")); m.linear_relation.bias.copy_(t("b_R"))
    g = Graph(torch.from_numpy(z["src"]), torch.from_numpy(z["dst"]), case["V"])
    X = t("X").requires_grad_(True)
    with torch.autocast("cuda", dtype=DT[dt]):
        Y = m(g, X)
    assert Y.dtype == DT[dt]                      # conv.py:65 under autocast: a half-precision linear
    Y.float().backward(t("dY"))
    got = {"Y": Y, "dX": X.grad, "dW_Q": m.linear_query.weight.grad, "db_Q": m.linear_query.bias.grad,
           "dW_K": m.linear_key.weight.grad, "dW_R": m.linear_relation.weight.grad,
           "db_R": m.linear_relation.bias.grad}
    amp = _reference_amp(case, z, DT[dt])
    for k, v in got.items():   # within tol, or comparable to the reference's own AMP dataflow (whose
        # error here is the same half-precision GEMMs': the two differ only by rounding noise)
        e, e_amp = rel_err(v.detach().float().cpu(), z[k]), rel_err(amp[k], z[k])
        assert e <= max(tol, AMP_SLACK * e_amp), f"{case['name']} {k}: relL2 {e:.3e} vs fp32 (reference AMP {e_amp:.3e})"


def _reference_amp(case, z, dt):
    """The reference's dataflow (oracle.SIRConvRef: gathers in half, sigma in half, fp32-promoted
    messages, index_add backward in half) under the same autocast, on the GPU (checker only)."""
    m = oracle.SIRConvRef(case["d"], case["H"], case["O"], ACTS[case["act"]], 0, agg_type=case["agg"]).to(DEV)
    t = lambda k: torch.from_numpy(np.ascontiguousarray(z[k])).to(DEV)
    with torch.no_grad():
        m.linear_query.weight.copy_(t("W_Q")); m.linear_query.bias.copy_(t("b_Q"))
        m.linear_key.weight.copy_(t("W_K"))
        m.linear_relation.weight.copy_(t("W_R")); m.linear_relation.bias.copy_(t("b_R"))
    g = Graph(torch.from_numpy(z["src"]), torch.from_numpy(z["dst"]), case["V"])
    X = t("X").requires_grad_(True)
    with torch.autocast("cuda", dtype=dt):
        Y = m(g, X)
    Y.float().backward(t("dY"))
    out = {"Y": Y, "dX": X.grad, "dW_Q": m.linear_query.weight.grad, "db_Q": m.linear_query.bias.grad,
           "dW_K": m.linear_key.weight.grad, "dW_R": m.linear_relation.weight.grad,
           "db_R": m.linear_relation.bias.grad}
    return {k: v.detach().float().cpu() for k, v in out.items()}


def test_amp_training_step_with_grad_scaler():
    """The heterophilous-datasets training step (train.py:75,92,106): fp16 autocast forward,
    GradScaler-scaled backward, unscale, step — gradients finite and close to fp32."""
    z = load_case("wide_sym_leaky_h256_f32")
    torch.manual_seed(0)
    m = SIRConv(64, 256, 64, nn.LeakyReLU(0.2), 0, agg_type="sym").to(DEV)
    m32 = SIRConv(64, 256, 64, nn.LeakyReLU(0.2), 0, agg_type="sym").to(DEV)
    m32.load_state_dict(m.state_dict())
    g = Graph(torch.from_numpy(z["src"]), torch.from_numpy(z["dst"]), 96)
    X = torch.from_numpy(z["X"]).to(DEV)
    dY = torch.from_numpy(z["dY"]).to(DEV)
    opt = torch.optim.SGD(m.parameters(), lr=0.0)
    scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 3)    # dW_R = dY^T S must stay inside fp16
    with torch.amp.autocast(device_type="cuda", enabled=True):
        loss = (m(g, X).float() * dY).sum()
    scaler.scale(loss).backward()
    scaler.unscale_(opt)
    (m32(g, X) * dY).sum().backward()
    mr = oracle.SIRConvRef(64, 256, 64, nn.LeakyReLU(0.2), 0, agg_type="sym").to(DEV)
    mr.load_state_dict(m32.state_dict())
    with torch.amp.autocast(device_type="cuda", enabled=True):      # the reference's AMP dataflow
        lr = (mr(g, X).float() * dY).sum()
    lr.backward()
    for (n, p), p32, pr in zip(m.named_parameters(), m32.parameters(), mr.parameters()):
        assert torch.isfinite(p.grad).all(), n
        e, e_ref = rel_err(p.grad.cpu(), p32.grad.cpu()), rel_err(pr.grad.cpu(), p32.grad.cpu())
        assert e <= max(1e-2, AMP_SLACK * e_ref), (n, e, e_ref)
    scaler.step(opt)
    scaler.update()


@pytest.mark.parametrize("dt", ["bf16", "f16"])
def test_autocast_layer_native_nt16_large(dt, monkeypatch):
    """Above linalg.MIN_ROWS_16 rows the autocast layer runs its four NT projections on the native
    16-bit kernel (X.to(dt) fused into the QK GEMM's loads, dX straight from the fp32 accumulator):
    every output and gradient within the AMP bar of the fp32 layer, and no worse than 1.25x the
    reference's own AMP dataflow (oracle.SIRConvRef under the same autocast)."""
    calls = []
    real = _native.gemm_nt16
    monkeypatch.setattr(_native, "gemm_nt16", lambda *a, **k: calls.append(1) or real(*a, **k))
    V, E, H = 20000, 200000, 256
    g = torch.Generator().manual_seed(21)
    src, dst = torch.randint(0, V, (E,), generator=g), torch.randint(0, V, (E,), generator=g)
    X = torch.randn(V, H, generator=g).to(DEV)
    dY = torch.randn(V, H, generator=g).to(DEV)
    torch.manual_seed(3)
    m = SIRConv(H, H, H, nn.LeakyReLU(0.2), 0, agg_type="sum").to(DEV)
    mr = oracle.SIRConvRef(H, H, H, nn.LeakyReLU(0.2), 0, agg_type="sum").to(DEV)
    mr.load_state_dict(m.state_dict())
    G = Graph(src, dst, V)

    def run(mod, amp):
        mod.zero_grad(set_to_none=True)
        x = X.clone().requires_grad_(True)
        if amp:
            with torch.autocast("cuda", dtype=DT[dt]):
                Y = mod(G, x)
        else:
            Y = mod(G, x)
        Y.backward(dY.to(Y.dtype))
        out = {"Y": Y, "dX": x.grad}
        out.update({n: p.grad for n, p in mod.named_parameters()})
        return {k: v.detach().double().cpu() for k, v in out.items()}

    ref32 = run(m, False)
    n0 = len(calls)
    got = run(m, True)
    assert len(calls) - n0 == 4, "QK, Y, G and dX on sir_gemm_nt16"
    amp = run(mr, True)
    tol = 2e-2 if dt == "bf16" else 1e-2
    for k, v in got.items():
        e, e_amp = rel_err(v, ref32[k]), rel_err(amp[k], ref32[k])
        assert e <= max(tol, AMP_SLACK * e_amp), f"{k}: relL2 {e:.3e} vs fp32 (reference AMP {e_amp:.3e})"


def _max16_graph(seed, V=400, E=5000):
    gen = torch.Generator().manual_seed(seed)
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V - 20, (E,), generator=gen)      # 20 isolated destinations
    dst[:600] = 5                                            # a hub row (split items / several stream blocks)
    return src, dst, V, gen


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("H,O,act", [(256, 256, "leaky"), (256, 40, "relu"), (512, 512, "leaky"), (64, 48, "relu"),
                                     (128, 200, "leaky")])
def test_max_forward_16bit_kernel_semantics(dt, H, O, act):
    """The 16-bit max forward (sir_edge_mlp_fwd_stream_st at H = 256, sir_edge_mlp_fwd_st per item otherwise)
    against its stated semantics in fp64 on the host: a = round_dt(act1(Q[v] + K[u]) in fp32) from the 16-bit
    rows, h = a round_dt(W)^T + round_dt(b), Y[v] = max_e h, arg = the first arg-max edge, empty rows 0 / -1.
    ReLU / LeakyReLU: a is bit-identical on both sides, so Y may differ only by the fp32 accumulation
    (<= 1e-5 of sum |a| |w| + |b|) and arg only where the row's two best h are closer than that."""
    from sirgcn import edgemlp
    from sirgcn.graph import get_plan
    src, dst, V, gen = _max16_graph(H + O)
    QK = (torch.randn(V, 2 * H, generator=gen) * 2).to(DT[dt]).to(DEV)
    W = (torch.randn(O, H, generator=gen) / H ** 0.5).to(DEV)
    b = torch.randn(O, generator=gen).to(DEV)
    code, slope = activation_code(ACTS[act])
    plan = get_plan(Graph(src, dst, V), torch.device(DEV))
    Y = torch.empty(V, O, device=DEV)
    arg = torch.empty(V, O, device=DEV, dtype=torch.int32)
    edgemlp._fwd_st(plan, QK[:, :H], QK[:, H:], W, b, code, slope, Y, arg)
    torch.cuda.synchronize()
    # host reference, edges in dst-CSR order (ascending edge id inside a row)
    order = torch.argsort(dst, stable=True)
    s_, d_ = src[order], dst[order]
    q, k = QK[:, :H].float().cpu(), QK[:, H:].float().cpu()
    z = q[d_] + k[s_]                                        # fp32, as the kernel
    a32 = torch.relu(z) if act == "relu" else torch.nn.functional.leaky_relu(z, slope)
    a = a32.to(DT[dt]).double()
    Wr, br = W.cpu().to(DT[dt]).double(), b.cpu().to(DT[dt]).double()
    h = a @ Wr.t() + br                                      # [E, O] fp64
    bound = 1e-5 * (a.abs() @ Wr.abs().t() + br.abs())
    Yr = torch.zeros(V, O, dtype=torch.float64)
    Ar = torch.full((V, O), -1, dtype=torch.int64)
    gap = torch.full((V, O), float("inf"), dtype=torch.float64)
    rp = torch.zeros(V + 1, dtype=torch.int64)
    rp[1:] = torch.cumsum(torch.bincount(d_, minlength=V), 0)
    for v in range(V):
        e0, e1 = int(rp[v]), int(rp[v + 1])
        if e0 == e1:
            continue
        hv = h[e0:e1]
        best, idx = hv.max(0)                                # torch.max returns the first maximal index
        Yr[v], Ar[v] = best, idx + e0
        if e1 - e0 > 1:
            top2 = hv.topk(2, dim=0).values
            gap[v] = top2[0] - top2[1]
    tol = torch.zeros(V, O, dtype=torch.float64)
    for v in range(V):
        e0, e1 = int(rp[v]), int(rp[v + 1])
        if e1 > e0:
            tol[v] = bound[e0:e1].max(0).values
    Yg, Ag = Y.double().cpu(), arg.long().cpu()
    assert ((Yg - Yr).abs() <= tol).all(), f"Y off by {(Yg - Yr).abs().max():.3e}"
    clear = gap > 2 * tol
    assert torch.equal(Ag[clear], Ar[clear]), int((Ag[clear] != Ar[clear]).sum())
    assert (Ag[rp[1:] == rp[:-1]] == -1).all()


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("H,O,act", [(256, 256, "gelu"), (512, 512, "gelu")])
def test_max_layer_under_autocast_runs_16bit_forward(dt, H, O, act, monkeypatch):
    """The reference's AMP max configs (heterophilous-datasets/README.md:8: roman-empire H = O = 512, GELU;
    amazon-ratings H = 256): SIRConv(agg_type='max') under autocast takes the 16-bit forward (16-bit Q / K
    rows, one 16-bit MFMA per product) — Y and every gradient within the AMP bar of the fp32 layer, or no
    worse than 1.25x the reference's own AMP dataflow."""
    from sirgcn import edgemlp
    calls = []
    orig = edgemlp._fwd_st
    monkeypatch.setattr(edgemlp, "_fwd_st", lambda *a: calls.append(a[0]) or orig(*a))
    src, dst, V, gen = _max16_graph(7 + H)
    d = 64
    X = torch.randn(V, d, generator=gen).to(DEV)
    dY = torch.randn(V, O, generator=gen).to(DEV)
    torch.manual_seed(9)
    m = SIRConv(d, H, O, ACTS[act], 0, agg_type="max").to(DEV)
    ref = oracle.SIRConvRef(d, H, O, ACTS[act], 0, agg_type="max").to(DEV)
    ref.load_state_dict(m.state_dict())
    g = Graph(src, dst, V)

    def run(mod, amp):
        for p in mod.parameters():
            p.grad = None
        x = X.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=DT[dt], enabled=amp):
            y = mod(g, x)
        y.float().backward(dY)
        out = {"Y": y.detach().float(), "dX": x.grad}
        out.update({n: p.grad for n, p in mod.named_parameters()})
        return {k: v.detach().float().cpu() for k, v in out.items()}

    got = run(m, True)
    assert len(calls) == 1, "the 16-bit max forward did not run"
    truth, amp = run(ref, False), run(ref, True)
    tol = 2e-2 if dt == "bf16" else 1e-2
    for k in truth:
        e, e_amp = rel_err(got[k], truth[k]), rel_err(amp[k], truth[k])
        assert e <= max(tol, AMP_SLACK * e_amp), f"max16 {k}: relL2 {e:.3e} (reference AMP {e_amp:.3e})"


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("agg,act,H,O", [("max", "gelu", 256, 256), ("max", "leaky", 128, 40),
                                         ("seq", "relu", 256, 128)])
def test_autocast_projections_native_nt16(dt, agg, act, H, O, monkeypatch):
    """The max / Sequential-sigma layers under autocast run their projections (QK = X [W_Q; W_K]^T + b,
    and linear_relation for the Sequential form) through linalg.linear's 16-bit route (_Linear16:
    sir_gemm_nt16 forward and dX, sir_gemm_tn16 weight gradients) instead of torch's bf16 GEMM plus
    casts — outputs and every gradient within the AMP bar of the fp32 layer, or no worse than 1.25x the
    reference's own AMP dataflow."""
    monkeypatch.setattr(linalg, "MIN_ROWS_16", 0)
    calls = {"nt": 0, "tn": 0}
    nt, tn = _native.gemm_nt16, _native.gemm_tn16
    monkeypatch.setattr(_native, "gemm_nt16", lambda *a, **k: calls.__setitem__("nt", calls["nt"] + 1) or nt(*a, **k))
    monkeypatch.setattr(_native, "gemm_tn16", lambda *a, **k: calls.__setitem__("tn", calls["tn"] + 1) or tn(*a, **k))
    src, dst, V, gen = _max16_graph(11 + H + O)
    d = 128
    X = torch.randn(V, d, generator=gen).to(DEV)
    dY = torch.randn(V, O, generator=gen).to(DEV)
    torch.manual_seed(5)
    if agg == "max":
        sig, kind = ACTS[act], "max"
    else:
        sig, kind = nn.Sequential(ACTS[act], nn.Linear(H, H), nn.ReLU()), "sum"
    m = SIRConv(d, H, O, sig, 0, agg_type=kind).to(DEV)
    ref = oracle.SIRConvRef(d, H, O, copy.deepcopy(sig), 0, agg_type=kind).to(DEV)
    ref.load_state_dict(m.state_dict())
    g = Graph(src, dst, V)

    def run(mod, amp):
        for p in mod.parameters():
            p.grad = None
        x = X.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=DT[dt], enabled=amp):
            y = mod(g, x)
        y.float().backward(dY)
        out = {"Y": y.detach().float(), "dX": x.grad}
        out.update({n: p.grad for n, p in mod.named_parameters()})
        return {k: v.detach().float().cpu() for k, v in out.items()}

    got = run(m, True)
    n_lin = 1 if agg == "max" else 2
    assert calls["nt"] == 2 * n_lin and calls["tn"] == n_lin, calls
    for n, p in m.named_parameters():
        assert p.grad.dtype == torch.float32, n
    truth, amp = run(ref, False), run(ref, True)
    tol = 2e-2 if dt == "bf16" else 1e-2
    for k in truth:
        e, e_amp = rel_err(got[k], truth[k]), rel_err(amp[k], truth[k])
        assert e <= max(tol, AMP_SLACK * e_amp), f"{agg} {k}: relL2 {e:.3e} (reference AMP {e_amp:.3e})"


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("form", ["max", "seq"])
def test_fused_edge_mlp_forms_under_autocast(form, dt):
    """agg='max' (conv.py:46-47, roman-empire trains it under AMP: the 16-bit forward) and the DictionaryLookup
    Sequential sigma (its per-edge Linear in fp32 even under autocast: sirgcn/edgemlp.py, a stated deviation):
    outputs and gradients within the AMP bar of the fp32 layer, or no worse than 1.25x the
    reference's own AMP dataflow (oracle.SIRConvRef under the same autocast)."""
    gen = torch.Generator().manual_seed(31 + len(dt))
    V, E, d, H, O = 300, 2400, 32, 64, 48
    src = torch.randint(0, V, (E,), generator=gen)
    dst = torch.randint(0, V - 10, (E,), generator=gen)
    dst[:300] = 4                                            # a split row
    X = torch.randn(V, d, generator=gen).to(DEV)
    dY = torch.randn(V, O, generator=gen).to(DEV)
    torch.manual_seed(5)
    if form == "max":
        act = nn.LeakyReLU(0.2)
        m = SIRConv(d, H, O, act, 0, agg_type="max").to(DEV)
    else:
        act = nn.Sequential(nn.ReLU(), nn.Linear(H, H), nn.ReLU())
        m = SIRConv(d, H, O, act, 0, agg_type="sum").to(DEV)
    ref = oracle.SIRConvRef(d, H, O, act, 0, agg_type=m._agg_type).to(DEV)
    ref.load_state_dict(m.state_dict())
    g = Graph(src, dst, V)

    def run(mod, amp):
        for p in mod.parameters():
            p.grad = None
        x = X.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=DT[dt], enabled=amp):
            y = mod(g, x)
        y.float().backward(dY)
        out = {"Y": y.detach().float(), "dX": x.grad}
        out.update({n: p.grad for n, p in mod.named_parameters()})
        return {k: v.detach().float().cpu() for k, v in out.items()}

    got, truth, amp = run(m, True), run(ref, False), run(ref, True)
    tol = 2e-2 if dt == "bf16" else 1e-2
    for k in truth:
        e, e_amp = rel_err(got[k], truth[k]), rel_err(amp[k], truth[k])
        assert e <= max(tol, AMP_SLACK * e_amp), f"{form} {k}: relL2 {e:.3e} (reference AMP {e_amp:.3e})"
