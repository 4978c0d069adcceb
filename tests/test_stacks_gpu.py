"""BASELINE configs 1, 2, 3 and 5 as multi-layer workloads on the HIP path (``sirgcn.workloads``),
against the same stacks built on the oracle's restated reference modules (``oracle.SIRConvRef``,
``oracle.GraphNormRef``, pinned to the reference's fixtures in test_oracle_golden.py), evaluated
in fp32 (the reference's own rounding) and fp64 (truth) with torch on the GPU — the checker only.

Tolerances: every output and gradient through ``assert_parity`` (1e-5 relative, or no worse than
twice the fp32 reference's own error against fp64, logged); the stack output h* strict at 1e-5
for the single-layer cfg1 (multi-layer stacks: envelope factor 4, errors compound over layers);
autocast (cfg2): relative L2 against fp64 within 2e-2 (bf16) / 1e-2 (fp16), or no worse
than 1.25x the reference's own AMP dataflow's error (the oracle stack under the same autocast; both
are dominated by the same half-precision GEMMs).
"""
import pytest
import torch

import oracle
from conftest import assert_parity, rel_err, tie_conditioned

from sirgcn import GraphNorm, SIRConv, _native
from sirgcn.workloads import CONFIGS, make_graph, make_inputs, make_stack

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need the MI355X box"
    _native.load()


def _run(stack, graph, X, dY, autocast=None):
    Xr = X.clone().requires_grad_(True)
    stack.zero_grad(set_to_none=True)
    if autocast is not None:
        with torch.autocast("cuda", dtype=autocast):
            Y = stack(graph, Xr)
    else:
        Y = stack(graph, Xr)
    Y.backward(dY.to(Y.dtype))
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().double().cpu() for n, p in stack.named_parameters() if p.grad is not None}
    return Y.detach().double().cpu(), Xr.grad.detach().double().cpu(), grads


def _stacks(name):
    ours = make_stack(name, SIRConv, GraphNorm).to(DEV)
    ref = make_stack(name, oracle.SIRConvRef, oracle.GraphNormRef)
    ref.load_state_dict(ours.state_dict())
    return ours, ref.to(DEV)


U32 = 2.0 ** -24


def _grad_abs_sums(stack):
    """Hooks recording sum_v |dL/dY_conv[v, :]| at every linear_relation (the terms its bias
    gradient db_R sums): the scale of an absolute rounding bound.  Only stacks with a norm after
    the conv (cfg5) have an analytically-zero db_R; elsewhere the conv output feeds an in-place
    activation, which a full backward hook does not allow."""
    sums = {}
    if stack.norms is None:
        return sums
    for i, conv in enumerate(stack.convs):
        conv.linear_relation.register_full_backward_hook(
            lambda mod, gin, gout, i=i: sums.__setitem__(f"convs.{i}.linear_relation.bias",
                                                         gout[0].detach().abs().sum(0).double().cpu()))
    return sums


class _Sites:
    """The stack's sigma' sites, as values: every conv's [Q | K] (the edge kernels' z = Q[v] + K[u])
    and every input of the between-layer activation.  ``record`` collects a run's values; ``inject``
    makes a reference stack run on given values (straight-through: the gradients still flow through
    the reference's own ops)."""

    def __init__(self, stack):
        self.stack = stack
        self.qk, self.act = [], []
        self.hooks = []

    def record_ours(self):
        import sirgcn.conv as sc
        sc.QK_TRACE = self.qk
        self.hooks.append(self.stack.activation.register_forward_pre_hook(
            lambda mod, args: self.act.append(args[0].detach().clone())))
        return self

    def _outside_convs(self):
        """The reference stack shares ONE activation module between the convs' sigma (per edge) and
        the layer loop: a flag set around every conv call tells the two apart."""
        inside = [False]
        for c in self.stack.convs:
            self.hooks.append(c.register_forward_pre_hook(lambda mod, args: inside.__setitem__(0, True)))
            self.hooks.append(c.register_forward_hook(lambda mod, args, out: inside.__setitem__(0, False)))
        return lambda: not inside[0]

    def record_ref(self):
        for c in self.stack.convs:
            c.qk_record = self.qk
        outside = self._outside_convs()

        def pre(mod, args):
            if outside():
                self.act.append(args[0].detach().clone())
        self.hooks.append(self.stack.activation.register_forward_pre_hook(pre))
        return self

    def inject(self, qk, act):
        for c, v in zip(self.stack.convs, qk):
            c.qk_inject = [v]
        vals = list(act)
        outside = self._outside_convs()

        def pre(mod, args):
            if not outside():
                return None
            x = args[0]
            v = vals.pop(0).to(device=x.device, dtype=x.dtype)
            return (x + (v - x).detach(),)
        self.hooks.append(self.stack.activation.register_forward_pre_hook(pre))
        return self

    def close(self):
        import sirgcn.conv as sc
        sc.QK_TRACE = None
        for h in self.hooks:
            h.remove()
        for c in self.stack.convs:
            if hasattr(c, "qk_record"):
                c.qk_record = c.qk_inject = None
        self.hooks = []


def _sign_flips(sites, graph):
    """(flips, flips beyond the noise) between our sigma' site values and the fp64 reference's: a
    flip is allowed where |truth| <= 4 max|ours - truth| of that site (the pre-activation lies inside
    our own fp32 error of it — a near-tie)."""
    src, dst = (torch.as_tensor(t, dtype=torch.int64).to(DEV) for t in graph.edges())
    n = bad = 0
    for kind, a_list, t_list in sites:
        for a, t in zip(a_list, t_list):
            a, t = a.to(DEV).double(), t.to(DEV).double()
            noise = (a - t).abs().max()
            if kind == "qk":           # z = Q[v] + K[u] per edge, in edge chunks
                H = a.shape[1] // 2
                for e0 in range(0, src.numel(), 1 << 20):
                    s_, d_ = src[e0:e0 + (1 << 20)], dst[e0:e0 + (1 << 20)]
                    za, zt = a[d_, :H] + a[s_, H:], t[d_, :H] + t[s_, H:]
                    f = (za > 0) != (zt > 0)
                    n += int(f.sum())
                    bad += int((f & (zt.abs() > 8 * noise)).sum())
            else:
                f = (a > 0) != (t > 0)
                n += int(f.sum())
                bad += int((f & (t.abs() > 4 * noise)).sum())
    return n, bad


def _check(name, small):
    g = make_graph(name, small=small)
    X, dY = make_inputs(name, g.num_nodes(), DEV)
    ours, ref = _stacks(name)
    so = _Sites(ours).record_ours()
    try:
        got = _run(ours, g, X, dY)
    finally:
        so.close()
    r32 = _run(ref, g, X, dY)
    ref64 = ref.double()
    gsum = _grad_abs_sums(ref64)
    sr = _Sites(ref64).record_ref()
    try:
        r64 = _run(ref64, g, X.double(), dY.double())
    finally:
        sr.close()
    n_flip, n_bad = _sign_flips([("qk", so.qk, sr.qk), ("act", so.act, sr.act)], g)
    assert n_bad == 0, f"{name}: {n_bad} of {n_flip} sigma' sign flips lie outside our own fp32 error of the site"
    if n_flip:
        # sigma' jumps at 0: a near-tie that our fp32 evaluation puts on the other side moves the
        # gradients by whole elements.  Score the gradients against the reference evaluated ON OUR
        # site values (fp64 truth and fp32 reference alike); h* stays on the unconditioned check.
        tie_conditioned(f"{name} stack", n_flip, 0.0)
        y64 = r64[0]
        ref32c = make_stack(name, oracle.SIRConvRef, oracle.GraphNormRef)
        ref32c.load_state_dict(ours.state_dict())
        ref32c = ref32c.to(DEV)
        sc32 = _Sites(ref32c).inject(so.qk, so.act)
        try:
            r32 = (r32[0],) + _run(ref32c, g, X, dY)[1:]
        finally:
            sc32.close()
        sc64 = _Sites(ref64).inject(so.qk, so.act)
        try:
            r64 = (y64,) + _run(ref64, g, X.double(), dY.double())[1:]
        finally:
            sc64.close()
    L = CONFIGS[name]["layers"]
    f = 2.0 if L == 1 else 4.0       # rounding differences compound over layers (each layer alone: 2x)
    assert_parity(got[0], r32[0], r64[0], 1e-5, f"{name} h*", strict=(L == 1), factor=f)
    assert_parity(got[1], r32[1], r64[1], 1e-5, f"{name} dX", factor=f)
    assert got[2].keys() == r64[2].keys()
    for k in got[2]:
        if k in gsum and r64[2][k].norm() <= 1e-6 * gsum[k].norm():
            # db_R behind a GraphNorm with mean_scale = 1 is analytically 0 (the norm removes any
            # per-feature constant): a relative bound is meaningless there.  Absolute bound instead:
            # the fp32 sum of V terms is within c * u * sum_v |term| (c = 64 covers the blocked
            # summation order with room; the reference's own fp32 result is held to it too).
            bound = 64 * U32 * gsum[k]
            assert torch.all((got[2][k] - r64[2][k]).abs() <= bound), \
                f"{name} d{k}: |err| {(got[2][k] - r64[2][k]).abs().max():.3e} > 64 u sum|dY| {bound.max():.3e}"
            assert torch.all((r32[2][k] - r64[2][k]).abs() <= bound)
            continue
        assert_parity(got[2][k], r32[2][k], r64[2][k], 1e-5, f"{name} d{k}", factor=f)
    return g


def test_cfg1_dictionary_lookup_seq_sigma():
    g = _check("cfg1", small=False)
    assert (g.num_nodes(), g.num_edges()) == (5120, 25600)


def test_cfg2_zinc_shaped_4_layers_fp32():
    g = _check("cfg2", small=False)
    assert 480_000 < g.num_edges() < 520_000


def test_cfg3_arxiv_shaped_3_layers_full_size():
    g = _check("cfg3", small=False)
    assert (g.num_nodes(), g.num_edges()) == (169_343, 1_166_243)


def test_cfg5_molhiv_shaped_5_layers_graphnorm():
    g = _check("cfg5", small=False)
    assert g.batch_size == 64


@pytest.mark.parametrize("dt,tol", [(torch.bfloat16, 2e-2), (torch.float16, 1e-2)], ids=["bf16", "f16"])
def test_cfg2_zinc_shaped_4_layers_autocast(dt, tol):
    """cfg2 at its BASELINE dtype: 16-bit storage kernels + autocast GEMMs vs the fp64 chain."""
    g = make_graph("cfg2")
    X, dY = make_inputs("cfg2", g.num_nodes(), DEV)
    ours, ref = _stacks("cfg2")
    seen = []
    orig = _native.edge_agg_fwd

    def spy(csr, Q, K, *a, **k):
        seen.append(Q.dtype)
        return orig(csr, Q, K, *a, **k)

    _native.edge_agg_fwd = spy
    try:
        got = _run(ours, g, X, dY, autocast=dt)
    finally:
        _native.edge_agg_fwd = orig
    assert seen == [dt] * 4, seen                      # the edge kernels ran on 16-bit rows
    amp = _run(ref, g, X, dY, autocast=dt)            # the reference's own AMP dataflow (restated)
    r64 = _run(ref.double(), g, X.double(), dY.double())
    # no worse than the reference's AMP path against fp64, or within the SURVEY §8c tolerance
    for what, a, r, t in [("h*", got[0], amp[0], r64[0]), ("dX", got[1], amp[1], r64[1])] + \
            [(k, got[2][k], amp[2][k], r64[2][k]) for k in got[2]]:
        e, e_amp = rel_err(a, t), rel_err(r, t)
        assert e <= max(tol, 1.25 * e_amp), (what, e, e_amp)


@pytest.mark.parametrize("name,autocast", [("cfg5", None), ("cfg2", None), ("cfg2", torch.bfloat16),
                                           ("cfg2", torch.float16), ("cfg3", None), ("cfg3", torch.bfloat16)])
def test_fused_norm_activation_residual_bit_identical(name, autocast, monkeypatch):
    """The stack's norm -> activation (-> + resid) as one GraphNorm kernel per direction
    (GraphNorm.forward_act: cfg5) and, without a norm, the residual + activation as one pass per
    direction (sirgcn.resact: cfg2's zinc order act(conv + h), cfg3's arxiv order act(conv) + h,
    under autocast with the 16-bit conv output) give the same bits as the separate torch steps,
    forward and every gradient."""
    import sirgcn.stacks as st
    g = make_graph(name, small=True)
    X, dY = make_inputs(name, g.num_nodes(), DEV)
    ours, _ = _stacks(name)
    for m in ours.modules():          # dropout off: the two runs must draw nothing
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    seen = []
    orig = st._resid_act
    def spy(*a):
        r = orig(*a)
        seen.append(r is not None)
        return r
    monkeypatch.setattr(st, "_resid_act", spy)
    fused = _run(ours, g, X, dY, autocast=autocast)
    assert name == "cfg5" or (seen and all(seen)), f"the fused residual pass did not run: {seen}"
    monkeypatch.setattr(GraphNorm, "forward_act", lambda self, *a, **k: None)
    monkeypatch.setattr(st, "_resid_act", lambda *a: None)
    plain = _run(ours, g, X, dY, autocast=autocast)
    assert torch.equal(fused[0], plain[0]) and torch.equal(fused[1], plain[1])
    for k in plain[2]:
        assert torch.equal(fused[2][k], plain[2][k]), k


@pytest.mark.parametrize("name,autocast", [("cfg2", None), ("cfg2", torch.bfloat16), ("cfg3", None),
                                           ("cfg3", torch.bfloat16)])
def test_residual_grad_link(name, autocast, monkeypatch):
    """The stacks without a norm (cfg2's zinc order act(conv(h) + h), cfg3's arxiv order act(conv(h)) + h)
    hand each layer's residual gradient to the previous layer's fused residual backward
    (sirgcn.resact.GradLink, D2 of sir_resid_act_bwd) instead of an autograd add: the link is used by every
    layer but the first, and the output and every gradient are the same bits as with the autograd add
    (SIRStack.link_residual_grads = False)."""
    from sirgcn.stacks import SIRStack
    g = make_graph(name, small=True)
    X, dY = make_inputs(name, g.num_nodes(), DEV)
    ours, _ = _stacks(name)
    for m in ours.modules():          # dropout off: the two runs must draw nothing
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    used = []
    orig = _native.resid_act_bwd
    monkeypatch.setattr(_native, "resid_act_bwd",
                        lambda *a, **k: used.append(k.get("D2") is not None) or orig(*a, **k))
    linked = _run(ours, g, X, dY, autocast=autocast)
    assert sorted(used) == [False] + [True] * (len(ours.convs) - 1), used
    monkeypatch.setattr(SIRStack, "link_residual_grads", False)
    plain = _run(ours, g, X, dY, autocast=autocast)
    assert torch.equal(linked[0], plain[0]) and torch.equal(linked[1], plain[1])
    for k in plain[2]:
        assert torch.equal(linked[2][k], plain[2][k]), k


@pytest.mark.parametrize("name", ["cfg1", "cfg5"])
def test_small_batches_on_the_product_gemm_route(name, monkeypatch):
    """The product's own GEMM routing (linalg.MIN_ROWS / MIN_ROWS_16 at their defaults — the suite
    lowers them to 0 elsewhere): the launch-bound batch sizes of cfg1 / cfg5 take the route the
    bench lines measure, and hold the same parity bar."""
    from sirgcn import linalg
    monkeypatch.setattr(linalg, "MIN_ROWS", linalg.DEFAULT_MIN_ROWS)
    monkeypatch.setattr(linalg, "MIN_ROWS_16", linalg.DEFAULT_MIN_ROWS_16)
    _check(name, small=False)


def test_cfg2_small_batch_autocast_on_the_product_gemm_route(monkeypatch):
    """A ZINC-shaped batch of 128 molecules (zinc/train.py:42) under bf16 autocast with the
    product's thresholds (below MIN_ROWS_16: the small-batch 16-bit route)."""
    from sirgcn import linalg
    monkeypatch.setattr(linalg, "MIN_ROWS", linalg.DEFAULT_MIN_ROWS)
    monkeypatch.setattr(linalg, "MIN_ROWS_16", linalg.DEFAULT_MIN_ROWS_16)
    from sirgcn.synth import molecule_batch
    g = molecule_batch(128, 23, seed=3)
    X, dY = make_inputs("cfg2", g.num_nodes(), DEV)
    ours, ref = _stacks("cfg2")
    got = _run(ours, g, X, dY, autocast=torch.bfloat16)
    amp = _run(ref, g, X, dY, autocast=torch.bfloat16)
    r64 = _run(ref.double(), g, X.double(), dY.double())
    for what, a, r, t in [("h*", got[0], amp[0], r64[0]), ("dX", got[1], amp[1], r64[1])] + \
            [(k, got[2][k], amp[2][k], r64[2][k]) for k in got[2]]:
        e, e_amp = rel_err(a, t), rel_err(r, t)
        assert e <= max(2e-2, 1.25 * e_amp), (what, e, e_amp)


def test_stack_draws_every_layer_dropout_seed_in_one_op(monkeypatch):
    """Training with feature dropout: the stack draws all layers' device seeds with one randint
    (one RNG launch per step, not one per layer), each layer gets its own seed, a fresh draw per
    step, and a re-seeded generator reproduces the step; the handed-in seeds are consumed."""
    g = make_graph("cfg5", small=True)
    X, dY = make_inputs("cfg5", g.num_nodes(), DEV)
    ours = make_stack("cfg5", SIRConv, GraphNorm, feat_dropout=0.2).to(DEV).train()
    calls = []
    orig = torch.randint

    def spy(*a, **k):
        out = orig(*a, **k)
        calls.append(out.numel())
        return out
    monkeypatch.setattr(torch, "randint", spy)
    torch.manual_seed(7)
    y1 = ours(g, X).detach()
    assert calls == [len(ours.convs)], calls
    assert all(c.step_seed is None for c in ours.convs)
    y2 = ours(g, X).detach()
    torch.manual_seed(7)
    y3 = ours(g, X).detach()
    assert not torch.equal(y1, y2) and torch.equal(y1, y3)
    # each layer's mask comes from its own seed: the layer outputs differ from a shared-seed run
    seen = []
    import sirgcn.conv as sc
    orig_drop = sc.SIRConv._drop
    monkeypatch.setattr(sc.SIRConv, "_drop", lambda self, dev: seen.append(orig_drop(self, dev)) or seen[-1])
    ours(g, X)
    ptrs = {d[0].data_ptr() for d in seen}
    assert len(seen) == len(ours.convs) and len(ptrs) == len(ours.convs)
