"""Pin the CPU oracle against the golden vectors produced by the reference's own conv.py.

CPU-only (no GPU): every golden case is re-derived by the oracle and compared.
"""
import numpy as np
import pytest
import torch

import oracle
from conftest import assert_close, golden_manifest, load_case

CASES = golden_manifest()
KERNEL_CASES = [c for c in CASES if c["agg"] in oracle.AGGS and c["act"] in oracle.ACTS]


def _t(x):
    return torch.from_numpy(np.ascontiguousarray(x))


@pytest.mark.parametrize("case", KERNEL_CASES, ids=[c["name"] for c in KERNEL_CASES])
def test_edge_agg_fwd_matches_reference(case):
    z = load_case(case["name"])
    S = oracle.edge_agg_fwd(z["src"], z["dst"], case["V"], _t(z["Q"]), _t(z["K"]),
                            case["agg"], case["act"], case["slope"])
    if case["act"] in ("relu", "leaky") and case["dtype"] == "float32":
        # same op order as the DGL edge-UDF path -> bit-exact
        assert torch.equal(S, _t(z["S"])), case["name"]
    else:
        assert_close(S, z["S"], 1e-6 if case["dtype"] == "float64" else 1e-6, case["name"])


@pytest.mark.parametrize("case", KERNEL_CASES, ids=[c["name"] for c in KERNEL_CASES])
def test_edge_agg_bwd_matches_reference(case):
    z = load_case(case["name"])
    dQ, dK = oracle.edge_agg_bwd(z["src"], z["dst"], case["V"], _t(z["Q"]), _t(z["K"]), _t(z["dS"]),
                                 case["agg"], case["act"], case["slope"])
    if case["act"] in ("relu", "leaky") and case["dtype"] == "float32":
        assert torch.equal(dQ, _t(z["dQ"])), case["name"]
        assert torch.equal(dK, _t(z["dK"])), case["name"]
    else:
        assert_close(dQ, z["dQ"], 1e-6, case["name"] + " dQ")
        assert_close(dK, z["dK"], 1e-6, case["name"] + " dK")


@pytest.mark.parametrize("case", KERNEL_CASES, ids=[c["name"] for c in KERNEL_CASES])
def test_layer_matches_reference(case):
    z = load_case(case["name"])
    args = [_t(z[k]) for k in ("X", "W_Q", "b_Q", "W_K", "W_R", "b_R", "dY")]
    out = oracle.layer_fwd_bwd(z["src"], z["dst"], case["V"], *args, case["agg"], case["act"], case["slope"])
    ref = oracle.reference_cpu_step(z["src"], z["dst"], case["V"], *args, case["agg"], case["act"], case["slope"])
    tol = 1e-12 if case["dtype"] == "float64" else 1e-5
    if case["dtype"] == "float64" and case["agg"] == "sym":
        tol = 1e-6   # reference norms are fp32 even in an fp64 model (conv.py:51-52)
    for key in ("Y", "dX", "dW_Q", "db_Q", "dW_K", "dW_R", "db_R"):
        assert_close(out[key], z[key], tol, f"{case['name']} {key} (analytic)")
        assert_close(ref[key], z[key], tol, f"{case['name']} {key} (autograd port)")


def test_csr_oracle_is_stable_by_edge_id():
    z = load_case("small_sum_leaky_f32")
    V = 64
    rowptr, col, eid = oracle.csr_by_dst(z["src"], z["dst"], V)
    assert rowptr[-1] == z["src"].size
    assert np.array_equal(np.diff(rowptr), z["in_deg"])
    for v in range(V):
        seg = eid[rowptr[v]:rowptr[v + 1]]
        assert np.all(np.diff(seg) > 0)
        assert np.all(z["dst"][seg] == v)
        assert np.array_equal(col[rowptr[v]:rowptr[v + 1]], z["src"][seg])
    rowptr_s, col_s, eid_s = oracle.csr_by_src(z["src"], z["dst"], V)
    assert np.array_equal(np.diff(rowptr_s), z["out_deg"])


def test_degree_norms_match_reference_shapes():
    z = load_case("small_sym_leaky_f32")
    in_norm, out_norm = oracle.degree_norms(z["in_deg"], z["out_deg"], "sym")
    assert in_norm.dtype == torch.float32 and out_norm.dtype == torch.float32
    # isolated destinations clamp to degree 1 -> norm 1 (conv.py:51)
    assert torch.all(in_norm[torch.from_numpy(z["in_deg"]) == 0] == 1.0)


def test_isolated_nodes_output_bias():
    """Appendix A.6: sum/mean/sym -> isolated destination outputs b_R."""
    z = load_case("empty_sum_leaky_f32")
    assert np.array_equal(z["Y"], np.broadcast_to(z["b_R"], z["Y"].shape))


# ------------------------------------------------------------------ max / sigma callables
def _act_from_case(case, z, dtype=None):
    from torch import nn
    if case["act"] == "tanh":
        return nn.Tanh()
    if case["act"] == "seq":
        lin = nn.Linear(case["H"], case["H"])
        with torch.no_grad():
            lin.weight.copy_(_t(z["act_W"])); lin.bias.copy_(_t(z["act_b"]))
        seq = nn.Sequential(nn.ReLU(), lin, nn.ReLU())
        return seq.to(dtype) if dtype is not None else seq
    return case["act"]


GENERIC = [c for c in CASES if c["agg"] == "max" or c["act"] in ("seq", "tanh")]


@pytest.mark.parametrize("case", GENERIC, ids=[c["name"] for c in GENERIC])
def test_generic_layer_matches_reference(case):
    """max (DGL first-arg-max) and sigma callables through the oracle's general UDF dataflow."""
    z = load_case(case["name"])
    args = [_t(z[k]) for k in ("X", "W_Q", "b_Q", "W_K", "W_R", "b_R", "dY")]
    act = _act_from_case(case, z)
    ref = oracle.reference_cpu_step(z["src"], z["dst"], case["V"], *args, case["agg"], act, case["slope"])
    assert_close(ref["Y"], z["Y"], 1e-5, f"{case['name']} Y")
    ties_possible = case["agg"] == "max" and not case["name"].startswith("nodup")
    if ties_possible:
        return      # duplicate edges tie in max: the shim splits tie gradients, DGL gives them to the first
    for key in ("dX", "dW_Q", "db_Q", "dW_K", "dW_R", "db_R"):
        assert_close(ref[key], z[key], 1e-5, f"{case['name']} {key}")


def test_max_first_wins_semantics():
    M = torch.tensor([[1.0, 5.0], [3.0, 5.0], [3.0, 0.0]])
    dst = torch.tensor([0, 0, 0])
    Y, arg = oracle.max_first_wins(dst, 2, M)
    assert Y.tolist() == [[3.0, 5.0], [0.0, 0.0]]
    assert arg.tolist() == [[1, 0], [-1, -1]]           # ties -> earliest edge; empty row -> -1


# ------------------------------------------------------------------ GraphNorm (models/norm.py:7-29)
GN = golden_manifest("graphnorm")


@pytest.mark.parametrize("case", GN, ids=[c["name"] for c in GN])
def test_graph_norm_oracle_matches_reference(case):
    z = load_case(case["name"])
    f = lambda k: _t(z[k]) if k in z else None
    Y, mean, std = oracle.graph_norm_fwd(f("X"), z["batch_num_nodes"], f("weight"), f("bias"), f("mean_scale"))
    assert torch.equal(Y, f("Y")), case["name"]           # same op order as the reference: bit-exact
    dX, dw, db, dms = oracle.graph_norm_bwd(f("X").double(), f("dY").double(), z["batch_num_nodes"],
                                            f("weight").double(),
                                            f("mean_scale").double() if "mean_scale" in z else None,
                                            mean.double(), std.double())
    assert_close(dX, z["dX"], 1e-5, "dX")
    assert_close(dw, z["dweight"], 1e-5, "dweight")
    if "dbias" in z:
        assert_close(db, z["dbias"], 1e-5, "dbias")
    if "dmean_scale" in z:   # a cancelling sum over graphs: the fp32 fixture is ~1e-6 off fp64 elementwise
        from conftest import rel_err
        assert rel_err(dms, z["dmean_scale"]) < 1e-5


# ------------------------------------------------------------------ SIREConv (models/conv.py:70-134)
SIRE = golden_manifest("sire")


@pytest.mark.parametrize("case", SIRE, ids=[c["name"] for c in SIRE])
def test_sire_oracle_matches_reference(case):
    z = load_case(case["name"])
    args = [_t(z[k]) for k in ("X", "efeat", "W_Q", "b_Q", "W_K", "W_E", "W_R", "b_R", "dY")]
    act = _act_from_case(case, z)
    ref = oracle.sire_reference_step(z["src"], z["dst"], case["V"], *args, case["agg"], act, case["slope"])
    tol = 1e-12 if case["dtype"] == "float64" else 1e-5
    for key in ("Y", "dX", "defeat", "dW_Q", "db_Q", "dW_K", "dW_E", "dW_R", "db_R"):
        assert_close(ref[key], z[key], tol, f"{case['name']} {key}")


# ------------------------------------------------------------------ differentiable oracle modules
def _oracle_act_module(case, z, dtype):
    from torch import nn
    a = _act_from_case(case, z, dtype)
    if not isinstance(a, str):
        return a
    return {"relu": nn.ReLU(), "leaky": nn.LeakyReLU(0.2), "gelu": nn.GELU()}[a]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_conv_module_matches_reference(case):
    """oracle.SIRConvRef (the chainable restatement used by the stack tests) vs every fixture."""
    from sirgcn.graph import Graph
    z = load_case(case["name"])
    dt = torch.float64 if case["dtype"] == "float64" else torch.float32
    m = oracle.SIRConvRef(case["d"], case["H"], case["O"], _oracle_act_module(case, z, dt), 0,
                          agg_type=case["agg"]).to(dt)
    with torch.no_grad():
        for mod, wk, bk in ((m.linear_query, "W_Q", "b_Q"), (m.linear_key, "W_K", None),
                            (m.linear_relation, "W_R", "b_R")):
            mod.weight.copy_(_t(z[wk]))
            if bk:
                mod.bias.copy_(_t(z[bk]))
    X = _t(z["X"]).requires_grad_(True)
    Y = m(Graph(_t(z["src"]).long(), _t(z["dst"]).long(), case["V"]), X)
    Y.backward(_t(z["dY"]))
    tol = 1e-12 if dt == torch.float64 else 1e-5
    if dt == torch.float64 and case["agg"] == "sym":
        tol = 1e-6
    assert_close(Y.detach(), z["Y"], tol, f"{case['name']} Y")
    if case["agg"] == "max" and not case["name"].startswith("nodup"):
        return      # tie gradients: see test_generic_layer_matches_reference
    for key, got in (("dX", X.grad), ("dW_Q", m.linear_query.weight.grad), ("db_Q", m.linear_query.bias.grad),
                     ("dW_K", m.linear_key.weight.grad), ("dW_R", m.linear_relation.weight.grad),
                     ("db_R", m.linear_relation.bias.grad)):
        assert_close(got, z[key], tol, f"{case['name']} {key}")


@pytest.mark.parametrize("case", GN, ids=[c["name"] for c in GN])
def test_oracle_graphnorm_module_matches_reference(case):
    from sirgcn.graph import Graph
    z = load_case(case["name"])
    n = int(z["batch_num_nodes"].sum())
    g = Graph(torch.zeros(0, dtype=torch.int64), torch.zeros(0, dtype=torch.int64), n, z["batch_num_nodes"])
    gn = oracle.GraphNormRef(case["F"], bias=case["bias"], mean_scale=case["mean_scale"])
    with torch.no_grad():
        gn.weight.copy_(_t(z["weight"]))
        if case["bias"]:
            gn.bias.copy_(_t(z["bias"]))
        if case["mean_scale"]:
            gn.mean_scale.copy_(_t(z["mean_scale"]))
    X = _t(z["X"]).requires_grad_(True)
    Y = gn(g, X)
    Y.backward(_t(z["dY"]))
    assert_close(Y.detach(), z["Y"], 1e-6, "Y")
    assert_close(X.grad, z["dX"], 1e-5, "dX")
    assert_close(gn.weight.grad, z["dweight"], 1e-5, "dweight")
