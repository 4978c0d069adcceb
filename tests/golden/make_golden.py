#!/usr/bin/env python3
"""Generate the golden SIRConv fixtures from the REFERENCE's own ``models/conv.py``.

Runs ONLY in the build container, where ``/root/reference`` (read-only) exists:

    python tests/golden/make_golden.py            # rewrites tests/golden/*.npz + manifest.json

How the reference is executed
-----------------------------
* ``/root/reference/models/conv.py`` is read as TEXT and compiled/executed from source
  (never from the reference's ``__pycache__``), with ``dgl`` resolved to the test-only
  DGL-2.1.0-semantics shim in ``tests/golden/dgl_shim`` (DGL is absent from the image; the
  shim restates ``update_all`` / ``fn.sum|mean|max`` / ``expand_as_pair``, see its docstring).
* The reference ``SIRConv`` (``conv.py:7-67``) is built exactly as callers build it
  (``SIRConv(d, H, O, activation, dropout, agg_type=...)``, e.g. ``zinc/model.py:36``), run in
  train mode with ``dropout=0``, and back-propagated with a random ``dY``.
* Hooks capture the kernel-level intermediates: Q/K (outputs of ``linear_query`` /
  ``linear_key``, ``conv.py:60-61``), S (input of ``linear_relation``, ``conv.py:65``) and
  their gradients dQ, dK, dS.

Only the produced ``.npz`` vectors are committed; no reference source enters the repo.
"""
import json
import os
import sys
import types

import numpy as np
import torch
from torch import nn

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
SHIM = os.path.join(HERE, "dgl_shim")


def load_reference_module(name):
    sys.dont_write_bytecode = True
    if SHIM not in sys.path:
        sys.path.insert(0, SHIM)
    import dgl  # noqa: F401  (the shim)

    path = os.path.join(REF, "models", name + ".py")
    with open(path, "r") as f:
        src = f.read()
    mod = types.ModuleType("ref_models_" + name)
    mod.__file__ = path
    exec(compile(src, path, "exec"), mod.__dict__)
    return mod


def run_graphnorm_case(norm_mod, name, sizes, F, bias, mean_scale, seed):
    """models/norm.py:7-29 GraphNorm on a dgl.batch of len(sizes) graphs (node features only)."""
    import dgl
    graphs = [dgl.graph((torch.zeros(0, dtype=torch.int64), torch.zeros(0, dtype=torch.int64)), num_nodes=n)
              for n in sizes]
    bg = dgl.batch(graphs)
    torch.manual_seed(seed)
    gn = norm_mod.GraphNorm(F, bias=bias, mean_scale=mean_scale)
    with torch.no_grad():   # non-trivial affine parameters
        gn.weight.copy_(torch.randn(F) * 0.5 + 1.0)
        if bias:
            gn.bias.copy_(torch.randn(F) * 0.1)
        if mean_scale:
            gn.mean_scale.copy_(torch.rand(F) + 0.25)
    gen = torch.Generator().manual_seed(seed + 1)
    X = (torch.randn(sum(sizes), F, generator=gen) * 2.0 + 0.5).requires_grad_(True)
    dY = torch.randn(sum(sizes), F, generator=gen)
    Y = gn(bg, X)
    Y.backward(dY)
    t = lambda x: x.detach().numpy()
    out = {"batch_num_nodes": np.asarray(sizes, np.int64), "X": t(X), "dY": t(dY), "Y": t(Y), "dX": t(X.grad),
           "weight": t(gn.weight), "dweight": t(gn.weight.grad)}
    if bias:
        out["bias"] = t(gn.bias); out["dbias"] = t(gn.bias.grad)
    if mean_scale:
        out["mean_scale"] = t(gn.mean_scale); out["dmean_scale"] = t(gn.mean_scale.grad)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    return {"name": name, "kind": "graphnorm", "sizes": list(map(int, sizes)), "F": F, "bias": bias,
            "mean_scale": mean_scale, "seed": seed, "agg": "graphnorm", "act": "none", "dtype": "float32",
            "keys": sorted(out.keys())}


def load_reference_conv():
    sys.dont_write_bytecode = True
    sys.path.insert(0, SHIM)
    import dgl  # noqa: F401  (the shim)

    path = os.path.join(REF, "models", "conv.py")
    with open(path, "r") as f:
        src = f.read()
    mod = types.ModuleType("ref_models_conv")
    mod.__file__ = path
    exec(compile(src, path, "exec"), mod.__dict__)
    return mod


# --------------------------------------------------------------------------------------
# graphs with the edge cases the survey lists: isolated destinations,
# zero out-degree sources, self-loops, duplicate edges, a hub row, a row longer than the
# kernel's split chunk, and the empty graph.
# --------------------------------------------------------------------------------------
def graph_small(seed=11):
    rng = np.random.default_rng(seed)
    V = 64
    src = list(rng.integers(0, 56, size=360))          # nodes 56..63 have out-degree 0
    dst = list(rng.integers(0, 60, size=360))          # nodes 60..63 have in-degree 0
    src += list(rng.integers(0, 56, size=100)); dst += [7] * 100   # hub row (in-degree >100)
    loops = rng.integers(0, 56, size=12)
    src += list(loops); dst += list(np.minimum(loops, 59))         # self-loops
    dup = rng.integers(0, len(src), size=40)
    src += [src[i] for i in dup]; dst += [dst[i] for i in dup]     # duplicate edges
    perm = rng.permutation(len(src))                               # shuffle edge ids
    src = np.asarray(src, np.int64)[perm]; dst = np.asarray(dst, np.int64)[perm]
    return V, src, dst


def graph_powerlaw(V, E, alpha, seed):
    g = torch.Generator().manual_seed(seed)
    p = (torch.arange(V, dtype=torch.float64) + 1.0).pow(-alpha)
    src = torch.multinomial(p, E, replacement=True, generator=g)
    dst = torch.multinomial(p, E, replacement=True, generator=g)
    relabel = torch.randperm(V, generator=g)
    return V, relabel[src].numpy().astype(np.int64), relabel[dst].numpy().astype(np.int64)


def graph_long(seed=13):
    rng = np.random.default_rng(seed)
    V = 40
    src = list(rng.integers(0, V, size=600)); dst = list(rng.integers(0, V, size=600))
    src += list(rng.integers(0, V, size=2100)); dst += [3] * 2100   # one row > 8 chunks of 256
    src += list(rng.integers(0, V, size=700)); dst += [21] * 700     # a second split row
    perm = rng.permutation(len(src))
    return V, np.asarray(src, np.int64)[perm], np.asarray(dst, np.int64)[perm]


def graph_small_nodup(seed=11):
    """graph_small without duplicate edges: continuous data then has no max ties, where the shim's
    amax backward (tie-splitting) and DGL's first-arg-max backward would differ."""
    V, src, dst = graph_small(seed)
    seen, keep = set(), []
    for i, (u, v) in enumerate(zip(src.tolist(), dst.tolist())):
        if (u, v) not in seen:
            seen.add((u, v))
            keep.append(i)
    keep = np.asarray(keep)
    return V, src[keep], dst[keep]


def graph_empty():
    return 16, np.zeros(0, np.int64), np.zeros(0, np.int64)


# --------------------------------------------------------------------------------------
def make_act(kind, H, seed):
    if kind == "relu":
        return nn.ReLU(), {}
    if kind == "leaky":
        return nn.LeakyReLU(0.2, inplace=True), {}
    if kind == "gelu":
        return nn.GELU(), {}
    if kind == "tanh":  # a sigma callable without a fused kernel (generic native path)
        return nn.Tanh(), {}
    if kind == "seq":  # dictionary-lookup/model.py:17
        torch.manual_seed(seed + 7)
        act = nn.Sequential(nn.ReLU(inplace=True), nn.Linear(H, H), nn.ReLU(inplace=True))
        return act, {"act_W": act[1].weight, "act_b": act[1].bias}
    raise ValueError(kind)


def run_case(conv_mod, name, graph, d, H, O, agg, act_kind, dtype, seed):
    import dgl
    V, src, dst = graph
    g = dgl.graph((torch.from_numpy(src), torch.from_numpy(dst)), num_nodes=V)
    act, act_params = make_act(act_kind, H, seed)
    torch.manual_seed(seed)
    m = conv_mod.SIRConv(d, H, O, act, 0, agg_type=agg)
    m = m.to(dtype)
    act = act.to(dtype)
    m.train()
    gen = torch.Generator().manual_seed(seed + 1)
    X = torch.randn(V, d, generator=gen, dtype=torch.float64).to(dtype).requires_grad_(True)
    dY = torch.randn(V, O, generator=gen, dtype=torch.float64).to(dtype)

    cap = {}

    def out_hook(key):
        def h(_mod, _inp, out):
            out.retain_grad()
            cap[key] = out
        return h

    def pre_hook(_mod, inp):
        if agg in ("sum", "mean", "sym"):
            inp[0].retain_grad()
            cap["S"] = inp[0]

    hs = [m.linear_query.register_forward_hook(out_hook("Q")),
          m.linear_key.register_forward_hook(out_hook("K")),
          m.linear_relation.register_forward_pre_hook(pre_hook)]
    Y = m(g, X)
    Y.backward(dY)
    for h in hs:
        h.remove()

    t = lambda x: x.detach().cpu().numpy()
    out = {
        "src": src, "dst": dst,
        "X": t(X), "W_Q": t(m.linear_query.weight), "b_Q": t(m.linear_query.bias),
        "W_K": t(m.linear_key.weight), "W_R": t(m.linear_relation.weight), "b_R": t(m.linear_relation.bias),
        "Y": t(Y), "dY": t(dY), "dX": t(X.grad),
        "dW_Q": t(m.linear_query.weight.grad), "db_Q": t(m.linear_query.bias.grad),
        "dW_K": t(m.linear_key.weight.grad),
        "dW_R": t(m.linear_relation.weight.grad), "db_R": t(m.linear_relation.bias.grad),
        "Q": t(cap["Q"]), "K": t(cap["K"]), "dQ": t(cap["Q"].grad), "dK": t(cap["K"].grad),
        "in_deg": t(g.in_degrees()), "out_deg": t(g.out_degrees()),
    }
    if "S" in cap:
        out["S"] = t(cap["S"])
        out["dS"] = t(cap["S"].grad)
    for k, p in act_params.items():
        out[k] = t(p.to(dtype))
        if p.grad is not None:
            out["d" + k] = t(p.grad)
    meta = {"name": name, "V": int(V), "E": int(src.size), "d": d, "H": H, "O": O, "agg": agg,
            "act": act_kind, "slope": 0.2 if act_kind == "leaky" else 0.0,
            "dtype": str(dtype).replace("torch.", ""), "seed": seed,
            "keys": sorted(out.keys())}
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    return meta


def run_sire_case(conv_mod, name, graph, d, de, H, O, agg, act_kind, dtype, seed):
    """models/conv.py:70-134 SIREConv: sigma((eq[v] + ek[u]) + e_uv) with e = linear_edge(efeat)."""
    import dgl
    V, src, dst = graph
    g = dgl.graph((torch.from_numpy(src), torch.from_numpy(dst)), num_nodes=V)
    act, _ = make_act(act_kind, H, seed)
    torch.manual_seed(seed)
    m = conv_mod.SIREConv(d, de, H, O, act, 0, agg_type=agg).to(dtype)
    m.train()
    gen = torch.Generator().manual_seed(seed + 1)
    X = torch.randn(V, d, generator=gen, dtype=torch.float64).to(dtype).requires_grad_(True)
    Ef = torch.randn(src.size, de, generator=gen, dtype=torch.float64).to(dtype).requires_grad_(True)
    dY = torch.randn(V, O, generator=gen, dtype=torch.float64).to(dtype)
    Y = m(g, X, Ef)
    Y.backward(dY)
    t = lambda x: x.detach().cpu().numpy()
    out = {
        "src": src, "dst": dst, "X": t(X), "efeat": t(Ef),
        "W_Q": t(m.linear_query.weight), "b_Q": t(m.linear_query.bias), "W_K": t(m.linear_key.weight),
        "W_E": t(m.linear_edge.weight), "W_R": t(m.linear_relation.weight), "b_R": t(m.linear_relation.bias),
        "Y": t(Y), "dY": t(dY), "dX": t(X.grad), "defeat": t(Ef.grad),
        "dW_Q": t(m.linear_query.weight.grad), "db_Q": t(m.linear_query.bias.grad),
        "dW_K": t(m.linear_key.weight.grad), "dW_E": t(m.linear_edge.weight.grad),
        "dW_R": t(m.linear_relation.weight.grad), "db_R": t(m.linear_relation.bias.grad),
    }
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    return {"name": name, "kind": "sire", "V": int(V), "E": int(src.size), "d": d, "de": de, "H": H, "O": O,
            "agg": agg, "act": act_kind, "slope": 0.2 if act_kind == "leaky" else 0.0,
            "dtype": str(dtype).replace("torch.", ""), "seed": seed, "keys": sorted(out.keys())}


def main():
    conv_mod = load_reference_conv()
    small = graph_small()
    wide = graph_powerlaw(96, 1600, 0.8, seed=21)
    long_ = graph_long()
    empty = graph_empty()
    cases = []
    seed = 100
    for agg in ("sum", "mean", "sym", "max"):
        for act in ("relu", "leaky", "gelu"):
            seed += 1
            cases.append(run_case(conv_mod, f"small_{agg}_{act}_f32", small, 16, 32, 8, agg, act, torch.float32, seed))
    for agg in ("sum", "mean", "sym"):
        seed += 1
        cases.append(run_case(conv_mod, f"small_{agg}_leaky_f64", small, 16, 32, 8, agg, "leaky", torch.float64, seed))
    seed += 1
    cases.append(run_case(conv_mod, "small_sum_seq_f32", small, 16, 32, 32, "sum", "seq", torch.float32, seed))
    for agg in ("sum", "mean", "sym"):
        seed += 1
        cases.append(run_case(conv_mod, f"wide_{agg}_leaky_h256_f32", wide, 64, 256, 64, agg, "leaky", torch.float32, seed))
    seed += 1
    cases.append(run_case(conv_mod, "wide_sum_leaky_d256_f32", wide, 256, 256, 256, "sum", "leaky", torch.float32, seed))
    seed += 1
    cases.append(run_case(conv_mod, "wide_sym_gelu_h256_f32", wide, 64, 256, 64, "sym", "gelu", torch.float32, seed))
    for H in (64, 128, 300):
        seed += 1
        cases.append(run_case(conv_mod, f"wide_sym_leaky_h{H}_f32", wide, 48, H, 48, "sym", "leaky", torch.float32, seed))
    for agg in ("sum", "mean", "sym"):
        seed += 1
        cases.append(run_case(conv_mod, f"long_{agg}_leaky_h256_f32", long_, 32, 256, 32, agg, "leaky", torch.float32, seed))
    seed += 1
    cases.append(run_case(conv_mod, "empty_sum_leaky_f32", empty, 16, 32, 8, "sum", "leaky", torch.float32, seed))
    seed += 1
    cases.append(run_case(conv_mod, "empty_sym_relu_f32", empty, 16, 32, 8, "sym", "relu", torch.float32, seed))
    # round-1 additions (appended so earlier fixtures keep their seeds): max aggregation on a
    # duplicate-free graph (no ties), and sigma callables without a fused kernel
    nodup = graph_small_nodup()
    for act in ("relu", "leaky", "gelu"):
        seed += 1
        cases.append(run_case(conv_mod, f"nodup_max_{act}_f32", nodup, 16, 32, 8, "max", act, torch.float32, seed))
    seed += 1
    cases.append(run_case(conv_mod, "nodup_max_leaky_h256_f32", nodup, 32, 256, 40, "max", "leaky", torch.float32, seed))
    seed += 1
    cases.append(run_case(conv_mod, "small_sym_tanh_f32", small, 16, 32, 8, "sym", "tanh", torch.float32, seed))
    seed += 1
    cases.append(run_case(conv_mod, "small_mean_seq_f32", small, 16, 64, 16, "mean", "seq", torch.float32, seed))
    # GraphNorm (models/norm.py:7-29), SURVEY §8(f) row 2: batched small graphs incl. a 1-node graph
    norm_mod = load_reference_module("norm")
    rng = np.random.default_rng(5)
    mol_sizes = [int(x) for x in rng.integers(5, 40, size=24)] + [1, 57]
    cases.append(run_graphnorm_case(norm_mod, "graphnorm_mol_f300", mol_sizes, 300, True, True, 501))
    cases.append(run_graphnorm_case(norm_mod, "graphnorm_mol_f64_nobias", mol_sizes[:10], 64, False, True, 502))
    cases.append(run_graphnorm_case(norm_mod, "graphnorm_f256_noscale", [3, 700, 12], 256, True, False, 503))
    cases.append(run_graphnorm_case(norm_mod, "graphnorm_f30_odd", [9, 4, 33], 30, True, True, 504))
    # SIREConv (models/conv.py:70-134), SURVEY §8(f) row 4: the edge-feature term
    seed = 700
    for agg in ("sum", "mean", "sym"):
        for act in ("relu", "leaky", "gelu"):
            seed += 1
            cases.append(run_sire_case(conv_mod, f"sire_small_{agg}_{act}_f32", small, 16, 6, 32, 8, agg, act,
                                       torch.float32, seed))
    for act in ("leaky", "gelu"):
        seed += 1
        cases.append(run_sire_case(conv_mod, f"sire_nodup_max_{act}_f32", nodup, 16, 6, 32, 8, "max", act,
                                   torch.float32, seed))
    seed += 1
    cases.append(run_sire_case(conv_mod, "sire_wide_sum_leaky_h256_f32", wide, 64, 16, 256, 64, "sum", "leaky",
                               torch.float32, seed))
    seed += 1
    cases.append(run_sire_case(conv_mod, "sire_long_sym_leaky_h256_f32", long_, 32, 8, 256, 32, "sym", "leaky",
                               torch.float32, seed))
    seed += 1
    cases.append(run_sire_case(conv_mod, "sire_small_sum_leaky_f64", small, 16, 6, 32, 8, "sum", "leaky",
                               torch.float64, seed))
    seed += 1
    cases.append(run_sire_case(conv_mod, "sire_empty_sum_relu_f32", empty, 16, 6, 32, 8, "sum", "relu",
                               torch.float32, seed))
    seed += 1
    cases.append(run_sire_case(conv_mod, "sire_small_sum_tanh_f32", small, 16, 6, 32, 8, "sum", "tanh",
                               torch.float32, seed))
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "reference": "briangodwinlim/SIR-GCN models/conv.py:7-134, models/norm.py:7-29 (snapshot 2025-08-24), via DGL-2.1.0 semantics shim",
                   "torch": torch.__version__, "cases": cases}, f, indent=1)
    print(f"wrote {len(cases)} cases")


if __name__ == "__main__":
    main()
