"""BASELINE.json configs as concrete workloads (shape-matched synthetic stand-ins; the real datasets
need network).  One definition serves ``bench.py --workload`` and the ``-m gpu`` stack tests, and
takes the conv / norm classes as parameters so the tests can build the identical stack on the
oracle's restated modules.

=======  ========================================================================================
name     what (reference)
=======  ========================================================================================
cfg1     DictionaryLookup n=10, batch 256 (V=5,120, E=25,600): 1 SIRConv, H=64, sum,
         sigma = Sequential(ReLU, Linear(H,H), ReLU) (``dictionary-lookup/model.py:17,20,30-32``,
         ``data.py:27-31``, ``train.py:108,114,119``)
cfg2     ZINC-shaped batch of 10,000 molecules (~231k nodes, ~497k edges): 4 layers, H=128, sym,
         LeakyReLU(0.2), identity residual (``zinc/model.py:50-56``); run under bf16 autocast
cfg3     ogbn-arxiv-shaped power-law graph (V=169,343, E=1,166,243): 3 layers, H=256, sym,
         LeakyReLU(0.2), residual (``ogbn-arxiv/model.py:65-73``)
cfg4     S2 power-law (V=2M, E=40M), 1 layer, H=256 (the headline; bench.py's default)
cfg5     ogbg-molhiv-shaped batch of 64 molecules per GPU (~1.6k nodes, ~3.5k edges): 5 layers,
         H=300, SIRConv -> GraphNorm -> LeakyReLU(0.2) -> +residual (``ogbg-molhiv/model.py:76-84``,
         ``norm.py:7-29``); data-parallel over GPUs (a different batch per rank)
=======  ========================================================================================
"""
import torch
from torch import nn

from .stacks import SIRStack
from .synth import NAMED, dictionary_lookup_batch, molecule_batch, powerlaw_graph

# feat_dropout: the SIRConv dropout the reference trains each config's source with
# (ogbn-arxiv/train.py:303 and ogbg-molhiv/train.py:249: 0.2; zinc/train.py:206: 0)
CONFIGS = {
    "cfg1": dict(hidden=64, layers=1, agg="sum", order="plain", dtype="f32", sigma="seq", feat_dropout=0.0),
    "cfg2": dict(hidden=128, layers=4, agg="sym", order="zinc", dtype="bf16", sigma="leaky", feat_dropout=0.0),
    "cfg3": dict(hidden=256, layers=3, agg="sym", order="arxiv", dtype="f32", sigma="leaky", feat_dropout=0.2),
    "cfg5": dict(hidden=300, layers=5, agg="sum", order="arxiv", dtype="f32", sigma="leaky", norm=True,
                 feat_dropout=0.2),
}
DTYPES = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}


def make_graph(name, seed=0, rank=0, small=False):
    """The workload's graph (``small``: a reduced instance of the same shape for quick tests)."""
    if name == "cfg1":
        return dictionary_lookup_batch(10, 16 if small else 256)
    if name == "cfg2":
        return molecule_batch(200 if small else 10_000, 23, seed=seed)
    if name == "cfg3":
        V, E, a = NAMED["arxiv"]
        return powerlaw_graph(V // 20, E // 20, a, seed) if small else powerlaw_graph(V, E, a, seed)
    if name == "cfg5":
        return molecule_batch(8 if small else 64, 25, seed=seed + 1000 * rank)
    raise KeyError(name)


def make_stack(name, conv_cls, norm_cls=None, seed=4, feat_dropout=0.0):
    """The config's layer stack on ``conv_cls`` (and ``norm_cls`` for cfg5), seeded init.
    ``feat_dropout``: the convs' Q/K dropout (0 for the parity tests; ``bench.py`` passes the
    config's trained value, ``CONFIGS[name]["feat_dropout"]``)."""
    c = CONFIGS[name]
    H = c["hidden"]
    torch.manual_seed(seed)
    act = nn.LeakyReLU(0.2, inplace=True)
    sigma = act
    if c["sigma"] == "seq":          # dictionary-lookup/model.py:17 (shared by every layer)
        sigma = nn.Sequential(nn.ReLU(inplace=True), nn.Linear(H, H), nn.ReLU(inplace=True))
    return SIRStack(conv_cls, H, c["layers"], act, c["agg"], c["order"],
                    norm_cls=norm_cls if c.get("norm") else None, conv_activation=sigma, feat_dropout=feat_dropout)


def make_inputs(name, num_nodes, device, seed=3):
    """X ~ N(0,1) [V, H] and dY ~ N(0,1), seeded on the host (identical on every machine)."""
    H = CONFIGS[name]["hidden"]
    gen = torch.Generator().manual_seed(seed)
    X = torch.randn(num_nodes, H, generator=gen).to(device)
    dY = torch.randn(num_nodes, H, generator=gen).to(device)
    return X, dY


def dp_replica(name, rank, world, device, conv_cls, norm_cls=None, feat_dropout=0.0, small=False):
    """One rank of a data-parallel workload (cfg5: a different batch of molecules per rank, the
    stack replicated with identical initial weights, gradients averaged by DDP's all-reduce —
    RCCL in ``bench.py --gpus N``, gloo in tests/test_ddp_gloo.py).  Returns (model, stack,
    graph, X, dY); ``model`` is the DDP wrapper when ``world > 1``."""
    g = make_graph(name, rank=rank, small=small)
    stack = make_stack(name, conv_cls, norm_cls, feat_dropout=feat_dropout).to(device)
    model = stack
    if world > 1:
        ids = [device.index] if torch.device(device).type == "cuda" else None
        model = torch.nn.parallel.DistributedDataParallel(stack, device_ids=ids)
    X, dY = make_inputs(name, g.num_nodes(), device, seed=3 + rank)
    return model, stack, g, X, dY
