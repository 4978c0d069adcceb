"""sirgcn — MI355X-native SIRConv (briangodwinlim/SIR-GCN ``models/conv.py``) hot path.

    import sys; sys.path.insert(0, "<repo>/sir-gcn_amd")
    from sirgcn import SIRConv, Graph      # drop-in for `from models.conv import SIRConv`
"""
from .conv import SIRConv, EdgeAggregate, activation_code  # noqa: F401
from .graph import Graph, GraphPlan, RowCSR, batch, get_plan, build_row_csr  # noqa: F401
from .norm import GraphNorm  # noqa: F401
from .econv import SIREConv  # noqa: F401
from . import _native  # noqa: F401

__all__ = ["SIRConv", "SIREConv", "GraphNorm", "Graph", "GraphPlan", "RowCSR", "EdgeAggregate", "batch", "get_plan",
           "build_row_csr"]
