"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference SIRConv path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / the timed CPU baseline.  The product path
(``sir-gcn_amd/sirgcn``) never imports it and has no CPU fallback.

Pinning: ``tests/test_oracle_golden.py`` checks every function here against the golden
vectors in ``tests/golden/*.npz``, which were produced by executing the reference's own
``models/conv.py`` (``tests/golden/make_golden.py``).
"""
from .sirconv_oracle import (  # noqa: F401
    ACTS, AGGS, act_fwd, act_bwd, csr_by_dst, csr_by_src, degree_norms,
    edge_agg_fwd, edge_agg_bwd, layer_fwd_bwd, max_first_wins, max_tie_flips, max_edge_values,
    sigma_tie_flips,
    reference_cpu_step,
)
from .graphnorm_oracle import graph_norm_fwd, graph_norm_bwd  # noqa: F401
from .sireconv_oracle import sire_reference_step  # noqa: F401
from .modules_oracle import SIRConvRef, GraphNormRef  # noqa: F401
