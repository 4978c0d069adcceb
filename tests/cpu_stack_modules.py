"""TEST INFRASTRUCTURE: CPU stand-ins for ``sirgcn.SIRConv`` / ``sirgcn.GraphNorm`` (the oracle's
restatements of ``models/conv.py`` / ``models/norm.py``), so that ``bench.py --gpus N --dist-backend
gloo --workload cfg5`` can rehearse the data-parallel launcher / DDP plumbing on a machine without a
GPU, the way ``cpu_edge_backend`` does for the cfg4 edge-cut.  Never used by the product path."""
import oracle

SIRConv = oracle.SIRConvRef
GraphNorm = oracle.GraphNormRef
