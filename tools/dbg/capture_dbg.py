import faulthandler, os, sys
faulthandler.enable()
import torch
from torch import nn
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "sir-gcn_amd"))
from sirgcn import SIRConv, Graph
import sirgcn.conv as conv
conv.OVERLAP_ROWS = int(os.environ.get("ROWS", "0"))
DEV = "cuda"
g = torch.Generator().manual_seed(11)
V, E, H = 1582, 3382, 300
graph = Graph(torch.randint(0, V, (E,), generator=g), torch.randint(0, V, (E,), generator=g), V)
X = torch.randn(V, H, generator=g).to(DEV)
dY = torch.randn(V, H, generator=g).to(DEV)
m = SIRConv(H, H, H, nn.LeakyReLU(0.2), 0.0, agg_type="sum").to(DEV)
static_x = X.clone().requires_grad_(True)
def step():
    m.zero_grad(set_to_none=True)
    static_x.grad = None
    m(graph, static_x).backward(dY)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
print("warm ok", flush=True)
cg = torch.cuda.CUDAGraph()
mode = os.environ.get("MODE", "fwd")
with torch.cuda.graph(cg):
    print("in capture", flush=True)
    if mode == "fwd":
        with torch.no_grad():
            Y = m(graph, static_x)
    else:
        step()
    print("captured body", flush=True)
print("capture ok", flush=True)
cg.replay()
torch.cuda.synchronize()
print("replay ok", flush=True)
