import glob
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sir-gcn_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


def golden_manifest(kind="sirconv"):
    """Fixture cases of one kind: "sirconv" (conv.py SIRConv), "sire" (SIREConv),
    "graphnorm" (norm.py GraphNorm); None = all."""
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        cases = json.load(f)["cases"]
    return [c for c in cases if kind is None or c.get("kind", "sirconv") == kind]


def load_case(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def manifest():
    return golden_manifest()


def rel_err(a, b):
    import torch
    a = torch.as_tensor(a).double()
    b = torch.as_tensor(b).double()
    den = b.norm().item()
    num = (a - b).norm().item()
    return num / den if den > 0 else num


def assert_close(actual, ref, rel=1e-5, what=""):
    """SURVEY.md §8c tolerance: ||d|| / ||ref|| <= rel AND allclose(rtol=rel, atol=1e-6*max|ref|)."""
    import torch
    a = torch.as_tensor(actual).double().cpu()
    r = torch.as_tensor(ref).double().cpu()
    assert a.shape == r.shape, (what, a.shape, r.shape)
    e = rel_err(a, r)
    assert e <= rel, f"{what}: relative L2 error {e:.3e} > {rel:.1e}"
    atol = 1e-6 * (r.abs().max().item() if r.numel() else 0.0) * (rel / 1e-5)
    assert torch.allclose(a, r, rtol=rel, atol=atol), f"{what}: allclose failed (max abs diff {(a - r).abs().max().item():.3e})"


def assert_parity(actual, ref32, truth64, rel=1e-5, what=""):
    """Accuracy-aware parity against the reference.

    ``ref32`` is the reference's own fp32 output (golden fixture / CPU oracle), ``truth64`` the
    same algorithm evaluated in fp64 (oracle).  Passes when the native result is within ``rel``
    of the reference, or — where the reference's own fp32 rounding (long hub sums) is already
    of that order — no worse than twice the reference's own error against fp64:
      per tensor : relL2(actual, truth) <= max(rel, 2 * relL2(ref32, truth))
      elementwise: |actual - truth| <= rel*|truth| + 1e-6*max|truth| + 4*max|ref32 - truth|
    """
    import torch
    a = torch.as_tensor(actual).double().cpu()
    r = torch.as_tensor(ref32).double().cpu()
    t = torch.as_tensor(truth64).double().cpu()
    assert a.shape == t.shape == r.shape, (what, a.shape, r.shape, t.shape)
    if rel_err(a, r) <= rel and torch.allclose(a, r, rtol=rel, atol=1e-6 * (r.abs().max().item() if r.numel() else 0)):
        return
    e_ref = rel_err(r, t)
    e_act = rel_err(a, t)
    assert e_act <= max(rel, 2 * e_ref), f"{what}: relL2 vs fp64 {e_act:.3e} > max({rel:.0e}, 2*ref {e_ref:.3e})"
    ref_abs = (r - t).abs().max().item() if r.numel() else 0.0
    tmax = t.abs().max().item() if t.numel() else 0.0
    bound = rel * t.abs() + 1e-6 * tmax + 4 * ref_abs
    bad = ((a - t).abs() > bound)
    assert not bad.any(), f"{what}: {int(bad.sum())} elements beyond the reference's own error envelope"
