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


def golden_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)["cases"]


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
