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


@pytest.fixture(autouse=True)
def _native_gemm_at_every_size():
    """Every fp32 GEMM the native kernels accept runs natively in the tests, as in the product
    (linalg.DEFAULT_MIN_ROWS = 0: small batches take the library's one-wave-per-tile kernels); the
    fixture pins that in case a caller raised the threshold."""
    from sirgcn import linalg
    old = linalg.MIN_ROWS
    linalg.MIN_ROWS = 0
    yield
    linalg.MIN_ROWS = old


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


PARITY_FALLBACKS = []      # (what, relL2 vs ref32, relL2 vs fp64, ref32's own relL2 vs fp64)


def assert_parity(actual, ref32, truth64, rel=1e-5, what="", strict=False, factor=2.0):
    """Accuracy-aware parity against the reference.

    ``ref32`` is the reference's own fp32 output (golden fixture / CPU oracle), ``truth64`` the
    same algorithm evaluated in fp64 (oracle).  Passes when the native result is within ``rel``
    of the reference (relative L2 and elementwise), or — where the reference's own fp32 rounding
    (long hub sums) is already of that order — no worse than twice the reference's own error
    against fp64:
      per tensor : relL2(actual, truth) <= max(rel, 2 * relL2(ref32, truth))
      elementwise: |actual - truth| <= rel*|truth| + 1e-6*max|truth| + 2*factor*max|ref32 - truth|
    Every case that passes only through that second criterion is recorded in PARITY_FALLBACKS and
    listed in the session summary.  ``strict=True`` (layer outputs h*, the north-star bar "within
    1e-5 rel"): relL2 to the reference <= ``rel`` is REQUIRED, and elements must lie inside the fp64
    envelope above (near-zero elements of a long fp32 sum are ill-posed for a pure rtol).
    ``factor`` (default 2) scales the envelope — the per-tensor and the elementwise term alike — for
    multi-layer stacks, where rounding differences of every layer compound.  (The elementwise term
    is set by the reference's own worst element, which moves run to run with torch's atomics: a
    4-layer element sat at 1.00-1.03x the unscaled bound across runs of the same build.)
    """
    import torch
    a = torch.as_tensor(actual).double().cpu()
    r = torch.as_tensor(ref32).double().cpu()
    t = torch.as_tensor(truth64).double().cpu()
    assert a.shape == t.shape == r.shape, (what, a.shape, r.shape, t.shape)
    e_r = rel_err(a, r)
    if e_r <= rel and torch.allclose(a, r, rtol=rel, atol=1e-6 * (r.abs().max().item() if r.numel() else 0)):
        return
    assert not strict or e_r <= rel, f"{what}: relL2 vs the reference {e_r:.3e} > {rel:.0e} (strict)"
    e_ref = rel_err(r, t)
    e_act = rel_err(a, t)
    assert strict or e_act <= max(rel, factor * e_ref), \
        f"{what}: relL2 vs fp64 {e_act:.3e} > max({rel:.0e}, {factor:g}*ref {e_ref:.3e})"
    ref_abs = (r - t).abs().max().item() if r.numel() else 0.0
    tmax = t.abs().max().item() if t.numel() else 0.0
    bound = rel * t.abs() + 1e-6 * tmax + 2 * factor * ref_abs
    bad = ((a - t).abs() > bound)
    if bad.any():
        i = int(((a - t).abs() - bound).argmax())
        af, rf, tf, bf = a.reshape(-1), r.reshape(-1), t.reshape(-1), bound.reshape(-1)
        raise AssertionError(f"{what}: {int(bad.sum())} elements beyond the reference's own error envelope "
                             f"(worst #{i}: ours {af[i].item():.6e} ref32 {rf[i].item():.6e} fp64 {tf[i].item():.6e} "
                             f"bound {bf[i].item():.2e}; max|ref32-fp64| {ref_abs:.2e})")
    PARITY_FALLBACKS.append((what + (" [strict: relL2 ok, elementwise via envelope]" if strict else ""),
                             e_r, e_act, e_ref))


TIE_CONDITIONED = []       # (what, sigma' flips, worst |z64| / ulp-mag, arg flips, worst gap / ulp-mag)


def tie_conditioned(what, n_sigma, w_sigma, n_arg=0, w_arg=0.0):
    """Record a case scored against the oracle conditioned on the kernel's own Q, K (and arg edges)
    because of near-ties (oracle.sigma_tie_flips / max_tie_flips)."""
    TIE_CONDITIONED.append((what, n_sigma, w_sigma, n_arg, w_arg))


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if TIE_CONDITIONED:
        terminalreporter.write_line(f"near-ties: {len(TIE_CONDITIONED)} case(s) scored against the oracle conditioned "
                                    "on the kernel's Q, K / arg edges (sigma' flips, worst |z|/(2^-24 mag), "
                                    "arg flips, worst gap/(2^-24 mag)):")
        for what, n_s, w_s, n_a, w_a in TIE_CONDITIONED:
            terminalreporter.write_line(f"  {what}: {n_s}, {w_s:.2f}, {n_a}, {w_a:.2f}")
    if PARITY_FALLBACKS:
        terminalreporter.write_line(f"assert_parity: {len(PARITY_FALLBACKS)} tensor(s) passed through the fp64 "
                                    "envelope (relL2 vs ref32 / vs fp64 / ref32's own vs fp64):")
        for what, e_r, e_a, e_ref in PARITY_FALLBACKS:
            terminalreporter.write_line(f"  {what}: {e_r:.2e} / {e_a:.2e} / {e_ref:.2e}")
