"""Host-side graph logic on CPU: CSR builder bit-exact vs the oracle (DGL's stable CSC order),
work-plan invariants (every edge in exactly one item, split bookkeeping), degrees/norms."""
import numpy as np
import pytest
import torch

import oracle
from conftest import golden_manifest, load_case

from sirgcn.graph import Graph, GraphPlan, build_row_csr, get_plan


def _check_plan(csr, rowptr_ref, chunk):
    n = csr.n_rows
    items = csr.items.cpu().numpy().astype(np.int64)
    rowptr = csr.rowptr.cpu().numpy().astype(np.int64)
    assert np.array_equal(rowptr, rowptr_ref)
    covered = np.zeros(rowptr[-1], dtype=np.int64)
    rows_seen = np.zeros(n, dtype=np.int64)
    for row, eb, ee, slot in items:
        assert rowptr[row] <= eb <= ee <= rowptr[row + 1]
        assert ee - eb <= chunk
        covered[eb:ee] += 1
        rows_seen[row] += 1
    assert np.all(covered == 1)
    assert np.all(rows_seen >= 1)
    deg = np.diff(rowptr)
    split_rows = np.nonzero(rows_seen > 1)[0]
    assert csr.n_splits == split_rows.size
    if csr.n_splits:
        sp = csr.splits.cpu().numpy().astype(np.int64)
        assert np.array_equal(sp[:, 0], split_rows)
        assert np.array_equal(sp[:, 3], deg[split_rows])
        slots = items[items[:, 3] >= 0]
        assert slots.shape[0] == csr.n_slots == sp[:, 2].sum()
        for row, s0, ns, _ in sp:
            mine = slots[slots[:, 0] == row]
            assert np.array_equal(np.sort(mine[:, 3]), np.arange(s0, s0 + ns))
    else:
        assert np.all(items[:, 3] == -1)


CASES = [c["name"] for c in golden_manifest() if c["name"].endswith("_f32")][:6] + \
        ["long_sum_leaky_h256_f32", "empty_sum_leaky_f32"]


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("chunk", [4, 256])
def test_row_csr_matches_oracle(name, chunk):
    z = load_case(name)
    V = int(z["in_deg"].size)
    src, dst = torch.from_numpy(z["src"]), torch.from_numpy(z["dst"])
    plan = GraphPlan(src, dst, V, "cpu", chunk=chunk)
    rowptr, col, eid = oracle.csr_by_dst(z["src"], z["dst"], V)
    assert np.array_equal(plan.dst.col.numpy(), col.astype(np.int32))
    assert np.array_equal(plan.dst.eid.numpy(), eid)
    _check_plan(plan.dst, rowptr, chunk)
    rowptr_s, col_s, eid_s = oracle.csr_by_src(z["src"], z["dst"], V)
    assert np.array_equal(plan.src.col.numpy(), col_s.astype(np.int32))
    assert np.array_equal(plan.src.eid.numpy(), eid_s)
    _check_plan(plan.src, rowptr_s, chunk)
    assert np.array_equal(plan.in_deg.numpy(), z["in_deg"])
    assert np.array_equal(plan.out_deg.numpy(), z["out_deg"])


def test_sym_norms_equal_reference_formula():
    z = load_case("small_sym_leaky_f32")
    V = int(z["in_deg"].size)
    plan = GraphPlan(torch.from_numpy(z["src"]), torch.from_numpy(z["dst"]), V, "cpu")
    in_norm, out_norm = plan.norms("sym")
    ref_in, ref_out = oracle.degree_norms(z["in_deg"], z["out_deg"], "sym")
    assert torch.equal(in_norm, ref_in) and torch.equal(out_norm, ref_out)
    assert plan.norms("sum") == (None, None)


def test_graph_surface_and_plan_cache():
    g = Graph([0, 1, 2, 2], [1, 2, 0, 0], num_nodes=4)
    assert g.num_nodes() == 4 and g.num_edges() == 4
    assert g.in_degrees().tolist() == [2, 1, 1, 0]
    assert g.out_degrees().tolist() == [1, 1, 2, 0]
    with g.local_scope():
        g.ndata["x"] = 1
    assert "x" not in g.ndata
    p1 = get_plan(g, "cpu")
    assert get_plan(g, "cpu") is p1
    assert p1.dst.rowptr.tolist() == [0, 2, 3, 4, 4]
    assert p1.dst.col.tolist() == [2, 2, 0, 1]


def test_duck_typed_graph_with_edges_only():
    class G:
        def __init__(self):
            self.s = torch.tensor([3, 0, 1]); self.d = torch.tensor([0, 0, 2])

        def edges(self):
            return self.s, self.d

        def num_nodes(self):
            return 4
    g = G()
    p = get_plan(g, "cpu")
    assert p.dst.col.tolist() == [3, 0, 1]
    assert get_plan(g, "cpu") is p


def test_hub_rows_are_split_and_bounded():
    V = 1000
    dst = torch.cat([torch.zeros(5000, dtype=torch.int64), torch.randint(0, V, (3000,), generator=torch.Generator().manual_seed(0))])
    src = torch.randint(0, V, (dst.numel(),), generator=torch.Generator().manual_seed(1))
    csr = build_row_csr(dst, src, V, chunk=256)
    assert csr.n_splits >= 1 and csr.max_degree >= 5000
    rowptr, _, _ = oracle.csr_by_dst(src.numpy(), dst.numpy(), V)
    _check_plan(csr, rowptr, 256)
