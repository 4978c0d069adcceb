"""GPU numerics of the split-fp16 MFMA projection GEMMs (sir_gemm_nt / sir_gemm_tn, through the
C ABI) against an fp64 evaluation, with torch's own fp32 GEMM as the yardstick.

Bar (the GEMMs of conv.py:60-61,65 and their autograd are floating point, so "parity" is
accuracy): per output element |C - C64| <= max(8e-7, 2x torch fp32 worst) * sum_k |a_ik||b_kj|, and
relative L2 error vs fp64 <= max(2 * torch fp32's, 1e-6).  The 8e-7 floor is the split's own
per-product bound: x*w is formed as hi*hi' + hi*lo' + lo*hi' with lo*lo' (< 2^-22 relative) dropped
and each lo rounded to fp16 (< 2^-22 each), i.e. <= 3 * 2^-22 = 7.2e-7 of |x||w| — visible alone
only when K (or R) is tiny, where fp32's single rounding is smaller; for real contraction lengths
the fp32 accumulation dominates both.  Runs: pytest tests -m gpu."""
import pytest
import torch

from sirgcn import _native

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need the MI355X box"
    _native.load()


def _rel(a, b):
    d = b.norm().item()
    return (a - b).norm().item() / d if d > 0 else (a - b).norm().item()


def _check(C, A64, B64, ref32, bias=None, what=""):
    """C vs fp64 A64 @ B64 (+bias); elementwise bound by the absolute-product sum."""
    C64 = A64 @ B64
    absum = A64.abs() @ B64.abs()
    if bias is not None:
        C64 = C64 + bias.double()
        absum = absum + bias.double().abs()
    den = absum + 1e-300
    worst = ((C.double() - C64).abs() / den).max().item() if C.numel() else 0.0
    worst_torch = ((ref32.double() - C64).abs() / den).max().item() if C.numel() else 0.0
    assert worst <= max(8e-7, 2 * worst_torch), \
        f"{what}: max |err| / sum|a||b| = {worst:.2e} (torch fp32: {worst_torch:.2e})"
    e_ours, e_torch = _rel(C.double(), C64), _rel(ref32.double(), C64)
    assert e_ours <= max(2 * e_torch, 1e-6), f"{what}: relL2 {e_ours:.2e} vs torch fp32 {e_torch:.2e}"
    return e_ours, e_torch


@pytest.mark.parametrize("M", [1, 255, 257, 4099])
@pytest.mark.parametrize("K,N", [(4, 4), (32, 64), (36, 132), (256, 256), (256, 512), (512, 256), (300, 300),
                                 (64, 128), (1024, 96)])
@pytest.mark.parametrize("with_bias", [True, False])
def test_gemm_nt_vs_fp64(M, K, N, with_bias):
    g = torch.Generator(device=DEV).manual_seed(M * 7 + K * 3 + N)
    A = torch.randn(M, K, device=DEV, generator=g)
    W = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
    b = torch.randn(N, device=DEV, generator=g) if with_bias else None
    C = _native.gemm_nt(A, _native.gemm_pack(W), b)
    ref = torch.addmm(b, A, W.t()) if with_bias else A @ W.t()
    _check(C, A.double(), W.double().t(), ref, b, f"nt M={M} K={K} N={N}")


@pytest.mark.parametrize("K,N", [(256, 256), (512, 256), (128, 64)])
def test_gemm_nt_transposed_weight(K, N):
    """B = W^T (W [K, N]): the x W form of G = dY W_R and dX = dQK [W_Q; W_K]."""
    g = torch.Generator(device=DEV).manual_seed(11)
    A = torch.randn(3001, K, device=DEV, generator=g)
    W = torch.randn(K, N, device=DEV, generator=g)
    C = _native.gemm_nt(A, _native.gemm_pack(W, trans=True))
    _check(C, A.double(), W.double(), A @ W, None, "nt trans")


def test_gemm_nt_wide_dynamic_range_and_running_scale():
    """Rows spanning 2^-40..2^40, zero rows, and rows whose maximum grows along K (every chunk
    raises the running scale: exercises the accumulator rescale), plus tiny/huge weights (all
    products stay inside the fp32 range)."""
    g = torch.Generator(device=DEV).manual_seed(5)
    M, K, N = 1500, 512, 256
    A = torch.randn(M, K, device=DEV, generator=g)
    A *= torch.exp2(torch.randint(-40, 40, (M, 1), device=DEV, generator=g).float())
    A[7] = 0
    ramp = torch.exp2(torch.linspace(-30, 30, K, device=DEV))
    A[100:300] *= ramp                      # maximum rises chunk after chunk
    A[300:400] *= ramp.flip(0)
    A[400:420, :96] = 0                     # leading zero chunks, then data: first scale set late
    A[420:440, :64] = 2.0 ** -130           # subnormal leading chunks, then normal-range data
    A[440:460, 32:] *= 2.0 ** 20            # a chunk far above the first one's headroom
    W = torch.randn(N, K, device=DEV, generator=g) * torch.exp2(torch.randint(-20, 20, (N, 1), device=DEV,
                                                                                generator=g).float())
    C = _native.gemm_nt(A, _native.gemm_pack(W))
    assert torch.all(C[7] == 0)
    _check(C, A.double(), W.double().t(), A @ W.t(), None, "nt dynamic range")


@pytest.mark.parametrize("M,K,N", [(70001, 256, 260), (513, 128, 512), (1, 512, 300), (66000, 512, 256)])
def test_gemm_nt_persistent_strided_out_and_ragged_tiles(M, K, N):
    """The persistent NT kernel (K = 128 / 256 / 512, N <= 512) writes through buffer stores whose
    range check drops rows past M and columns past N: C as a column slice of a wider tensor
    (ldc > N) keeps its neighbours, and a partial last data tile / feature tile is exact."""
    g = torch.Generator(device=DEV).manual_seed(M + K + N)
    A = torch.randn(M, K, device=DEV, generator=g)
    W = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
    b = torch.randn(N, device=DEV, generator=g)
    wide = torch.full((M, N + 44), 7.0, device=DEV)
    C = _native.gemm_nt(A, _native.gemm_pack(W), b, out=wide[:, 8:8 + N])
    assert torch.all(wide[:, :8] == 7.0) and torch.all(wide[:, 8 + N:] == 7.0)
    _check(C, A.double(), W.double().t(), torch.addmm(b, A, W.t()), b, f"nt strided M={M} K={K} N={N}")
    C0 = _native.gemm_nt(A, _native.gemm_pack(W))          # no bias: the epilogue adds -0 (an identity)
    _check(C0, A.double(), W.double().t(), A @ W.t(), None, f"nt no bias M={M}")


@pytest.mark.parametrize("R", [0, 1, 31, 33, 1000, 70001])
@pytest.mark.parametrize("M,N", [(4, 4), (32, 36), (256, 256), (512, 256), (300, 100)])
def test_gemm_tn_vs_fp64(R, M, N):
    g = torch.Generator(device=DEV).manual_seed(R + 3 * M + N)
    A = torch.randn(R, M, device=DEV, generator=g)
    B = torch.randn(R, N, device=DEV, generator=g)
    C = _native.gemm_tn(A, B)
    if R == 0:
        assert torch.all(C == 0)
        return
    _check(C, A.double().t(), B.double(), A.t() @ B, None, f"tn R={R} M={M} N={N}")


@pytest.mark.parametrize("R,M,N,mean", [(0, 8, 4, 0), (1, 256, 256, 0), (1000, 512, 256, 0), (70001, 256, 256, 0),
                                        (4099, 300, 100, 0), (231000, 256, 128, 3.0), (9000, 300, 300, 3.0)])
def test_gemm_tn_column_sums(R, M, N, mean):
    """colsum_a: the bias gradient (sum over rows of A) from the weight-gradient pass, vs fp64 with
    torch's fp32 column sum as the yardstick; the product must be unchanged by asking for it.
    Columns with a non-zero mean (the partial sums grow with the row count: cfg2's db_Q at 231k
    rows) stress the accumulation order — per-chunk sums Kahan-added."""
    g = torch.Generator(device=DEV).manual_seed(R + M)
    A = torch.randn(R, M, device=DEV, generator=g) + mean
    B = torch.randn(R, N, device=DEV, generator=g)
    C, cs = _native.gemm_tn(A, B, colsum=True)
    assert torch.equal(C, _native.gemm_tn(A, B))
    if R == 0:
        assert torch.all(cs == 0)
        return
    ref64 = A.double().sum(0)
    e_ours, e_torch = _rel(cs.double(), ref64), _rel(A.sum(0).double(), ref64)
    assert e_ours <= max(2 * e_torch, 1e-6), (e_ours, e_torch)
    assert torch.equal(cs, _native.gemm_tn(A, B, colsum=True)[1]), "column sums must be deterministic"


def test_gemm_tn_dynamic_range_strided_and_deterministic():
    g = torch.Generator(device=DEV).manual_seed(9)
    R = 50000
    A0 = torch.randn(R, 600, device=DEV, generator=g)
    A = A0[:, 40:552]                                       # lda = 600, 512 columns
    A *= torch.exp2(torch.randint(-40, 40, (1, 512), device=DEV, generator=g).float())
    B = torch.randn(R, 256, device=DEV, generator=g)
    B[20000:21000] *= 2.0 ** 30                             # a late row block raises the B scales
    B[:3000, :17] = 0                                       # leading zero rows of some B columns
    C1 = _native.gemm_tn(A, B)
    C2 = _native.gemm_tn(A, B)
    assert torch.equal(C1, C2), "TN GEMM must be run-to-run deterministic"
    _check(C1, A.double().t(), B.double(), A.t() @ B, None, "tn dynamic range")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("R,M,N", [(0, 8, 4), (1, 256, 256), (31, 32, 36), (1000, 512, 256), (70001, 256, 256),
                                   (4099, 300, 100), (20000, 128, 128), (66000, 512, 256)])
def test_gemm_tn16_vs_fp64(dt, R, M, N):
    """sir_gemm_tn16 (the autocast weight gradients): 16-bit A, B; every product exact in fp32, so
    the bar is the fp32 GEMM's on the widened values — vs fp64 of the same (exactly widened)
    values, torch's fp32 A.float()^T B.float() as the yardstick; column sums likewise; the product
    unchanged by asking for the column sums; run-to-run deterministic."""
    g = torch.Generator(device=DEV).manual_seed(R + 5 * M + N)
    A = torch.randn(R, M, device=DEV, generator=g).to(dt)
    B = torch.randn(R, N, device=DEV, generator=g).to(dt)
    C, cs = _native.gemm_tn16(A, B, colsum=True)
    if R == 0:
        assert torch.all(C == 0) and torch.all(cs == 0)
        return
    assert torch.equal(C, _native.gemm_tn16(A, B)), "product must not depend on colsum / must be deterministic"
    _check(C, A.double().t(), B.double(), A.float().t() @ B.float(), None, f"tn16 {dt} R={R} M={M} N={N}")
    ref64 = A.double().sum(0)
    e_ours, e_torch = _rel(cs.double(), ref64), _rel(A.float().sum(0).double(), ref64)
    assert e_ours <= max(2 * e_torch, 1e-6), (e_ours, e_torch)


@pytest.mark.parametrize("R,M,N", [(60000, 256, 128), (229532, 128, 128), (5000, 100, 300), (3000, 128, 512)])
def test_gemm_tn16_narrow_tiles_bit_identical(R, M, N, monkeypatch):
    """The 128 x 128-tile TN16 kernel (taken when M or N <= 128: config 2's H = 128 gradients) sums
    the same rows, chunks and MFMAs per output as the 256 x 256 one: bit-identical, column sums too."""
    g = torch.Generator(device=DEV).manual_seed(R + M + N)
    A = torch.randn(R, M, device=DEV, generator=g).to(torch.bfloat16)
    B = torch.randn(R, N, device=DEV, generator=g).to(torch.bfloat16)
    out = {}
    for v in ("1", "0"):
        monkeypatch.setenv("SIR_TN16_NARROW", v)
        out[v] = _native.gemm_tn16(A, B, colsum=True)
    assert torch.equal(out["1"][0], out["0"][0]) and torch.equal(out["1"][1], out["0"][1])
    _check(out["1"][0], A.double().t(), B.double(), A.float().t() @ B.float(), None, f"tn16 narrow R={R}")


def test_gemm_tn16_strided_and_wide_range():
    """lda > M (a column slice of a wider tensor, as dQK[:, :H]), values spread over many binades
    (bf16 keeps fp32's exponent range; no scaling is involved), and errors are loud."""
    g = torch.Generator(device=DEV).manual_seed(11)
    R = 40000
    A0 = torch.randn(R, 600, device=DEV, generator=g)
    A0 *= torch.exp2(torch.randint(-60, 60, (1, 600), device=DEV, generator=g).float())
    A = A0.to(torch.bfloat16)[:, 40:552]
    B = torch.randn(R, 256, device=DEV, generator=g).to(torch.bfloat16)
    C = _native.gemm_tn16(A, B)
    _check(C, A.double().t(), B.double(), A.float().t() @ B.float(), None, "tn16 strided wide range")
    with pytest.raises(RuntimeError, match="even"):
        _native.gemm_tn16(torch.zeros(10, 3, device=DEV, dtype=torch.bfloat16),
                          torch.zeros(10, 4, device=DEV, dtype=torch.bfloat16))


def test_gemm_errors_are_loud():
    A = torch.randn(10, 6, device=DEV)
    pk = _native.gemm_pack(torch.randn(8, 6, device=DEV))
    with pytest.raises(RuntimeError, match="multiples of 4"):
        _native.gemm_nt(A, pk)


# ---------------------------------------------------------------------------- 16-bit NT (autocast)
def _nt16_ref(A, W, bias, dt, trans):
    """fp64 of autocast's half-precision nn.Linear on the rounded operands: A.to(dt), W.to(dt),
    bias.to(dt) (each 16-bit product exact; fp64 sums)."""
    Wd = W.to(dt).double()
    B = Wd.t() if trans else Wd
    ref = A.to(dt).double() @ B.t()
    if bias is not None:
        ref = ref + bias.to(dt).double()
    return ref


@pytest.mark.parametrize("M,K,N", [(229532, 128, 128), (70001, 256, 128), (4133, 512, 96), (300, 128, 8)])
@pytest.mark.parametrize("a32,c32", [(False, False), (True, False), (False, True)])
def test_gemm_nt16_narrow_tiles_bit_identical(M, K, N, a32, c32, monkeypatch):
    """The 128-feature-tile NT16 kernel (taken for N <= 128: config 2's Y, G and dX) computes every
    output with the same chunks, MFMAs and epilogue as the 256-wide one: bit-identical (16-bit and
    fp32 outputs, the rounded A copy, bias, the dropout epilogue)."""
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(M + K + N)
    A = torch.randn(M, K, device=DEV, generator=g)
    if not a32:
        A = A.to(dt)
    W = torch.randn(N, K, device=DEV, generator=g) * K ** -0.5
    b = torch.randn(N, device=DEV, generator=g).to(dt).float()
    pk = _native.gemm_pack16(W, dt)
    out = {}
    for v in ("1", "0"):
        monkeypatch.setenv("SIR_NT16_NARROW", v)
        acopy = torch.full((M, K), 7.0, device=DEV, dtype=dt) if a32 else None
        C = _native.gemm_nt16(A, pk, b, torch.float32 if c32 else None, acopy, drop=(3, 0.25))
        out[v] = (C, acopy)
    assert torch.equal(out["1"][0], out["0"][0])
    if a32:
        assert torch.equal(out["1"][1], out["0"][1])


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("a32", [False, True])
@pytest.mark.parametrize("M,K,N,trans,with_bias", [(4133, 256, 512, False, True), (2000, 256, 256, False, True),
                                                   (517, 512, 256, True, False), (300, 256, 256, True, False),
                                                   (1000, 128, 104, False, True), (70, 256, 8, False, False),
                                                   (0, 256, 256, False, True), (33000, 256, 256, False, True)])
def test_gemm_nt16_vs_fp64(dt, a32, M, K, N, trans, with_bias):
    """sir_gemm_nt16 (the autocast forward projections and input gradients) against fp64 of the
    same rounded operands: the fp32-output result within the fp32 accumulation bound, the 16-bit
    output within one unit of its last place of the correctly rounded value (the fp32 sum may sit
    on the other side of a rounding boundary), and — for an fp32 A — the rounded copy equal to
    A.to(dt) bit for bit."""
    g = torch.Generator(device=DEV).manual_seed(M + 3 * K + N)
    A = torch.randn(M, K, device=DEV, generator=g)
    if not a32:
        A = A.to(dt)
    W = torch.randn(K, N, device=DEV, generator=g) if trans else torch.randn(N, K, device=DEV, generator=g)
    W *= K ** -0.5
    bias = torch.randn(N, device=DEV, generator=g) if with_bias else None
    pk = _native.gemm_pack16(W, dt, trans=trans)
    b = bias.to(dt).float() if bias is not None else None
    acopy = torch.full((M, K), 7.0, device=DEV, dtype=dt) if a32 else None
    C32 = _native.gemm_nt16(A, pk, b, torch.float32, acopy)
    C16 = _native.gemm_nt16(A, pk, b)
    assert C16.dtype == dt and C32.dtype == torch.float32
    if M == 0:
        return
    if a32:
        assert torch.equal(acopy, A.to(dt)), "rounded copy of A"
    ref = _nt16_ref(A, W, bias, dt, trans)
    absum = A.to(dt).double().abs() @ (W.to(dt).double().t() if trans else W.to(dt).double()).abs().t()
    err = (C32.double() - ref).abs()
    assert torch.all(err <= 4 * K * 2.0 ** -24 * absum + 1e-30), f"nt16 fp32 out: max err {err.max().item():.3e}"
    # 16-bit output: within 1 ulp of the correctly rounded reference
    r16 = ref.to(dt)
    ulp = (r16.double().abs() * 2.0 ** (-7 if dt == torch.bfloat16 else -10)).clamp_min(2.0 ** -126)
    d16 = (C16.double() - r16.double()).abs()
    assert torch.all(d16 <= ulp + 4 * K * 2.0 ** -24 * absum), f"nt16 16-bit out: max diff {d16.max().item():.3e}"
    assert torch.equal(C16, _native.gemm_nt16(A, pk, b)), "deterministic"


def test_gemm_nt16_strided_rows_and_errors():
    """lda > K (a column slice of a wider 16-bit tensor), ldc > N, and loud errors."""
    g = torch.Generator(device=DEV).manual_seed(12)
    A0 = torch.randn(5000, 640, device=DEV, generator=g).to(torch.bfloat16)
    A = A0[:, 64:320]
    W = torch.randn(256, 256, device=DEV, generator=g) * 0.0625
    pk = _native.gemm_pack16(W, torch.bfloat16)
    C = _native.gemm_nt16(A, pk, None, torch.float32)
    ref = A.double() @ W.to(torch.bfloat16).double().t()
    assert _rel(C.double(), ref) < 1e-6
    with pytest.raises(RuntimeError, match="bad shape"):
        _native.gemm_nt16(torch.zeros(10, 96, device=DEV, dtype=torch.bfloat16),
                          _native.gemm_pack16(torch.zeros(8, 96, device=DEV), torch.bfloat16))
    with pytest.raises(RuntimeError, match="multiples of 16 B"):     # 16-bit C rows in 16-B pieces
        _native.gemm_nt16(torch.zeros(10, 256, device=DEV, dtype=torch.bfloat16),
                          _native.gemm_pack16(torch.zeros(12, 256, device=DEV), torch.bfloat16))


@pytest.mark.parametrize("M,K,N", [(70001, 256, 256), (4099, 256, 512), (3001, 128, 256), (66000, 512, 256),
                                   (513, 256, 300), (1, 512, 256), (255, 128, 512)])
def test_gemm_nt_block_routes_wide_range_strided(M, K, N, monkeypatch):
    """The block-tiled NT kernels (persistent k_gemm_nt_p for K in {128, 256, 512}, N in (128, 512];
    tiled k_gemm_nt otherwise) within the fp64 bound on rows spanning 2^60 of range, rows whose maximum
    grows by 2^40 along K (the rescale branch), a strided C (the columns around it untouched) and a
    ragged last tile."""
    g = torch.Generator(device=DEV).manual_seed(M * 7 + K)
    A = torch.randn(M, K, device=DEV, generator=g)
    A *= torch.exp2(torch.randint(-30, 30, (M, 1), device=DEV, generator=g).float())
    if M > 300:
        A[100:300] *= torch.exp2(torch.linspace(-20, 20, K, device=DEV))
    W = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
    b = torch.randn(N, device=DEV, generator=g)
    pk = _native.gemm_pack(W)
    monkeypatch.setenv("SIR_GEMM_SMALL_ROWS", "0")   # block-tiled routes at every M (not k_gemm_nt_s)
    wide = torch.full((M, N + 12), 7.0, device=DEV)
    C = _native.gemm_nt(A, pk, b, out=wide[:, 4:4 + N])
    torch.cuda.synchronize()
    _check(C, A.double(), W.double().t(), torch.addmm(b, A, W.t()), b, f"nt block M={M} K={K} N={N}")
    assert torch.all(wide[:, :4] == 7.0) and torch.all(wide[:, 4 + N:] == 7.0)


# ---------------------------------------------------------------------------- small-batch route
# Below SIR_SMALL_ROWS (16384) node rows the NT / TN GEMMs run one wave per output tile
# (k_gemm_nt_s / k_gemm_tn_s: config 5's 1.6k-node molecule batches, config 1's 5k-node batches).
# SIR_GEMM_SMALL_ROWS in the environment moves the threshold per call: "0" forces the block-tiled
# kernels, a huge value the one-wave ones.
ROUTES = {"small": "1000000000", "block": "0"}


@pytest.mark.parametrize("M,K,N", [(1582, 256, 512), (1582, 512, 256), (5120, 128, 256), (1, 256, 300),
                                   (33, 128, 64), (70001, 256, 256), (4099, 64, 128), (3000, 1024, 96)])
@pytest.mark.parametrize("trans,with_bias,drop", [(False, True, False), (True, False, False), (False, True, True)])
def test_gemm_nt_small_route_bit_identical_to_block_route(M, K, N, trans, with_bias, drop, monkeypatch):
    """k_gemm_nt_s splits, scales and multiplies each row exactly as the block-tiled kernels do (same
    32-k chunks, same running scale, the three MFMAs in the same order per accumulator, the same
    epilogue arithmetic incl. the dropout mask): the two routes agree bit for bit, on rows spanning
    2^60 and rows whose maximum grows along K; both within the fp64 bound."""
    g = torch.Generator(device=DEV).manual_seed(M + 5 * K + N)
    A = torch.randn(M, K, device=DEV, generator=g)
    A *= torch.exp2(torch.randint(-30, 30, (M, 1), device=DEV, generator=g).float())
    if M > 300:
        A[100:300] *= torch.exp2(torch.linspace(-20, 20, K, device=DEV))
        A[17] = 0
    W = (torch.randn(K, N, device=DEV, generator=g) if trans else torch.randn(N, K, device=DEV, generator=g)) / K ** 0.5
    b = torch.randn(N, device=DEV, generator=g) if with_bias else None
    pk = _native.gemm_pack(W, trans=trans)
    dr = (1234, 0.25) if drop else None
    outs = {}
    for name, v in ROUTES.items():
        monkeypatch.setenv("SIR_GEMM_SMALL_ROWS", v)
        outs[name] = _native.gemm_nt(A, pk, b, drop=dr)
    assert torch.equal(outs["small"], outs["block"]), \
        f"small vs block route differ: relL2 {_rel(outs['small'].double(), outs['block'].double()):.2e}"
    if not drop:
        Wt = W if trans else W.t()
        ref = torch.addmm(b, A, Wt) if with_bias else A @ Wt
        _check(outs["small"], A.double(), Wt.double(), ref, b, f"nt small M={M} K={K} N={N}")


@pytest.mark.parametrize("M,K,N", [(1582, 300, 600), (1582, 600, 300), (777, 36, 132), (5, 300, 300),
                                   (2000, 100, 12)])
def test_gemm_nt_small_route_ragged_k(M, K, N, monkeypatch):
    """K not a multiple of 32 (config 5: H = 300): the last chunk's columns past K (the next row's
    values, or past the buffer) must not enter the row scale or the products; vs fp64, and an
    A slice of a wider tensor (lda > K) whose neighbouring columns hold huge values."""
    monkeypatch.setenv("SIR_GEMM_SMALL_ROWS", ROUTES["small"])
    g = torch.Generator(device=DEV).manual_seed(M + K)
    A0 = torch.full((M, K + 8), 3e37, device=DEV)
    A = A0[:, 4:4 + K]
    A.copy_(torch.randn(M, K, device=DEV, generator=g))
    W = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
    b = torch.randn(N, device=DEV, generator=g)
    C = _native.gemm_nt(A, _native.gemm_pack(W), b)
    _check(C, A.double(), W.double().t(), torch.addmm(b, A, W.t()), b, f"nt small ragged M={M} K={K} N={N}")


@pytest.mark.parametrize("R,M,N", [(0, 8, 4), (1, 300, 300), (37, 64, 128), (1582, 600, 300), (1582, 300, 300),
                                   (5120, 128, 64), (16000, 256, 256), (70, 36, 100)])
@pytest.mark.parametrize("route", ["small", "block"])
def test_gemm_tn_small_and_block_routes_vs_fp64(R, M, N, route, monkeypatch):
    """k_gemm_tn_s (one wave per 32 x 64 tile, >= 1024 waves over row splits) and the block-tiled
    k_gemm_tn on the same small-batch shapes: vs fp64 on columns spanning 2^60, a late row block that
    raises the B scales, leading zero rows; column sums (the bias gradient) vs fp64; run-to-run
    deterministic, and the product unchanged by asking for the column sums."""
    monkeypatch.setenv("SIR_GEMM_SMALL_ROWS", ROUTES[route])
    g = torch.Generator(device=DEV).manual_seed(R + 3 * M + N)
    A = torch.randn(R, M, device=DEV, generator=g)
    A *= torch.exp2(torch.randint(-30, 30, (1, M), device=DEV, generator=g).float())
    B = torch.randn(R, N, device=DEV, generator=g)
    if R > 100:
        B[R // 2:R // 2 + 40] *= 2.0 ** 30
        B[:50, :7] = 0
    C, cs = _native.gemm_tn(A, B, colsum=True)
    if R == 0:
        assert torch.all(C == 0) and torch.all(cs == 0)
        return
    assert torch.equal(C, _native.gemm_tn(A, B)), "deterministic / independent of colsum"
    _check(C, A.double().t(), B.double(), A.t() @ B, None, f"tn {route} R={R} M={M} N={N}")
    ref64 = A.double().sum(0)
    e_ours, e_torch = _rel(cs.double(), ref64), _rel(A.sum(0).double(), ref64)
    assert e_ours <= max(2 * e_torch, 1e-6), (e_ours, e_torch)


@pytest.mark.parametrize("M,K,N", [(1582, 300, 600), (1582, 300, 300), (1582, 600, 300), (5120, 64, 128),
                                   (1, 256, 256), (33, 36, 12), (8191, 512, 256), (2000, 1024, 96)])
@pytest.mark.parametrize("trans,with_bias", [(False, True), (True, False), (False, False)])
def test_gemm_nt_direct_vs_fp64(M, K, N, trans, with_bias):
    """sir_gemm_nt_direct (the small-batch route of nn.Linear: the fp32 weight split in the kernel,
    running scales on both operands; the LDS-tiled k_gemm_lt by default) vs fp64, on rows and
    weight rows spanning 2^60, rows whose maximum grows along K, a zero row; strided A (lda > K)."""
    g = torch.Generator(device=DEV).manual_seed(M + 7 * K + N)
    A0 = torch.randn(M, K + 8, device=DEV, generator=g)
    A = A0[:, 4:4 + K]
    A *= torch.exp2(torch.randint(-30, 30, (M, 1), device=DEV, generator=g).float())
    if M > 300:
        A[100:300] *= torch.exp2(torch.linspace(-20, 20, K, device=DEV))
        A[17] = 0
    W = (torch.randn(K, N, device=DEV, generator=g) if trans else torch.randn(N, K, device=DEV, generator=g)) / K ** 0.5
    W *= torch.exp2(torch.randint(-15, 15, (1, N) if trans else (N, 1), device=DEV, generator=g).float())
    b = torch.randn(N, device=DEV, generator=g) if with_bias else None
    C = _native.gemm_nt_direct(A, W, trans, b)
    Wt = W if trans else W.t()
    ref = torch.addmm(b, A, Wt) if with_bias else A @ Wt
    _check(C, A.double(), Wt.double(), ref, b, f"nt direct M={M} K={K} N={N} trans={trans}")
    assert torch.equal(C, _native.gemm_nt_direct(A, W, trans, b)), "deterministic"


@pytest.mark.parametrize("cfg", ["0", "1", "2", "3", "4", "5", "6", "7", "8"])
@pytest.mark.parametrize("M,K,N", [(1582, 300, 600), (1582, 600, 300), (33, 36, 12), (97, 68, 132), (1, 32, 4)])
@pytest.mark.parametrize("trans", [False, True])
def test_gemm_nt_direct_lt_arrangements(cfg, M, K, N, trans, monkeypatch):
    """Every wave arrangement of the LDS-tiled small kernel (SIR_LT_NT: 1 = 2x2 tiles, 2 = 1x2 tiles x
    2 k-ways, 3 = 2x1 x 2, 4 = 1 tile x 4 k-ways, 5 = 1x4; 8 waves: 6 = 2x1 x 4, 7 = 1x2 x 4, 8 = 2x2 x 2;
    0 = the 4-wave k_gemm_nt_sw) vs fp64 with
    bias and dropout, ragged tiles, a row whose scale grows along K; a weight view not 16-byte aligned
    takes k_gemm_nt_sw whatever the setting."""
    monkeypatch.setenv("SIR_LT_NT", cfg)
    g = torch.Generator(device=DEV).manual_seed(M + K + N + int(cfg))
    A = torch.randn(M, K, device=DEV, generator=g)
    A *= torch.exp2(torch.randint(-20, 20, (M, 1), device=DEV, generator=g).float())
    A[M // 2] *= torch.exp2(torch.linspace(-20, 20, K, device=DEV))
    W = (torch.randn(K, N, device=DEV, generator=g) if trans else torch.randn(N, K, device=DEV, generator=g)) / K ** 0.5
    b = torch.randn(N, device=DEV, generator=g)
    Wt = W if trans else W.t()
    C = _native.gemm_nt_direct(A, W, trans, b)
    _check(C, A.double(), Wt.double(), torch.addmm(b, A, Wt), b, f"nt lt{cfg} M={M} K={K} N={N} trans={trans}")
    if not trans:
        Cd = _native.gemm_nt_direct(A, W, False, b, drop=(5, 0.25))
        keep = Cd != 0
        assert torch.equal(Cd[keep], C[keep] * (1.0 / 0.75))
    # 4-byte-aligned weight view (k_gemm_nt_sw)
    Wb = torch.empty(W.numel() + 1, device=DEV)[1:].view_as(W).copy_(W)
    C2 = _native.gemm_nt_direct(A, Wb, trans, b)
    _check(C2, A.double(), Wt.double(), torch.addmm(b, A, Wt), b, f"nt unaligned lt{cfg}")


@pytest.mark.parametrize("cfg", ["0", "1", "2", "3", "4", "5"])
@pytest.mark.parametrize("R,M,N", [(1582, 600, 300), (1582, 300, 300), (37, 64, 128), (70, 36, 100), (3000, 4, 8)])
def test_gemm_tn_small_lt_arrangements(cfg, R, M, N, monkeypatch):
    """The small TN route per LDS arrangement (SIR_LT_TN: 1 = 2x2 tiles, 2 = 1x2 x 2 k-ways, 3 = 1 x 4
    k-ways; 8 waves: 4 = 1x2 x 4, 5 = 2x2 x 2; 0 = k_gemm_tn_s): product and column sums vs fp64,
    deterministic, ragged rows and tiles."""
    monkeypatch.setenv("SIR_LT_TN", cfg)
    monkeypatch.setenv("SIR_GEMM_SMALL_ROWS", ROUTES["small"])
    g = torch.Generator(device=DEV).manual_seed(R + M + N + int(cfg))
    A = torch.randn(R, M, device=DEV, generator=g)
    A *= torch.exp2(torch.randint(-30, 30, (1, M), device=DEV, generator=g).float())
    B = torch.randn(R, N, device=DEV, generator=g)
    B[R // 2:R // 2 + 20] *= 2.0 ** 20
    C, cs = _native.gemm_tn(A, B, colsum=True)
    assert torch.equal(C, _native.gemm_tn(A, B)), "deterministic / independent of colsum"
    _check(C, A.double().t(), B.double(), A.t() @ B, None, f"tn lt{cfg} R={R} M={M} N={N}")
    # column sums per column against sum |a| (a relative L2 over a few columns is decided by the one
    # whose sum cancels most): the fp32 chain of 16 plain adds + compensated adds stays <= 2e-7
    ref64, absum = A.double().sum(0), A.double().abs().sum(0)
    e_ours = ((cs.double() - ref64).abs() / absum).max().item()
    e_torch = ((A.sum(0).double() - ref64).abs() / absum).max().item()
    assert e_ours <= max(2 * e_torch, 2e-7), (e_ours, e_torch)


@pytest.mark.parametrize("M,n1,n2,K", [(1582, 300, 300, 300), (97, 36, 100, 68), (1, 4, 8, 4), (4099, 128, 64, 256)])
@pytest.mark.parametrize("trans", [False, True])
def test_gemm_nt_direct2_two_part_weight_bit_identical(M, n1, n2, K, trans):
    """sir_gemm_nt_direct2 reads [W; W2] in place (split inside a tile for 300 = 4 x 64 + 44) and adds
    the bias to the first rows' outputs only: the same bits as sir_gemm_nt_direct on the
    concatenated weight with the zero-padded bias (dropout included)."""
    g = torch.Generator(device=DEV).manual_seed(M + n1 + n2 + K)
    if trans:   # weight [K1 + K2, N]: A has K1 + K2 columns
        A = torch.randn(M, n1 + n2, device=DEV, generator=g)
        W = torch.randn(n1, K, device=DEV, generator=g)
        W2 = torch.randn(n2, K, device=DEV, generator=g)
        ref = _native.gemm_nt_direct(A, torch.cat([W, W2], 0), True)
        got = _native.gemm_nt_direct2(A, W, W2, True)
        assert torch.equal(got, ref)
        return
    A = torch.randn(M, K, device=DEV, generator=g)
    W = torch.randn(n1, K, device=DEV, generator=g)
    W2 = torch.randn(n2, K, device=DEV, generator=g)
    b = torch.randn(n1, device=DEV, generator=g)
    Wc, bc = torch.cat([W, W2], 0), torch.nn.functional.pad(b, (0, n2))
    for drop in (None, (9, 0.3)):
        ref = _native.gemm_nt_direct(A, Wc, False, bc, drop=drop)
        got = _native.gemm_nt_direct2(A, W, W2, False, b, drop=drop)
        assert torch.equal(got, ref)
    assert torch.equal(_native.gemm_nt_direct2(A, W, W2), _native.gemm_nt_direct(A, Wc, False))
    with pytest.raises(RuntimeError, match="split"):
        _native.gemm_nt_direct2(A, W[:0], W2, False)


@pytest.mark.parametrize("lt", ["0", "-1"])
def test_pair_projections_fall_back_off_the_lds_kernel(lt, monkeypatch):
    """linalg.mm_wt_pair / mm_w_pair (the layer's QK and dX on small batches) take the two-part
    weight only where the LDS-tiled kernel runs; with it switched off (SIR_LT_NT=0) they take the
    cat + pad route instead of raising (advisor r05 finding) and return the same product."""
    from sirgcn import linalg
    monkeypatch.setenv("SIR_LT_NT", lt)
    g = torch.Generator(device=DEV).manual_seed(5)
    M, d, H = 1582, 300, 300
    X = torch.randn(M, d, device=DEV, generator=g)
    WQ, WK = torch.randn(H, d, device=DEV, generator=g), torch.randn(H, d, device=DEV, generator=g)
    bQ = torch.randn(H, device=DEV, generator=g)
    qk = linalg.mm_wt_pair(X, WQ, WK, bQ)
    ref = torch.cat([X.double() @ WQ.double().t() + bQ.double(), X.double() @ WK.double().t()], 1)
    assert _rel(qk.double(), ref) < 1e-6
    dQK = torch.randn(M, 2 * H, device=DEV, generator=g)
    dX = linalg.mm_w_pair(dQK, WQ, WK)
    assert _rel(dX.double(), dQK.double() @ torch.cat([WQ, WK], 0).double()) < 1e-6


def test_gemm_nt_direct_dropout_epilogue_and_errors():
    """The QK dropout in the direct kernel's epilogue: the kept entries are exactly the undropped
    result times 1/(1-p), the same hashed mask as the packed-weight kernels, ~p dropped."""
    g = torch.Generator(device=DEV).manual_seed(3)
    A = torch.randn(1582, 300, device=DEV, generator=g)
    W = torch.randn(600, 300, device=DEV, generator=g) / 17.0
    b = torch.randn(600, device=DEV, generator=g)
    p = 0.2
    C0 = _native.gemm_nt_direct(A, W, False, b)
    Cd = _native.gemm_nt_direct(A, W, False, b, drop=(77, p))
    Cp = _native.gemm_nt(A, _native.gemm_pack(W), b, drop=(77, p))
    keep = Cd != 0
    assert torch.equal(keep, Cp != 0), "same mask as the packed-weight kernel"
    assert torch.equal(Cd[keep], C0[keep] * (1.0 / (1.0 - p)))
    frac = 1.0 - keep.float().mean().item()
    assert abs(frac - p) < 0.01, frac
    with pytest.raises(RuntimeError, match="multiples of 4"):
        _native.gemm_nt_direct(torch.zeros(10, 6, device=DEV), torch.zeros(8, 6, device=DEV))


@pytest.mark.parametrize("M,K,N", [(40000, 256, 256), (20000, 512, 256), (20000, 256, 64), (3000, 256, 256)])
@pytest.mark.parametrize("act,slope", [(_native.ACT_LEAKY, 0.2), (_native.ACT_RELU, 0.0)])
def test_gemm_nt_dact_equals_gemm_then_activation_backward(M, K, N, act, slope):
    """sir_gemm_nt_dact (sigma'(gate) applied in k_gemm_nt_p's epilogue, or after the GEMM on the other
    routes) is bit-identical to the native packed-weight GEMM followed by torch's threshold /
    leaky_relu backward."""
    from sirgcn import linalg
    g = torch.Generator(device="cuda").manual_seed(M + N)
    A = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(K, N, device="cuda", generator=g) / K ** 0.5
    gate = torch.randn(M, N, device="cuda", generator=g)
    got = linalg.mm_w_dact(A, W, gate, act, slope)
    ref = _native.gemm_nt(A, _native.gemm_pack(W, trans=True))
    ref = (torch.ops.aten.threshold_backward(ref, gate, 0.0) if act == _native.ACT_RELU
           else torch.ops.aten.leaky_relu_backward(ref, gate, slope, False))
    assert torch.equal(got, ref)
    if N == 256:                            # the gate as sign words (sir_edge_gather_act's mask)
        bits = (gate > 0).reshape(M, 64, 4).permute(0, 2, 1).long()
        words = (bits << torch.arange(64, device="cuda")).sum(-1).contiguous()
        got_m = linalg.mm_w_dact(A, W, gate, act, slope, gate_mask=words)
        assert torch.equal(got_m, ref)
