// sirconv_gemm16.hip — the weight-gradient GEMMs of the autocast path (conv.py:60-61,65 under
// torch.autocast, heterophilous-datasets/train.py:75) on 16-bit operands:
//   part[p] = A[rows_p]^T B[rows_p],  A [R, Mc], B [R, Nc] bf16 or fp16, fp32 result,
// i.e. dW_R = dY^T S and [dW_Q; dW_K] = [dQ dK]^T X with dY, S, dQK, X as the 16-bit tensors the
// autocast layer holds.  A product of two bf16 (or two fp16) values is exact in fp32, so ONE
// v_mfma_f32_32x32x16_{bf16,f16} per 32x32x16 step with fp32 accumulation gives the accuracy of
// the fp32 split GEMM run on the widened values (which splits every 16-bit value into hi = value,
// lo = 0) at a third of the MFMA work, half the bytes, and with no fp32 copies of the operands.
//
// Tiling (per 512-thread block, one (row split p, 256 x 256 output tile)): 2 x 4 waves, 128 x 64
// outputs per wave (4 x 2 MFMA tiles).  Chunks of 32 node rows: a thread loads one column PAIR
// (one dword) of 16 rows — a wave instruction reads 256 contiguous bytes of a row — and
// transposes the pair in registers (v_perm) into two fragment pieces of 8 rows per column,
// stored in the fimg LDS order (conflict-free ds_read_b128 operands).  Three register sets keep
// two to three chunks' loads in flight while the current chunk is multiplied; the steady-state
// steps carry no conditional load (a load skipped on one path makes the compiler's wait-count
// merge drain the queue), rows past the split's end read as 0 through the buffer range check.
// The column sums of A (the bias gradient of the same linear) are summed from the loaded
// values in fp32, in row order.  Partials are added in split order by k_gemm_reduce
// (sirconv_gemm.hip): deterministic.
#include "sirconv.h"
#include "sirconv_internal.h"
#include "sirconv_gemm_util.h"

namespace sir {
namespace {
using namespace gemm;

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

constexpr int KC16 = 32;       // node rows per chunk (two k16 MFMA steps)
constexpr int NSET = 3;        // register sets of chunk loads

template <bool BF>
__device__ inline f16v mfma16(u4v a, u4v b, f16v c) {
    if constexpr (BF)
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}

template <bool BF>
__device__ inline float widen(uint32_t bits16) {
    if constexpr (BF)
        return __uint_as_float(bits16 << 16);
    else
        return (float)__builtin_bit_cast(_Float16, (unsigned short)bits16);
}

template <bool BF>
__global__ void __launch_bounds__(512)
k_gemm_tn16(const unsigned short* __restrict__ A, int64_t lda, const unsigned short* __restrict__ B, int64_t ldb,
            int64_t R, int Mc, int Nc, float* __restrict__ part, float* __restrict__ csum_part, int n_mtiles,
            int n_ntiles, int64_t rows_per_split) {
    constexpr int WN = 4, TMT = 4, TNT = 2;
    constexpr int BM = 256, BN = 256;
    constexpr int PLANE_A = BM * 32, PLANE_B = BN * 32;          // one k16 step: 32 B per column
    constexpr int A_BYTES = 2 * PLANE_A, B_BYTES = 2 * PLANE_B;
    constexpr int STAGE = A_BYTES + B_BYTES;
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

    const int t = threadIdx.x;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int tiles = n_mtiles * n_ntiles;
    const int p = wg / tiles, tile = wg % tiles;
    const int m0 = (tile / n_ntiles) * BM, n0 = (tile % n_ntiles) * BN;
    const int64_t v_begin = (int64_t)p * rows_per_split;
    const int64_t v_end = (v_begin + rows_per_split < R) ? v_begin + rows_per_split : R;
    const int nc = v_end > v_begin ? (int)((v_end - v_begin + KC16 - 1) / KC16) : 0;

    // loader: slot = column pair (slots [0, 128) of A, [128, 256) of B: wave-uniform), kse = which
    // 16 rows of the chunk (= the k16 step whose plane the pair's pieces go to)
    const int slot = t & 255, kse = t >> 8;
    const bool is_a = (__builtin_amdgcn_readfirstlane(t >> 6) & 2) == 0;    // slot < 128, wave-uniform
    const int pr = is_a ? slot : slot - BM / 2;
    const int c0 = 2 * pr;
    const bool col_ok = is_a ? (m0 + c0 < Mc) : (n0 + c0 < Nc);
    const unsigned short* xbase = is_a ? A : B;
    const int64_t ldx = is_a ? lda : ldb;
    const int voff = ((is_a ? m0 : n0) + (col_ok ? c0 : 0)) * 2 + kse * 16 * (int)ldx * 2;
    const int img = (is_a ? 0 : A_BYTES) + kse * (is_a ? PLANE_A : PLANE_B);

    const int w = t >> 6, l = t & 63, r = l & 31, h = l >> 5;
    const int m_w = (w / WN) * TMT * 32, n_w = (w % WN) * TNT * 32;

    const int rstride = (int)ldx * 2;
    uint32_t xs[NSET][16];
    auto load = [&](int set, int c) {
        const int64_t vc = v_begin + (int64_t)c * KC16;
        const int64_t nrow = v_end - vc;
        // one resource per chunk: rows past v_end (and chunks past the split) read as 0
        const rsrc_t rs = mk_rsrc(xbase + vc * ldx, nrow <= 0 ? 0u : (uint32_t)((nrow < KC16 ? nrow : KC16) * ldx * 2));
        // row offsets stepped in one SGPR (the compiler would otherwise keep all 16 live)
        int so = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            xs[set][j] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, so, 0);
            so += rstride;
            asm volatile("" : "+s"(so));
        }
    };
    float cs0 = 0.f, cs1 = 0.f;
    const bool do_cs = csum_part != nullptr && is_a;
    auto store = [&](int set, int buf) {
        char* st = lds + buf * STAGE + img;
        u4v lo0, lo1, hi0, hi1;       // column c0 (low halves) / c0 + 1 (high halves), rows 0-7 / 8-15
        uint32_t* q[4] = {(uint32_t*)&lo0, (uint32_t*)&lo1, (uint32_t*)&hi0, (uint32_t*)&hi1};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            q[0][i] = __builtin_amdgcn_perm(xs[set][2 * i + 1], xs[set][2 * i], 0x05040100u);
            q[1][i] = __builtin_amdgcn_perm(xs[set][2 * i + 9], xs[set][2 * i + 8], 0x05040100u);
            q[2][i] = __builtin_amdgcn_perm(xs[set][2 * i + 1], xs[set][2 * i], 0x07060302u);
            q[3][i] = __builtin_amdgcn_perm(xs[set][2 * i + 9], xs[set][2 * i + 8], 0x07060302u);
        }
        *reinterpret_cast<u4v*>(st + fimg(c0, 0)) = lo0;
        *reinterpret_cast<u4v*>(st + fimg(c0, 1)) = lo1;
        *reinterpret_cast<u4v*>(st + fimg(c0 + 1, 0)) = hi0;
        *reinterpret_cast<u4v*>(st + fimg(c0 + 1, 1)) = hi1;
        if (do_cs) {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                cs0 += widen<BF>(xs[set][j] & 0xffffu);
                cs1 += widen<BF>(xs[set][j] >> 16);
            }
        }
    };

    f16v acc[TMT][TNT];
#pragma unroll
    for (int a = 0; a < TMT; ++a)
#pragma unroll
        for (int b = 0; b < TNT; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

    auto mfma = [&](int buf) {
        const char* st = lds + buf * STAGE;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            u4v af[TMT], bf[TNT];
#pragma unroll
            for (int a = 0; a < TMT; ++a)
                af[a] = *reinterpret_cast<const u4v*>(st + ks * PLANE_A + fimg(m_w + 32 * a + r, h));
#pragma unroll
            for (int b = 0; b < TNT; ++b)
                bf[b] = *reinterpret_cast<const u4v*>(st + A_BYTES + ks * PLANE_B + fimg(n_w + 32 * b + r, h));
#pragma unroll
            for (int a = 0; a < TMT; ++a)
#pragma unroll
                for (int b = 0; b < TNT; ++b) acc[a][b] = mfma16<BF>(af[a], bf[b], acc[a][b]);
        }
    };

    // step c: set c % 3 is free (chunk c is in LDS buffer c & 1), sets (c+1) % 3, (c+2) % 3 hold
    // chunks c+1, c+2 in flight.  Issue chunk c+3, multiply chunk c, then write chunk c+1 into the
    // other buffer (its wait leaves chunks c+2, c+3 in flight).
    auto step_full = [&](int c, int s) {
        load(s, c + 3);
        mfma(c & 1);
        store((s + 1) % NSET, (c + 1) & 1);
        __syncthreads();
    };
    auto step_tail = [&](int c, int s) {
        mfma(c & 1);
        if (c + 1 < nc) store((s + 1) % NSET, (c + 1) & 1);
        __syncthreads();
    };
    if (nc > 0) {
        load(0, 0);
        load(1, 1);
        load(2, 2);
        store(0, 0);
        __syncthreads();
        int c = 0;
        for (; c + 3 < nc; c += 3) {
            step_full(c, 0);
            step_full(c + 1, 1);
            step_full(c + 2, 2);
        }
        step_tail(c, 0);
        if (c + 1 < nc) step_tail(c + 1, 1);
        if (c + 2 < nc) step_tail(c + 2, 2);
    }

    float* out = part + (int64_t)p * Mc * Nc;
#pragma unroll
    for (int b = 0; b < TNT; ++b) {
        const int n = n0 + n_w + 32 * b + r;
#pragma unroll
        for (int a = 0; a < TMT; ++a) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int m = m0 + m_w + 32 * a + (i & 3) + 8 * (i >> 2) + 4 * h;
                if (m < Mc && n < Nc) out[(int64_t)m * Nc + n] = acc[a][b][i];
            }
        }
    }
    if (csum_part != nullptr && tile % n_ntiles == 0) {
        // rows 0-15 (kse 0) + rows 16-31 (kse 1) of every chunk, through LDS (partners in other waves)
        float* cl = reinterpret_cast<float*>(lds);
        __syncthreads();
        if (is_a && kse == 1) { cl[c0] = cs0; cl[c0 + 1] = cs1; }
        __syncthreads();
        if (is_a && kse == 0) {
            if (m0 + c0 < Mc) csum_part[(int64_t)p * Mc + m0 + c0] = cs0 + cl[c0];
            if (m0 + c0 + 1 < Mc) csum_part[(int64_t)p * Mc + m0 + c0 + 1] = cs1 + cl[c0 + 1];
        }
    }
}

}  // namespace

hipError_t run_gemm_tn16(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t R, int Mc, int Nc, int dtype,
                         float* C, int64_t ldc, float* colsum, void* workspace, hipStream_t st) {
    if (Mc == 0 || Nc == 0) return hipSuccess;
    const int P = gemm_tn_splits(R, Mc, Nc);
    const int64_t rps = (R + P - 1) / P;
    const int nmt = (Mc + 255) / 256, nnt = (Nc + 255) / 256;
    float* part = static_cast<float*>(workspace);
    float* cpart = colsum != nullptr ? part + (int64_t)P * Mc * Nc : nullptr;
    const auto* a = static_cast<const unsigned short*>(A);
    const auto* b = static_cast<const unsigned short*>(B);
    const dim3 grid((unsigned)(P * nmt * nnt));
    if (dtype == SIR_DTYPE_BF16)
        hipLaunchKernelGGL(k_gemm_tn16<true>, grid, dim3(512), 0, st, a, lda, b, ldb, R, Mc, Nc, part, cpart, nmt, nnt,
                           rps);
    else
        hipLaunchKernelGGL(k_gemm_tn16<false>, grid, dim3(512), 0, st, a, lda, b, ldb, R, Mc, Nc, part, cpart, nmt, nnt,
                           rps);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = run_gemm_reduce(part, P, (int64_t)Mc * Nc, Nc, C, ldc, st);
    if (e != hipSuccess || colsum == nullptr) return e;
    return run_gemm_reduce(cpart, P, (int64_t)Mc, Mc, colsum, 0, st);
}

}  // namespace sir
