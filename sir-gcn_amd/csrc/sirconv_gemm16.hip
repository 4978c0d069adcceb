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
#include "sirconv_dropout.h"

#include <type_traits>

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

// x rounded to the 16-bit output type (identity for an fp32 output)
template <bool BF, bool C32>
__device__ inline float rnd16(float x) {
    if constexpr (C32) return x;
    else if constexpr (BF) return (float)(__bf16)x;
    else return (float)(_Float16)x;
}

template <bool BF>
__device__ inline float widen(uint32_t bits16) {
    if constexpr (BF)
        return __uint_as_float(bits16 << 16);
    else
        return (float)__builtin_bit_cast(_Float16, (unsigned short)bits16);
}

// BM x BN output tile per block of BM + BN threads: 256 x 256 (8 waves of 128 x 64, TMT x TNT = 4 x 2
// MFMA tiles) or, for the narrow gradients of H <= 128 layers (config 2's 128 x 128 and 256 x 128),
// 128 x 128 (4 waves of 64 x 64) — the 256-wide tile left three quarters of its MFMAs and half its
// loads on columns past Mc / Nc there.
template <bool BF, int BM = 256, int BN = 256, int WN = 4, int TMT = 4, int TNT = 2>
__global__ void __launch_bounds__(BM + BN)
k_gemm_tn16(const unsigned short* __restrict__ A, int64_t lda, const unsigned short* __restrict__ B, int64_t ldb,
            int64_t R, int Mc, int Nc, float* __restrict__ part, float* __restrict__ csum_part, int n_mtiles,
            int n_ntiles, int64_t rows_per_split) {
    constexpr int SLOTS = BM / 2 + BN / 2;                       // column pairs per block (a power of 2)
    constexpr int PLANE_A = BM * 32, PLANE_B = BN * 32;          // one k16 step: 32 B per column
    constexpr int A_BYTES = 2 * PLANE_A, B_BYTES = 2 * PLANE_B;
    constexpr int STAGE = A_BYTES + B_BYTES;
    static_assert((SLOTS & (SLOTS - 1)) == 0 && (BM / 2) % 64 == 0, "slot layout");
    static_assert((BM / (TMT * 32)) * (BN / (TNT * 32)) == (BM + BN) / 64 && BN / (TNT * 32) == WN, "wave tiling");
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

    const int t = threadIdx.x;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int tiles = n_mtiles * n_ntiles;
    const int p = wg / tiles, tile = wg % tiles;
    const int m0 = (tile / n_ntiles) * BM, n0 = (tile % n_ntiles) * BN;
    const int64_t v_begin = (int64_t)p * rows_per_split;
    const int64_t v_end = (v_begin + rows_per_split < R) ? v_begin + rows_per_split : R;
    const int nc = v_end > v_begin ? (int)((v_end - v_begin + KC16 - 1) / KC16) : 0;

    // loader: slot = column pair (slots [0, BM/2) of A, the rest of B: wave-uniform), kse = which
    // 16 rows of the chunk (= the k16 step whose plane the pair's pieces go to)
    const int slot = t & (SLOTS - 1), kse = t / SLOTS;
    const bool is_a = (__builtin_amdgcn_readfirstlane(t >> 6) % (SLOTS / 64)) < (BM / 2) / 64;   // wave-uniform
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

// ------------------------------------------------------------------------------------------
// NT GEMM on 16-bit MFMA: the autocast layer's forward projections and input gradients
// (QK = X [W_Q; W_K]^T + b, Y = S W_R^T + b, G = dY W_R, dX = dQK [W_Q; W_K]):
//   C[M, N] = A[M, K] B[N, K]^T (+ bias),  B packed 16-bit in fragment order (k_pack16),
// A in the 16-bit type, or fp32 rounded (RNE) to it on load — the autocast cast X.to(dt) fused
// into the GEMM; the rounded copy can be written out (Acopy, the first feature tile only) for the
// weight-gradient GEMM.  C in the 16-bit type (RNE of the fp32 accumulator, what the library
// GEMM returns) or fp32 (dX: the fp32 gradient of an fp32 input, without the 16-bit rounding and
// the separate .to(float32) pass).  One 16-bit MFMA per 32x32x16 step, fp32 accumulation.
//
// Persistent: one 512-thread block per CU walks a contiguous range of 256 x 256 output tiles;
// 8 waves, 128 x 64 outputs each (4 x 2 MFMA tiles, MFMA rows = features, columns = data rows).
// Chunks of KC k-values: a thread loads half of one row's chunk (KC/2 values) and the same
// number of packed weight bytes into a register set, two sets alternate (two chunks in flight
// while one is multiplied out of LDS), and the pipeline runs on across tile boundaries.
#ifndef SIR_NT16_EPI
#define SIR_NT16_EPI 1          // 16-bit NT epilogue through LDS with whole-row stores (1) or fragment stores (0)
#endif
#ifndef SIR_NT16_ABL
#define SIR_NT16_ABL 0          // timing-only ablations: 1 = A loads dropped, 2 = C stores dropped, 4 = no MFMAs
#endif

template <int I, int N_, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N_) {
        f(std::integral_constant<int, I>());
        static_for<I + 1, N_>(f);
    }
}

__device__ inline uint32_t pack2(float a, float b, bool bf) {
    if (bf) return (uint32_t)__builtin_bit_cast(unsigned short, (__bf16)a) |
                   ((uint32_t)__builtin_bit_cast(unsigned short, (__bf16)b) << 16);
    return (uint32_t)__builtin_bit_cast(unsigned short, (_Float16)a) |
           ((uint32_t)__builtin_bit_cast(unsigned short, (_Float16)b) << 16);
}

template <bool BF, bool A32, bool C32, int KC, int NC, int NS, int BFT = 256>
__global__ void __launch_bounds__(512)
k_gemm_nt16(const void* __restrict__ A, int64_t lda, int64_t M, const u4v* __restrict__ Wp, int Npad,
            const float* __restrict__ bias, int N, void* __restrict__ C, int64_t ldc, unsigned short* __restrict__ Acopy,
            int64_t ldac, int n_ftiles, int n_tiles, int tiles_per_block, Drop drop) {
    drop = drop_resolve(drop);
    // BFT features per tile: 256, or 128 for the narrow outputs of H <= 128 layers (config 2's Y, G
    // and dX), where the 256-wide tile spent half its MFMAs and weight loads past N
    constexpr int BD = 256, TFT = 2, WF = BFT / (TFT * 32), WD = 8 / WF, TDT = BD / (WD * 32);
    constexpr int KS = KC / 16;                       // k16 planes per chunk
    constexpr int PLANE = 256 * 32;                   // one k16 plane of the 256 data rows
    constexpr int PLANE_W = BFT * 32;                 // one k16 plane of the tile's weight rows
    constexpr int STAGE = KS * (PLANE + PLANE_W);     // A planes, then W planes
    constexpr int EA = A32 ? 4 : 2;                   // bytes per A element
    constexpr int AV = (KC / 2) * EA / 16;            // u4v A loads per thread and chunk
    constexpr int WV = KS * PLANE_W / (16 * 512);     // u4v W pieces per thread and chunk
    constexpr int EC = C32 ? 4 : 2;
    static_assert(KC == 32 || KC == 64, "chunk");
    static_assert(BFT == 256 || BFT == 128, "feature tile");
    static_assert(WV >= 1, "weight loader");
    static_assert(NS >= 2 && NS <= NC && NC % NS == 0, "register sets: a tile's chunks map to sets the same way");
    constexpr int IMG_ROWS = 32 * WD;                 // epilogue image: one 32-row band per data wave
    constexpr int EPITCH = BFT * EC + 16;             // epilogue image row pitch (bytes)
    constexpr int EPI_BYTES = SIR_NT16_EPI ? IMG_ROWS * EPITCH : 0;
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE + 512 * 4 + EPI_BYTES];
    float* const bias_l = reinterpret_cast<float*>(lds + 2 * STAGE);
    char* const epi = lds + 2 * STAGE + 512 * 4;

    const int t = threadIdx.x;
    const int tb = blockIdx.x * tiles_per_block;
    const int te = (tb + tiles_per_block < n_tiles) ? tb + tiles_per_block : n_tiles;
    if (tb >= te) return;
    // x + (-0) == x for every x: without a bias the epilogue adds -0 (no branch)
    for (int n = t; n < Npad; n += 512) bias_l[n] = (bias != nullptr && n < N) ? bias[n] : -0.f;

    // loader role: row rho of the tile, k half kh of the chunk (planes kh*KS/2 ..)
    const int rho = t >> 1, kh = t & 1;
    const int aoff = (int)(rho * lda + kh * (KC / 2)) * EA;
    const int coff = (int)(rho * ldac + kh * (KC / 2)) * 2;
    const rsrc_t wrs = mk_rsrc(Wp, (uint32_t)((int64_t)NC * KS * Npad * 32));
    struct TileP { rsrc_t a; rsrc_t cp; int64_t d0; int f0; int rows; };
    auto tile_p = [&](int tt) {      // a tile past the block's range loads zeros (0-record resource)
        TileP p;
        if (tt < te) {
            p.d0 = (int64_t)(tt / n_ftiles) * BD;
            p.f0 = (tt % n_ftiles) * BFT;
            p.rows = (M - p.d0 < BD) ? (int)(M - p.d0) : BD;
            p.a = mk_rsrc(static_cast<const char*>(A) + p.d0 * lda * EA, (SIR_NT16_ABL & 1) ? 0u : (uint32_t)(p.rows * lda * EA));
            p.cp = mk_rsrc(Acopy + p.d0 * ldac, (Acopy != nullptr && p.f0 == 0) ? (uint32_t)(p.rows * ldac * 2) : 0u);
        } else {
            p.d0 = 0;
            p.f0 = 0;
            p.rows = 0;
            p.a = mk_rsrc(A, 0u);
            p.cp = mk_rsrc(A, 0u);
        }
        return p;
    };

    const int w = t >> 6, l = t & 63, r = l & 31, h = l >> 5;
    const int d_w = (w / WF) * TDT * 32, f_w = (w % WF) * TFT * 32;

    u4v av[NS][AV], wv[NS][WV];
    auto load = [&](int set, const TileP& p, int c) {
#pragma unroll
        for (int i = 0; i < AV; ++i) av[set][i] = __builtin_amdgcn_raw_buffer_load_b128(p.a, aoff + 16 * i, c * KC * EA, 0);
#pragma unroll
        for (int i = 0; i < WV; ++i)
            wv[set][i] = __builtin_amdgcn_raw_buffer_load_b128(wrs, ((i * 512 + t) / (PLANE_W / 16)) * Npad * 32 +
                                                                         ((i * 512 + t) % (PLANE_W / 16)) * 16,
                                                              (c * KS * Npad + p.f0) * 32, 0);
    };
    auto store = [&](int set, int buf, const TileP& p, int c) {
        char* st = lds + buf * STAGE;
        u4v q[KC / 16];                                // this thread's KC/2 values as 16-bit, in k order
        if constexpr (A32) {
#pragma unroll
            for (int i = 0; i < KC / 16; ++i) {
                const u4v x0 = av[set][2 * i], x1 = av[set][2 * i + 1];
                q[i].x = pack2(__uint_as_float(x0.x), __uint_as_float(x0.y), BF);
                q[i].y = pack2(__uint_as_float(x0.z), __uint_as_float(x0.w), BF);
                q[i].z = pack2(__uint_as_float(x1.x), __uint_as_float(x1.y), BF);
                q[i].w = pack2(__uint_as_float(x1.z), __uint_as_float(x1.w), BF);
            }
#pragma unroll
            for (int i = 0; i < KC / 16; ++i)       // the rounded copy (first feature tile only)
                __builtin_amdgcn_raw_buffer_store_b128(q[i], p.cp, coff + 16 * i, c * KC * 2, 0);
        } else {
#pragma unroll
            for (int i = 0; i < KC / 16; ++i) q[i] = av[set][i];
        }
        // piece i covers k = kh*KC/2 + 8i .. +7: plane kh*KS/2 + i/2, half i%2
#pragma unroll
        for (int i = 0; i < KC / 16; ++i)
            *reinterpret_cast<u4v*>(st + (kh * (KS / 2) + (i >> 1)) * PLANE + fimg(rho, i & 1)) = q[i];
#pragma unroll
        for (int i = 0; i < WV; ++i) *reinterpret_cast<u4v*>(st + KS * PLANE + (i * 512 + t) * 16) = wv[set][i];   // W planes
    };

    f16v acc[TFT][TDT];
    auto mfma = [&](int buf, bool zinit) {
        const char* st = lds + buf * STAGE;
        const f16v zero = {};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            u4v wf[TFT], df[TDT];
#pragma unroll
            for (int a = 0; a < TFT; ++a)
                wf[a] = *reinterpret_cast<const u4v*>(st + KS * PLANE + ks * PLANE_W + fimg(f_w + 32 * a + r, h));
#pragma unroll
            for (int b = 0; b < TDT; ++b)
                df[b] = *reinterpret_cast<const u4v*>(st + ks * PLANE + fimg(d_w + 32 * b + r, h));
#if SIR_NT16_ABL & 4
#pragma unroll
            for (int a = 0; a < TFT; ++a)
#pragma unroll
                for (int b = 0; b < TDT; ++b) {
                    asm volatile("" :: "v"(wf[a]), "v"(df[b]));      // timing-only: no MFMAs
                    if (zinit && ks == 0) acc[a][b] = zero;
                }
#else
#pragma unroll
            for (int a = 0; a < TFT; ++a)
#pragma unroll
                for (int b = 0; b < TDT; ++b)
                    acc[a][b] = mfma16<BF>(wf[a], df[b], (zinit && ks == 0) ? zero : acc[a][b]);
#endif
        }
    };
    // C[m][n] = acc + bias[n]; rows past M fall outside the store's range, columns past N are
    // sent past its end (dropped).  Lane indices re-derived from an opaque threadIdx copy so that
    // they do not hold VGPRs through the steps.
#if !SIR_NT16_EPI
#error "the fragment-store 16-bit NT epilogue has no dropout"
#endif
#if SIR_NT16_EPI
    // Epilogue through LDS: per round b, every wave writes its 32-row band b (bias added, rounded
    // to the output type) into a row-major image of 64 tile rows, then the block stores whole
    // output rows — each wave-instruction writes 1 KiB of contiguous row bytes (2 bf16 / 1 fp32
    // rows) instead of 32 rows x 16 B (the fragment-order stores made the 16-bit Y GEMM spend 45 %
    // of its time on its stores: timing ablation, profiles/r02_ab_nt16.txt).
    auto epilogue = [&](const TileP& p) {
        int tq = threadIdx.x;
        asm volatile("" : "+v"(tq));
        const int lq = tq & 63, rq = lq & 31, hq = lq >> 5, wq = tq >> 6;
        const int f_wq = (wq % WF) * TFT * 32;
        const uint32_t ldcb = (uint32_t)ldc * EC;
        const uint32_t nrec = (uint32_t)p.rows * ldcb;
        const rsrc_t crs = mk_rsrc(static_cast<char*>(C) + p.d0 * ldc * EC, (SIR_NT16_ABL & 2) ? 0u : nrec);
        char* const wrow = epi + ((wq / WF) * 32 + rq) * EPITCH + (f_wq + 4 * hq) * EC;
#pragma unroll
        for (int b = 0; b < TDT; ++b) {
#pragma unroll
            for (int a = 0; a < TFT; ++a) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int nl = f_wq + 32 * a + 8 * g + 4 * hq;
                    const float4 bb = *reinterpret_cast<const float4*>(bias_l + p.f0 + nl);
                    float o0 = acc[a][b][4 * g + 0] + bb.x, o1 = acc[a][b][4 * g + 1] + bb.y;
                    float o2 = acc[a][b][4 * g + 2] + bb.z, o3 = acc[a][b][4 * g + 3] + bb.w;
                    if (drop.on()) {
                        // dropout of autocast's dt output: round to dt, scale in fp32, round again
                        // (the reference's Dropout on the half-precision Linear output)
                        const uint32_t rh = drop_row_hash(drop, p.d0 + (wq / WF) * (TDT * 32) + 32 * b + rq);
                        const int cc = drop.col0 + p.f0 + nl;
                        o0 = drop_keep(drop, rh, cc + 0) ? rnd16<BF, C32>(o0) * drop.scale : 0.f;
                        o1 = drop_keep(drop, rh, cc + 1) ? rnd16<BF, C32>(o1) * drop.scale : 0.f;
                        o2 = drop_keep(drop, rh, cc + 2) ? rnd16<BF, C32>(o2) * drop.scale : 0.f;
                        o3 = drop_keep(drop, rh, cc + 3) ? rnd16<BF, C32>(o3) * drop.scale : 0.f;
                    }
                    char* d = wrow + (32 * a + 8 * g) * EC;
                    if constexpr (C32) {
                        *reinterpret_cast<float4*>(d) = make_float4(o0, o1, o2, o3);
                    } else {
                        typedef unsigned int u2v __attribute__((ext_vector_type(2)));
                        u2v ov;
                        ov.x = pack2(o0, o1, BF);
                        ov.y = pack2(o2, o3, BF);
                        *reinterpret_cast<u2v*>(d) = ov;
                    }
                }
            }
            __syncthreads();
            constexpr int PR = BFT * EC / 16;                 // 16-B pieces per image row
#pragma unroll
            for (int i = 0; i < IMG_ROWS * PR / 512; ++i) {
                const int q = tq + 512 * i;
                const int ir = q / PR, c16 = q % PR;
                const u4v v = *reinterpret_cast<const u4v*>(epi + ir * EPITCH + c16 * 16);
                const int ml = (ir >> 5) * (TDT * 32) + 32 * b + (ir & 31);      // row within the tile
                const int n = p.f0 + c16 * (16 / EC);
                const uint32_t off = (n < N) ? (uint32_t)ml * ldcb + (uint32_t)c16 * 16u : nrec;
                __builtin_amdgcn_raw_buffer_store_b128(v, crs, off, p.f0 * EC, 0);
                // the store reads its data VGPRs over several cycles: keep the next writes of
                // them away (see k_gemm_nt_p's epilogue)
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_nop 1" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
            }
            __syncthreads();
        }
    };
#else
    auto epilogue = [&](const TileP& p) {
        int tq = threadIdx.x;
        asm volatile("" : "+v"(tq));
        const int lq = tq & 63, rq = lq & 31, hq = lq >> 5, wq = tq >> 6;
        const int d_wq = (wq / WF) * TDT * 32, f_wq = (wq % WF) * TFT * 32;
        const uint32_t ldcb = (uint32_t)ldc * EC;
        const uint32_t nrec = (uint32_t)p.rows * ldcb;
        const rsrc_t crs = mk_rsrc(static_cast<char*>(C) + p.d0 * ldc * EC, (SIR_NT16_ABL & 2) ? 0u : nrec);
        const uint32_t rv = (uint32_t)(d_wq + rq) * ldcb + (uint32_t)(f_wq + 4 * hq) * EC;
#pragma unroll
        for (int b = 0; b < TDT; ++b) {
            const uint32_t rb = rv + (uint32_t)(32 * b) * ldcb;
#pragma unroll
            for (int a = 0; a < TFT; ++a) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int nc0 = p.f0 + 32 * a + 8 * g;
                    const int n = nc0 + f_wq + 4 * hq;
                    const float4 bb = *reinterpret_cast<const float4*>(bias_l + n);
                    const float o0 = acc[a][b][4 * g + 0] + bb.x, o1 = acc[a][b][4 * g + 1] + bb.y;
                    const float o2 = acc[a][b][4 * g + 2] + bb.z, o3 = acc[a][b][4 * g + 3] + bb.w;
                    const uint32_t off = (n < N) ? rb : nrec;
                    if constexpr (C32) {
                        u4v ov;
                        ov.x = __float_as_uint(o0); ov.y = __float_as_uint(o1);
                        ov.z = __float_as_uint(o2); ov.w = __float_as_uint(o3);
                        __builtin_amdgcn_raw_buffer_store_b128(ov, crs, off, nc0 * EC, 0);
                    } else {
                        typedef unsigned int u2v __attribute__((ext_vector_type(2)));
                        u2v ov;
                        ov.x = pack2(o0, o1, BF);
                        ov.y = pack2(o2, o3, BF);
                        __builtin_amdgcn_raw_buffer_store_b64(ov, crs, off, nc0 * EC, 0);
                    }
                    // the store reads its data VGPRs over several cycles: keep the next writes of
                    // them away (see k_gemm_nt_p's epilogue)
                    __builtin_amdgcn_sched_barrier(0);
                    asm volatile("s_nop 1" ::: "memory");
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
    };

#endif

    // step c: chunk c is multiplied out of LDS buffer c & 1, chunks c+1 .. c+NS are in flight in
    // register sets (c+1) % NS .. c % NS; chunk c+NS is issued into set c % NS (chunk c's, already
    // in LDS), chunk c+1 is written into the other buffer.  Chunks past the tile's last come from
    // the next tile (NC % NS == 0: its chunk i lands in set i % NS).
    TileP cu = tile_p(tb), nx = tile_p(tb + 1);
    static_for<0, NS>([&](auto I_) { load(decltype(I_)::value, cu, decltype(I_)::value); });
    store(0, 0, cu, 0);
    __syncthreads();
    for (int j = 0; tb + j < te; ++j) {
        const TileP nn = tile_p(tb + j + 2);
        static_for<0, NC>([&](auto C_) {
            constexpr int c = decltype(C_)::value;
            constexpr int s = c % NS;
            if constexpr (c + NS < NC) load(s, cu, c + NS);
            else load(s, nx, c + NS - NC);
            mfma(c & 1, c == 0);
            if constexpr (c == NC - 1) epilogue(cu);
            if constexpr (c + 1 < NC) store((c + 1) % NS, (c + 1) & 1, cu, c + 1);
            else store(0, 0, nx, 0);
            __syncthreads();
        });
        cu = nx;
        nx = nn;
    }
}

// 16-bit weight operand of k_gemm_nt16: B[n][k] (W[n][k], or W[k][n] with trans) rounded to the
// MFMA type, in planes of 16 k: plane P = k / 16 holds the Npad rows in fimg order.
__global__ void __launch_bounds__(64)
k_pack16(const float* __restrict__ W, int64_t ldw, int N, int K, int trans, int bf, int Npad, unsigned short* __restrict__ out) {
    const int n = blockIdx.x;
    for (int k = threadIdx.x; k < K; k += 64) {
        const float x = (n < N) ? (trans ? W[(int64_t)k * ldw + n] : W[(int64_t)n * ldw + k]) : 0.f;
        const unsigned short b = bf ? __builtin_bit_cast(unsigned short, (__bf16)x) : __builtin_bit_cast(unsigned short, (_Float16)x);
        const int P = k >> 4, j = k & 15;
        out[((int64_t)P * Npad * 32 + fimg(n, j >> 3)) / 2 + (j & 7)] = b;
    }
}

}  // namespace

#ifndef SIR_TN16_NARROW
#define SIR_TN16_NARROW 1       // 128 x 128 tiles when Mc or Nc <= 128 (env SIR_TN16_NARROW=0: always 256 x 256)
#endif
static bool tn16_narrow(int Mc, int Nc) {
    const char* e = getenv("SIR_TN16_NARROW");
    const int on = (e != nullptr && e[0] != 0) ? atoi(e) : SIR_TN16_NARROW;
    return on && (Mc <= 128 || Nc <= 128);
}

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
    if (tn16_narrow(Mc, Nc)) {      // 128 x 128 tiles, same row splits (the workspace is unchanged)
        const int nm = (Mc + 127) / 128, nn = (Nc + 127) / 128;
        const dim3 grid((unsigned)(P * nm * nn));
        if (dtype == SIR_DTYPE_BF16)
            hipLaunchKernelGGL((k_gemm_tn16<true, 128, 128, 2, 2, 2>), grid, dim3(256), 0, st, a, lda, b, ldb, R, Mc, Nc,
                               part, cpart, nm, nn, rps);
        else
            hipLaunchKernelGGL((k_gemm_tn16<false, 128, 128, 2, 2, 2>), grid, dim3(256), 0, st, a, lda, b, ldb, R, Mc, Nc,
                               part, cpart, nm, nn, rps);
    } else {
        const dim3 grid((unsigned)(P * nmt * nnt));
        if (dtype == SIR_DTYPE_BF16)
            hipLaunchKernelGGL(k_gemm_tn16<true>, grid, dim3(512), 0, st, a, lda, b, ldb, R, Mc, Nc, part, cpart, nmt, nnt,
                               rps);
        else
            hipLaunchKernelGGL(k_gemm_tn16<false>, grid, dim3(512), 0, st, a, lda, b, ldb, R, Mc, Nc, part, cpart, nmt, nnt,
                               rps);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = run_gemm_reduce(part, P, (int64_t)Mc * Nc, Nc, C, ldc, st);
    if (e != hipSuccess || colsum == nullptr) return e;
    return run_gemm_reduce(cpart, P, (int64_t)Mc, Mc, colsum, 0, st);
}


// ------------------------------------------------------------------------------------------
// feature dropout in place on an [M, N] block (the QK of a path whose projection is not native)
namespace {
template <int DT>
__global__ void __launch_bounds__(256)
k_dropout_apply(void* __restrict__ X, int64_t ldx, int64_t M, int N, Drop drop) {
    drop = drop_resolve(drop);
    const int64_t m = blockIdx.y;
    const uint32_t rh = drop_row_hash(drop, m);
    for (int n = blockIdx.x * 256 + threadIdx.x; n < N; n += gridDim.x * 256) {
        const bool k = drop_keep(drop, rh, drop.col0 + n);
        if constexpr (DT == SIR_DTYPE_F32) {
            float* p = static_cast<float*>(X) + m * ldx + n;
            *p = k ? *p * drop.scale : 0.f;
        } else if constexpr (DT == SIR_DTYPE_BF16) {
            __bf16* p = static_cast<__bf16*>(X) + m * ldx + n;
            *p = k ? (__bf16)((float)*p * drop.scale) : (__bf16)0.f;
        } else {
            _Float16* p = static_cast<_Float16*>(X) + m * ldx + n;
            *p = k ? (_Float16)((float)*p * drop.scale) : (_Float16)0.f;
        }
    }
}
}  // namespace

hipError_t run_dropout_apply(void* X, int64_t ldx, int64_t M, int N, int dtype, const Drop& drop, hipStream_t st) {
    if (M == 0 || N == 0 || !drop.on()) return hipSuccess;
    if (M > 2147483647) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((N + 255) / 256 < 4 ? (N + 255) / 256 : 4), (unsigned)M);
    if (dtype == SIR_DTYPE_F32) hipLaunchKernelGGL(k_dropout_apply<SIR_DTYPE_F32>, grid, dim3(256), 0, st, X, ldx, M, N, drop);
    else if (dtype == SIR_DTYPE_BF16) hipLaunchKernelGGL(k_dropout_apply<SIR_DTYPE_BF16>, grid, dim3(256), 0, st, X, ldx, M, N, drop);
    else hipLaunchKernelGGL(k_dropout_apply<SIR_DTYPE_F16>, grid, dim3(256), 0, st, X, ldx, M, N, drop);
    return hipGetLastError();
}

int64_t gemm_pack16_bytes(int64_t N, int64_t K) { return (N + 255) / 256 * 256 * K * 2; }

hipError_t run_gemm_pack16(const float* W, int64_t ldw, int N, int K, int trans, int dtype, void* packed, hipStream_t st) {
    const int np = (N + 255) / 256 * 256;
    hipLaunchKernelGGL(k_pack16, dim3(np), dim3(64), 0, st, W, ldw, N, K, trans, dtype == SIR_DTYPE_BF16 ? 1 : 0, np,
                       static_cast<unsigned short*>(packed));
    return hipGetLastError();
}

#ifndef SIR_NT16_KC
#define SIR_NT16_KC 32          // k values per chunk of the 16-bit NT GEMM (32 or 64; 16-bit A only)
#endif
#ifndef SIR_NT16_NS
#define SIR_NT16_NS 2           // register sets (chunks in flight) of the 16-bit NT GEMM, 16-bit A
#endif
#ifndef SIR_NT16_NS32
#define SIR_NT16_NS32 2         // the same for an fp32 A
#endif

#ifndef SIR_NT16_NARROW
#define SIR_NT16_NARROW 1       // 128-feature tiles for N <= 128 (env SIR_NT16_NARROW=0: always 256)
#endif
template <bool BF, bool A32, bool C32, int BFT>
static hipError_t launch_nt16_w(const void* A, int64_t lda, int64_t M, int K, const void* packed, int N, const float* bias,
                                void* C, int64_t ldc, unsigned short* Acopy, int64_t ldac, hipStream_t st, const Drop& drop) {
    const int np = (N + 255) / 256 * 256, nft = (N + BFT - 1) / BFT;
    const int64_t ntiles = (M + 255) / 256 * nft;
    const int ncu = device_cu_count();
    const int tpb = (int)((ntiles + ncu - 1) / ncu);
    const int nblk = (int)((ntiles + tpb - 1) / tpb);
    const auto* wp = static_cast<const u4v*>(packed);
    constexpr int KC = (SIR_NT16_KC == 64 && !A32) ? 64 : 32;
    constexpr int NS = A32 ? SIR_NT16_NS32 : SIR_NT16_NS;
    const int nc = K / KC;
#define SIR_NT16_L(NCV, NSV)                                                                                   \
    hipLaunchKernelGGL((k_gemm_nt16<BF, A32, C32, KC, NCV, NSV, BFT>), dim3((unsigned)nblk), dim3(512), 0, st, A, lda, \
                       M, wp, np, bias, N, C, ldc, Acopy, ldac, nft, (int)ntiles, tpb, drop)
    if (nc == 256 / KC) SIR_NT16_L(256 / KC, (NS <= 256 / KC ? NS : 256 / KC));
    else if (nc == 512 / KC) SIR_NT16_L(512 / KC, NS);
    else if (nc == 128 / KC) SIR_NT16_L(128 / KC, (NS <= 128 / KC ? NS : 128 / KC));
    else return hipErrorInvalidValue;
#undef SIR_NT16_L
    return hipGetLastError();
}

template <bool BF, bool A32, bool C32>
static hipError_t launch_nt16(const void* A, int64_t lda, int64_t M, int K, const void* packed, int N, const float* bias,
                              void* C, int64_t ldc, unsigned short* Acopy, int64_t ldac, hipStream_t st, const Drop& drop) {
    const char* e = getenv("SIR_NT16_NARROW");
    const int narrow = (e != nullptr && e[0] != 0) ? atoi(e) : SIR_NT16_NARROW;
    if (narrow && N <= 128)
        return launch_nt16_w<BF, A32, C32, 128>(A, lda, M, K, packed, N, bias, C, ldc, Acopy, ldac, st, drop);
    return launch_nt16_w<BF, A32, C32, 256>(A, lda, M, K, packed, N, bias, C, ldc, Acopy, ldac, st, drop);
}

hipError_t run_gemm_nt16(const void* A, int64_t lda, int a_dtype, int64_t M, int K, const void* packed, int N, int dtype,
                         const float* bias, void* C, int64_t ldc, int c_dtype, void* Acopy, int64_t ldac, hipStream_t st,
                         const Drop& drop) {
    if (M == 0) return hipSuccess;
    const bool bf = dtype == SIR_DTYPE_BF16, a32 = a_dtype == SIR_DTYPE_F32, c32 = c_dtype == SIR_DTYPE_F32;
    auto* acp = static_cast<unsigned short*>(Acopy);
#define SIR_NT16_D(B, A3, C3) \
    if (bf == B && a32 == A3 && c32 == C3) return launch_nt16<B, A3, C3>(A, lda, M, K, packed, N, bias, C, ldc, acp, ldac, st, drop)
    SIR_NT16_D(true, false, false);
    SIR_NT16_D(true, false, true);
    SIR_NT16_D(true, true, false);
    SIR_NT16_D(true, true, true);
    SIR_NT16_D(false, false, false);
    SIR_NT16_D(false, false, true);
    SIR_NT16_D(false, true, false);
    SIR_NT16_D(false, true, true);
#undef SIR_NT16_D
    return hipErrorInvalidValue;
}

}  // namespace sir
