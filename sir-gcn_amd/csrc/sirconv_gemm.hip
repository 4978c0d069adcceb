// sirconv_gemm.hip — the layer's projection GEMMs (conv.py:60-61,65 and their autograd) on
// gfx950 fp16 MFMA with a two-term operand split: fp32 accuracy at ~16x the f32-MFMA rate.
//
// Numerics.  Every operand element x is represented as (hi + lo) / s with hi = fp16(x*s),
// lo = fp16(x*s - hi) and s a power of two chosen per operand row (the contraction runs along
// the row), so that |x*s| < 2^15.  The product x*w is then hi*hi' + hi*lo' + lo*hi' (the lo*lo'
// term, < 2^-22 relative, is dropped), each fp16 x fp16 product exact in the fp32 MFMA
// accumulator: three v_mfma_f32_32x32x16_f16 per 32x32x16 step and ~22 significant bits per
// operand — an error comparable to an fp32 GEMM's own rounding (tests/test_gemm_gpu.py holds
// it to <= 2x torch fp32's error against fp64).  The scale of a data row is not known before
// its last k-chunk has been read, so it is a RUNNING scale: when a chunk's values would leave
// the fp16 range under the current scale, the scale is reset (with 2^SIR_HR headroom, see
// next_se) and the accumulators of that row are multiplied by the (exact, power of two) ratio of
// the new and old scales before the chunk is added.
//
// Kernels
//   k_pack_weight : B[n][k] (= W or W^T) -> fp16 hi/lo in MFMA fragment order + 1/scale per n
//   k_gemm_nt     : C[M,N] = A[M,K] B[N,K]^T + bias   (QK = X [W_Q;W_K]^T, Y = S W_R^T,
//                   G = dY W_R, dX = [dQ dK][W_Q;W_K]).  MFMA rows = features (packed B),
//                   MFMA columns = data rows, so a lane's accumulator column IS the data row
//                   whose running scale it needs.  A streamed once per feature tile (the
//                   feature tiles of one data tile run back to back on one XCD: L2 reuse).
//   k_gemm_tn     : part[p] = A[rows_p]^T B[rows_p]  (the weight gradients dW_R = dY^T S,
//                   [dW_Q; dW_K] = [dQ dK]^T X; contraction over the V node rows, split over
//                   P row ranges), running scales per column of A and of B.
//                   With csum_part the same pass also sums the columns of A (the bias gradient
//                   of that linear: db_R = sum dY, db_Q = sum dQ) from the loaded fp32 values.
//   k_gemm_reduce : C = sum_p part[p] in p order (deterministic).
// LDS stage image (both kernels): [part hi/lo][k-step 0/1][rows in fimg order] — one k-step of
// 32 rows is 1 KiB contiguous, exactly one ds_read_b128 per lane, in lane order (conflict-free).
#include <type_traits>
#include <algorithm>

#include "sirconv_internal.h"
#include "sirconv_gemm_util.h"
#include "sirconv_dropout.h"

namespace sir {
namespace {
using namespace gemm;

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

constexpr int KC = 32;          // contraction elements per LDS stage (two k16 MFMA steps)

#ifndef SIR_ABL_TN
#define SIR_ABL_TN 0            // timing-only ablation: TN loads dropped (zero-record descriptors)
#endif
#ifndef SIR_ABL_NT
#define SIR_ABL_NT 0            // timing-only ablations: 1 = NT data loads dropped, 2 = NT C stores dropped,
                                // persistent NT only: 4 = no split arithmetic, 8 = no MFMAs
#endif
#ifndef SIR_HR
#define SIR_HR 8                // headroom bits of a reset running scale (see next_se)
#endif
#ifndef SIR_TN_CFG
#define SIR_TN_CFG 2            // TN tiling: 1 = 16 waves 64x64 (4 per SIMD), 2 = 8 waves 128x64 (2 per SIMD)
#endif
#ifndef SIR_TN_PF
#define SIR_TN_PF 2             // TN chunks in flight in registers (1 or 2; 2: -3..-5 %, profiles/r02_ab_tn_pf2.txt)
#endif
#ifndef SIR_NT_PF
#define SIR_NT_PF 2             // NT chunks in flight in registers ahead of the LDS stage (1 or 2)
#endif
#ifndef SIR_NT_EPI
#define SIR_NT_EPI 1            // 1: NT epilogue through LDS, full-row stores; 0: fragment stores
#endif

// Smallest e with |m| < 2^e for normal m (e = -126 for 0 and subnormals, 129 for inf/nan).
__device__ inline int bexp(float m) { return (int)((__float_as_uint(m) >> 23) & 255u) - 126; }
// scale exponent for a running binade e: |x| * 2^(15 - e) < 2^15, clamped to a normal float
__device__ inline int scale_exp(int e) { int s = 15 - e; return s > 126 ? 126 : s; }
// Running scale of a data row / column with hysteresis: a chunk whose binade e_c still fits
// (|x| * 2^se < 2^15) keeps the current scale; otherwise the scale is reset with SIR_HR bits of
// headroom, so a row's scale changes (and its accumulators are rescaled) only when a chunk
// exceeds the row's earlier maximum by more than 2^SIR_HR — once per row in practice, at its
// first chunk.  Scaled values stay in [2^-14, 2^15) over >= 20 binades below the maximum, where
// the fp16 hi/lo pair is exact to ~22 bits; the split is scale-invariant there, so the result
// does not depend on which power-of-two scale was in force.
constexpr int SE_INIT = 127;    // no chunk seen yet
__device__ inline int next_se(int se_old, int e_c) {
    if (e_c + se_old <= 15) return se_old;
    const int s = 15 - SIR_HR - e_c;
    return s > 126 ? 126 : s;
}
// compensated (Kahan) accumulation: s += x with the rounding error carried in c (no fp contraction
// in this file, so the compensation is not optimised away)
__device__ inline void kahan_add(float& s, float& c, float x) {
    const float y = x - c;
    const float t = s + y;
    c = (t - s) - y;
    s = t;
}
__device__ inline float pow2(int e) { e = e < -126 ? -126 : (e > 127 ? 127 : e); return __uint_as_float((uint32_t)(e + 127) << 23); }
// feature dropout of QK (sirconv_dropout.h) on 4 consecutive output columns n .. n+3 of one row
__device__ inline void drop4(const Drop& d, int64_t row, int n, float4& o) {
    const uint32_t rh = drop_row_hash(d, row);
    const int c = d.col0 + n;
    o.x = drop_keep(d, rh, c + 0) ? o.x * d.scale : 0.f;
    o.y = drop_keep(d, rh, c + 1) ? o.y * d.scale : 0.f;
    o.z = drop_keep(d, rh, c + 2) ? o.z * d.scale : 0.f;
    o.w = drop_keep(d, rh, c + 3) ? o.w * d.scale : 0.f;
}

// sigma'(z) * x from the sign of the gate (z or sigma(z): the same sign for the ReLU family)
__device__ inline float gate_dact(float g, float x, int relu, float slope) {
    return g > 0.f ? x : (relu ? 0.f : x * slope);
}
// in place, the sign-bit gate (N = 256; see k_gemm_nt_p GATE 2)
__global__ void __launch_bounds__(256)
k_gate_dact_bits(float* __restrict__ C, int64_t ldc, const uint64_t* __restrict__ mask, int64_t M, int relu, float slope) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= M * 256) return;
    const int64_t r = i >> 8;
    const int c = (int)(i & 255);
    const bool pos = (mask[r * 4 + (c & 3)] >> (c >> 2)) & 1u;
    C[r * ldc + c] = gate_dact(pos ? 1.f : -1.f, C[r * ldc + c], relu, slope);
}
// in place: C = sigma'(gate) * C (the gated GEMM's epilogue for the routes without it)
__global__ void __launch_bounds__(256)
k_gate_dact(float* __restrict__ C, int64_t ldc, const float* __restrict__ gate, int64_t M, int N, int relu, float slope) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= M * N) return;
    const int64_t r = i / N, c = i % N;
    C[r * ldc + c] = gate_dact(gate[r * ldc + c], C[r * ldc + c], relu, slope);
}

#ifndef SIR_SPLIT_MIX
#define SIR_SPLIT_MIX 1         // TN loaders: 1 = the split by v_fma_mix (2 VALU per element), 0 = plain C (~4.5)
#endif                          // (the NT kernels keep the C form: the asm one costs them a spill in the loop)
// hi/lo fp16 split of 8 floats scaled by s (exact power of two)
// hi = fp16(x s), lo = fp16(x s - hi), one v_fma_mix each, written into the halves of the fragment
// registers (x s is exact, and x s - hi is exact in the fused op: the same bits as rounding y = x s
// and y - hi separately, sirconv_gemm_w.hip).  s_nop 1: the VALU-write -> MFMA-read wait states
// (the hazard recognizer does not look inside inline asm).
__device__ inline void split8_mix(float4 a, float4 b, float s, h8& hi, h8& lo) {
    uint32_t h0, h1, h2, h3, l0, l1, l2, l3;
    asm volatile(
        "v_fma_mixlo_f16 %0, %8, %16, 0\n\tv_fma_mixhi_f16 %0, %9, %16, 0\n\t"
        "v_fma_mixlo_f16 %1, %10, %16, 0\n\tv_fma_mixhi_f16 %1, %11, %16, 0\n\t"
        "v_fma_mixlo_f16 %2, %12, %16, 0\n\tv_fma_mixhi_f16 %2, %13, %16, 0\n\t"
        "v_fma_mixlo_f16 %3, %14, %16, 0\n\tv_fma_mixhi_f16 %3, %15, %16, 0\n\t"
        "v_fma_mixlo_f16 %4, %8, %16, -%0 op_sel_hi:[0,0,1]\n\tv_fma_mixhi_f16 %4, %9, %16, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %5, %10, %16, -%1 op_sel_hi:[0,0,1]\n\tv_fma_mixhi_f16 %5, %11, %16, -%1 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %6, %12, %16, -%2 op_sel_hi:[0,0,1]\n\tv_fma_mixhi_f16 %6, %13, %16, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %7, %14, %16, -%3 op_sel_hi:[0,0,1]\n\tv_fma_mixhi_f16 %7, %15, %16, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "s_nop 1"
        : "=&v"(h0), "=&v"(h1), "=&v"(h2), "=&v"(h3), "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3)
        : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w), "v"(s));
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    hi = __builtin_bit_cast(h8, u4{h0, h1, h2, h3});
    lo = __builtin_bit_cast(h8, u4{l0, l1, l2, l3});
}
// the same split written as fused ops for the backend's v_fma_mix patterns (x s exact: fma(x, s, -hi)
// == x s - hi, one rounding to fp16 either way)
#define SIR_SPLIT1F(x, i) { const _Float16 h_ = (_Float16)__builtin_fmaf((x), s, 0.f); hi[i] = h_; lo[i] = (_Float16)__builtin_fmaf((x), s, -(float)h_); }
__device__ inline void split8_fma(float4 a, float4 b, float s, h8& hi, h8& lo) {
    SIR_SPLIT1F(a.x, 0) SIR_SPLIT1F(a.y, 1) SIR_SPLIT1F(a.z, 2) SIR_SPLIT1F(a.w, 3)
    SIR_SPLIT1F(b.x, 4) SIR_SPLIT1F(b.y, 5) SIR_SPLIT1F(b.z, 6) SIR_SPLIT1F(b.w, 7)
}
#undef SIR_SPLIT1F
#define SIR_SPLIT1(x, i) { const float y_ = (x) * s; const _Float16 h_ = (_Float16)y_; hi[i] = h_; lo[i] = (_Float16)(y_ - (float)h_); }
__device__ inline void split8(float4 a, float4 b, float s, h8& hi, h8& lo) {
    SIR_SPLIT1(a.x, 0) SIR_SPLIT1(a.y, 1) SIR_SPLIT1(a.z, 2) SIR_SPLIT1(a.w, 3)
    SIR_SPLIT1(b.x, 4) SIR_SPLIT1(b.y, 5) SIR_SPLIT1(b.z, 6) SIR_SPLIT1(b.w, 7)
}
#undef SIR_SPLIT1

// m = max(m, |v|) in two v_max3_f32 with |.| source modifiers (fmaxf makes hipcc canonicalise every
// input first)
__device__ inline float fmax4_mix(float m, float4 v) {
    asm("v_max3_f32 %0, %0, |%1|, |%2|\n\tv_max3_f32 %0, %0, |%3|, |%4|" : "+v"(m) : "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
    return m;
}
__device__ inline float fmax4(float m, float4 v) {
    return fmaxf(fmaxf(m, fmaxf(fabsf(v.x), fabsf(v.y))), fmaxf(fabsf(v.z), fabsf(v.w)));
}

// ------------------------------------------------------------------------------------------
// weight packing: one block of 64 threads per feature n (Npad blocks)
// out layout: halves [Kc][2 part][2 ks][Npad rows in fimg order], then float inv_scale[Npad]
__global__ void __launch_bounds__(64)
k_pack_weight(const float* __restrict__ W, int64_t ldw, int N, int K, int trans, int Npad, int Kc,
              _Float16* __restrict__ out, float* __restrict__ inv_scale) {
    const int n = blockIdx.x, l = threadIdx.x;
    float m = 0.f;
    if (n < N)
        for (int k = l; k < K; k += 64) m = fmaxf(m, fabsf(trans ? W[(int64_t)k * ldw + n] : W[(int64_t)n * ldw + k]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    const int se = scale_exp(bexp(m));
    const float s = pow2(se);
    for (int k = l; k < Kc * KC; k += 64) {
        float x = 0.f;
        if (n < N && k < K) x = trans ? W[(int64_t)k * ldw + n] : W[(int64_t)n * ldw + k];
        const float y = x * s;
        const _Float16 h = (_Float16)y;
        const int kc = k / KC, ks = (k / 16) & 1, j = k & 15;
        const int64_t at = fimg(n, j >> 3) / 2 + (j & 7);
        out[(((int64_t)kc * 2 + 0) * 2 + ks) * Npad * 16 + at] = h;
        out[(((int64_t)kc * 2 + 1) * 2 + ks) * Npad * 16 + at] = (_Float16)(y - (float)h);
    }
    if (l == 0) inv_scale[n] = (n < N) ? pow2(-se) : 0.f;
}

// ------------------------------------------------------------------------------------------
// NT GEMM.  WD x WF waves, each TDT x TFT tiles of 32 data rows x 32 features.
// KFULL: K is a multiple of KC, so no column past K is ever loaded (no per-element select: the
// compiler turns that select into exec-masked branches with a vmcnt(0) inside, draining the
// prefetch queue every chunk).
template <int WD, int WF, int TDT, int TFT, bool KFULL>
__global__ void __launch_bounds__(64 * WD * WF)
k_gemm_nt(const float* __restrict__ A, int64_t lda, int64_t M, int K,
          const u4v* __restrict__ Wp, int Npad, const float* __restrict__ inv_t,
          const float* __restrict__ bias, int N, float* __restrict__ C, int64_t ldc, int n_ftiles, Drop drop) {
    drop = drop_resolve(drop);
    constexpr int NT = 64 * WD * WF;
    constexpr int BD = 32 * TDT * WD;        // data rows per block
    constexpr int BF = 32 * TFT * WF;        // features per block
    constexpr int TPR = NT / BD;             // loader threads per data row
    static_assert(TPR == 1 || TPR == 2 || TPR == 4, "loader mapping");
    constexpr int FPT = KC / TPR;            // floats per loader thread per stage
    constexpr int WPT = BF * 8 / NT;         // 16-B weight pieces per thread per stage
    static_assert(WPT >= 1 && BF * 8 % NT == 0, "weight loader mapping");
    constexpr int D_BYTES = BD * 128, W_BYTES = BF * 128;
    constexpr int STAGE = D_BYTES + W_BYTES + BD * 4;
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

    const int t = threadIdx.x;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t d0 = (int64_t)(wg / n_ftiles) * BD;
    const int f0 = (wg % n_ftiles) * BF;
    const int nc = (K + KC - 1) / KC;

    // loader role: buffer loads off wave-uniform bases (rows past M read as 0 by the range check)
    const int rho = t / TPR, kp = t % TPR;
    const int64_t rows_here = (M - d0 < BD) ? M - d0 : BD;
    const rsrc_t arsrc = mk_rsrc(A + d0 * lda, (SIR_ABL_NT & 1) ? 0u : (uint32_t)(rows_here * lda * 4));
    const int aoff = (rho * (int)lda + kp * FPT) * 4;
    const rsrc_t wrsrc = mk_rsrc(Wp, (uint32_t)((int64_t)nc * Npad * 128));
    int woff[WPT];
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
        const int p = t + i * NT;
        // LDS piece p of the stage's weight image: plane p / (2 BF), then fimg order
        const int plane = p / (BF * 2), rem = p % (BF * 2);
        const int nl = (rem >> 6) * 32 + (rem & 31), q = (rem >> 5) & 1;
        woff[i] = plane * Npad * 32 + fimg(f0 + nl, q);
    }
    int se_run = SE_INIT;                   // running scale exponent of this data row

    // compute role
    const int w = t >> 6, l = t & 63, r = l & 31, h = l >> 5;
    const int d_w = (w / WF) * TDT * 32, f_w = (w % WF) * TFT * 32;

    // register sets for data chunks in flight: chunk j lands in set j % SIR_NT_PF.  The packed
    // weights come from L2 (one set, loaded one chunk ahead).
    float4 dv[2][FPT / 4];
    u4v wv[WPT];

    auto load_a = [&](int set, int c) {
#pragma unroll
        for (int i = 0; i < FPT / 4; ++i) {
            const int k = c * KC + kp * FPT + 4 * i;
            const u4v u = __builtin_amdgcn_raw_buffer_load_b128(arsrc, aoff + 16 * i, c * KC * 4, 0);
            dv[set][i] = (KFULL || k < K) ? make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z),
                                               __uint_as_float(u.w))
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto load_w = [&](int c) {
#pragma unroll
        for (int i = 0; i < WPT; ++i)
            wv[i] = __builtin_amdgcn_raw_buffer_load_b128(wrsrc, woff[i], c * Npad * 128, 0);
    };
    auto load = [&](int set, int c) { load_a(set, c); load_w(c); };

    // split the loaded chunk of register set `set` into stage `buf` (with the row's rescale
    // factor; 1 for the first chunk, whose accumulators are still zero)
    auto store = [&](int set, int buf, bool first = false) {
        char* st = lds + buf * STAGE;
        float m = 0.f;
#pragma unroll
        for (int i = 0; i < FPT / 4; ++i) m = fmax4(m, dv[set][i]);
        if (TPR > 1) m = fmaxf(m, __shfl_xor(m, 1));
        if (TPR > 2) m = fmaxf(m, __shfl_xor(m, 2));
        const int se_old = se_run, se = next_se(se_old, bexp(m));
        se_run = se;
        const float s = pow2(se);
        // k_local = kp*FPT + j -> ks = k_local / 16, position k_local % 16
#pragma unroll
        for (int j = 0; j < FPT; j += 8) {
            const int kl = kp * FPT + j, ks = kl >> 4, pos = kl & 15;
            h8 hv, lv;
            split8(dv[set][j / 4], dv[set][j / 4 + 1], s, hv, lv);
            *reinterpret_cast<h8*>(st + (0 * 2 + ks) * BD * 32 + fimg(rho, pos >> 3)) = hv;
            *reinterpret_cast<h8*>(st + (1 * 2 + ks) * BD * 32 + fimg(rho, pos >> 3)) = lv;
        }
        // every loader thread of the row holds the same factor: a branch-free (same-value) store
        reinterpret_cast<float*>(st + D_BYTES + W_BYTES)[rho] = first ? 1.f : pow2(se - se_old);
#pragma unroll
        for (int i = 0; i < WPT; ++i)
            *reinterpret_cast<u4v*>(st + D_BYTES + (t + i * NT) * 16) = wv[i];
    };

    f16v acc[TFT][TDT];
#pragma unroll
    for (int a = 0; a < TFT; ++a)
#pragma unroll
        for (int b = 0; b < TDT; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

    // rows whose scale rose with the chunk in stage `buf` carry a factor != 1: each wave checks
    // its own rows (a ballot, no block-wide reduction) and rescales only when one changed
    auto rescale = [&](int buf) {
        const float* fac = reinterpret_cast<const float*>(lds + buf * STAGE + D_BYTES + W_BYTES);
        float f[TDT];
        bool ch = false;
#pragma unroll
        for (int b = 0; b < TDT; ++b) { f[b] = fac[d_w + 32 * b + r]; ch |= f[b] != 1.f; }
        if (__builtin_amdgcn_ballot_w64(ch) != 0) {
#pragma unroll
            for (int b = 0; b < TDT; ++b)
#pragma unroll
                for (int a = 0; a < TFT; ++a) acc[a][b] *= f[b];
        }
    };
    auto mfma = [&](int buf) {
        const char* st = lds + buf * STAGE;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            h8 wf[TFT][2], df[TDT][2];
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) {
#pragma unroll
                for (int a = 0; a < TFT; ++a)
                    wf[a][pt] = *reinterpret_cast<const h8*>(st + D_BYTES + (pt * 2 + ks) * BF * 32 + fimg(f_w + 32 * a + r, h));
#pragma unroll
                for (int b = 0; b < TDT; ++b)
                    df[b][pt] = *reinterpret_cast<const h8*>(st + (pt * 2 + ks) * BD * 32 + fimg(d_w + 32 * b + r, h));
            }
#pragma unroll
            for (int a = 0; a < TFT; ++a)
#pragma unroll
                for (int b = 0; b < TDT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[a][0], df[b][0], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TFT; ++a)
#pragma unroll
                for (int b = 0; b < TDT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[a][0], df[b][1], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TFT; ++a)
#pragma unroll
                for (int b = 0; b < TDT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[a][1], df[b][0], acc[a][b], 0, 0, 0);
        }
    };
    auto compute = [&](int buf) {
        rescale(buf);
        mfma(buf);
    };

    load(0, 0);
    store(0, 0, true);
#if SIR_NT_PF == 2
    // two data chunks in flight: at step c the registers hold chunks c+1 (set (c+1)&1) and c+2
    // (set c&1); chunk c+1 is split into the free stage, then W(c+2) and A(c+3) (into the freed
    // set) are issued in that order, so that the wait for A(c+1), W(c+1) leaves A(c+2) in flight.
    // The steady-state steps (and the path into them) carry no conditional loads: a load skipped
    // on one path makes the compiler's wait-count merge assume the worst and drain the queue
    // (vmcnt(0)) every step.
    auto step_full = [&](int c, int set) {        // set = (c + 1) & 1, static; needs c + 3 < nc
        compute(c & 1);
        store(set, (c & 1) ^ 1);
        load_w(c + 2);
        load_a(set, c + 3);
        __syncthreads();
    };
    auto step_tail = [&](int c, int set) {
        compute(c & 1);
        if (c + 1 < nc) {
            store(set, (c & 1) ^ 1);
            if (c + 2 < nc) load_w(c + 2);
            if (c + 3 < nc) load_a(set, c + 3);
        }
        __syncthreads();
    };
    int c = 0;
    if (nc > 4) {
        load_a(1, 1);
        load_w(1);
        load_a(0, 2);
        __syncthreads();
        for (; c + 4 < nc; c += 2) {
            step_full(c, 1);
            step_full(c + 1, 0);
        }
    } else {
        if (nc > 1) { load_a(1, 1); load_w(1); }
        if (nc > 2) load_a(0, 2);
        __syncthreads();
    }
    for (; c < nc; c += 2) {
        step_tail(c, 1);
        if (c + 1 < nc) step_tail(c + 1, 0);
    }
#elif SIR_NT_PF == 3
    // two data chunks in flight, and the split of chunk c+1 into the free stage happens BEFORE
    // the MFMAs of chunk c (the free stage was last read before the previous barrier), in one
    // basic block with them so the scheduler can interleave its VALU/LDS work with the MFMAs.
    // Issue order per step: W(c+2) then A(c+3), so the next step's wait for A(c+2), W(c+2)
    // leaves A(c+3) in flight.
    if (nc > 1) { load_a(1, 1); load_w(1); }
    if (nc > 2) load_a(0, 2);
    __syncthreads();
    auto step_full = [&](int c, int set) {        // requires c + 3 < nc
        const int buf = c & 1;
        rescale(buf);
        store(set, buf ^ 1);
        load_w(c + 2);
        load_a(set, c + 3);
        mfma(buf);
        __syncthreads();
    };
    auto step_tail = [&](int c, int set) {
        const int buf = c & 1;
        rescale(buf);
        if (c + 1 < nc) store(set, buf ^ 1);
        if (c + 2 < nc) load_w(c + 2);
        if (c + 3 < nc) load_a(set, c + 3);
        mfma(buf);
        __syncthreads();
    };
    int c = 0;
    for (; c + 4 < nc; c += 2) {
        step_full(c, 1);
        step_full(c + 1, 0);
    }
    for (; c < nc; c += 2) {
        step_tail(c, 1);
        if (c + 1 < nc) step_tail(c + 1, 0);
    }
#else
    __syncthreads();
    for (int c = 0; c < nc; ++c) {
        const int buf = c & 1;
        const bool more = c + 1 < nc;
        if (more) load(0, c + 1);
        compute(buf);
        if (more) store(0, buf ^ 1);
        __syncthreads();
    }
#endif

    // epilogue: C[m][n] = acc * 2^-se(m) * inv_t[n] + bias[n]
#if SIR_NT_EPI != 1
#error "the fragment-store NT epilogue has no dropout"
#endif
#if SIR_NT_EPI == 1
    // Through LDS, one 32-row band of every wave per round: the waves write their scaled float4
    // fragments into a row-major image (row pitch BF*4 + 16 B: conflict-free ds_write_b128), then
    // the block stores whole output rows — every wave-instruction writes BF*4 contiguous bytes
    // (full cache lines) instead of 32 rows x 32 B.
    constexpr int RR = WD * 32, PITCH = BF * 4 + 16;
    constexpr int SC_OFF = STAGE + D_BYTES + W_BYTES;
    static_assert(RR * PITCH <= SC_OFF, "epilogue image overlaps the scale row");
    static_assert((RR * BF / 4) % NT == 0, "epilogue copy mapping");
    float* sc = reinterpret_cast<float*>(lds + SC_OFF);
    if (kp == 0) sc[rho] = pow2(-se_run);
    __syncthreads();
#pragma unroll
    for (int b = 0; b < TDT; ++b) {
        const int dl = d_w + 32 * b + r;
        const float is = sc[dl];
        char* rowp = lds + ((w / WF) * 32 + r) * PITCH;
#pragma unroll
        for (int a = 0; a < TFT; ++a) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int nl = f_w + 32 * a + 8 * g + 4 * h;
                const int n = f0 + nl;
                const float4 it = *reinterpret_cast<const float4*>(inv_t + n);
                float4 o;
                o.x = acc[a][b][4 * g + 0] * is * it.x;
                o.y = acc[a][b][4 * g + 1] * is * it.y;
                o.z = acc[a][b][4 * g + 2] * is * it.z;
                o.w = acc[a][b][4 * g + 3] * is * it.w;
                if (bias != nullptr && n < N) {
                    const float4 bb = *reinterpret_cast<const float4*>(bias + n);
                    o.x += bb.x; o.y += bb.y; o.z += bb.z; o.w += bb.w;
                }
                if (drop.on()) drop4(drop, d0 + dl, n, o);
                *reinterpret_cast<float4*>(rowp + nl * 4) = o;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < RR * BF / 4 / NT; ++k) {
            const int idx = t + k * NT;
            const int row = idx / (BF / 4), c4 = idx % (BF / 4);
            const int64_t m = d0 + (row >> 5) * (TDT * 32) + 32 * b + (row & 31);
            const int n = f0 + c4 * 4;
            const float4 o = *reinterpret_cast<const float4*>(lds + row * PITCH + c4 * 16);
            if (!(SIR_ABL_NT & 2) && m < M && n < N) *reinterpret_cast<float4*>(C + m * ldc + n) = o;
        }
        __syncthreads();
    }
}
#else
    float* sc = reinterpret_cast<float*>(lds);
    if (kp == 0) sc[rho] = pow2(-se_run);
    __syncthreads();
#pragma unroll
    for (int b = 0; b < TDT; ++b) {
        const int dl = d_w + 32 * b + r;
        const int64_t m = d0 + dl;
        const float is = sc[dl];
#pragma unroll
        for (int a = 0; a < TFT; ++a) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = f0 + f_w + 32 * a + 8 * g + 4 * h;
                const float4 it = *reinterpret_cast<const float4*>(inv_t + n);
                float4 o;
                o.x = acc[a][b][4 * g + 0] * is * it.x;
                o.y = acc[a][b][4 * g + 1] * is * it.y;
                o.z = acc[a][b][4 * g + 2] * is * it.z;
                o.w = acc[a][b][4 * g + 3] * is * it.w;
                if (bias != nullptr && n < N) {
                    const float4 bb = *reinterpret_cast<const float4*>(bias + n);
                    o.x += bb.x; o.y += bb.y; o.z += bb.z; o.w += bb.w;
                }
                if (m < M && n < N) *reinterpret_cast<float4*>(C + m * ldc + n) = o;
            }
        }
    }
}
#endif

// ------------------------------------------------------------------------------------------
// Persistent NT GEMM (N <= NT_P_NMAX, K = 32 * NCT).  k_gemm_nt's tiles are short at the layer's
// shapes (K = 256: 8 chunks), and with one block per CU every tile paid the pipeline fill (one
// memory latency) and an epilogue during which the CU's MFMAs idled: a fixed ~11 us per tile
// against ~23 us of chunk work (fit over K = 256 / 512 on MI355X).  Here one 512-thread block per
// CU walks a contiguous range of 256 x 256 output tiles (both feature tiles of a data tile back to
// back, so A's second read is an L2 hit), the chunk pipeline runs on across tile boundaries (the
// next tile's first chunks are loaded and split while the current tile's last ones are
// multiplied), and the epilogue stores straight from the accumulators with buffer stores — rows
// past M and columns past N fall outside the store's range and are dropped, so no store is
// guarded by a branch and the compiler's wait counts stay exact.  Per-tile data and arithmetic
// are those of k_gemm_nt<2, 4, 4, 2, true>: results are bit-identical.
#ifndef SIR_NT_PERSIST
#define SIR_NT_PERSIST 1
#endif
#ifndef SIR_NT_PRIO
#define SIR_NT_PRIO 0           // 1: s_setprio 1 around each step's MFMA cluster; 2: waves 4-7 at priority 1
#endif
#ifndef SIR_NT_P_UNROLL
#define SIR_NT_P_UNROLL 1       // the steps between the first and the last three fully unrolled
#endif
#ifndef SIR_NT_STAGGER
#define SIR_NT_STAGGER 0        // 1: waves 4-7 split / load before their MFMAs (see step)
#endif
#ifndef SIR_NT_P_KSB
#define SIR_NT_P_KSB 1
#endif
#ifndef SIR_NT_MAX3
#define SIR_NT_MAX3 1           // 1: the row maximum of a chunk by v_max3 with |.| modifiers (fmax4_mix)
#endif
// hi / lo split of the persistent NT kernel: 1 = v_fma_mix in asm (split8_mix), 2 = the same as fused C ops
// (split8_fma), 0 = plain C; all bit-identical.  Round-6 A/B over QK / Y / G / dX at S2: 5.71 ms (0) ->
// 5.57 ms (1 with SIR_NT_MAX3; 2 VGPRs spilled outside the chunk loop), fused C 5.72, MAX3 alone 5.65
// (profiles/r06_ab_gemm_nt_split.txt)
#ifndef SIR_NT_SPLIT_MIX
#define SIR_NT_SPLIT_MIX 1
#endif
#ifndef SIR_NT_P_EPI
#define SIR_NT_P_EPI 1          // persistent NT epilogue through LDS with whole-row stores (1) or fragment stores (0)
#endif
constexpr int NT_P_NMAX = 512;

// GATE: C = sigma'(gate) * (A B^T) (gate [M, N] with C's leading dimension; ReLU: gate > 0 ? x : 0,
// LeakyReLU: gate > 0 ? x : x * slope — torch's threshold / leaky_relu backward with the activation's
// output or input as `gate`: the same sign): the materialised max backward's dZ = sigma'(z) * (dM W_R)
// in the GEMM's epilogue instead of an [E, H] elementwise pass
// GATE 2: the gate as sign bits (sir_edge_gather_act's mask: N = 256, 4 words per row, bit l of word
// x = gate(4 l + x) > 0): 32 B per output row instead of the row's 1 KiB of gate values
template <int NCT, int GATE>
__global__ void __launch_bounds__(512)
k_gemm_nt_p(const float* __restrict__ A, int64_t lda, int64_t M, const u4v* __restrict__ Wp, int Npad,
            const float* __restrict__ inv_t, const float* __restrict__ bias, int N, float* __restrict__ C,
            int64_t ldc, int n_ftiles, int n_tiles, int tiles_per_block, Drop drop, const float* __restrict__ gate,
            int gate_relu, float gate_slope) {
    drop = drop_resolve(drop);
    constexpr int WF = 4, TDT = 4, TFT = 2;
    constexpr int NT = 512, BD = 256, BF = 256, TPR = NT / BD, FPT = KC / TPR, WPT = BF * 8 / NT;
    static_assert(TPR == 2 && WPT == 4 && NCT >= 4 && NCT % 2 == 0, "mapping");
    constexpr int D_BYTES = BD * 128, W_BYTES = BF * 128;
    constexpr int STAGE = D_BYTES + W_BYTES + BD * 4;
    constexpr int FIN_OFF = 2 * STAGE;                // [2][BD]: 2^-se of the rows of the last two tiles
    constexpr int EPI_OFF = FIN_OFF + 2 * BD * 4;     // inv_t[NT_P_NMAX], bias[NT_P_NMAX]
    __shared__ __attribute__((aligned(16))) char lds[EPI_OFF + 2 * NT_P_NMAX * 4];

    const int t = threadIdx.x;
    const int tb = blockIdx.x * tiles_per_block;
    const int te = (tb + tiles_per_block < n_tiles) ? tb + tiles_per_block : n_tiles;
    if (tb >= te) return;
    float* const inv_l = reinterpret_cast<float*>(lds + EPI_OFF);
    float* const bias_l = inv_l + NT_P_NMAX;
    float* const fin = reinterpret_cast<float*>(lds + FIN_OFF);
    // x + (-0) == x for every x (-0 included): without a bias the epilogue adds -0, which leaves
    // the result bit-identical to adding nothing (no branch around the stores)
    for (int n = t; n < Npad; n += NT) {          // visible after the prologue's barrier
        inv_l[n] = inv_t[n];
        bias_l[n] = (bias != nullptr && n < N) ? bias[n] : -0.f;
    }

    // loader role
    const int rho = t / TPR, kp = t % TPR;
    const int aoff = (rho * (int)lda + kp * FPT) * 4;
    const rsrc_t wrsrc = mk_rsrc(Wp, (uint32_t)((int64_t)NCT * Npad * 128));
    // weight piece t + i*NT of a stage: plane i (BF * 2 == NT), row nl / half q from t; with
    // fimg(f0 + nl, q) = f0 * 32 + fimg(nl, q) (f0 % 256 == 0) the plane and the tile's f0 go to
    // the scalar offset and one VGPR holds the lane's part
    static_assert(BF * 2 == NT, "one weight plane per loader pass");
    const int woff = fimg((t >> 6) * 32 + (t & 31), (t >> 5) & 1);
    struct TileP { rsrc_t a; int64_t d0; int f0; int rows; };
    auto tile_p = [&](int tt) {   // a tile past the block's range loads zeros (0-record resource)
        TileP p;
        if (tt < te) {
            p.d0 = (int64_t)(tt / n_ftiles) * BD;
            p.f0 = (tt % n_ftiles) * BF;
            p.rows = (M - p.d0 < BD) ? (int)(M - p.d0) : BD;
            p.a = mk_rsrc(A + p.d0 * lda, (SIR_ABL_NT & 1) ? 0u : (uint32_t)(p.rows * lda * 4));
        } else {
            p.d0 = 0;
            p.f0 = 0;
            p.rows = 0;
            p.a = mk_rsrc(A, 0u);
        }
        return p;
    };
    int se_run = SE_INIT;

    // compute role
    const int w = t >> 6, l = t & 63, r = l & 31, h = l >> 5;
    const int d_w = (w / WF) * TDT * 32, f_w = (w % WF) * TFT * 32;

    float4 dv[2][FPT / 4];
    u4v wv[WPT];
    auto load_a = [&](int set, const TileP& p, int c) {
#pragma unroll
        for (int i = 0; i < FPT / 4; ++i) {
            const u4v u = __builtin_amdgcn_raw_buffer_load_b128(p.a, aoff + 16 * i, c * KC * 4, 0);
            dv[set][i] = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z),
                                     __uint_as_float(u.w));
        }
    };
    auto load_w = [&](const TileP& p, int c) {
#pragma unroll
        for (int i = 0; i < WPT; ++i)
            wv[i] = __builtin_amdgcn_raw_buffer_load_b128(wrsrc, woff, c * Npad * 128 + i * Npad * 32 + p.f0 * 32, 0);
    };
    // split chunk of register set `set` into stage `buf`; first: a tile's first chunk (fresh row
    // scale, factor 1); last: a tile's last chunk (its final row scale goes to fin[slot])
    auto store = [&](int set, int buf, bool first, bool last, int slot) {
        char* st = lds + buf * STAGE;
        float m = 0.f;
#pragma unroll
        for (int i = 0; i < FPT / 4; ++i) m = SIR_NT_MAX3 ? fmax4_mix(m, dv[set][i]) : fmax4(m, dv[set][i]);
        m = fmaxf(m, __shfl_xor(m, 1));
        const int se_old = first ? SE_INIT : se_run, se = next_se(se_old, bexp(m));
        se_run = se;
        const float s = pow2(se);
#pragma unroll
        for (int j = 0; j < FPT; j += 8) {
            const int kl = kp * FPT + j, ks = kl >> 4, pos = kl & 15;
            h8 hv, lv;
#if SIR_ABL_NT & 4
            hv = __builtin_bit_cast(h8, dv[set][j / 4]);         // timing-only: no split arithmetic
            lv = __builtin_bit_cast(h8, dv[set][j / 4 + 1]);
#else
#if SIR_NT_SPLIT_MIX == 1
            split8_mix(dv[set][j / 4], dv[set][j / 4 + 1], s, hv, lv);
#elif SIR_NT_SPLIT_MIX == 2
            split8_fma(dv[set][j / 4], dv[set][j / 4 + 1], s, hv, lv);
#else
            split8(dv[set][j / 4], dv[set][j / 4 + 1], s, hv, lv);
#endif
#endif
            *reinterpret_cast<h8*>(st + (0 * 2 + ks) * BD * 32 + fimg(rho, pos >> 3)) = hv;
            *reinterpret_cast<h8*>(st + (1 * 2 + ks) * BD * 32 + fimg(rho, pos >> 3)) = lv;
        }
        reinterpret_cast<float*>(st + D_BYTES + W_BYTES)[rho] = first ? 1.f : pow2(se - se_old);
        if (last) {
            int rq = threadIdx.x;                     // recomputed here: see the epilogue
            asm volatile("" : "+v"(rq));
            fin[slot * BD + rq / TPR] = pow2(-se);
        }
#pragma unroll
        for (int i = 0; i < WPT; ++i)
            *reinterpret_cast<u4v*>(st + D_BYTES + (t + i * NT) * 16) = wv[i];
    };

    f16v acc[TFT][TDT];
    auto rescale = [&](int buf) {
        const float* fac = reinterpret_cast<const float*>(lds + buf * STAGE + D_BYTES + W_BYTES);
        float f[TDT];
        bool ch = false;
#pragma unroll
        for (int b = 0; b < TDT; ++b) { f[b] = fac[d_w + 32 * b + r]; ch |= f[b] != 1.f; }
        if (__builtin_amdgcn_ballot_w64(ch) != 0) {
#pragma unroll
            for (int b = 0; b < TDT; ++b)
#pragma unroll
                for (int a = 0; a < TFT; ++a) acc[a][b] *= f[b];
        }
    };
    auto mfma = [&](int buf, bool zinit) {       // zinit: a tile's first chunk starts from zero
        const char* st = lds + buf * STAGE;
        const f16v zero = {};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#if SIR_NT_P_KSB
            if (ks == 1) __builtin_amdgcn_sched_barrier(0);   // ks 1's fragments not loaded under ks 0's MFMAs
#endif
            h8 wf[TFT][2], df[TDT][2];
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) {
#pragma unroll
                for (int a = 0; a < TFT; ++a)
                    wf[a][pt] = *reinterpret_cast<const h8*>(st + D_BYTES + (pt * 2 + ks) * BF * 32 + fimg(f_w + 32 * a + r, h));
#pragma unroll
                for (int b = 0; b < TDT; ++b)
                    df[b][pt] = *reinterpret_cast<const h8*>(st + (pt * 2 + ks) * BD * 32 + fimg(d_w + 32 * b + r, h));
            }
#if SIR_ABL_NT & 8
#pragma unroll
            for (int a = 0; a < TFT; ++a)
#pragma unroll
                for (int b = 0; b < TDT; ++b)
                    asm volatile("" :: "v"(wf[a][0]), "v"(wf[a][1]), "v"(df[b][0]), "v"(df[b][1]));   // timing-only
            continue;
#endif
#pragma unroll
            for (int a = 0; a < TFT; ++a)
#pragma unroll
                for (int b = 0; b < TDT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[a][0], df[b][0],
                                                                       (zinit && ks == 0) ? zero : acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TFT; ++a)
#pragma unroll
                for (int b = 0; b < TDT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[a][0], df[b][1], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TFT; ++a)
#pragma unroll
                for (int b = 0; b < TDT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[a][1], df[b][0], acc[a][b], 0, 0, 0);
        }
    };
    // C[m][n] = acc * 2^-se(m) * inv_t[n] + bias[n], one buffer store per float4
    // Store offsets: the lane's row (voffset, so the range check drops rows past M) plus the
    // lane's column; the static column parts and f0 go to the scalar offset.  The lane indices are
    // re-derived from an opaque copy of threadIdx.x inside the epilogue: hoisted out of the tile
    // loop, its addresses and offsets would hold VGPRs through every step and force spills
    // (whose reloads, vector-memory ops, drain the load queue).
#if !SIR_NT_P_EPI
#error "the fragment-store persistent NT epilogue has no dropout"
#endif
#if SIR_NT_P_EPI
    // Epilogue through LDS (stage 1: free after a tile's last step — the next tile's first chunk
    // is in stage 0 — and the 64-row image of pitch BF*4 + 16 is exactly STAGE bytes): per round b
    // every wave writes its 32-row band b, then the block stores whole output rows (one 1-KiB row
    // per wave-instruction instead of 32 rows x 32 B; the 16-bit kernel's timing ablation put 45 %
    // of a GEMM on the fragment-order stores).  Called after the tile's last step; it ends with a
    // barrier, so the next tile's first split into stage 1 follows it.
    auto epilogue = [&](const TileP& p, int slot) {
        int tq = threadIdx.x;
        asm volatile("" : "+v"(tq));
        const int lq = tq & 63, rq = lq & 31, hq = lq >> 5, wq = tq >> 6;
        const int d_wq = (wq / WF) * TDT * 32, f_wq = (wq % WF) * TFT * 32;
        constexpr int PITCH = BF * 4 + 16;
        static_assert(64 * PITCH <= STAGE, "epilogue image fits the free stage");
        char* const img = lds + STAGE;
        const uint32_t ldc4 = (uint32_t)ldc * 4u;
        const uint32_t nrec = (uint32_t)p.rows * ldc4;
        const rsrc_t crs = mk_rsrc(C + p.d0 * ldc, (SIR_ABL_NT & 2) ? 0u : nrec);
        const rsrc_t grs = GATE == 2 ? mk_rsrc(reinterpret_cast<const char*>(gate) + p.d0 * 32, (uint32_t)p.rows * 32u)
                                     : mk_rsrc(GATE ? gate + p.d0 * ldc : C, GATE ? nrec : 0u);
        const float* sc = fin + slot * BD;
        char* const wrow = img + ((wq / WF) * 32 + rq) * PITCH + (f_wq + 4 * hq) * 4;
#pragma unroll
        for (int b = 0; b < TDT; ++b) {
            const float is = sc[d_wq + 32 * b + rq];
#pragma unroll
            for (int a = 0; a < TFT; ++a) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int n = p.f0 + f_wq + 32 * a + 8 * g + 4 * hq;
                    const float4 it = *reinterpret_cast<const float4*>(inv_l + n);
                    const float4 bb = *reinterpret_cast<const float4*>(bias_l + n);   // -0 without bias
                    float4 o;
                    o.x = acc[a][b][4 * g + 0] * is * it.x + bb.x;
                    o.y = acc[a][b][4 * g + 1] * is * it.y + bb.y;
                    o.z = acc[a][b][4 * g + 2] * is * it.z + bb.z;
                    o.w = acc[a][b][4 * g + 3] * is * it.w + bb.w;
                    if (drop.on()) drop4(drop, p.d0 + d_wq + 32 * b + rq, n, o);
                    *reinterpret_cast<float4*>(wrow + (32 * a + 8 * g) * 4) = o;
                }
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int ir = wq + 8 * i, c16 = lq;                 // image row, 16-B piece of it
                u4v v = *reinterpret_cast<const u4v*>(img + ir * PITCH + c16 * 16);
                const int ml = (ir >> 5) * (TDT * 32) + 32 * b + (ir & 31);
                const int n = p.f0 + 4 * c16;
                const uint32_t off = (n < N) ? (uint32_t)ml * ldc4 + (uint32_t)c16 * 16u : nrec;
                if constexpr (GATE == 2) {          // N = 256, f0 = 0: lane c16's 4 features 4 c16 + x
                    const u4v m01 = __builtin_amdgcn_raw_buffer_load_b128(grs, (uint32_t)ml * 32u, 0, 0);
                    const u4v m23 = __builtin_amdgcn_raw_buffer_load_b128(grs, (uint32_t)ml * 32u + 16u, 0, 0);
                    const int sh = c16 & 31;
                    const uint32_t w0 = c16 < 32 ? m01.x : m01.y, w1 = c16 < 32 ? m01.z : m01.w;
                    const uint32_t w2 = c16 < 32 ? m23.x : m23.y, w3 = c16 < 32 ? m23.z : m23.w;
                    const float g0 = ((w0 >> sh) & 1u) ? 1.f : -1.f, g1 = ((w1 >> sh) & 1u) ? 1.f : -1.f;
                    const float g2 = ((w2 >> sh) & 1u) ? 1.f : -1.f, g3 = ((w3 >> sh) & 1u) ? 1.f : -1.f;
                    v.x = __float_as_uint(gate_dact(g0, __uint_as_float(v.x), gate_relu, gate_slope));
                    v.y = __float_as_uint(gate_dact(g1, __uint_as_float(v.y), gate_relu, gate_slope));
                    v.z = __float_as_uint(gate_dact(g2, __uint_as_float(v.z), gate_relu, gate_slope));
                    v.w = __float_as_uint(gate_dact(g3, __uint_as_float(v.w), gate_relu, gate_slope));
                } else if constexpr (GATE == 1) {
                    const u4v gv = __builtin_amdgcn_raw_buffer_load_b128(grs, off, p.f0 * 4, 0);
                    v.x = __float_as_uint(gate_dact(__uint_as_float(gv.x), __uint_as_float(v.x), gate_relu, gate_slope));
                    v.y = __float_as_uint(gate_dact(__uint_as_float(gv.y), __uint_as_float(v.y), gate_relu, gate_slope));
                    v.z = __float_as_uint(gate_dact(__uint_as_float(gv.z), __uint_as_float(v.z), gate_relu, gate_slope));
                    v.w = __float_as_uint(gate_dact(__uint_as_float(gv.w), __uint_as_float(v.w), gate_relu, gate_slope));
                }
                __builtin_amdgcn_raw_buffer_store_b128(v, crs, off, p.f0 * 4, 0);
                // a 16-byte store reads its data VGPRs over several cycles (see below)
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_nop 1" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
            }
            __syncthreads();
        }
    };
#else
    auto epilogue = [&](const TileP& p, int slot) {
        int tq = threadIdx.x;
        asm volatile("" : "+v"(tq));
        const int lq = tq & 63, rq = lq & 31, hq = lq >> 5, wq = tq >> 6;
        const int d_wq = (wq / WF) * TDT * 32, f_wq = (wq % WF) * TFT * 32;
        const uint32_t ldc4 = (uint32_t)ldc * 4u;
        const uint32_t nrec = (uint32_t)p.rows * ldc4;
        const rsrc_t crs = mk_rsrc(C + p.d0 * ldc, (SIR_ABL_NT & 2) ? 0u : nrec);
        const float* sc = fin + slot * BD;
        // < 2^30: row < 256, ldc <= SIR_GEMM_MAX_LD
        const uint32_t rv = (uint32_t)(d_wq + rq) * ldc4 + (uint32_t)(f_wq + 4 * hq) * 4u;
#pragma unroll
        for (int b = 0; b < TDT; ++b) {
            const float is = sc[d_wq + 32 * b + rq];
            const uint32_t rb = rv + (uint32_t)(32 * b) * ldc4;
#pragma unroll
            for (int a = 0; a < TFT; ++a) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int nc0 = p.f0 + 32 * a + 8 * g;                 // wave-uniform column part
                    const int n = nc0 + f_wq + 4 * hq;
                    const float4 it = *reinterpret_cast<const float4*>(inv_l + n);
                    float4 o;
                    o.x = acc[a][b][4 * g + 0] * is * it.x;
                    o.y = acc[a][b][4 * g + 1] * is * it.y;
                    o.z = acc[a][b][4 * g + 2] * is * it.z;
                    o.w = acc[a][b][4 * g + 3] * is * it.w;
                    const float4 bb = *reinterpret_cast<const float4*>(bias_l + n);   // -0 without bias
                    o.x += bb.x; o.y += bb.y; o.z += bb.z; o.w += bb.w;
                    u4v ov;
                    ov.x = __float_as_uint(o.x); ov.y = __float_as_uint(o.y);
                    ov.z = __float_as_uint(o.z); ov.w = __float_as_uint(o.w);
                    // columns past N: an offset at the end of the range (dropped)
                    __builtin_amdgcn_raw_buffer_store_b128(ov, crs, (n < N) ? rb : nrec, nc0 * 4, 0);
                    // A 16-byte store reads its data VGPRs over several cycles: hipcc (ROCm 7.2) put a
                    // v_pk_mul_f32 overwriting them right after the store with no wait state, and
                    // lanes 12-15 of each 16-lane group stored the new value (measured on MI355X).
                    // Pin the order and pad the window.
                    __builtin_amdgcn_sched_barrier(0);
                    asm volatile("s_nop 1" ::: "memory");
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
    };

#endif

#if SIR_NT_PRIO == 2
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
#endif
    TileP cur = tile_p(tb), nxt = tile_p(tb + 1);
    load_a(0, cur, 0);
    load_w(cur, 0);
    store(0, 0, true, false, 0);
    load_a(1, cur, 1);
    load_w(cur, 1);
    load_a(0, cur, 2);
    __syncthreads();
    // step c: chunk c is multiplied out of stage c&1; chunk c+1 (registers, set (c+1)&1) is split
    // into the other stage; W(c+2) and A(c+3) (into the freed set) are issued.  Chunks past the
    // tile's last belong to the next tile.  Steps 0 and NCT-3 .. NCT-1 are written out (first
    // chunk / tile crossing); the ones between run as a loop of step pairs (static set parity).
    // SK: 0 store chunk c+1 of this tile, 1 the same as the tile's last chunk, 2 the next tile's
    // chunk 0; WN / AN: W(c+2) / A(c+3) come from the next tile.
    typedef std::integral_constant<int, 0> I0;
    typedef std::integral_constant<int, 1> I1;
    typedef std::integral_constant<int, 2> I2;
    // LATE (SIR_NT_STAGGER, waves 4-7 = the second wave of every SIMD): split the next chunk
    // BEFORE the MFMAs of the step instead of after, so that on each SIMD one wave's MFMAs run
    // beside its partner's split VALU / LDS writes rather than both waves doing the same phase
    // together (MI355X_MICROARCH.md "Two waves per SIMD" item 9).  Within a step the order is
    // free: the MFMAs read stage P, the split writes stage P^1, the barrier closes the step.
    auto step = [&](int c, int j, const TileP& cu, const TileP& nx, auto P_, auto Z_, auto SK_, auto WN_, auto AN_,
                    auto L_) {
        constexpr int P = decltype(P_)::value, SK = decltype(SK_)::value;
        constexpr bool Z = decltype(Z_)::value != 0, WN = decltype(WN_)::value != 0, AN = decltype(AN_)::value != 0;
        constexpr bool LATE = decltype(L_)::value != 0;
        if constexpr (!Z) rescale(P);
        auto split = [&]() {
            if constexpr (SK == 2) store(0, 0, true, false, 0);
            else store(P ^ 1, P ^ 1, false, SK == 1, j & 1);
        };
        if constexpr (LATE) split();
#if SIR_NT_STAGGER == 3
        const bool late_w = __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256;
        if (late_w) split();
#endif
#if SIR_NT_PRIO == 1
        __builtin_amdgcn_s_setprio(1);
#endif
        mfma(P, Z);
#if SIR_NT_PRIO == 1
        __builtin_amdgcn_s_setprio(0);
#endif
#if SIR_NT_STAGGER == 3
        if (!late_w) split();
#else
        if constexpr (!LATE) split();
#endif
        if constexpr (WN) load_w(nx, c + 2 - NCT);
        else load_w(cu, c + 2);
        if constexpr (AN) load_a(P ^ 1, nx, c + 3 - NCT);
        else load_a(P ^ 1, cu, c + 3);
        __syncthreads();
    };
    auto run = [&](auto L_) {
        TileP cu = cur, nx = nxt;
        for (int j = 0; tb + j < te; ++j) {
            const TileP nn = tile_p(tb + j + 2);
            step(0, j, cu, nx, I0(), I1(), I0(), I0(), I0(), L_);
#if SIR_NT_P_UNROLL
#pragma unroll
#endif
            for (int c = 1; c + 1 <= NCT - 4; c += 2) {
                step(c, j, cu, nx, I1(), I0(), I0(), I0(), I0(), L_);
                step(c + 1, j, cu, nx, I0(), I0(), I0(), I0(), I0(), L_);
            }
            step(NCT - 3, j, cu, nx, I1(), I0(), I0(), I0(), I1(), L_);
            step(NCT - 2, j, cu, nx, I0(), I0(), I1(), I1(), I1(), L_);
            step(NCT - 1, j, cu, nx, I1(), I0(), I2(), I1(), I1(), L_);
            epilogue(cu, j & 1);
            cu = nx;
            nx = nn;
        }
    };
#if SIR_NT_STAGGER == 2
    run(I1());
#elif SIR_NT_STAGGER == 3
    run(I0());
#elif SIR_NT_STAGGER
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) run(I1());
    else run(I0());
#else
    run(I0());
#endif
}

// ------------------------------------------------------------------------------------------
// TN GEMM (split over row ranges).  WM x WN waves, each TMT x TNT tiles of 32 x 32.
// Loader: one slot per thread — threads [0, 2BM) own column t/2 of the A block, threads
// [2BM, 2BM+2BN) column (t-2BM)/2 of the B block; t&1 selects the k-step (16 rows of the chunk).
template <int WM, int WN, int TMT, int TNT>
__global__ void __launch_bounds__(64 * WM * WN)
k_gemm_tn(const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb,
          int64_t R, int Mc, int Nc, float* __restrict__ part, float* __restrict__ csum_part,
          int n_mtiles, int n_ntiles, int64_t rows_per_split) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BM = 32 * TMT * WM, BN = 32 * TNT * WN;
    // loader: one column slot per KSPT threads — KSPT = 1: a thread loads one k-step (16 rows)
    // of its column, its partner (t ^ 1) the other; KSPT = 2: a thread loads all 32 rows
    constexpr int KSPT = 2 * (BM + BN) / NT;
    static_assert(KSPT * NT == 2 * (BM + BN) && (KSPT == 1 || KSPT == 2), "loader mapping");
    constexpr int XR = 16 * KSPT;            // rows of its column a thread loads per chunk
    constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
    constexpr int STAGE = A_BYTES + B_BYTES + (BM + BN) * 4;
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE + 16];
    // per stage: index of the chunk in it if some column's scale changed with that chunk (a
    // same-value store by every such thread; no reset needed, chunk indices are unique)
    int* const rescaled = reinterpret_cast<int*>(lds + 2 * STAGE);

    const int t = threadIdx.x;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int tiles = n_mtiles * n_ntiles;
    const int p = wg / tiles, tile = wg % tiles;
    const int m0 = (tile / n_ntiles) * BM, n0 = (tile % n_ntiles) * BN;
    const int64_t v_begin = (int64_t)p * rows_per_split;
    const int64_t v_end = (v_begin + rows_per_split < R) ? v_begin + rows_per_split : R;
    const int nc = (int)((v_end - v_begin + KC - 1) / KC);

    // loader slot (A or B is wave-uniform: waves [0, BM/32) load A)
    const int slot = KSPT == 1 ? (t >> 1) : t;
    const bool is_a = __builtin_amdgcn_readfirstlane(t >> 6) < BM * (2 / KSPT) / 64;
    const int cl = is_a ? slot : slot - BM, kse = KSPT == 1 ? (t & 1) : 0;
    const bool col_ok = is_a ? (m0 + cl < Mc) : (n0 + cl < Nc);
    const float* xbase = is_a ? A : B;
    const int ldx = (int)(is_a ? lda : ldb);
    const int xoff = 16 * kse * ldx + (is_a ? m0 : n0) + (col_ok ? cl : 0);   // within a chunk
    const int img = is_a ? 0 : A_BYTES, rows_img = is_a ? BM : BN, fac_off = is_a ? cl : BM + cl;
    // this thread's LDS destinations within a stage, folded into two offsets (fewer live VGPRs)
    const int hi_off = img + kse * rows_img * 32 + fimg(cl, 0);
    const int lo_delta = 2 * rows_img * 32;
    const int fac_byte = A_BYTES + B_BYTES + fac_off * 4;
    int se_run = SE_INIT;

    const int w = t >> 6, l = t & 63, r = l & 31, h = l >> 5;
    const int m_w = (w / WN) * TMT * 32, n_w = (w % WN) * TNT * 32;

    float4 xv_[SIR_TN_PF][XR / 4];
    // bias gradient of the same linear (column sums of A) rides on the A loads: one partial row
    // per split, written by the blocks of the first n-tile
    const bool do_cs = csum_part != nullptr && is_a;
    float cs = 0.f, csc = 0.f;
    auto load = [&](int set, int c) {
        float4 (&xv)[XR / 4] = xv_[set];
        const int64_t vc = v_begin + (int64_t)c * KC;
        const float* src = xbase + vc * ldx;                 // wave-uniform chunk base
        float x[XR];
#if SIR_TN_PF == 2
        // one branch-free form for every chunk (a load on only one side of a branch makes the
        // compiler's wait counts pessimistic): rows past v_end, and whole chunks past the split,
        // fail the range check and read as 0
        const int64_t nrow = v_end - vc;
        const rsrc_t rs = mk_rsrc(src, (SIR_ABL_TN || nrow <= 0) ? 0u : (uint32_t)((nrow < KC ? nrow : KC) * ldx * 4));
#pragma unroll
        for (int j = 0; j < XR; ++j)
            x[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, xoff * 4, j * ldx * 4, 0));
#else
        if (vc + KC <= v_end) {
            const rsrc_t rs = mk_rsrc(src, SIR_ABL_TN ? 0u : (uint32_t)(KC * ldx * 4));
#pragma unroll
            for (int j = 0; j < XR; ++j)
                x[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, xoff * 4, j * ldx * 4, 0));
        } else {   // tail chunk: rows past v_end fail the range check and read as 0
            const rsrc_t rs = mk_rsrc(src, SIR_ABL_TN ? 0u : (uint32_t)((v_end - vc) * ldx * 4));
            int o = xoff * 4;
            asm volatile("" : "+v"(o));      // keep the offsets out of the loop preheader
#pragma unroll
            for (int j = 0; j < XR; ++j)
                x[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, o + j * ldx * 4, 0, 0));
        }
#endif
        // no zeroing of columns past Mc / Nc (they re-read column 0): such a column only feeds
        // its own output row / column, which is never stored, under its own scale.  A select
        // here would make the compiler wait for the loads right after issuing them.
#pragma unroll
        for (int j = 0; j < XR / 4; ++j) xv[j] = make_float4(x[4 * j], x[4 * j + 1], x[4 * j + 2], x[4 * j + 3]);
    };
    auto store = [&](int set, int buf, int chunk, bool first = false) {   // first chunk: factor 1 (acc is zero)
        const float4 (&xv)[XR / 4] = xv_[set];
        char* st = lds + buf * STAGE;
        float m = 0.f;
#pragma unroll
        for (int j = 0; j < XR / 4; ++j) m = SIR_SPLIT_MIX ? fmax4_mix(m, xv[j]) : fmax4(m, xv[j]);
        if (KSPT == 1) m = fmaxf(m, __shfl_xor(m, 1));
        const int se_old = se_run, se = next_se(se_old, bexp(m));
        se_run = se;
        const float s = pow2(se);
#pragma unroll
        for (int q = 0; q < KSPT; ++q) {      // k-step kse + q: rows 16q .. 16q+15 of x
            h8 hv[2], lv[2];
            if constexpr (SIR_SPLIT_MIX) {
                split8_mix(xv[4 * q + 0], xv[4 * q + 1], s, hv[0], lv[0]);
                split8_mix(xv[4 * q + 2], xv[4 * q + 3], s, hv[1], lv[1]);
            } else {
                split8(xv[4 * q + 0], xv[4 * q + 1], s, hv[0], lv[0]);
                split8(xv[4 * q + 2], xv[4 * q + 3], s, hv[1], lv[1]);
            }
            char* hd = st + hi_off + q * rows_img * 32;    // fimg(cl, 1) = fimg(cl, 0) + 512
            *reinterpret_cast<h8*>(hd) = hv[0];
            *reinterpret_cast<h8*>(hd + 512) = hv[1];
            *reinterpret_cast<h8*>(hd + lo_delta) = lv[0];
            *reinterpret_cast<h8*>(hd + lo_delta + 512) = lv[1];
        }
        if (kse == 0) *reinterpret_cast<float*>(st + fac_byte) = first ? 1.f : pow2(se - se_old);
        if (do_cs) {           // column sums of A from the fp32 values: per-chunk sum, Kahan-added to the total
            float t = 0.f;
#pragma unroll
            for (int j = 0; j < XR / 4; ++j) { t += xv[j].x; t += xv[j].y; t += xv[j].z; t += xv[j].w; }
            kahan_add(cs, csc, t);
        }
        if (!first && se != se_old) rescaled[buf] = chunk;
    };

    f16v acc[TMT][TNT];
#pragma unroll
    for (int a = 0; a < TMT; ++a)
#pragma unroll
        for (int b = 0; b < TNT; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

    auto compute = [&](int c) {
        const int buf = c & 1;
        const char* st = lds + buf * STAGE;
        if (rescaled[buf] == c) {
            const float* fac = reinterpret_cast<const float*>(st + A_BYTES + B_BYTES);
#pragma unroll
            for (int a = 0; a < TMT; ++a) {
                float fa[16];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 f4 = *reinterpret_cast<const float4*>(fac + m_w + 32 * a + 8 * g + 4 * h);
                    fa[4 * g] = f4.x; fa[4 * g + 1] = f4.y; fa[4 * g + 2] = f4.z; fa[4 * g + 3] = f4.w;
                }
#pragma unroll
                for (int b = 0; b < TNT; ++b) {
                    const float fb = fac[BM + n_w + 32 * b + r];
#pragma unroll
                    for (int i = 0; i < 16; ++i) acc[a][b][i] *= fa[i] * fb;
                }
            }
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            __builtin_amdgcn_sched_barrier(0);
            h8 af[TMT][2], bf[TNT][2];
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) {
#pragma unroll
                for (int a = 0; a < TMT; ++a)
                    af[a][pt] = *reinterpret_cast<const h8*>(st + (pt * 2 + ks) * BM * 32 + fimg(m_w + 32 * a + r, h));
#pragma unroll
                for (int b = 0; b < TNT; ++b)
                    bf[b][pt] = *reinterpret_cast<const h8*>(st + A_BYTES + (pt * 2 + ks) * BN * 32 + fimg(n_w + 32 * b + r, h));
            }
#pragma unroll
            for (int a = 0; a < TMT; ++a)
#pragma unroll
                for (int b = 0; b < TNT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[a][0], bf[b][0], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TMT; ++a)
#pragma unroll
                for (int b = 0; b < TNT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[a][0], bf[b][1], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < TMT; ++a)
#pragma unroll
                for (int b = 0; b < TNT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[a][1], bf[b][0], acc[a][b], 0, 0, 0);
        }
    };

    if (t < 2) rescaled[t] = -1;
#if SIR_TN_PF == 2
    // two chunks in flight: step c multiplies chunk c (stage c&1) while chunks c+1 (set (c+1)&1)
    // and c+2 (set c&1, issued at the top of the step) load; chunks past the split load as zeros
    // (empty range), so every step issues the same loads and the wait counts stay exact.
    if (nc > 0) {
        load(0, 0);
        load(1, 1);
        store(0, 0, 0, true);
    }
    __syncthreads();
    auto step = [&](int c, int set) {            // set = c & 1 (static)
        load(set, c + 2);
        compute(c);
        if (c + 1 < nc) store(set ^ 1, (c + 1) & 1, c + 1);
        __syncthreads();
    };
    int c = 0;
    for (; c + 2 <= nc; c += 2) {
        step(c, 0);
        step(c + 1, 1);
    }
    if (c < nc) step(c, 0);
#else
    if (nc > 0) {
        load(0, 0);
        store(0, 0, 0, true);
    }
    __syncthreads();
    for (int c = 0; c < nc; ++c) {
        const bool more = c + 1 < nc;
        if (more) load(0, c + 1);
        compute(c);
        if (more) store(0, (c & 1) ^ 1, c + 1);
        __syncthreads();
    }
#endif

    // epilogue: part[p][m][n] = acc * 2^-se_a(m) * 2^-se_b(n)
    float* sc = reinterpret_cast<float*>(lds);
    if (kse == 0) sc[fac_off] = pow2(-se_run);
    __syncthreads();
    float* out = part + (int64_t)p * Mc * Nc;
#pragma unroll
    for (int b = 0; b < TNT; ++b) {
        const int nl = n_w + 32 * b + r;
        const int n = n0 + nl;
        const float ib = sc[BM + nl];
#pragma unroll
        for (int a = 0; a < TMT; ++a) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int ml = m_w + 32 * a + (i & 3) + 8 * (i >> 2) + 4 * h;
                const int m = m0 + ml;
                if (m < Mc && n < Nc) out[(int64_t)m * Nc + n] = acc[a][b][i] * sc[ml] * ib;
            }
        }
    }
    if (do_cs && tile % n_ntiles == 0) {
        // KSPT = 1: the partner thread holds rows 16..31 of each chunk
        const float other = KSPT == 1 ? __shfl_xor(cs, 1) : 0.f;
        if (kse == 0 && col_ok) csum_part[(int64_t)p * Mc + m0 + cl] = KSPT == 1 ? cs + other : cs;
    }
}

// Partials added in split order; the loads are issued 16 at a time ahead of the (sequential,
// same-order) adds — a dependent one-load-per-add loop kept one load in flight per thread and
// took ~50 us per call at P = 256 (and longer for the many-split small shapes).
__global__ void __launch_bounds__(256)
k_gemm_reduce(const float* __restrict__ part, int P, int64_t count, int Nc, float* __restrict__ C, int64_t ldc) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    float s = 0.f;
    int q = 0;
    for (; q + 16 <= P; q += 16) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = part[(int64_t)(q + j) * count + i];
#pragma unroll
        for (int j = 0; j < 16; ++j) s += v[j];
    }
    for (; q < P; ++q) s += part[(int64_t)q * count + i];
    C[(i / Nc) * ldc + i % Nc] = s;
}

// ------------------------------------------------------------------------------------------
// Small-batch GEMMs (fewer than gemm_small_rows() node rows: config-5 / config-1 / ZINC batches of
// a few thousand nodes).  The block-tiled kernels above have 256-row tiles: a 1.6k-row batch is 7
// tiles on a 256-CU chip.  Here ONE WAVE owns one small output tile and runs alone — no LDS stage,
// no barrier: its operand fragments come straight from global memory into registers (the data
// rows' fp32 values, split in registers; the packed weight's fragments, in lane order, from L2),
// the next 32-k chunk in flight while the current one is multiplied.  Same split, running-scale
// rule and MFMA order per accumulator as k_gemm_nt_p / k_gemm_tn, so the NT result is
// bit-identical to k_gemm_nt_p's (tests/test_gemm_gpu.py).
//
// k_gemm_nt_s: wave = 32 data rows x 32*S_FT features.  Lane l = 32h + r holds row r's k-range
// 8h .. 8h+7 of each k16 step (the MFMA B-operand fragment), i.e. two 32-B pieces per 32-k chunk.
constexpr int S_FT = 2;

template <bool KFULL>
__global__ void __launch_bounds__(256)
k_gemm_nt_s(const float* __restrict__ A, int64_t lda, int64_t M, int K, const u4v* __restrict__ Wp, int Npad, int Kc,
            const float* __restrict__ inv_t, const float* __restrict__ bias, int N, float* __restrict__ C, int64_t ldc,
            int nfg, int64_t n_waves, Drop drop) {
    drop = drop_resolve(drop);
    const int l = threadIdx.x & 63, r = l & 31, h = l >> 5;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= n_waves) return;                       // whole waves (4 per block)
    const int64_t d0 = (w / nfg) * 32;
    const int f0 = (int)(w % nfg) * S_FT;           // first 32-feature tile
    const int rows = (M - d0 < 32) ? (int)(M - d0) : 32;
    const rsrc_t ars = mk_rsrc(A + d0 * lda, (uint32_t)(rows * lda * 4));
    const rsrc_t wrs = mk_rsrc(Wp, (uint32_t)((int64_t)Kc * 4 * Npad * 32));
    const int aoff = (r * (int)lda + 8 * h) * 4;
    const int woff = 16 * l;
    float4 av[2][4];                                // [set][ks * 2 + q]: k = 32c + 16ks + 8h + 4q + (0..3)
    u4v wv[2][S_FT][2][2];                          // [set][tile][part][ks]
    auto load = [&](int set, int c) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u4v u = __builtin_amdgcn_raw_buffer_load_b128(ars, aoff + ((i >> 1) * 16 + (i & 1) * 4) * 4, c * KC * 4, 0);
            av[set][i] = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
        }
#pragma unroll
        for (int a = 0; a < S_FT; ++a)
#pragma unroll
            for (int pt = 0; pt < 2; ++pt)
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
                    wv[set][a][pt][ks] = __builtin_amdgcn_raw_buffer_load_b128(
                        wrs, woff, ((c * 2 + pt) * 2 + ks) * Npad * 32 + (f0 + a) * 1024, 0);
    };
    f16v acc[S_FT];
#pragma unroll
    for (int a = 0; a < S_FT; ++a)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[a][i] = 0.f;
    int se_run = SE_INIT;
    auto chunk = [&](int set, int c, bool first) {
        float4 x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = av[set][i];
        if (!KFULL && c == Kc - 1) {                 // columns past K (the next row's values) read as 0
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int k = c * KC + (i >> 1) * 16 + 8 * h + (i & 1) * 4;
                x[i].x = k + 0 < K ? x[i].x : 0.f;
                x[i].y = k + 1 < K ? x[i].y : 0.f;
                x[i].z = k + 2 < K ? x[i].z : 0.f;
                x[i].w = k + 3 < K ? x[i].w : 0.f;
            }
        }
        float m = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) m = fmax4(m, x[i]);
        m = fmaxf(m, __shfl_xor(m, 32));
        const int se_old = first ? SE_INIT : se_run, se = next_se(se_old, bexp(m));
        se_run = se;
        if (!first) {
            const float f = pow2(se - se_old);
            if (__builtin_amdgcn_ballot_w64(f != 1.f) != 0) {
#pragma unroll
                for (int a = 0; a < S_FT; ++a) acc[a] *= f;
            }
        }
        const float s = pow2(se);
        h8 dh[2], dl[2];
        split8(x[0], x[1], s, dh[0], dl[0]);
        split8(x[2], x[3], s, dh[1], dl[1]);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int a = 0; a < S_FT; ++a)
                acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, wv[set][a][0][ks]), dh[ks], acc[a], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < S_FT; ++a)
                acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, wv[set][a][0][ks]), dl[ks], acc[a], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < S_FT; ++a)
                acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, wv[set][a][1][ks]), dh[ks], acc[a], 0, 0, 0);
        }
    };
    // chunk pairs with static register sets; every pair issues its loads (the last chunk's are
    // re-issued past the end: same addresses, unused), so the wait counts stay exact
    load(0, 0);
    int c = 0;
    for (; c + 2 <= Kc; c += 2) {
        load(1, c + 1);
        chunk(0, c, c == 0);
        load(0, (c + 2 < Kc) ? c + 2 : Kc - 1);
        chunk(1, c + 1, false);
    }
    if (c < Kc) chunk(0, c, c == 0);

    // C[m][n] = acc * 2^-se(m) * inv_t[n] + bias[n] (k_gemm_nt_p's epilogue arithmetic)
    const float is = pow2(-se_run);
    const int64_t row = d0 + r;
    if (row < M) {
#pragma unroll
        for (int a = 0; a < S_FT; ++a) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = (f0 + a) * 32 + 8 * g + 4 * h;
                if (n < N) {
                    const float4 it = *reinterpret_cast<const float4*>(inv_t + n);
                    const float4 bb = bias != nullptr ? *reinterpret_cast<const float4*>(bias + n)
                                                      : make_float4(-0.f, -0.f, -0.f, -0.f);
                    float4 o;
                    o.x = acc[a][4 * g + 0] * is * it.x + bb.x;
                    o.y = acc[a][4 * g + 1] * is * it.y + bb.y;
                    o.z = acc[a][4 * g + 2] * is * it.z + bb.z;
                    o.w = acc[a][4 * g + 3] * is * it.w + bb.w;
                    if (drop.on()) drop4(drop, row, n, o);
                    *reinterpret_cast<float4*>(C + row * ldc + n) = o;
                }
            }
        }
    }
}

// Small contractions with both operands split in the kernel (no packed weight): a block of 4 waves
// owns one 32 x 32 output tile, the waves take the 32-k chunks c = q, q + 4, ... of the contraction
// (up to 4 chunks' operands loaded at once: one memory latency per 4 chunks, not one per chunk), each
// with running scales on both operands (k_gemm_tn's rule), and the 4 partial tiles are added in wave
// order through LDS.  Operand line j (an MFMA row of src0 / column of src1) of lane l = 32h + j holds
// k = 32c + 16ks + 8h + (0..7): CONTIG lines run along k in memory (x[j * ld + k]: A rows, an
// nn.Linear weight's rows), strided ones across it (x[k * ld + j]: the node-row contraction of the
// weight gradients, a transposed weight).
//   k_gemm_nt_sw : C = A W^T + bias (or A W), W read as fp32 (sir_gemm_nt_direct)
//   k_gemm_tn_s  : part[p] = A[rows_p]^T B[rows_p] (+ column sums of A)
template <bool CONTIG>
struct SOp {
    const float* x;      // element (line 0, k 0) of the tile
    int64_t ld;          // elements between lines (CONTIG) / between k (strided)
    int lines, klen;     // valid lines, contraction length
    int j;               // this lane's line, clamped to a valid one
    // the lane's 16 values of chunk c (zeros past klen; lines past `lines` re-read line 0's values:
    // they feed only their own outputs, which are never stored)
    __device__ __forceinline__ void load(float (&v)[16], int c, bool live, int h) const {
        if constexpr (CONTIG) {
            const rsrc_t rs = mk_rsrc(x, live ? (uint32_t)((int64_t)lines * ld * 4) : 0u);
            const int voff = (int)((j * ld + 8 * h) * 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const u4v u = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, (c * KC + (i >> 1) * 16 + (i & 1) * 4) * 4, 0);
                v[4 * i + 0] = __uint_as_float(u.x); v[4 * i + 1] = __uint_as_float(u.y);
                v[4 * i + 2] = __uint_as_float(u.z); v[4 * i + 3] = __uint_as_float(u.w);
            }
        } else {
            const int64_t k0 = (int64_t)c * KC;
            const int64_t left = klen - k0;
            const uint32_t kr = (!live || left <= 0) ? 0u : (uint32_t)(left < KC ? left : KC);
            const rsrc_t rs = mk_rsrc(x + (kr ? k0 : 0) * ld, kr * (uint32_t)ld * 4u);
            const int voff = (int)((8 * h * ld + j) * 4);
#pragma unroll
            for (int i = 0; i < 16; ++i)
                v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, ((i >> 3) * 16 + (i & 7)) * (int)ld * 4, 0));
        }
    }
    // CONTIG: k past klen inside the last chunk reads the next line's values -> zero them
    __device__ __forceinline__ void mask_tail(float (&v)[16], int c, int h) const {
        if constexpr (CONTIG) {
            if ((c + 1) * KC > klen) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int k = c * KC + (i >> 3) * 16 + 8 * h + (i & 7);
                    v[i] = k < klen ? v[i] : 0.f;
                }
            }
        }
    }
};

// One wave's 32 x 32 split-fp16 tile, fed one 32-k chunk at a time: x0 = the lane's 16 values of
// its src0 line (MFMA row), x1 of its src1 line (MFMA column), each line with its running scale
// (k_gemm_tn's rule); with CS also the Kahan sum of the lane's src0 values.
struct SplitTile {
    f16v acc;
    int se0 = SE_INIT, se1 = SE_INIT;
    bool first = true;
    float cs = 0.f, csc = 0.f;
    __device__ __forceinline__ SplitTile() {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    }
    static __device__ __forceinline__ float colmax(const float (&x)[16]) {
        float mm = 0.f;
#pragma unroll
        for (int i = 0; i < 16; i += 4) mm = fmax4(mm, make_float4(x[i], x[i + 1], x[i + 2], x[i + 3]));
        // with the partner half (lane ^ 32): v_permlane32_swap, no LDS round trip
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mm), __float_as_uint(mm), false, false);
        return fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    template <bool CS>
    __device__ __forceinline__ void step(const float (&x0)[16], const float (&x1)[16], int h) {
        const int s0 = first ? SE_INIT : se0, s1 = first ? SE_INIT : se1;
        se0 = next_se(s0, bexp(colmax(x0)));
        se1 = next_se(s1, bexp(colmax(x1)));
        if (!first) {
            const float f0 = pow2(se0 - s0), f1 = pow2(se1 - s1);
            if (__builtin_amdgcn_ballot_w64(f0 != 1.f || f1 != 1.f) != 0) {
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[i] *= __shfl(f0, (i & 3) + 8 * (i >> 2) + 4 * h) * f1;
            }
        }
        first = false;
        if constexpr (CS) {
            float t = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) t += x0[i];
            kahan_add(cs, csc, t);
        }
        h8 ah[2], al[2], bh[2], bl[2];
        const float sa = pow2(se0), sb = pow2(se1);
        split8(make_float4(x0[0], x0[1], x0[2], x0[3]), make_float4(x0[4], x0[5], x0[6], x0[7]), sa, ah[0], al[0]);
        split8(make_float4(x0[8], x0[9], x0[10], x0[11]), make_float4(x0[12], x0[13], x0[14], x0[15]), sa, ah[1], al[1]);
        split8(make_float4(x1[0], x1[1], x1[2], x1[3]), make_float4(x1[4], x1[5], x1[6], x1[7]), sb, bh[0], bl[0]);
        split8(make_float4(x1[8], x1[9], x1[10], x1[11]), make_float4(x1[12], x1[13], x1[14], x1[15]), sb, bh[1], bl[1]);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[ks], bh[ks], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[ks], bl[ks], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[ks], bh[ks], acc, 0, 0, 0);
        }
    }
    // the tile in true scale: acc * 2^-se0(row i) * 2^-se1(lane column)
    __device__ __forceinline__ void result(float (&p)[16], int h) const {
        const float i0 = pow2(-se0), i1 = pow2(-se1);
#pragma unroll
        for (int i = 0; i < 16; ++i) p[i] = acc[i] * __shfl(i0, (i & 3) + 8 * (i >> 2) + 4 * h) * i1;
    }
};

// The contraction of one wave: chunks q, q + 4, ... < nc; returns the partial tile in true scale
// in p, and (if CS) the sums of the lane's src0 values.
template <bool C0, bool C1, bool CS>
__device__ __forceinline__ void small_contract(const SOp<C0>& o0, const SOp<C1>& o1, int nc, int q, int h,
                                               float (&p)[16], float& cs) {
    SplitTile t;
    for (int cb = q; cb < nc; cb += 16) {
        float x0[4][16], x1[4][16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int c = cb + 4 * g;
            o0.load(x0[g], c, c < nc, h);
            o1.load(x1[g], c, c < nc, h);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int c = cb + 4 * g;
            if (c >= nc) break;
            o0.mask_tail(x0[g], c, h);
            o1.mask_tail(x1[g], c, h);
            t.step<CS>(x0[g], x1[g], h);
        }
    }
    t.result(p, h);
    cs = t.cs;
}

// C[d0 + r][n0 + n] = sum_k A[d0 + r][k] W(n0 + n, k) + bias: src0 = W lines (features), src1 = A rows
template <bool TRANS>
__global__ void __launch_bounds__(256)
k_gemm_nt_sw(const float* __restrict__ A, int64_t lda, int64_t M, int K, const float* __restrict__ W, int64_t ldw,
             int N, const float* __restrict__ bias, float* __restrict__ C, int64_t ldc, int nft, Drop drop) {
    drop = drop_resolve(drop);
    __shared__ float red[4][16][64];
    const int l = threadIdx.x & 63, r = l & 31, h = l >> 5, q = threadIdx.x >> 6;
    const int64_t d0 = (int64_t)(blockIdx.x / nft) * 32;
    const int n0 = (int)(blockIdx.x % nft) * 32;
    const int rows = (M - d0 < 32) ? (int)(M - d0) : 32, feats = (N - n0 < 32) ? N - n0 : 32;
    SOp<true> oa{A + d0 * lda, lda, rows, K, r < rows ? r : 0};
    SOp<!TRANS> ow{TRANS ? W + n0 : W + (int64_t)n0 * ldw, ldw, feats, K, r < feats ? r : 0};
    float p[16], cs = 0.f;
    small_contract<!TRANS, true, false>(ow, oa, (K + KC - 1) / KC, q, h, p, cs);
#pragma unroll
    for (int i = 0; i < 16; ++i) red[q][i][l] = p[i];
    __syncthreads();
    // wave q: acc elements 4q .. 4q+3 = features n0 + 8q + 4h + (0..3) of data row d0 + r
    const int64_t row = d0 + r;
    const int n = n0 + 8 * q + 4 * h;
    if (row < M && n < N) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int i = 4 * q + e;
            v[e] = ((red[0][i][l] + red[1][i][l]) + red[2][i][l]) + red[3][i][l];
        }
        const float4 bb = bias != nullptr ? *reinterpret_cast<const float4*>(bias + n) : make_float4(-0.f, -0.f, -0.f, -0.f);
        float4 o = make_float4(v[0] + bb.x, v[1] + bb.y, v[2] + bb.z, v[3] + bb.w);
        if (drop.on()) drop4(drop, row, n, o);
        *reinterpret_cast<float4*>(C + row * ldc + n) = o;
    }
}

// part[p][m0 + m][n0 + n] = sum over the split's rows of A[v][m0 + m] B[v][n0 + n]: src0 = A columns,
// src1 = B columns (both strided: the contraction runs over the node rows)
__global__ void __launch_bounds__(256)
k_gemm_tn_s(const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb, int64_t R, int Mc,
            int Nc, float* __restrict__ part, float* __restrict__ csum_part, int nmt, int nnt, int64_t rps) {
    __shared__ float red[4][16][64];
    __shared__ float cred[4][64];
    const int l = threadIdx.x & 63, r = l & 31, h = l >> 5, q = threadIdx.x >> 6;
    const int tiles = nmt * nnt;
    const int64_t p = blockIdx.x / tiles;
    const int mt = (int)(blockIdx.x % tiles) / nnt, nt = (int)(blockIdx.x % tiles) % nnt;
    const int m0 = mt * 32, n0 = nt * 32;
    const int64_t v0 = p * rps, v1 = (v0 + rps < R) ? v0 + rps : R;
    const int klen = v1 > v0 ? (int)(v1 - v0) : 0;
    const int mcols = (Mc - m0 < 32) ? Mc - m0 : 32, ncols = (Nc - n0 < 32) ? Nc - n0 : 32;
    SOp<false> oa{A + (klen ? v0 : 0) * lda + m0, lda, mcols, klen, r < mcols ? r : 0};
    SOp<false> ob{B + (klen ? v0 : 0) * ldb + n0, ldb, ncols, klen, r < ncols ? r : 0};
    const bool do_cs = csum_part != nullptr && nt == 0;
    float pv[16], cs = 0.f;
    if (do_cs) small_contract<false, false, true>(oa, ob, (klen + KC - 1) / KC, q, h, pv, cs);
    else small_contract<false, false, false>(oa, ob, (klen + KC - 1) / KC, q, h, pv, cs);
#pragma unroll
    for (int i = 0; i < 16; ++i) red[q][i][l] = pv[i];
    cred[q][l] = cs;
    __syncthreads();
    // wave q: acc elements 4q .. 4q+3 = A columns m0 + 8q + 4h + (0..3), B column n0 + r
    float* out = part + p * (int64_t)Mc * Nc;
    const int n = n0 + r;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int i = 4 * q + e, m = m0 + 8 * q + 4 * h + e;
        const float v = ((red[0][i][l] + red[1][i][l]) + red[2][i][l]) + red[3][i][l];
        if (m < Mc && n < Nc) out[(int64_t)m * Nc + n] = v;
    }
    if (do_cs && q == 0 && h == 0 && r < mcols) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) t += cred[w][r] + cred[w][r + 32];
        csum_part[p * Mc + m0 + r] = t;
    }
}

// k_gemm_reduce over the product partials [P][count] and, in the same launch (blocks past the
// product's), the column-sum partials [P][Mc]: one launch fewer per weight gradient
__global__ void __launch_bounds__(256)
k_gemm_reduce2(const float* __restrict__ part, int P, int64_t count, int Nc, float* __restrict__ C, int64_t ldc,
               const float* __restrict__ cpart, int Mc, float* __restrict__ colsum, int64_t nb_main) {
    const bool cs = blockIdx.x >= nb_main;
    const int64_t i = (int64_t)(cs ? blockIdx.x - nb_main : blockIdx.x) * 256 + threadIdx.x;
    const float* src = cs ? cpart : part;
    const int64_t cnt = cs ? (int64_t)Mc : count;
    if (i >= cnt) return;
    // the P split partials in split order: sums of 16, Kahan-added (a column sum of a few hundred
    // partials of mixed sign loses ~P ulps of the largest partial in a plain sequential sum)
    float s = 0.f, c = 0.f;
    int q = 0;
    for (; q + 16 <= P; q += 16) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = src[(int64_t)(q + j) * cnt + i];
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) t += v[j];
        kahan_add(s, c, t);
    }
    for (; q < P; ++q) kahan_add(s, c, src[(int64_t)q * cnt + i]);
    if (cs) colsum[i] = s;
    else C[(i / Nc) * ldc + i % Nc] = s;
}

// ------------------------------------------------------------------------------------------
// LDS-tiled small GEMMs (the small-batch route: config 5's 1.6k-node batches).  A block of 4 waves
// owns a (32 W0) x (32 W1) output tile: W0 x W1 waves of 32 x 32, times WK waves that take the
// 32-k chunks of each step in turn (partials added in LDS, in wave order).  The operands' k-slices
// of a step (32 WK k) go global -> LDS by LDS-DMA (global_load_lds_dwordx4: no registers, whole
// 128-byte lines per 8 lanes) into a ring of NS stage buffers, NS - 1 steps in flight ahead of the
// one being read (counted vmcnt + a raw barrier; the 4-wave k_gemm_nt_sw / k_gemm_tn_s load 16
// scattered bytes per line and lane, every wave its own copy, one memory latency per 4 chunks);
// each wave then reads its lines in the MFMA operand layout and runs SplitTile on them.
// Operand 0 feeds the MFMA rows, operand 1 the columns.  CONTIG operands are line-major in memory
// (x[line * ld + k]: A rows, an nn.Linear weight), imaged [line][32 WK k] with the 16-byte slots of
// each line XOR-swizzled (the DMA writes lane-linear; the swizzle goes on the source address, the
// reads undo it: conflict-free ds_read_b128); strided ones are k-major (x[k * ld + line]: the
// node-row contraction of the weight gradients, a transposed weight), imaged [k][line].
//   EPI 0 (NT): C[op1 line][op0 line] = sum_k + bias, dropout  (op0 = W lines, op1 = A rows)
//   EPI 1 (TN): part[p][op0 line][op1 line] (+ column sums of op0)  (op0 = A cols, op1 = B cols)
template <bool C0, bool C1, int W0, int W1, int WK, int NS>
struct Lt {
    static constexpr int NT = 64 * W0 * W1 * WK;                              // threads (4 or 8 waves)
    static constexpr int L0 = 32 * W0, L1 = 32 * W1, KS = 32 * WK;
    static constexpr int F0 = L0 * KS, F1 = L1 * KS;                          // floats per stage image
    static constexpr int BUF = F0 + F1;
    static constexpr int N0 = L0 * KS / (4 * NT), N1 = L1 * KS / (4 * NT);    // DMAs per thread per step
    static constexpr int D = N0 + N1;
    static constexpr int RED = (WK - 1) * W0 * W1 * 16 * 64;                  // partial-tile floats
    static constexpr int CRED = 2 * W0 * 32 * WK;                             // column-sum halves
    static constexpr int LDS = (NS * BUF > RED + CRED ? NS * BUF : RED + CRED);
    static_assert(NT == 256 || NT == 512, "4 or 8 waves");
    static_assert(N0 >= 1 && N1 >= 1 && N0 * 4 * NT == L0 * KS && N1 * 4 * NT == L1 * KS, "whole DMAs per thread");
    static_assert(NS >= 2 && (NS - 2) * D <= 63, "vmcnt range");
    static_assert(LDS * 4 <= 160 * 1024, "LDS");
};

__device__ __attribute__((aligned(16))) float g_lt_zero[4];    // source of the DMAs past the operand

// one operand of the block: element (line, k) of the block's tile at x[line * ld + k] (CONTIG) or
// x[k * ld + line]; lines >= `lines` and k >= `klen` read as zeros (k in 4-aligned groups: klen % 4 == 0
// for CONTIG operands, checked by the launchers).  Thread t of NT fills the 16-byte slots u = t + NT i
// (i < N) of every step's image (wave-instruction i of wave w: slots NT i + 64 w + lane); the
// slot's source at step 0 and its k offset are set up once, a step adds s * KS (CONTIG) or
// s * KS * ld (strided) elements.  TWO: the operand's weight-row index (the line for CONTIG, k for
// strided) continues from `split` on in a second array x2 (row r >= split at x2 + (r - split) ld2):
// the layer's [W_Q; W_K] read as it lies, no concatenated copy.  `row0`: the weight row of the
// tile's line / k 0; x2 is offset to the tile along the other index (k for CONTIG, line otherwise).
template <bool CONTIG, int L, int KS, int NT, bool TWO = false>
struct LtOp {
    static constexpr int NC = KS / 4;                                 // 16-byte slots per image line
    static constexpr int N = L * KS / (4 * NT);
    static constexpr bool SPLIT_K = TWO && !CONTIG;                  // the part is chosen per step
    const float* src[N];
    const float* src2[SPLIT_K ? N : 1];
    int kof[N];                                                       // slot k at step 0 (INT_MAX: dead line)
    int64_t step, step2;                                              // elements per step
    int klen, ksplit;
    __device__ __forceinline__ static int swz(int line) { return KS == 32 ? (line >> 1) & 7 : line & (NC - 1); }
    __device__ __forceinline__ LtOp(const float* x, int64_t ld, int lines, int klen_, int t, const float* x2 = nullptr,
                                    int64_t ld2 = 0, int64_t split = 0, int64_t row0 = 0)
        : klen(klen_), ksplit(0x7fffffff) {
        step = CONTIG ? (int64_t)KS : (int64_t)KS * ld;
        step2 = (int64_t)KS * ld2;
        if constexpr (SPLIT_K) {
            const int64_t ks = split - row0;
            ksplit = ks < 0 ? 0 : (ks > 0x7fffffff ? 0x7fffffff : (int)ks);
        }
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const int u = t + NT * i;
            int line, k;
            if constexpr (CONTIG) { line = u / NC; k = 4 * ((u % NC) ^ swz(u / NC)); }
            else { k = u / (L / 4); line = 4 * (u % (L / 4)); }
            if constexpr (CONTIG) {
                src[i] = (TWO && row0 + line >= split) ? x2 + (row0 + line - split) * ld2 + k : x + (int64_t)line * ld + k;
            } else {
                src[i] = x + (int64_t)k * ld + line;
                if constexpr (SPLIT_K) src2[i] = x2 + (row0 + k - split) * ld2 + line;
            }
            kof[i] = line < lines ? k : 0x7fffffff - KS * 4096;
        }
    }
    __device__ __forceinline__ const float* at(int i, int s) const {
        const int k = s * KS + kof[i];
        if (k >= klen) return g_lt_zero;
        if constexpr (SPLIT_K) {
            if (k >= ksplit) return src2[i] + s * step2;
        }
        return src[i] + s * step;
    }
    // the lane's 16 values of its line j, chunk kc of the step (k = 32 kc + 16 (i >> 3) + 8 h + (i & 7))
    __device__ __forceinline__ static void read(const float* img, int j, int kc, int h, float (&x)[16]) {
        if constexpr (CONTIG) {
            const int sw = swz(j);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c = 8 * kc + 4 * (i >> 1) + 2 * h + (i & 1);
                const float4 v = *reinterpret_cast<const float4*>(img + j * KS + 4 * (c ^ sw));
                x[4 * i + 0] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = img[(32 * kc + (i >> 3) * 16 + 8 * h + (i & 7)) * L + j];
        }
    }
};

// One LDS-DMA wave-instruction: lane l's 16 bytes at g go to LDS lds_wave_base + 16 l.  Inline asm,
// not the builtin: hipcc makes every ds_read wait vmcnt(0) behind a visible LDS-DMA (the ring's
// later steps would drain at each read); the waits are ours (wait_vm), M0 saved around the
// statement (the compiler does not preserve it for us).
__device__ __forceinline__ void dma16(const float* g, float* lds_wave_base) {
    const uint32_t dst = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds_wave_base);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(dst) : "memory");
}
// LDS barrier without the vector-memory drain of __syncthreads (the DMAs of later steps stay in flight)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }

// tools/dbg/lt_trace.hip: per-block phase clocks (s_memtime) of k_gemm_lt, wave 0 lane 0
#ifdef SIR_LT_TRACE
__device__ uint64_t* g_lt_trace;
#define SIR_LT_TRACE_AT(i, v) do { if (threadIdx.x == 0) g_lt_trace[blockIdx.x * 24 + (i)] = (v); } while (0)
#else
#define SIR_LT_TRACE_AT(i, v) do { } while (0)
#endif
template <bool C0, bool C1, int W0, int W1, int WK, int NS, int EPI>
__global__ void __launch_bounds__(64 * W0 * W1 * WK)
k_gemm_lt(const float* __restrict__ X0, int64_t ld0, const float* __restrict__ X1, int64_t ld1, int64_t n0lines,
          int64_t n1lines, int64_t klen_all, int nt0, int nt1, int64_t rps, const float* __restrict__ bias,
          float* __restrict__ C, int64_t ldc, float* __restrict__ csum_part, Drop drop,
          const float* __restrict__ X0b = nullptr, int64_t ld0b = 0, int64_t split0 = INT64_MAX,
          int64_t bias_cols = INT64_MAX) {
    using G = Lt<C0, C1, W0, W1, WK, NS>;
    __shared__ __attribute__((aligned(16))) float lds[G::LDS];
    const int t = threadIdx.x, l = t & 63, j = l & 31, h = l >> 5, w = t >> 6;
    const int w0 = w % W0, w1 = (w / W0) % W1, wk = w / (W0 * W1);
    const int tiles = nt0 * nt1;
    // XCD-aware: consecutive ids on one XCD, so an XCD's blocks share their op1 rows (NT: A row
    // tiles, each read by the XCD that owns it; TN: row splits) and only the small op0 is read by
    // all eight L2s
    const int bid = xcd_remap((int)blockIdx.x, (int)gridDim.x);
    const int64_t p = bid / tiles;                              // TN: the row split
    const int t0 = (bid % tiles) % nt0, t1 = (bid % tiles) / nt0;
    const int64_t a0 = (int64_t)t0 * G::L0, a1 = (int64_t)t1 * G::L1;    // first line of each operand
    const int lines0 = (int)(n0lines - a0 < G::L0 ? n0lines - a0 : G::L0);
    const int lines1 = (int)(n1lines - a1 < G::L1 ? n1lines - a1 : G::L1);
    const int64_t v0 = p * rps;
    const int klen = (int)(klen_all - v0 < rps ? klen_all - v0 : rps);
    // NT (EPI 0): op0 is the weight, possibly in two parts (X0 rows < split0, X0b the rest)
    const LtOp<C0, G::L0, G::KS, G::NT, EPI == 0> o0(C0 ? X0 + a0 * ld0 + v0 : X0 + v0 * ld0 + a0, ld0, lines0, klen, t,
                                              X0b == nullptr ? nullptr : (C0 ? X0b + v0 : X0b + a0), ld0b, split0,
                                              C0 ? a0 : v0);
    const LtOp<C1, G::L1, G::KS, G::NT> o1(C1 ? X1 + a1 * ld1 + v0 : X1 + v0 * ld1 + a1, ld1, lines1, klen, t);
    const int nsteps = klen > 0 ? (klen + G::KS - 1) / G::KS : 0;
    constexpr bool CS = EPI == 1;
    const bool do_cs = CS && csum_part != nullptr && t1 == 0 && w1 == 0;

    // step s's DMAs into stage buffer s % NS (steps past the last read zeros into a free buffer, so
    // every step issues the same count and the waits stay compile-time)
    auto issue = [&](int s) {
        float* img = lds + (s % NS) * G::BUF;
#pragma unroll
        for (int i = 0; i < G::N0; ++i) dma16(o0.at(i, s), img + (G::NT * i + 64 * w) * 4);
#pragma unroll
        for (int i = 0; i < G::N1; ++i) dma16(o1.at(i, s), img + G::F0 + (G::NT * i + 64 * w) * 4);
    };
    // the epilogue's bias and dropout seed, loaded ahead of the loop (their latency off the tail)
    float4 bb[4];
    if constexpr (EPI == 0) {
        drop = drop_resolve(drop);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int64_t n = a0 + 32 * w0 + 8 * g + 4 * h;
            // past bias_cols: + 0 (the zeros of a padded bias); no bias: - 0 (x + -0 = x)
            bb[g] = (bias != nullptr && n < n0lines && n < bias_cols) ? *reinterpret_cast<const float4*>(bias + n)
                    : (bias != nullptr ? make_float4(0.f, 0.f, 0.f, 0.f) : make_float4(-0.f, -0.f, -0.f, -0.f));
        }
    }
    SplitTile tile;
    SIR_LT_TRACE_AT(0, __builtin_amdgcn_s_memrealtime());
    SIR_LT_TRACE_AT(1, __builtin_amdgcn_s_memtime());
    if (nsteps > 0) {
#pragma unroll
        for (int q = 0; q < NS - 1; ++q) issue(q);
    }
    SIR_LT_TRACE_AT(2, __builtin_amdgcn_s_memtime());
    for (int s = 0; s < nsteps; ++s) {
        wait_vm<(NS - 2) * G::D>();                             // this thread's DMAs of step s landed
        lds_barrier();                                          // everyone's; step s - 1's reads done
        SIR_LT_TRACE_AT(4 + 2 * (s & 7), __builtin_amdgcn_s_memtime());
        issue(s + NS - 1);                                      // into the buffer step s - 1 used
        if (s == 1) SIR_LT_TRACE_AT(22, __builtin_amdgcn_s_memtime());
        const float* img = lds + (s % NS) * G::BUF;
        if ((s * WK + wk) * 32 < klen) {
            float x0[16], x1[16];
            LtOp<C0, G::L0, G::KS, G::NT, EPI == 0>::read(img, w0 * 32 + j, wk, h, x0);
            LtOp<C1, G::L1, G::KS, G::NT>::read(img + G::F0, w1 * 32 + j, wk, h, x1);
#ifdef SIR_LT_TRACE
            if (s == 1) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("" :: "v"(x0[0]), "v"(x1[0]), "v"(x0[15]), "v"(x1[15]));
                SIR_LT_TRACE_AT(23, __builtin_amdgcn_s_memtime());
            }
#endif
            if (do_cs) tile.step<true>(x0, x1, h);
            else tile.step<false>(x0, x1, h);
        }
        SIR_LT_TRACE_AT(5 + 2 * (s & 7), __builtin_amdgcn_s_memtime());
    }
    SIR_LT_TRACE_AT(3, __builtin_amdgcn_s_memtime());
    float pv[16];
    tile.result(pv, h);
    wait_vm<0>();                                               // the trailing DMAs too
    __syncthreads();                                            // the images are free: partials go there
    float* red = lds;
    float* cred = lds + G::RED;                                 // [WK][32 W0][2] column-sum halves
    const int tile_id = w0 + W0 * w1;
    if (wk > 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) red[(((wk - 1) * W0 * W1 + tile_id) * 16 + i) * 64 + l] = pv[i];
    }
    if (do_cs) cred[(wk * G::L0 + w0 * 32 + j) * 2 + h] = tile.cs;
    __syncthreads();
    if (wk == 0) {
#pragma unroll
        for (int q = 1; q < WK; ++q) {
#pragma unroll
            for (int i = 0; i < 16; ++i) pv[i] += red[(((q - 1) * W0 * W1 + tile_id) * 16 + i) * 64 + l];
        }
        // acc element i of lane (j, h): op0 line 32 w0 + (i & 3) + 8 (i >> 2) + 4 h, op1 line 32 w1 + j
        const int64_t r1 = a1 + 32 * w1 + j;
        if constexpr (EPI == 0) {
            if (r1 < n1lines) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int64_t n = a0 + 32 * w0 + 8 * g + 4 * h;
                    if (n < n0lines) {
                        float4 o = make_float4(pv[4 * g] + bb[g].x, pv[4 * g + 1] + bb[g].y, pv[4 * g + 2] + bb[g].z,
                                               pv[4 * g + 3] + bb[g].w);
                        if (drop.on()) drop4(drop, r1, (int)n, o);
                        *reinterpret_cast<float4*>(C + r1 * ldc + n) = o;
                    }
                }
            }
        } else {
            float* out = C + p * n0lines * n1lines;
            if (r1 < n1lines) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int64_t m = a0 + 32 * w0 + (i & 3) + 8 * (i >> 2) + 4 * h;
                    if (m < n0lines) out[m * n1lines + r1] = pv[i];
                }
            }
        }
    }
    SIR_LT_TRACE_AT(20, __builtin_amdgcn_s_memtime());
    SIR_LT_TRACE_AT(21, __builtin_amdgcn_s_memrealtime());
    if (do_cs && t < G::L0 && a0 + t < n0lines) {
        float sum = 0.f;
#pragma unroll
        for (int q = 0; q < WK; ++q) sum += cred[(q * G::L0 + t) * 2] + cred[(q * G::L0 + t) * 2 + 1];
        csum_part[p * n0lines + a0 + t] = sum;
    }
}

}  // namespace

#ifndef SIR_SMALL_ROWS
#define SIR_SMALL_ROWS 16384    // fewest node rows for the block-tiled GEMMs; below: k_gemm_nt_s / k_gemm_tn_s
#endif
// env SIR_GEMM_SMALL_ROWS overrides the threshold per call (A/B and the route tests)
static int64_t gemm_small_rows() {
    const char* e = getenv("SIR_GEMM_SMALL_ROWS");
    return (e != nullptr && e[0] != 0) ? atoll(e) : (int64_t)SIR_SMALL_ROWS;
}

#ifndef SIR_TN_S_ROWS
#define SIR_TN_S_ROWS 512       // k_gemm_tn_s: node rows per split (<= 16 splits)
#endif
// LDS-tiled small GEMMs (k_gemm_lt) and their wave arrangement (W0 x W1 tiles of 32 x 32, WK
// k-ways).  NT: 1 = 2x2x1, 2 = 1x2x2, 3 = 2x1x2 (64 weight lines x 32 rows), 4 = 1x1x4, 5 = 1x4x1,
// 8 waves: 6 = 2x1x4, 7 = 1x2x4, 8 = 2x2x2; default by shape (nt_lt_auto); TN: 1 = 2x2x1, 2 = 1x2x2 (default),
// 3 = 1x1x4, 8 waves: 4 = 1x2x4, 5 = 2x2x2; 0 = the 4-wave k_gemm_nt_sw /
// k_gemm_tn_s.  env SIR_LT_NT / SIR_LT_TN override per call (A/B runs, the arrangement tests);
// measured in profiles/r05_small_gemm.txt.
#ifndef SIR_LT_NT
#define SIR_LT_NT -1            // -1: by shape (nt_lt_auto)
#endif
#ifndef SIR_LT_TN
#define SIR_LT_TN 2
#endif
static int lt_env(const char* name, int dflt) {
    const char* e = getenv(name);
    return (e != nullptr && e[0] != 0) ? atoi(e) : dflt;
}
#ifndef SIR_LT_BLOCKS
#define SIR_LT_BLOCKS 512       // k_gemm_lt TN: row splits until about this many blocks
#endif
static bool aligned16(const void* p, int64_t ld) { return ((uintptr_t)p & 15u) == 0 && ld % 4 == 0; }
// TN row splits of k_gemm_lt: each split a multiple of KS rows, at most 32 splits
static int gemm_tn_splits_lt(int64_t R, int64_t tiles, int KS, int64_t* rps) {
    int64_t P = (SIR_LT_BLOCKS + tiles - 1) / tiles;
    const int64_t pmax = (R + KS - 1) / KS;
    if (P > pmax) P = pmax;
    if (P > 32) P = 32;
    if (P < 1) P = 1;
    int64_t r = (R + P - 1) / P;
    r = (r + KS - 1) / KS * KS;
    *rps = r > 0 ? r : KS;
    P = (R + *rps - 1) / *rps;
    return (int)(P < 1 ? 1 : P);
}

static int gemm_tn_splits_s(int64_t R, int64_t, int64_t) {
    int64_t P = (R + SIR_TN_S_ROWS - 1) / SIR_TN_S_ROWS;
    if (P > 16) P = 16;
    if (P < 1) P = 1;
    return (int)P;
}

static hipError_t run_gemm_nt_s(const float* A, int64_t lda, int64_t M, int K, const void* packed, int N,
                                const float* bias, float* C, int64_t ldc, hipStream_t st, const Drop& drop) {
    const int np = (int)gemm_pack_npad(N), kc = (K + KC - 1) / KC;
    const u4v* wp = static_cast<const u4v*>(packed);
    const float* inv = reinterpret_cast<const float*>(static_cast<const char*>(packed) + (int64_t)kc * 4 * np * 32);
    const int nfg = (N + 32 * S_FT - 1) / (32 * S_FT);
    const int64_t waves = (M + 31) / 32 * nfg;
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    if (K % KC == 0)
        hipLaunchKernelGGL(k_gemm_nt_s<true>, dim3(blocks), dim3(256), 0, st, A, lda, M, K, wp, np, kc, inv, bias, N, C,
                           ldc, nfg, waves, drop);
    else
        hipLaunchKernelGGL(k_gemm_nt_s<false>, dim3(blocks), dim3(256), 0, st, A, lda, M, K, wp, np, kc, inv, bias, N, C,
                           ldc, nfg, waves, drop);
    return hipGetLastError();
}

#ifndef SIR_LT_NS
#define SIR_LT_NS 3             // k_gemm_lt stage buffers (NS - 1 steps in flight)
#endif
struct NtW {            // the weight of an NT product: rows < split from W, the rest from W2
    const float* W;
    int64_t ldw;
    const float* W2;
    int64_t ldw2, split, bias_cols;
};
template <bool TRANS, int W0, int W1, int WK>
static void launch_nt_lt(const float* A, int64_t lda, int64_t M, int K, const NtW& w, int N, const float* bias,
                         float* C, int64_t ldc, hipStream_t st, const Drop& drop) {
    using G = Lt<!TRANS, true, W0, W1, WK, SIR_LT_NS>;
    const int nt0 = (N + G::L0 - 1) / G::L0;
    const int64_t nt1 = (M + G::L1 - 1) / G::L1;
    hipLaunchKernelGGL((k_gemm_lt<!TRANS, true, W0, W1, WK, SIR_LT_NS, 0>), dim3((unsigned)(nt0 * nt1)), dim3(G::NT), 0, st,
                       w.W, w.ldw, A, lda, (int64_t)N, M, (int64_t)K, nt0, (int)nt1, (int64_t)K, bias, C, ldc, nullptr,
                       drop, w.W2, w.ldw2, w.split, w.bias_cols);
}

// The arrangement by shape: every block is latency-bound (one block's steps set the time, not the
// CU's bandwidth: half the rows take as long), so the most k-ways whose grid still fits one round
// on the CUs wins — 8 waves as 32 features x 64 rows x 4 k-ways (7), else 64 x 64 x 2 k-ways (8),
// else the 4-wave 64 x 32 x 2 (3) at 2+ blocks per CU (profiles/r05_small_gemm.txt: config 5's
// QK 11.9 -> 10.3 us, R / dY W_R 8.5 / 9.4 -> 7.8 / 8.0, dX 15.1 -> 11.2).
static int nt_lt_auto(int64_t M, int N) {
    const int64_t ncu = device_cu_count();
    if ((int64_t)((N + 31) / 32) * ((M + 63) / 64) <= ncu) return 7;
    if ((int64_t)((N + 63) / 64) * ((M + 63) / 64) <= ncu) return 8;
    return 3;
}

hipError_t run_gemm_nt_direct(const float* A, int64_t lda, int64_t M, int K, const float* W, int64_t ldw, int trans,
                              int N, const float* bias, float* C, int64_t ldc, hipStream_t st, const Drop& drop,
                              const float* W2, int64_t ldw2, int64_t split, int64_t bias_cols) {
    if (M == 0 || N == 0) return hipSuccess;
    int lt = lt_env("SIR_LT_NT", SIR_LT_NT);
    if (lt < 0) lt = nt_lt_auto(M, N);
    const NtW w{W, ldw, W2, ldw2, W2 != nullptr ? split : INT64_MAX, bias_cols};
    // k_gemm_lt: 16-byte loads of both operands (and of W2), every byte offset of a tile's resource in 31 bits
    if (lt > 0 && K % 4 == 0 && N % 4 == 0 && aligned16(A, lda) && aligned16(W, ldw) && ((uintptr_t)bias & 15u) == 0
        && (W2 == nullptr || aligned16(W2, ldw2)) && 128 * lda < ((int64_t)1 << 29)
        && (trans ? (int64_t)K * ldw : 128 * ldw) < ((int64_t)1 << 29)
        && (M + 31) / 32 * ((N + 31) / 32) < ((int64_t)1 << 31)) {
        switch (lt * 2 + (trans ? 1 : 0)) {
        case 2: launch_nt_lt<false, 2, 2, 1>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 3: launch_nt_lt<true, 2, 2, 1>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 4: launch_nt_lt<false, 1, 2, 2>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 5: launch_nt_lt<true, 1, 2, 2>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 6: launch_nt_lt<false, 2, 1, 2>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 7: launch_nt_lt<true, 2, 1, 2>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 8: launch_nt_lt<false, 1, 1, 4>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 9: launch_nt_lt<true, 1, 1, 4>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 10: launch_nt_lt<false, 1, 4, 1>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 11: launch_nt_lt<true, 1, 4, 1>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 12: launch_nt_lt<false, 2, 1, 4>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;   // 8 waves
        case 13: launch_nt_lt<true, 2, 1, 4>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 14: launch_nt_lt<false, 1, 2, 4>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 15: launch_nt_lt<true, 1, 2, 4>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 16: launch_nt_lt<false, 2, 2, 2>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        case 17: launch_nt_lt<true, 2, 2, 2>(A, lda, M, K, w, N, bias, C, ldc, st, drop); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    // the two-part weight and the partial bias are the LDS-tiled kernel's only
    if (W2 != nullptr || bias_cols < N) return hipErrorInvalidValue;
    const int nft = (N + 31) / 32;
    const int64_t blocks = (M + 31) / 32 * nft;
    if (trans)
        hipLaunchKernelGGL(k_gemm_nt_sw<true>, dim3((unsigned)blocks), dim3(256), 0, st, A, lda, M, K, W, ldw, N, bias, C,
                           ldc, nft, drop);
    else
        hipLaunchKernelGGL(k_gemm_nt_sw<false>, dim3((unsigned)blocks), dim3(256), 0, st, A, lda, M, K, W, ldw, N, bias,
                           C, ldc, nft, drop);
    return hipGetLastError();
}

int64_t gemm_pack_npad(int64_t N) { return (N + 255) / 256 * 256; }
// the packed weight: the k_gemm_nt / k_gemm_nt_p fragment image, then the per-feature inverse scales
int64_t gemm_pack_bytes(int64_t N, int64_t K) {
    const int64_t np = gemm_pack_npad(N), kc = (K + KC - 1) / KC;
    return (kc * 4 * np * 32 + np * 4 + 15) / 16 * 16;
}

hipError_t run_gemm_pack(const float* W, int64_t ldw, int N, int K, int trans, void* packed, hipStream_t st) {
    const int np = (int)gemm_pack_npad(N), kc = (K + KC - 1) / KC;
    _Float16* out = static_cast<_Float16*>(packed);
    float* inv = reinterpret_cast<float*>(static_cast<char*>(packed) + (int64_t)kc * 4 * np * 32);
    hipLaunchKernelGGL(k_pack_weight, dim3(np), dim3(64), 0, st, W, ldw, N, K, trans, np, kc, out, inv);
    return hipGetLastError();
}

hipError_t run_gemm_nt(const float* A, int64_t lda, int64_t M, int K, const void* packed, int N,
                       const float* bias, float* C, int64_t ldc, hipStream_t st, const Drop& drop, const float* gate,
                       int gate_relu, float gate_slope, const uint64_t* gate_mask) {
    if (M == 0 || N == 0) return hipSuccess;
    if (gate_mask != nullptr && N != 256) return hipErrorInvalidValue;
    if (gate != nullptr || gate_mask != nullptr) {   // fused in k_gemm_nt_p's epilogue; other routes: afterwards
        const int np = (int)gemm_pack_npad(N), kc = (K + KC - 1) / KC;
        if (M >= gemm_small_rows() && N > 128 && np <= NT_P_NMAX && K % KC == 0 && (kc == 4 || kc == 8 || kc == 16)) {
            const u4v* wp = static_cast<const u4v*>(packed);
            const float* inv = reinterpret_cast<const float*>(static_cast<const char*>(packed) + (int64_t)kc * 4 * np * 32);
            constexpr int BD = 256, BF = 256;
            const int nft = (N + BF - 1) / BF;
            const int64_t ntiles = (M + BD - 1) / BD * nft;
            const int ncu = device_cu_count();
            if (ntiles < (int64_t)1 << 30) {
                const int tpb = (int)((ntiles + ncu - 1) / ncu);
                const int nblk = (int)((ntiles + tpb - 1) / tpb);
                if (gate_mask != nullptr) {
                    auto kern = kc == 4 ? k_gemm_nt_p<4, 2> : (kc == 8 ? k_gemm_nt_p<8, 2> : k_gemm_nt_p<16, 2>);
                    hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(512), 0, st, A, lda, M, wp, np, inv, bias, N, C,
                                       ldc, nft, (int)ntiles, tpb, drop, reinterpret_cast<const float*>(gate_mask),
                                       gate_relu, gate_slope);
                } else {
                    auto kern = kc == 4 ? k_gemm_nt_p<4, 1> : (kc == 8 ? k_gemm_nt_p<8, 1> : k_gemm_nt_p<16, 1>);
                    hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(512), 0, st, A, lda, M, wp, np, inv, bias, N, C,
                                       ldc, nft, (int)ntiles, tpb, drop, gate, gate_relu, gate_slope);
                }
                return hipGetLastError();
            }
        }
        hipError_t err = run_gemm_nt(A, lda, M, K, packed, N, bias, C, ldc, st, drop, nullptr, 0, 0.f, nullptr);
        if (err != hipSuccess) return err;
        const int64_t cnt = M * N;
        if (gate_mask != nullptr)
            hipLaunchKernelGGL(k_gate_dact_bits, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, C, ldc, gate_mask, M,
                               gate_relu, gate_slope);
        else
            hipLaunchKernelGGL(k_gate_dact, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, C, ldc, gate, M, N,
                               gate_relu, gate_slope);
        return hipGetLastError();
    }
    const int np = (int)gemm_pack_npad(N), kc = (K + KC - 1) / KC;
    const u4v* wp = static_cast<const u4v*>(packed);
    const float* inv = reinterpret_cast<const float*>(static_cast<const char*>(packed) + (int64_t)kc * 4 * np * 32);
    const bool kfull = K % KC == 0;
    if (M < gemm_small_rows()) return run_gemm_nt_s(A, lda, M, K, packed, N, bias, C, ldc, st, drop);
    if (SIR_NT_PERSIST && N > 128 && np <= NT_P_NMAX && kfull && (kc == 4 || kc == 8 || kc == 16)) {
        constexpr int BD = 256, BF = 256;
        const int nft = (N + BF - 1) / BF;
        const int64_t ntiles = (M + BD - 1) / BD * nft;
        const int ncu = device_cu_count();
        if (ntiles < (int64_t)1 << 30) {
            const int tpb = (int)((ntiles + ncu - 1) / ncu);
            const int nblk = (int)((ntiles + tpb - 1) / tpb);
            auto kern = kc == 4 ? k_gemm_nt_p<4, 0> : (kc == 8 ? k_gemm_nt_p<8, 0> : k_gemm_nt_p<16, 0>);
            hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(512), 0, st, A, lda, M, wp, np, inv, bias, N, C, ldc,
                               nft, (int)ntiles, tpb, drop, nullptr, 0, 0.f);
            return hipGetLastError();
        }
    }
    if (N > 128) {
        constexpr int BD = 256, BF = 256;
        const int nft = (N + BF - 1) / BF;
        const int64_t nblk = (M + BD - 1) / BD * nft;
        if (kfull)
            hipLaunchKernelGGL((k_gemm_nt<2, 4, 4, 2, true>), dim3((unsigned)nblk), dim3(512), 0, st,
                               A, lda, M, K, wp, np, inv, bias, N, C, ldc, nft, drop);
        else
            hipLaunchKernelGGL((k_gemm_nt<2, 4, 4, 2, false>), dim3((unsigned)nblk), dim3(512), 0, st,
                               A, lda, M, K, wp, np, inv, bias, N, C, ldc, nft, drop);
    } else {
        constexpr int BD = 256, BF = 128;
        const int nft = (N + BF - 1) / BF;
        const int64_t nblk = (M + BD - 1) / BD * nft;
        if (kfull)
            hipLaunchKernelGGL((k_gemm_nt<4, 2, 2, 2, true>), dim3((unsigned)nblk), dim3(512), 0, st,
                               A, lda, M, K, wp, np, inv, bias, N, C, ldc, nft, drop);
        else
            hipLaunchKernelGGL((k_gemm_nt<4, 2, 2, 2, false>), dim3((unsigned)nblk), dim3(512), 0, st,
                               A, lda, M, K, wp, np, inv, bias, N, C, ldc, nft, drop);
    }
    return hipGetLastError();
}

hipError_t run_gemm_reduce(const float* part, int P, int64_t count, int Nc, float* C, int64_t ldc, hipStream_t st) {
    if (count > 0)
        hipLaunchKernelGGL(k_gemm_reduce, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, part, P, count, Nc, C,
                           ldc);
    return hipGetLastError();
}

#ifndef SIR_TN_MINROWS
#define SIR_TN_MINROWS 1024     // fewest node rows per split of the TN GEMMs (1024: cfg2 TN16 -30 %, profiles/r02_ab_tn_reduce.txt)
#endif
int gemm_tn_splits(int64_t R, int64_t Mc, int64_t Nc) {
    const int64_t tiles = ((Mc + 255) / 256) * ((Nc + 255) / 256);
    int64_t P = (256 + tiles - 1) / tiles;
    const int64_t pmax = (R + SIR_TN_MINROWS - 1) / SIR_TN_MINROWS;      // >= SIR_TN_MINROWS rows per split
    if (P > pmax) P = pmax;
    if (P < 1) P = 1;
    return (int)P;
}

int64_t gemm_tn_workspace(int64_t R, int64_t Mc, int64_t Nc) {
    int64_t P = gemm_tn_splits(R, Mc, Nc);                 // the block-tiled kernels (fp32 and 16-bit)
    if (R < gemm_small_rows()) {
        const int64_t ps = gemm_tn_splits_s(R, Mc, Nc);    // k_gemm_tn_s
        if (ps > P) P = ps;
        if (P < 32) P = 32;                                // k_gemm_lt: at most 32 splits
    }
    return P * (Mc * Nc + Mc) * 4;                         // partial products + column sums
}

// k_gemm_lt TN arrangements (SIR_LT_TN): 1 = 2x2x1, 2 = 1x2x2, 3 = 1x1x4, 4 = 1x2x4 and 5 = 2x2x2 (8 waves)
static int lt_tn_w0(int lt) { return (lt == 1 || lt == 5) ? 2 : 1; }
static int lt_tn_w1(int lt) { return lt == 3 ? 1 : 2; }
static int lt_tn_ks(int lt) { return 32 * (lt == 1 ? 1 : (lt == 2 || lt == 5) ? 2 : 4); }
static int64_t lt_tn_tiles(int lt, int Mc, int Nc) {
    const int a = 32 * lt_tn_w0(lt), b = 32 * lt_tn_w1(lt);
    return (int64_t)((Mc + a - 1) / a) * ((Nc + b - 1) / b);
}
template <int W0, int W1, int WK>
static void launch_tn_lt(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t R, int Mc, int Nc,
                         float* part, bool colsum, hipStream_t st) {
    using G = Lt<false, false, W0, W1, WK, SIR_LT_NS>;
    const int nt0 = (Mc + G::L0 - 1) / G::L0, nt1 = (Nc + G::L1 - 1) / G::L1;
    const int64_t tiles = (int64_t)nt0 * nt1;
    int64_t rl = 0;
    const int Pl = gemm_tn_splits_lt(R, tiles, G::KS, &rl);
    float* cp = colsum ? part + (int64_t)Pl * Mc * Nc : nullptr;
    hipLaunchKernelGGL((k_gemm_lt<false, false, W0, W1, WK, SIR_LT_NS, 1>), dim3((unsigned)(Pl * tiles)), dim3(G::NT), 0,
                       st, A, lda, B, ldb, (int64_t)Mc, (int64_t)Nc, R, nt0, nt1, rl, nullptr, part, (int64_t)0, cp,
                       Drop{});
}

hipError_t run_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t R, int Mc, int Nc,
                       float* C, int64_t ldc, float* colsum, void* workspace, hipStream_t st) {
    if (Mc == 0 || Nc == 0) return hipSuccess;
    const bool small = R < gemm_small_rows();
    const int P = small ? gemm_tn_splits_s(R, Mc, Nc) : gemm_tn_splits(R, Mc, Nc);
    const int64_t rps = (R + P - 1) / P;
    const int nmt = (Mc + 255) / 256, nnt = (Nc + 255) / 256;
    float* part = static_cast<float*>(workspace);
    float* cpart = colsum != nullptr ? part + (int64_t)P * Mc * Nc : nullptr;
    const int lt = lt_env("SIR_LT_TN", SIR_LT_TN);
    if (small && lt > 0 && lt <= 5 && aligned16(A, lda) && aligned16(B, ldb) && (Mc + 31) / 32 * ((Nc + 31) / 32) < (1 << 24)) {
        switch (lt) {
        case 1: launch_tn_lt<2, 2, 1>(A, lda, B, ldb, R, Mc, Nc, part, colsum != nullptr, st); break;
        case 2: launch_tn_lt<1, 2, 2>(A, lda, B, ldb, R, Mc, Nc, part, colsum != nullptr, st); break;
        case 3: launch_tn_lt<1, 1, 4>(A, lda, B, ldb, R, Mc, Nc, part, colsum != nullptr, st); break;
        case 4: launch_tn_lt<1, 2, 4>(A, lda, B, ldb, R, Mc, Nc, part, colsum != nullptr, st); break;   // 8 waves
        default: launch_tn_lt<2, 2, 2>(A, lda, B, ldb, R, Mc, Nc, part, colsum != nullptr, st); break;  // 8 waves
        }
        const int64_t tiles = lt_tn_tiles(lt, Mc, Nc);
        int64_t rl = 0;
        const int Pl = gemm_tn_splits_lt(R, tiles, lt_tn_ks(lt), &rl);
        float* cp = colsum != nullptr ? part + (int64_t)Pl * Mc * Nc : nullptr;
        const int64_t count = (int64_t)Mc * Nc;
        const int64_t nbm = (count + 255) / 256, nbc = colsum != nullptr ? (Mc + 255) / 256 : 0;
        hipLaunchKernelGGL(k_gemm_reduce2, dim3((unsigned)(nbm + nbc)), dim3(256), 0, st, part, Pl, count, Nc, C, ldc,
                           cp, Mc, colsum, nbm);
        return hipGetLastError();
    }
    if (small) {
        const int smt = (Mc + 31) / 32, snt = (Nc + 31) / 32;
        hipLaunchKernelGGL(k_gemm_tn_s, dim3((unsigned)((int64_t)P * smt * snt)), dim3(256), 0, st, A, lda, B, ldb, R,
                           Mc, Nc, part, cpart, smt, snt, rps);
    } else
#if SIR_TN_CFG == 2
    // 8 waves (2 per SIMD, 256 registers), 128x64 per wave, a thread loads a whole column chunk
    hipLaunchKernelGGL((k_gemm_tn<2, 4, 4, 2>), dim3((unsigned)(P * nmt * nnt)), dim3(512), 0, st,
                       A, lda, B, ldb, R, Mc, Nc, part, cpart, nmt, nnt, rps);
#else
    hipLaunchKernelGGL((k_gemm_tn<4, 4, 2, 2>), dim3((unsigned)(P * nmt * nnt)), dim3(1024), 0, st,
                       A, lda, B, ldb, R, Mc, Nc, part, cpart, nmt, nnt, rps);
#endif
    // C = sum_p part[p] and colsum = sum_p cpart[p], in split order, one launch
    const int64_t count = (int64_t)Mc * Nc;
    const int64_t nbm = (count + 255) / 256, nbc = colsum != nullptr ? (Mc + 255) / 256 : 0;
    hipLaunchKernelGGL(k_gemm_reduce2, dim3((unsigned)(nbm + nbc)), dim3(256), 0, st, part, P, count, Nc, C, ldc, cpart,
                       Mc, colsum, nbm);
    return hipGetLastError();
}

}  // namespace sir
