// sirconv_gemm_w.hip — weight-resident NT GEMM for the layer's node projections (conv.py:60-61,65 and
// the input gradients of their autograd): C[M, N] = A[M, K] B[N, K]^T + bias, fp32 in and out, on
// gfx950 fp16 MFMA with the two-term operand split of sirconv_gemm.hip (x = (hi + lo) / s per
// data row, hi*hi' + hi*lo' + lo*hi', fp32 accumulation; same running row scale with hysteresis).
//
// Why a second NT kernel.  k_gemm_nt_p stages both operands in LDS per 32-k chunk: every step the
// two waves of a SIMD split A, write the LDS image, meet at a barrier and multiply — in lock-step,
// so the MFMA pipe idles while both split (its Y GEMM without loads or stores still took 2x its
// MFMA time).  Here the weights never move during the main loop:
//  * a block owns a feature SLICE of F features (F*K*4 B of packed hi/lo fp16 = 128 KiB, the whole
//    contraction) and keeps it in LDS for the life of the block; 8 waves, 2 per SIMD;
//  * every wave walks its own 32-row data tiles: it loads its rows straight into registers in MFMA
//    fragment shape (no LDS image of A), splits them itself and multiplies them against the
//    resident slice (ds_read_b128 of lane-linear fragment images: conflict-free);
//  * there is NO barrier after the slice is loaded: the two waves of a SIMD drift apart on their
//    own, so one's split / loads / stores run under the other's MFMAs.
// The cost is that each data row is read (and split) once per slice: N / F times (2 for Y and G,
// 4 for QK and dX).  The slice-blocks of one row group sit on one XCD (block id = 8q + x: equal x
// <=> same XCD under round-robin dispatch — for speed only) and walk the same rows in the same order,
// so the re-reads are L2 hits and HBM sees A once.
//
// Memory access shape.  MFMA operands are fragment-shaped (lane = row), and a 16-B load per lane in
// fragment shape puts 16 different rows in every 16-lane group: 64 separate requests per wave
// instruction (an earlier version of this kernel spent most of its time there).  So every global
// access here is coalesced — a wave instruction reads / writes 8 whole 128-B row pieces — and
// each wave transposes through a private 4-KiB LDS slot: A chunks (32 rows x 32 k) on the way in,
// the output tile (32 rows x 32 features at a time) on the way out.  The slot is the wave's own,
// so no barrier is needed (LDS operations of one wave complete in order).
#include "sirconv_internal.h"
#include "sirconv_gemm_util.h"
#include "sirconv_dropout.h"

#include <cstdlib>

namespace sir {
namespace {
using namespace gemm;

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

#ifndef SIR_NTW_PD
#define SIR_NTW_PD 2            // 32-k chunks of A in flight ahead of the one being multiplied (1..3)
#endif

#ifndef SIR_NTW_ABL
#define SIR_NTW_ABL 0           // timing-only ablations: 1 no A loads, 2 no C stores, 4 no MFMAs, 8 no split
#endif

constexpr int WKC = 32;         // contraction elements per chunk
constexpr int WNS = 4;          // register sets for chunks (PD + 1 <= 4)
static_assert(SIR_NTW_PD >= 1 && SIR_NTW_PD < WNS, "prefetch depth");

// ---- split helpers (the numerics of sirconv_gemm.hip; see its header) ----
__device__ inline int bexp(float m) { return (int)((__float_as_uint(m) >> 23) & 255u) - 126; }
constexpr int SE_INIT = 127;
#ifndef SIR_HR
#define SIR_HR 8
#endif
__device__ inline int next_se(int se_old, int e_c) {
    if (e_c + se_old <= 15) return se_old;
    const int s = 15 - SIR_HR - e_c;
    return s > 126 ? 126 : s;
}
__device__ inline int scale_exp(int e) { int s = 15 - e; return s > 126 ? 126 : s; }
__device__ inline float pow2(int e) { e = e < -126 ? -126 : (e > 127 ? 127 : e); return __uint_as_float((uint32_t)(e + 127) << 23); }
// m = max(m, |v.x|, |v.y|, |v.z|, |v.w|) in two v_max3_f32 with |.| source modifiers (fmaxf makes
// hipcc canonicalise every input first: 2 VALU per element instead of 0.5)
__device__ inline float fmax4(float m, float4 v) {
    asm("v_max3_f32 %0, %0, |%1|, |%2|\n\tv_max3_f32 %0, %0, |%3|, |%4|" : "+v"(m) : "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
    return m;
}
// hi = fp16(x s), lo = fp16(x s - hi): x s is exact (power-of-two s), so each is ONE fused
// multiply-add with an fp16 result written into a half of the fragment register
// (v_fma_mixlo/hi_f16, the second reading hi as an fp16 source): the same values as rounding
// y = x s and y - hi separately, in 2 VALU operations per element instead of 3.5 (hipcc builds hi
// twice: once packed by v_cvt_pk_f16_f32 for the MFMA operand and once as a scalar fp16 for the
// subtraction).  The closing s_nop 1 gives the 2 wait states a VALU write needs before an MFMA
// reads the register (the hazard recognizer does not look inside inline asm).
__device__ inline void split8(float4 a, float4 b, float s, h8& hi, h8& lo) {
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
__device__ inline float4 as_f4(u4v u) {
    return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
}

// ------------------------------------------------------------------------------------------
// weight packing: one 64-thread block per (padded) feature n.  Output: nsl slice images of
// K*F*2 halves, each [g = k16 step][part hi/lo][feature tile a][lane][j], then inv_scale[Npad].
__global__ void __launch_bounds__(64)
k_pack_w(const float* __restrict__ W, int64_t ldw, int N, int K, int trans, int F, _Float16* __restrict__ out,
         float* __restrict__ inv_scale) {
    const int n = blockIdx.x, l = threadIdx.x;
    float m = 0.f;
    if (n < N)
        for (int k = l; k < K; k += 64) m = fmaxf(m, fabsf(trans ? W[(int64_t)k * ldw + n] : W[(int64_t)n * ldw + k]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    const int se = scale_exp(bexp(m));
    const float s = pow2(se);
    const int FT = F / 32, sl = n / F, a = (n % F) / 32, rr = n % 32;
    _Float16* img = out + (int64_t)sl * K * F * 2;
    for (int k = l; k < K; k += 64) {
        const float x = (n < N) ? (trans ? W[(int64_t)k * ldw + n] : W[(int64_t)n * ldw + k]) : 0.f;
        const float y = x * s;
        const _Float16 hh = (_Float16)y;
        const int g = k >> 4, kk = k & 15, h = kk >> 3, j = kk & 7;
        const int lane = h * 32 + rr;
        img[((int64_t)(g * 2 + 0) * FT + a) * 512 + lane * 8 + j] = hh;
        img[((int64_t)(g * 2 + 1) * FT + a) * 512 + lane * 8 + j] = (_Float16)(y - (float)hh);
    }
    if (l == 0) inv_scale[n] = (n < N) ? pow2(-se) : 0.f;
}

// ------------------------------------------------------------------------------------------
// Per-wave LDS slot (4 KiB): 32 rows x 128 B, 16-B piece p of row r at r*128 + (p ^ ((r>>1)&7))*16 —
// conflict-free for the coalesced writes (8 lanes per row) and for the fragment reads
// (ds_read_b128 lane groups hit 16 distinct 16-B bank groups).
__device__ inline int slot_off(int row, int piece) { return row * 128 + ((piece ^ ((row >> 1) & 7)) << 4); }

template <int K, int F>
__global__ void __launch_bounds__(512)
k_gemm_nt_w(const float* __restrict__ A, int64_t lda, int64_t M, const u4v* __restrict__ Wimg,
            const float* __restrict__ inv_t, const float* __restrict__ bias, int N, float* __restrict__ C,
            int64_t ldc, int nsl, int nrg, int ntiles, Drop drop) {
    constexpr int FT = F / 32, NCH = K / WKC, IMG = K * F * 4, SLOT = 4096;
    static_assert(NCH % WNS == 0, "chunk count must be a multiple of the register sets");
    static_assert(IMG + 8 * SLOT <= 160 * 1024, "slice image + wave slots fit LDS");
    __shared__ __attribute__((aligned(16))) char lds[IMG + 8 * SLOT];

    const int bid = blockIdx.x, x8 = bid & 7, q = bid >> 3;
    const int sl = q % nsl, rg = (q / nsl) * 8 + x8;
    const int f0 = sl * F;
    {
        const u4v* src = Wimg + (int64_t)sl * (IMG / 16);
        u4v* dst = reinterpret_cast<u4v*>(lds);
#pragma unroll 4
        for (int i = threadIdx.x; i < IMG / 16; i += 512) dst[i] = src[i];
    }
    __syncthreads();

    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int l = threadIdx.x & 63, r = l & 31, h = l >> 5;
    const int lr = l >> 3, lp = l & 7;       // coalesced role: row lr + 8i, 16-B piece lp
    int t = rg * 8 + w;
    if (t >= ntiles) return;                 // no barrier below this point
    const int tstr = nrg * 8;
    char* const slot = lds + IMG + w * SLOT;
    auto mk_a = [&](int tt) {                // a tile past the end loads zeros (0-record resource)
        uint32_t bytes = 0;
        if (tt < ntiles) {
            const int64_t rows = M - (int64_t)tt * 32;
            bytes = (SIR_NTW_ABL & 1) ? 0u : (uint32_t)((rows < 32 ? rows : 32) * lda * 4);
        }
        return mk_rsrc(A + (int64_t)(tt < ntiles ? tt : 0) * 32 * lda, bytes);
    };
    // rows in voffset (the range check drops rows past M), the chunk's column offset in soffset
    uint32_t voffa[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) voffa[i] = (uint32_t)(((lr + 8 * i) * lda) * 4 + lp * 16);

    float4 d[WNS][4];
    auto load = [&](int set, rsrc_t rs, int c) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            d[set][i] = as_f4(__builtin_amdgcn_raw_buffer_load_b128(rs, voffa[i], c * WKC * 4, 0));
    };

    rsrc_t ca = mk_a(t), na = mk_a(t + tstr);
#pragma unroll
    for (int p = 0; p < SIR_NTW_PD; ++p) load(p, ca, p);

    // bias: a 0-record resource without one (reads 0)
    const rsrc_t brs = mk_rsrc(bias, bias != nullptr ? (uint32_t)N * 4u : 0u);
    const char* wl = lds + l * 16;
    while (true) {
        f16v acc[FT];
#pragma unroll
        for (int a = 0; a < FT; ++a)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[a][i] = 0.f;
        int se = SE_INIT;
        uint64_t over = 0;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int set = c % WNS;
            {
                const int cp = c + SIR_NTW_PD;
                if (cp < NCH) load(cp % WNS, ca, cp);
                else load(cp % WNS, na, cp - NCH);
            }
            // transpose the chunk through the wave's slot: lane (r, h) takes row r, floats
            // 16 s + 8 h .. +8 of k16 step s (natural MFMA k order)
#pragma unroll
            for (int i = 0; i < 4; ++i) *reinterpret_cast<float4*>(slot + slot_off(lr + 8 * i, lp)) = d[set][i];
            float4 fr[2][2];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    fr[s2][u] = *reinterpret_cast<const float4*>(slot + slot_off(r, 4 * s2 + 2 * h + u));
            // row scale.  Fast path: the scale of the tile's first chunk (with 2^SIR_HR headroom) is
            // kept for the whole tile; a later chunk that would leave the fp16 range under it only
            // raises a wave-uniform flag (a ballot OR-ed on the scalar unit) — no branch, so the
            // whole tile is one scheduling region and chunk c+1's transpose / split interleave with
            // chunk c's MFMAs.  This is exactly the running scale with hysteresis as long as no
            // scale change is due; a flagged tile is recomputed with it below (rare: a row whose
            // maximum grows by more than 2^SIR_HR along K).
            float m = 0.f;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) m = fmax4(fmax4(m, fr[s2][0]), fr[s2][1]);
            {
                const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
                m = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
            }
            if (c == 0) se = next_se(SE_INIT, bexp(m));
            else over |= __builtin_amdgcn_ballot_w64(bexp(m) + se > 15);
            const float s = pow2(se);
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                h8 dh, dl;
#if SIR_NTW_ABL & 8
                dh = __builtin_bit_cast(h8, fr[s2][0]);
                dl = __builtin_bit_cast(h8, fr[s2][1]);
#else
                split8(fr[s2][0], fr[s2][1], s, dh, dl);
#endif
                const int g = 2 * c + s2;
#pragma unroll
                for (int a = 0; a < FT; ++a) {
                    const h8 wh = *reinterpret_cast<const h8*>(wl + ((g * 2 + 0) * FT + a) * 1024);
                    const h8 wo = *reinterpret_cast<const h8*>(wl + ((g * 2 + 1) * FT + a) * 1024);
#if SIR_NTW_ABL & 4
                    asm volatile("" :: "v"(wh), "v"(wo), "v"(dh), "v"(dl));
#else
                    acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, dh, acc[a], 0, 0, 0);
                    acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, dl, acc[a], 0, 0, 0);
                    acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wo, dh, acc[a], 0, 0, 0);
#endif
                }
            }
        }
        if (over != 0) {
            // exact running scale with hysteresis (sirconv_gemm.hip's algorithm): recompute the
            // tile, its rows read straight in fragment shape (the prefetched chunks of the next
            // tile stay untouched in their registers)
#pragma unroll
            for (int a = 0; a < FT; ++a)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[a][i] = 0.f;
            const uint32_t vf = (uint32_t)((r * lda + 8 * h) * 4);
#pragma unroll 1
            for (int c = 0; c < NCH; ++c) {
                float4 fr[2][2];
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                    for (int u = 0; u < 2; ++u)
                        fr[s2][u] = as_f4(__builtin_amdgcn_raw_buffer_load_b128(ca, vf + 64 * s2 + 16 * u, c * WKC * 4, 0));
                float m = 0.f;
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) m = fmax4(fmax4(m, fr[s2][0]), fr[s2][1]);
                {
                    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
                    m = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
                }
                const int se_new = next_se(c == 0 ? SE_INIT : se, bexp(m));
                if (c > 0) {
                    const float fac = pow2(se_new - se);
                    if (__builtin_amdgcn_ballot_w64(fac != 1.f) != 0) {
#pragma unroll
                        for (int a = 0; a < FT; ++a) acc[a] *= fac;
                    }
                }
                se = se_new;
                const float s = pow2(se);
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    h8 dh, dl;
                    split8(fr[s2][0], fr[s2][1], s, dh, dl);
                    const int g = 2 * c + s2;
#pragma unroll
                    for (int a = 0; a < FT; ++a) {
                        const h8 wh = *reinterpret_cast<const h8*>(wl + ((g * 2 + 0) * FT + a) * 1024);
                        const h8 wo = *reinterpret_cast<const h8*>(wl + ((g * 2 + 1) * FT + a) * 1024);
                        acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, dh, acc[a], 0, 0, 0);
                        acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, dl, acc[a], 0, 0, 0);
                        acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wo, dh, acc[a], 0, 0, 0);
                    }
                }
            }
        }
        // epilogue: C[m][n] = acc * 2^-se(m) * inv_t[n] + bias[n].  Per feature tile the row-scaled
        // fragments go through the slot (lane (r, h) holds row r, features 8 g4 + 4 h .. +4), and the
        // wave stores 8 whole 128-B row pieces per instruction.
        {
            const float is = pow2(-se);
            const int64_t rows = M - (int64_t)t * 32;
            const uint32_t ldc4 = (uint32_t)ldc * 4u;
            const uint32_t nrec = (uint32_t)(rows < 32 ? rows : 32) * ldc4;
            const rsrc_t crs = mk_rsrc(C + (int64_t)t * 32 * ldc, (SIR_NTW_ABL & 2) ? 0u : nrec);
#pragma unroll
            for (int a = 0; a < FT; ++a) {
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    float4 o;
                    o.x = acc[a][4 * g4 + 0] * is;
                    o.y = acc[a][4 * g4 + 1] * is;
                    o.z = acc[a][4 * g4 + 2] * is;
                    o.w = acc[a][4 * g4 + 3] * is;
                    *reinterpret_cast<float4*>(slot + slot_off(r, 2 * g4 + h)) = o;
                }
                const int fl = f0 + 32 * a + 4 * lp;           // this lane's 4 output features
                const float4 it = *reinterpret_cast<const float4*>(inv_t + fl);
                const float4 bb = as_f4(__builtin_amdgcn_raw_buffer_load_b128(brs, (uint32_t)fl * 4u, 0, 0));
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float4 v = *reinterpret_cast<const float4*>(slot + slot_off(lr + 8 * i, lp));
                    u4v ov;
                    float4 o = make_float4(v.x * it.x + bb.x, v.y * it.y + bb.y, v.z * it.z + bb.z, v.w * it.w + bb.w);
                    if (drop.on()) {           // feature dropout of QK (sirconv_dropout.h)
                        const uint32_t rh = drop_row_hash(drop, (int64_t)t * 32 + lr + 8 * i);
                        const int cc = drop.col0 + fl;
                        o.x = drop_keep(drop, rh, cc + 0) ? o.x * drop.scale : 0.f;
                        o.y = drop_keep(drop, rh, cc + 1) ? o.y * drop.scale : 0.f;
                        o.z = drop_keep(drop, rh, cc + 2) ? o.z * drop.scale : 0.f;
                        o.w = drop_keep(drop, rh, cc + 3) ? o.w * drop.scale : 0.f;
                    }
                    ov.x = __float_as_uint(o.x);
                    ov.y = __float_as_uint(o.y);
                    ov.z = __float_as_uint(o.z);
                    ov.w = __float_as_uint(o.w);
                    const uint32_t off = (fl < N) ? (uint32_t)(lr + 8 * i) * ldc4 + (uint32_t)(32 * a + 4 * lp) * 4u : nrec;
                    __builtin_amdgcn_raw_buffer_store_b128(ov, crs, off, f0 * 4, 0);
                    // a 16-byte store reads its data VGPRs over several cycles (sirconv_gemm.hip):
                    // pin the order and pad the window
                    __builtin_amdgcn_sched_barrier(0);
                    asm volatile("s_nop 1" ::: "memory");
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        t += tstr;
        if (t >= ntiles) break;
        ca = na;
        na = mk_a(t + tstr);
    }
}

}  // namespace

// ------------------------------------------------------------------------------------------
static int ntw_feat(int K) { return K <= 256 ? 128 : 64; }

// the shapes the kernel handles: Y, G (N <= 256: two slices) and K <= 256 only — with four slices
// (QK at N = 512, dX at K = 512) the per-slice re-reads of A no longer hit in L2 and k_gemm_nt_p is
// faster (r03 A/B).  The packed weight always carries the image for these shapes, whatever the
// route switch says at pack time (the switch is read again at every launch).
static bool gemm_nt_w_shape(int N, int K) {
    return N > 0 && N % 4 == 0 && N <= 2 * ntw_feat(K) && (K == 128 || K == 256);
}

bool gemm_nt_w_ok(int N, int K) {
#ifdef SIR_NT_W
    if (!SIR_NT_W) return false;
#endif
    // OPT-IN (SIR_NT_W=1 in the environment, read per call so a process can A/B it): stand-alone
    // the kernel beats k_gemm_nt_p on Y / G (0.98 vs 1.04 ms at S2), but inside the S2 step it is
    // slower (1.08-1.12 vs 0.95 ms; step 21.6 vs 21.3 ms, r03 A/B on one box), so the default
    // route stays k_gemm_nt_p.
    const char* e = getenv("SIR_NT_W");
    if (e == nullptr || e[0] != '1') return false;
    return gemm_nt_w_shape(N, K);
}

int64_t gemm_pack_w_bytes(int N, int K) {
    if (!gemm_nt_w_shape(N, K)) return 0;
    const int F = ntw_feat(K);
    const int64_t np = (int64_t)(N + F - 1) / F * F;
    return np * K * 4 + np * 4;
}

hipError_t run_gemm_pack_w(const float* W, int64_t ldw, int N, int K, int trans, void* packed, hipStream_t st) {
    const int F = ntw_feat(K);
    const int np = (N + F - 1) / F * F;
    _Float16* out = static_cast<_Float16*>(packed);
    float* inv = reinterpret_cast<float*>(static_cast<char*>(packed) + (int64_t)np * K * 4);
    hipLaunchKernelGGL(k_pack_w, dim3(np), dim3(64), 0, st, W, ldw, N, K, trans, F, out, inv);
    return hipGetLastError();
}

hipError_t run_gemm_nt_w(const float* A, int64_t lda, int64_t M, int K, const void* packed, int N,
                         const float* bias, float* C, int64_t ldc, hipStream_t st, const Drop& drop) {
    if (M == 0) return hipSuccess;
    const int F = ntw_feat(K);
    const int nsl = (N + F - 1) / F, np = nsl * F;
    const int64_t ntiles = (M + 31) / 32;
    if (ntiles >= ((int64_t)1 << 30)) return hipErrorInvalidValue;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        ncu = 256;
    int64_t nrg = (ncu / nsl) / 8 * 8;
    if (nrg < 8) nrg = 8;
    const int64_t need = (ntiles + 7) / 8;             // 8 waves per block, one tile each per round
    if (need < nrg) nrg = (need + 7) / 8 * 8;
    const u4v* img = static_cast<const u4v*>(packed);
    const float* inv = reinterpret_cast<const float*>(static_cast<const char*>(packed) + (int64_t)np * K * 4);
    const dim3 grid((unsigned)(nsl * nrg)), blk(512);
    if (K == 256)
        hipLaunchKernelGGL((k_gemm_nt_w<256, 128>), grid, blk, 0, st, A, lda, M, img, inv, bias, N, C, ldc, nsl,
                           (int)nrg, (int)ntiles, drop);
    else if (K == 512)
        hipLaunchKernelGGL((k_gemm_nt_w<512, 64>), grid, blk, 0, st, A, lda, M, img, inv, bias, N, C, ldc, nsl,
                           (int)nrg, (int)ntiles, drop);
    else
        hipLaunchKernelGGL((k_gemm_nt_w<128, 128>), grid, blk, 0, st, A, lda, M, img, inv, bias, N, C, ldc, nsl,
                           (int)nrg, (int)ntiles, drop);
    return hipGetLastError();
}

}  // namespace sir
