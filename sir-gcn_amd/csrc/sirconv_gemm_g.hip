// sirconv_gemm_g.hip — the layer's fp32 node projections (conv.py:60-61,65 and their input gradients:
// QK = X [W_Q; W_K]^T + b, Y = S W_R^T + b_R, G = dY W_R, dX = [dQ dK] [W_Q; W_K]) as a persistent NT
// GEMM whose operands reach LDS by DMA (buffer_load ... lds), several stages ahead of the MFMAs.
//
// Numerics: the two-term fp16 split of sirconv_gemm.hip (x = (hi + lo) / s, s a power of two per
// data row with the same running-scale-with-hysteresis rule; products hi*hi' + hi*lo' + lo*hi' on
// v_mfma_f32_32x32x16_f16, fp32 accumulation).  The scale is decided per 16-k stage here (per 32-k
// chunk there); inside the fp16 normal range the split does not depend on the scale in force, so the
// results agree with k_gemm_nt_p (tests/test_gemm_gpu.py holds both to <= 2x torch fp32's error).
//
// Why a third NT kernel.  k_gemm_nt_p stages the split A image and the weights in LDS through
// registers: its loads sit in VGPRs (two 32-k chunks deep, the register file is full), both waves
// of a SIMD split / write / wait in lock-step between barriers, and loads and MFMAs barely overlap
// (timing ablations, profiles/r02_ab_gemm_nt_persist.txt: QK 2.09 ms, 1.20 ms without its loads and
// stores, 1.58 ms without its MFMAs).  Here:
//  * A (fp32, raw) and the packed weights go global -> LDS by LDS-DMA into a ring of 4 stages of
//    16 k each (A 16 KiB + W 16 KiB per stage): 3 stages in flight while one is multiplied, no VGPR
//    holds a load, no ds_write for the operands;
//  * every wave reads its own rows' fp32 fragments from the stage and splits them in registers
//    (a data row is split by the 2 waves that share it), so there is no split-image pass and no
//    second barrier per stage;
//  * one raw s_barrier per stage with COUNTED vmcnt waits (the DMA of stage s+1 is waited for at
//    the end of stage s; the epilogue's stores are counted in), so the DMAs stay in flight across
//    barriers (cdna_hip_programming.md §5 "Pipelining across barriers");
//  * the epilogue goes through a per-wave LDS slot (no barrier) and stores 64-B row pieces.
// Tile: 256 data rows x 256 features per block-tile, 8 waves of 64 rows x 128 features (2 x 4 MFMA
// tiles, 128 accumulator registers), one 512-thread block per CU walking a contiguous tile range.
#include "sirconv_internal.h"
#include "sirconv_gemm_util.h"
#include "sirconv_dropout.h"

#include <cstdlib>

#ifndef SIR_NT_G
// OPT-IN (SIR_NT_G=1 in the environment, read per call; 0 here disables it entirely): measured slower than
// k_gemm_nt_p on every S2 shape (profiles/r03_ab_gemm_dma.txt: QK 2.10 vs 1.96, Y 1.06 vs 0.99, dX 1.92
// vs 1.74 ms) — each data row is split by the two waves that share it and the split runs between the
// barrier and the MFMAs of every 16-k stage, so the DMA depth does not pay for it
#define SIR_NT_G 1
#endif

namespace sir {
namespace {
using namespace gemm;

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int GST = 4;                          // LDS stages (GST - 1 in flight)
constexpr int GSTAGE = 32768;                   // A 16 KiB (256 rows x 16 k fp32) + W 16 KiB (hi | lo)
constexpr int GA = 0, GW = 16384, GWLO = 8192;  // offsets inside a stage
constexpr int GSLOT = 2048;                     // per-wave epilogue slot (32 rows x 16 features fp32)
constexpr int GSLOT_OFF = GST * GSTAGE;
constexpr int GEPI_OFF = GSLOT_OFF + 8 * GSLOT; // inv_t[512], bias[512]
constexpr int GLDS = GEPI_OFF + 2 * 512 * 4;
static_assert(GLDS <= 160 * 1024, "LDS budget");
constexpr int GOPS = 4;                         // DMA instructions per wave per stage (2 A + 2 W)
constexpr int GSTORES = 32;                     // epilogue stores per wave per tile
#ifndef SIR_NTG_TB
#define SIR_NTG_TB 1            // 32-row MFMA tiles per wave: 1 = 32 rows x 256 features (each row split once),
#endif                          // 2 = 64 rows x 128 features (each row split by the two waves sharing it)
constexpr int GTB = SIR_NTG_TB, GTA = 8 / GTB, GWF = 8 / GTA;   // row tiles, feature tiles, waves along features

#ifndef SIR_HR
#define SIR_HR 8
#endif
constexpr int SE_INIT = 127;
__device__ inline int bexp(float m) { return (int)((__float_as_uint(m) >> 23) & 255u) - 126; }
__device__ inline int next_se(int se_old, int e_c) {
    if (e_c + se_old <= 15) return se_old;
    const int s = 15 - SIR_HR - e_c;
    return s > 126 ? 126 : s;
}
__device__ inline float pow2(int e) { e = e < -126 ? -126 : (e > 127 ? 127 : e); return __uint_as_float((uint32_t)(e + 127) << 23); }
// m = max(m, |v|) over a float4 (two v_max3_f32 with |.| source modifiers)
__device__ inline float fmax4(float m, float4 v) {
    asm("v_max3_f32 %0, %0, |%1|, |%2|\n\tv_max3_f32 %0, %0, |%3|, |%4|" : "+v"(m) : "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
    return m;
}
// hi = fp16(x s), lo = fp16(x s - hi), one v_fma_mix each (see sirconv_gemm_w.hip); the closing
// s_nop 1 covers the VALU-write -> MFMA-read wait states (the hazard recognizer does not look inside
// inline asm)
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
// Buffer resource as four SGPRs for inline asm (base, stride 0, num_records, gfx9 word3): loads past
// num_records return 0
__device__ inline u4v rsrc4(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)p;
    u4v r;
    r.x = (uint32_t)a;
    r.y = (uint32_t)(a >> 32) & 0xFFFFu;
    r.z = bytes;
    r.w = 0x00020000u;
    return r;
}
// One LDS-DMA wave instruction: lane i's 16 bytes at rsrc + voff land at lds_base + 16 i.  Written as
// inline asm so that the compiler does not see an LDS write in flight: with the builtin it puts
// s_waitcnt vmcnt(0) in front of every ds_read, draining the stages in flight (checked in the .s);
// the waits are counted by hand instead (wait_vm).  The kernel uses M0 for nothing else.
__device__ inline void dma16(const u4v& rs, uint32_t voff, const void* lds_base) {
    const uint32_t m = (uint32_t)(uintptr_t)(lds_void*)lds_base;
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" :: "v"(voff), "s"(rs), "s"(m)
                 : "memory");
}
template <int N>
__device__ inline void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }
// a raw barrier the scheduler cannot move memory operations across (no vmcnt drain: the DMAs of
// later stages stay in flight)
__device__ inline void stage_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

template <int NST>
__global__ void __launch_bounds__(512)
k_gemm_nt_g(const float* __restrict__ A, int64_t lda, int64_t M, const char* __restrict__ Wp, int Npad,
            const float* __restrict__ inv_t, const float* __restrict__ bias, int N, float* __restrict__ C,
            int64_t ldc, int n_ftiles, int n_tiles, int tiles_per_block, Drop drop) {
    static_assert(NST >= 4, "the vmcnt accounting assumes at most one epilogue per 3 stages");
    __shared__ __attribute__((aligned(16))) char lds[GLDS];
    const int t = threadIdx.x;
    const int tb = blockIdx.x * tiles_per_block;
    const int te = (tb + tiles_per_block < n_tiles) ? tb + tiles_per_block : n_tiles;
    if (tb >= te) return;
    float* const inv_l = reinterpret_cast<float*>(lds + GEPI_OFF);
    float* const bias_l = inv_l + 512;
    // x + (-0) == x for every x: without a bias the epilogue adds -0 (no branch)
    inv_l[t] = (t < Npad) ? inv_t[t] : 0.f;
    bias_l[t] = (bias != nullptr && t < N) ? bias[t] : -0.f;

    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int l = t & 63, r = l & 31, h = l >> 5;
    const int d_w = (w / GWF) * 32 * GTB, f_w = (w % GWF) * 32 * GTA;
    const uint32_t wbytes = (uint32_t)((int64_t)(NST / 2) * 4 * Npad * 32);

    // ---- DMA of stage s (block-local stage sequence: tile tb + s / NST, k16 step s % NST) ----
    // A: wave w copies rows 32w .. 32w+31 (2 instructions of 16 rows x 64 B); lane l of instruction i
    // lands at LDS row 32w + 16i + l/4, slot l%4, and fetches the 16-B piece (l%4) ^ ((row/4)%4)
    // of that row (row/4 % 4 = (l/16) % 4): the fragment reads of a 16-lane group then hit 16
    // different bank groups.  Rows past M re-read the tile's last row (never stored).
    // W: wave w copies 1 KiB of the hi plane and 1 KiB of the lo plane of the k16 step (fimg order,
    // lane-linear, as packed by k_pack_weight).
    auto dma = [&](int s) {
        const int j = s / NST, g = s - j * NST;
        const int tt = tb + j;
        char* const st = lds + (s & (GST - 1)) * GSTAGE;
        int64_t d0 = 0;
        int f0 = 0, rows = 1;
        uint32_t abytes = 0;
        if (tt < te) {
            d0 = (int64_t)(tt / n_ftiles) * 256;
            f0 = (tt % n_ftiles) * 256;
            rows = (M - d0 < 256) ? (int)(M - d0) : 256;
            abytes = (uint32_t)(rows * lda * 4);
        }
        const u4v ars = rsrc4(A + d0 * lda, abytes);
        const u4v wrs = rsrc4(Wp, tt < te ? wbytes : 0u);          // stages past the block's range load nothing
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            int row = 32 * w + 16 * i + (l >> 2);
            row = row < rows ? row : rows - 1;
            const int p = (l & 3) ^ ((l >> 4) & 3);
            const uint32_t vo = (uint32_t)((row * (int)lda + 16 * g + 4 * p) * 4);
            dma16(ars, vo, st + GA + (32 * w + 16 * i) * 64);
        }
        const uint32_t hi_off = (uint32_t)((((g >> 1) * 2 + 0) * 2 + (g & 1)) * Npad * 32 + f0 * 32);
        const uint32_t lo_off = (uint32_t)((((g >> 1) * 2 + 1) * 2 + (g & 1)) * Npad * 32 + f0 * 32);
        const uint32_t wo = (uint32_t)(w * 1024 + l * 16);
        dma16(wrs, wo + hi_off, st + GW + w * 1024);
        dma16(wrs, wo + lo_off, st + GW + GWLO + w * 1024);
    };

    f16v acc[GTA][GTB];
    int se[GTB];
#pragma unroll
    for (int b = 0; b < GTB; ++b) se[b] = SE_INIT;
    const int sw = (r >> 2) & 3;                  // A piece swizzle of this lane's rows

    // multiply the k16 step in stage slot `slot`; first: the tile's first step (zero accumulators).
    // The (rare) rescale is one branch ahead of the splits and MFMAs, which then form one basic block
    // the scheduler can interleave (fragment reads and splits under the MFMAs).
    auto compute = [&](int slot, bool first) {
        const char* st = lds + slot * GSTAGE;
        float4 av[GTB][2];
#pragma unroll
        for (int b = 0; b < GTB; ++b)
#pragma unroll
            for (int u = 0; u < 2; ++u)
                av[b][u] = *reinterpret_cast<const float4*>(st + GA + (d_w + 32 * b + r) * 64 + (((2 * h + u) ^ sw) << 4));
        h8 wh[GTA], wl[GTA];
#pragma unroll
        for (int a = 0; a < GTA; ++a) {
            wh[a] = *reinterpret_cast<const h8*>(st + GW + fimg(f_w + 32 * a + r, h));
            wl[a] = *reinterpret_cast<const h8*>(st + GW + GWLO + fimg(f_w + 32 * a + r, h));
        }
        int se_new[GTB];
        bool ch = false;
#pragma unroll
        for (int b = 0; b < GTB; ++b) {
            float m = fmax4(fmax4(0.f, av[b][0]), av[b][1]);
            const auto sx = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
            m = fmaxf(__uint_as_float(sx[0]), __uint_as_float(sx[1]));
            se_new[b] = next_se(first ? SE_INIT : se[b], bexp(m));
            ch |= se_new[b] != se[b];
        }
        if (!first && __builtin_amdgcn_ballot_w64(ch) != 0) {     // rare: a row's maximum rose past 2^SIR_HR
#pragma unroll
            for (int b = 0; b < GTB; ++b) {
                const float fac = pow2(se_new[b] - se[b]);
#pragma unroll
                for (int a = 0; a < GTA; ++a) acc[a][b] *= fac;
            }
        }
        h8 dh[GTB], dl[GTB];
#pragma unroll
        for (int b = 0; b < GTB; ++b) {
            se[b] = se_new[b];
            split8(av[b][0], av[b][1], pow2(se_new[b]), dh[b], dl[b]);
        }
        const f16v zero = {};
#pragma unroll
        for (int a = 0; a < GTA; ++a)
#pragma unroll
            for (int b = 0; b < GTB; ++b) {
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh[a], dh[b], first ? zero : acc[a][b], 0, 0, 0);
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh[a], dl[b], acc[a][b], 0, 0, 0);
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl[a], dh[b], acc[a][b], 0, 0, 0);
            }
    };

    // C[m][n] = acc * 2^-se(m) * inv_t[n] + bias[n] (+ dropout), through the wave's slot: per round
    // 32 rows x 16 features (rows scaled in fragment order, written by 16-B pieces with the A swizzle,
    // read back as 4 lanes per row and stored as 64-B row pieces).  2 stores per round, 16 rounds.
    auto epilogue = [&](int tt) {
        const int64_t d0 = (int64_t)(tt / n_ftiles) * 256;
        const int f0 = (tt % n_ftiles) * 256;
        const int rows = (M - d0 < 256) ? (int)(M - d0) : 256;
        const uint32_t ldc4 = (uint32_t)ldc * 4u;
        const uint32_t nrec = (uint32_t)rows * ldc4;
        const rsrc_t crs = mk_rsrc(C + d0 * ldc, nrec);
        char* const slot = lds + GSLOT_OFF + w * GSLOT;
        const int rq = l >> 2, pq = l & 3;            // read-back role: row rq (+16), piece pq
#pragma unroll
        for (int b = 0; b < GTB; ++b) {
            const float is = pow2(-se[b]);
#pragma unroll
            for (int q = 0; q < 2 * GTA; ++q) {
                const int a = q >> 1;
#pragma unroll
                for (int gg = 0; gg < 2; ++gg) {
                    const int g = 2 * (q & 1) + gg;
                    float4 o;
                    o.x = acc[a][b][4 * g + 0] * is;
                    o.y = acc[a][b][4 * g + 1] * is;
                    o.z = acc[a][b][4 * g + 2] * is;
                    o.w = acc[a][b][4 * g + 3] * is;
                    *reinterpret_cast<float4*>(slot + r * 64 + (((2 * gg + h) ^ sw) << 4)) = o;
                }
                const int n = f0 + f_w + 16 * q + 4 * pq;
                const float4 it = *reinterpret_cast<const float4*>(inv_l + n);
                const float4 bb = *reinterpret_cast<const float4*>(bias_l + n);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int row = rq + 16 * i;
                    const float4 v = *reinterpret_cast<const float4*>(slot + row * 64 + ((pq ^ ((row >> 2) & 3)) << 4));
                    float4 o;
                    o.x = v.x * it.x + bb.x;
                    o.y = v.y * it.y + bb.y;
                    o.z = v.z * it.z + bb.z;
                    o.w = v.w * it.w + bb.w;
                    const int ml = d_w + 32 * b + row;
                    if (drop.on()) {                 // feature dropout of QK (sirconv_dropout.h)
                        const uint32_t rh = drop_row_hash(drop, d0 + ml);
                        const int cc = drop.col0 + n;
                        o.x = drop_keep(drop, rh, cc + 0) ? o.x * drop.scale : 0.f;
                        o.y = drop_keep(drop, rh, cc + 1) ? o.y * drop.scale : 0.f;
                        o.z = drop_keep(drop, rh, cc + 2) ? o.z * drop.scale : 0.f;
                        o.w = drop_keep(drop, rh, cc + 3) ? o.w * drop.scale : 0.f;
                    }
                    u4v ov;
                    ov.x = __float_as_uint(o.x);
                    ov.y = __float_as_uint(o.y);
                    ov.z = __float_as_uint(o.z);
                    ov.w = __float_as_uint(o.w);
                    const uint32_t off = (n < N) ? (uint32_t)ml * ldc4 + (uint32_t)n * 4u : nrec;
                    __builtin_amdgcn_raw_buffer_store_b128(ov, crs, off, 0, 0);
                    // a 16-byte store reads its data VGPRs over several cycles (sirconv_gemm.hip)
                    __builtin_amdgcn_sched_barrier(0);
                    asm volatile("s_nop 1" ::: "memory");
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
    };

    // prologue: stages 0, 1, 2 in flight, wait for stage 0
    dma(0);
    dma(1);
    dma(2);
    wait_vm<2 * GOPS>();
    stage_barrier();                 // also publishes inv_l / bias_l (lgkmcnt(0) before the barrier)

    // Stage s: barrier (stage s landed for every wave; stage s-1's slot is free) -> DMA of stage
    // s+3 into that slot -> multiply stage s -> (tile end: epilogue) -> wait for stage s+1.  The wait
    // leaves the DMAs of stages s+2, s+3 in flight, plus the epilogue stores when one was issued
    // after stage s+1's DMA (at step s, s-1 or s-2: never the block's first tile's first steps).
    int s = 0;
    for (int j = 0; tb + j < te; ++j) {
        const bool later = j > 0;
#pragma unroll
        for (int g = 0; g < NST; ++g, ++s) {
            if (g > 0 || j > 0) stage_barrier();
            dma(s + 3);
            compute(s & (GST - 1), g == 0);
            if (g == NST - 1) {
                epilogue(tb + j);
                wait_vm<2 * GOPS + GSTORES>();
            } else if (g <= 1) {
                if (later) wait_vm<2 * GOPS + GSTORES>();
                else wait_vm<2 * GOPS>();
            } else {
                wait_vm<2 * GOPS>();
            }
        }
    }
}

}  // namespace

// the shapes k_gemm_nt_g takes: K = 128 / 256 / 512, 128 < N <= 512, 16-B aligned rows of A and C
bool gemm_nt_g_ok(const float* A, int64_t lda, int K, int N, const float* C, int64_t ldc) {
    if (!SIR_NT_G) return false;
    const char* e = getenv("SIR_NT_G");       // "1": this kernel (read per call, for A/B in one process)
    if (e == nullptr || e[0] != '1') return false;
    return (K == 128 || K == 256 || K == 512) && N > 128 && gemm_pack_npad(N) <= 512 && lda % 4 == 0 &&
           ldc % 4 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)C & 15) == 0 && (int64_t)256 * lda * 4 < ((int64_t)1 << 32);
}

hipError_t run_gemm_nt_g(const float* A, int64_t lda, int64_t M, int K, const void* packed, int N,
                         const float* bias, float* C, int64_t ldc, hipStream_t st, const Drop& drop) {
    if (M == 0 || N == 0) return hipSuccess;
    const int np = (int)gemm_pack_npad(N), kc = (K + 31) / 32;
    const char* wp = static_cast<const char*>(packed);
    const float* inv = reinterpret_cast<const float*>(wp + (int64_t)kc * 4 * np * 32);
    const int nft = np / 256;
    const int64_t ntiles = (M + 255) / 256 * nft;
    if (ntiles >= ((int64_t)1 << 30)) return hipErrorInvalidValue;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        ncu = 256;
    const int tpb = (int)((ntiles + ncu - 1) / ncu);
    const int nblk = (int)((ntiles + tpb - 1) / tpb);
    const int ti = (int)ntiles;
    if (K == 256)
        hipLaunchKernelGGL(k_gemm_nt_g<16>, dim3(nblk), dim3(512), 0, st, A, lda, M, wp, np, inv, bias, N, C, ldc, nft,
                           ti, tpb, drop);
    else if (K == 512)
        hipLaunchKernelGGL(k_gemm_nt_g<32>, dim3(nblk), dim3(512), 0, st, A, lda, M, wp, np, inv, bias, N, C, ldc, nft,
                           ti, tpb, drop);
    else
        hipLaunchKernelGGL(k_gemm_nt_g<8>, dim3(nblk), dim3(512), 0, st, A, lda, M, wp, np, inv, bias, N, C, ldc, nft,
                           ti, tpb, drop);
    return hipGetLastError();
}

}  // namespace sir
