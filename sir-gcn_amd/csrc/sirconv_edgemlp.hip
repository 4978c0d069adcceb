// sirconv_edgemlp.hip — a dense layer INSIDE the edge loop, fused with the gather and the reduce:
//
//   z_e = Q[v] + K[u],  a_e = act1(z_e),  h_e = W a_e + b,  m_e = act2(h_e)
//   SUM / MEAN / SYM:  out[v] = sum_e c_e * m_e   (c_e = out_norm[u] * in_norm[v] for SYM, mean / deg)
//   MAX:               out[v] = max_e m_e, arg[v] = first arg-max edge (DGL fn.max; empty rows 0 / -1)
//
// Two reference call sites are exactly this shape:
//   * conv.py:45 with sigma = Sequential(ReLU, Linear(H, H), ReLU) (dictionary-lookup/model.py:17):
//     act1 = ReLU, (W, b) = the sigma Linear, act2 = ReLU, reduce = sum/mean/sym;
//   * conv.py:46-47 (agg_type='max'): the per-edge linear_relation: act1 = sigma, (W, b) = W_R, b_R,
//     act2 = identity, reduce = max.
// The reference materialises a_e and m_e as [E, H] / [E, F] tensors (DGL edge UDF); here a block
// owns a work item (a destination row, or a <= chunk-edge piece of a hub row) or, at H = 256, a range
// of the dst-CSR edge stream (k_mlp_fwd16r), stages 32 edges' a_e in LDS, runs h = a W^T on
// split-fp16 MFMA (three v_mfma_f32_32x32x16_f16 per 16 k on hi / lo parts: fp32-accurate products,
// fp32 accumulation) and reduces m_e in registers — no [E, *] tensor in HBM.
//
// Backward of the sum family (H, F <= 256): a destination pass (dQ, and per-block partial dW / db of
// the layer) and a source pass (dK), each recomputing z, a, h for its edges:
//   dm_e = g[v] * c_e,  dh_e = act2'(h_e) dm_e,  da_e = dh_e W,  dz_e = act1'(z_e) da_e,
//   dQ[v] = sum dz_e,  dK[u] = sum dz_e,  dW = sum dh_e (x) a_e,  db = sum dh_e.
// MAX (agg_type='max', act2 = identity, W = W_R): no h is needed — dm_e[n] = dY[v][n] when e is the
// first arg-max edge of (v, n) (the forward's arg), else 0 — and the same passes give dQ, dK and the
// per-block partial dW_R / db_R without any [E, *] tensor (the source pass finds its edges' arg
// status through the source CSR's perm = dst-CSR position).
// Accumulation orders are fixed (no atomics): run-to-run deterministic.
#include "sirconv_edge_impl.h"

namespace sir {
namespace {

typedef float mf16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ mf16 mfma32(float a, float b, mf16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// D-layout row (edge within the 32-edge tile) of accumulator register r in lane l
__device__ __forceinline__ int drow(int r, int l) { return 8 * (r >> 2) + 4 * (l >> 5) + (r & 3); }

template <int ACT>
__device__ __forceinline__ float act_f(float z, float slope) {
    return sig<ACT>(z, slope);
}

// ------------------------------------------------------------------------------ weight packing
// Forward operand B[k][n] = W[n][k] (W: [F, H] row-major, an nn.Linear weight): float4 per lane,
// packed[(t * (HP / 8) + q) * 64 + l] = {W[32t + l%32][8q + 2j + l/32], j = 0..3}, 0 outside.
__global__ void k_mlp_pack(const float* __restrict__ W, int H, int F, int HP, int FP, float4* __restrict__ out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int nq = HP / 8;
    const int64_t total = (int64_t)(FP / 32) * nq * 64;
    if (idx >= total) return;
    const int l = (int)(idx & 63);
    const int q = (int)((idx >> 6) % nq);
    const int t = (int)((idx >> 6) / nq);
    const int n = 32 * t + (l & 31);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int k = 8 * q + 2 * j + (l >> 5);
        v[j] = (n < F && k < H) ? W[(int64_t)n * H + k] : 0.f;
    }
    out[idx] = make_float4(v[0], v[1], v[2], v[3]);
}

// ------------------------------------------------------------------------------ forward, split-fp16 MFMA
// One block per work item (a destination row or a chunk of a hub row): its waves stage 32 edges' a_e
// rows in LDS and compute h = a W^T on v_mfma_f32_32x32x16_f16 with the two-term operand
// split of the projection GEMMs (sirconv_gemm.hip): a = (a_hi + a_lo) / s_e with one power-of-two
// scale per edge row (the whole row is staged before it is split), W = (w_hi + w_lo) / s_n per
// feature (packed once, k_mlp_pack16), h = (a_hi w_hi + a_hi w_lo + a_lo w_hi) / (s_e s_n) with fp32
// accumulation: per product <= 3 * 2^-22 relative (tests/test_gemm_gpu.py's bound), 3 MFMAs of 32
// cycles per 16 k instead of 8 fp32 MFMAs of 64 cycles (5.3x fewer MFMA cycles).
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
__device__ __forceinline__ int mlp_bexp(float m) { return (int)((__float_as_uint(m) >> 23) & 255u) - 126; }
__device__ __forceinline__ float mlp_pow2(int e) {
    e = e < -126 ? -126 : (e > 127 ? 127 : e);
    return __uint_as_float((uint32_t)(e + 127) << 23);
}
// scale exponent with |x| * 2^se < 2^15 for the row maximum m (clamped to a normal float)
__device__ __forceinline__ int mlp_scale_exp(float m) { const int s = 15 - mlp_bexp(m); return s > 126 ? 126 : s; }
// fragment image of one 16-k step plane: piece (row, h) of 16 B at (row / 32) * 1024 + h * 512 + (row % 32) * 16
__device__ __forceinline__ int mlp_fimg(int row, int h) { return ((row >> 5) << 10) + (h << 9) + ((row & 31) << 4); }
// The stream forward's image (32 rows): mlp_fimg with the row's 16-B slot XORed by f = 2 (g & 3) + h.  A
// staging store (ds_write_b64, one edge row a wave, lane l: k-group g = l / 4, half h = (l / 2) & 1) then
// puts the 16 lanes of each store group on 16 distinct 8-B positions of the 128-B bank period (unswizzled:
// all on the row's one slot, 8-way), and the MFMA fragment read (lane l: row l & 31, half l / 32, one g a
// read) still takes 32 distinct slots of its 512-B half (the XOR is a bijection on the slot).
#ifndef SIR_MLP_SWZ
#define SIR_MLP_SWZ 1
#endif
#ifndef SIR_MLP_SPLIT_WALK
#define SIR_MLP_SPLIT_WALK 1    // stream max forward: interior tiles walked by both half-waves (16 edges each)
#endif
#ifndef SIR_MLP_SPLIT_MIX
#define SIR_MLP_SPLIT_MIX 1     // stream forward staging: hi / lo split by v_fma_mix (2 VALU per element)
#endif
// hi = fp16(x s), lo = fp16(x s - hi) of 4 floats (s an exact power of two), one v_fma_mix each into the
// halves of the packed registers: x s is exact and x s - hi exact inside the fused op, so the bits are
// those of rounding y = x s and y - hi separately.  s_nop 1: VALU-write wait states the hazard recognizer
// does not see inside inline asm.
__device__ inline void split4_mix(float4 a, float s, uint2& hi, uint2& lo) {
    uint32_t h0, h1, l0, l1;
    asm volatile(
        "v_fma_mixlo_f16 %0, %4, %8, 0\n\tv_fma_mixhi_f16 %0, %5, %8, 0\n\t"
        "v_fma_mixlo_f16 %1, %6, %8, 0\n\tv_fma_mixhi_f16 %1, %7, %8, 0\n\t"
        "v_fma_mixlo_f16 %2, %4, %8, -%0 op_sel_hi:[0,0,1]\n\tv_fma_mixhi_f16 %2, %5, %8, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %3, %6, %8, -%1 op_sel_hi:[0,0,1]\n\tv_fma_mixhi_f16 %3, %7, %8, -%1 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "s_nop 1"
        : "=&v"(h0), "=&v"(h1), "=&v"(l0), "=&v"(l1)
        : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(s));
    hi = make_uint2(h0, h1);
    lo = make_uint2(l0, l1);
}
__device__ __forceinline__ int mlp_fimg_sw(int row, int h, int g) {
    return (h << 9) + (((row & 31) << 4) ^ (SIR_MLP_SWZ ? ((h << 4) | ((g & 3) << 5)) : 0));
}

// pack: out16[((t * NG + g) * 2 + p) * 64 + l] = 8 halves of part p (hi / lo) of W[32t + l%32][16g + 8(l/32) + j]
// scaled by 2^se(n); inv[n] = 2^-se(n) (0 past F).  One 64-thread block per padded feature.
__global__ void __launch_bounds__(64)
k_mlp_pack16(const float* __restrict__ W, int H, int F, int NG, _Float16* __restrict__ out16, float* __restrict__ inv) {
    const int n = blockIdx.x, l = threadIdx.x;
    float m = 0.f;
    if (n < F)
        for (int k = l; k < H; k += 64) m = fmaxf(m, fabsf(W[(int64_t)n * H + k]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    const int se = mlp_scale_exp(m);
    const float s = mlp_pow2(se);
    const int t = n >> 5, r = n & 31;
    for (int k = l; k < NG * 16; k += 64) {
        const float x = (n < F && k < H) ? W[(int64_t)n * H + k] : 0.f;
        const float y = x * s;
        const _Float16 hh = (_Float16)y;
        const int g = k >> 4, h = (k >> 3) & 1, j = k & 7;
        const int lane = h * 32 + r;
        out16[(((int64_t)t * NG + g) * 2 + 0) * 512 + lane * 8 + j] = hh;
        out16[(((int64_t)t * NG + g) * 2 + 1) * 512 + lane * 8 + j] = (_Float16)(y - (float)hh);
    }
    if (l == 0) inv[n] = (n < F) ? mlp_pow2(-se) : 0.f;
}

// 16-bit storage (autocast, SIR_DTYPE_BF16 / F16): Q / K rows are read in the storage type (half the gather
// bytes of fp32 rows), z and act1 are evaluated in fp32, a is rounded once to the storage type (autocast's
// half-precision message) and h = a W^T runs as ONE 16-bit MFMA per 16 k on W rounded to it (autocast's
// W.to(dtype); k_mlp_pack_st) with fp32 accumulation — the half-precision Linear of the reference's AMP
// path, no operand split.
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
template <int ST>
__device__ __forceinline__ mf16 mfma16_st(h8v a, h8v b, mf16 c) {
    if constexpr (ST == ST_BF16)
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8v, a), __builtin_bit_cast(bf8v, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
// four fp32 values rounded to the storage type, as 8 B (the a image of the 16-bit forms)
template <int ST>
__device__ __forceinline__ uint2 pack4_st(float4 a) {
    return make_uint2(f2h<ST>(a.x) | (f2h<ST>(a.y) << 16), f2h<ST>(a.z) | (f2h<ST>(a.w) << 16));
}
// the weight of the 16-bit forms in k_mlp_pack16's layout: plane 0 = W rounded to the storage type,
// plane 1 = 0, inverse scales 1 (0 past F)
template <int ST>
__global__ void __launch_bounds__(64)
k_mlp_pack_st(const float* __restrict__ W, int H, int F, int NG, uint16_t* __restrict__ out16, float* __restrict__ inv) {
    const int n = blockIdx.x, l = threadIdx.x;
    const int t = n >> 5, r = n & 31;
    for (int k = l; k < NG * 16; k += 64) {
        const float x = (n < F && k < H) ? W[(int64_t)n * H + k] : 0.f;
        const int g = k >> 4, h = (k >> 3) & 1, j = k & 7;
        const int lane = h * 32 + r;
        out16[(((int64_t)t * NG + g) * 2 + 0) * 512 + lane * 8 + j] = (uint16_t)f2h<ST>(x);
        out16[(((int64_t)t * NG + g) * 2 + 1) * 512 + lane * 8 + j] = 0;
    }
    if (l == 0) inv[n] = (n < F) ? 1.f : 0.f;
}

// RPW = rows of the 32-edge tile per wave (32 / NW), C4 = float4 chunks of 256 features per row (HP16 / 256)
template <int ACT1, int ACT2, int RED, int NW, int TPW, int C4, int ST = ST_F32>
__global__ void __launch_bounds__(64 * NW)
k_mlp_fwd16(const int* __restrict__ rowptr, const int* __restrict__ col, const int4* __restrict__ items,
            const typename Stor<ST>::T* __restrict__ Q, int64_t ldq, const typename Stor<ST>::T* __restrict__ K,
            int64_t ldk,
            const float* __restrict__ norm_row, const float* __restrict__ norm_col, float slope,
            int H, int NG, int F, const h8v* __restrict__ Wp16, const float* __restrict__ winv,
            const float* __restrict__ bias, float* __restrict__ out, int64_t ldo, int* __restrict__ arg, int64_t lda,
            float* __restrict__ pval, int* __restrict__ parg) {
    constexpr int RPW = 32 / NW;
    constexpr bool X16 = ST != ST_F32;                 // 16-bit storage: one image, one MFMA per 16 k
    extern __shared__ float smem[];
    char* const img = reinterpret_cast<char*>(smem);                // [NG][2][32 rows fimg] halves
    float* const sInv = reinterpret_cast<float*>(img + NG * 2048);  // [32] 2^-se of the edge rows
    float* const sC = sInv + 32;                                    // [32] c_e (0 past the tile's last edge)
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int4 it = uniform_item(items, blockIdx.x);
    const int row = it.x, e0 = it.y, e1 = it.z, slot = it.w;
    const float nr = (RED == AGG_SYM) ? norm_row[row] : 1.f;
    const auto* qp = Q + (int64_t)row * ldq;
    const int ntile = (F + 31) / 32;

    float racc[TPW], best[TPW], bb[TPW], iw[TPW];
    int bidx[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
        racc[j] = 0.f; best[j] = -INFINITY; bidx[j] = INT_MAX;
        const int n = 32 * (w + NW * j) + (l & 31);
        bb[j] = (bias != nullptr && n < F) ? round_st<ST>(bias[n]) : 0.f;
        iw[j] = (n < F) ? winv[n] : 0.f;
    }
    float4 q4[C4];
#pragma unroll
    for (int c = 0; c < C4; ++c) {
        const int k = 256 * c + 4 * l;
        if constexpr (X16) {
            float t4[4] = {0.f, 0.f, 0.f, 0.f};
            if (k < H) tload_p<ST, 4, false>(t4, qp + k);
            q4[c] = make_float4(t4[0], t4[1], t4[2], t4[3]);
        } else {
            q4[c] = (k < H) ? *reinterpret_cast<const float4*>(qp + k) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }

    for (int t0 = e0; t0 < e1; t0 += 32) {
        const int nv = (e1 - t0) < 32 ? (e1 - t0) : 32;
        // ---- stage: this wave's rows i = w + NW * ii; every K row gathered before any is used
        float4 kv[RPW][C4];
#pragma unroll
        for (int ii = 0; ii < RPW; ++ii) {
            const int i = w + NW * ii;
            const int u = col[t0 + (i < nv ? i : 0)];
#pragma unroll
            for (int c = 0; c < C4; ++c) {
                const int k = 256 * c + 4 * l;
                if constexpr (X16) {
                    float t4[4] = {0.f, 0.f, 0.f, 0.f};
                    if (k < H) tload_p<ST, 4, false>(t4, K + (int64_t)u * ldk + k);
                    kv[ii][c] = make_float4(t4[0], t4[1], t4[2], t4[3]);
                } else {
                    kv[ii][c] = (k < H) ? *reinterpret_cast<const float4*>(K + (int64_t)u * ldk + k)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
        }
#pragma unroll
        for (int ii = 0; ii < RPW; ++ii) {
            const int i = w + NW * ii;
            float4 a4[C4];
            float m = 0.f;
#pragma unroll
            for (int c = 0; c < C4; ++c) {
                const int k = 256 * c + 4 * l;
                const bool ok = i < nv && k < H;
                a4[c].x = ok ? act_f<ACT1>(q4[c].x + kv[ii][c].x, slope) : 0.f;
                a4[c].y = ok ? act_f<ACT1>(q4[c].y + kv[ii][c].y, slope) : 0.f;
                a4[c].z = ok ? act_f<ACT1>(q4[c].z + kv[ii][c].z, slope) : 0.f;
                a4[c].w = ok ? act_f<ACT1>(q4[c].w + kv[ii][c].w, slope) : 0.f;
                m = fmaxf(m, fmaxf(fmaxf(fabsf(a4[c].x), fabsf(a4[c].y)), fmaxf(fabsf(a4[c].z), fabsf(a4[c].w))));
            }
            if constexpr (X16) {
#pragma unroll
                for (int c = 0; c < C4; ++c) {
                    const int k = 256 * c + 4 * l;
                    if (k < NG * 16) {
                        const int g = k >> 4, h = (k >> 3) & 1, j8 = k & 7;
                        *reinterpret_cast<uint2*>(img + g * 2048 + mlp_fimg(i, h) + j8 * 2) = pack4_st<ST>(a4[c]);
                    }
                }
                if (l == 0) sInv[i] = 1.f;
                continue;
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
            const int se = mlp_scale_exp(m);
            const float sc = mlp_pow2(se);
#pragma unroll
            for (int c = 0; c < C4; ++c) {
                const int k = 256 * c + 4 * l;
                if (k < NG * 16) {
                    const float y[4] = {a4[c].x * sc, a4[c].y * sc, a4[c].z * sc, a4[c].w * sc};
                    _Float16 hv[4], lv[4];
#pragma unroll
                    for (int x = 0; x < 4; ++x) { hv[x] = (_Float16)y[x]; lv[x] = (_Float16)(y[x] - (float)hv[x]); }
                    const int g = k >> 4, h = (k >> 3) & 1, j8 = k & 7;
                    char* d = img + g * 2048 + mlp_fimg(i, h) + j8 * 2;
                    *reinterpret_cast<uint2*>(d) = __builtin_bit_cast(uint2, hv);
                    *reinterpret_cast<uint2*>(d + 1024) = __builtin_bit_cast(uint2, lv);
                }
            }
            if (l == 0) sInv[i] = mlp_pow2(-se);
        }
        if (w == 0 && l < 32) {
            float c = 0.f;
            if (l < nv) c = (RED == AGG_SYM) ? norm_col[col[t0 + l]] * nr : 1.f;   // conv.py:45 operand order
            sC[l] = c;
        }
        __syncthreads();
        // ---- h = a W^T on split-fp16 MFMA (this wave's output tiles)
        mf16 acc[TPW];
#pragma unroll
        for (int j = 0; j < TPW; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
        const int fo = mlp_fimg(l & 31, l >> 5);
        for (int g = 0; g < NG; ++g) {
            const h8v ahi = *reinterpret_cast<const h8v*>(img + g * 2048 + fo);
            const h8v alo = X16 ? h8v{} : *reinterpret_cast<const h8v*>(img + g * 2048 + 1024 + fo);
#pragma unroll
            for (int j = 0; j < TPW; ++j) {
                const int t = w + NW * j;
                if (t >= ntile) continue;            // wave-uniform: tiles past F have no packed W
                const h8v whi = Wp16[(((int64_t)t * NG + g) * 2 + 0) * 64 + l];
                if constexpr (X16) {
                    acc[j] = mfma16_st<ST>(ahi, whi, acc[j]);
                } else {
                    const h8v wlo = Wp16[(((int64_t)t * NG + g) * 2 + 1) * 64 + l];
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, whi, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, wlo, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, whi, acc[j], 0, 0, 0);
                }
            }
        }
        // ---- m = act2(h + b), reduced in edge order within the lane
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = drow(r, l);
                if (i < nv) {
                    const float m = act_f<ACT2>(acc[j][r] * sInv[i] * iw[j] + bb[j], slope);
                    if constexpr (RED == 3) {
                        if (m > best[j]) { best[j] = m; bidx[j] = t0 + i; }    // strict >: first wins
                    } else {
                        racc[j] += sC[i] * m;
                    }
                }
            }
        }
        __syncthreads();
    }
    // ---- the two half-waves hold interleaved edge groups of the same columns: combine, store
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
        const int n = 32 * (w + NW * j) + (l & 31);
        if constexpr (RED == 3) {
            const float ob = __shfl_xor(best[j], 32);
            const int oi = __shfl_xor(bidx[j], 32);
            if (ob > best[j] || (ob == best[j] && oi < bidx[j])) { best[j] = ob; bidx[j] = oi; }
            if (l < 32 && n < F) {
                const bool any = bidx[j] != INT_MAX;
                if (slot < 0) {
                    out[(int64_t)row * ldo + n] = any ? best[j] : 0.f;
                    arg[(int64_t)row * lda + n] = any ? bidx[j] : -1;
                } else {
                    pval[(int64_t)slot * F + n] = best[j];
                    parg[(int64_t)slot * F + n] = bidx[j];
                }
            }
        } else {
            const float other = __shfl_xor(racc[j], 32);
            float v = (l < 32) ? racc[j] + other : other + racc[j];
            if (l < 32 && n < F) {
                if (slot < 0) {
                    if constexpr (RED == AGG_MEAN) {
                        const int d = e1 - e0;
                        v = v / (float)(d > 1 ? d : 1);
                    }
                    out[(int64_t)row * ldo + n] = v;
                } else {
                    pval[(int64_t)slot * F + n] = v;
                }
            }
        }
    }
}

// Persistent form for H <= 128, F <= 256 (the DictionaryLookup sigma of config 1):
// 8 waves, wave w owns feature tile w and keeps its whole weight slice (hi and lo, NGT k16 steps:
// 8 NGT VGPRs) in registers for the life of the block, which walks work items b, b + grid, ...  The
// weight is read once per block instead of once per 32-edge tile (k_mlp_fwd16 streamed the packed W
// from L2 for every tile: ~128 GB of L2 reads per S1 forward).  Everything else is k_mlp_fwd16.
template <int ACT1, int ACT2, int RED, int NGT>
__global__ void __launch_bounds__(512)
k_mlp_fwd16p(const int* __restrict__ rowptr, const int* __restrict__ col, const int4* __restrict__ items,
             int64_t n_items, const float* __restrict__ Q, int64_t ldq, const float* __restrict__ K, int64_t ldk,
             const float* __restrict__ norm_row, const float* __restrict__ norm_col, float slope,
             int H, int F, const h8v* __restrict__ Wp16, const float* __restrict__ winv,
             const float* __restrict__ bias, float* __restrict__ out, int64_t ldo, int* __restrict__ arg, int64_t lda,
             float* __restrict__ pval, int* __restrict__ parg) {
    constexpr int NW = 8, RPW = 4;
    constexpr int NG = NGT;
    __shared__ __attribute__((aligned(16))) char img[NG * 2048];
    __shared__ float sInv[32], sC[32];
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ntile = (F + 31) / 32;
    const bool has_t = w < ntile;                 // wave-uniform: waves past F only stage
    const int n = 32 * w + (l & 31);
    const float bbv = (bias != nullptr && n < F) ? bias[n] : 0.f;
    const float iwv = (n < F) ? winv[n] : 0.f;
    h8v whi[NG], wlo[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        if (has_t) {
            whi[g] = Wp16[(((int64_t)w * NG + g) * 2 + 0) * 64 + l];
            wlo[g] = Wp16[(((int64_t)w * NG + g) * 2 + 1) * 64 + l];
        } else {
            whi[g] = h8v{};
            wlo[g] = h8v{};
        }
    }
    const int fo = mlp_fimg(l & 31, l >> 5);
    for (int64_t itx = blockIdx.x; itx < n_items; itx += gridDim.x) {
        const int4 it = uniform_item(items, itx);
        const int row = it.x, e0 = it.y, e1 = it.z, slot = it.w;
        const float nr = (RED == AGG_SYM) ? norm_row[row] : 1.f;
        const float* qp = Q + (int64_t)row * ldq;
        const int k4 = 4 * l;
        const float4 q4 = (k4 < H) ? *reinterpret_cast<const float4*>(qp + k4) : make_float4(0.f, 0.f, 0.f, 0.f);
        float racc = 0.f, best = -INFINITY;
        int bidx = INT_MAX;
        for (int t0 = e0; t0 < e1; t0 += 32) {
            const int nv = (e1 - t0) < 32 ? (e1 - t0) : 32;
            float4 kv[RPW];
#pragma unroll
            for (int ii = 0; ii < RPW; ++ii) {
                const int i = w + NW * ii;
                const int u = col[t0 + (i < nv ? i : 0)];
                kv[ii] = (k4 < H) ? *reinterpret_cast<const float4*>(K + (int64_t)u * ldk + k4)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int ii = 0; ii < RPW; ++ii) {
                const int i = w + NW * ii;
                const bool ok = i < nv && k4 < H;
                float4 a4;
                a4.x = ok ? act_f<ACT1>(q4.x + kv[ii].x, slope) : 0.f;
                a4.y = ok ? act_f<ACT1>(q4.y + kv[ii].y, slope) : 0.f;
                a4.z = ok ? act_f<ACT1>(q4.z + kv[ii].z, slope) : 0.f;
                a4.w = ok ? act_f<ACT1>(q4.w + kv[ii].w, slope) : 0.f;
                float m = fmaxf(fmaxf(fabsf(a4.x), fabsf(a4.y)), fmaxf(fabsf(a4.z), fabsf(a4.w)));
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
                const int se = mlp_scale_exp(m);
                const float sc = mlp_pow2(se);
                if (k4 < NG * 16) {
                    const float y[4] = {a4.x * sc, a4.y * sc, a4.z * sc, a4.w * sc};
                    _Float16 hv[4], lv[4];
#pragma unroll
                    for (int x = 0; x < 4; ++x) { hv[x] = (_Float16)y[x]; lv[x] = (_Float16)(y[x] - (float)hv[x]); }
                    const int g = k4 >> 4, h = (k4 >> 3) & 1, j8 = k4 & 7;
                    char* d = img + g * 2048 + mlp_fimg(i, h) + j8 * 2;
                    *reinterpret_cast<uint2*>(d) = __builtin_bit_cast(uint2, hv);
                    *reinterpret_cast<uint2*>(d + 1024) = __builtin_bit_cast(uint2, lv);
                }
                if (l == 0) sInv[i] = mlp_pow2(-se);
            }
            if (w == 0 && l < 32) {
                float c = 0.f;
                if (l < nv) c = (RED == AGG_SYM) ? norm_col[col[t0 + l]] * nr : 1.f;   // conv.py:45 operand order
                sC[l] = c;
            }
            __syncthreads();
            if (has_t) {
                mf16 acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
                for (int g = 0; g < NG; ++g) {
                    const h8v ahi = *reinterpret_cast<const h8v*>(img + g * 2048 + fo);
                    const h8v alo = *reinterpret_cast<const h8v*>(img + g * 2048 + 1024 + fo);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, whi[g], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, wlo[g], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, whi[g], acc, 0, 0, 0);
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int i = drow(r, l);
                    if (i < nv) {
                        const float m = act_f<ACT2>(acc[r] * sInv[i] * iwv + bbv, slope);
                        if constexpr (RED == 3) {
                            if (m > best) { best = m; bidx = t0 + i; }    // strict >: first wins
                        } else {
                            racc += sC[i] * m;
                        }
                    }
                }
            }
            __syncthreads();
        }
        if (has_t) {
            if constexpr (RED == 3) {
                const float ob = __shfl_xor(best, 32);
                const int oi = __shfl_xor(bidx, 32);
                if (ob > best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
                if (l < 32 && n < F) {
                    const bool any = bidx != INT_MAX;
                    if (slot < 0) {
                        out[(int64_t)row * ldo + n] = any ? best : 0.f;
                        arg[(int64_t)row * lda + n] = any ? bidx : -1;
                    } else {
                        pval[(int64_t)slot * F + n] = best;
                        parg[(int64_t)slot * F + n] = bidx;
                    }
                }
            } else {
                const float other = __shfl_xor(racc, 32);
                float v = (l < 32) ? racc + other : other + racc;
                if (l < 32 && n < F) {
                    if (slot < 0) {
                        if constexpr (RED == AGG_MEAN) {
                            const int d = e1 - e0;
                            v = v / (float)(d > 1 ? d : 1);
                        }
                        out[(int64_t)row * ldo + n] = v;
                    } else {
                        pval[(int64_t)slot * F + n] = v;
                    }
                }
            }
        }
    }
}

// max over the 64 lanes (non-negative values: exact in any order): DPP within each 16-lane row, then
// the four rows' maxima by v_readlane — no LDS round trip (ds_bpermute) per level
__device__ __forceinline__ float wave_max64(float m) {
    m = fmaxf(m, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, m), 0xB1, 0xF, 0xF, false)));
    m = fmaxf(m, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, m), 0x4E, 0xF, 0xF, false)));
    m = fmaxf(m, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, m), 0x141, 0xF, 0xF, false)));
    m = fmaxf(m, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, m), 0x140, 0xF, 0xF, false)));
    const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, m), 0));
    const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, m), 16));
    const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, m), 32));
    const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, m), 48));
    return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}

// Pipelined persistent form (H <= 256, F <= 256; the S1 / S2 max shape): k_mlp_fwd16p's register-
// resident weights, with the block's stream of 32-edge tiles (item after item, b, b + grid, ...)
// software-pipelined so that no gather latency is exposed: while tile i is multiplied and reduced,
// the K rows of tile i + 1 (and its Q row, its norms) are in flight in registers, and the column
// indices of tile i + 2 are loaded one tile earlier still (each wave takes its rows' source ids from
// that vector by v_readlane).  k_mlp_fwd16p issued each tile's gathers and waited for them right
// away (one memory latency per tile on a CU holding one block).  Per tile and edge the arithmetic,
// its order and the reduction order are k_mlp_fwd16p's: the results are bit-identical.
template <int ACT1, int ACT2, int RED, int NGT, bool HF>
__global__ void __launch_bounds__(512)
k_mlp_fwd16q(const int* __restrict__ col, const int4* __restrict__ items, int64_t n_items, const float* __restrict__ Q,
             int64_t ldq, const float* __restrict__ K, int64_t ldk, const float* __restrict__ norm_row,
             const float* __restrict__ norm_col, float slope, int H, int F, const h8v* __restrict__ Wp16,
             const float* __restrict__ winv, const float* __restrict__ bias, float* __restrict__ out, int64_t ldo,
             int* __restrict__ arg, int64_t lda, float* __restrict__ pval, int* __restrict__ parg) {
    constexpr int NW = 8, RPW = 4;
    constexpr int NG = NGT;
    constexpr int C4 = (NG * 16 + 255) / 256;       // float4 chunks of 256 features per row (1 up to H = 256)
    static_assert(C4 == 1, "H <= 256");
    // two LDS images: tile i is multiplied out of one while tile i + 1 is staged into the other
    __shared__ __attribute__((aligned(16))) char img[2][NG * 2048];
    __shared__ __attribute__((aligned(16))) float sInv[2][32];
    __shared__ __attribute__((aligned(16))) float sC[2][32];
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ntile = (F + 31) / 32;
    const bool has_t = w < ntile;
    const int n = 32 * w + (l & 31);
    const float bbv = (bias != nullptr && n < F) ? bias[n] : 0.f;
    const float iwv = (n < F) ? winv[n] : 0.f;
    h8v whi[NG], wlo[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        if (has_t) {
            whi[g] = Wp16[(((int64_t)w * NG + g) * 2 + 0) * 64 + l];
            wlo[g] = Wp16[(((int64_t)w * NG + g) * 2 + 1) * 64 + l];
        } else {
            whi[g] = h8v{};
            wlo[g] = h8v{};
        }
    }
    const int fo = mlp_fimg(l & 31, l >> 5);
    const int k4 = 4 * l;
    // HF: H == 16 NG == 64 * 4 (H = 256, the S1 / S2 shape): every lane's 4 features exist, no masked load
    const bool kin = HF || k4 < H;
    // The block's items b, b + grid, ... come 64 at a time as one vector load (lane j: the block's
    // item 64 q + j), two batches held, read by v_readlane: no scalar load (and no lgkmcnt wait that
    // the LDS reads of the MFMA phase would share) per tile.
    auto load_batch = [&](int q) {
        const int64_t itx = blockIdx.x + (int64_t)(64 * q + l) * gridDim.x;
        return itx < n_items ? items[itx] : make_int4(0, 0, 0, -1);
    };
    int bq = 0;
    int4 ib0 = load_batch(0), ib1 = load_batch(1);
    // tile cursor (wave-uniform): the block's item ordinal k, its row / edges / slot, the tile's first
    // edge; a cursor past the last item reads row 0, edge 0 (valid addresses; nothing of it is used)
    struct Cur { int k; int64_t itx; int row, e0, e1, slot, t0; };
    auto first_of = [&](int k) {
        const int64_t itx = blockIdx.x + (int64_t)k * gridDim.x;
        Cur c;
        if (itx < n_items) {
            const int j = k & 63;
            const bool in0 = (k >> 6) == bq;
            const int x = __builtin_amdgcn_readlane(in0 ? ib0.x : ib1.x, j);
            const int y = __builtin_amdgcn_readlane(in0 ? ib0.y : ib1.y, j);
            const int z = __builtin_amdgcn_readlane(in0 ? ib0.z : ib1.z, j);
            const int wv = __builtin_amdgcn_readlane(in0 ? ib0.w : ib1.w, j);
            c = Cur{k, itx, x, y, z, wv, y};
        } else {
            c = Cur{k, n_items, 0, 0, 0, -1, 0};
        }
        return c;
    };
    auto advance = [&](const Cur& c) {   // the next tile: the next 32 edges of the item, or the block's next item
        if (c.itx < n_items && c.t0 + 32 < c.e1) {
            Cur d = c;
            d.t0 += 32;
            return d;
        }
        return first_of(c.itx < n_items ? c.k + 1 : c.k);
    };
    // lane l (mod 32) of the tile's column vector: col[t0 + min(l, nv - 1)], col[0] for an empty tile
    auto load_col = [&](const Cur& c) {
        const int nv = c.e1 - c.t0 < 32 ? c.e1 - c.t0 : 32;
        const int li = l & 31;
        return col[nv > 0 ? c.t0 + (li < nv ? li : nv - 1) : 0];
    };
    float4 kv[RPW];
    float4 q4;
    float cn = 0.f;
    auto gather = [&](const Cur& c, int colv) {
#pragma unroll
        for (int ii = 0; ii < RPW; ++ii) {
            const int u = __builtin_amdgcn_readlane(colv, w + NW * ii);
            kv[ii] = kin ? *reinterpret_cast<const float4*>(K + (int64_t)u * ldk + k4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        q4 = kin ? *reinterpret_cast<const float4*>(Q + (int64_t)c.row * ldq + k4) : make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (RED == AGG_SYM) cn = norm_col[colv] * norm_row[c.row];   // conv.py:45 operand order
    };
    // stage tile c (its rows in kv / q4 / cn) into image buffer bf: a = act1(q + k), one power-of-two
    // scale per edge row (its max over the 64 lanes), fp16 hi / lo pieces in fragment order
    auto stage = [&](int bf, const Cur& c) {
        const int nv = (c.e1 - c.t0) < 32 ? (c.e1 - c.t0) : 32;
#pragma unroll
        for (int ii = 0; ii < RPW; ++ii) {
            const int i = w + NW * ii;
            const bool ok = i < nv && kin;
            float4 a4;
            a4.x = ok ? act_f<ACT1>(q4.x + kv[ii].x, slope) : 0.f;
            a4.y = ok ? act_f<ACT1>(q4.y + kv[ii].y, slope) : 0.f;
            a4.z = ok ? act_f<ACT1>(q4.z + kv[ii].z, slope) : 0.f;
            a4.w = ok ? act_f<ACT1>(q4.w + kv[ii].w, slope) : 0.f;
            const float m = wave_max64(fmaxf(fmaxf(fabsf(a4.x), fabsf(a4.y)), fmaxf(fabsf(a4.z), fabsf(a4.w))));
            const int se = mlp_scale_exp(m);
            const float sc = mlp_pow2(se);
            if (NG * 16 >= 256 || k4 < NG * 16) {
                const float y[4] = {a4.x * sc, a4.y * sc, a4.z * sc, a4.w * sc};
                _Float16 hv[4], lv[4];
#pragma unroll
                for (int x = 0; x < 4; ++x) { hv[x] = (_Float16)y[x]; lv[x] = (_Float16)(y[x] - (float)hv[x]); }
                const int g = k4 >> 4, h = (k4 >> 3) & 1, j8 = k4 & 7;
                char* d = img[bf] + g * 2048 + mlp_fimg(i, h) + j8 * 2;
                *reinterpret_cast<uint2*>(d) = __builtin_bit_cast(uint2, hv);
                *reinterpret_cast<uint2*>(d + 1024) = __builtin_bit_cast(uint2, lv);
            }
            if (l == 0) sInv[bf][i] = mlp_pow2(-se);
        }
        if (w == 0 && l < 32) sC[bf][l] = (l < nv) ? ((RED == AGG_SYM) ? cn : 1.f) : 0.f;
    };

    Cur cur = first_of(0);
    Cur n1 = advance(cur);
    Cur n2 = advance(n1);
    int colv_n2 = load_col(n2);
    gather(cur, load_col(cur));
    const int colv_n1 = load_col(n1);
    stage(0, cur);
    gather(n1, colv_n1);
    __syncthreads();
    float racc = 0.f, best = -INFINITY;
    int bidx = INT_MAX;
    int bf = 0;
    while (cur.itx < n_items) {
        const int nv = (cur.e1 - cur.t0) < 32 ? (cur.e1 - cur.t0) : 32;
        // ---- tile cur's MFMAs (image bf) and tile n1's staging (image bf ^ 1, rows in kv) in one block:
        // the staging VALU / LDS writes fill the MFMA issue gaps
        // (unconditional: a wave past F multiplies its zero weights — no branch splits the block)
        mf16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const h8v ahi = *reinterpret_cast<const h8v*>(img[bf] + g * 2048 + fo);
            const h8v alo = *reinterpret_cast<const h8v*>(img[bf] + g * 2048 + 1024 + fo);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, whi[g], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, wlo[g], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, whi[g], acc, 0, 0, 0);
        }
        stage(bf ^ 1, n1);
        // ---- tile n2's rows in flight from here to the next iteration's staging; n3's column ids
        const Cur n3 = advance(n2);
        const int colv_n3 = load_col(n3);
        gather(n2, colv_n2);
        if (has_t) {
            // branch-free: the lane's 16 edge rows are 8 g + 4 (l / 32) + (0..3), g = 0..3 — their scales
            // (and c_e) come as four 16-B LDS reads; rows past the tile's last edge are masked by select
            const int hb = 4 * (l >> 5);
            float4 inv4[4], c4[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                inv4[g] = *reinterpret_cast<const float4*>(sInv[bf] + 8 * g + hb);
                if constexpr (RED != 3) c4[g] = *reinterpret_cast<const float4*>(sC[bf] + 8 * g + hb);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = drow(r, l);
                const float iv = r % 4 == 0 ? inv4[r / 4].x : r % 4 == 1 ? inv4[r / 4].y : r % 4 == 2 ? inv4[r / 4].z : inv4[r / 4].w;
                const float m = act_f<ACT2>(acc[r] * iv * iwv + bbv, slope);
                if constexpr (RED == 3) {
                    const bool take = i < nv && m > best;         // strict >: first wins
                    best = take ? m : best;
                    bidx = take ? cur.t0 + i : bidx;
                } else {
                    const float cv = r % 4 == 0 ? c4[r / 4].x : r % 4 == 1 ? c4[r / 4].y : r % 4 == 2 ? c4[r / 4].z : c4[r / 4].w;
                    racc += (i < nv) ? cv * m : 0.f;
                }
            }
            if (n1.itx != cur.itx) {                 // the item's last tile: combine the half-waves, store
                const int row = cur.row, slot = cur.slot;
                if constexpr (RED == 3) {
                    const float ob = __shfl_xor(best, 32);
                    const int oi = __shfl_xor(bidx, 32);
                    if (ob > best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
                    if (l < 32 && n < F) {
                        const bool any = bidx != INT_MAX;
                        if (slot < 0) {
                            out[(int64_t)row * ldo + n] = any ? best : 0.f;
                            arg[(int64_t)row * lda + n] = any ? bidx : -1;
                        } else {
                            pval[(int64_t)slot * F + n] = best;
                            parg[(int64_t)slot * F + n] = bidx;
                        }
                    }
                } else {
                    const float other = __shfl_xor(racc, 32);
                    float v = (l < 32) ? racc + other : other + racc;
                    if (l < 32 && n < F) {
                        if (slot < 0) {
                            if constexpr (RED == AGG_MEAN) {
                                const int d = cur.e1 - cur.e0;
                                v = v / (float)(d > 1 ? d : 1);
                            }
                            out[(int64_t)row * ldo + n] = v;
                        } else {
                            pval[(int64_t)slot * F + n] = v;
                        }
                    }
                }
                racc = 0.f;
                best = -INFINITY;
                bidx = INT_MAX;
            }
        }
        __syncthreads();
        cur = n1;
        n1 = n2;
        n2 = n3;
        colv_n2 = colv_n3;
        bf ^= 1;
        if ((cur.k >> 6) > bq) {             // cur entered the second batch: n3 (<= cur + 3 items) stays within it
            ++bq;
            ib0 = ib1;
            ib1 = load_batch(bq + 1);
        }
    }
}


// ------------------------------------------------------------------------------ forward, edge stream
// The same per-edge layer with the 32-edge MFMA tiles taken from the dst-CSR edge STREAM instead of
// per work item: block b owns edges [E b / nb, E (b + 1) / nb), its tiles are consecutive 32-edge
// windows of it, so a tile holds the edges of several short rows (S1: median in-degree 8 — the
// per-item tiles of k_mlp_fwd16q were 47 % full) and a long row runs through several tiles.  Each
// edge brings its own Q row (erow: the row of every edge).  After the MFMAs every wave writes its
// 32 features x 32 edges of m (c_e m for the sum family) to an LDS tile [feature][edge], and lane n
// walks the tile's edges in order, reducing runs of equal row (max: strict >, first arg-max wins;
// sum: in edge order) and storing a row when its run ends.  A row cut by the block's first or last
// edge writes its partial to the block's slot 2b / 2b + 1 (with its row id in prow), and
// k_mlp_stream_combine merges the slots of each row in block (= edge) order; rows with no edge are
// written by k_mlp_empty_rows.  H = 256 (the S1 / S2 shape), F <= 256; the rest is k_mlp_fwd16q's
// pipeline (weights in registers, two images, next tile's gathers in flight).
template <int ACT1, int ACT2, int RED, int ST = ST_F32>
__global__ void __launch_bounds__(512)
k_mlp_fwd16r(const int* __restrict__ col, const int* __restrict__ erow, const int* __restrict__ rowptr, int64_t E,
             const typename Stor<ST>::T* __restrict__ Q, int64_t ldq, const typename Stor<ST>::T* __restrict__ K,
             int64_t ldk,
             const float* __restrict__ norm_row, const float* __restrict__ norm_col, float slope, int F,
             const h8v* __restrict__ Wp16, const float* __restrict__ winv, const float* __restrict__ bias,
             float* __restrict__ out, int64_t ldo, int* __restrict__ arg, int64_t lda, float* __restrict__ pval,
             int* __restrict__ parg, int* __restrict__ prow) {
    constexpr int NW = 8, RPW = 4, NG = 16, MP = 36;   // MP: pitch of the m tile (floats), bank-rotating
    constexpr bool X16 = ST != ST_F32;                 // 16-bit storage: one image, one MFMA per 16 k
    __shared__ __attribute__((aligned(16))) char img[2][NG * 2048];
    __shared__ __attribute__((aligned(16))) float sInv[2][32];
    __shared__ __attribute__((aligned(16))) float sC[2][32];
    __shared__ __attribute__((aligned(16))) float mt[NW][32 * MP];
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.x, nb = gridDim.x;
    const int64_t eb = E * b / nb, ee = E * (b + 1) / nb;
    if (threadIdx.x == 0) { prow[2 * b] = -1; prow[2 * b + 1] = -1; }
    if (eb >= ee) return;                                    // block-uniform, before any barrier
    const int row_before = eb > 0 ? erow[eb - 1] : -1;       // a run continuing from the previous block
    const int row_after = ee < E ? erow[ee] : -1;            // ... into the next block
    const int n = 32 * w + (l & 31);
    const bool fo_ok = (l < 32) && n < F;                    // the lane that owns feature n's walk / stores
    // 16-bit forms: the bias rounded to the storage type (autocast's bias.to(dtype))
    const float bbv = (bias != nullptr && n < F) ? round_st<ST>(bias[n]) : 0.f;
    const float iwv = (n < F) ? winv[n] : 0.f;
    h8v whi[NG], wlo[NG];
    const bool has_t = w < (F + 31) / 32;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        if (has_t) {
            whi[g] = Wp16[(((int64_t)w * NG + g) * 2 + 0) * 64 + l];
            wlo[g] = X16 ? h8v{} : Wp16[(((int64_t)w * NG + g) * 2 + 1) * 64 + l];
        } else {
            whi[g] = h8v{};
            wlo[g] = h8v{};
        }
    }
    int fos[4];                                             // the lane's fragment slot for g & 3 = 0..3
#pragma unroll
    for (int q = 0; q < 4; ++q) fos[q] = mlp_fimg_sw(l & 31, l >> 5, q);
    const int k4 = 4 * l;
    const int sg = k4 >> 4, sh = (k4 >> 3) & 1, sj8 = k4 & 7;  // the lane's staging k-group / half / offset
    const int T = (int)((ee - eb + 31) / 32);
    // lane l (mod 32) of tile j's column / row vectors (clamped: any index is a valid edge)
    auto tile_t0 = [&](int j) { return eb + 32 * (int64_t)j; };
    auto tile_nv = [&](int j) { const int64_t r = ee - tile_t0(j); return r <= 0 ? 0 : (r < 32 ? (int)r : 32); };
    auto edge_of = [&](int j) {
        const int nv = tile_nv(j);
        const int li = l & 31;
        const int64_t e = nv > 0 ? tile_t0(j) + (li < nv ? li : nv - 1) : ee - 1;
        return e;
    };
    float4 kv[RPW], qv[RPW];
    float cn = 0.f;
    auto gather = [&](int colv, int rowv) {
#pragma unroll
        for (int ii = 0; ii < RPW; ++ii) {
            const int u = __builtin_amdgcn_readlane(colv, w + NW * ii);
            const int r = __builtin_amdgcn_readlane(rowv, w + NW * ii);
            if constexpr (X16) {
                float t4[4];
                tload_p<ST, 4, false>(t4, K + (int64_t)u * ldk + k4);
                kv[ii] = make_float4(t4[0], t4[1], t4[2], t4[3]);
                tload_p<ST, 4, false>(t4, Q + (int64_t)r * ldq + k4);
                qv[ii] = make_float4(t4[0], t4[1], t4[2], t4[3]);
            } else {
                kv[ii] = *reinterpret_cast<const float4*>(K + (int64_t)u * ldk + k4);
                qv[ii] = *reinterpret_cast<const float4*>(Q + (int64_t)r * ldq + k4);
            }
        }
        if constexpr (RED == AGG_SYM) cn = norm_col[colv] * norm_row[rowv];   // conv.py:45 operand order
    };
    auto stage = [&](int bf, int nv) {
#pragma unroll
        for (int ii = 0; ii < RPW; ++ii) {
            const int i = w + NW * ii;
            const bool ok = i < nv;
            float4 a4;
            a4.x = ok ? act_f<ACT1>(qv[ii].x + kv[ii].x, slope) : 0.f;
            a4.y = ok ? act_f<ACT1>(qv[ii].y + kv[ii].y, slope) : 0.f;
            a4.z = ok ? act_f<ACT1>(qv[ii].z + kv[ii].z, slope) : 0.f;
            a4.w = ok ? act_f<ACT1>(qv[ii].w + kv[ii].w, slope) : 0.f;
            char* const d = img[bf] + sg * 2048 + mlp_fimg_sw(i, sh, sg) + sj8 * 2;
            if constexpr (X16) {
                *reinterpret_cast<uint2*>(d) = pack4_st<ST>(a4);
                if (l == 0) sInv[bf][i] = 1.f;
                continue;
            }
            const float m = wave_max64(fmaxf(fmaxf(fabsf(a4.x), fabsf(a4.y)), fmaxf(fabsf(a4.z), fabsf(a4.w))));
            const int se = mlp_scale_exp(m);
            const float sc = mlp_pow2(se);
            if constexpr (SIR_MLP_SPLIT_MIX) {
                uint2 hv, lv;
                split4_mix(a4, sc, hv, lv);
                *reinterpret_cast<uint2*>(d) = hv;
                *reinterpret_cast<uint2*>(d + 1024) = lv;
            } else {
                const float y[4] = {a4.x * sc, a4.y * sc, a4.z * sc, a4.w * sc};
                _Float16 hv[4], lv[4];
#pragma unroll
                for (int x = 0; x < 4; ++x) { hv[x] = (_Float16)y[x]; lv[x] = (_Float16)(y[x] - (float)hv[x]); }
                *reinterpret_cast<uint2*>(d) = __builtin_bit_cast(uint2, hv);
                *reinterpret_cast<uint2*>(d + 1024) = __builtin_bit_cast(uint2, lv);
            }
            if (l == 0) sInv[bf][i] = mlp_pow2(-se);
        }
        if (w == 0 && l < 32) sC[bf][l] = (l < nv) ? ((RED == AGG_SYM) ? cn : 1.f) : 0.f;
    };

    int colv0 = col[edge_of(0)], rowv0 = erow[edge_of(0)];
    int colv1 = col[edge_of(1)], rowv1 = erow[edge_of(1)];
    int colv2 = col[edge_of(2)], rowv2 = erow[edge_of(2)];
    gather(colv0, rowv0);
    stage(0, tile_nv(0));
    gather(colv1, rowv1);
    __syncthreads();
    float racc = 0.f, best = -INFINITY;
    int bidx = INT_MAX;
    bool first_run = true;
    int bf = 0;
    float* const mw = mt[w];
    for (int j = 0; j < T; ++j) {
        const int nv = tile_nv(j);
        const int64_t t0 = tile_t0(j);
        mf16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const h8v ahi = *reinterpret_cast<const h8v*>(img[bf] + g * 2048 + fos[g & 3]);
            if constexpr (X16) {
                acc = mfma16_st<ST>(ahi, whi[g], acc);
            } else {
                const h8v alo = *reinterpret_cast<const h8v*>(img[bf] + g * 2048 + 1024 + fos[g & 3]);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, whi[g], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, wlo[g], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, whi[g], acc, 0, 0, 0);
            }
        }
        stage(bf ^ 1, tile_nv(j + 1));
        const int colv3 = col[edge_of(j + 3)], rowv3 = erow[edge_of(j + 3)];
        gather(colv2, rowv2);
        // ---- m (or c_e m) of this wave's 32 features x the tile's 32 edges -> mw[feature][edge]
        {
            const int hb = 4 * (l >> 5);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 iv = *reinterpret_cast<const float4*>(sInv[bf] + 8 * g + hb);
                float4 o;
                o.x = act_f<ACT2>(acc[4 * g + 0] * iv.x * iwv + bbv, slope);
                o.y = act_f<ACT2>(acc[4 * g + 1] * iv.y * iwv + bbv, slope);
                o.z = act_f<ACT2>(acc[4 * g + 2] * iv.z * iwv + bbv, slope);
                o.w = act_f<ACT2>(acc[4 * g + 3] * iv.w * iwv + bbv, slope);
                if constexpr (RED != 3) {
                    const float4 cv = *reinterpret_cast<const float4*>(sC[bf] + 8 * g + hb);
                    o.x = cv.x * o.x; o.y = cv.y * o.y; o.z = cv.z * o.z; o.w = cv.w * o.w;
                }
                *reinterpret_cast<float4*>(mw + (l & 31) * MP + 8 * g + hb) = o;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);          // lgkmcnt(0): this wave's tile writes done
        __builtin_amdgcn_wave_barrier();
        const int next_first = (j + 1 < T) ? __builtin_amdgcn_readlane(rowv1, 0) : row_after;
        // run ends of the tile as one ballot (bit e: edge e is the last of its row's run here): the row
        // changes after it, or the block ends there
        const int li = l & 31;
        const int r_next = __shfl(rowv0, (li + 1) & 31);
        const bool end_l = li < nv && ((li + 1 < nv ? r_next : next_first) != rowv0 || (li + 1 == nv && t0 + nv == ee));
        const uint32_t bnd = (uint32_t)__builtin_amdgcn_ballot_w64(l < 32 && end_l);
        if constexpr (RED == 3 && SIR_MLP_SPLIT_WALK) {
            if (!first_run && t0 + 32 < ee) {
                // max over a full interior tile (no block-boundary slot can end here): the two half-waves
                // walk edges 0-15 and 16-31 of the same features.  Half 1's first run may have begun in
                // half 0 (or earlier), so its result waits for half 0's trailing state; max with the
                // first arg-max edge merges exactly (strict >: ties keep the earlier half), so the
                // values and arg edges are those of the one-lane walk.
                const int h = l >> 5;
                float mh[16];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 v = *reinterpret_cast<const float4*>(mw + li * MP + 16 * h + 4 * q);
                    mh[4 * q + 0] = v.x; mh[4 * q + 1] = v.y; mh[4 * q + 2] = v.z; mh[4 * q + 3] = v.w;
                }
                const uint32_t bh = bnd >> (16 * h);
                const int eb = (int)t0 + 16 * h;
                float hb_ = h ? -INFINITY : best;
                int hi_ = h ? INT_MAX : bidx;
                float pb = -INFINITY;                 // half 1: its first run, held back
                int pi = INT_MAX, pr = 0;
                bool seen = false;
                const bool fo_n = n < F;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float v = mh[i];
                    const bool take = v > hb_;
                    hb_ = take ? v : hb_;
                    hi_ = take ? eb + i : hi_;
                    // the rows of edges i and 16 + i by readlane (read whatever the EXEC mask: a cross-lane
                    // read inside the divergent branch would see the other half's lanes disabled)
                    const int re0 = __builtin_amdgcn_readlane(rowv0, i);
                    const int re1 = __builtin_amdgcn_readlane(rowv0, 16 + i);
                    if ((bh >> i) & 1u) {
                        const int re = h ? re1 : re0;
                        if (h == 1 && !seen) {
                            pb = hb_; pi = hi_; pr = re;
                        } else if (fo_n) {
                            const bool any = hi_ != INT_MAX;
                            out[(int64_t)re * ldo + n] = any ? hb_ : 0.f;
                            arg[(int64_t)re * lda + n] = any ? hi_ : -1;
                        }
                        seen = true;
                        hb_ = -INFINITY;
                        hi_ = INT_MAX;
                    }
                }
                // half 0's trailing state <-> half 1's
                const float ob = __shfl_xor(hb_, 32);
                const int oi = __shfl_xor(hi_, 32);
                if (h == 1 && (bh & 0xffffu) != 0u) {                 // half 1 had a run end: its first
                    const bool t1 = pb > ob;                         // run continues half 0's trailing one
                    const float mb = t1 ? pb : ob;
                    const int mi = t1 ? pi : oi;
                    if (fo_n) {
                        const bool any = mi != INT_MAX;
                        out[(int64_t)pr * ldo + n] = any ? mb : 0.f;
                        arg[(int64_t)pr * lda + n] = any ? mi : -1;
                    }
                }
                // the carry into the next tile (both halves): half 1's trailing run, or, without a run end
                // in half 1, half 0's trailing run continued through half 1
                const float b0 = h ? ob : hb_, b1 = h ? hb_ : ob;
                const int i0 = h ? oi : hi_, i1 = h ? hi_ : oi;
                const bool end1 = (bnd >> 16) != 0u;
                const bool t1 = end1 || b1 > b0;
                best = t1 ? b1 : b0;
                bidx = t1 ? i1 : i0;
                goto tile_done;
            }
        }
        {
        float mv[32];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float4 v = *reinterpret_cast<const float4*>(mw + (l & 31) * MP + 4 * q);
            mv[4 * q + 0] = v.x; mv[4 * q + 1] = v.y; mv[4 * q + 2] = v.z; mv[4 * q + 3] = v.w;
        }
        // ---- walk the tile's edges in order; a run of equal rows ends where the row changes
#pragma unroll
        for (int e = 0; e < 32; ++e) {
            if (e < nv) {
                const float v = mv[e];
                if constexpr (RED == 3) {
                    const bool take = v > best;           // strict >: the first arg-max edge wins
                    best = take ? v : best;
                    bidx = take ? (int)(t0 + e) : bidx;
                } else {
                    racc += v;
                }
                if ((bnd >> e) & 1u) {
                    const int re = __builtin_amdgcn_readlane(rowv0, e);
                    const bool last_in_block = t0 + e + 1 == ee;
                    const bool cut0 = first_run && re == row_before;
                    const bool cut1 = last_in_block && re == row_after;
                    if (cut0 || cut1) {
                        const int slot = cut0 ? 2 * b : 2 * b + 1;
                        if (fo_ok) {
                            pval[(int64_t)slot * F + n] = RED == 3 ? best : racc;
                            if constexpr (RED == 3) parg[(int64_t)slot * F + n] = bidx;
                        }
                        if (w == 0 && l == 0) prow[slot] = re;
                    } else if (fo_ok) {
                        if constexpr (RED == 3) {
                            const bool any = bidx != INT_MAX;
                            out[(int64_t)re * ldo + n] = any ? best : 0.f;
                            arg[(int64_t)re * lda + n] = any ? bidx : -1;
                        } else {
                            float vv = racc;
                            if constexpr (RED == AGG_MEAN) {
                                const int d = rowptr[re + 1] - rowptr[re];
                                vv = vv / (float)(d > 1 ? d : 1);
                            }
                            out[(int64_t)re * ldo + n] = vv;
                        }
                    }
                    racc = 0.f;
                    best = -INFINITY;
                    bidx = INT_MAX;
                    first_run = false;
                }
            }
        }
        }
    tile_done:
        __syncthreads();
        colv0 = colv1; rowv0 = rowv1;
        colv1 = colv2; rowv1 = rowv2;
        colv2 = colv3; rowv2 = rowv3;
        bf ^= 1;
    }
}

// rows without an edge: out = 0 (and arg = -1 for MAX), as DGL's reduce leaves them
__global__ void __launch_bounds__(256)
k_mlp_empty_rows(const int* __restrict__ rowptr, int64_t n_rows, int F, float* __restrict__ out, int64_t ldo,
                 int* __restrict__ arg, int64_t lda) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_rows || rowptr[r + 1] != rowptr[r]) return;
    for (int f = threadIdx.x & 63; f < F; f += 64) {
        out[r * ldo + f] = 0.f;
        if (arg != nullptr) arg[r * lda + f] = -1;
    }
}

// merge the boundary slots of the stream forward: slots in block order, runs of equal row merged (MAX:
// strict >, the earlier slot = the earlier edges wins ties; sum family: added in slot order)
template <int RED>
__global__ void __launch_bounds__(256)
k_mlp_stream_combine(const float* __restrict__ pval, const int* __restrict__ parg, const int* __restrict__ prow,
                     int n_slots, int F, const int* __restrict__ rowptr, float* __restrict__ out, int64_t ldo,
                     int* __restrict__ arg, int64_t lda) {
    for (int f = threadIdx.x; f < F; f += 256) {
        int cur = -1, ba = INT_MAX;
        float bv = 0.f;
        for (int s = 0; s <= n_slots; ++s) {
            const int r = s < n_slots ? prow[s] : -2;
            if (r == -1) continue;
            if (r != cur) {
                if (cur >= 0) {
                    if constexpr (RED == 3) {
                        out[(int64_t)cur * ldo + f] = ba != INT_MAX ? bv : 0.f;
                        arg[(int64_t)cur * lda + f] = ba != INT_MAX ? ba : -1;
                    } else {
                        float v = bv;
                        if constexpr (RED == AGG_MEAN) {
                            const int d = rowptr[cur + 1] - rowptr[cur];
                            v = v / (float)(d > 1 ? d : 1);
                        }
                        out[(int64_t)cur * ldo + f] = v;
                    }
                }
                if (r < 0) break;
                cur = r;
                bv = pval[(int64_t)s * F + f];
                if constexpr (RED == 3) ba = parg[(int64_t)s * F + f];
            } else {
                const float v = pval[(int64_t)s * F + f];
                if constexpr (RED == 3) {
                    if (v > bv) { bv = v; ba = parg[(int64_t)s * F + f]; }
                } else {
                    bv += v;
                }
            }
        }
    }
}

// max: combine the chunk partials of split rows in chunk (= edge) order, strict > (first wins)
__global__ void k_mlp_max_combine(const int4* __restrict__ splits, int F, const float* __restrict__ pval,
                                  const int* __restrict__ parg, float* __restrict__ Y, int64_t ldy,
                                  int* __restrict__ arg, int64_t lda) {
    const int4 sp = splits[blockIdx.x];
    for (int f = threadIdx.x; f < F; f += blockDim.x) {
        float b = pval[(int64_t)sp.y * F + f];
        int a = parg[(int64_t)sp.y * F + f];
        for (int k = 1; k < sp.z; ++k) {
            const float v = pval[(int64_t)(sp.y + k) * F + f];
            if (v > b) { b = v; a = parg[(int64_t)(sp.y + k) * F + f]; }
        }
        Y[(int64_t)sp.x * ldy + f] = b;
        arg[(int64_t)sp.x * lda + f] = a;
    }
}

// sum family: add the partial rows of split rows in slot order (mean: / degree)
template <bool MEAN_DIV>
__global__ void k_mlp_sum_combine(const int4* __restrict__ splits, int F, const float* __restrict__ pval,
                                  float* __restrict__ out, int64_t ldo) {
    const int4 sp = splits[blockIdx.x];
    for (int f = threadIdx.x; f < F; f += blockDim.x) {
        float s = 0.f;
        for (int k = 0; k < sp.z; ++k) s += pval[(int64_t)(sp.y + k) * F + f];
        if (MEAN_DIV) s = s / (float)(sp.w > 1 ? sp.w : 1);
        out[(int64_t)sp.x * ldo + f] = s;
    }
}

// ------------------------------------------------------------------------------ backward (sum family)
// One block of NW waves per work item (persistent over items) shares the LDS image of a 32-edge
// tile: z (pre-activation of act1) and a = act1(z) [32 x 32 NW], dh [32 x 32 NW], and the g rows
// (source pass: the gathered G[v] rows; destination pass: the one row g[v]).  H, F <= 32 NW.  The
// waves split the work by 32-wide tiles — h / dh: feature tile w; da / dz and the dQ / dK columns:
// a-column tile w; the block's partial dW: tiles (tf, th) = w, w + NW, ... — so no two waves ever
// write the same accumulator and the per-block partials are summed in block order afterwards.
template <int ACT1, int ACT2, int RED, bool DST, int NW>
__global__ void __launch_bounds__(64 * NW)
k_mlp_bwd(const int* __restrict__ rowptr, const int* __restrict__ col, const int4* __restrict__ items,
          int64_t n_items, const float* __restrict__ Q, int64_t ldq, const float* __restrict__ K, int64_t ldk,
          const float* __restrict__ G, int64_t ldg, const float* __restrict__ norm_row,
          const float* __restrict__ norm_col, float slope, int H, int HP, int F,
          const float4* __restrict__ Wp, const float* __restrict__ W, const float* __restrict__ bias,
          float* __restrict__ out, int64_t ldo, float* __restrict__ partial, float* __restrict__ Gm,
          float* __restrict__ wpart, const int* __restrict__ argm, int64_t lda, const int* __restrict__ perm) {
    constexpr int P = 32 * NW + 1;               // row pitch of every LDS tile (odd: conflict-free columns)
    constexpr int DWW = NW;                      // dW tiles per wave: (NW x NW tiles) / NW waves
    constexpr bool MAXR = RED == 3;              // agg max: dh = dY routed to the first arg-max edge
    __shared__ float sZ[32 * P], sA[32 * P], sDH[32 * P], sG[DST ? P : 32 * P], sC[32];
    __shared__ int sArg[(MAXR && DST) ? P : 1];
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nt = (F + 31) / 32, nh = (HP + 31) / 32;
    const int nq = HP / 8;
    const int tf_own = w, th_own = w;            // this wave's h / dh tile and da / dz tile
    mf16 dw[DWW];
    float db = 0.f;
#pragma unroll
    for (int d = 0; d < DWW; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) dw[d][r] = 0.f;
    const int nown = 32 * tf_own + (l & 31);     // this lane's feature column in the h / dh tile
    const float bb = (bias != nullptr && nown < F) ? bias[nown] : 0.f;
    const int kk = 32 * th_own + (l & 31);       // this lane's a column in the da / dz tile
    for (int64_t wi = blockIdx.x; wi < n_items; wi += gridDim.x) {
        const int4 it = uniform_item(items, wi);
        const int row = it.x, e0 = it.y, e1 = it.z, slot = it.w;
        const float nr = (RED == AGG_SYM) ? norm_row[row] : 1.f;
        // row-side vector: destination pass Q[v], source pass K[u]; 4 columns per lane
        const float* rp = DST ? Q + (int64_t)row * ldq : K + (int64_t)row * ldk;
        const int k4 = 4 * l;
        float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (k4 < H) rv = *reinterpret_cast<const float4*>(rp + k4);
        if (DST) {                               // g[v] (mean: / deg; the first chunk also writes Gm)
            float degf = 1.f;
            bool first = true;
            if (RED == AGG_MEAN) {
                const int rs = rowptr[row];
                const int d = rowptr[row + 1] - rs;
                degf = (float)(d > 1 ? d : 1);
                first = (e0 == rs);
            }
            for (int n = threadIdx.x; n < 32 * nt; n += 64 * NW) {
                float g = 0.f;
                if (n < F) {
                    g = G[(int64_t)row * ldg + n];
                    if (RED == AGG_MEAN) {
                        g = g / degf;
                        if (Gm != nullptr && first) Gm[(int64_t)row * F + n] = g;
                    }
                }
                sG[n] = g;
                if constexpr (MAXR && DST) sArg[n] = (n < F) ? argm[(int64_t)row * lda + n] : -2;
            }
        }
        float dacc = 0.f;                        // dQ / dK of column kk (this lane's rows)
        for (int t0 = e0; t0 < e1; t0 += 32) {
            const int nv = (e1 - t0) < 32 ? (e1 - t0) : 32;
            // ---- stage z, a (rows w, w + NW, ...; columns past H and rows past nv: zeros)
            if (k4 < 32 * nh) {
                for (int i = w; i < 32; i += NW) {
                    float4 z = make_float4(0.f, 0.f, 0.f, 0.f), a = z;
                    if (i < nv && k4 < H) {
                        const int o = col[t0 + i];
                        const float4 ov = DST ? *reinterpret_cast<const float4*>(K + (int64_t)o * ldk + k4)
                                              : *reinterpret_cast<const float4*>(Q + (int64_t)o * ldq + k4);
                        // z = Q[v] + K[u] in the reference's operand order either way
                        z = DST ? make_float4(rv.x + ov.x, rv.y + ov.y, rv.z + ov.z, rv.w + ov.w)
                                : make_float4(ov.x + rv.x, ov.y + rv.y, ov.z + rv.z, ov.w + rv.w);
                        a = make_float4(act_f<ACT1>(z.x, slope), act_f<ACT1>(z.y, slope), act_f<ACT1>(z.z, slope),
                                        act_f<ACT1>(z.w, slope));
                    }
                    float* dz = sZ + i * P + k4;
                    float* da = sA + i * P + k4;
                    dz[0] = z.x; dz[1] = z.y; dz[2] = z.z; dz[3] = z.w;
                    da[0] = a.x; da[1] = a.y; da[2] = a.z; da[3] = a.w;
                }
            }
            if (!DST) {                          // the gathered g rows of the tile's destinations
                for (int i = w; i < 32; i += NW) {
                    const int o = (i < nv) ? col[t0 + i] : 0;
                    if constexpr (MAXR) {        // dY[v] where this edge (dst-CSR position pos) is the arg-max
                        const int pos = (i < nv) ? perm[t0 + i] : -3;
                        for (int n = l; n < 32 * nt; n += 64)
                            sG[i * P + n] = (i < nv && n < F && argm[(int64_t)o * lda + n] == pos)
                                                ? G[(int64_t)o * ldg + n] : 0.f;
                    } else {
                        for (int n = l; n < 32 * nt; n += 64)
                            sG[i * P + n] = (i < nv && n < F) ? G[(int64_t)o * ldg + n] : 0.f;
                    }
                }
            }
            if (threadIdx.x < 32) {
                float c = 0.f;
                if ((int)threadIdx.x < nv) {
                    if (RED == AGG_SYM) {
                        const int o = col[t0 + threadIdx.x];
                        c = DST ? norm_col[o] * nr : nr * norm_col[o];     // out_norm[u] * in_norm[v]
                    } else {
                        c = 1.f;
                    }
                }
                sC[threadIdx.x] = c;
            }
            __syncthreads();
            // ---- h = a W^T + b (MFMA, this wave's feature tile), dh = act2'(h) * (g * c) -> sDH[i][n]
            if (MAXR && tf_own < nt) {           // max: dh = dm (act2 = identity, no h needed)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int i = drow(r, l);
                    float dh = 0.f;
                    if (i < nv && nown < F) {
                        if constexpr (DST) dh = (sArg[nown] == t0 + i) ? sG[nown] : 0.f;
                        else dh = sG[i * P + nown];
                    }
                    sDH[i * P + nown] = dh;
                    if (DST) db += dh;
                }
            } else if (tf_own < nt) {
                mf16 acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = 0.f;
                const float* arow = sA + (l & 31) * P + (l >> 5);
                for (int q = 0; q < nq; ++q) {
                    const float4 b4 = Wp[(int64_t)(tf_own * nq + q) * 64 + l];
                    acc = mfma32(arow[8 * q + 0], b4.x, acc);
                    acc = mfma32(arow[8 * q + 2], b4.y, acc);
                    acc = mfma32(arow[8 * q + 4], b4.z, acc);
                    acc = mfma32(arow[8 * q + 6], b4.w, acc);
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int i = drow(r, l);
                    float dh = 0.f;
                    if (i < nv && nown < F) {
                        const float gi = DST ? sG[nown] : sG[i * P + nown];
                        const float dm = gi * sC[i];                 // autograd of c * m: grad * c
                        dh = dsig<ACT2>(acc[r] + bb, dm, slope);
                    }
                    sDH[i * P + nown] = dh;
                    if (DST) db += dh;
                }
            }
            __syncthreads();
            // ---- destination pass: dW[n][k] += sum_i dh[i][n] a[i][k]  (K = edges, 2 per MFMA)
            if (DST) {
#pragma unroll
                for (int d = 0; d < DWW; ++d) {
                    const int idx = w + NW * d;
                    const int tf = idx / NW, th = idx % NW;
                    if (tf < nt && th < nh) {
                        for (int s2 = 0; s2 < 16; ++s2) {
                            const int i = 2 * s2 + (l >> 5);
                            dw[d] = mfma32(sDH[i * P + 32 * tf + (l & 31)], sA[i * P + 32 * th + (l & 31)], dw[d]);
                        }
                    }
                }
            }
            // ---- da[i][k] = sum_n dh[i][n] W[n][k]  (K = features), dz = act1'(z) da, summed per lane
            if (th_own < nh) {
                mf16 da;
#pragma unroll
                for (int r = 0; r < 16; ++r) da[r] = 0.f;
                for (int s2 = 0; s2 < 16 * nt; ++s2) {
                    const int n = 2 * s2 + (l >> 5);
                    const float bv = (n < F && kk < H) ? W[(int64_t)n * H + kk] : 0.f;
                    da = mfma32(sDH[(l & 31) * P + n], bv, da);
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int i = drow(r, l);
                    if (i < nv && kk < H) dacc += dsig<ACT1>(sZ[i * P + kk], da[r], slope);
                }
            }
            __syncthreads();
        }
        // ---- dQ[v] (destination pass) / dK[u] (source pass): combine the half-waves, store
        const float v = dacc + __shfl_xor(dacc, 32);
        if (th_own < nh && l < 32 && kk < H) {
            if (slot < 0) out[(int64_t)row * ldo + kk] = v;
            else partial[(int64_t)slot * H + kk] = v;
        }
    }
    if (DST) {   // this block's partial dW [FP x HP] (row-major n, k) and db [FP]
        const int FP = nt * 32;
        const int64_t stride = (int64_t)FP * HP + FP;
        float* wp = wpart + (int64_t)blockIdx.x * stride;
#pragma unroll
        for (int d = 0; d < DWW; ++d) {
            const int idx = w + NW * d;
            const int tf = idx / NW, th = idx % NW;
            if (tf < nt && th < nh) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int n = 32 * tf + drow(r, l);      // MFMA rows = n, columns = k
                    const int k = 32 * th + (l & 31);
                    if (k < HP) wp[(int64_t)n * HP + k] = dw[d][r];
                }
            }
        }
        const float v = db + __shfl_xor(db, 32);
        if (tf_own < nt && l < 32) wp[(int64_t)FP * HP + nown] = v;
    }
}

int mlp_ng(int H) { return (H + 15) / 16; }
int64_t mlp_pack16_bytes(int H, int F) {
    const int FP = (F + 31) / 32 * 32;
    return (int64_t)FP * mlp_ng(H) * 16 * 2 * 2 + (int64_t)FP * 4;
}

#ifndef SIR_MLP_RESIDENT
// 1: H <= 128, F <= 256 on k_mlp_fwd16p (weights resident in registers, persistent blocks): cfg1 0.302 ->
// 0.294 ms; at H = 256 it was slower than the per-item kernel (S1 max forward 15.5 vs 14.4 ms,
// profiles/r03_ab_mlp_resident.txt: the W stream from L2 was not the bound), so NG = 16 stays per-item
#define SIR_MLP_RESIDENT 1
#endif
#ifndef SIR_MLP_PIPE
#define SIR_MLP_PIPE 1          // 1: 128 < H <= 256, F <= 256 on k_mlp_fwd16q (S1 max forward 13.69 -> 10.02 ms,
                                // profiles/r04_ab_mlp_fwd.txt; at H <= 128 k_mlp_fwd16p stays faster)
#endif
// the 16-bit storage forms (max, act2 = identity) on k_mlp_fwd16
template <int ACT1, int ST>
hipError_t mlp_fwd16_st(int nt, dim3 grid, hipStream_t st, const EdgeMlpArgs& a, const void* p16) {
    const int NG = mlp_ng(a.H), FP = (a.F + 31) / 32 * 32;
    const h8v* w16 = static_cast<const h8v*>(p16);
    const float* winv = reinterpret_cast<const float*>(static_cast<const char*>(p16) + (int64_t)FP * NG * 64);
    const auto* Q = reinterpret_cast<const typename Stor<ST>::T*>(a.Q);
    const auto* K = reinterpret_cast<const typename Stor<ST>::T*>(a.K);
    const size_t lds = (size_t)NG * 2048 + 64 * sizeof(float);
#define SIR_MLP_FWD16S(NWV, TPWV, C4V)                                                                           \
    hipLaunchKernelGGL((k_mlp_fwd16<ACT1, ACT_IDENTITY, 3, NWV, TPWV, C4V, ST>), grid, dim3(64 * NWV), lds, st,    \
                       a.rowptr, a.col, reinterpret_cast<const int4*>(a.items), Q, a.ldq, K, a.ldk, a.norm_row,    \
                       a.norm_col, a.slope, a.H, NG, a.F, w16, winv, a.bias, a.out, a.ldo, a.arg, a.lda, a.pval,   \
                       a.parg)
    if (NG * 16 <= 256) {
        if (nt <= 4) SIR_MLP_FWD16S(4, 1, 1);
        else SIR_MLP_FWD16S(8, 2, 1);
    } else {
        if (nt <= 8) SIR_MLP_FWD16S(4, 2, 2);
        else SIR_MLP_FWD16S(8, 2, 2);
    }
#undef SIR_MLP_FWD16S
    return hipGetLastError();
}

template <int ACT1, int ACT2, int RED>
hipError_t mlp_fwd16_nt(int nt, dim3 grid, hipStream_t st, const EdgeMlpArgs& a, const void* p16) {
    const int NG = mlp_ng(a.H), FP = (a.F + 31) / 32 * 32;
    const h8v* w16 = static_cast<const h8v*>(p16);
    const float* winv = reinterpret_cast<const float*>(static_cast<const char*>(p16) + (int64_t)FP * NG * 64);
    if (SIR_MLP_PIPE && a.col != nullptr && a.F <= 256 && NG == 16) {
        const int ncu = device_cu_count();
        // resident blocks only (a persistent block never yields its CU): one 512-thread block per CU
        const int64_t cap = (int64_t)ncu;
        const int64_t nb = a.n_items < cap ? a.n_items : cap;
        const dim3 g((unsigned)nb);
#define SIR_MLP_FWD16Q(NGV, HFV)                                                                                    \
        hipLaunchKernelGGL((k_mlp_fwd16q<ACT1, ACT2, RED, NGV, HFV>), g, dim3(512), 0, st, a.col,                      \
                           reinterpret_cast<const int4*>(a.items), a.n_items, a.Q, a.ldq, a.K, a.ldk, a.norm_row,      \
                           a.norm_col, a.slope, a.H, a.F, w16, winv, a.bias, a.out, a.ldo, a.arg, a.lda, a.pval, a.parg)
        if (a.H == 256) SIR_MLP_FWD16Q(16, true);
        else SIR_MLP_FWD16Q(16, false);
#undef SIR_MLP_FWD16Q
        return hipGetLastError();
    }
    if (SIR_MLP_RESIDENT && a.F <= 256 && (NG == 4 || NG == 8)) {
        const int ncu = device_cu_count();
        // resident blocks only (a persistent block never yields its CU): NG = 16 takes ~208 VGPRs (one
        // 512-thread block per CU), NG <= 8 fits two
        const int64_t cap = (int64_t)ncu * (NG == 16 ? 1 : 2);
        const int64_t nb = a.n_items < cap ? a.n_items : cap;
        const dim3 g((unsigned)nb);
#define SIR_MLP_FWD16P(NGV)                                                                                         \
        hipLaunchKernelGGL((k_mlp_fwd16p<ACT1, ACT2, RED, NGV>), g, dim3(512), 0, st, a.rowptr, a.col,                 \
                           reinterpret_cast<const int4*>(a.items), a.n_items, a.Q, a.ldq, a.K, a.ldk, a.norm_row,      \
                           a.norm_col, a.slope, a.H, a.F, w16, winv, a.bias, a.out, a.ldo, a.arg, a.lda, a.pval, a.parg)
        if (NG == 4) SIR_MLP_FWD16P(4);
        else SIR_MLP_FWD16P(8);
#undef SIR_MLP_FWD16P
        return hipGetLastError();
    }
    const size_t lds = (size_t)NG * 2048 + 64 * sizeof(float);
#define SIR_MLP_FWD16(NWV, TPWV, C4V)                                                                            \
    hipLaunchKernelGGL((k_mlp_fwd16<ACT1, ACT2, RED, NWV, TPWV, C4V>), grid, dim3(64 * NWV), lds, st, a.rowptr,     \
                       a.col, reinterpret_cast<const int4*>(a.items), a.Q, a.ldq, a.K, a.ldk, a.norm_row, a.norm_col, \
                       a.slope, a.H, NG, a.F, w16, winv, a.bias, a.out, a.ldo, a.arg, a.lda, a.pval, a.parg)
    if (NG * 16 <= 256) {
        if (nt <= 1) SIR_MLP_FWD16(1, 1, 1);
        else if (nt <= 2) SIR_MLP_FWD16(2, 1, 1);
        else if (nt <= 4) SIR_MLP_FWD16(4, 1, 1);
        else if (nt <= 8) SIR_MLP_FWD16(4, 2, 1);
        else SIR_MLP_FWD16(8, 2, 1);
    } else {
        if (nt <= 4) SIR_MLP_FWD16(4, 1, 2);
        else if (nt <= 8) SIR_MLP_FWD16(4, 2, 2);
        else SIR_MLP_FWD16(8, 2, 2);
    }
#undef SIR_MLP_FWD16
    return hipGetLastError();
}

template <int ACT1, int ACT2>
hipError_t mlp_fwd16_red(int red, int nt, dim3 grid, hipStream_t st, const EdgeMlpArgs& a, const void* p16) {
    switch (red) {
        case AGG_SUM: return mlp_fwd16_nt<ACT1, ACT2, AGG_SUM>(nt, grid, st, a, p16);
        case AGG_MEAN: return mlp_fwd16_nt<ACT1, ACT2, AGG_MEAN>(nt, grid, st, a, p16);
        case AGG_SYM: return mlp_fwd16_nt<ACT1, ACT2, AGG_SYM>(nt, grid, st, a, p16);
        default: return mlp_fwd16_nt<ACT1, ACT2, 3>(nt, grid, st, a, p16);
    }
}

// waves per block: the larger of the feature / a-column tile counts (H, F <= 32 NW)
int mlp_bwd_nw(int H, int F) {
    const int HP = (H + 7) / 8 * 8;
    const int t = (F + 31) / 32 > (HP + 31) / 32 ? (F + 31) / 32 : (HP + 31) / 32;
    return t <= 2 ? 2 : (t <= 4 ? 4 : 8);
}

template <int ACT1, int ACT2, int RED, bool DST>
hipError_t mlp_bwd_launch(dim3 grid, hipStream_t st, const EdgeMlpArgs& a) {
#define SIR_MLP_BWD(NWV)                                                                                            \
    hipLaunchKernelGGL((k_mlp_bwd<ACT1, ACT2, RED, DST, NWV>), grid, dim3(64 * NWV), 0, st, a.rowptr, a.col,           \
                       reinterpret_cast<const int4*>(a.items), a.n_items, a.Q, a.ldq, a.K, a.ldk, a.G, a.ldg,          \
                       a.norm_row, a.norm_col, a.slope, a.H, a.HP, a.F, reinterpret_cast<const float4*>(a.Wp), a.W,   \
                       a.bias, a.out, a.ldo, a.pval, a.Gm, a.wpart, a.arg, a.lda, a.perm)
    const int nw = mlp_bwd_nw(a.H, a.F);
    if (nw == 2) SIR_MLP_BWD(2);
    else if (nw == 4) SIR_MLP_BWD(4);
    else SIR_MLP_BWD(8);
#undef SIR_MLP_BWD
    return hipGetLastError();
}

template <int ACT1, int ACT2, bool DST>
hipError_t mlp_bwd_red(int red, dim3 grid, hipStream_t st, const EdgeMlpArgs& a) {
    switch (red) {
        case AGG_SUM: return mlp_bwd_launch<ACT1, ACT2, AGG_SUM, DST>(grid, st, a);
        case AGG_MEAN: return mlp_bwd_launch<ACT1, ACT2, AGG_MEAN, DST>(grid, st, a);
        case AGG_SYM: return mlp_bwd_launch<ACT1, ACT2, AGG_SYM, DST>(grid, st, a);
        default:
            if constexpr (ACT2 == ACT_IDENTITY) return mlp_bwd_launch<ACT1, ACT2, 3, DST>(grid, st, a);
            else return hipErrorInvalidValue;
    }
}

// act1 in {identity, relu, leaky, gelu, gelu_tanh} x act2 in {identity, relu}
template <typename Fn>
hipError_t by_acts(int act1, int act2, Fn&& fn) {
#define SIR_ACT2(A1)                                                               \
    return act2 == ACT_RELU ? fn(std::integral_constant<int, A1>{}, std::integral_constant<int, ACT_RELU>{}) \
                            : fn(std::integral_constant<int, A1>{}, std::integral_constant<int, ACT_IDENTITY>{})
    switch (act1) {
        case ACT_IDENTITY: SIR_ACT2(ACT_IDENTITY);
        case ACT_RELU: SIR_ACT2(ACT_RELU);
        case ACT_LEAKY: SIR_ACT2(ACT_LEAKY);
        case ACT_GELU: SIR_ACT2(ACT_GELU);
        default: SIR_ACT2(ACT_GELU_TANH);
    }
#undef SIR_ACT2
}

}  // namespace

// the packed weight: the fp32 fragment image (k_mlp_pack: the backward and the fp32 forward), then,
// 16-B aligned, the split-fp16 image + inverse scales of the forward (k_mlp_pack16)
static int64_t mlp_pack32_floats(int H, int F) {
    const int HP = (H + 7) / 8 * 8, FP = (F + 31) / 32 * 32;
    return (int64_t)(FP / 32) * (HP / 8) * 64 * 4;
}
int64_t mlp_pack_floats(int H, int F) { return mlp_pack32_floats(H, F) + (mlp_pack16_bytes(H, F) + 3) / 4; }
static const void* mlp_p16(const void* packed, int H, int F) {
    return static_cast<const char*>(packed) + mlp_pack32_floats(H, F) * 4;
}

hipError_t run_mlp_pack(const float* W, int H, int F, void* packed, hipStream_t st) {
    const int HP = (H + 7) / 8 * 8, FP = (F + 31) / 32 * 32;
    const int64_t n = (int64_t)(FP / 32) * (HP / 8) * 64;
    hipLaunchKernelGGL(k_mlp_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, W, H, F, HP, FP,
                       static_cast<float4*>(packed));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    char* p16 = static_cast<char*>(packed) + mlp_pack32_floats(H, F) * 4;
    const int NG = mlp_ng(H);
    hipLaunchKernelGGL(k_mlp_pack16, dim3((unsigned)FP), dim3(64), 0, st, W, H, F, NG,
                       reinterpret_cast<_Float16*>(p16), reinterpret_cast<float*>(p16 + (int64_t)FP * NG * 64));
    return hipGetLastError();
}

hipError_t run_mlp_pack_st(const float* W, int H, int F, int dtype, void* packed, hipStream_t st) {
    if (dtype != ST_BF16 && dtype != ST_F16) return hipErrorInvalidValue;
    const int FP = (F + 31) / 32 * 32, NG = mlp_ng(H);
    char* p16 = static_cast<char*>(packed) + mlp_pack32_floats(H, F) * 4;
    uint16_t* o16 = reinterpret_cast<uint16_t*>(p16);
    float* inv = reinterpret_cast<float*>(p16 + (int64_t)FP * NG * 64);
    if (dtype == ST_BF16)
        hipLaunchKernelGGL(k_mlp_pack_st<ST_BF16>, dim3((unsigned)FP), dim3(64), 0, st, W, H, F, NG, o16, inv);
    else
        hipLaunchKernelGGL(k_mlp_pack_st<ST_F16>, dim3((unsigned)FP), dim3(64), 0, st, W, H, F, NG, o16, inv);
    return hipGetLastError();
}

hipError_t run_mlp_fwd(const EdgeMlpArgs& a, int red, int act1, int act2, hipStream_t st) {
    if (a.st != ST_F32 && (red != 3 || act2 != ACT_IDENTITY)) return hipErrorInvalidValue;
    if (a.n_items > 0) {
        if (a.H > 512) return hipErrorInvalidValue;           // the ABI's limit (sirconv.h)
        const int nt = (a.F + 31) / 32;
        const dim3 grid((unsigned)a.n_items);
        hipError_t err;
        if (a.st != ST_F32)
            err = by_acts(act1, ACT_IDENTITY, [&](auto A1, auto) {
                constexpr int X1 = decltype(A1)::value;
                return a.st == ST_BF16 ? mlp_fwd16_st<X1, ST_BF16>(nt, grid, st, a, mlp_p16(a.Wp, a.H, a.F))
                                       : mlp_fwd16_st<X1, ST_F16>(nt, grid, st, a, mlp_p16(a.Wp, a.H, a.F));
            });
        else
            err = by_acts(act1, act2, [&](auto A1, auto A2) {
                return mlp_fwd16_red<decltype(A1)::value, decltype(A2)::value>(red, nt, grid, st, a,
                                                                               mlp_p16(a.Wp, a.H, a.F));
            });
        if (err != hipSuccess) return err;
    }
    if (a.n_splits > 0) {
        const dim3 g((unsigned)a.n_splits);
        if (red == 3)
            hipLaunchKernelGGL(k_mlp_max_combine, g, dim3(256), 0, st, reinterpret_cast<const int4*>(a.splits), a.F,
                               a.pval, a.parg, a.out, a.ldo, a.arg, a.lda);
        else if (red == AGG_MEAN)
            hipLaunchKernelGGL(k_mlp_sum_combine<true>, g, dim3(256), 0, st, reinterpret_cast<const int4*>(a.splits),
                               a.F, a.pval, a.out, a.ldo);
        else
            hipLaunchKernelGGL(k_mlp_sum_combine<false>, g, dim3(256), 0, st, reinterpret_cast<const int4*>(a.splits),
                               a.F, a.pval, a.out, a.ldo);
        return hipGetLastError();
    }
    return hipSuccess;
}

// the stream forward's grid (one 512-thread block per CU) and its boundary-slot workspace
static int mlp_stream_blocks() {
    const int ncu = device_cu_count();
    return ncu > 1024 ? 1024 : ncu;
}
int64_t mlp_stream_work_bytes(int F) {
    const int64_t slots = 2 * 1024;
    return slots * F * 8 + slots * 4;
}

hipError_t run_mlp_fwd_stream(const EdgeMlpArgs& a, int red, int act1, int act2, hipStream_t st) {
    if (a.n_rows == 0) return hipSuccess;
    const int nb = mlp_stream_blocks();
    const int slots = 2 * nb;
    float* pval = static_cast<float*>(a.work);
    int* parg = reinterpret_cast<int*>(pval + (int64_t)2 * 1024 * a.F);
    int* prow = parg + (int64_t)2 * 1024 * a.F;
    const int FP = (a.F + 31) / 32 * 32;
    const h8v* w16 = static_cast<const h8v*>(mlp_p16(a.Wp, a.H, a.F));
    const float* winv = reinterpret_cast<const float*>(reinterpret_cast<const char*>(w16) + (int64_t)FP * mlp_ng(a.H) * 64);
    hipLaunchKernelGGL(k_mlp_empty_rows, dim3((unsigned)((a.n_rows + 3) / 4)), dim3(256), 0, st, a.rowptr, a.n_rows,
                       a.F, a.out, a.ldo, red == 3 ? a.arg : nullptr, a.lda);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess || a.n_edges == 0) return err;
    if (a.st != ST_F32) {
        if (red != 3 || act2 != ACT_IDENTITY) return hipErrorInvalidValue;
        return by_acts(act1, ACT_IDENTITY, [&](auto A1, auto) {
            constexpr int X1 = decltype(A1)::value;
            auto launch = [&](auto S) {
                constexpr int SV = decltype(S)::value;
                using T = typename Stor<SV>::T;
                hipLaunchKernelGGL((k_mlp_fwd16r<X1, ACT_IDENTITY, 3, SV>), dim3((unsigned)nb), dim3(512), 0, st, a.col,
                                   a.erow, a.rowptr, a.n_edges, reinterpret_cast<const T*>(a.Q), a.ldq,
                                   reinterpret_cast<const T*>(a.K), a.ldk, a.norm_row, a.norm_col, a.slope, a.F, w16,
                                   winv, a.bias, a.out, a.ldo, a.arg, a.lda, pval, parg, prow);
                hipLaunchKernelGGL((k_mlp_stream_combine<3>), dim3(1), dim3(256), 0, st, pval, parg, prow, slots, a.F,
                                   a.rowptr, a.out, a.ldo, a.arg, a.lda);
                return hipGetLastError();
            };
            return a.st == ST_BF16 ? launch(std::integral_constant<int, ST_BF16>())
                                   : launch(std::integral_constant<int, ST_F16>());
        });
    }
    err = by_acts(act1, act2, [&](auto A1, auto A2) {
        constexpr int X1 = decltype(A1)::value, X2 = decltype(A2)::value;
        auto launch = [&](auto R) {
            constexpr int RV = decltype(R)::value;
            hipLaunchKernelGGL((k_mlp_fwd16r<X1, X2, RV>), dim3((unsigned)nb), dim3(512), 0, st, a.col, a.erow, a.rowptr,
                               a.n_edges, a.Q, a.ldq, a.K, a.ldk, a.norm_row, a.norm_col, a.slope, a.F, w16, winv,
                               a.bias, a.out, a.ldo, a.arg, a.lda, pval, parg, prow);
            hipLaunchKernelGGL((k_mlp_stream_combine<RV>), dim3(1), dim3(256), 0, st, pval, parg, prow, slots, a.F,
                               a.rowptr, a.out, a.ldo, a.arg, a.lda);
            return hipGetLastError();
        };
        switch (red) {
            case AGG_SUM: return launch(std::integral_constant<int, AGG_SUM>());
            case AGG_MEAN: return launch(std::integral_constant<int, AGG_MEAN>());
            case AGG_SYM: return launch(std::integral_constant<int, AGG_SYM>());
            default: return launch(std::integral_constant<int, 3>());
        }
    });
    return err;
}

// blocks of the backward grid = rows of the destination pass's dW partials: 2048 waves' worth of
// blocks (about 8 waves per CU), fewer when there are fewer work items
int mlp_bwd_blocks(int64_t n_items, int H, int F) {
    const int cap = 2048 / mlp_bwd_nw(H, F);
    return (int)(n_items < cap ? (n_items > 0 ? n_items : 1) : cap);
}

hipError_t run_mlp_bwd(const EdgeMlpArgs& a, bool dst, int red, int act1, int act2, hipStream_t st) {
    if (a.n_items > 0) {
        const dim3 grid((unsigned)mlp_bwd_blocks(a.n_items, a.H, a.F));
        hipError_t err = by_acts(act1, act2, [&](auto A1, auto A2) {
            return dst ? mlp_bwd_red<decltype(A1)::value, decltype(A2)::value, true>(red, grid, st, a)
                       : mlp_bwd_red<decltype(A1)::value, decltype(A2)::value, false>(red, grid, st, a);
        });
        if (err != hipSuccess) return err;
    }
    if (a.n_splits > 0) {      // the rows' partial dQ / dK (H wide) in slot order
        hipLaunchKernelGGL(k_mlp_sum_combine<false>, dim3((unsigned)a.n_splits), dim3(256), 0, st,
                           reinterpret_cast<const int4*>(a.splits), a.H, a.pval, a.out, a.ldo);
        return hipGetLastError();
    }
    return hipSuccess;
}

}  // namespace sir
