// sirconv_edge_impl.h — gfx950 (MI355X, CDNA4) edge-aggregation kernels for SIRConv.
//
// Reference path: briangodwinlim/SIR-GCN models/conv.py:43-45 (message UDF) + conv.py:63
// (graph.update_all -> DGL 2.1.0 gather + GSpMM copy_e/sum; autograd -> gsddmm + index_add).
//
// Design:
//  * Row-CSR, atomics-free.  A "row" is the node reduced INTO: dst for the forward and the dQ
//    pass, src for the dK pass.  One wave (or a 4..32-lane sub-wave when H is small) owns one
//    work item {row, e_begin, e_end, slot}; the row-side vector (Q[v] or K[u], and G[v]) stays in
//    registers, each edge gathers ONE (fwd, dQ) or TWO (dK) contiguous H-float rows with 16-B
//    per-lane loads (1 KiB per wave-instruction at H=256), UNROLL edges in flight per wave.
//  * sigma, sigma', the norm product and the mean division are applied in registers; fp32
//    accumulation sequentially in edge order => an unsplit row reproduces DGL/torch's CPU
//    summation order bit-for-bit (built with -ffp-contract=off).
//  * Power-law hubs: rows longer than the plan chunk are split into several items writing
//    partial rows; a combine kernel adds the partials in slot order (deterministic).
//  * The edge loop's indices are wave-uniform when LPR == 64 (readfirstlane), so col[e],
//    norm_col[u] and the item descriptor come through the scalar unit (s_load).
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma once
#include "sirconv_internal.h"
#include "sirconv_gemm_util.h"

namespace sir {

// ------------------------------------------------------------------------------ sigma
// Formulas follow torch's CPU/GPU kernels (aten Activation.cpp) operation for operation.
template <int ACT>
__device__ __forceinline__ float sig(float z, float slope) {
    if constexpr (ACT == ACT_IDENTITY) {
        return z;
    } else if constexpr (ACT == ACT_RELU) {
        return z > 0.f ? z : 0.f;
    } else if constexpr (ACT == ACT_LEAKY) {
        return z > 0.f ? z : z * slope;
    } else if constexpr (ACT == ACT_GELU) {
        const float kAlpha = 0.70710678118654752440f;  // M_SQRT1_2
        return z * 0.5f * (1.0f + erff(z * kAlpha));
    } else {  // GELU tanh
        const float kBeta = 0.79788456080286535588f;   // M_SQRT2 * M_2_SQRTPI * 0.5
        const float kKappa = 0.044715f;
        const float inner = kBeta * (z + kKappa * z * z * z);
        return 0.5f * z * (1.0f + tanhf(inner));
    }
}

// sigma'(z) applied to an incoming gradient t (torch backward formulas).
template <int ACT>
__device__ __forceinline__ float dsig(float z, float t, float slope) {
    if constexpr (ACT == ACT_IDENTITY) {
        return t;
    } else if constexpr (ACT == ACT_RELU) {
        return z > 0.f ? t : 0.f;        // threshold_backward: result <= 0 -> 0
    } else if constexpr (ACT == ACT_LEAKY) {
        return z > 0.f ? t : t * slope;  // leaky_relu_backward
    } else if constexpr (ACT == ACT_GELU) {
        const float kAlpha = 0.70710678118654752440f;
        const float kBeta = 0.39894228040143267794f;   // M_2_SQRTPI * M_SQRT1_2 * 0.5
        const float cdf = 0.5f * (1.0f + erff(z * kAlpha));
        const float pdf = kBeta * expf(z * z * -0.5f);
        return t * (cdf + z * pdf);
    } else {
        const float kBeta = 0.79788456080286535588f;
        const float kKappa = 0.044715f;
        const float x_sq = z * z;
        const float x_cube = x_sq * z;
        const float inner = kBeta * (z + kKappa * x_cube);
        const float tanh_inner = tanhf(inner);
        const float left = 0.5f * z;
        const float right = 1.0f + tanh_inner;
        const float left_derivative = 0.5f * right;
        const float tanh_derivative = 1.0f - tanh_inner * tanh_inner;
        const float inner_derivative = kBeta * (1.0f + 3.0f * kKappa * x_sq);
        const float right_derivative = left * tanh_derivative * inner_derivative;
        return t * (left_derivative + right_derivative);
    }
}

// ------------------------------------------------------------------------------ storage dtype
// Feature rows (Q, K, G, S, dQ, dK, Gm) are stored as fp32, bf16 or fp16 (SIR_DTYPE_*; the AMP
// path of the reference, heterophilous-datasets/train.py:75, runs the layer under autocast).  Every
// value is converted to fp32 on load; sigma, sigma', the norm product and the accumulation run in
// fp32 (the reference accumulates its promoted fp32 messages), and results are
// rounded once (RNE) on store.  Partial rows of split items stay fp32.
template <int ST> struct Stor { typedef float T; };
template <> struct Stor<ST_BF16> { typedef __bf16 T; };
template <> struct Stor<ST_F16> { typedef _Float16 T; };

typedef unsigned int sir_u2 __attribute__((ext_vector_type(2)));
typedef unsigned int sir_u4 __attribute__((ext_vector_type(4)));

template <int ST>
__device__ __forceinline__ float h2f(uint32_t bits16) {
    if constexpr (ST == ST_BF16) return __uint_as_float(bits16 << 16);
    else return (float)__builtin_bit_cast(_Float16, (uint16_t)bits16);
}
template <int ST>
__device__ __forceinline__ uint32_t f2h(float x) {
    if constexpr (ST == ST_BF16) return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)x);
    else return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)x);
}
// fp32 value rounded to the storage precision (what a store + reload yields)
template <int ST>
__device__ __forceinline__ float round_st(float x) {
    if constexpr (ST == ST_F32) return x;
    else return h2f<ST>(f2h<ST>(x));
}

// backward of the feature dropout on Q / K (sirconv_dropout.h): row `row`, features c0 .. c0+VW-1 of
// dQ (drop.col0 = 0) or dK (drop.col0 = H); 16-bit storage scales the value rounded to it (the
// reference's grad is the half-precision tensor), the store rounds again
template <int ST, int VW>
__device__ __forceinline__ void drop_vec(const Drop& d, int64_t row, int c0, float (&v)[VW]) {
    const uint32_t rh = drop_row_hash(d, row);
#pragma unroll
    for (int w = 0; w < VW; ++w) v[w] = drop_keep(d, rh, d.col0 + c0 + w) ? round_st<ST>(v[w]) * d.scale : 0.f;
}

// ------------------------------------------------------------------------------ vectors
// Cache-policy experiment knobs (tools/edge_ab.py builds them as separate libraries):
//   SIR_NT_STREAM = 1: non-temporal loads/stores for the once-touched row-side streams
//                      (Q/G rows read, S/dQ/dK/partial rows and the sign mask written);
//   SIR_NT_GATHER = 1: non-temporal loads for the gathered rows too.
#ifndef SIR_NT_STREAM
#define SIR_NT_STREAM 0
#endif
#ifndef SIR_NT_GATHER
#define SIR_NT_GATHER 0
#endif
#ifndef SIR_FWD_PF
#define SIR_FWD_PF 1            // row-CSR edge loop (full-wave rows, fp32): next batch's col[] prefetched per lane
#endif
#ifndef SIR_FWD_BUFGATHER
#define SIR_FWD_BUFGATHER 1     // fp32 forward (mask mode): K rows gathered by 16-B buffer loads (not narrowed)
#endif
#ifndef SIR_MASK_WRITELANE
#define SIR_MASK_WRITELANE 1    // forward sign-mask words built by v_writelane (1) or per-lane selects (0)
#endif
typedef float sir_f4 __attribute__((ext_vector_type(4)));

template <int VW, bool NT>
__device__ __forceinline__ void vload_p(float (&d)[VW], const float* __restrict__ p) {
    if constexpr (VW == 4 && NT) {
        const sir_f4 t = __builtin_nontemporal_load(reinterpret_cast<const sir_f4*>(p));
        d[0] = t.x; d[1] = t.y; d[2] = t.z; d[3] = t.w;
    } else if constexpr (VW == 4) {
        const float4 t = *reinterpret_cast<const float4*>(p);
        d[0] = t.x; d[1] = t.y; d[2] = t.z; d[3] = t.w;
    } else {
#pragma unroll
        for (int w = 0; w < VW; ++w) d[w] = NT ? __builtin_nontemporal_load(p + w) : p[w];
    }
}

template <int VW, bool NT>
__device__ __forceinline__ void vstore_p(float* __restrict__ p, const float (&s)[VW]) {
    if constexpr (VW == 4 && NT) {
        sir_f4 t;
        t.x = s[0]; t.y = s[1]; t.z = s[2]; t.w = s[3];
        __builtin_nontemporal_store(t, reinterpret_cast<sir_f4*>(p));
    } else if constexpr (VW == 4) {
        *reinterpret_cast<float4*>(p) = make_float4(s[0], s[1], s[2], s[3]);
    } else {
#pragma unroll
        for (int w = 0; w < VW; ++w) {
            if constexpr (NT) __builtin_nontemporal_store(s[w], p + w);
            else p[w] = s[w];
        }
    }
}

// typed loads / stores: fp32 as above; 16-bit storage as one 8-B access per 4 values
template <int ST, int VW, bool NT>
__device__ __forceinline__ void tload_p(float (&d)[VW], const typename Stor<ST>::T* __restrict__ p) {
    if constexpr (ST == ST_F32) {
        vload_p<VW, NT>(d, p);
    } else if constexpr (VW == 4) {
        const sir_u2* q = reinterpret_cast<const sir_u2*>(p);
        const sir_u2 t = NT ? __builtin_nontemporal_load(q) : *q;
        d[0] = h2f<ST>(t.x & 0xffffu); d[1] = h2f<ST>(t.x >> 16);
        d[2] = h2f<ST>(t.y & 0xffffu); d[3] = h2f<ST>(t.y >> 16);
    } else {
        const uint16_t* q = reinterpret_cast<const uint16_t*>(p);
#pragma unroll
        for (int w = 0; w < VW; ++w) d[w] = h2f<ST>(q[w]);
    }
}

template <int ST, int VW, bool NT>
__device__ __forceinline__ void tstore_p(typename Stor<ST>::T* __restrict__ p, const float (&s)[VW]) {
    if constexpr (ST == ST_F32) {
        vstore_p<VW, NT>(p, s);
    } else if constexpr (VW == 4) {
        sir_u2 t;
        t.x = f2h<ST>(s[0]) | (f2h<ST>(s[1]) << 16);
        t.y = f2h<ST>(s[2]) | (f2h<ST>(s[3]) << 16);
        if constexpr (NT) __builtin_nontemporal_store(t, reinterpret_cast<sir_u2*>(p));
        else *reinterpret_cast<sir_u2*>(p) = t;
    } else {
        uint16_t* q = reinterpret_cast<uint16_t*>(p);
#pragma unroll
        for (int w = 0; w < VW; ++w) q[w] = (uint16_t)f2h<ST>(s[w]);
    }
}

// row-side streams (read or written once) and gathered rows
template <int ST, int VW>
__device__ __forceinline__ void vload_row(float (&d)[VW], const typename Stor<ST>::T* __restrict__ p) { tload_p<ST, VW, SIR_NT_STREAM>(d, p); }
template <int ST, int VW>
__device__ __forceinline__ void vstore_row(typename Stor<ST>::T* __restrict__ p, const float (&s)[VW]) { tstore_p<ST, VW, SIR_NT_STREAM>(p, s); }
template <int VW>
__device__ __forceinline__ void vstore_part(float* __restrict__ p, const float (&s)[VW]) { vstore_p<VW, SIR_NT_STREAM>(p, s); }
template <int ST, int VW>
__device__ __forceinline__ void vload_gather(float (&d)[VW], const typename Stor<ST>::T* __restrict__ p) { tload_p<ST, VW, SIR_NT_GATHER>(d, p); }

template <int VW>
__device__ __forceinline__ void vload(float (&d)[VW], const float* __restrict__ p) {
    if constexpr (VW == 4) {
        const float4 t = *reinterpret_cast<const float4*>(p);
        d[0] = t.x; d[1] = t.y; d[2] = t.z; d[3] = t.w;
    } else {
#pragma unroll
        for (int w = 0; w < VW; ++w) d[w] = p[w];
    }
}

template <int VW>
__device__ __forceinline__ void vstore(float* __restrict__ p, const float (&s)[VW]) {
    if constexpr (VW == 4) {
        *reinterpret_cast<float4*>(p) = make_float4(s[0], s[1], s[2], s[3]);
    } else {
#pragma unroll
        for (int w = 0; w < VW; ++w) p[w] = s[w];
    }
}

// lane K of v takes the wave-uniform x (v_writelane_b32; this clang has no builtin for it)
// (k must fold to a constant after unrolling: an inline-constant lane select, no hazard)
__device__ __forceinline__ void writelane(uint32_t& v, uint32_t x, int k) {
    asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(x), "i"(k));
}

// ------------------------------------------------------------------------------ edge batch
// Processes UU consecutive edges [e, e+UU) of one row: all gathers issued before any use.
// Sub-wave rows (LPR < 64, H <= 128) in sign-mask mode: one record of MW uint32 per edge (>= 8 B),
// bit (w * LPR + li) = (z of feature 4 li + w) > 0, i.e. per vector slot w an LPR-bit field of the
// row's lanes.  The forward extracts each sub-row's field from the wave ballot (shift by the
// sub-row's first lane), the backward passes read the record with one 8- or 16-B load per lane.
template <int LPR, int VW> constexpr int sub_mask_words() { return LPR * VW >= 64 ? LPR * VW / 32 : 2; }

// MK: 0 = no sign mask, 1 = write it (forward, ReLU family), 2 = read it (backward passes of sub-wave
// rows: no Q / K gathered; the full-wave rows' mask backward is k_edge_mask below)
template <int ST, int MODE, int ACT, int AGG, int LPR, int NV, int VW, int UU, int MK>
__device__ __forceinline__ void edge_batch(int e, const int* __restrict__ col,
                                           const typename Stor<ST>::T* __restrict__ C, int64_t ldc,
                                           const typename Stor<ST>::T* __restrict__ G, int64_t ldg,
                                           const float* __restrict__ norm_col, float nr, float slope,
                                           int li, int HC,
                                           const float (&rv)[NV][VW], const float (&gv)[NV][VW],
                                           float (&acc)[NV][VW], uint64_t* __restrict__ mask, int lane,
                                           const int* __restrict__ upre = nullptr,
                                           const int* __restrict__ perm = nullptr) {
    constexpr bool MASKW = MK == 1, MASKR = MK == 2;
    static_assert(!MASKR || (LPR < 64 && NV == 1 && VW == 4 && MODE != MODE_FWD), "mask-read rows are sub-wave float4 rows");
    int u[UU];
#pragma unroll
    for (int i = 0; i < UU; ++i) u[i] = (upre != nullptr) ? upre[i] : col[e + i];
    constexpr bool kBufGather = SIR_FWD_BUFGATHER && MODE == MODE_FWD && ST == ST_F32 && VW == 4 && LPR == 64 && MASKW;
    constexpr int MWS = sub_mask_words<LPR, VW>();
    uint32_t mr[MASKR ? UU : 1][MWS];
    if constexpr (MASKR) {
        // the batch's mask records (edge position: e + i in the dst CSR; perm[e + i] for the source pass)
#pragma unroll
        for (int i = 0; i < UU; ++i) {
            const int p = (MODE == MODE_BWD_SRC) ? perm[e + i] : e + i;
            const uint32_t* rp = reinterpret_cast<const uint32_t*>(mask) + (int64_t)p * MWS;
            if constexpr (MWS == 8) {
                const sir_u4 t = reinterpret_cast<const sir_u4*>(rp)[0];
                const sir_u4 t2 = reinterpret_cast<const sir_u4*>(rp)[1];
                mr[i][0] = t.x; mr[i][1] = t.y; mr[i][2] = t.z; mr[i][3] = t.w;
                mr[i][4] = t2.x; mr[i][5] = t2.y; mr[i][6] = t2.z; mr[i][7] = t2.w;
            } else if constexpr (MWS == 4) {
                const sir_u4 t = *reinterpret_cast<const sir_u4*>(rp);
                mr[i][0] = t.x; mr[i][1] = t.y; mr[i][2] = t.z; mr[i][3] = t.w;
            } else {
                const sir_u2 t = *reinterpret_cast<const sir_u2*>(rp);
                mr[i][0] = t.x; mr[i][1] = t.y;
            }
        }
    }
    float cv[MASKR ? 1 : UU][NV][VW];
    float gc[(MODE == MODE_BWD_SRC) ? UU : 1][NV][VW];
#pragma unroll
    for (int i = 0; i < UU; ++i) {
      if constexpr (!MASKR) {
        // gathers are unconditional: lanes past the row (c >= HC) re-read column 0 and their
        // values are never used.  A guarded load becomes an exec-masked branch whose result the
        // compiler may copy inside the branch, i.e. wait for right after issuing it — that
        // serialised the gathers of some instances (sym forward: +50%).
        const auto* cp = C + (int64_t)u[i] * ldc;
        if constexpr (kBufGather) {
            // one 16-B buffer load per lane off the (wave-uniform) row base; lanes past the row
            // fail the range check and read 0.  A plain float4 load whose halves feed packed
            // (v_pk_*) math only is narrowed by the DAG into two 8-B loads, the second issued
            // after a wait for the first (fp32 forward +20 %, measured)
            const gemm::rsrc_t rs = gemm::mk_rsrc(cp, (uint32_t)(HC * 16));
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                const sir_u4 t = __builtin_amdgcn_raw_buffer_load_b128(rs, (li + LPR * j) * 16, 0, 0);
                cv[i][j][0] = __uint_as_float(t.x); cv[i][j][1] = __uint_as_float(t.y);
                cv[i][j][2] = __uint_as_float(t.z); cv[i][j][3] = __uint_as_float(t.w);
            }
        } else {
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                const int c = li + LPR * j;
                vload_gather<ST, VW>(cv[i][j], cp + (c < HC ? c : 0) * VW);
            }
        }
      }
        if constexpr (MODE == MODE_BWD_SRC) {
            const auto* gp = G + (int64_t)u[i] * ldg;
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                const int c = li + LPR * j;
                vload_gather<ST, VW>(gc[i][j], gp + (c < HC ? c : 0) * VW);
            }
        }
    }
    // sym norms after the row gathers are issued: their (scalar) loads then overlap the gathers
    // instead of the wait for them preceding the gather issue
    float cf[UU];
    if constexpr (AGG == AGG_SYM) {
#pragma unroll
        for (int i = 0; i < UU; ++i) cf[i] = norm_col[u[i]] * nr;  // out_norm[u] * in_norm[v]
    }
    if constexpr (MASKW && LPR < 64) {
        // sub-wave rows: this sub-row's LPR-bit field of each slot's ballot (shifted down by its first
        // lane), packed into the edge's record; lane li stores record word li (several rounds when the
        // batch's words outnumber the sub-row's lanes)
        static_assert(VW == 4 && NV == 1, "sub-wave mask rows are float4 rows");
        constexpr uint32_t FM = (LPR == 32) ? 0xffffffffu : ((1u << LPR) - 1u);
        const int sh = lane - li;
        uint32_t wd[UU][MWS];
#pragma unroll
        for (int i = 0; i < UU; ++i) {
#pragma unroll
            for (int k = 0; k < MWS; ++k) wd[i][k] = 0u;
#pragma unroll
            for (int w = 0; w < VW; ++w) {
                const uint64_t b = __builtin_amdgcn_ballot_w64(li < HC && (rv[0][w] + cv[i][0][w]) > 0.f);
                wd[i][(w * LPR) / 32] |= ((uint32_t)(b >> sh) & FM) << ((w * LPR) % 32);
            }
        }
        uint32_t* mrec = reinterpret_cast<uint32_t*>(mask) + (int64_t)e * MWS;
        constexpr int NWB = UU * MWS;
#pragma unroll
        for (int r = 0; r < (NWB + LPR - 1) / LPR; ++r) {
            uint32_t mine = 0u;
#pragma unroll
            for (int i = 0; i < UU; ++i)
#pragma unroll
                for (int k = 0; k < MWS; ++k)
                    if ((i * MWS + k) / LPR == r) mine = (li == (i * MWS + k) % LPR) ? wd[i][k] : mine;
            const int q = r * LPR + li;
            if (q < NWB) mrec[q] = mine;
        }
    } else if constexpr (MASKW) {
        // sign mask of z for the sign-mask backward: word (j*4+w), bit lane = z[(lane+64j)*4+w] > 0.
        // The UU edges' words are contiguous; lane k takes word k (uniform -> per-lane select)
        // and ONE store writes the batch's UU*NW*8 bytes.
        static_assert(LPR == 64 && VW == 4, "mask layout needs full-wave rows of float4");
        constexpr int NW = NV * VW;
        static_assert(UU * NW <= 64, "one mask store per batch");
#if SIR_MASK_WRITELANE
        // The compare IS the ballot (v_cmp writes the 64-lane mask to SGPRs; the row's column-range
        // mask is ANDed on the scalar unit) and v_writelane drops each word into its lane: 3 VALU
        // per word.  The select form (lane == k ? b : mine) compiled to ~8 VALU per word (the compare
        // materialised as 0/1 and re-compared, SGPR->VGPR moves, per-lane selects) — more VALU per
        // edge than sigma and the sum together.
        uint32_t mlo = 0, mhi = 0;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const uint64_t okm = __builtin_amdgcn_ballot_w64((li + LPR * j) < HC);
#pragma unroll
            for (int i = 0; i < UU; ++i) {
#pragma unroll
                for (int w = 0; w < VW; ++w) {
                    const uint64_t b = __builtin_amdgcn_ballot_w64((rv[j][w] + cv[i][j][w]) > 0.f) & okm;
                    writelane(mlo, (uint32_t)b, i * NW + j * VW + w);
                    writelane(mhi, (uint32_t)(b >> 32), i * NW + j * VW + w);
                }
            }
        }
        const uint64_t mine = ((uint64_t)mhi << 32) | mlo;
#else
        uint64_t mine = 0;
#pragma unroll
        for (int i = 0; i < UU; ++i) {
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                const bool ok = (li + LPR * j) < HC;
#pragma unroll
                for (int w = 0; w < VW; ++w) {
                    const uint64_t b = __ballot(ok && (rv[j][w] + cv[i][j][w]) > 0.f);
                    mine = (lane == i * NW + j * VW + w) ? b : mine;
                }
            }
        }
#endif
        if (lane < UU * NW) {
            if constexpr (SIR_NT_STREAM) __builtin_nontemporal_store(mine, mask + (int64_t)e * NW + lane);
            else mask[(int64_t)e * NW + lane] = mine;
        }
    }
#pragma unroll
    for (int i = 0; i < UU; ++i) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = li + LPR * j;
            if (c < HC) {
#pragma unroll
                for (int w = 0; w < VW; ++w) {
                    if constexpr (MODE == MODE_FWD) {
                        const float z = rv[j][w] + cv[i][j][w];        // eq[v] + ek[u]
                        float m = sig<ACT>(z, slope);
                        if constexpr (AGG == AGG_SYM) m = cf[i] * m;
                        acc[j][w] += m;
                    } else if constexpr (MASKR) {
                        // sigma'(z) from the stored sign: bit (w * LPR + li) of the record
                        float t = (MODE == MODE_BWD_SRC) ? gc[i][j][w] : gv[j][w];
                        if constexpr (AGG == AGG_SYM) t = t * cf[i];
                        const int wi = (w * LPR) / 32;
                        const bool pos = (mr[i][wi] >> (((w * LPR) % 32) + li)) & 1u;
                        acc[j][w] += pos ? t : (ACT == ACT_RELU ? 0.f : t * slope);
                    } else if constexpr (MODE == MODE_BWD_DST) {
                        const float z = rv[j][w] + cv[i][j][w];
                        float t = gv[j][w];
                        if constexpr (AGG == AGG_SYM) t = t * cf[i];
                        acc[j][w] += dsig<ACT>(z, t, slope);
                    } else {
                        const float z = cv[i][j][w] + rv[j][w];        // Q[v] + K[u]
                        float t = gc[i][j][w];
                        if constexpr (AGG == AGG_SYM) t = t * cf[i];
                        acc[j][w] += dsig<ACT>(z, t, slope);
                    }
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------ main kernel
// MODE_FWD:     R = Q (rows = dst), C = K (gathered by src), out = S
// MODE_BWD_DST: R = Q, C = K, G = dS rows (row-side), out = dQ, optional Gm = G/deg (MEAN)
// MODE_BWD_SRC: R = K (rows = src), C = Q (gathered by dst), G = Gd (gathered), out = dK
// One wave's items (64 / LPR consecutive items, one per sub-row) of a pass; `wave` is the wave's
// index among the pass's waves.
template <int ST, int MODE, int ACT, int AGG, int LPR, int NV, int VW, int U, int MK>
__device__ __forceinline__ void
edge_wave(int64_t wave, const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ perm,
          const int4* __restrict__ items, int64_t n_items,
          const typename Stor<ST>::T* __restrict__ R, int64_t ldr,
          const typename Stor<ST>::T* __restrict__ C, int64_t ldc,
          const typename Stor<ST>::T* __restrict__ G, int64_t ldg,
          const float* __restrict__ norm_row, const float* __restrict__ norm_col,
          float slope, int H,
          typename Stor<ST>::T* __restrict__ out, int64_t ldo, float* __restrict__ partial,
          typename Stor<ST>::T* __restrict__ Gm, int64_t ldgm, uint64_t* __restrict__ mask, const Drop& drop,
          int accumulate = 0) {
    // MK bit 2 (forward only): the segmented forward's accumulate form (S[v] += this call's sum), a
    // separate instantiation so that the plain forward carries no read of the old row
    constexpr int MKB = MK & 3;
    constexpr bool ACC = (MK & 4) != 0;
    constexpr int RPW = 64 / LPR;
    const int lane = threadIdx.x & 63;
    const int sub = lane / LPR;
    const int li = lane - sub * LPR;
    const int64_t idx = wave * RPW + sub;
    if (idx >= n_items) return;
    int4 it = items[idx];
    if constexpr (LPR == 64) {
        it.x = __builtin_amdgcn_readfirstlane(it.x);
        it.y = __builtin_amdgcn_readfirstlane(it.y);
        it.z = __builtin_amdgcn_readfirstlane(it.z);
        it.w = __builtin_amdgcn_readfirstlane(it.w);
    }
    const int row = it.x, e0 = it.y, e1 = it.z, slot = it.w;
    const int HC = H / VW;

    float rv[NV][VW];
    float gv[NV][VW];
    float acc[NV][VW];
    const auto* rp = R + (int64_t)row * ldr;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int c = li + LPR * j;
#pragma unroll
        for (int w = 0; w < VW; ++w) { acc[j][w] = 0.f; rv[j][w] = 0.f; gv[j][w] = 0.f; }
        if (MKB != 2 && c < HC) vload_row<ST, VW>(rv[j], rp + c * VW);     // mask-read passes need no Q / K row
    }
    if constexpr (MODE == MODE_BWD_DST) {
        const auto* gp = G + (int64_t)row * ldg;
        float degf = 1.f;
        bool first = true;
        if constexpr (AGG == AGG_MEAN) {
            const int rs = rowptr[row];
            const int d = rowptr[row + 1] - rs;
            degf = (float)(d > 1 ? d : 1);
            first = (e0 == rs);
        }
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = li + LPR * j;
            if (c < HC) {
                vload_row<ST, VW>(gv[j], gp + c * VW);
                if constexpr (AGG == AGG_MEAN) {
                    // DivBackward: grad / deg (16-bit storage: rounded like the Gm copy the src pass reads)
#pragma unroll
                    for (int w = 0; w < VW; ++w) gv[j][w] = round_st<ST>(gv[j][w] / degf);
                    if (Gm != nullptr && first) vstore_row<ST, VW>(Gm + (int64_t)row * ldgm + c * VW, gv[j]);
                }
            }
        }
    }
    float nr = 1.f;
    if constexpr (AGG == AGG_SYM) nr = norm_row[row];

    int e = e0;
    if constexpr (SIR_FWD_PF && LPR == 64 && ST == ST_F32) {
        // software-pipelined column indices (as in the dK pass): the next batch's col[] by one
        // per-lane load issued with the current batch's gathers, moved to SGPRs by v_readlane
        // (S2 forward f32 sum -2 %, mean -2 %, sym -1 %; 16-bit storage +10 %: fp32 only,
        // profiles/r02_ab_index_prefetch.txt)
        if (e + U <= e1) {
            auto load_col = [&](int eb) {
                const int q0 = eb + (lane < U ? lane : 0);
                return col[q0 < e1 ? q0 : e1 - 1];
            };
            int vc = load_col(e);
            for (; e + U <= e1; e += U) {
                int uc[U];
#pragma unroll
                for (int i = 0; i < U; ++i) uc[i] = __builtin_amdgcn_readlane(vc, i);
                vc = load_col(e + U);
                edge_batch<ST, MODE, ACT, AGG, LPR, NV, VW, U, MKB>(e, col, C, ldc, G, ldg, norm_col, nr, slope, li, HC,
                                                                  rv, gv, acc, mask, lane, uc, perm);
            }
        }
    } else {
        for (; e + U <= e1; e += U)
            edge_batch<ST, MODE, ACT, AGG, LPR, NV, VW, U, MKB>(e, col, C, ldc, G, ldg, norm_col, nr, slope, li, HC, rv, gv,
                                                              acc, mask, lane, nullptr, perm);
    }
    if constexpr (U > 8) {
        if (e + 8 <= e1) {
            edge_batch<ST, MODE, ACT, AGG, LPR, NV, VW, 8, MKB>(e, col, C, ldc, G, ldg, norm_col, nr, slope, li, HC, rv, gv, acc, mask, lane, nullptr, perm);
            e += 8;
        }
    }
    if constexpr (U > 4) {
        if (e + 4 <= e1) {
            edge_batch<ST, MODE, ACT, AGG, LPR, NV, VW, 4, MKB>(e, col, C, ldc, G, ldg, norm_col, nr, slope, li, HC, rv, gv, acc, mask, lane, nullptr, perm);
            e += 4;
        }
    }
    if constexpr (U > 2) {
        if (e + 2 <= e1) {
            edge_batch<ST, MODE, ACT, AGG, LPR, NV, VW, 2, MKB>(e, col, C, ldc, G, ldg, norm_col, nr, slope, li, HC, rv, gv, acc, mask, lane, nullptr, perm);
            e += 2;
        }
    }
    if (e < e1)
        edge_batch<ST, MODE, ACT, AGG, LPR, NV, VW, 1, MKB>(e, col, C, ldc, G, ldg, norm_col, nr, slope, li, HC, rv, gv, acc, mask, lane, nullptr, perm);

    if (slot < 0) {
        if constexpr (MODE == MODE_FWD && AGG == AGG_MEAN) {
            const int d = e1 - e0;                      // unsplit: the whole row
            const float degf = (float)(d > 1 ? d : 1);
#pragma unroll
            for (int j = 0; j < NV; ++j)
#pragma unroll
                for (int w = 0; w < VW; ++w) acc[j][w] = acc[j][w] / degf;
        }
        auto* op = out + (int64_t)row * ldo;
        if constexpr (MODE != MODE_FWD) {
            if (drop.on()) {
#pragma unroll
                for (int j = 0; j < NV; ++j) drop_vec<ST, VW>(drop, row, (li + LPR * j) * VW, acc[j]);
            }
        } else {
            if constexpr (ACC) {    // segmented forward (sirgcn.dist): S[v] = S[v] + this segment's sum
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                    const int c = li + LPR * j;
                    if (c < HC) {
                        float prev[VW];
                        vload_row<ST, VW>(prev, op + c * VW);
#pragma unroll
                        for (int w = 0; w < VW; ++w) acc[j][w] = prev[w] + acc[j][w];
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = li + LPR * j;
            if (c < HC) vstore_row<ST, VW>(op + c * VW, acc[j]);
        }
    } else {
        float* pp = partial + (int64_t)slot * H;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = li + LPR * j;
            if (c < HC) vstore_part<VW>(pp + c * VW, acc[j]);
        }
    }
}

template <int ST, int MODE, int ACT, int AGG, int LPR, int NV, int VW, int U, int MK>
__global__ void __launch_bounds__(256)
k_edge(const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ perm,
       const int4* __restrict__ items, int64_t n_items,
       const typename Stor<ST>::T* __restrict__ R, int64_t ldr,
       const typename Stor<ST>::T* __restrict__ C, int64_t ldc,
       const typename Stor<ST>::T* __restrict__ G, int64_t ldg,
       const float* __restrict__ norm_row, const float* __restrict__ norm_col,
       float slope, int H,
       typename Stor<ST>::T* __restrict__ out, int64_t ldo, float* __restrict__ partial,
       typename Stor<ST>::T* __restrict__ Gm, int64_t ldgm, uint64_t* __restrict__ mask, Drop drop, int accumulate) {
    drop = drop_resolve(drop);
    int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if constexpr (LPR == 64) wave = __builtin_amdgcn_readfirstlane((int)wave);
    edge_wave<ST, MODE, ACT, AGG, LPR, NV, VW, U, MK>(wave, rowptr, col, perm, items, n_items, R, ldr, C, ldc, G, ldg,
                                                     norm_row, norm_col, slope, H, out, ldo, partial, Gm, ldgm, mask,
                                                     drop, accumulate);
}

// ------------------------------------------------------------------------------ sign-mask backward
// For sigma in {ReLU, LeakyReLU} sigma'(z) depends only on sign(z), which the forward stored as
// one bit per (edge, element) (k_edge<MODE_FWD, ..., MASKW>).  The backward then never
// re-gathers Q or K:
//   MODE_BWD_DST: dQ[v] = sum_e sel(bit, t_e), t_e = g[v] (* c_e)      -> reads only the mask
//   MODE_BWD_SRC: dK[u] = sum_e sel(bit, t_e), t_e = Gd[v] (* c_e)     -> one gathered row + mask
// with sel(bit, t) = bit ? t : t*slope (LeakyReLU) / 0 (ReLU): exactly dsig<ACT>(z, t), so the
// result is bit-identical to the recompute path.  Full-wave rows of float4 only (LPR = 64).
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Per-lane select by a wave-uniform 64-bit lane mask: lane l gets (m >> l) & 1 ? if1 : if0.
// A ballot word is exactly an EXEC-style lane mask, so it is v_cndmask's condition operand
// (one VALU op instead of shift/and/compare/select).  Pure asm: no memory, freely schedulable.
__device__ __forceinline__ float lane_select(uint64_t m, float if0, float if1) {
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(m));
    return r;
}

template <int ACT>
__device__ __forceinline__ float sel_mask(uint64_t m, float t, float slope) {
    if constexpr (ACT == ACT_RELU) return lane_select(m, 0.f, t);
    else return lane_select(m, t * slope, t);
}

#ifndef SIR_DK_PF
#define SIR_DK_PF 1             // dK pass: the next batch's col / perm indices loaded with the current batch's rows
#endif

// wave-uniform (scalar) edge indices of one batch: source / destination id and dst-CSR position
template <int UU> struct EdgeIdx { int v[UU]; int p[UU]; };
#ifndef SIR_DQ_VMASK
#define SIR_DQ_VMASK 1          // dQ pass: mask words by one vector load + v_readlane (1; -9% sum, -19% sym) or scalar loads (0)
#endif

template <int ST, int MODE, int ACT, int AGG, int NV, int UU, bool PRE = false, bool PIDX = false>
__device__ __forceinline__ void mask_batch(int e, const int* __restrict__ col, const int* __restrict__ perm,
                                           const typename Stor<ST>::T* __restrict__ G, int64_t ldg,
                                           const uint64_t* __restrict__ mask,
                                           const float* __restrict__ norm_col, float nr, float slope,
                                           int lane, int HC, const float (&gv)[NV][4], float (&acc)[NV][4],
                                           uint64_t pre = 0, int pre_lane = 0, float cfw = 0.f, int cf_lane = 0,
                                           const EdgeIdx<UU>* idx = nullptr) {
    constexpr int NW = NV * 4;
    int p[UU];
    int v[UU];
#pragma unroll
    for (int i = 0; i < UU; ++i) {
        if constexpr (MODE == MODE_BWD_SRC && PIDX) {
            v[i] = idx->v[i];
            p[i] = idx->p[i];
        } else if constexpr (MODE == MODE_BWD_SRC) {
            v[i] = __builtin_amdgcn_readfirstlane(col[e + i]);
            p[i] = __builtin_amdgcn_readfirstlane(perm[e + i]);
        } else {
            p[i] = e + i;
            if constexpr (AGG == AGG_SYM && !PRE) v[i] = __builtin_amdgcn_readfirstlane(col[e + i]);
        }
    }
    uint64_t wd[UU][NW];
    if constexpr (PRE) {
        // words already in registers (one per lane, prefetched by mask_item_dst): edge e's word
        // k is in lane pre_lane + i*NW + k
        const int mlo = (int)(uint32_t)pre, mhi = (int)(uint32_t)(pre >> 32);
#pragma unroll
        for (int i = 0; i < UU; ++i)
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(mlo, pre_lane + i * NW + k);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane(mhi, pre_lane + i * NW + k);
                wd[i][k] = ((uint64_t)hi << 32) | lo;
            }
    } else if constexpr (SIR_DQ_VMASK && MODE == MODE_BWD_DST && UU * NW <= 64) {
        // the batch's UU*NW words are contiguous: one 8-B vector load per lane, then broadcast
        // each word to SGPRs (v_readlane) for the lane-mask selects
        const uint64_t mv = (lane < UU * NW) ? mask[(int64_t)e * NW + lane] : 0ull;
        const int mlo = (int)(uint32_t)mv, mhi = (int)(uint32_t)(mv >> 32);
#pragma unroll
        for (int i = 0; i < UU; ++i)
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(mlo, i * NW + k);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane(mhi, i * NW + k);
                wd[i][k] = ((uint64_t)hi << 32) | lo;
            }
    } else {
#pragma unroll
    for (int i = 0; i < UU; ++i)
#pragma unroll
        for (int k = 0; k < NW; ++k) wd[i][k] = uniform64(mask[(int64_t)p[i] * NW + k]);
    }
    float cf[UU];
    if constexpr (AGG == AGG_SYM && PRE) {
        // norms already gathered one per lane (mask_item_dst_wide): edge e+i's in lane cf_lane + i
#pragma unroll
        for (int i = 0; i < UU; ++i)
            cf[i] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cfw), cf_lane + i)) * nr;
    } else if constexpr (AGG == AGG_SYM) {
#pragma unroll
        for (int i = 0; i < UU; ++i) cf[i] = norm_col[v[i]] * nr;
    }
    float gc[(MODE == MODE_BWD_SRC) ? UU : 1][NV][4];
    if constexpr (MODE == MODE_BWD_SRC) {
#pragma unroll
        for (int i = 0; i < UU; ++i) {
            const auto* gp = G + (int64_t)v[i] * ldg;
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                const int c = lane + 64 * j;
                vload_gather<ST, 4>(gc[i][j], gp + (c < HC ? c : 0) * 4);   // unconditional (see edge_batch)
            }
        }
    }
#pragma unroll
    for (int i = 0; i < UU; ++i) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = lane + 64 * j;
            if (c < HC) {
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    float t;
                    if constexpr (MODE == MODE_BWD_SRC) t = gc[i][j][w];
                    else t = gv[j][w];
                    if constexpr (AGG == AGG_SYM) t = t * cf[i];
                    acc[j][w] += sel_mask<ACT>(wd[i][j * 4 + w], t, slope);
                }
            }
        }
    }
}

// The edge loop of one item (UNROLL-edge batches, then a binary tail).
template <int ST, int MODE, int ACT, int AGG, int NV, int U>
__device__ __forceinline__ void mask_item(int e0, int e1, const int* __restrict__ col, const int* __restrict__ perm,
                                          const typename Stor<ST>::T* __restrict__ G, int64_t ldg,
                                          const uint64_t* __restrict__ mask,
                                          const float* __restrict__ norm_col, float nr, float slope,
                                          int lane, int HC, const float (&gv)[NV][4], float (&acc)[NV][4]) {
    int e = e0;
    if constexpr (SIR_DK_PF && MODE == MODE_BWD_SRC) {
        // software-pipelined indices: the next batch's col / perm are fetched by one per-lane
        // vector load (lane i < U: edge eb + i, clamped to the item) issued with the current
        // batch's mask words and rows, and moved to SGPRs by v_readlane when the batch starts; a
        // batch then costs one memory latency instead of two (index load, then the gathers), and
        // the prefetched indices hold 2 VGPRs instead of 2U SGPRs
        if (e + U <= e1) {
            auto load_idx = [&](int eb, int& vc, int& pc) {
                const int q0 = eb + (lane < U ? lane : 0);
                const int q = q0 < e1 ? q0 : e1 - 1;
                vc = col[q];
                pc = perm[q];
            };
            int vc, pc;
            load_idx(e, vc, pc);
            for (; e + U <= e1; e += U) {
                EdgeIdx<U> cur;
#pragma unroll
                for (int i = 0; i < U; ++i) {
                    cur.v[i] = __builtin_amdgcn_readlane(vc, i);
                    cur.p[i] = __builtin_amdgcn_readlane(pc, i);
                }
                load_idx(e + U, vc, pc);
                mask_batch<ST, MODE, ACT, AGG, NV, U, false, true>(e, col, perm, G, ldg, mask, norm_col, nr, slope, lane,
                                                                   HC, gv, acc, 0, 0, 0.f, 0, &cur);
            }
        }
    } else {
        for (; e + U <= e1; e += U)
            mask_batch<ST, MODE, ACT, AGG, NV, U>(e, col, perm, G, ldg, mask, norm_col, nr, slope, lane, HC, gv, acc);
    }
    if constexpr (U > 8) {
        if (e + 8 <= e1) {
            mask_batch<ST, MODE, ACT, AGG, NV, 8>(e, col, perm, G, ldg, mask, norm_col, nr, slope, lane, HC, gv, acc);
            e += 8;
        }
    }
    if constexpr (U > 4) {
        if (e + 4 <= e1) {
            mask_batch<ST, MODE, ACT, AGG, NV, 4>(e, col, perm, G, ldg, mask, norm_col, nr, slope, lane, HC, gv, acc);
            e += 4;
        }
    }
    if constexpr (U > 2) {
        if (e + 2 <= e1) {
            mask_batch<ST, MODE, ACT, AGG, NV, 2>(e, col, perm, G, ldg, mask, norm_col, nr, slope, lane, HC, gv, acc);
            e += 2;
        }
    }
    if (e < e1)
        mask_batch<ST, MODE, ACT, AGG, NV, 1>(e, col, perm, G, ldg, mask, norm_col, nr, slope, lane, HC, gv, acc);
}

#ifndef SIR_DQ_PF
#define SIR_DQ_PF 1             // dQ pass: next batch's mask words loaded before the current batch is summed
#endif

// dQ pass (no col/perm reads for sum/mean): the mask words of the NEXT U-edge batch are loaded
// while the current batch is summed, so a wave no longer waits one memory latency per batch.
// A full batch is loaded whole; the row's final partial batch (and a row shorter than U) is
// loaded lane-guarded, so no load leaves the row.  Every batch's words start at lane 0, so the
// readlane lane indices are compile-time constants (a runtime lane index costs ~20%); the final
// partial batch is summed edge by edge under uniform guards.
template <int ST, int ACT, int AGG, int NV, int U>
__device__ __forceinline__ void mask_item_dst(int e0, int e1, const int* __restrict__ col,
                                              const uint64_t* __restrict__ mask,
                                              const float* __restrict__ norm_col, float nr, float slope,
                                              int lane, int HC, const float (&gv)[NV][4], float (&acc)[NV][4]) {
    constexpr int NW = NV * 4, BW = U * NW;       // words per edge, per batch (BW <= 64)
    const int wl = lane % BW;
    auto load_batch = [&](int eb) -> uint64_t {
        const int n = e1 - eb;
        if (n >= U) return mask[(int64_t)eb * NW + wl];
        return (lane < n * NW) ? mask[(int64_t)eb * NW + lane] : 0ull;
    };
    uint64_t cur = load_batch(e0);
    int e = e0;
    for (; e + U <= e1; e += U) {
        const uint64_t nxt = load_batch(e + U);
        mask_batch<ST, MODE_BWD_DST, ACT, AGG, NV, U, true>(e, col, nullptr, nullptr, 0, mask, norm_col, nr, slope,
                                                        lane, HC, gv, acc, cur, 0);
        cur = nxt;
    }
    const int r = e1 - e;                         // 0 .. U-1 edges left, their words in cur
#pragma unroll
    for (int i = 0; i < U - 1; ++i)
        if (i < r)
            mask_batch<ST, MODE_BWD_DST, ACT, AGG, NV, 1, true>(e + i, col, nullptr, nullptr, 0, mask, norm_col, nr,
                                                            slope, lane, HC, gv, acc, cur, i * NW);
}

#ifndef SIR_DQ_WIDE
#define SIR_DQ_WIDE 1           // dQ pass: a whole wave of mask words per load (mask_item_dst_wide)
#endif

// dQ pass, wide form: the per-batch loads of mask_item_dst leave a wave one U-edge batch (U*NW*8 B)
// in flight, so a row of ~20 edges costs ~4 serial memory latencies and the pass is latency-bound.
// Here every load fetches a full chunk of CH = 64/NW edges (all 64 lanes: 512 B for H = 256), the
// row's first two chunks are loaded together and the next chunk is in flight while one is summed (a
// row of <= 2*CH edges costs one latency); a chunk is summed in SB-edge sub-batches
// (compile-time readlane lanes, SB*NW word pairs of SGPRs).  Same per-column edge order as
// mask_item_dst, so the sums are bit-identical.
template <int ST, int ACT, int AGG, int NV>
__device__ __forceinline__ void mask_item_dst_wide(int e0, int e1, const int* __restrict__ col,
                                                   const uint64_t* __restrict__ mask,
                                                   const float* __restrict__ norm_col, float nr, float slope, int lane,
                                                   int HC, const float (&gv)[NV][4], float (&acc)[NV][4]) {
    constexpr int NW = NV * 4, CH = 64 / NW, SB = (NV == 1) ? 4 : (NV == 2 ? 2 : 1);
    static_assert(CH % SB == 0, "sub-batches tile a chunk");
    constexpr bool kSym = (AGG == AGG_SYM);
    if (e0 >= e1) return;
    // Loads are unconditional (lanes past the row re-read edge e0's first word, whose value is never
    // used): a lane-guarded load compiles to a branch that may skip it, and the compiler then waits
    // for every outstanding load (vmcnt(0)) instead of the oldest chunk only.
    auto load_chunk = [&](int eb) -> uint64_t {
        const int n = e1 - eb;
        const int lim = (n >= CH ? CH : n) * NW;
        return mask[(lane < lim) ? (int64_t)eb * NW + lane : (int64_t)e0 * NW];
    };
    // SYM: lane i < CH also fetches the chunk's edge i source id, then its norm (one gather per chunk
    // instead of two dependent scalar loads per edge); the norm of the next chunk is gathered while
    // the current one is summed
    auto load_col = [&](int eb) -> int {
        const int n = e1 - eb;
        return col[(lane < (n >= CH ? CH : n)) ? eb + lane : e0];
    };
    auto gather_norm = [&](int c) -> float { return norm_col[c]; };
    auto full = [&](uint64_t c, int eb, float f) {
#pragma unroll
        for (int s = 0; s < CH / SB; ++s)
            mask_batch<ST, MODE_BWD_DST, ACT, AGG, NV, SB, true>(eb + s * SB, nullptr, nullptr, nullptr, 0, mask,
                                                                 nullptr, nr, slope, lane, HC, gv, acc, c, s * SB * NW,
                                                                 f, s * SB);
    };
    auto tail = [&](uint64_t c, int eb, float f) {   // 0 .. CH-1 edges
        const int r = e1 - eb;
#pragma unroll
        for (int i = 0; i < CH - 1; ++i)
            if (i < r)
                mask_batch<ST, MODE_BWD_DST, ACT, AGG, NV, 1, true>(eb + i, nullptr, nullptr, nullptr, 0, mask, nullptr,
                                                                nr, slope, lane, HC, gv, acc, c, i * NW, f, i);
    };
    // chunk registers a / b alternate roles in a loop unrolled by two over the row's full chunks (a
    // register copy of a value still being loaded would make the compiler wait for that load)
    const int nfull = (e1 - e0) / CH;
    uint64_t ca = load_chunk(e0);
    int ka = 0, kb = 0;
    if constexpr (kSym) ka = load_col(e0);
    uint64_t cb = load_chunk(e0 + CH);
    if constexpr (kSym) kb = load_col(e0 + CH);
    float fa = 0.f, fb = 0.f;
    if constexpr (kSym) fa = gather_norm(ka);
    int e = e0;
    for (int k = 2; k <= nfull; k += 2) {
        full(ca, e, fa);
        if constexpr (kSym) fb = gather_norm(kb);
        ca = load_chunk(e + 2 * CH);
        if constexpr (kSym) ka = load_col(e + 2 * CH);
        full(cb, e + CH, fb);
        if constexpr (kSym) fa = gather_norm(ka);
        cb = load_chunk(e + 3 * CH);
        if constexpr (kSym) kb = load_col(e + 3 * CH);
        e += 2 * CH;
    }
    if (nfull & 1) {
        full(ca, e, fa);
        if constexpr (kSym) fb = gather_norm(kb);
        tail(cb, e + CH, fb);
    } else {
        tail(ca, e, fa);
    }
}

#ifndef SIR_DQ_SMEM
#define SIR_DQ_SMEM 0           // 1: dQ pass (sum / mean, H <= 256) mask words by prefetched scalar loads (+13 %: rejected, profiles/r02_ab_dq_smem2.txt)
#endif

// dQ pass, scalar form (sum / mean, NV = 1: 4 words per edge): the mask words of a 4-edge
// sub-batch (128 B, contiguous) come by two s_load_dwordx16 straight into SGPRs — the selects'
// lane-mask operands — so no v_readlane is needed (8 per edge in the vector forms: the pass was
// VALU-bound on them).  Scalar loads may return out of order (one lgkmcnt for all), so the next
// sub-batch's loads are issued only after the current one's words have arrived, then overlap
// its selects and adds.  Same per-column edge order as the other forms: bit-identical.
template <int ST, int ACT, int AGG>
__device__ __forceinline__ void mask_item_dst_smem(int e0, int e1, const uint64_t* __restrict__ mask, float slope,
                                                   int HC, int lane, const float (&gv)[1][4], float (&acc)[1][4]) {
    struct W16 { uint64_t w[16]; };
    auto load = [&](int eb) {
        W16 x;
        const uint64_t* p = mask + (int64_t)__builtin_amdgcn_readfirstlane(eb) * 4;
#pragma unroll
        for (int k = 0; k < 16; ++k) x.w[k] = p[k];
        return x;
    };
    auto arrived = [&](const W16& x) {       // wait for x (and nothing else is in flight)
#pragma unroll
        for (int k = 0; k < 16; ++k) asm volatile("" :: "s"(x.w[k]) : "memory");
    };
    const bool ok = lane < HC;
    auto compute = [&](const W16& x, int n) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i < n && ok) {
#pragma unroll
                for (int w = 0; w < 4; ++w) acc[0][w] += sel_mask<ACT>(x.w[4 * i + w], gv[0][w], slope);
            }
        }
    };
    int e = e0;
    if (e + 4 <= e1) {
        W16 a = load(e);
        for (; e + 8 <= e1; e += 8) {
            arrived(a);
            const W16 b = load(e + 4);
            compute(a, 4);
            arrived(b);
            if (e + 12 <= e1) a = load(e + 8);
            compute(b, 4);
        }
        if (e + 4 <= e1) {
            arrived(a);
            compute(a, 4);
            e += 4;
        }
    }
    for (; e < e1; ++e) {                    // 0 .. 3 edges
        uint64_t wd[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) wd[k] = uniform64(mask[(int64_t)e * 4 + k]);
        if (ok) {
#pragma unroll
            for (int w = 0; w < 4; ++w) acc[0][w] += sel_mask<ACT>(wd[w], gv[0][w], slope);
        }
    }
}

__device__ __forceinline__ int4 uniform_item(const int4* __restrict__ items, int64_t i) {
    int4 it = items[i];
    it.x = __builtin_amdgcn_readfirstlane(it.x);
    it.y = __builtin_amdgcn_readfirstlane(it.y);
    it.z = __builtin_amdgcn_readfirstlane(it.z);
    it.w = __builtin_amdgcn_readfirstlane(it.w);
    return it;
}

// One work item of a sign-mask backward pass (one wave).
template <int ST, int MODE, int ACT, int AGG, int NV, int U>
__device__ __forceinline__ void
mask_pass_item(int64_t wave, const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ perm,
               const int4* __restrict__ items,
               const typename Stor<ST>::T* __restrict__ G, int64_t ldg, const uint64_t* __restrict__ mask,
               const float* __restrict__ norm_row, const float* __restrict__ norm_col,
               float slope, int H, typename Stor<ST>::T* __restrict__ out, int64_t ldo, float* __restrict__ partial,
               typename Stor<ST>::T* __restrict__ Gm, int64_t ldgm, const Drop& drop) {
    const int lane = threadIdx.x & 63;
    const int4 it = uniform_item(items, wave);
    const int row = it.x, e0 = it.y, e1 = it.z, slot = it.w;
    const int HC = H / 4;
    float gv[NV][4];
    float acc[NV][4];
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int w = 0; w < 4; ++w) { acc[j][w] = 0.f; gv[j][w] = 0.f; }
    if constexpr (MODE == MODE_BWD_DST) {
        const auto* gp = G + (int64_t)row * ldg;
        float degf = 1.f;
        bool first = true;
        if constexpr (AGG == AGG_MEAN) {
            const int rs = rowptr[row];
            const int d = rowptr[row + 1] - rs;
            degf = (float)(d > 1 ? d : 1);
            first = (e0 == rs);
        }
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = lane + 64 * j;
            if (c < HC) {
                vload_row<ST, 4>(gv[j], gp + c * 4);
                if constexpr (AGG == AGG_MEAN) {
#pragma unroll
                    for (int w = 0; w < 4; ++w) gv[j][w] = round_st<ST>(gv[j][w] / degf);
                    if (Gm != nullptr && first) vstore_row<ST, 4>(Gm + (int64_t)row * ldgm + c * 4, gv[j]);
                }
            }
        }
    }
    float nr = 1.f;
    if constexpr (AGG == AGG_SYM) nr = norm_row[row];
    if constexpr (SIR_DQ_SMEM && MODE == MODE_BWD_DST && AGG != AGG_SYM && NV == 1)
        mask_item_dst_smem<ST, ACT, AGG>(e0, e1, mask, slope, HC, lane, gv, acc);
    else if constexpr (SIR_DQ_WIDE && MODE == MODE_BWD_DST)
        mask_item_dst_wide<ST, ACT, AGG, NV>(e0, e1, col, mask, norm_col, nr, slope, lane, HC, gv, acc);
    else if constexpr (SIR_DQ_PF && MODE == MODE_BWD_DST && AGG != AGG_SYM && U * NV * 4 <= 64)
        mask_item_dst<ST, ACT, AGG, NV, U>(e0, e1, col, mask, norm_col, nr, slope, lane, HC, gv, acc);
    else
        mask_item<ST, MODE, ACT, AGG, NV, U>(e0, e1, col, perm, G, ldg, mask, norm_col, nr, slope, lane, HC, gv, acc);
    if (slot < 0) {
        auto* op = out + (int64_t)row * ldo;
        if (drop.on()) {
#pragma unroll
            for (int j = 0; j < NV; ++j) drop_vec<ST, 4>(drop, row, (lane + 64 * j) * 4, acc[j]);
        }
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = lane + 64 * j;
            if (c < HC) vstore_row<ST, 4>(op + c * 4, acc[j]);
        }
    } else {
        float* op = partial + (int64_t)slot * H;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = lane + 64 * j;
            if (c < HC) vstore_part<4>(op + c * 4, acc[j]);
        }
    }
}

template <int ST, int MODE, int ACT, int AGG, int NV, int U>
__global__ void __launch_bounds__(256)
k_edge_mask(const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ perm,
            const int4* __restrict__ items, int64_t n_items,
            const typename Stor<ST>::T* __restrict__ G, int64_t ldg, const uint64_t* __restrict__ mask,
            const float* __restrict__ norm_row, const float* __restrict__ norm_col,
            float slope, int H, typename Stor<ST>::T* __restrict__ out, int64_t ldo, float* __restrict__ partial,
            typename Stor<ST>::T* __restrict__ Gm, int64_t ldgm, Drop drop) {
    drop = drop_resolve(drop);
    const int64_t wave = __builtin_amdgcn_readfirstlane((int)((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
    if (wave >= n_items) return;
    mask_pass_item<ST, MODE, ACT, AGG, NV, U>(wave, rowptr, col, perm, items, G, ldg, mask, norm_row, norm_col, slope, H,
                                              out, ldo, partial, Gm, ldgm, drop);
}

#ifndef SIR_DUAL_PRIO
#define SIR_DUAL_PRIO 0         // one-launch backward wave priority: 1 = dK waves first, 2 = dQ waves first
#endif
// Both sign-mask backward passes in ONE launch (SUM / SYM: the dK pass does not need the dQ pass's
// Gm).  The dQ pass is VALU-bound (v_readlane + select + add per element and edge) and reads 32 B
// per edge; the dK pass is HBM-bound (one gathered G row per edge).  Interleaving their waves
// (even waves dQ items, odd waves dK items, then the rest of the larger set) puts both kinds on
// every CU at once, so the dQ pass's VALU work hides under the dK pass's memory time instead of
// running as a separate launch.  Each wave still runs exactly the single-pass code, so results are
// bit-identical to the two launches.
// DR: a dropout seed lives in device memory (drop_resolve at the start); a separate instantiation —
// the resolve code alone made the SYM one-launch backward 5 % slower (profiles/r04_ab_devseed.txt)
template <int ST, int ACT, int AGG, int NV, int UD, int US, bool DR>
__global__ void __launch_bounds__(256)
k_edge_mask_dual(const int* __restrict__ rowptr, const int* __restrict__ col, const int4* __restrict__ items,
                 int64_t n_items, float* __restrict__ partial, typename Stor<ST>::T* __restrict__ dQ, int64_t lddq,
                 const int* __restrict__ rowptr_s, const int* __restrict__ col_s, const int* __restrict__ perm_s,
                 const int4* __restrict__ items_s, int64_t n_items_s, float* __restrict__ partial_s,
                 typename Stor<ST>::T* __restrict__ dK, int64_t lddk,
                 const typename Stor<ST>::T* __restrict__ G, int64_t ldg, const uint64_t* __restrict__ mask,
                 const float* __restrict__ in_norm, const float* __restrict__ out_norm, float slope, int H,
                 Drop drop_q, Drop drop_k) {
    if constexpr (DR) {
        drop_q = drop_resolve(drop_q);
        drop_k = drop_resolve(drop_k);
    }
    const int64_t w = __builtin_amdgcn_readfirstlane((int)((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
    const int64_t nmin = n_items < n_items_s ? n_items : n_items_s;
    bool dst;
    int64_t idx;
    if (w < 2 * nmin) {
        dst = (w & 1) == 0;
        idx = w >> 1;
    } else {
        dst = n_items > n_items_s;
        idx = nmin + (w - 2 * nmin);
        if (idx >= (dst ? n_items : n_items_s)) return;
    }
#if SIR_DUAL_PRIO == 1
    if (!dst) __builtin_amdgcn_s_setprio(1);       // dK waves (memory-bound) issue first
#elif SIR_DUAL_PRIO == 2
    if (dst) __builtin_amdgcn_s_setprio(1);        // dQ waves (VALU-bound) issue first
#endif
    if (dst)
        mask_pass_item<ST, MODE_BWD_DST, ACT, AGG, NV, UD>(idx, rowptr, col, nullptr, items, G, ldg, mask, in_norm,
                                                           out_norm, slope, H, dQ, lddq, partial, nullptr, H, drop_q);
    else
        mask_pass_item<ST, MODE_BWD_SRC, ACT, AGG, NV, US>(idx, rowptr_s, col_s, perm_s, items_s, G, ldg, mask,
                                                           out_norm, in_norm, slope, H, dK, lddk, partial_s, nullptr, H,
                                                           drop_k);
}

#ifndef SIR_COMBINE_PF
#define SIR_COMBINE_PF 4        // partial rows in flight per thread in k_combine (8: +0..1 %, rejected)
#endif
// Combine the partial rows of split rows (deterministic, no atomics).  One 1024-thread block
// per split row: threads cover the row's columns (VW floats each); the remaining thread
// dimension takes slices of the partial slots (slot s -> slice s % nslice, SIR_COMBINE_PF
// loads in flight); the slices are added in slice order through LDS.  MEAN_DIV divides by the degree.
template <int ST, bool MEAN_DIV, int VW>
__global__ void __launch_bounds__(1024)
k_combine(const int4* __restrict__ splits, const float* __restrict__ partial,
          int H, typename Stor<ST>::T* __restrict__ out, int64_t ldo, Drop drop, int accumulate) {
    drop = drop_resolve(drop);
    __shared__ float red[1024 * VW];
    const int4 sp = splits[blockIdx.x];
    const int HC = H / VW;
    const int cols = HC < 1024 ? HC : 1024;
    const int nslice = 1024 / cols;
    const int t = threadIdx.x;
    const int slice = t / cols;
    const float degf = (float)(sp.w > 1 ? sp.w : 1);
    for (int c0 = 0; c0 < HC; c0 += cols) {
        const int c = c0 + (t % cols);
        float acc[VW];
#pragma unroll
        for (int w = 0; w < VW; ++w) acc[w] = 0.f;
        if (slice < nslice && c < HC) {
            const float* base = partial + (int64_t)sp.y * H + c * VW;
            int s = slice;
            for (; s + (SIR_COMBINE_PF - 1) * nslice < sp.z; s += SIR_COMBINE_PF * nslice) {
                float v[SIR_COMBINE_PF][VW];
#pragma unroll
                for (int i = 0; i < SIR_COMBINE_PF; ++i) vload<VW>(v[i], base + (int64_t)(s + i * nslice) * H);
#pragma unroll
                for (int i = 0; i < SIR_COMBINE_PF; ++i)
#pragma unroll
                    for (int w = 0; w < VW; ++w) acc[w] += v[i][w];
            }
            for (; s < sp.z; s += nslice) {
                float v[VW];
                vload<VW>(v, base + (int64_t)s * H);
#pragma unroll
                for (int w = 0; w < VW; ++w) acc[w] += v[w];
            }
        }
#pragma unroll
        for (int w = 0; w < VW; ++w) red[t * VW + w] = acc[w];
        __syncthreads();
        if (t < cols && c < HC) {
            float r[VW];
#pragma unroll
            for (int w = 0; w < VW; ++w) r[w] = red[t * VW + w];
            for (int k = 1; k < nslice; ++k)
#pragma unroll
                for (int w = 0; w < VW; ++w) r[w] += red[(k * cols + t) * VW + w];
            if constexpr (MEAN_DIV) {
#pragma unroll
                for (int w = 0; w < VW; ++w) r[w] = r[w] / degf;
            }
            if (drop.on()) drop_vec<ST, VW>(drop, sp.x, c * VW, r);      // backward passes only (host)
            if (accumulate) {           // segmented forward: prior S row + this segment's sum
                float prev[VW];
                tload_p<ST, VW, false>(prev, out + (int64_t)sp.x * ldo + c * VW);
#pragma unroll
                for (int w = 0; w < VW; ++w) r[w] = prev[w] + r[w];
            }
            tstore_p<ST, VW, false>(out + (int64_t)sp.x * ldo + c * VW, r);
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------ per-mode launch
// Gathered rows in flight per wave for NV == 1 shapes, per pass (A/B-tuned on MI355X with
// tools/edge_ab.py: more rows in flight per wave than this only adds cache pressure).
#ifndef SIR_UNROLL_FWD
#define SIR_UNROLL_FWD 6         // with the buffer-load gathers + col prefetch: S2 forward 5.86 -> 5.61 ms (profiles/r02_ab_unroll_fwd.txt)
#endif
#ifndef SIR_UNROLL_DST
#define SIR_UNROLL_DST 6
#endif
#ifndef SIR_UNROLL_SRC
#define SIR_UNROLL_SRC 8
#endif
// 16-bit storage (A/B on MI355X, profiles/r02_ab_dq_smem_unroll.txt: twice the rows in flight per
// wave made the bf16 passes 17-40% slower, like fp32 UNROLL 8 in round 1)
#ifndef SIR_UNROLL_FWD_H
#define SIR_UNROLL_FWD_H 4
#endif
#ifndef SIR_UNROLL_DST_H
#define SIR_UNROLL_DST_H 6
#endif
#ifndef SIR_UNROLL_SRC_H
#define SIR_UNROLL_SRC_H 4       // with the prefetched indices: one-launch bf16 backward 5.50 -> 4.86 ms (profiles/r02_ab_unroll_src.txt)
#endif
#if SIR_UNROLL_FWD > 16 || SIR_UNROLL_DST > 16 || SIR_UNROLL_SRC > 16 || SIR_UNROLL_FWD_H > 16 || \
    SIR_UNROLL_DST_H > 16 || SIR_UNROLL_SRC_H > 16
#error "unroll must be <= 16 (the tail covers < 16 edges)"
#endif
template <int MODE, int ST>
constexpr int unroll_of() {
    if constexpr (ST == ST_F32)
        return MODE == MODE_FWD ? SIR_UNROLL_FWD : (MODE == MODE_BWD_DST ? SIR_UNROLL_DST : SIR_UNROLL_SRC);
    else
        return MODE == MODE_FWD ? SIR_UNROLL_FWD_H : (MODE == MODE_BWD_DST ? SIR_UNROLL_DST_H : SIR_UNROLL_SRC_H);
}

template <int ST> using TP = typename Stor<ST>::T;
template <int ST> __host__ inline const TP<ST>* cp_(const void* p) { return static_cast<const TP<ST>*>(p); }
template <int ST> __host__ inline TP<ST>* mp_(void* p) { return static_cast<TP<ST>*>(p); }

template <int ST, int MODE, int ACT, int AGG, int LPR, int NV, int VW>
static hipError_t launch_edge_t(const EdgeArgs& a, hipStream_t st) {
    constexpr int U = (NV == 1) ? unroll_of<MODE, ST>() : 4;
    constexpr int RPW = 64 / LPR;
    const int64_t waves = (a.n_items + RPW - 1) / RPW;
    const int64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    constexpr bool kReluFamily = (ACT == ACT_RELU || ACT == ACT_LEAKY) && VW == 4 && (LPR == 64 || NV == 1);
    constexpr bool kMaskable = (MODE == MODE_FWD) && kReluFamily;
    if constexpr (kMaskable) {
        if (a.mask_out != nullptr) {
#define SIR_EDGE_FWD_MASK(MKV)                                                                                       \
            hipLaunchKernelGGL((k_edge<ST, MODE, ACT, AGG, LPR, NV, VW, U, MKV>), dim3((unsigned)blocks), dim3(256), 0,   \
                               st, a.rowptr, a.col, nullptr, reinterpret_cast<const int4*>(a.items), a.n_items,        \
                               cp_<ST>(a.R), a.ldr, cp_<ST>(a.C), a.ldc, cp_<ST>(a.G), a.ldg, a.norm_row, a.norm_col,  \
                               a.slope, a.H, mp_<ST>(a.out), a.ldo, a.partial, mp_<ST>(a.Gm), a.ldgm, a.mask_out,      \
                               a.drop, a.accumulate)
            if (a.accumulate) SIR_EDGE_FWD_MASK(1 | 4);
            else SIR_EDGE_FWD_MASK(1);
#undef SIR_EDGE_FWD_MASK
            return hipGetLastError();
        }
    } else {
        if (a.mask_out != nullptr) return hipErrorInvalidValue;
    }
    if constexpr (MODE != MODE_FWD && kReluFamily && LPR < 64) {
        if (a.mask_in != nullptr) {          // sub-wave rows, sign-mask backward
            hipLaunchKernelGGL((k_edge<ST, MODE, ACT, AGG, LPR, NV, VW, U, 2>), dim3((unsigned)blocks), dim3(256), 0, st,
                               a.rowptr, a.col, a.perm, reinterpret_cast<const int4*>(a.items), a.n_items,
                               cp_<ST>(a.R), a.ldr, cp_<ST>(a.C), a.ldc, cp_<ST>(a.G), a.ldg, a.norm_row, a.norm_col,
                               a.slope, a.H, mp_<ST>(a.out), a.ldo, a.partial, mp_<ST>(a.Gm), a.ldgm,
                               const_cast<uint64_t*>(a.mask_in), a.drop, 0);
            return hipGetLastError();
        }
    }
    if (a.mask_in != nullptr) return hipErrorInvalidValue;
#define SIR_EDGE_PLAIN(MKV)                                                                                           \
    hipLaunchKernelGGL((k_edge<ST, MODE, ACT, AGG, LPR, NV, VW, U, MKV>), dim3((unsigned)blocks), dim3(256), 0, st,   \
                       a.rowptr, a.col, nullptr, reinterpret_cast<const int4*>(a.items), a.n_items,                   \
                       cp_<ST>(a.R), a.ldr, cp_<ST>(a.C), a.ldc, cp_<ST>(a.G), a.ldg, a.norm_row, a.norm_col,         \
                       a.slope, a.H, mp_<ST>(a.out), a.ldo, a.partial, mp_<ST>(a.Gm), a.ldgm, nullptr, a.drop,        \
                       a.accumulate)
    if constexpr (MODE == MODE_FWD) {
        if (a.accumulate) SIR_EDGE_PLAIN(4);
        else SIR_EDGE_PLAIN(0);
    } else {
        SIR_EDGE_PLAIN(0);
    }
#undef SIR_EDGE_PLAIN
    return hipGetLastError();
}

template <int ST, int MODE, int ACT, int AGG, int NV>
static hipError_t launch_mask_t(const EdgeArgs& a, hipStream_t st) {
    constexpr int U = (NV == 1) ? unroll_of<MODE, ST>() : (NV == 2 ? 4 : 2);
    const int64_t blocks = (a.n_items + 3) / 4;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL((k_edge_mask<ST, MODE, ACT, AGG, NV, U>), dim3((unsigned)blocks), dim3(256), 0, st,
                       a.rowptr, a.col, a.perm, reinterpret_cast<const int4*>(a.items), a.n_items,
                       cp_<ST>(a.G), a.ldg, a.mask_in, a.norm_row, a.norm_col, a.slope, a.H,
                       mp_<ST>(a.out), a.ldo, a.partial, mp_<ST>(a.Gm), a.ldgm, a.drop);
    return hipGetLastError();
}

// a: the destination pass (dQ), b: the source pass (dK); mask mode, SUM / SYM
template <int ST, int ACT, int AGG, int NV>
static hipError_t launch_dual_t(const EdgeArgs& a, const EdgeArgs& b, hipStream_t st) {
    constexpr int UD = (NV == 1) ? unroll_of<MODE_BWD_DST, ST>() : (NV == 2 ? 4 : 2);
    constexpr int US = (NV == 1) ? unroll_of<MODE_BWD_SRC, ST>() : (NV == 2 ? 4 : 2);
    const int64_t blocks = (a.n_items + b.n_items + 3) / 4;
    if (blocks == 0) return hipSuccess;
#define SIR_DUAL(DRV)                                                                                               \
    hipLaunchKernelGGL((k_edge_mask_dual<ST, ACT, AGG, NV, UD, US, DRV>), dim3((unsigned)blocks), dim3(256), 0, st,  \
                       a.rowptr, a.col, reinterpret_cast<const int4*>(a.items), a.n_items, a.partial,              \
                       mp_<ST>(a.out), a.ldo,                                                                      \
                       b.rowptr, b.col, b.perm, reinterpret_cast<const int4*>(b.items), b.n_items, b.partial,      \
                       mp_<ST>(b.out), b.ldo, cp_<ST>(a.G), a.ldg, a.mask_in, a.norm_row, a.norm_col, a.slope, a.H, \
                       a.drop, b.drop)
    if (a.drop.sptr != nullptr || b.drop.sptr != nullptr) SIR_DUAL(true);
    else SIR_DUAL(false);
#undef SIR_DUAL
    return hipGetLastError();
}

template <int ST, int ACT, int AGG>
static hipError_t launch_dual_shape(const EdgeArgs& a, const EdgeArgs& b, Shape s, hipStream_t st) {
    switch (s.nv) {
        case 1: return launch_dual_t<ST, ACT, AGG, 1>(a, b, st);
        case 2: return launch_dual_t<ST, ACT, AGG, 2>(a, b, st);
        case 3: return launch_dual_t<ST, ACT, AGG, 3>(a, b, st);
        default: return launch_dual_t<ST, ACT, AGG, 4>(a, b, st);
    }
}

template <int ST>
static hipError_t launch_edge_dual_st(const EdgeArgs& a, const EdgeArgs& b, int agg, int act, Shape s, hipStream_t st) {
    if (s.vw != 4 || (agg != AGG_SUM && agg != AGG_SYM) || (act != ACT_RELU && act != ACT_LEAKY))
        return hipErrorInvalidValue;
    if (s.lpr < 64) {
        // sub-wave rows: the two mask-read passes one after the other (one launch with the waves
        // interleaved, as for full-wave rows, measured 8 % slower on config 2's molecule batch: the
        // combined kernel's register budget lowers the occupancy of both latency-bound passes)
        hipError_t e2 = launch_edge_pass<ST, MODE_BWD_DST>(a, agg, act, s, st);
        if (e2 != hipSuccess) return e2;
        return launch_edge_pass<ST, MODE_BWD_SRC>(b, agg, act, s, st);
    }
    if (act == ACT_RELU)
        return agg == AGG_SUM ? launch_dual_shape<ST, ACT_RELU, AGG_SUM>(a, b, s, st)
                              : launch_dual_shape<ST, ACT_RELU, AGG_SYM>(a, b, s, st);
    return agg == AGG_SUM ? launch_dual_shape<ST, ACT_LEAKY, AGG_SUM>(a, b, s, st)
                          : launch_dual_shape<ST, ACT_LEAKY, AGG_SYM>(a, b, s, st);
}

template <int ST, int MODE, int ACT, int AGG>
static hipError_t launch_mask_shape(const EdgeArgs& a, Shape s, hipStream_t st) {
    switch (s.nv) {
        case 1: return launch_mask_t<ST, MODE, ACT, AGG, 1>(a, st);
        case 2: return launch_mask_t<ST, MODE, ACT, AGG, 2>(a, st);
        case 3: return launch_mask_t<ST, MODE, ACT, AGG, 3>(a, st);
        default: return launch_mask_t<ST, MODE, ACT, AGG, 4>(a, st);
    }
}

template <int ST, int MODE, int ACT, int AGG>
static hipError_t launch_edge_shape(const EdgeArgs& a, Shape s, hipStream_t st) {
    if constexpr (MODE != MODE_FWD && (ACT == ACT_RELU || ACT == ACT_LEAKY)) {
        if (a.mask_in != nullptr) {
            if (s.vw != 4) return hipErrorInvalidValue;
            if (s.lpr == 64) return launch_mask_shape<ST, MODE, ACT, AGG>(a, s, st);
            // sub-wave rows: k_edge in mask-read mode (below)
        }
    } else if constexpr (MODE != MODE_FWD) {
        if (a.mask_in != nullptr) return hipErrorInvalidValue;
    }
    if (s.vw == 4) {
        if (s.lpr == 4) return launch_edge_t<ST, MODE, ACT, AGG, 4, 1, 4>(a, st);
        if (s.lpr == 8) return launch_edge_t<ST, MODE, ACT, AGG, 8, 1, 4>(a, st);
        if (s.lpr == 16) return launch_edge_t<ST, MODE, ACT, AGG, 16, 1, 4>(a, st);
        if (s.lpr == 32) return launch_edge_t<ST, MODE, ACT, AGG, 32, 1, 4>(a, st);
        switch (s.nv) {
            case 1: return launch_edge_t<ST, MODE, ACT, AGG, 64, 1, 4>(a, st);
            case 2: return launch_edge_t<ST, MODE, ACT, AGG, 64, 2, 4>(a, st);
            case 3: return launch_edge_t<ST, MODE, ACT, AGG, 64, 3, 4>(a, st);
            default: return launch_edge_t<ST, MODE, ACT, AGG, 64, 4, 4>(a, st);
        }
    }
    if constexpr (ST != ST_F32) {
        return hipErrorInvalidValue;        // 16-bit storage: H % 4 == 0 and 8-B aligned rows only
    } else {
        switch (s.nv) {
            case 1: return launch_edge_t<ST, MODE, ACT, AGG, 64, 1, 1>(a, st);
            case 2: return launch_edge_t<ST, MODE, ACT, AGG, 64, 2, 1>(a, st);
            default: return launch_edge_t<ST, MODE, ACT, AGG, 64, 4, 1>(a, st);
        }
    }
}

template <int ST, int MODE, int ACT>
static hipError_t launch_edge_agg(const EdgeArgs& a, int agg, Shape s, hipStream_t st) {
    switch (agg) {
        case AGG_SUM: return launch_edge_shape<ST, MODE, ACT, AGG_SUM>(a, s, st);
        case AGG_MEAN: return launch_edge_shape<ST, MODE, ACT, AGG_MEAN>(a, s, st);
        default: return launch_edge_shape<ST, MODE, ACT, AGG_SYM>(a, s, st);
    }
}

template <int ST, int MODE>
static hipError_t launch_edge_mode(const EdgeArgs& a, int agg, int act, Shape s, hipStream_t st) {
    switch (act) {
        case ACT_IDENTITY: return launch_edge_agg<ST, MODE, ACT_IDENTITY>(a, agg, s, st);
        case ACT_RELU: return launch_edge_agg<ST, MODE, ACT_RELU>(a, agg, s, st);
        case ACT_LEAKY: return launch_edge_agg<ST, MODE, ACT_LEAKY>(a, agg, s, st);
        case ACT_GELU: return launch_edge_agg<ST, MODE, ACT_GELU>(a, agg, s, st);
        default: return launch_edge_agg<ST, MODE, ACT_GELU_TANH>(a, agg, s, st);
    }
}

}  // namespace sir
