// sirconv_kernels.hip — gfx950 (MI355X, CDNA4) edge-aggregation kernels for SIRConv.
//
// Reference path: briangodwinlim/SIR-GCN models/conv.py:43-45 (message UDF) + conv.py:63
// (graph.update_all -> DGL 2.1.0 gather + GSpMM copy_e/sum; autograd -> gsddmm + index_add).
//
// Design:
//  * Row-CSR, atomics-free.  A "row" is the node reduced INTO: dst for the forward and the dQ
//    pass, src for the dK pass.  One wave (or a 16/32-lane sub-wave when H is small) owns one
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

#include "sirconv_internal.h"

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

// ------------------------------------------------------------------------------ vectors
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

// ------------------------------------------------------------------------------ edge batch
// Processes UU consecutive edges [e, e+UU) of one row: all gathers issued before any use.
template <int MODE, int ACT, int AGG, int LPR, int NV, int VW, int UU>
__device__ __forceinline__ void edge_batch(int e, const int* __restrict__ col,
                                           const float* __restrict__ C, int64_t ldc,
                                           const float* __restrict__ G, int64_t ldg,
                                           const float* __restrict__ norm_col, float nr, float slope,
                                           int li, int HC,
                                           const float (&rv)[NV][VW], const float (&gv)[NV][VW],
                                           float (&acc)[NV][VW]) {
    int u[UU];
#pragma unroll
    for (int i = 0; i < UU; ++i) u[i] = col[e + i];
    float cf[UU];
    if constexpr (AGG == AGG_SYM) {
#pragma unroll
        for (int i = 0; i < UU; ++i) cf[i] = norm_col[u[i]] * nr;  // out_norm[u] * in_norm[v]
    }
    float cv[UU][NV][VW];
    float gc[(MODE == MODE_BWD_SRC) ? UU : 1][NV][VW];
#pragma unroll
    for (int i = 0; i < UU; ++i) {
        const float* cp = C + (int64_t)u[i] * ldc;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = li + LPR * j;
            if (NV == 1 || c < HC) vload<VW>(cv[i][j], cp + c * VW);
        }
        if constexpr (MODE == MODE_BWD_SRC) {
            const float* gp = G + (int64_t)u[i] * ldg;
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                const int c = li + LPR * j;
                if (NV == 1 || c < HC) vload<VW>(gc[i][j], gp + c * VW);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < UU; ++i) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = li + LPR * j;
            if (NV == 1 || c < HC) {
#pragma unroll
                for (int w = 0; w < VW; ++w) {
                    if constexpr (MODE == MODE_FWD) {
                        const float z = rv[j][w] + cv[i][j][w];        // eq[v] + ek[u]
                        float m = sig<ACT>(z, slope);
                        if constexpr (AGG == AGG_SYM) m = cf[i] * m;
                        acc[j][w] += m;
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
template <int MODE, int ACT, int AGG, int LPR, int NV, int VW, int U>
__global__ void __launch_bounds__(256)
k_edge(const int* __restrict__ rowptr, const int* __restrict__ col,
       const int4* __restrict__ items, int64_t n_items,
       const float* __restrict__ R, int64_t ldr,
       const float* __restrict__ C, int64_t ldc,
       const float* __restrict__ G, int64_t ldg,
       const float* __restrict__ norm_row, const float* __restrict__ norm_col,
       float slope, int H,
       float* __restrict__ out, int64_t ldo, float* __restrict__ partial,
       float* __restrict__ Gm, int64_t ldgm) {
    constexpr int RPW = 64 / LPR;
    const int lane = threadIdx.x & 63;
    const int sub = lane / LPR;
    const int li = lane - sub * LPR;
    int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if constexpr (LPR == 64) wave = __builtin_amdgcn_readfirstlane((int)wave);
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
    const float* rp = R + (int64_t)row * ldr;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int c = li + LPR * j;
#pragma unroll
        for (int w = 0; w < VW; ++w) { acc[j][w] = 0.f; rv[j][w] = 0.f; gv[j][w] = 0.f; }
        if (NV == 1 || c < HC) vload<VW>(rv[j], rp + c * VW);
    }
    if constexpr (MODE == MODE_BWD_DST) {
        const float* gp = G + (int64_t)row * ldg;
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
            if (NV == 1 || c < HC) {
                vload<VW>(gv[j], gp + c * VW);
                if constexpr (AGG == AGG_MEAN) {
#pragma unroll
                    for (int w = 0; w < VW; ++w) gv[j][w] = gv[j][w] / degf;   // DivBackward: grad / deg
                    if (Gm != nullptr && first) vstore<VW>(Gm + (int64_t)row * ldgm + c * VW, gv[j]);
                }
            }
        }
    }
    float nr = 1.f;
    if constexpr (AGG == AGG_SYM) nr = norm_row[row];

    int e = e0;
    for (; e + U <= e1; e += U)
        edge_batch<MODE, ACT, AGG, LPR, NV, VW, U>(e, col, C, ldc, G, ldg, norm_col, nr, slope, li, HC, rv, gv, acc);
    if constexpr (U > 4) {
        if (e + 4 <= e1) {
            edge_batch<MODE, ACT, AGG, LPR, NV, VW, 4>(e, col, C, ldc, G, ldg, norm_col, nr, slope, li, HC, rv, gv, acc);
            e += 4;
        }
    }
    if constexpr (U > 2) {
        if (e + 2 <= e1) {
            edge_batch<MODE, ACT, AGG, LPR, NV, VW, 2>(e, col, C, ldc, G, ldg, norm_col, nr, slope, li, HC, rv, gv, acc);
            e += 2;
        }
    }
    if (e < e1)
        edge_batch<MODE, ACT, AGG, LPR, NV, VW, 1>(e, col, C, ldc, G, ldg, norm_col, nr, slope, li, HC, rv, gv, acc);

    if (slot < 0) {
        if constexpr (MODE == MODE_FWD && AGG == AGG_MEAN) {
            const int d = e1 - e0;                      // unsplit: the whole row
            const float degf = (float)(d > 1 ? d : 1);
#pragma unroll
            for (int j = 0; j < NV; ++j)
#pragma unroll
                for (int w = 0; w < VW; ++w) acc[j][w] = acc[j][w] / degf;
        }
        float* op = out + (int64_t)row * ldo;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = li + LPR * j;
            if (NV == 1 || c < HC) vstore<VW>(op + c * VW, acc[j]);
        }
    } else {
        float* pp = partial + (int64_t)slot * H;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = li + LPR * j;
            if (NV == 1 || c < HC) vstore<VW>(pp + c * VW, acc[j]);
        }
    }
}

// Combine the partial rows of split rows in slot order; MEAN_DIV divides by the degree.
template <bool MEAN_DIV, int LPR, int NV, int VW>
__global__ void __launch_bounds__(256)
k_combine(const int4* __restrict__ splits, int64_t n_splits, const float* __restrict__ partial,
          int H, float* __restrict__ out, int64_t ldo) {
    constexpr int RPW = 64 / LPR;
    const int lane = threadIdx.x & 63;
    const int sub = lane / LPR;
    const int li = lane - sub * LPR;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t idx = wave * RPW + sub;
    if (idx >= n_splits) return;
    const int4 sp = splits[idx];
    const int HC = H / VW;
    float acc[NV][VW];
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int w = 0; w < VW; ++w) acc[j][w] = 0.f;
    for (int s = 0; s < sp.z; ++s) {
        const float* pp = partial + (int64_t)(sp.y + s) * H;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = li + LPR * j;
            if (NV == 1 || c < HC) {
                float v[VW];
                vload<VW>(v, pp + c * VW);
#pragma unroll
                for (int w = 0; w < VW; ++w) acc[j][w] += v[w];
            }
        }
    }
    const float degf = (float)(sp.w > 1 ? sp.w : 1);
    float* op = out + (int64_t)sp.x * ldo;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int c = li + LPR * j;
        if (NV == 1 || c < HC) {
            if constexpr (MEAN_DIV) {
#pragma unroll
                for (int w = 0; w < VW; ++w) acc[j][w] = acc[j][w] / degf;
            }
            vstore<VW>(op + c * VW, acc[j]);
        }
    }
}

// ------------------------------------------------------------------------------ dispatch
struct Shape {
    int lpr, nv, vw;
};

template <int MODE, int ACT, int AGG, int LPR, int NV, int VW>
static hipError_t launch_edge_t(const EdgeArgs& a, hipStream_t st) {
    constexpr int U = (NV == 1) ? 8 : 4;
    constexpr int RPW = 64 / LPR;
    const int64_t waves = (a.n_items + RPW - 1) / RPW;
    const int64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL((k_edge<MODE, ACT, AGG, LPR, NV, VW, U>), dim3((unsigned)blocks), dim3(256), 0, st,
                       a.rowptr, a.col, reinterpret_cast<const int4*>(a.items), a.n_items,
                       a.R, a.ldr, a.C, a.ldc, a.G, a.ldg, a.norm_row, a.norm_col, a.slope, a.H,
                       a.out, a.ldo, a.partial, a.Gm, a.ldgm);
    return hipGetLastError();
}

template <int MODE, int ACT, int AGG>
static hipError_t launch_edge_shape(const EdgeArgs& a, Shape s, hipStream_t st) {
    if (s.vw == 4) {
        if (s.lpr == 16) return launch_edge_t<MODE, ACT, AGG, 16, 1, 4>(a, st);
        if (s.lpr == 32) return launch_edge_t<MODE, ACT, AGG, 32, 1, 4>(a, st);
        switch (s.nv) {
            case 1: return launch_edge_t<MODE, ACT, AGG, 64, 1, 4>(a, st);
            case 2: return launch_edge_t<MODE, ACT, AGG, 64, 2, 4>(a, st);
            case 3: return launch_edge_t<MODE, ACT, AGG, 64, 3, 4>(a, st);
            default: return launch_edge_t<MODE, ACT, AGG, 64, 4, 4>(a, st);
        }
    }
    switch (s.nv) {
        case 1: return launch_edge_t<MODE, ACT, AGG, 64, 1, 1>(a, st);
        case 2: return launch_edge_t<MODE, ACT, AGG, 64, 2, 1>(a, st);
        default: return launch_edge_t<MODE, ACT, AGG, 64, 4, 1>(a, st);
    }
}

template <int MODE, int ACT>
static hipError_t launch_edge_agg(const EdgeArgs& a, int agg, Shape s, hipStream_t st) {
    switch (agg) {
        case AGG_SUM: return launch_edge_shape<MODE, ACT, AGG_SUM>(a, s, st);
        case AGG_MEAN: return launch_edge_shape<MODE, ACT, AGG_MEAN>(a, s, st);
        default: return launch_edge_shape<MODE, ACT, AGG_SYM>(a, s, st);
    }
}

template <int MODE>
static hipError_t launch_edge_mode(const EdgeArgs& a, int agg, int act, Shape s, hipStream_t st) {
    switch (act) {
        case ACT_IDENTITY: return launch_edge_agg<MODE, ACT_IDENTITY>(a, agg, s, st);
        case ACT_RELU: return launch_edge_agg<MODE, ACT_RELU>(a, agg, s, st);
        case ACT_LEAKY: return launch_edge_agg<MODE, ACT_LEAKY>(a, agg, s, st);
        case ACT_GELU: return launch_edge_agg<MODE, ACT_GELU>(a, agg, s, st);
        default: return launch_edge_agg<MODE, ACT_GELU_TANH>(a, agg, s, st);
    }
}

template <bool MEAN_DIV, int LPR, int NV, int VW>
static hipError_t launch_combine_t(const int32_t* splits, int64_t n, const float* partial, int H,
                                   float* out, int64_t ldo, hipStream_t st) {
    constexpr int RPW = 64 / LPR;
    const int64_t waves = (n + RPW - 1) / RPW;
    const int64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL((k_combine<MEAN_DIV, LPR, NV, VW>), dim3((unsigned)blocks), dim3(256), 0, st,
                       reinterpret_cast<const int4*>(splits), n, partial, H, out, ldo);
    return hipGetLastError();
}

template <bool MEAN_DIV>
static hipError_t launch_combine_shape(const int32_t* splits, int64_t n, const float* partial, int H,
                                       float* out, int64_t ldo, Shape s, hipStream_t st) {
    if (s.vw == 4) {
        if (s.lpr == 16) return launch_combine_t<MEAN_DIV, 16, 1, 4>(splits, n, partial, H, out, ldo, st);
        if (s.lpr == 32) return launch_combine_t<MEAN_DIV, 32, 1, 4>(splits, n, partial, H, out, ldo, st);
        switch (s.nv) {
            case 1: return launch_combine_t<MEAN_DIV, 64, 1, 4>(splits, n, partial, H, out, ldo, st);
            case 2: return launch_combine_t<MEAN_DIV, 64, 2, 4>(splits, n, partial, H, out, ldo, st);
            case 3: return launch_combine_t<MEAN_DIV, 64, 3, 4>(splits, n, partial, H, out, ldo, st);
            default: return launch_combine_t<MEAN_DIV, 64, 4, 4>(splits, n, partial, H, out, ldo, st);
        }
    }
    switch (s.nv) {
        case 1: return launch_combine_t<MEAN_DIV, 64, 1, 1>(splits, n, partial, H, out, ldo, st);
        case 2: return launch_combine_t<MEAN_DIV, 64, 2, 1>(splits, n, partial, H, out, ldo, st);
        default: return launch_combine_t<MEAN_DIV, 64, 4, 1>(splits, n, partial, H, out, ldo, st);
    }
}

static bool aligned16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Vector width 4 needs every row start 16-B aligned.
bool pick_shape(int H, bool vec4_ok, Shape* s) {
    if (H <= 0) return false;
    if (vec4_ok && (H % 4) == 0) {
        const int hc = H / 4;
        s->vw = 4;
        if (hc <= 16) { s->lpr = 16; s->nv = 1; return true; }
        if (hc <= 32) { s->lpr = 32; s->nv = 1; return true; }
        s->lpr = 64;
        s->nv = (hc + 63) / 64;
        return s->nv <= 4;
    }
    s->vw = 1;
    s->lpr = 64;
    s->nv = (H + 63) / 64;
    if (s->nv == 3) s->nv = 4;
    return s->nv <= 4;
}

hipError_t run_edge(int mode, const EdgeArgs& a, int agg, int act,
                    const int32_t* splits, int64_t n_splits, float* out_final, int64_t ld_final,
                    bool mean_div, hipStream_t st, const char** why) {
    const bool v4 = aligned16(a.R) && aligned16(a.C) && aligned16(a.G) && aligned16(a.out) &&
                    aligned16(a.partial) && aligned16(a.Gm) &&
                    (a.ldr % 4 == 0) && (a.ldc % 4 == 0) && (a.ldg % 4 == 0) && (a.ldo % 4 == 0) &&
                    (a.ldgm % 4 == 0);
    Shape s;
    if (!pick_shape(a.H, v4, &s)) {
        *why = "unsupported hidden size (H must be <= 1024 with H%4==0 and 16-B aligned rows, else <= 256)";
        return hipErrorInvalidValue;
    }
    hipError_t err;
    switch (mode) {
        case MODE_FWD: err = launch_edge_mode<MODE_FWD>(a, agg, act, s, st); break;
        case MODE_BWD_DST: err = launch_edge_mode<MODE_BWD_DST>(a, agg, act, s, st); break;
        default: err = launch_edge_mode<MODE_BWD_SRC>(a, agg, act, s, st); break;
    }
    if (err != hipSuccess) return err;
    if (n_splits > 0) {
        err = mean_div ? launch_combine_shape<true>(splits, n_splits, a.partial, a.H, out_final, ld_final, s, st)
                       : launch_combine_shape<false>(splits, n_splits, a.partial, a.H, out_final, ld_final, s, st);
    }
    return err;
}

}  // namespace sir
