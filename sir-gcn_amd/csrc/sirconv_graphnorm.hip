// sirconv_graphnorm.hip — fused GraphNorm (reference models/norm.py:7-29) for batched graphs.
//
// Nodes of graph b are rows [off[b], off[b+1]).  One wave per (graph, 64-lane column chunk); the
// graph's rows are walked sequentially, so every per-graph sum is taken in node order — the
// order of the reference's CPU scatter_add_ (norm.py:20,26) — and the forward reproduces it.
//   forward : mean = sum x / n;  d = x - mean * ms;  std = sqrt(sum d^2 / n + eps);
//             y = (w * d) / std + b                        (three passes over the graph's rows)
//   backward: A = sum gy*d, G = sum gy;  gd = w*gy/std - w*d*A/(n*std^3);  Bs = sum gd;
//             dx = gd - ms*Bs/n;  per-graph partials A/std, -mean*Bs, G for dw, dms, db
//             (reduced over graphs by the host with the deterministic column sum).
// The whole graph is re-read from L2 by each pass (molecule-sized graphs: a few KB), 32 (forward) / 16
// (backward, two arrays) rows' loads in flight at a time (walk_rows).  One wave per block (spread
// over the CUs), one column per lane by default (gn_wide below).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sirconv.h"
#include "sirconv_internal.h"

namespace sir {
namespace {

template <int VW>
__device__ __forceinline__ void gld(float (&d)[VW], const float* __restrict__ p) {
    if constexpr (VW == 4) {
        const float4 t = *reinterpret_cast<const float4*>(p);
        d[0] = t.x; d[1] = t.y; d[2] = t.z; d[3] = t.w;
    } else {
        d[0] = p[0];
    }
}

template <int VW>
__device__ __forceinline__ void gst(float* __restrict__ p, const float (&s)[VW]) {
    if constexpr (VW == 4) *reinterpret_cast<float4*>(p) = make_float4(s[0], s[1], s[2], s[3]);
    else p[0] = s[0];
}


// Walk rows [r0, r1) in node order, RB rows' loads in flight at a time (a molecule has ~25 rows: the
// forward's passes take one memory latency each, the backward's two; a one-load-per-iteration loop
// paid one latency per row and pass, ~40 us per launch on cfg5);
// f(i, v) is applied in row order, so every per-graph sum keeps the reference's node order.
template <int VW, int RB = 32, typename Fn>
__device__ __forceinline__ void walk_rows(int64_t r0, int64_t r1, const float* __restrict__ base, int64_t ld, int c,
                                          Fn f) {
    int64_t i = r0;
    for (; i + RB <= r1; i += RB) {
        float v[RB][VW];
#pragma unroll
        for (int k = 0; k < RB; ++k) gld<VW>(v[k], base + (i + k) * ld + c * VW);
#pragma unroll
        for (int k = 0; k < RB; ++k) f(i + k, v[k]);
    }
    if (i < r1) {
        const int n = (int)(r1 - i);
        float v[RB][VW];
#pragma unroll
        for (int k = 0; k < RB; ++k) gld<VW>(v[k], base + (i + (k < n ? k : 0)) * ld + c * VW);
#pragma unroll
        for (int k = 0; k < RB; ++k)
            if (k < n) f(i + k, v[k]);
    }
}
// the same over two row-aligned arrays (X and dY)
template <int VW, int RB = 16, typename Fn>
__device__ __forceinline__ void walk_rows2(int64_t r0, int64_t r1, const float* __restrict__ a, int64_t lda,
                                           const float* __restrict__ b, int64_t ldb, int c, Fn f) {
    int64_t i = r0;
    for (; i + RB <= r1; i += RB) {
        float u[RB][VW], v[RB][VW];
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            gld<VW>(u[k], a + (i + k) * lda + c * VW);
            gld<VW>(v[k], b + (i + k) * ldb + c * VW);
        }
#pragma unroll
        for (int k = 0; k < RB; ++k) f(i + k, u[k], v[k]);
    }
    if (i < r1) {
        const int n = (int)(r1 - i);
        float u[RB][VW], v[RB][VW];
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int64_t q = i + (k < n ? k : 0);
            gld<VW>(u[k], a + q * lda + c * VW);
            gld<VW>(v[k], b + q * ldb + c * VW);
        }
#pragma unroll
        for (int k = 0; k < RB; ++k)
            if (k < n) f(i + k, u[k], v[k]);
    }
}

// the stack's activation after the norm (ogbn-arxiv/model.py:65-73: h = act(norm(h)) + resid), the
// ops of torch's relu / leaky_relu and their backward (x > 0 ? g : 0 / g * slope)
template <int ACT>
__device__ __forceinline__ float gn_act(float y, float slope) {
    if constexpr (ACT == SIR_ACT_RELU) return y > 0.f ? y : 0.f;
    else if constexpr (ACT == SIR_ACT_LEAKY_RELU) return y > 0.f ? y : y * slope;
    else return y;
}
template <int ACT>
__device__ __forceinline__ float gn_act_bwd(float y, float g, float slope) {
    if constexpr (ACT == SIR_ACT_RELU) return y > 0.f ? g : 0.f;
    else if constexpr (ACT == SIR_ACT_LEAKY_RELU) return y > 0.f ? g : g * slope;
    else return g;
}

template <int VW, int ACT>
__global__ void __launch_bounds__(64)
k_gn_fwd(const int64_t* __restrict__ off, int64_t B, int F, int n_cc,
         const float* __restrict__ X, int64_t ldx, const float* __restrict__ w, const float* __restrict__ bias,
         const float* __restrict__ ms, float eps, float slope, const float* __restrict__ R, int64_t ldr,
         float* __restrict__ Y, int64_t ldy, float* __restrict__ mean_out, float* __restrict__ std_out) {
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (wave >= B * n_cc) return;
    const int64_t b = wave / n_cc;
    const int cc = (int)(wave - b * n_cc);
    const int c = cc * 64 + (threadIdx.x & 63);          // in units of VW floats
    if (c * VW >= F) return;
    const int64_t r0 = off[b], r1 = off[b + 1];
    const float nf = (float)(r1 - r0);
    float s[VW], q[VW], t[VW], wv[VW], bv[VW], mv[VW];
#pragma unroll
    for (int x = 0; x < VW; ++x) { s[x] = 0.f; q[x] = 0.f; }
    walk_rows<VW>(r0, r1, X, ldx, c, [&](int64_t, const float (&v)[VW]) {   // norm.py:20 scatter_add_ (node order)
#pragma unroll
        for (int x = 0; x < VW; ++x) s[x] += v[x];
    });
    gld<VW>(wv, w + c * VW);
    if (bias) gld<VW>(bv, bias + c * VW);
    if (ms) gld<VW>(mv, ms + c * VW);
#pragma unroll
    for (int x = 0; x < VW; ++x) {
        s[x] = (r1 > r0) ? s[x] / nf : 0.f;               // norm.py:21 mean
        t[x] = ms ? s[x] * mv[x] : s[x];                  // norm.py:23 mean * mean_scale
    }
    walk_rows<VW>(r0, r1, X, ldx, c, [&](int64_t, const float (&v)[VW]) {   // norm.py:26 scatter_add_(demean^2)
#pragma unroll
        for (int x = 0; x < VW; ++x) {
            const float d = v[x] - t[x];
            q[x] += d * d;
        }
    });
    float sd[VW];
#pragma unroll
    for (int x = 0; x < VW; ++x) sd[x] = (r1 > r0) ? sqrtf(q[x] / nf + eps) : 0.f;   // norm.py:27
    auto norm_row = [&](const float (&v)[VW], float (&y)[VW]) {   // norm.py:29, then the activation
#pragma unroll
        for (int x = 0; x < VW; ++x) {
            const float d = v[x] - t[x];
            y[x] = wv[x] * d / sd[x];
            if (bias) y[x] = y[x] + bv[x];
            y[x] = gn_act<ACT>(y[x], slope);
        }
    };
    if (R == nullptr) {
        walk_rows<VW>(r0, r1, X, ldx, c, [&](int64_t i, const float (&v)[VW]) {
            float y[VW];
            norm_row(v, y);
            gst<VW>(Y + i * ldy + c * VW, y);
        });
    } else {                                              // + resid (model.py:73)
        walk_rows2<VW>(r0, r1, X, ldx, R, ldr, c, [&](int64_t i, const float (&v)[VW], const float (&r)[VW]) {
            float y[VW];
            norm_row(v, y);
#pragma unroll
            for (int x = 0; x < VW; ++x) y[x] = y[x] + r[x];
            gst<VW>(Y + i * ldy + c * VW, y);
        });
    }
    gst<VW>(mean_out + b * F + c * VW, s);
    gst<VW>(std_out + b * F + c * VW, sd);
}

// ACT: dY is the gradient of act(y); the kernel takes g = act'(y) dY with y = the forward's norm output,
// recomputed by the forward's own ops (same bits, so the same side of 0)
template <int VW, int ACT>
__global__ void __launch_bounds__(64)
k_gn_bwd(const int64_t* __restrict__ off, int64_t B, int F, int n_cc,
         const float* __restrict__ X, int64_t ldx, const float* __restrict__ dY, int64_t ldg,
         const float* __restrict__ w, const float* __restrict__ bias, const float* __restrict__ ms,
         const float* __restrict__ mean, const float* __restrict__ sdv, float slope, float* __restrict__ dX,
         int64_t lddx, float* __restrict__ dw_part, float* __restrict__ dms_part, float* __restrict__ db_part) {
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (wave >= B * n_cc) return;
    const int64_t b = wave / n_cc;
    const int cc = (int)(wave - b * n_cc);
    const int c = cc * 64 + (threadIdx.x & 63);
    if (c * VW >= F) return;
    const int64_t r0 = off[b], r1 = off[b + 1];
    const float nf = (float)(r1 - r0);
    float wv[VW], mv[VW], mu[VW], sd[VW], t[VW], A[VW], G[VW], Bs[VW], bv[VW];
    gld<VW>(wv, w + c * VW);
    if (ACT != SIR_ACT_IDENTITY && bias != nullptr) gld<VW>(bv, bias + c * VW);
    if (ms) gld<VW>(mv, ms + c * VW);
    else {
#pragma unroll
        for (int x = 0; x < VW; ++x) mv[x] = 1.f;
    }
    gld<VW>(mu, mean + b * F + c * VW);
    gld<VW>(sd, sdv + b * F + c * VW);
#pragma unroll
    for (int x = 0; x < VW; ++x) { t[x] = ms ? mu[x] * mv[x] : mu[x]; A[x] = 0.f; G[x] = 0.f; Bs[x] = 0.f; }
    // act'(y) dY for the row (y: the forward's norm output, same ops)
    auto gate = [&](const float (&v)[VW], const float (&g0)[VW], float (&g)[VW]) {
#pragma unroll
        for (int x = 0; x < VW; ++x) {
            if constexpr (ACT == SIR_ACT_IDENTITY) {
                g[x] = g0[x];
            } else {
                float y = wv[x] * (v[x] - t[x]) / sd[x];
                if (bias) y = y + bv[x];
                g[x] = gn_act_bwd<ACT>(y, g0[x], slope);
            }
        }
    };
    walk_rows2<VW>(r0, r1, X, ldx, dY, ldg, c, [&](int64_t, const float (&v)[VW], const float (&g0)[VW]) {
        float g[VW];
        gate(v, g0, g);
#pragma unroll
        for (int x = 0; x < VW; ++x) { A[x] += g[x] * (v[x] - t[x]); G[x] += g[x]; }
    });
    float k1[VW], k2[VW];
#pragma unroll
    for (int x = 0; x < VW; ++x) {
        k1[x] = wv[x] / sd[x];                                       // w / s
        k2[x] = wv[x] * A[x] / (nf * sd[x] * sd[x] * sd[x]);          // w A / (n s^3)
    }
    walk_rows2<VW>(r0, r1, X, ldx, dY, ldg, c, [&](int64_t, const float (&v)[VW], const float (&g0)[VW]) {
        float g[VW];
        gate(v, g0, g);
#pragma unroll
        for (int x = 0; x < VW; ++x) Bs[x] += k1[x] * g[x] - k2[x] * (v[x] - t[x]);
    });
    walk_rows2<VW>(r0, r1, X, ldx, dY, ldg, c, [&](int64_t i, const float (&v)[VW], const float (&g0)[VW]) {
        float g[VW];
        gate(v, g0, g);
        float o[VW];
#pragma unroll
        for (int x = 0; x < VW; ++x) o[x] = (k1[x] * g[x] - k2[x] * (v[x] - t[x])) - mv[x] * Bs[x] / nf;
        gst<VW>(dX + i * lddx + c * VW, o);
    });
    float pw[VW], pm[VW];
#pragma unroll
    for (int x = 0; x < VW; ++x) {
        pw[x] = (r1 > r0) ? A[x] / sd[x] : 0.f;
        pm[x] = -(mu[x] * Bs[x]);
    }
    gst<VW>(dw_part + b * F + c * VW, pw);
    if (dms_part) gst<VW>(dms_part + b * F + c * VW, pm);
    gst<VW>(db_part + b * F + c * VW, G);
}

bool al(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// One column per lane (VW 1) by default: a wave walks its graph's rows in order three times, so
// its time is its instruction latency over the rows — 16-byte columns (VW 4) give each wave 4x the
// work and 4x fewer waves: config 5 (64 molecules, F = 300) 10.96 -> 6.48 us forward, 9.66 -> 6.63
// backward; 10,000 graphs at F = 128: 68.7 -> 54.5 forward, 108 vs 111 backward
// (tools/dbg/gn_probe.hip, profiles/r05_graphnorm.txt).  env SIR_GN_VW=4 takes the wide kernels.
bool gn_wide(int64_t, int) {
    const char* e = getenv("SIR_GN_VW");
    return e != nullptr && atoi(e) == 4;
}

}  // namespace

template <int ACT>
static void launch_gn_fwd(bool v4, unsigned blocks, hipStream_t st, const int64_t* off, int64_t B, int F, int n_cc,
                          const float* X, int64_t ldx, const float* w, const float* bias, const float* ms, float eps,
                          float slope, const float* R, int64_t ldr, float* Y, int64_t ldy, float* mean, float* sd) {
    if (v4)
        hipLaunchKernelGGL((k_gn_fwd<4, ACT>), dim3(blocks), dim3(64), 0, st, off, B, F, n_cc, X, ldx, w, bias, ms,
                           eps, slope, R, ldr, Y, ldy, mean, sd);
    else
        hipLaunchKernelGGL((k_gn_fwd<1, ACT>), dim3(blocks), dim3(64), 0, st, off, B, F, n_cc, X, ldx, w, bias, ms,
                           eps, slope, R, ldr, Y, ldy, mean, sd);
}

hipError_t run_graph_norm_fwd(const int64_t* off, int64_t B, int F, const float* X, int64_t ldx,
                              const float* w, const float* bias, const float* ms, float eps, int act, float slope,
                              const float* R, int64_t ldr, float* Y, int64_t ldy, float* mean, float* sd,
                              hipStream_t st) {
    if (B == 0) return hipSuccess;
    const bool v4 = F % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && (R == nullptr || ldr % 4 == 0) && al(X) && al(Y) &&
                    al(R) && al(w) && al(bias) && al(ms) && al(mean) && al(sd) && gn_wide(B, F);
    const int vw = v4 ? 4 : 1;
    const int n_cc = (F / vw + 63) / 64;
    const unsigned blocks = (unsigned)(B * n_cc);
    switch (act) {
    case SIR_ACT_IDENTITY:
        launch_gn_fwd<SIR_ACT_IDENTITY>(v4, blocks, st, off, B, F, n_cc, X, ldx, w, bias, ms, eps, slope, R, ldr, Y, ldy, mean, sd);
        break;
    case SIR_ACT_RELU:
        launch_gn_fwd<SIR_ACT_RELU>(v4, blocks, st, off, B, F, n_cc, X, ldx, w, bias, ms, eps, slope, R, ldr, Y, ldy, mean, sd);
        break;
    case SIR_ACT_LEAKY_RELU:
        launch_gn_fwd<SIR_ACT_LEAKY_RELU>(v4, blocks, st, off, B, F, n_cc, X, ldx, w, bias, ms, eps, slope, R, ldr, Y, ldy,
                                          mean, sd);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int ACT>
static void launch_gn_bwd(bool v4, unsigned blocks, hipStream_t st, const int64_t* off, int64_t B, int F, int n_cc,
                          const float* X, int64_t ldx, const float* dY, int64_t ldg, const float* w, const float* bias,
                          const float* ms, const float* mean, const float* sd, float slope, float* dX, int64_t lddx,
                          float* dw_part, float* dms_part, float* db_part) {
    if (v4)
        hipLaunchKernelGGL((k_gn_bwd<4, ACT>), dim3(blocks), dim3(64), 0, st, off, B, F, n_cc, X, ldx, dY, ldg, w, bias,
                           ms, mean, sd, slope, dX, lddx, dw_part, dms_part, db_part);
    else
        hipLaunchKernelGGL((k_gn_bwd<1, ACT>), dim3(blocks), dim3(64), 0, st, off, B, F, n_cc, X, ldx, dY, ldg, w, bias,
                           ms, mean, sd, slope, dX, lddx, dw_part, dms_part, db_part);
}

hipError_t run_graph_norm_bwd(const int64_t* off, int64_t B, int F, const float* X, int64_t ldx,
                              const float* dY, int64_t ldg, const float* w, const float* bias, const float* ms,
                              const float* mean, const float* sd, int act, float slope, float* dX, int64_t lddx,
                              float* dw_part, float* dms_part, float* db_part, hipStream_t st) {
    if (B == 0) return hipSuccess;
    const bool v4 = F % 4 == 0 && ldx % 4 == 0 && ldg % 4 == 0 && lddx % 4 == 0 && al(X) && al(dY) && al(dX) &&
                    al(w) && al(bias) && al(ms) && al(mean) && al(sd) && al(dw_part) && al(dms_part) && al(db_part) &&
                    gn_wide(B, F);
    const int vw = v4 ? 4 : 1;
    const int n_cc = (F / vw + 63) / 64;
    const unsigned blocks = (unsigned)(B * n_cc);
    switch (act) {
    case SIR_ACT_IDENTITY:
        launch_gn_bwd<SIR_ACT_IDENTITY>(v4, blocks, st, off, B, F, n_cc, X, ldx, dY, ldg, w, bias, ms, mean, sd, slope, dX,
                                        lddx, dw_part, dms_part, db_part);
        break;
    case SIR_ACT_RELU:
        launch_gn_bwd<SIR_ACT_RELU>(v4, blocks, st, off, B, F, n_cc, X, ldx, dY, ldg, w, bias, ms, mean, sd, slope, dX,
                                    lddx, dw_part, dms_part, db_part);
        break;
    case SIR_ACT_LEAKY_RELU:
        launch_gn_bwd<SIR_ACT_LEAKY_RELU>(v4, blocks, st, off, B, F, n_cc, X, ldx, dY, ldg, w, bias, ms, mean, sd, slope,
                                          dX, lddx, dw_part, dms_part, db_part);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sir
