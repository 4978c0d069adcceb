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
// (backward, two arrays) rows' loads in flight at a time (walk_rows).
#include <hip/hip_runtime.h>
#include <stdint.h>

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

template <int VW>
__global__ void __launch_bounds__(256)
k_gn_fwd(const int64_t* __restrict__ off, int64_t B, int F, int n_cc,
         const float* __restrict__ X, int64_t ldx, const float* __restrict__ w, const float* __restrict__ bias,
         const float* __restrict__ ms, float eps, float* __restrict__ Y, int64_t ldy,
         float* __restrict__ mean_out, float* __restrict__ std_out) {
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
    walk_rows<VW>(r0, r1, X, ldx, c, [&](int64_t i, const float (&v)[VW]) {   // norm.py:29
        float y[VW];
#pragma unroll
        for (int x = 0; x < VW; ++x) {
            const float d = v[x] - t[x];
            y[x] = wv[x] * d / sd[x];
            if (bias) y[x] = y[x] + bv[x];
        }
        gst<VW>(Y + i * ldy + c * VW, y);
    });
    gst<VW>(mean_out + b * F + c * VW, s);
    gst<VW>(std_out + b * F + c * VW, sd);
}

template <int VW>
__global__ void __launch_bounds__(256)
k_gn_bwd(const int64_t* __restrict__ off, int64_t B, int F, int n_cc,
         const float* __restrict__ X, int64_t ldx, const float* __restrict__ dY, int64_t ldg,
         const float* __restrict__ w, const float* __restrict__ ms, const float* __restrict__ mean,
         const float* __restrict__ sdv, float* __restrict__ dX, int64_t lddx,
         float* __restrict__ dw_part, float* __restrict__ dms_part, float* __restrict__ db_part) {
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (wave >= B * n_cc) return;
    const int64_t b = wave / n_cc;
    const int cc = (int)(wave - b * n_cc);
    const int c = cc * 64 + (threadIdx.x & 63);
    if (c * VW >= F) return;
    const int64_t r0 = off[b], r1 = off[b + 1];
    const float nf = (float)(r1 - r0);
    float wv[VW], mv[VW], mu[VW], sd[VW], t[VW], A[VW], G[VW], Bs[VW];
    gld<VW>(wv, w + c * VW);
    if (ms) gld<VW>(mv, ms + c * VW);
    else {
#pragma unroll
        for (int x = 0; x < VW; ++x) mv[x] = 1.f;
    }
    gld<VW>(mu, mean + b * F + c * VW);
    gld<VW>(sd, sdv + b * F + c * VW);
#pragma unroll
    for (int x = 0; x < VW; ++x) { t[x] = ms ? mu[x] * mv[x] : mu[x]; A[x] = 0.f; G[x] = 0.f; Bs[x] = 0.f; }
    walk_rows2<VW>(r0, r1, X, ldx, dY, ldg, c, [&](int64_t, const float (&v)[VW], const float (&g)[VW]) {
#pragma unroll
        for (int x = 0; x < VW; ++x) { A[x] += g[x] * (v[x] - t[x]); G[x] += g[x]; }
    });
    float k1[VW], k2[VW];
#pragma unroll
    for (int x = 0; x < VW; ++x) {
        k1[x] = wv[x] / sd[x];                                       // w / s
        k2[x] = wv[x] * A[x] / (nf * sd[x] * sd[x] * sd[x]);          // w A / (n s^3)
    }
    walk_rows2<VW>(r0, r1, X, ldx, dY, ldg, c, [&](int64_t, const float (&v)[VW], const float (&g)[VW]) {
#pragma unroll
        for (int x = 0; x < VW; ++x) Bs[x] += k1[x] * g[x] - k2[x] * (v[x] - t[x]);
    });
    walk_rows2<VW>(r0, r1, X, ldx, dY, ldg, c, [&](int64_t i, const float (&v)[VW], const float (&g)[VW]) {
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

}  // namespace

hipError_t run_graph_norm_fwd(const int64_t* off, int64_t B, int F, const float* X, int64_t ldx,
                              const float* w, const float* bias, const float* ms, float eps,
                              float* Y, int64_t ldy, float* mean, float* sd, hipStream_t st) {
    if (B == 0) return hipSuccess;
    const bool v4 = F % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && al(X) && al(Y) && al(w) && al(bias) &&
                    al(ms) && al(mean) && al(sd);
    const int vw = v4 ? 4 : 1;
    const int n_cc = (F / vw + 63) / 64;
    const int64_t waves = B * n_cc;
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    if (v4)
        hipLaunchKernelGGL((k_gn_fwd<4>), dim3(blocks), dim3(256), 0, st, off, B, F, n_cc, X, ldx, w, bias, ms,
                           eps, Y, ldy, mean, sd);
    else
        hipLaunchKernelGGL((k_gn_fwd<1>), dim3(blocks), dim3(256), 0, st, off, B, F, n_cc, X, ldx, w, bias, ms,
                           eps, Y, ldy, mean, sd);
    return hipGetLastError();
}

hipError_t run_graph_norm_bwd(const int64_t* off, int64_t B, int F, const float* X, int64_t ldx,
                              const float* dY, int64_t ldg, const float* w, const float* ms,
                              const float* mean, const float* sd, float* dX, int64_t lddx,
                              float* dw_part, float* dms_part, float* db_part, hipStream_t st) {
    if (B == 0) return hipSuccess;
    const bool v4 = F % 4 == 0 && ldx % 4 == 0 && ldg % 4 == 0 && lddx % 4 == 0 && al(X) && al(dY) && al(dX) &&
                    al(w) && al(ms) && al(mean) && al(sd) && al(dw_part) && al(dms_part) && al(db_part);
    const int vw = v4 ? 4 : 1;
    const int n_cc = (F / vw + 63) / 64;
    const int64_t waves = B * n_cc;
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    if (v4)
        hipLaunchKernelGGL((k_gn_bwd<4>), dim3(blocks), dim3(256), 0, st, off, B, F, n_cc, X, ldx, dY, ldg, w, ms,
                           mean, sd, dX, lddx, dw_part, dms_part, db_part);
    else
        hipLaunchKernelGGL((k_gn_bwd<1>), dim3(blocks), dim3(256), 0, st, off, B, F, n_cc, X, ldx, dY, ldg, w, ms,
                           mean, sd, dX, lddx, dw_part, dms_part, db_part);
    return hipGetLastError();
}

}  // namespace sir
