// sirconv_resact.hip — the stack loop's residual + activation around a SIRConv layer, one pass per
// direction (the layer loops sirgcn.stacks restates; reference zinc/model.py:53-56 and
// ogbn-arxiv/model.py:65-73 without a norm):
//   order 0 (zinc) : out = act(y + r)            backward: g = act'(y + r) dout;  dy = g, dr = g
//   order 1 (arxiv): out = act(y) + r            backward: dy = act'(y) dout;     dr = dout (the caller's)
// y is the conv output in its storage type (fp32, or bf16 / fp16 under autocast), r and out fp32.
// Each value goes through the ops torch's add / relu / leaky_relu and their autograd apply, in the
// same order and types, so the result is bit-identical to the separate torch kernels they replace
// (two passes forward, two or three backward, plus the 16-bit cast of the gradient): under autocast
// an arxiv-order activation runs on the 16-bit y and rounds to it (torch's opmath), and the
// gradient of a 16-bit y is rounded once from fp32.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sirconv.h"
#include "sirconv_internal.h"

namespace sir {
namespace {

template <int DT>
struct Elt;
template <>
struct Elt<SIR_DTYPE_F32> {
    typedef float T;
    static __device__ __forceinline__ float up(float x) { return x; }
    static __device__ __forceinline__ float down(float x) { return x; }
};
template <>
struct Elt<SIR_DTYPE_BF16> {
    typedef __bf16 T;
    static __device__ __forceinline__ float up(__bf16 x) { return (float)x; }
    static __device__ __forceinline__ __bf16 down(float x) { return (__bf16)x; }
};
template <>
struct Elt<SIR_DTYPE_F16> {
    typedef _Float16 T;
    static __device__ __forceinline__ float up(_Float16 x) { return (float)x; }
    static __device__ __forceinline__ _Float16 down(float x) { return (_Float16)x; }
};

template <int ACT>
__device__ __forceinline__ float act_f(float x, float slope) {
    if constexpr (ACT == SIR_ACT_RELU) return x > 0.f ? x : 0.f;
    else if constexpr (ACT == SIR_ACT_LEAKY_RELU) return x > 0.f ? x : x * slope;
    else return x;
}
template <int ACT>
__device__ __forceinline__ float act_b(float x, float g, float slope) {
    if constexpr (ACT == SIR_ACT_RELU) return x > 0.f ? g : 0.f;
    else if constexpr (ACT == SIR_ACT_LEAKY_RELU) return x > 0.f ? g : g * slope;
    else return g;
}

// 4 consecutive elements per thread, rows of N (N % 4 == 0) — grid-stride over M * N / 4
template <int DT, int ACT, int ORDER>
__global__ void __launch_bounds__(256)
k_resact_fwd(const void* __restrict__ Y, int64_t ldy, const float* __restrict__ R, int64_t ldr, float* __restrict__ O,
             int64_t ldo, int64_t M, int N, float slope) {
    using E = Elt<DT>;
    typedef typename E::T T;
    const int nq = N / 4;
    const int64_t total = M * nq;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
        const int64_t m = q / nq;
        const int n = (int)(q - m * nq) * 4;
        const T* y = static_cast<const T*>(Y) + m * ldy + n;
        const float4 r = *reinterpret_cast<const float4*>(R + m * ldr + n);
        float yv[4];
        if constexpr (DT == SIR_DTYPE_F32) {
            const float4 t = *reinterpret_cast<const float4*>(y);
            yv[0] = t.x; yv[1] = t.y; yv[2] = t.z; yv[3] = t.w;
        } else {
            typedef T T4 __attribute__((ext_vector_type(4)));
            const T4 t = *reinterpret_cast<const T4*>(y);
            yv[0] = E::up(t[0]); yv[1] = E::up(t[1]); yv[2] = E::up(t[2]); yv[3] = E::up(t[3]);
        }
        const float rv[4] = {r.x, r.y, r.z, r.w};
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if constexpr (ORDER == 0) o[i] = act_f<ACT>(yv[i] + rv[i], slope);                  // act(y + r)
            else o[i] = E::up(E::down(act_f<ACT>(yv[i], slope))) + rv[i];                         // act(y) + r
        }
        *reinterpret_cast<float4*>(O + m * ldo + n) = make_float4(o[0], o[1], o[2], o[3]);
    }
}

template <int DT, int ACT, int ORDER>
__global__ void __launch_bounds__(256)
k_resact_bwd(const float* __restrict__ D, int64_t ldd, const float* __restrict__ D2, int64_t ldd2,
             const void* __restrict__ Y, int64_t ldy,
             const float* __restrict__ R, int64_t ldr, void* __restrict__ DY, int64_t lddy, float* __restrict__ DR,
             int64_t lddr, int64_t M, int N, float slope) {
    using E = Elt<DT>;
    typedef typename E::T T;
    const int nq = N / 4;
    const int64_t total = M * nq;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
        const int64_t m = q / nq;
        const int n = (int)(q - m * nq) * 4;
        float4 d = *reinterpret_cast<const float4*>(D + m * ldd + n);
        if (D2 != nullptr) {           // a second gradient of the output: the sum autograd would form
            const float4 d2 = *reinterpret_cast<const float4*>(D2 + m * ldd2 + n);
            d.x += d2.x; d.y += d2.y; d.z += d2.z; d.w += d2.w;
        }
        const T* y = static_cast<const T*>(Y) + m * ldy + n;
        float yv[4];
        if constexpr (DT == SIR_DTYPE_F32) {
            const float4 t = *reinterpret_cast<const float4*>(y);
            yv[0] = t.x; yv[1] = t.y; yv[2] = t.z; yv[3] = t.w;
        } else {
            typedef T T4 __attribute__((ext_vector_type(4)));
            const T4 t = *reinterpret_cast<const T4*>(y);
            yv[0] = E::up(t[0]); yv[1] = E::up(t[1]); yv[2] = E::up(t[2]); yv[3] = E::up(t[3]);
        }
        const float dv[4] = {d.x, d.y, d.z, d.w};
        float g[4];
        if constexpr (ORDER == 0) {
            const float4 r = *reinterpret_cast<const float4*>(R + m * ldr + n);
            const float rv[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) g[i] = act_b<ACT>(yv[i] + rv[i], dv[i], slope);
            if (DR != nullptr) *reinterpret_cast<float4*>(DR + m * lddr + n) = make_float4(g[0], g[1], g[2], g[3]);
        } else {
            // the 16-bit activation's backward runs on the gradient rounded to its type (autograd
            // casts the add's fp32 gradient for the 16-bit operand), in opmath, rounded once more
#pragma unroll
            for (int i = 0; i < 4; ++i) g[i] = act_b<ACT>(yv[i], E::up(E::down(dv[i])), slope);
            // R's gradient is dout itself: written only when it is a sum formed here (D2)
            if (D2 != nullptr && DR != nullptr) *reinterpret_cast<float4*>(DR + m * lddr + n) = d;
        }
        if constexpr (DT == SIR_DTYPE_F32) {
            *reinterpret_cast<float4*>(static_cast<float*>(DY) + m * lddy + n) = make_float4(g[0], g[1], g[2], g[3]);
        } else {
            typedef T T4 __attribute__((ext_vector_type(4)));
            T4 o;
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = E::down(g[i]);
            *reinterpret_cast<T4*>(static_cast<T*>(DY) + m * lddy + n) = o;
        }
    }
}

unsigned resact_grid(int64_t M, int N) {
    const int64_t q = M * (N / 4);
    const int64_t b = (q + 255) / 256;
    const int64_t cap = 8 * (int64_t)device_cu_count();
    return (unsigned)(b < 1 ? 1 : (b > cap ? cap : b));
}

template <int DT, int ORDER>
hipError_t resact_fwd_t(int act, const void* Y, int64_t ldy, const float* R, int64_t ldr, float* O, int64_t ldo,
                        int64_t M, int N, float slope, hipStream_t st) {
    const dim3 grid(resact_grid(M, N));
    switch (act) {
    case SIR_ACT_IDENTITY:
        hipLaunchKernelGGL((k_resact_fwd<DT, SIR_ACT_IDENTITY, ORDER>), grid, dim3(256), 0, st, Y, ldy, R, ldr, O, ldo, M, N, slope);
        break;
    case SIR_ACT_RELU:
        hipLaunchKernelGGL((k_resact_fwd<DT, SIR_ACT_RELU, ORDER>), grid, dim3(256), 0, st, Y, ldy, R, ldr, O, ldo, M, N, slope);
        break;
    case SIR_ACT_LEAKY_RELU:
        hipLaunchKernelGGL((k_resact_fwd<DT, SIR_ACT_LEAKY_RELU, ORDER>), grid, dim3(256), 0, st, Y, ldy, R, ldr, O, ldo, M, N,
                           slope);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int DT, int ORDER>
hipError_t resact_bwd_t(int act, const float* D, int64_t ldd, const float* D2, int64_t ldd2, const void* Y, int64_t ldy,
                        const float* R, int64_t ldr,
                        void* DY, int64_t lddy, float* DR, int64_t lddr, int64_t M, int N, float slope, hipStream_t st) {
    const dim3 grid(resact_grid(M, N));
    switch (act) {
    case SIR_ACT_IDENTITY:
        hipLaunchKernelGGL((k_resact_bwd<DT, SIR_ACT_IDENTITY, ORDER>), grid, dim3(256), 0, st, D, ldd, D2, ldd2, Y, ldy, R, ldr, DY,
                           lddy, DR, lddr, M, N, slope);
        break;
    case SIR_ACT_RELU:
        hipLaunchKernelGGL((k_resact_bwd<DT, SIR_ACT_RELU, ORDER>), grid, dim3(256), 0, st, D, ldd, D2, ldd2, Y, ldy, R, ldr, DY, lddy,
                           DR, lddr, M, N, slope);
        break;
    case SIR_ACT_LEAKY_RELU:
        hipLaunchKernelGGL((k_resact_bwd<DT, SIR_ACT_LEAKY_RELU, ORDER>), grid, dim3(256), 0, st, D, ldd, D2, ldd2, Y, ldy, R, ldr, DY,
                           lddy, DR, lddr, M, N, slope);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace

hipError_t run_resid_act_fwd(const void* Y, int64_t ldy, int dtype, const float* R, int64_t ldr, float* O, int64_t ldo,
                             int64_t M, int N, int act, float slope, int order, hipStream_t st) {
    if (M == 0 || N == 0) return hipSuccess;
    if (dtype == SIR_DTYPE_F32)
        return order ? resact_fwd_t<SIR_DTYPE_F32, 1>(act, Y, ldy, R, ldr, O, ldo, M, N, slope, st)
                     : resact_fwd_t<SIR_DTYPE_F32, 0>(act, Y, ldy, R, ldr, O, ldo, M, N, slope, st);
    if (dtype == SIR_DTYPE_BF16)
        return order ? resact_fwd_t<SIR_DTYPE_BF16, 1>(act, Y, ldy, R, ldr, O, ldo, M, N, slope, st)
                     : resact_fwd_t<SIR_DTYPE_BF16, 0>(act, Y, ldy, R, ldr, O, ldo, M, N, slope, st);
    return order ? resact_fwd_t<SIR_DTYPE_F16, 1>(act, Y, ldy, R, ldr, O, ldo, M, N, slope, st)
                 : resact_fwd_t<SIR_DTYPE_F16, 0>(act, Y, ldy, R, ldr, O, ldo, M, N, slope, st);
}

hipError_t run_resid_act_bwd(const float* D, int64_t ldd, const float* D2, int64_t ldd2, const void* Y, int64_t ldy,
                             int dtype, const float* R, int64_t ldr, void* DY, int64_t lddy, float* DR, int64_t lddr,
                             int64_t M, int N, int act, float slope, int order, hipStream_t st) {
    if (M == 0 || N == 0) return hipSuccess;
#define SIR_RESACT_BWD(DTV, ORD) resact_bwd_t<DTV, ORD>(act, D, ldd, D2, ldd2, Y, ldy, R, ldr, DY, lddy, DR, lddr, M, N, slope, st)
    if (dtype == SIR_DTYPE_F32) return order ? SIR_RESACT_BWD(SIR_DTYPE_F32, 1) : SIR_RESACT_BWD(SIR_DTYPE_F32, 0);
    if (dtype == SIR_DTYPE_BF16) return order ? SIR_RESACT_BWD(SIR_DTYPE_BF16, 1) : SIR_RESACT_BWD(SIR_DTYPE_BF16, 0);
    return order ? SIR_RESACT_BWD(SIR_DTYPE_F16, 1) : SIR_RESACT_BWD(SIR_DTYPE_F16, 0);
#undef SIR_RESACT_BWD
}

}  // namespace sir
