// sirconv_dispatch.hip — shape selection, combine kernel launch, and the per-pass dispatch.
#include "sirconv_edge_impl.h"

namespace sir {

// conv.py:51-57 — fp32 degree norms clamp(deg, 1)^-1/2 computed as IEEE 1/sqrt (what CPU
// torch.pow(x, -0.5) returns bit-for-bit); one launch covers both CSRs.
__global__ void __launch_bounds__(256)
k_degree_norms(const int* __restrict__ rowptr_a, float* __restrict__ norm_a,
               const int* __restrict__ rowptr_b, float* __restrict__ norm_b, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int da = rowptr_a[i + 1] - rowptr_a[i];
    norm_a[i] = 1.0f / sqrtf((float)(da > 1 ? da : 1));
    if (rowptr_b != nullptr) {
        const int db = rowptr_b[i + 1] - rowptr_b[i];
        norm_b[i] = 1.0f / sqrtf((float)(db > 1 ? db : 1));
    }
}

// Column sums of a tall row-major matrix (the bias gradients db_R = sum_v dY[v], db_Q = sum_v dQ[v]).
// Deterministic two-pass: pass 1 gives each of `nb` blocks a contiguous range of rows and writes
// one partial row per block; pass 2 adds the nb partials in block order.  float4 columns.
__global__ void __launch_bounds__(256)
k_colsum_partial(const float* __restrict__ X, int64_t ld, int64_t n_rows, int n_cols,
                 int64_t rows_per_block, float* __restrict__ part) {
    const int c4 = n_cols / 4;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = (r0 + rows_per_block < n_rows) ? r0 + rows_per_block : n_rows;
    for (int cb = 0; cb < c4; cb += 64) {
        const int c = cb + (threadIdx.x & 63);
        const int slice = threadIdx.x >> 6;          // 4 waves take rows r0+slice, +4, ...
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c < c4) {
            int64_t r = r0 + slice;
            for (; r + 12 < r1; r += 16) {
                float4 v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const float4*>(X + (r + 4 * i) * ld + 4 * c);
#pragma unroll
                for (int i = 0; i < 4; ++i) { acc.x += v[i].x; acc.y += v[i].y; acc.z += v[i].z; acc.w += v[i].w; }
            }
            for (; r < r1; r += 4) {
                const float4 v = *reinterpret_cast<const float4*>(X + r * ld + 4 * c);
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            }
        }
        __shared__ float4 red[256];
        red[threadIdx.x] = acc;
        __syncthreads();
        if (threadIdx.x < 64 && c < c4) {
            float4 t = red[threadIdx.x];
#pragma unroll
            for (int k = 1; k < 4; ++k) {
                const float4 u = red[threadIdx.x + 64 * k];
                t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
            }
            *reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * n_cols + 4 * c) = t;
        }
        __syncthreads();
    }
}

// 64 columns x 16 slices per block; slice k adds partials k, k+16, ... (8 loads in flight),
// then the 16 slice sums are added in slice order.
__global__ void __launch_bounds__(1024)
k_colsum_final(const float* __restrict__ part, int nb, int n_cols, float* __restrict__ out) {
    __shared__ float red[1024];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const int slice = threadIdx.x >> 6;
    float acc = 0.f;
    if (c < n_cols) {
        int b = slice;
        for (; b + 7 * 16 < nb; b += 8 * 16) {
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = part[(int64_t)(b + 16 * i) * n_cols + c];
#pragma unroll
            for (int i = 0; i < 8; ++i) acc += v[i];
        }
        for (; b < nb; b += 16) acc += part[(int64_t)b * n_cols + c];
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < 64 && c < n_cols) {
        float t = red[threadIdx.x];
        for (int k = 1; k < 16; ++k) t += red[threadIdx.x + 64 * k];
        out[c] = t;
    }
}

hipError_t run_colsum(const float* X, int64_t ld, int64_t n_rows, int n_cols, float* out,
                      float* workspace, int nb, hipStream_t st) {
    if (n_cols <= 0) return hipSuccess;
    const int64_t rpb = (n_rows + nb - 1) / nb;
    if (n_rows > 0)
        hipLaunchKernelGGL(k_colsum_partial, dim3((unsigned)nb), dim3(256), 0, st, X, ld, n_rows, n_cols, rpb, workspace);
    else
        return hipMemsetAsync(out, 0, sizeof(float) * n_cols, st);
    hipLaunchKernelGGL(k_colsum_final, dim3((unsigned)((n_cols + 63) / 64)), dim3(1024), 0, st,
                       workspace, nb, n_cols, out);
    return hipGetLastError();
}

template <int ST, bool MEAN_DIV>
static hipError_t launch_combine(const int32_t* splits, int64_t n, const float* partial, int H,
                                 void* out, int64_t ldo, int vw, hipStream_t st, const Drop& drop, int accumulate = 0) {
    if (n == 0) return hipSuccess;
    TP<ST>* o = static_cast<TP<ST>*>(out);
    if (vw == 4)
        hipLaunchKernelGGL((k_combine<ST, MEAN_DIV, 4>), dim3((unsigned)n), dim3(1024), 0, st,
                           reinterpret_cast<const int4*>(splits), partial, H, o, ldo, drop, accumulate);
    else
        hipLaunchKernelGGL((k_combine<ST, MEAN_DIV, 1>), dim3((unsigned)n), dim3(1024), 0, st,
                           reinterpret_cast<const int4*>(splits), partial, H, o, ldo, drop, accumulate);
    return hipGetLastError();
}

template <int ST>
static hipError_t run_edge_t(int mode, const EdgeArgs& a, int agg, int act, Shape s,
                             const int32_t* splits, int64_t n_splits, void* out_final, int64_t ld_final,
                             bool mean_div, hipStream_t st) {
    hipError_t err;
    switch (mode) {
        case MODE_FWD: err = launch_edge_pass<ST, MODE_FWD>(a, agg, act, s, st); break;
        case MODE_BWD_DST: err = launch_edge_pass<ST, MODE_BWD_DST>(a, agg, act, s, st); break;
        default: err = launch_edge_pass<ST, MODE_BWD_SRC>(a, agg, act, s, st); break;
    }
    if (err != hipSuccess || n_splits == 0) return err;
    return mean_div ? launch_combine<ST, true>(splits, n_splits, a.partial, a.H, out_final, ld_final, s.vw, st, a.drop)
                    : launch_combine<ST, false>(splits, n_splits, a.partial, a.H, out_final, ld_final, s.vw, st, a.drop,
                                                a.accumulate);
}

hipError_t run_degree_norms(const int* rowptr_a, float* norm_a, const int* rowptr_b, float* norm_b,
                            int64_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_degree_norms, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       rowptr_a, norm_a, rowptr_b, norm_b, n);
    return hipGetLastError();
}

static bool aligned_to(const void* p, uintptr_t b) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & (b - 1)) == 0; }

// Vector width 4 needs every row start 16-B aligned (fp32) / 8-B aligned (16-bit).  (16-bit rows with
// 8 values per lane on sub-wave rows were measured 2-3x slower on the power-law graph, forward slower on
// molecule batches too: profiles/r04_ab_vw8_16bit.txt.)
bool pick_shape(int H, bool vec4_ok, Shape* s) {
    if (H <= 0) return false;
    if (vec4_ok && (H % 4) == 0) {
        const int hc = H / 4;
        s->vw = 4;
        if (hc <= 4) { s->lpr = 4; s->nv = 1; return true; }
        if (hc <= 8) { s->lpr = 8; s->nv = 1; return true; }
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

hipError_t run_edge(int mode, int dtype, const EdgeArgs& a, int agg, int act,
                    const int32_t* splits, int64_t n_splits, void* out_final, int64_t ld_final,
                    bool mean_div, hipStream_t st, const char** why) {
    // 4-wide vectors need every feature row start aligned to 4 elements (16 B fp32, 8 B 16-bit)
    const uintptr_t vb = (dtype == ST_F32) ? 16 : 8;
    const bool v4 = aligned_to(a.R, vb) && aligned_to(a.C, vb) && aligned_to(a.G, vb) && aligned_to(a.out, vb) &&
                    aligned_to(a.partial, 16) && aligned_to(a.Gm, vb) &&
                    (a.ldr % 4 == 0) && (a.ldc % 4 == 0) && (a.ldg % 4 == 0) && (a.ldo % 4 == 0) &&
                    (a.ldgm % 4 == 0);
    Shape s;
    if (!pick_shape(a.H, v4, &s)) {
        *why = "unsupported hidden size (H must be <= 1024 with H%4==0 and 16-B aligned rows, else <= 256)";
        return hipErrorInvalidValue;
    }
    if (dtype != ST_F32 && s.vw != 4) {
        *why = "bf16/fp16 storage needs H % 4 == 0 and 8-B aligned rows (leading dimensions multiples of 4)";
        return hipErrorInvalidValue;
    }
    switch (dtype) {
        case ST_BF16: return run_edge_t<ST_BF16>(mode, a, agg, act, s, splits, n_splits, out_final, ld_final, mean_div, st);
        case ST_F16: return run_edge_t<ST_F16>(mode, a, agg, act, s, splits, n_splits, out_final, ld_final, mean_div, st);
        default: return run_edge_t<ST_F32>(mode, a, agg, act, s, splits, n_splits, out_final, ld_final, mean_div, st);
    }
}

hipError_t run_edge_dual(int dtype, const EdgeArgs& a, const int32_t* splits, int64_t n_splits,
                         const EdgeArgs& b, const int32_t* splits_s, int64_t n_splits_s,
                         int agg, int act, hipStream_t st, const char** why) {
    const uintptr_t vb = (dtype == ST_F32) ? 16 : 8;
    const bool v4 = aligned_to(a.G, vb) && aligned_to(a.out, vb) && aligned_to(b.out, vb) &&
                    aligned_to(a.partial, 16) && aligned_to(b.partial, 16) &&
                    (a.ldg % 4 == 0) && (a.ldo % 4 == 0) && (b.ldo % 4 == 0);
    Shape s;
    if (!pick_shape(a.H, v4, &s) || s.vw != 4) {
        *why = "the sign-mask backward needs H % 4 == 0, H <= 1024 and aligned rows";
        return hipErrorInvalidValue;
    }
    hipError_t err;
    switch (dtype) {
        case ST_BF16: err = launch_edge_dual<ST_BF16>(a, b, agg, act, s, st); break;
        case ST_F16: err = launch_edge_dual<ST_F16>(a, b, agg, act, s, st); break;
        default: err = launch_edge_dual<ST_F32>(a, b, agg, act, s, st); break;
    }
    if (err != hipSuccess) {
        if (err == hipErrorInvalidValue) *why = "the one-launch backward covers SUM/SYM with ReLU/LeakyReLU only";
        return err;
    }
    auto combine = [&](const int32_t* sp, int64_t n, const EdgeArgs& x) -> hipError_t {
        if (n == 0) return hipSuccess;
        switch (dtype) {
            case ST_BF16: return launch_combine<ST_BF16, false>(sp, n, x.partial, x.H, x.out, x.ldo, 4, st, x.drop);
            case ST_F16: return launch_combine<ST_F16, false>(sp, n, x.partial, x.H, x.out, x.ldo, 4, st, x.drop);
            default: return launch_combine<ST_F32, false>(sp, n, x.partial, x.H, x.out, x.ldo, 4, st, x.drop);
        }
    };
    if ((err = combine(splits, n_splits, a)) != hipSuccess) return err;
    return combine(splits_s, n_splits_s, b);
}

}  // namespace sir
