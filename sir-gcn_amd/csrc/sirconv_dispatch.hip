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

template <bool MEAN_DIV>
static hipError_t launch_combine(const int32_t* splits, int64_t n, const float* partial, int H,
                                 float* out, int64_t ldo, int vw, hipStream_t st) {
    if (n == 0) return hipSuccess;
    if (vw == 4)
        hipLaunchKernelGGL((k_combine<MEAN_DIV, 4>), dim3((unsigned)n), dim3(1024), 0, st,
                           reinterpret_cast<const int4*>(splits), partial, H, out, ldo);
    else
        hipLaunchKernelGGL((k_combine<MEAN_DIV, 1>), dim3((unsigned)n), dim3(1024), 0, st,
                           reinterpret_cast<const int4*>(splits), partial, H, out, ldo);
    return hipGetLastError();
}

hipError_t run_degree_norms(const int* rowptr_a, float* norm_a, const int* rowptr_b, float* norm_b,
                            int64_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_degree_norms, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       rowptr_a, norm_a, rowptr_b, norm_b, n);
    return hipGetLastError();
}

static bool aligned16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Vector width 4 needs every row start 16-B aligned.
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
        case MODE_FWD: err = launch_mode_fwd(a, agg, act, s, st); break;
        case MODE_BWD_DST: err = launch_mode_bwd_dst(a, agg, act, s, st); break;
        default: err = launch_mode_bwd_src(a, agg, act, s, st); break;
    }
    if (err != hipSuccess) return err;
    if (n_splits > 0) {
        err = mean_div ? launch_combine<true>(splits, n_splits, a.partial, a.H, out_final, ld_final, s.vw, st)
                       : launch_combine<false>(splits, n_splits, a.partial, a.H, out_final, ld_final, s.vw, st);
    }
    return err;
}

}  // namespace sir
