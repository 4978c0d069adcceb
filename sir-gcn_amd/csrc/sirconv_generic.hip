// sirconv_generic.hip — edge-materialised kernels for the variants the fused path does not cover:
// agg_type='max' (conv.py:46-47: per-edge linear_relation, then DGL's max reduce) and an arbitrary
// sigma callable (e.g. DictionaryLookup's Sequential(ReLU, Linear, ReLU), dictionary-lookup/model.py:17).
//
// The reference's DGL edge-UDF dataflow is kept (gather -> UDF -> reduce), but every sparse step is
// a native kernel over the row-CSR work plan (same items / split rows as the fused kernels):
//   k_gather_add      Z[e] = Q[row] + K[col[e]]              (edges in dst-CSR order)
//   k_seg_sum         out[row] = sum_e c_e * X[idx(e)]       (idx = e or perm[e]; c_e = norm product)
//   k_edge_bcast      dM[e] = c_e * dS[row] (/deg for mean)  (backward of k_seg_sum)
//   k_seg_max         Y[row] = max_e M[e], arg = first arg-max edge (DGL SpMMCmpCsr), 0 if no edge
//   k_seg_max_bwd     dM[e] = (arg[row] == e) ? dY[row] : 0
// Deterministic, atomics-free, fp32 accumulation in edge order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sirconv_internal.h"

namespace sir {
namespace {

template <int VW>
__device__ __forceinline__ void ld(float (&d)[VW], const float* __restrict__ p) {
    if constexpr (VW == 4) {
        const float4 t = *reinterpret_cast<const float4*>(p);
        d[0] = t.x; d[1] = t.y; d[2] = t.z; d[3] = t.w;
    } else {
        d[0] = p[0];
    }
}

template <int VW>
__device__ __forceinline__ void st(float* __restrict__ p, const float (&s)[VW]) {
    if constexpr (VW == 4) *reinterpret_cast<float4*>(p) = make_float4(s[0], s[1], s[2], s[3]);
    else p[0] = s[0];
}

struct Item {
    int row, e0, e1, slot;
};

__device__ __forceinline__ Item load_item(const int4* __restrict__ items, int64_t w) {
    int4 it = items[w];
    return {__builtin_amdgcn_readfirstlane(it.x), __builtin_amdgcn_readfirstlane(it.y),
            __builtin_amdgcn_readfirstlane(it.z), __builtin_amdgcn_readfirstlane(it.w)};
}

__device__ __forceinline__ int64_t wave_id() {
    return __builtin_amdgcn_readfirstlane((int)((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
}

// ---------------------------------------------------------------------------------------- gather
// ACT: ACT_IDENTITY (Z = the sum), ACT_RELU / ACT_LEAKY (A = sigma of it: torch's relu / leaky_relu)
// SM: also the sign bits of the 256 features of each edge (F = 256, one float4 per lane): 4 words per
// edge, bit l of word x = (value of feature 4 l + x) > 0 — one ballot per word (sir_gemm_nt_dact's gate)
template <int NV, int VW, int ACT, bool SM>
__global__ void __launch_bounds__(256)
k_gather_add(const int* __restrict__ col, const int4* __restrict__ items, int64_t n_items, int F,
             const float* __restrict__ Q, int64_t ldq, const float* __restrict__ K, int64_t ldk,
             float* __restrict__ Z, int64_t ldz, float slope, uint64_t* __restrict__ smask) {
    const int64_t w = wave_id();
    if (w >= n_items) return;
    const Item it = load_item(items, w);
    const int lane = threadIdx.x & 63;
    const int FC = F / VW;
    float q[NV][VW];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int c = lane + 64 * j;
        if (c < FC) ld<VW>(q[j], Q + (int64_t)it.row * ldq + c * VW);
    }
    for (int e = it.e0; e < it.e1; ++e) {
        const int u = __builtin_amdgcn_readfirstlane(col[e]);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = lane + 64 * j;
            if (c < FC) {
                float k[VW];
                ld<VW>(k, K + (int64_t)u * ldk + c * VW);
#pragma unroll
                for (int x = 0; x < VW; ++x) {
                    k[x] = q[j][x] + k[x];                                 // eq[v] + ek[u] (conv.py:45)
                    if constexpr (ACT == ACT_RELU) k[x] = k[x] > 0.f ? k[x] : 0.f;
                    else if constexpr (ACT == ACT_LEAKY) k[x] = k[x] > 0.f ? k[x] : k[x] * slope;
                }
                if constexpr (SM) {
                    uint64_t b[VW];
#pragma unroll
                    for (int x = 0; x < VW; ++x) b[x] = __builtin_amdgcn_ballot_w64(k[x] > 0.f);
                    if (lane < VW) smask[(int64_t)e * VW + lane] = lane == 0 ? b[0] : lane == 1 ? b[1 % VW] : lane == 2 ? b[2 % VW] : b[3 % VW];
                }
                st<VW>(Z + (int64_t)e * ldz + c * VW, k);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------- seg sum
// out[row] = sum_{e in item} coef_e * X[idx(e)], coef_e = norm_col[col[e]] * norm_row[row] (if norms)
template <int NV, int VW>
__global__ void __launch_bounds__(256)
k_seg_sum(const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ perm,
          const int4* __restrict__ items, int64_t n_items, int F,
          const float* __restrict__ X, int64_t ldx, const float* __restrict__ norm_row,
          const float* __restrict__ norm_col, int mean, float* __restrict__ out, int64_t ldo,
          float* __restrict__ partial) {
    const int64_t w = wave_id();
    if (w >= n_items) return;
    const Item it = load_item(items, w);
    const int lane = threadIdx.x & 63;
    const int FC = F / VW;
    float acc[NV][VW];
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int x = 0; x < VW; ++x) acc[j][x] = 0.f;
    const float nr = norm_row ? norm_row[it.row] : 1.f;
    for (int e = it.e0; e < it.e1; ++e) {
        const int src = perm ? __builtin_amdgcn_readfirstlane(perm[e]) : e;
        float c = 1.f;
        if (norm_row) c = norm_col[__builtin_amdgcn_readfirstlane(col[e])] * nr;   // out_norm[u]*in_norm[v]
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int cc = lane + 64 * j;
            if (cc < FC) {
                float v[VW];
                ld<VW>(v, X + (int64_t)src * ldx + cc * VW);
#pragma unroll
                for (int x = 0; x < VW; ++x) acc[j][x] += norm_row ? c * v[x] : v[x];
            }
        }
    }
    float* op;
    if (it.slot < 0) {
        op = out + (int64_t)it.row * ldo;
        if (mean) {
            const int d = it.e1 - it.e0;
            const float degf = (float)(d > 1 ? d : 1);
#pragma unroll
            for (int j = 0; j < NV; ++j)
#pragma unroll
                for (int x = 0; x < VW; ++x) acc[j][x] = acc[j][x] / degf;
        }
    } else {
        op = partial + (int64_t)it.slot * F;
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int cc = lane + 64 * j;
        if (cc < FC) st<VW>(op + cc * VW, acc[j]);
    }
    (void)rowptr;
}

// ------------------------------------------------------------------------------------ broadcast
// dM[e] = c_e * g,  g = dS[row] (mean: dS[row] / max(deg, 1), deg from rowptr)
template <int NV, int VW>
__global__ void __launch_bounds__(256)
k_edge_bcast(const int* __restrict__ rowptr, const int* __restrict__ col, const int4* __restrict__ items,
             int64_t n_items, int F, const float* __restrict__ dS, int64_t lds,
             const float* __restrict__ norm_row, const float* __restrict__ norm_col, int mean,
             float* __restrict__ dM, int64_t ldm) {
    const int64_t w = wave_id();
    if (w >= n_items) return;
    const Item it = load_item(items, w);
    const int lane = threadIdx.x & 63;
    const int FC = F / VW;
    float g[NV][VW];
    float degf = 1.f;
    if (mean) {
        const int d = rowptr[it.row + 1] - rowptr[it.row];
        degf = (float)(d > 1 ? d : 1);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int c = lane + 64 * j;
        if (c < FC) {
            ld<VW>(g[j], dS + (int64_t)it.row * lds + c * VW);
            if (mean) {
#pragma unroll
                for (int x = 0; x < VW; ++x) g[j][x] = g[j][x] / degf;
            }
        }
    }
    const float nr = norm_row ? norm_row[it.row] : 1.f;
    for (int e = it.e0; e < it.e1; ++e) {
        float c = 1.f;
        if (norm_row) c = norm_col[__builtin_amdgcn_readfirstlane(col[e])] * nr;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int cc = lane + 64 * j;
            if (cc < FC) {
                float v[VW];
#pragma unroll
                for (int x = 0; x < VW; ++x) v[x] = norm_row ? g[j][x] * c : g[j][x];   // grad * other
                st<VW>(dM + (int64_t)e * ldm + cc * VW, v);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------- seg max
// Y[row] = max_e M[e] with the FIRST arg-max edge kept on ties (strict >, DGL SpMMCmpCsr);
// rows without edges: Y = 0, arg = -1.  Split rows: per-slot (value, arg) partials.
template <int NV, int VW>
__global__ void __launch_bounds__(256)
k_seg_max(const int4* __restrict__ items, int64_t n_items, int F, const float* __restrict__ M, int64_t ldm,
          float* __restrict__ Y, int64_t ldy, int* __restrict__ arg, int64_t lda,
          float* __restrict__ pval, int* __restrict__ parg) {
    const int64_t w = wave_id();
    if (w >= n_items) return;
    const Item it = load_item(items, w);
    const int lane = threadIdx.x & 63;
    const int FC = F / VW;
    float best[NV][VW];
    int barg[NV][VW];
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int x = 0; x < VW; ++x) { best[j][x] = 0.f; barg[j][x] = -1; }
    for (int e = it.e0; e < it.e1; ++e) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = lane + 64 * j;
            if (c < FC) {
                float v[VW];
                ld<VW>(v, M + (int64_t)e * ldm + c * VW);
#pragma unroll
                for (int x = 0; x < VW; ++x)
                    if (barg[j][x] < 0 || v[x] > best[j][x]) { best[j][x] = v[x]; barg[j][x] = e; }
            }
        }
    }
    float* yp = (it.slot < 0) ? Y + (int64_t)it.row * ldy : pval + (int64_t)it.slot * F;
    int* ap = (it.slot < 0) ? arg + (int64_t)it.row * lda : parg + (int64_t)it.slot * F;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int c = lane + 64 * j;
        if (c < FC) {
            st<VW>(yp + c * VW, best[j]);
#pragma unroll
            for (int x = 0; x < VW; ++x) ap[c * VW + x] = barg[j][x];
        }
    }
}

// combine split rows: slots in edge order, strict > keeps the first arg-max
__global__ void __launch_bounds__(256)
k_seg_max_combine(const int4* __restrict__ splits, int64_t n_splits, int F, const float* __restrict__ pval,
                  const int* __restrict__ parg, float* __restrict__ Y, int64_t ldy, int* __restrict__ arg,
                  int64_t lda) {
    const int64_t s = blockIdx.x;
    if (s >= n_splits) return;
    const int4 sp = splits[s];
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

// dM[e] = (arg[row] == e) ? dY[row] : 0   for every edge e of the item
template <int NV, int VW>
__global__ void __launch_bounds__(256)
k_seg_max_bwd(const int4* __restrict__ items, int64_t n_items, int F, const int* __restrict__ arg, int64_t lda,
              const float* __restrict__ dY, int64_t ldy, float* __restrict__ dM, int64_t ldm) {
    const int64_t w = wave_id();
    if (w >= n_items) return;
    const Item it = load_item(items, w);
    const int lane = threadIdx.x & 63;
    const int FC = F / VW;
    float g[NV][VW];
    int a[NV][VW];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int c = lane + 64 * j;
        if (c < FC) {
            ld<VW>(g[j], dY + (int64_t)it.row * ldy + c * VW);
#pragma unroll
            for (int x = 0; x < VW; ++x) a[j][x] = arg[(int64_t)it.row * lda + c * VW + x];
        }
    }
    for (int e = it.e0; e < it.e1; ++e) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int c = lane + 64 * j;
            if (c < FC) {
                float v[VW];
#pragma unroll
                for (int x = 0; x < VW; ++x) v[x] = (a[j][x] == e) ? g[j][x] : 0.f;
                st<VW>(dM + (int64_t)e * ldm + c * VW, v);
            }
        }
    }
}

template <int VW>
__global__ void __launch_bounds__(1024)
k_sum_combine(const int4* __restrict__ splits, const float* __restrict__ partial, int F, int mean,
              float* __restrict__ out, int64_t ldo) {
    const int4 sp = splits[blockIdx.x];
    const float degf = (float)(sp.w > 1 ? sp.w : 1);
    for (int c = threadIdx.x; c < F / VW; c += blockDim.x) {
        float acc[VW];
#pragma unroll
        for (int x = 0; x < VW; ++x) acc[x] = 0.f;
        for (int k = 0; k < sp.z; ++k) {
            float v[VW];
            ld<VW>(v, partial + (int64_t)(sp.y + k) * F + c * VW);
#pragma unroll
            for (int x = 0; x < VW; ++x) acc[x] += v[x];
        }
        if (mean) {
#pragma unroll
            for (int x = 0; x < VW; ++x) acc[x] = acc[x] / degf;
        }
        st<VW>(out + (int64_t)sp.x * ldo + c * VW, acc);
    }
}

// ---------------------------------------------------------------------------------------- dispatch
struct GShape {
    int nv, vw;
};

bool gshape(int F, bool v4, GShape* s) {
    if (F <= 0) return false;
    if (v4 && F % 4 == 0) {
        s->vw = 4;
        s->nv = (F / 4 + 63) / 64;
    } else {
        s->vw = 1;
        s->nv = (F + 63) / 64;
    }
    if (s->nv == 3) s->nv = 4;
    return s->nv <= 4 && s->nv >= 1;
}

inline unsigned blocks_for(int64_t n_items) { return (unsigned)((n_items + 3) / 4); }

template <class Fn>
void gdispatch(GShape s, Fn&& fn) {
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I4 = std::integral_constant<int, 4>;
    if (s.vw == 4) {
        if (s.nv == 1) fn(I1{}, I4{});
        else if (s.nv == 2) fn(I2{}, I4{});
        else fn(I4{}, I4{});
    } else {
        if (s.nv == 1) fn(I1{}, I1{});
        else if (s.nv == 2) fn(I2{}, I1{});
        else fn(I4{}, I1{});
    }
}

bool al16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace

hipError_t run_gather_add(const GenericArgs& a, hipStream_t st, int act, float slope, uint64_t* smask) {
    GShape s;
    const bool v4 = al16(a.X) && al16(a.X2) && al16(a.out) && a.ldx % 4 == 0 && a.ldx2 % 4 == 0 && a.ldo % 4 == 0;
    if (!gshape(a.F, v4, &s)) return hipErrorInvalidValue;
    if (act != ACT_IDENTITY && act != ACT_RELU && act != ACT_LEAKY) return hipErrorInvalidValue;
    if (smask != nullptr && !(a.F == 256 && s.nv == 1 && s.vw == 4)) return hipErrorInvalidValue;
    if (a.n_items == 0) return hipSuccess;
    gdispatch(s, [&](auto nv_, auto vw_) {
        constexpr int NV_ = decltype(nv_)::value, VW_ = decltype(vw_)::value;
        const dim3 grid(blocks_for(a.n_items));
#define SIR_GATHER(ACTV, SMV)                                                                                   \
        hipLaunchKernelGGL((k_gather_add<NV_, VW_, ACTV, SMV>), grid, dim3(256), 0, st, a.col,                  \
                           reinterpret_cast<const int4*>(a.items), a.n_items, a.F, a.X, a.ldx, a.X2, a.ldx2, a.out, \
                           a.ldo, slope, smask)
        if constexpr (NV_ == 1 && VW_ == 4) {
            if (smask != nullptr) {
                if (act == ACT_RELU) SIR_GATHER(ACT_RELU, true);
                else if (act == ACT_LEAKY) SIR_GATHER(ACT_LEAKY, true);
                else SIR_GATHER(ACT_IDENTITY, true);
                return;
            }
        }
        if (act == ACT_RELU) SIR_GATHER(ACT_RELU, false);
        else if (act == ACT_LEAKY) SIR_GATHER(ACT_LEAKY, false);
        else SIR_GATHER(ACT_IDENTITY, false);
#undef SIR_GATHER
    });
    return hipGetLastError();
}

hipError_t run_seg_sum(const GenericArgs& a, hipStream_t st) {
    GShape s;
    const bool v4 = al16(a.X) && al16(a.out) && al16(a.partial) && a.ldx % 4 == 0 && a.ldo % 4 == 0;
    if (!gshape(a.F, v4, &s)) return hipErrorInvalidValue;
    if (a.n_items == 0) return hipSuccess;
    gdispatch(s, [&](auto nv_, auto vw_) {
        constexpr int NV_ = decltype(nv_)::value, VW_ = decltype(vw_)::value;
        hipLaunchKernelGGL((k_seg_sum<NV_, VW_>), dim3(blocks_for(a.n_items)), dim3(256), 0, st,
                                        a.rowptr, a.col, a.perm, reinterpret_cast<const int4*>(a.items), a.n_items,
                                        a.F, a.X, a.ldx, a.norm_row, a.norm_col, a.mean, a.out, a.ldo, a.partial);
    });
    hipError_t err = hipGetLastError();
    if (err != hipSuccess || a.n_splits == 0) return err;
    if (s.vw == 4)
        hipLaunchKernelGGL((k_sum_combine<4>), dim3((unsigned)a.n_splits), dim3(1024), 0, st,
                           reinterpret_cast<const int4*>(a.splits), a.partial, a.F, a.mean, a.out, a.ldo);
    else
        hipLaunchKernelGGL((k_sum_combine<1>), dim3((unsigned)a.n_splits), dim3(1024), 0, st,
                           reinterpret_cast<const int4*>(a.splits), a.partial, a.F, a.mean, a.out, a.ldo);
    return hipGetLastError();
}

hipError_t run_edge_bcast(const GenericArgs& a, hipStream_t st) {
    GShape s;
    const bool v4 = al16(a.X) && al16(a.out) && a.ldx % 4 == 0 && a.ldo % 4 == 0;
    if (!gshape(a.F, v4, &s)) return hipErrorInvalidValue;
    if (a.n_items == 0) return hipSuccess;
    gdispatch(s, [&](auto nv_, auto vw_) {
        constexpr int NV_ = decltype(nv_)::value, VW_ = decltype(vw_)::value;
        hipLaunchKernelGGL((k_edge_bcast<NV_, VW_>), dim3(blocks_for(a.n_items)), dim3(256), 0, st,
                                        a.rowptr, a.col, reinterpret_cast<const int4*>(a.items), a.n_items, a.F,
                                        a.X, a.ldx, a.norm_row, a.norm_col, a.mean, a.out, a.ldo);
    });
    return hipGetLastError();
}

hipError_t run_seg_max(const GenericArgs& a, hipStream_t st) {
    GShape s;
    const bool v4 = al16(a.X) && al16(a.out) && al16(a.partial) && a.ldx % 4 == 0 && a.ldo % 4 == 0;
    if (!gshape(a.F, v4, &s)) return hipErrorInvalidValue;
    if (a.n_items == 0) return hipSuccess;
    gdispatch(s, [&](auto nv_, auto vw_) {
        constexpr int NV_ = decltype(nv_)::value, VW_ = decltype(vw_)::value;
        hipLaunchKernelGGL((k_seg_max<NV_, VW_>), dim3(blocks_for(a.n_items)), dim3(256), 0, st,
                                        reinterpret_cast<const int4*>(a.items), a.n_items, a.F, a.X, a.ldx,
                                        a.out, a.ldo, a.arg, a.lda, a.partial, a.parg);
    });
    hipError_t err = hipGetLastError();
    if (err != hipSuccess || a.n_splits == 0) return err;
    hipLaunchKernelGGL(k_seg_max_combine, dim3((unsigned)a.n_splits), dim3(256), 0, st,
                       reinterpret_cast<const int4*>(a.splits), a.n_splits, a.F, a.partial, a.parg,
                       a.out, a.ldo, a.arg, a.lda);
    return hipGetLastError();
}

hipError_t run_seg_max_bwd(const GenericArgs& a, hipStream_t st) {
    GShape s;
    const bool v4 = al16(a.X) && al16(a.out) && a.ldx % 4 == 0 && a.ldo % 4 == 0;
    if (!gshape(a.F, v4, &s)) return hipErrorInvalidValue;
    if (a.n_items == 0) return hipSuccess;
    gdispatch(s, [&](auto nv_, auto vw_) {
        constexpr int NV_ = decltype(nv_)::value, VW_ = decltype(vw_)::value;
        hipLaunchKernelGGL((k_seg_max_bwd<NV_, VW_>), dim3(blocks_for(a.n_items)), dim3(256), 0, st,
                                        reinterpret_cast<const int4*>(a.items), a.n_items, a.F, a.arg, a.lda,
                                        a.X, a.ldx, a.out, a.ldo);
    });
    return hipGetLastError();
}

}  // namespace sir
