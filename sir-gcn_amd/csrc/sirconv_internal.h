// Internal declarations shared by the kernel TU and the C-ABI TU (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sirconv_dropout.h"

namespace sir {

enum { AGG_SUM = 0, AGG_MEAN = 1, AGG_SYM = 2 };
enum { ACT_IDENTITY = 0, ACT_RELU = 1, ACT_LEAKY = 2, ACT_GELU = 3, ACT_GELU_TANH = 4 };
enum { MODE_FWD = 0, MODE_BWD_DST = 1, MODE_BWD_SRC = 2 };
enum { ST_F32 = 0, ST_BF16 = 1, ST_F16 = 2 };     // feature storage dtype (SIR_DTYPE_*)

// Feature pointers carry the storage dtype of the call (ST_*); norms and partial rows are fp32.
struct EdgeArgs {
    const int* rowptr;
    const int* col;
    const int32_t* items;
    int64_t n_items;
    const void* R;  int64_t ldr;      // row-side features
    const void* C;  int64_t ldc;      // gathered (col-side) features
    const void* G;  int64_t ldg;      // gradient rows (row-side for BWD_DST, gathered for BWD_SRC)
    const float* norm_row;
    const float* norm_col;
    float slope;
    int H;
    void* out;  int64_t ldo;
    float* partial;
    void* Gm;  int64_t ldgm;
    uint64_t* mask_out;          // forward: write the sign mask (ReLU family, full-wave rows)
    const uint64_t* mask_in;     // backward: sign-mask mode (Q/K not read)
    const int* perm;             // BWD_SRC mask mode: src-CSR position -> dst-CSR position
    Drop drop;                   // backward passes: feature dropout on the output rows (sirconv_dropout.h)
    int accumulate;              // forward: out[v] = out[v] + sum (rows of the items only; segmented forward)
};

struct Shape {
    int lpr, nv, vw;   // lanes per row, float-vectors per lane, floats per vector
};

// one TU per (pass, storage dtype) instantiates these (parallel builds)
template <int ST, int MODE>
hipError_t launch_edge_pass(const EdgeArgs& a, int agg, int act, Shape s, hipStream_t st);
#define SIR_DECL_PASS(ST_, MODE_) \
    template <> hipError_t launch_edge_pass<ST_, MODE_>(const EdgeArgs&, int, int, Shape, hipStream_t);
SIR_DECL_PASS(ST_F32, MODE_FWD) SIR_DECL_PASS(ST_F32, MODE_BWD_DST) SIR_DECL_PASS(ST_F32, MODE_BWD_SRC)
SIR_DECL_PASS(ST_BF16, MODE_FWD) SIR_DECL_PASS(ST_BF16, MODE_BWD_DST) SIR_DECL_PASS(ST_BF16, MODE_BWD_SRC)
SIR_DECL_PASS(ST_F16, MODE_FWD) SIR_DECL_PASS(ST_F16, MODE_BWD_DST) SIR_DECL_PASS(ST_F16, MODE_BWD_SRC)
#undef SIR_DECL_PASS
// both sign-mask backward passes in one launch (a = destination pass, b = source pass)
template <int ST>
hipError_t launch_edge_dual(const EdgeArgs& a, const EdgeArgs& b, int agg, int act, Shape s, hipStream_t st);
template <> hipError_t launch_edge_dual<ST_F32>(const EdgeArgs&, const EdgeArgs&, int, int, Shape, hipStream_t);
template <> hipError_t launch_edge_dual<ST_BF16>(const EdgeArgs&, const EdgeArgs&, int, int, Shape, hipStream_t);
template <> hipError_t launch_edge_dual<ST_F16>(const EdgeArgs&, const EdgeArgs&, int, int, Shape, hipStream_t);
hipError_t run_edge_dual(int dtype, const EdgeArgs& a, const int32_t* splits, int64_t n_splits,
                         const EdgeArgs& b, const int32_t* splits_s, int64_t n_splits_s,
                         int agg, int act, hipStream_t st, const char** why);

// edge-materialised (generic) path, sirconv_generic.hip
struct GenericArgs {
    const int* rowptr;
    const int* col;
    const int* perm;
    const int32_t* items;
    int64_t n_items;
    const int32_t* splits;
    int64_t n_splits;
    int F;
    const float* X;  int64_t ldx;
    const float* X2; int64_t ldx2;
    const float* norm_row;
    const float* norm_col;
    int mean;
    float* out;  int64_t ldo;
    float* partial;
    int* arg;  int64_t lda;
    int* parg;
};

hipError_t run_gather_add(const GenericArgs& a, hipStream_t st, int act = ACT_IDENTITY, float slope = 0.f,
                          uint64_t* smask = nullptr);
hipError_t run_seg_sum(const GenericArgs& a, hipStream_t st);
hipError_t run_edge_bcast(const GenericArgs& a, hipStream_t st);
hipError_t run_seg_max(const GenericArgs& a, hipStream_t st);
hipError_t run_seg_max_bwd(const GenericArgs& a, hipStream_t st);

hipError_t run_resid_act_fwd(const void* Y, int64_t ldy, int dtype, const float* R, int64_t ldr, float* O, int64_t ldo,
                             int64_t M, int N, int act, float slope, int order, hipStream_t st);
hipError_t run_resid_act_bwd(const float* D, int64_t ldd, const float* D2, int64_t ldd2, const void* Y, int64_t ldy,
                             int dtype, const float* R, int64_t ldr, void* DY, int64_t lddy, float* DR, int64_t lddr,
                             int64_t M, int N, int act, float slope, int order, hipStream_t st);
hipError_t run_graph_norm_fwd(const int64_t* off, int64_t B, int F, const float* X, int64_t ldx,
                              const float* w, const float* bias, const float* ms, float eps, int act, float slope,
                              const float* R, int64_t ldr, float* Y, int64_t ldy, float* mean, float* sd,
                              hipStream_t st);
hipError_t run_graph_norm_bwd(const int64_t* off, int64_t B, int F, const float* X, int64_t ldx,
                              const float* dY, int64_t ldg, const float* w, const float* bias, const float* ms,
                              const float* mean, const float* sd, int act, float slope, float* dX, int64_t lddx,
                              float* dw_part, float* dms_part, float* db_part, hipStream_t st);

hipError_t run_degree_norms(const int* rowptr_a, float* norm_a, const int* rowptr_b, float* norm_b,
                            int64_t n, hipStream_t st);

hipError_t run_colsum(const float* X, int64_t ld, int64_t n_rows, int n_cols, float* out,
                      float* workspace, int nb, hipStream_t st);

hipError_t run_edge(int mode, int dtype, const EdgeArgs& a, int agg, int act,
                    const int32_t* splits, int64_t n_splits, void* out_final, int64_t ld_final,
                    bool mean_div, hipStream_t st, const char** why);

int64_t csr_build_workspace(int64_t n_rows, int64_t E);
hipError_t run_csr_build(const int64_t* rows, const int64_t* cols, int64_t E, int64_t n_rows, int64_t n_cols,
                         int chunk, int* rowptr, int* col, int64_t* eid, int32_t* items, int32_t* splits,
                         int64_t* counts, void* ws, int64_t ws_bytes, hipStream_t st);
hipError_t run_csr_perm(const int64_t* eid_a, const int64_t* eid_b, int64_t E, int* pos_ws, int* perm,
                        hipStream_t st);

// per-edge dense layer fused with the gather and the reduce, sirconv_edgemlp.hip
struct EdgeMlpArgs {
    const int* rowptr;
    const int* col;
    const int32_t* items;
    int64_t n_items;
    const int32_t* splits;
    int64_t n_splits;
    const float* Q;  int64_t ldq;
    const float* K;  int64_t ldk;
    const float* G;  int64_t ldg;        // backward: dS rows (destination pass) / G or Gm rows (source pass)
    const float* norm_row;
    const float* norm_col;
    float slope;                        // act1's LeakyReLU slope
    int H, HP, F;                       // a width, a width padded to 8, output width
    const void* Wp;                     // packed W (run_mlp_pack)
    const float* W;                     // W [F, H] row-major (backward)
    const float* bias;                  // [F] or NULL
    float* out;  int64_t ldo;           // forward: [rows, F]; backward: dQ / dK [rows, H]
    int* arg;  int64_t lda;             // MAX: forward output / backward input (first arg-max edges)
    const int* perm;                    // MAX backward, source pass: source-CSR position -> dst-CSR position
    float* pval;                        // split partials (values)
    int* parg;                          // split partials (MAX args)
    float* Gm;                          // backward destination pass, MEAN: g / deg rows [rows, F]
    float* wpart;                       // backward destination pass: per-wave partial [dW | db]
    // edge-stream forward (run_mlp_fwd_stream): the destination row of every dst-CSR edge, sizes, and
    // the per-block boundary slots (mlp_stream_work_bytes)
    const int* erow;
    int64_t n_rows, n_edges;
    void* work;
    // forward: storage type of Q / K (ST_F32, or ST_BF16 / ST_F16 with the 16-bit weight of run_mlp_pack_st:
    // max reduce, act2 = identity only; Q / K then point at 16-bit rows)
    int st = 0;
};
int64_t mlp_stream_work_bytes(int F);
hipError_t run_mlp_fwd_stream(const EdgeMlpArgs& a, int red, int act1, int act2, hipStream_t st);
int64_t mlp_pack_floats(int H, int F);
hipError_t run_mlp_pack(const float* W, int H, int F, void* packed, hipStream_t st);
hipError_t run_mlp_pack_st(const float* W, int H, int F, int dtype, void* packed, hipStream_t st);
hipError_t run_mlp_fwd(const EdgeMlpArgs& a, int red, int act1, int act2, hipStream_t st);
int mlp_bwd_blocks(int64_t n_items, int H, int F);
hipError_t run_mlp_bwd(const EdgeMlpArgs& a, bool dst, int red, int act1, int act2, hipStream_t st);

// agg_type='max' backward from the arg-max routing (sirconv_maxbwd.hip): no [E, *] tensor
struct MaxBwdArgs {
    const int* rowptr_d; const int* col_d; const int32_t* items_d; int64_t n_items_d;
    const int32_t* splits_d; int64_t n_splits_d;
    const int* col_s; const int32_t* items_s; int64_t n_items_s; const int32_t* splits_s; int64_t n_splits_s;
    const int* pinv;                    // dst-CSR position -> src-CSR position
    int H, O; int64_t V;                // V = destination rows
    const float* Q; int64_t ldq; const float* K; int64_t ldk;
    const float* dY; int64_t ldy; const int* arg; int64_t lda;
    int act1; float slope; const float* W;
    float* dQ; int64_t lddq; float* dK; int64_t lddk;
    float* partial;                     // split rows: max(n_slots) * H
    void* ent;                          // int2 [V * O]
    void* ecnt_d; void* ecnt_s;         // int2 [E] each
    float* dbpart; int64_t route_blocks;   // [route_blocks, O]
    float* wpart;                       // [maxb_dw_ranges(V), O, H]
};
int64_t maxb_dw_ranges(int64_t V);
int64_t max_dw_rows_ranges(int64_t V, int H);
hipError_t run_max_dw_qk(const int* rowptr, const int* col, int64_t V, const int* arg, int64_t lda, const float* dY,
                         int64_t ldy, const float* Q, int64_t ldq, const float* K, int64_t ldk, int O, int H, int act1,
                         float slope, float* wpart, int64_t ldw, hipStream_t st);
hipError_t run_max_dw_rows(const int* rowptr, int64_t V, const int* arg, int64_t lda, const float* dY, int64_t ldy,
                           const float* A, int64_t ldA, int O, int H, float* wpart, int64_t ldw, hipStream_t st);
hipError_t run_max_bwd_sparse(const MaxBwdArgs& a, hipStream_t st);

// projection GEMMs, sirconv_gemm.hip
int64_t gemm_pack_bytes(int64_t N, int64_t K);
hipError_t run_gemm_pack(const float* W, int64_t ldw, int N, int K, int trans, void* packed, hipStream_t st);
hipError_t run_gemm_nt(const float* A, int64_t lda, int64_t M, int K, const void* packed, int N,
                       const float* bias, float* C, int64_t ldc, hipStream_t st, const Drop& drop = Drop(),
                       const float* gate = nullptr, int gate_relu = 0, float gate_slope = 0.f,
                       const uint64_t* gate_mask = nullptr);
hipError_t run_gemm_nt_direct(const float* A, int64_t lda, int64_t M, int K, const float* W, int64_t ldw, int trans,
                              int N, const float* bias, float* C, int64_t ldc, hipStream_t st, const Drop& drop,
                              const float* W2 = nullptr, int64_t ldw2 = 0, int64_t split = 0,
                              int64_t bias_cols = INT64_MAX);
int64_t gemm_tn_workspace(int64_t R, int64_t Mc, int64_t Nc);
hipError_t run_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t R, int Mc, int Nc,
                       float* C, int64_t ldc, float* colsum, void* workspace, hipStream_t st);
int gemm_tn_splits(int64_t R, int64_t Mc, int64_t Nc);
int64_t gemm_pack_npad(int64_t N);
// C = sum_p part[p] (count elements of rows of Nc, C row stride ldc), p in order
hipError_t run_gemm_reduce(const float* part, int P, int64_t count, int Nc, float* C, int64_t ldc, hipStream_t st);
// 16-bit TN GEMM (sirconv_gemm16.hip): A, B bf16 (dtype SIR_DTYPE_BF16) or fp16, fp32 result
hipError_t run_gemm_tn16(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t R, int Mc, int Nc, int dtype,
                         float* C, int64_t ldc, float* colsum, void* workspace, hipStream_t st);
// 16-bit NT GEMM (sirconv_gemm16.hip): packed 16-bit weights, A 16-bit or fp32, C 16-bit or fp32
int64_t gemm_pack16_bytes(int64_t N, int64_t K);
hipError_t run_gemm_pack16(const float* W, int64_t ldw, int N, int K, int trans, int dtype, void* packed, hipStream_t st);
hipError_t run_gemm_nt16(const void* A, int64_t lda, int a_dtype, int64_t M, int K, const void* packed, int N, int dtype,
                         const float* bias, void* C, int64_t ldc, int c_dtype, void* Acopy, int64_t ldac, hipStream_t st,
                         const Drop& drop = Drop());
// feature dropout applied in place to an [M, N] block of QK (the forward of paths whose QK GEMM
// is not native): X[m][n] = keep(m, col0 + n) ? X[m][n] * scale : 0, storage dtype SIR_DTYPE_*
hipError_t run_dropout_apply(void* X, int64_t ldx, int64_t M, int N, int dtype, const Drop& drop, hipStream_t st);

// compute units of the current device (persistent-grid sizing), queried once per device: the
// attribute query is not free and the launch paths run it on every call otherwise
inline int device_cu_count() {
    static int cached[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
    if (dev < 64 && cached[dev] > 0) return cached[dev];
    int ncu = 256;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
    if (dev < 64) cached[dev] = ncu;
    return ncu;
}

}  // namespace sir
