// sirconv_abi.cpp — the extern "C" boundary declared in include/sirconv.h.
//
// Synchronous argument checks, then asynchronous launches on the caller's stream (the edge
// kernel, plus the split-row combine when the plan has split rows).  No allocation, no device
// sync, no hipSetDevice: the caller (the Python host layer) selects the device and owns every
// buffer.
#include <hip/hip_runtime.h>

#include <climits>
#include <string>

#include "sirconv.h"
#include "sirconv_internal.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fn, const char* msg) {
    g_last_error = std::string(fn) + ": " + msg;
    return code;
}

int check_common(const char* fn, const int32_t* rowptr, const int32_t* col, const int32_t* items,
                 int64_t n_items, const int32_t* splits, int64_t n_splits, int64_t H, int dtype,
                 int agg, int act, const float* norm_row, const float* norm_col, const void* out,
                 const float* partial) {
    if (dtype != SIR_DTYPE_F32 && dtype != SIR_DTYPE_BF16 && dtype != SIR_DTYPE_F16)
        return fail(SIR_EINVAL, fn, "dtype must be SIR_DTYPE_F32, _BF16 or _F16");
    if (agg < SIR_AGG_SUM || agg > SIR_AGG_SYM) return fail(SIR_EINVAL, fn, "agg must be SUM, MEAN or SYM");
    if (act < SIR_ACT_IDENTITY || act > SIR_ACT_GELU_TANH) return fail(SIR_EINVAL, fn, "unknown activation");
    if (H <= 0 || H > 1024) return fail(SIR_EINVAL, fn, "H must be in [1, 1024]");
    if (n_items < 0 || n_splits < 0) return fail(SIR_EINVAL, fn, "negative item/split count");
    if (n_items > 0 && (rowptr == nullptr || items == nullptr || out == nullptr))
        return fail(SIR_EINVAL, fn, "rowptr/items/output must be non-NULL");
    (void)col;  // may be NULL exactly when the graph has no edges (every item is empty)
    if (n_splits > 0 && (splits == nullptr || partial == nullptr))
        return fail(SIR_EINVAL, fn, "split rows need `splits` and a `partial` workspace");
    if (agg == SIR_AGG_SYM && n_items > 0 && (norm_row == nullptr || norm_col == nullptr))
        return fail(SIR_EINVAL, fn, "SYM needs norm_row and norm_col");
    return SIR_OK;
}

int check_mask(const char* fn, int64_t H, int act) {
    if (sir_mask_words(H, act) == 0)
        return fail(SIR_EUNSUPPORTED, fn, "sign mask needs act RELU/LEAKY_RELU, H % 4 == 0 and H <= 1024");
    return SIR_OK;
}

// the kernels' Drop of an ABI dropout argument (NULL / p <= 0: none); col0 = first QK column written
sir::Drop to_drop(const sir_dropout_t* d, int64_t col0) {
    if (d == nullptr || !(d->p > 0.0)) return sir::Drop();
    return sir::make_drop(d->p, d->seed, (int)col0, d->seed_ptr);
}

int finish(const char* fn, hipError_t err, const char* why) {
    if (err == hipSuccess) return SIR_OK;
    if (err == hipErrorInvalidValue && why) return fail(SIR_EUNSUPPORTED, fn, why);
    if (err == hipErrorInvalidValue)
        return fail(SIR_EUNSUPPORTED, fn, "sign-mask mode needs 16-B aligned full-wave rows");
    return fail(SIR_ELAUNCH, fn, hipGetErrorString(err));
}

}  // namespace

extern "C" {

int sir_abi_version(void) { return SIR_ABI_VERSION; }

#ifndef SIR_SRC_HASH
#define SIR_SRC_HASH "unknown"
#endif
const char* sir_source_hash(void) { return SIR_SRC_HASH; }

const char* sir_last_error(void) { return g_last_error.c_str(); }

int64_t sir_mask_words(int64_t H, int act) {
    if (act != SIR_ACT_RELU && act != SIR_ACT_LEAKY_RELU) return 0;
    if (H % 4 != 0 || H <= 0 || H > 1024) return 0;
    if (H > 128) return 4 * ((H + 255) / 256);       // full-wave rows: one 64-bit ballot per 256 features x 4 slots
    // sub-wave rows (LPR = 4, 8, 16, 32 lanes of float4): an H-bit record, at least 8 bytes
    const int64_t hc = H / 4;
    const int64_t lpr = hc <= 4 ? 4 : (hc <= 8 ? 8 : (hc <= 16 ? 16 : 32));
    return lpr >= 16 ? lpr / 16 : 1;
}

int sir_degree_norms(const int32_t* rowptr_dst, float* in_norm,
                     const int32_t* rowptr_src, float* out_norm, int64_t n, void* stream) {
    const char* fn = "sir_degree_norms";
    if (n < 0) return fail(SIR_EINVAL, fn, "negative node count");
    if (n > 0 && (rowptr_dst == nullptr || in_norm == nullptr)) return fail(SIR_EINVAL, fn, "NULL rowptr/norm");
    if ((rowptr_src == nullptr) != (out_norm == nullptr)) return fail(SIR_EINVAL, fn, "rowptr_src/out_norm pairing");
    hipError_t err = sir::run_degree_norms(rowptr_dst, in_norm, rowptr_src, out_norm, n,
                                           static_cast<hipStream_t>(stream));
    return finish(fn, err, nullptr);
}

int sir_col_sum(const float* X, int64_t ld, int64_t n_rows, int64_t n_cols, float* out,
                float* workspace, void* stream) {
    const char* fn = "sir_col_sum";
    if (n_rows < 0 || n_cols < 0 || n_cols > (1 << 20)) return fail(SIR_EINVAL, fn, "bad shape");
    if (n_cols % 4 != 0 || ld % 4 != 0 || ld < n_cols) return fail(SIR_EINVAL, fn, "n_cols and ld must be multiples of 4, ld >= n_cols");
    if (n_cols > 0 && (out == nullptr || workspace == nullptr || (n_rows > 0 && X == nullptr)))
        return fail(SIR_EINVAL, fn, "NULL buffer");
    if ((reinterpret_cast<uintptr_t>(X) & 15u) != 0) return fail(SIR_EINVAL, fn, "X must be 16-B aligned");
    hipError_t err = sir::run_colsum(X, ld, n_rows, (int)n_cols, out, workspace, SIR_COLSUM_BLOCKS,
                                     static_cast<hipStream_t>(stream));
    return finish(fn, err, nullptr);
}

int sir_edge_agg_fwd(const int32_t* rowptr, const int32_t* col,
                     const int32_t* items, int64_t n_items,
                     const int32_t* splits, int64_t n_splits,
                     int64_t H, int dtype,
                     const void* Q, int64_t ldq, const void* K, int64_t ldk,
                     const float* norm_row, const float* norm_col,
                     int agg, int act, float slope,
                     void* S, int64_t lds, uint64_t* mask_out, float* partial, void* stream) {
    const char* fn = "sir_edge_agg_fwd";
    const int accumulate = (agg & SIR_AGG_ACCUMULATE) != 0;
    agg &= ~SIR_AGG_ACCUMULATE;
    if (accumulate && agg == SIR_AGG_MEAN)
        return fail(SIR_EUNSUPPORTED, fn, "SIR_AGG_ACCUMULATE: segment sums of SUM / SYM only (divide afterwards for MEAN)");
    int rc = check_common(fn, rowptr, col, items, n_items, splits, n_splits, H, dtype, agg, act,
                          norm_row, norm_col, S, partial);
    if (rc) return rc;
    if (ldq < H || ldk < H || lds < H) return fail(SIR_EINVAL, fn, "leading dimensions must be >= H");
    if (n_items > 0 && (Q == nullptr || K == nullptr)) return fail(SIR_EINVAL, fn, "Q/K must be non-NULL");
    if (mask_out != nullptr && (rc = check_mask(fn, H, act))) return rc;
    sir::EdgeArgs a{};
    a.rowptr = rowptr; a.col = col; a.items = items; a.n_items = n_items;
    a.R = Q; a.ldr = ldq;
    a.C = K; a.ldc = ldk;
    a.G = nullptr; a.ldg = H;
    a.norm_row = norm_row; a.norm_col = norm_col; a.slope = slope; a.H = (int)H;
    a.out = S; a.ldo = lds; a.partial = partial; a.Gm = nullptr; a.ldgm = H;
    a.mask_out = mask_out;
    a.accumulate = accumulate;
    const char* why = nullptr;
    hipError_t err = sir::run_edge(sir::MODE_FWD, dtype, a, agg, act, splits, n_splits, S, lds,
                                   agg == SIR_AGG_MEAN, static_cast<hipStream_t>(stream), &why);
    return finish(fn, err, why);
}

int sir_edge_agg_bwd_dst(const int32_t* rowptr, const int32_t* col,
                         const int32_t* items, int64_t n_items,
                         const int32_t* splits, int64_t n_splits,
                         int64_t H, int dtype,
                         const void* Q, int64_t ldq, const void* K, int64_t ldk,
                         const uint64_t* mask,
                         const void* G, int64_t ldg,
                         const float* norm_row, const float* norm_col,
                         int agg, int act, float slope,
                         void* dQ, int64_t lddq, void* Gm, int64_t ldgm,
                         float* partial, const sir_dropout_t* drop, void* stream) {
    const char* fn = "sir_edge_agg_bwd_dst";
    int rc = check_common(fn, rowptr, col, items, n_items, splits, n_splits, H, dtype, agg, act,
                          norm_row, norm_col, dQ, partial);
    if (rc) return rc;
    if (ldg < H || lddq < H) return fail(SIR_EINVAL, fn, "leading dimensions must be >= H");
    if (Gm != nullptr && ldgm < H) return fail(SIR_EINVAL, fn, "ldgm must be >= H");
    if (n_items > 0 && G == nullptr) return fail(SIR_EINVAL, fn, "G must be non-NULL");
    if (mask != nullptr) {
        if ((rc = check_mask(fn, H, act))) return rc;
    } else {
        if (ldq < H || ldk < H) return fail(SIR_EINVAL, fn, "leading dimensions must be >= H");
        if (n_items > 0 && (Q == nullptr || K == nullptr)) return fail(SIR_EINVAL, fn, "Q/K must be non-NULL");
    }
    sir::EdgeArgs a{};
    a.rowptr = rowptr; a.col = col; a.items = items; a.n_items = n_items;
    a.R = Q; a.ldr = mask ? H : ldq;
    a.C = K; a.ldc = mask ? H : ldk;
    a.G = G; a.ldg = ldg;
    a.norm_row = norm_row; a.norm_col = norm_col; a.slope = slope; a.H = (int)H;
    a.out = dQ; a.ldo = lddq; a.partial = partial;
    a.Gm = (agg == SIR_AGG_MEAN) ? Gm : nullptr; a.ldgm = Gm ? ldgm : H;
    a.mask_in = mask;
    a.drop = to_drop(drop, 0);              // dQ = QK columns 0 .. H-1
    const char* why = nullptr;
    hipError_t err = sir::run_edge(sir::MODE_BWD_DST, dtype, a, agg, act, splits, n_splits, dQ, lddq, false,
                                   static_cast<hipStream_t>(stream), &why);
    return finish(fn, err, why);
}

int sir_edge_agg_bwd_src(const int32_t* rowptr_s, const int32_t* col_s, const int32_t* perm_s,
                         const int32_t* items, int64_t n_items,
                         const int32_t* splits, int64_t n_splits,
                         int64_t H, int dtype,
                         const void* K, int64_t ldk, const void* Q, int64_t ldq,
                         const uint64_t* mask,
                         const void* Gd, int64_t ldg,
                         const float* norm_row, const float* norm_col,
                         int agg, int act, float slope,
                         void* dK, int64_t lddk, float* partial, const sir_dropout_t* drop, void* stream) {
    const char* fn = "sir_edge_agg_bwd_src";
    int rc = check_common(fn, rowptr_s, col_s, items, n_items, splits, n_splits, H, dtype, agg, act,
                          norm_row, norm_col, dK, partial);
    if (rc) return rc;
    if (ldg < H || lddk < H) return fail(SIR_EINVAL, fn, "leading dimensions must be >= H");
    if (n_items > 0 && Gd == nullptr) return fail(SIR_EINVAL, fn, "Gd must be non-NULL");
    if (mask != nullptr) {
        if ((rc = check_mask(fn, H, act))) return rc;
        if (n_items > 0 && col_s != nullptr && perm_s == nullptr) return fail(SIR_EINVAL, fn, "sign-mask mode needs perm_s");
    } else {
        if (ldq < H || ldk < H) return fail(SIR_EINVAL, fn, "leading dimensions must be >= H");
        if (n_items > 0 && (Q == nullptr || K == nullptr)) return fail(SIR_EINVAL, fn, "K/Q must be non-NULL");
    }
    sir::EdgeArgs a{};
    a.rowptr = rowptr_s; a.col = col_s; a.items = items; a.n_items = n_items;
    a.R = K; a.ldr = mask ? H : ldk;
    a.C = Q; a.ldc = mask ? H : ldq;
    a.G = Gd; a.ldg = ldg;
    a.norm_row = norm_row; a.norm_col = norm_col; a.slope = slope; a.H = (int)H;
    a.out = dK; a.ldo = lddk; a.partial = partial; a.Gm = nullptr; a.ldgm = H;
    a.mask_in = mask; a.perm = perm_s;
    a.drop = to_drop(drop, H);              // dK = QK columns H .. 2H-1
    const char* why = nullptr;
    hipError_t err = sir::run_edge(sir::MODE_BWD_SRC, dtype, a, agg, act, splits, n_splits, dK, lddk, false,
                                   static_cast<hipStream_t>(stream), &why);
    return finish(fn, err, why);
}

int sir_edge_agg_bwd(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                     const int32_t* splits, int64_t n_splits,
                     const int32_t* rowptr_s, const int32_t* col_s, const int32_t* perm_s,
                     const int32_t* items_s, int64_t n_items_s, const int32_t* splits_s, int64_t n_splits_s,
                     int64_t H, int dtype, const uint64_t* mask, const void* G, int64_t ldg,
                     const float* in_norm, const float* out_norm, int agg, int act, float slope,
                     void* dQ, int64_t lddq, void* dK, int64_t lddk, float* partial, float* partial_s,
                     const sir_dropout_t* drop, void* stream) {
    const char* fn = "sir_edge_agg_bwd";
    int rc = check_common(fn, rowptr, col, items, n_items, splits, n_splits, H, dtype, agg, act, in_norm, out_norm,
                          dQ, partial);
    if (rc) return rc;
    rc = check_common(fn, rowptr_s, col_s, items_s, n_items_s, splits_s, n_splits_s, H, dtype, agg, act, out_norm,
                      in_norm, dK, partial_s);
    if (rc) return rc;
    if (agg == SIR_AGG_MEAN)
        return fail(SIR_EUNSUPPORTED, fn, "MEAN: the source pass needs the destination pass's Gm (two calls)");
    if (mask == nullptr) return fail(SIR_EINVAL, fn, "the one-launch backward is the sign-mask mode: mask required");
    if ((rc = check_mask(fn, H, act))) return rc;
    if (ldg < H || lddq < H || lddk < H) return fail(SIR_EINVAL, fn, "leading dimensions must be >= H");
    if ((n_items > 0 || n_items_s > 0) && G == nullptr) return fail(SIR_EINVAL, fn, "G must be non-NULL");
    if (n_items_s > 0 && col_s != nullptr && perm_s == nullptr) return fail(SIR_EINVAL, fn, "sign-mask mode needs perm_s");
    if (n_items > INT32_MAX || n_items_s > INT32_MAX || n_items + n_items_s > (int64_t)INT32_MAX)
        return fail(SIR_EINVAL, fn, "too many work items for one launch");
    sir::EdgeArgs a{};
    a.rowptr = rowptr; a.col = col; a.items = items; a.n_items = n_items;
    a.G = G; a.ldg = ldg; a.norm_row = in_norm; a.norm_col = out_norm; a.slope = slope; a.H = (int)H;
    a.out = dQ; a.ldo = lddq; a.partial = partial; a.mask_in = mask; a.ldr = H; a.ldc = H; a.ldgm = H;
    sir::EdgeArgs b{};
    b.rowptr = rowptr_s; b.col = col_s; b.perm = perm_s; b.items = items_s; b.n_items = n_items_s;
    b.G = G; b.ldg = ldg; b.norm_row = out_norm; b.norm_col = in_norm; b.slope = slope; b.H = (int)H;
    b.out = dK; b.ldo = lddk; b.partial = partial_s; b.mask_in = mask; b.ldr = H; b.ldc = H; b.ldgm = H;
    a.drop = to_drop(drop, 0);
    b.drop = to_drop(drop, H);
    const char* why = nullptr;
    hipError_t err = sir::run_edge_dual(dtype, a, splits, n_splits, b, splits_s, n_splits_s, agg, act,
                                        static_cast<hipStream_t>(stream), &why);
    return finish(fn, err, why);
}

// ------------------------------------------------------------------------------ generic path
static int check_generic(const char* fn, int64_t n_items, int64_t F, const int32_t* items) {
    if (F <= 0 || F > 1024) return fail(SIR_EINVAL, fn, "F must be in [1, 1024]");
    if (n_items < 0) return fail(SIR_EINVAL, fn, "negative item count");
    if (n_items > 0 && items == nullptr) return fail(SIR_EINVAL, fn, "NULL items");
    return SIR_OK;
}

int sir_edge_gather_add(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                        int64_t F, const float* Q, int64_t ldq, const float* K, int64_t ldk,
                        float* Z, int64_t ldz, void* stream) {
    const char* fn = "sir_edge_gather_add";
    int rc = check_generic(fn, n_items, F, items);
    if (rc) return rc;
    if (ldq < F || ldk < F || ldz < F) return fail(SIR_EINVAL, fn, "leading dimensions must be >= F");
    if (n_items > 0 && (Q == nullptr || K == nullptr)) return fail(SIR_EINVAL, fn, "NULL Q/K");
    sir::GenericArgs a{};
    a.rowptr = rowptr; a.col = col; a.items = items; a.n_items = n_items; a.F = (int)F;
    a.X = Q; a.ldx = ldq; a.X2 = K; a.ldx2 = ldk; a.out = Z; a.ldo = ldz;
    return finish(fn, sir::run_gather_add(a, static_cast<hipStream_t>(stream)), "unsupported F / alignment");
}

int sir_edge_gather_act(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                        int64_t F, const float* Q, int64_t ldq, const float* K, int64_t ldk, int act, float slope,
                        float* A, int64_t lda, uint64_t* sign_mask, void* stream) {
    const char* fn = "sir_edge_gather_act";
    int rc = check_generic(fn, n_items, F, items);
    if (rc) return rc;
    if (act != SIR_ACT_IDENTITY && act != SIR_ACT_RELU && act != SIR_ACT_LEAKY_RELU)
        return fail(SIR_EINVAL, fn, "act must be identity, ReLU or LeakyReLU");
    if (ldq < F || ldk < F || lda < F) return fail(SIR_EINVAL, fn, "leading dimensions must be >= F");
    if (n_items > 0 && (Q == nullptr || K == nullptr)) return fail(SIR_EINVAL, fn, "NULL Q/K");
    sir::GenericArgs a{};
    a.rowptr = rowptr; a.col = col; a.items = items; a.n_items = n_items; a.F = (int)F;
    a.X = Q; a.ldx = ldq; a.X2 = K; a.ldx2 = ldk; a.out = A; a.ldo = lda;
    if (sign_mask != nullptr && F != 256) return fail(SIR_EUNSUPPORTED, fn, "sign_mask needs F = 256");
    return finish(fn, sir::run_gather_add(a, static_cast<hipStream_t>(stream), act, slope, sign_mask),
                  "unsupported F / alignment");
}

int sir_segment_sum(const int32_t* rowptr, const int32_t* col, const int32_t* perm,
                    const int32_t* items, int64_t n_items, const int32_t* splits, int64_t n_splits,
                    int64_t F, const float* X, int64_t ldx, const float* norm_row, const float* norm_col,
                    int mean, float* out, int64_t ldo, float* partial, void* stream) {
    const char* fn = "sir_segment_sum";
    int rc = check_generic(fn, n_items, F, items);
    if (rc) return rc;
    if (ldx < F || ldo < F) return fail(SIR_EINVAL, fn, "leading dimensions must be >= F");
    if ((norm_row == nullptr) != (norm_col == nullptr)) return fail(SIR_EINVAL, fn, "norm_row/norm_col pairing");
    if (n_splits > 0 && (splits == nullptr || partial == nullptr)) return fail(SIR_EINVAL, fn, "split rows need splits + partial");
    if (n_items > 0 && out == nullptr) return fail(SIR_EINVAL, fn, "NULL out");
    sir::GenericArgs a{};
    a.rowptr = rowptr; a.col = col; a.perm = perm; a.items = items; a.n_items = n_items;
    a.splits = splits; a.n_splits = n_splits; a.F = (int)F; a.X = X; a.ldx = ldx;
    a.norm_row = norm_row; a.norm_col = norm_col; a.mean = mean; a.out = out; a.ldo = ldo; a.partial = partial;
    return finish(fn, sir::run_seg_sum(a, static_cast<hipStream_t>(stream)), "unsupported F / alignment");
}

int sir_edge_broadcast(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                       int64_t F, const float* dS, int64_t lds, const float* norm_row, const float* norm_col,
                       int mean, float* dM, int64_t ldm, void* stream) {
    const char* fn = "sir_edge_broadcast";
    int rc = check_generic(fn, n_items, F, items);
    if (rc) return rc;
    if (lds < F || ldm < F) return fail(SIR_EINVAL, fn, "leading dimensions must be >= F");
    if ((norm_row == nullptr) != (norm_col == nullptr)) return fail(SIR_EINVAL, fn, "norm_row/norm_col pairing");
    if (mean && rowptr == nullptr && n_items > 0) return fail(SIR_EINVAL, fn, "mean needs rowptr");
    sir::GenericArgs a{};
    a.rowptr = rowptr; a.col = col; a.items = items; a.n_items = n_items; a.F = (int)F;
    a.X = dS; a.ldx = lds; a.norm_row = norm_row; a.norm_col = norm_col; a.mean = mean; a.out = dM; a.ldo = ldm;
    return finish(fn, sir::run_edge_bcast(a, static_cast<hipStream_t>(stream)), "unsupported F / alignment");
}

int sir_segment_max(const int32_t* items, int64_t n_items, const int32_t* splits, int64_t n_splits,
                    int64_t F, const float* M, int64_t ldm, float* Y, int64_t ldy, int32_t* arg, int64_t lda,
                    float* pval, int32_t* parg, void* stream) {
    const char* fn = "sir_segment_max";
    int rc = check_generic(fn, n_items, F, items);
    if (rc) return rc;
    if (ldm < F || ldy < F || lda < F) return fail(SIR_EINVAL, fn, "leading dimensions must be >= F");
    if (n_splits > 0 && (splits == nullptr || pval == nullptr || parg == nullptr))
        return fail(SIR_EINVAL, fn, "split rows need splits + pval + parg");
    sir::GenericArgs a{};
    a.items = items; a.n_items = n_items; a.splits = splits; a.n_splits = n_splits; a.F = (int)F;
    a.X = M; a.ldx = ldm; a.out = Y; a.ldo = ldy; a.arg = arg; a.lda = lda; a.partial = pval; a.parg = parg;
    return finish(fn, sir::run_seg_max(a, static_cast<hipStream_t>(stream)), "unsupported F / alignment");
}

int sir_segment_max_bwd(const int32_t* items, int64_t n_items, int64_t F, const int32_t* arg, int64_t lda,
                        const float* dY, int64_t ldy, float* dM, int64_t ldm, void* stream) {
    const char* fn = "sir_segment_max_bwd";
    int rc = check_generic(fn, n_items, F, items);
    if (rc) return rc;
    if (ldm < F || ldy < F || lda < F) return fail(SIR_EINVAL, fn, "leading dimensions must be >= F");
    sir::GenericArgs a{};
    a.items = items; a.n_items = n_items; a.F = (int)F; a.arg = const_cast<int*>(arg); a.lda = lda;
    a.X = dY; a.ldx = ldy; a.out = dM; a.ldo = ldm;
    return finish(fn, sir::run_seg_max_bwd(a, static_cast<hipStream_t>(stream)), "unsupported F / alignment");
}

// ------------------------------------------------------------------------------ fused per-edge dense layer
static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

static int check_mlp(const char* fn, const int32_t* rowptr, const int32_t* items, int64_t n_items,
                     const int32_t* splits, int64_t n_splits, int64_t H, int64_t F, const float* Q, int64_t ldq,
                     const float* K, int64_t ldk, int agg, int act1, int act2, const void* packed,
                     const float* norm_row, const float* norm_col, bool bwd, bool rows16 = false) {
    if (agg < SIR_AGG_SUM || agg > SIR_AGG_MAX || (bwd && agg == SIR_AGG_MAX))
        return fail(SIR_EINVAL, fn, bwd ? "agg must be SUM, MEAN or SYM" : "agg must be SUM, MEAN, SYM or MAX");
    if (act1 < SIR_ACT_IDENTITY || act1 > SIR_ACT_GELU_TANH) return fail(SIR_EINVAL, fn, "unknown act1");
    if (act2 != SIR_ACT_IDENTITY && act2 != SIR_ACT_RELU) return fail(SIR_EUNSUPPORTED, fn, "act2 must be IDENTITY or RELU");
    if (H <= 0 || H % 4 != 0 || H > (bwd ? 256 : 512)) return fail(SIR_EUNSUPPORTED, fn, bwd ? "H % 4 == 0 and H <= 256" : "H % 4 == 0 and H <= 512");
    if (F <= 0 || F > (bwd ? 256 : 512)) return fail(SIR_EUNSUPPORTED, fn, bwd ? "F <= 256" : "F <= 512");
    if (n_items < 0 || n_splits < 0 || n_items > INT32_MAX) return fail(SIR_EINVAL, fn, "bad item count");
    if (n_items > 0 && (rowptr == nullptr || items == nullptr || packed == nullptr || Q == nullptr || K == nullptr))
        return fail(SIR_EINVAL, fn, "NULL buffer");
    if (rows16) {      // 16-bit rows: 8-B aligned
        if (ldq < H || ldk < H || ldq % 4 || ldk % 4 || (reinterpret_cast<uintptr_t>(Q) & 7u) ||
            (reinterpret_cast<uintptr_t>(K) & 7u))
            return fail(SIR_EUNSUPPORTED, fn, "Q/K rows must be 8-B aligned (ld % 4 == 0, ld >= H)");
    } else if (ldq < H || ldk < H || ldq % 4 || ldk % 4 || !al16(Q) || !al16(K)) {
        return fail(SIR_EUNSUPPORTED, fn, "Q/K rows must be 16-B aligned (ld % 4 == 0, ld >= H)");
    }
    if (n_splits > 0 && splits == nullptr) return fail(SIR_EINVAL, fn, "NULL splits");
    if (agg == SIR_AGG_SYM && n_items > 0 && (norm_row == nullptr || norm_col == nullptr))
        return fail(SIR_EINVAL, fn, "SYM needs norm_row and norm_col");
    return SIR_OK;
}

int64_t sir_edge_mlp_pack_bytes(int64_t H, int64_t F) {
    if (H <= 0 || F <= 0 || H > 512 || F > 512) return 0;
    return sir::mlp_pack_floats((int)H, (int)F) * 4;
}

int sir_edge_mlp_pack(const float* W, int64_t H, int64_t F, void* packed, void* stream) {
    const char* fn = "sir_edge_mlp_pack";
    if (H <= 0 || F <= 0 || H > 512 || F > 512) return fail(SIR_EINVAL, fn, "H <= 512, F <= 512");
    if (W == nullptr || packed == nullptr || !al16(packed)) return fail(SIR_EINVAL, fn, "NULL / unaligned buffer");
    return finish(fn, sir::run_mlp_pack(W, (int)H, (int)F, packed, static_cast<hipStream_t>(stream)), nullptr);
}

int sir_edge_mlp_fwd(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                     const int32_t* splits, int64_t n_splits, int64_t H, int64_t F,
                     const float* Q, int64_t ldq, const float* K, int64_t ldk,
                     const float* norm_row, const float* norm_col, int agg, int act1, float slope, int act2,
                     const void* packed, const float* bias, float* out, int64_t ldo, int32_t* arg, int64_t lda,
                     float* pval, int32_t* parg, void* stream) {
    const char* fn = "sir_edge_mlp_fwd";
    int rc = check_mlp(fn, rowptr, items, n_items, splits, n_splits, H, F, Q, ldq, K, ldk, agg, act1, act2, packed,
                       norm_row, norm_col, false);
    if (rc) return rc;
    if (n_items > 0 && (out == nullptr || ldo < F)) return fail(SIR_EINVAL, fn, "out / ldo");
    if (agg == SIR_AGG_MAX && n_items > 0 && (arg == nullptr || lda < F)) return fail(SIR_EINVAL, fn, "MAX needs arg");
    if (n_splits > 0 && (pval == nullptr || (agg == SIR_AGG_MAX && parg == nullptr)))
        return fail(SIR_EINVAL, fn, "split rows need pval (and parg for MAX)");
    sir::EdgeMlpArgs a{};
    a.rowptr = rowptr; a.col = col; a.items = items; a.n_items = n_items; a.splits = splits; a.n_splits = n_splits;
    a.Q = Q; a.ldq = ldq; a.K = K; a.ldk = ldk; a.norm_row = norm_row; a.norm_col = norm_col; a.slope = slope;
    a.H = (int)H; a.HP = (int)((H + 7) / 8 * 8); a.F = (int)F; a.Wp = packed; a.bias = bias;
    a.out = out; a.ldo = ldo; a.arg = arg; a.lda = lda; a.pval = pval; a.parg = parg;
    return finish(fn, sir::run_mlp_fwd(a, agg, act1, act2, static_cast<hipStream_t>(stream)), nullptr);
}

int64_t sir_edge_mlp_stream_work_bytes(int64_t F) {
    if (F <= 0 || F > 512) return 0;
    return sir::mlp_stream_work_bytes((int)F);
}

int sir_edge_mlp_fwd_stream(const int32_t* rowptr, const int32_t* col, const int32_t* erow, int64_t n_rows,
                            int64_t n_edges, int64_t H, int64_t F, const float* Q, int64_t ldq, const float* K,
                            int64_t ldk, const float* norm_row, const float* norm_col, int agg, int act1, float slope,
                            int act2, const void* packed, const float* bias, float* out, int64_t ldo, int32_t* arg,
                            int64_t lda, void* work, void* stream) {
    const char* fn = "sir_edge_mlp_fwd_stream";
    if (H != 256 || F <= 0 || F > 256) return fail(SIR_EUNSUPPORTED, fn, "H = 256, F <= 256");
    if (n_rows < 0 || n_edges < 0 || n_edges >= INT32_MAX) return fail(SIR_EINVAL, fn, "bad sizes");
    if (agg != SIR_AGG_SUM && agg != SIR_AGG_MEAN && agg != SIR_AGG_SYM && agg != SIR_AGG_MAX)
        return fail(SIR_EINVAL, fn, "agg");
    if (act1 < SIR_ACT_IDENTITY || act1 > SIR_ACT_GELU_TANH || act2 < SIR_ACT_IDENTITY || act2 > SIR_ACT_GELU_TANH)
        return fail(SIR_EINVAL, fn, "act");
    if (n_rows > 0 && (rowptr == nullptr || out == nullptr || ldo < F || packed == nullptr || work == nullptr))
        return fail(SIR_EINVAL, fn, "NULL buffer / ldo");
    if (n_edges > 0 && (col == nullptr || erow == nullptr || Q == nullptr || K == nullptr))
        return fail(SIR_EINVAL, fn, "NULL col / erow / Q / K");
    if (ldq < H || ldk < H || ldq % 4 || ldk % 4 || !al16(Q) || !al16(K))
        return fail(SIR_EUNSUPPORTED, fn, "Q/K rows must be 16-B aligned (ld % 4 == 0, ld >= H)");
    if (agg == SIR_AGG_MAX && n_rows > 0 && (arg == nullptr || lda < F)) return fail(SIR_EINVAL, fn, "MAX needs arg");
    if (agg == SIR_AGG_SYM && n_edges > 0 && (norm_row == nullptr || norm_col == nullptr))
        return fail(SIR_EINVAL, fn, "SYM needs norm_row and norm_col");
    sir::EdgeMlpArgs a{};
    a.rowptr = rowptr; a.col = col; a.erow = erow; a.n_rows = n_rows; a.n_edges = n_edges;
    a.Q = Q; a.ldq = ldq; a.K = K; a.ldk = ldk; a.norm_row = norm_row; a.norm_col = norm_col; a.slope = slope;
    a.H = (int)H; a.HP = (int)((H + 7) / 8 * 8); a.F = (int)F; a.Wp = packed; a.bias = bias;
    a.out = out; a.ldo = ldo; a.arg = arg; a.lda = lda; a.work = work;
    return finish(fn, sir::run_mlp_fwd_stream(a, agg, act1, act2, static_cast<hipStream_t>(stream)), nullptr);
}

int sir_edge_mlp_pack_st(const float* W, int64_t H, int64_t F, int dtype, void* packed, void* stream) {
    const char* fn = "sir_edge_mlp_pack_st";
    if (H <= 0 || F <= 0 || H > 512 || F > 512) return fail(SIR_EINVAL, fn, "H <= 512, F <= 512");
    if (dtype != SIR_DTYPE_BF16 && dtype != SIR_DTYPE_F16) return fail(SIR_EINVAL, fn, "dtype must be BF16 or F16");
    if (W == nullptr || packed == nullptr || !al16(packed)) return fail(SIR_EINVAL, fn, "NULL / unaligned buffer");
    return finish(fn, sir::run_mlp_pack_st(W, (int)H, (int)F, dtype, packed, static_cast<hipStream_t>(stream)), nullptr);
}

static int check_st(const char* fn, int dtype, int agg, int act2, const void* Q, int64_t ldq, const void* K, int64_t ldk,
                    int64_t H) {
    if (dtype != SIR_DTYPE_BF16 && dtype != SIR_DTYPE_F16) return fail(SIR_EINVAL, fn, "dtype must be BF16 or F16");
    if (agg != SIR_AGG_MAX || act2 != SIR_ACT_IDENTITY)
        return fail(SIR_EUNSUPPORTED, fn, "16-bit storage: agg MAX and act2 IDENTITY only");
    if (ldq < H || ldk < H || ldq % 4 || ldk % 4 || (reinterpret_cast<uintptr_t>(Q) & 7u) ||
        (reinterpret_cast<uintptr_t>(K) & 7u))
        return fail(SIR_EUNSUPPORTED, fn, "Q/K rows must be 8-B aligned (ld % 4 == 0, ld >= H)");
    return SIR_OK;
}

int sir_edge_mlp_fwd_st(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                        const int32_t* splits, int64_t n_splits, int64_t H, int64_t F, const void* Q, int64_t ldq,
                        const void* K, int64_t ldk, int dtype, int agg, int act1, float slope, int act2,
                        const void* packed, const float* bias, float* out, int64_t ldo, int32_t* arg, int64_t lda,
                        float* pval, int32_t* parg, void* stream) {
    const char* fn = "sir_edge_mlp_fwd_st";
    int rc = check_st(fn, dtype, agg, act2, Q, ldq, K, ldk, H);
    if (rc) return rc;
    rc = check_mlp(fn, rowptr, items, n_items, splits, n_splits, H, F, static_cast<const float*>(Q), ldq,
                   static_cast<const float*>(K), ldk, agg, act1, act2, packed, nullptr, nullptr, false, true);
    if (rc) return rc;
    if (n_items > 0 && (out == nullptr || ldo < F || arg == nullptr || lda < F)) return fail(SIR_EINVAL, fn, "out / arg");
    if (n_splits > 0 && (pval == nullptr || parg == nullptr)) return fail(SIR_EINVAL, fn, "split rows need pval and parg");
    sir::EdgeMlpArgs a{};
    a.rowptr = rowptr; a.col = col; a.items = items; a.n_items = n_items; a.splits = splits; a.n_splits = n_splits;
    a.Q = static_cast<const float*>(Q); a.ldq = ldq; a.K = static_cast<const float*>(K); a.ldk = ldk;
    a.slope = slope; a.H = (int)H; a.HP = (int)((H + 7) / 8 * 8); a.F = (int)F; a.Wp = packed; a.bias = bias;
    a.out = out; a.ldo = ldo; a.arg = arg; a.lda = lda; a.pval = pval; a.parg = parg; a.st = dtype;
    return finish(fn, sir::run_mlp_fwd(a, agg, act1, act2, static_cast<hipStream_t>(stream)), nullptr);
}

int sir_edge_mlp_fwd_stream_st(const int32_t* rowptr, const int32_t* col, const int32_t* erow, int64_t n_rows,
                               int64_t n_edges, int64_t H, int64_t F, const void* Q, int64_t ldq, const void* K,
                               int64_t ldk, int dtype, int agg, int act1, float slope, int act2, const void* packed,
                               const float* bias, float* out, int64_t ldo, int32_t* arg, int64_t lda, void* work,
                               void* stream) {
    const char* fn = "sir_edge_mlp_fwd_stream_st";
    int rc = check_st(fn, dtype, agg, act2, Q, ldq, K, ldk, H);
    if (rc) return rc;
    if (H != 256 || F <= 0 || F > 256) return fail(SIR_EUNSUPPORTED, fn, "H = 256, F <= 256");
    if (n_rows < 0 || n_edges < 0 || n_edges >= INT32_MAX) return fail(SIR_EINVAL, fn, "bad sizes");
    if (act1 < SIR_ACT_IDENTITY || act1 > SIR_ACT_GELU_TANH) return fail(SIR_EINVAL, fn, "act");
    if (n_rows > 0 && (rowptr == nullptr || out == nullptr || ldo < F || packed == nullptr || work == nullptr ||
                       arg == nullptr || lda < F))
        return fail(SIR_EINVAL, fn, "NULL buffer / ldo / lda");
    if (n_edges > 0 && (col == nullptr || erow == nullptr || Q == nullptr || K == nullptr))
        return fail(SIR_EINVAL, fn, "NULL col / erow / Q / K");
    sir::EdgeMlpArgs a{};
    a.rowptr = rowptr; a.col = col; a.erow = erow; a.n_rows = n_rows; a.n_edges = n_edges;
    a.Q = static_cast<const float*>(Q); a.ldq = ldq; a.K = static_cast<const float*>(K); a.ldk = ldk;
    a.slope = slope; a.H = (int)H; a.HP = (int)((H + 7) / 8 * 8); a.F = (int)F; a.Wp = packed; a.bias = bias;
    a.out = out; a.ldo = ldo; a.arg = arg; a.lda = lda; a.work = work; a.st = dtype;
    return finish(fn, sir::run_mlp_fwd_stream(a, agg, act1, act2, static_cast<hipStream_t>(stream)), nullptr);
}

int64_t sir_edge_mlp_bwd_parts(int64_t n_items, int64_t H, int64_t F) {
    if (H <= 0 || F <= 0 || H > 256 || F > 256) return 0;
    return sir::mlp_bwd_blocks(n_items, (int)H, (int)F);
}

int sir_edge_mlp_bwd_dst(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                         const int32_t* splits, int64_t n_splits, int64_t H, int64_t F,
                         const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* G, int64_t ldg,
                         const float* norm_row, const float* norm_col, int agg, int act1, float slope, int act2,
                         const void* packed, const float* W, const float* bias, float* dQ, int64_t lddq,
                         float* Gm, float* partial, float* wpart, void* stream) {
    const char* fn = "sir_edge_mlp_bwd_dst";
    int rc = check_mlp(fn, rowptr, items, n_items, splits, n_splits, H, F, Q, ldq, K, ldk, agg, act1, act2, packed,
                       norm_row, norm_col, true);
    if (rc) return rc;
    if (n_items > 0 && (G == nullptr || ldg < F || W == nullptr || dQ == nullptr || lddq < H || wpart == nullptr))
        return fail(SIR_EINVAL, fn, "G / W / dQ / wpart");
    if (n_splits > 0 && partial == nullptr) return fail(SIR_EINVAL, fn, "split rows need partial");
    sir::EdgeMlpArgs a{};
    a.rowptr = rowptr; a.col = col; a.items = items; a.n_items = n_items; a.splits = splits; a.n_splits = n_splits;
    a.Q = Q; a.ldq = ldq; a.K = K; a.ldk = ldk; a.G = G; a.ldg = ldg; a.norm_row = norm_row; a.norm_col = norm_col;
    a.slope = slope; a.H = (int)H; a.HP = (int)((H + 7) / 8 * 8); a.F = (int)F; a.Wp = packed; a.W = W; a.bias = bias;
    a.out = dQ; a.ldo = lddq; a.pval = partial; a.Gm = (agg == SIR_AGG_MEAN) ? Gm : nullptr; a.wpart = wpart;
    return finish(fn, sir::run_mlp_bwd(a, true, agg, act1, act2, static_cast<hipStream_t>(stream)), nullptr);
}

int sir_edge_mlp_bwd_src(const int32_t* rowptr_s, const int32_t* col_s, const int32_t* items, int64_t n_items,
                         const int32_t* splits, int64_t n_splits, int64_t H, int64_t F,
                         const float* K, int64_t ldk, const float* Q, int64_t ldq, const float* Gd, int64_t ldg,
                         const float* norm_row, const float* norm_col, int agg, int act1, float slope, int act2,
                         const void* packed, const float* W, const float* bias, float* dK, int64_t lddk,
                         float* partial, void* stream) {
    const char* fn = "sir_edge_mlp_bwd_src";
    int rc = check_mlp(fn, rowptr_s, items, n_items, splits, n_splits, H, F, Q, ldq, K, ldk, agg, act1, act2, packed,
                       norm_row, norm_col, true);
    if (rc) return rc;
    if (n_items > 0 && (Gd == nullptr || ldg < F || W == nullptr || dK == nullptr || lddk < H))
        return fail(SIR_EINVAL, fn, "Gd / W / dK");
    if (n_splits > 0 && partial == nullptr) return fail(SIR_EINVAL, fn, "split rows need partial");
    sir::EdgeMlpArgs a{};
    a.rowptr = rowptr_s; a.col = col_s; a.items = items; a.n_items = n_items; a.splits = splits; a.n_splits = n_splits;
    a.Q = Q; a.ldq = ldq; a.K = K; a.ldk = ldk; a.G = Gd; a.ldg = ldg; a.norm_row = norm_row; a.norm_col = norm_col;
    a.slope = slope; a.H = (int)H; a.HP = (int)((H + 7) / 8 * 8); a.F = (int)F; a.Wp = packed; a.W = W; a.bias = bias;
    a.out = dK; a.ldo = lddk; a.pval = partial; a.wpart = nullptr;
    return finish(fn, sir::run_mlp_bwd(a, false, agg, act1, act2, static_cast<hipStream_t>(stream)), nullptr);
}

int sir_edge_max_bwd_dst(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                         const int32_t* splits, int64_t n_splits, int64_t H, int64_t O,
                         const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* dY, int64_t ldy,
                         const int32_t* arg, int64_t lda, int act1, float slope, const float* W,
                         float* dQ, int64_t lddq, float* partial, float* wpart, void* stream) {
    const char* fn = "sir_edge_max_bwd_dst";
    if (act1 < SIR_ACT_IDENTITY || act1 > SIR_ACT_GELU_TANH) return fail(SIR_EINVAL, fn, "unknown act1");
    if (H <= 0 || H % 4 != 0 || H > 256 || O <= 0 || O > 256) return fail(SIR_EUNSUPPORTED, fn, "H % 4 == 0, H <= 256, O <= 256");
    if (n_items < 0 || n_splits < 0 || n_items > INT32_MAX) return fail(SIR_EINVAL, fn, "bad item count");
    if (ldq < H || ldk < H || ldq % 4 || ldk % 4 || !al16(Q) || !al16(K))
        return fail(SIR_EUNSUPPORTED, fn, "Q/K rows must be 16-B aligned (ld % 4 == 0, ld >= H)");
    if (n_items > 0 && (rowptr == nullptr || items == nullptr || Q == nullptr || K == nullptr || dY == nullptr ||
                        ldy < O || arg == nullptr || lda < O || W == nullptr || dQ == nullptr || lddq < H ||
                        wpart == nullptr))
        return fail(SIR_EINVAL, fn, "NULL buffer / leading dimension");
    if (n_splits > 0 && (splits == nullptr || partial == nullptr)) return fail(SIR_EINVAL, fn, "split rows need partial");
    sir::EdgeMlpArgs a{};
    a.rowptr = rowptr; a.col = col; a.items = items; a.n_items = n_items; a.splits = splits; a.n_splits = n_splits;
    a.Q = Q; a.ldq = ldq; a.K = K; a.ldk = ldk; a.G = dY; a.ldg = ldy; a.slope = slope;
    a.H = (int)H; a.HP = (int)((H + 7) / 8 * 8); a.F = (int)O; a.W = W;
    a.out = dQ; a.ldo = lddq; a.pval = partial; a.wpart = wpart; a.arg = const_cast<int*>(arg); a.lda = lda;
    return finish(fn, sir::run_mlp_bwd(a, true, SIR_AGG_MAX, act1, SIR_ACT_IDENTITY, static_cast<hipStream_t>(stream)),
                  nullptr);
}

#ifndef SIR_MAXB_ROUTE_CAP
#define SIR_MAXB_ROUTE_CAP 4096   // routing-table blocks (4 waves, ~12 KB of LDS each): 16 a CU in one round
#endif
static int64_t maxb_route_blocks(int64_t n_items) {
    const int64_t b = (n_items + 3) / 4;
    return b < 1 ? 1 : (b > SIR_MAXB_ROUTE_CAP ? SIR_MAXB_ROUTE_CAP : b);
}

int sir_edge_max_bwd_sparse_parts(int64_t n_items_d, int64_t V, int64_t* route_blocks, int64_t* dw_ranges) {
    const char* fn = "sir_edge_max_bwd_sparse_parts";
    if (route_blocks == nullptr || dw_ranges == nullptr || n_items_d < 0 || V < 0)
        return fail(SIR_EINVAL, fn, "bad argument");
    *route_blocks = maxb_route_blocks(n_items_d);
    *dw_ranges = sir::maxb_dw_ranges(V);
    return SIR_OK;
}

int sir_edge_max_bwd_sparse(const int32_t* rowptr_d, const int32_t* col_d, const int32_t* items_d, int64_t n_items_d,
                            const int32_t* splits_d, int64_t n_splits_d, const int32_t* col_s,
                            const int32_t* items_s, int64_t n_items_s, const int32_t* splits_s, int64_t n_splits_s,
                            const int32_t* pinv, int64_t V, int64_t E, int64_t H, int64_t O,
                            const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* dY, int64_t ldy,
                            const int32_t* arg, int64_t lda, int act1, float slope, const float* W,
                            float* dQ, int64_t lddq, float* dK, int64_t lddk, float* partial, void* ent,
                            void* ecnt_d, void* ecnt_s, float* dbpart, float* wpart, void* stream) {
    const char* fn = "sir_edge_max_bwd_sparse";
    if (act1 < SIR_ACT_IDENTITY || act1 > SIR_ACT_GELU_TANH) return fail(SIR_EINVAL, fn, "unknown act1");
    if (H <= 0 || H % 4 != 0 || H > 512 || O <= 0 || O > 256)
        return fail(SIR_EUNSUPPORTED, fn, "H % 4 == 0, H <= 512, O <= 256");
    if (V < 0 || E < 0 || n_items_d < 0 || n_items_s < 0 || n_splits_d < 0 || n_splits_s < 0 ||
        n_items_d > INT32_MAX || n_items_s > INT32_MAX || E > INT32_MAX)
        return fail(SIR_EINVAL, fn, "bad size");
    if (V * O >= (int64_t)INT32_MAX) return fail(SIR_EUNSUPPORTED, fn, "V * O must be < 2^31");
    if (ldq < H || ldk < H || ldq % 4 || ldk % 4 || lddq < H || lddk < H || lddq % 4 || lddk % 4 || !al16(Q) ||
        !al16(K) || !al16(W) || !al16(dQ) || !al16(dK))
        return fail(SIR_EUNSUPPORTED, fn, "Q / K / W / dQ / dK rows must be 16-B aligned (ld % 4 == 0, ld >= H)");
    if (V > 0 && (rowptr_d == nullptr || items_d == nullptr || Q == nullptr || dY == nullptr || ldy < O ||
                  arg == nullptr || lda < O || W == nullptr || dQ == nullptr || dbpart == nullptr ||
                  ent == nullptr))
        return fail(SIR_EINVAL, fn, "NULL buffer / leading dimension");
    if (E > 0 && (col_d == nullptr || col_s == nullptr || items_s == nullptr || pinv == nullptr || K == nullptr ||
                  dK == nullptr || ecnt_d == nullptr || ecnt_s == nullptr))
        return fail(SIR_EINVAL, fn, "NULL edge buffer");
    if ((n_splits_d > 0 && splits_d == nullptr) || (n_splits_s > 0 && splits_s == nullptr) ||
        ((n_splits_d > 0 || n_splits_s > 0) && partial == nullptr))
        return fail(SIR_EINVAL, fn, "split rows need partial");
    sir::MaxBwdArgs a{};
    a.rowptr_d = rowptr_d; a.col_d = col_d; a.items_d = items_d; a.n_items_d = n_items_d;
    a.splits_d = splits_d; a.n_splits_d = n_splits_d;
    a.col_s = col_s; a.items_s = items_s; a.n_items_s = n_items_s; a.splits_s = splits_s; a.n_splits_s = n_splits_s;
    a.pinv = pinv; a.H = (int)H; a.O = (int)O; a.V = V;
    a.Q = Q; a.ldq = ldq; a.K = K; a.ldk = ldk; a.dY = dY; a.ldy = ldy; a.arg = arg; a.lda = lda;
    a.act1 = act1; a.slope = slope; a.W = W; a.dQ = dQ; a.lddq = lddq; a.dK = dK; a.lddk = lddk;
    a.partial = partial; a.ent = ent; a.ecnt_d = ecnt_d; a.ecnt_s = ecnt_s; a.dbpart = dbpart;
    a.route_blocks = maxb_route_blocks(n_items_d); a.wpart = wpart;
    return finish(fn, sir::run_max_bwd_sparse(a, static_cast<hipStream_t>(stream)), nullptr);
}

int64_t sir_max_dw_rows_parts(int64_t V, int64_t H) {
    if (V < 0 || H <= 0) return 0;
    return sir::max_dw_rows_ranges(V, (int)H);
}

int sir_max_dw_rows(const int32_t* rowptr, int64_t V, const int32_t* arg, int64_t lda, const float* dY, int64_t ldy,
                    const float* A, int64_t ldA, int64_t O, int64_t H, float* wpart, int64_t ldw, void* stream) {
    const char* fn = "sir_max_dw_rows";
    if (O <= 0 || O > 256 || H <= 0 || H % 4 != 0 || H > INT32_MAX) return fail(SIR_EUNSUPPORTED, fn, "O <= 256, H % 4 == 0");
    if (V < 0 || V > INT32_MAX) return fail(SIR_EINVAL, fn, "bad V");
    if (ldw < O * H + ((O + 3) / 4) * 4 || ldw % 4) return fail(SIR_EINVAL, fn, "ldw >= O * H + O4, ldw % 4 == 0");
    if (ldA < H || ldA % 4 || !al16(A) || !al16(wpart)) return fail(SIR_EUNSUPPORTED, fn, "A rows 16-B aligned");
    if (V > 0 && (rowptr == nullptr || arg == nullptr || lda < O || dY == nullptr || ldy < O || wpart == nullptr))
        return fail(SIR_EINVAL, fn, "NULL buffer / leading dimension");
    return finish(fn, sir::run_max_dw_rows(rowptr, V, arg, lda, dY, ldy, A, ldA, (int)O, (int)H, wpart, ldw,
                                           static_cast<hipStream_t>(stream)), nullptr);
}

int sir_max_dw_qk(const int32_t* rowptr, const int32_t* col, int64_t V, const int32_t* arg, int64_t lda,
                  const float* dY, int64_t ldy, const float* Q, int64_t ldq, const float* K, int64_t ldk, int64_t O,
                  int64_t H, int act1, float slope, float* wpart, int64_t ldw, void* stream) {
    const char* fn = "sir_max_dw_qk";
    if (act1 < SIR_ACT_IDENTITY || act1 > SIR_ACT_GELU_TANH) return fail(SIR_EINVAL, fn, "unknown act1");
    if (O <= 0 || O > 256 || H <= 0 || H % 4 != 0 || H > INT32_MAX) return fail(SIR_EUNSUPPORTED, fn, "O <= 256, H % 4 == 0");
    if (V < 0 || V > INT32_MAX) return fail(SIR_EINVAL, fn, "bad V");
    if (ldw < O * H + ((O + 3) / 4) * 4 || ldw % 4) return fail(SIR_EINVAL, fn, "ldw >= O * H + O4, ldw % 4 == 0");
    if (ldq < H || ldk < H || ldq % 4 || ldk % 4 || !al16(Q) || !al16(K) || !al16(wpart))
        return fail(SIR_EUNSUPPORTED, fn, "Q / K rows 16-B aligned");
    if (V > 0 && (rowptr == nullptr || col == nullptr || arg == nullptr || lda < O || dY == nullptr || ldy < O ||
                  wpart == nullptr))
        return fail(SIR_EINVAL, fn, "NULL buffer / leading dimension");
    return finish(fn, sir::run_max_dw_qk(rowptr, col, V, arg, lda, dY, ldy, Q, ldq, K, ldk, (int)O, (int)H, act1, slope,
                                         wpart, ldw, static_cast<hipStream_t>(stream)), nullptr);
}

int sir_edge_max_bwd_src(const int32_t* rowptr_s, const int32_t* col_s, const int32_t* perm_s,
                         const int32_t* items, int64_t n_items, const int32_t* splits, int64_t n_splits,
                         int64_t H, int64_t O, const float* K, int64_t ldk, const float* Q, int64_t ldq,
                         const float* dY, int64_t ldy, const int32_t* arg, int64_t lda, int act1, float slope,
                         const float* W, float* dK, int64_t lddk, float* partial, void* stream) {
    const char* fn = "sir_edge_max_bwd_src";
    if (act1 < SIR_ACT_IDENTITY || act1 > SIR_ACT_GELU_TANH) return fail(SIR_EINVAL, fn, "unknown act1");
    if (H <= 0 || H % 4 != 0 || H > 256 || O <= 0 || O > 256) return fail(SIR_EUNSUPPORTED, fn, "H % 4 == 0, H <= 256, O <= 256");
    if (n_items < 0 || n_splits < 0 || n_items > INT32_MAX) return fail(SIR_EINVAL, fn, "bad item count");
    if (ldq < H || ldk < H || ldq % 4 || ldk % 4 || !al16(Q) || !al16(K))
        return fail(SIR_EUNSUPPORTED, fn, "Q/K rows must be 16-B aligned (ld % 4 == 0, ld >= H)");
    if (n_items > 0 && (rowptr_s == nullptr || items == nullptr || Q == nullptr || K == nullptr || dY == nullptr ||
                        ldy < O || arg == nullptr || lda < O || W == nullptr || dK == nullptr || lddk < H))
        return fail(SIR_EINVAL, fn, "NULL buffer / leading dimension");
    if (n_items > 0 && col_s != nullptr && perm_s == nullptr) return fail(SIR_EINVAL, fn, "NULL perm");
    if (n_splits > 0 && (splits == nullptr || partial == nullptr)) return fail(SIR_EINVAL, fn, "split rows need partial");
    sir::EdgeMlpArgs a{};
    a.rowptr = rowptr_s; a.col = col_s; a.items = items; a.n_items = n_items; a.splits = splits; a.n_splits = n_splits;
    a.Q = Q; a.ldq = ldq; a.K = K; a.ldk = ldk; a.G = dY; a.ldg = ldy; a.slope = slope;
    a.H = (int)H; a.HP = (int)((H + 7) / 8 * 8); a.F = (int)O; a.W = W;
    a.out = dK; a.ldo = lddk; a.pval = partial; a.wpart = nullptr; a.arg = const_cast<int*>(arg); a.lda = lda;
    a.perm = perm_s;
    return finish(fn, sir::run_mlp_bwd(a, false, SIR_AGG_MAX, act1, SIR_ACT_IDENTITY, static_cast<hipStream_t>(stream)),
                  nullptr);
}

// ------------------------------------------------------------------------------ GraphNorm
int sir_graph_norm_fwd(const int64_t* off, int64_t B, int64_t F, const float* X, int64_t ldx,
                       const float* weight, const float* bias, const float* mean_scale, float eps,
                       float* Y, int64_t ldy, float* mean, float* std_, void* stream) {
    const char* fn = "sir_graph_norm_fwd";
    if (B < 0 || F <= 0 || F > 65536) return fail(SIR_EINVAL, fn, "bad shape");
    if (ldx < F || ldy < F) return fail(SIR_EINVAL, fn, "leading dimensions must be >= F");
    if (B > 0 && (off == nullptr || X == nullptr || weight == nullptr || Y == nullptr || mean == nullptr ||
                  std_ == nullptr))
        return fail(SIR_EINVAL, fn, "NULL buffer");
    return finish(fn, sir::run_graph_norm_fwd(off, B, (int)F, X, ldx, weight, bias, mean_scale, eps, SIR_ACT_IDENTITY,
                                              0.f, nullptr, 0, Y, ldy, mean, std_, static_cast<hipStream_t>(stream)),
                  nullptr);
}


int sir_resid_act_fwd(const void* Y, int64_t ldy, int dtype, const float* R, int64_t ldr, float* out, int64_t ldo,
                      int64_t M, int64_t N, int act, float slope, int order, void* stream) {
    const char* fn = "sir_resid_act_fwd";
    if (M < 0 || N <= 0 || N % 4 != 0 || N > (1 << 30)) return fail(SIR_EINVAL, fn, "bad shape (N % 4 == 0)");
    if (dtype != SIR_DTYPE_F32 && dtype != SIR_DTYPE_BF16 && dtype != SIR_DTYPE_F16) return fail(SIR_EINVAL, fn, "bad dtype");
    if (act != SIR_ACT_IDENTITY && act != SIR_ACT_RELU && act != SIR_ACT_LEAKY_RELU)
        return fail(SIR_EINVAL, fn, "act must be identity, relu or leaky_relu");
    if (order != 0 && order != 1) return fail(SIR_EINVAL, fn, "order must be 0 (zinc) or 1 (arxiv)");
    if (ldy < N || ldr < N || ldo < N || ldy % 4 || ldr % 4 || ldo % 4)
        return fail(SIR_EINVAL, fn, "leading dimensions must be >= N and multiples of 4");
    if (M > 0 && (Y == nullptr || R == nullptr || out == nullptr)) return fail(SIR_EINVAL, fn, "NULL buffer");
    if (!al16(R) || !al16(out) || (dtype == SIR_DTYPE_F32 ? !al16(Y) : (reinterpret_cast<uintptr_t>(Y) & 7u) != 0))
        return fail(SIR_EINVAL, fn, "rows must be 16-B aligned (8-B for 16-bit Y)");
    return finish(fn, sir::run_resid_act_fwd(Y, ldy, dtype, R, ldr, out, ldo, M, (int)N, act, slope, order,
                                             static_cast<hipStream_t>(stream)), nullptr);
}

int sir_resid_act_bwd(const float* D, int64_t ldd, const float* D2, int64_t ldd2, const void* Y, int64_t ldy, int dtype,
                      const float* R, int64_t ldr, void* dY, int64_t lddy, float* dR, int64_t lddr, int64_t M, int64_t N,
                      int act, float slope, int order, void* stream) {
    const char* fn = "sir_resid_act_bwd";
    if (M < 0 || N <= 0 || N % 4 != 0 || N > (1 << 30)) return fail(SIR_EINVAL, fn, "bad shape (N % 4 == 0)");
    if (dtype != SIR_DTYPE_F32 && dtype != SIR_DTYPE_BF16 && dtype != SIR_DTYPE_F16) return fail(SIR_EINVAL, fn, "bad dtype");
    if (act != SIR_ACT_IDENTITY && act != SIR_ACT_RELU && act != SIR_ACT_LEAKY_RELU)
        return fail(SIR_EINVAL, fn, "act must be identity, relu or leaky_relu");
    if (order != 0 && order != 1) return fail(SIR_EINVAL, fn, "order must be 0 (zinc) or 1 (arxiv)");
    if (D2 != nullptr && (ldd2 < N || ldd2 % 4 || !al16(D2) || (order == 1 && dR == nullptr)))
        return fail(SIR_EINVAL, fn, "D2: rows 16-B aligned, ldd2 >= N, ldd2 % 4 == 0 (order 1: with dR for the sum)");
    const bool want_dr = order == 0 || D2 != nullptr;        // order 1 writes dR only as the sum D + D2
    if (ldd < N || ldy < N || lddy < N || ldd % 4 || ldy % 4 || lddy % 4 || (order == 0 && (ldr < N || ldr % 4)) ||
        (want_dr && dR != nullptr && (lddr < N || lddr % 4)))
        return fail(SIR_EINVAL, fn, "leading dimensions must be >= N and multiples of 4");
    if (M > 0 && (D == nullptr || Y == nullptr || dY == nullptr || (order == 0 && R == nullptr)))
        return fail(SIR_EINVAL, fn, "NULL buffer");
    const bool y16 = dtype != SIR_DTYPE_F32;
    if (!al16(D) || (y16 ? (reinterpret_cast<uintptr_t>(Y) & 7u) || (reinterpret_cast<uintptr_t>(dY) & 7u)
                         : !al16(Y) || !al16(dY)) || (order == 0 && !al16(R)) || (want_dr && !al16(dR)))
        return fail(SIR_EINVAL, fn, "rows must be 16-B aligned (8-B for 16-bit Y, dY)");
    return finish(fn, sir::run_resid_act_bwd(D, ldd, D2, ldd2, Y, ldy, dtype, R, ldr, dY, lddy, want_dr ? dR : nullptr, lddr, M,
                                             (int)N, act, slope, order, static_cast<hipStream_t>(stream)), nullptr);
}

int sir_graph_norm_act_fwd(const int64_t* off, int64_t B, int64_t F, const float* X, int64_t ldx,
                           const float* weight, const float* bias, const float* mean_scale, float eps, int act,
                           float slope, const float* R, int64_t ldr, float* Y, int64_t ldy, float* mean, float* std_,
                           void* stream) {
    const char* fn = "sir_graph_norm_act_fwd";
    if (B < 0 || F <= 0 || F > 65536) return fail(SIR_EINVAL, fn, "bad shape");
    if (ldx < F || ldy < F || (R != nullptr && ldr < F)) return fail(SIR_EINVAL, fn, "leading dimensions must be >= F");
    if (act != SIR_ACT_IDENTITY && act != SIR_ACT_RELU && act != SIR_ACT_LEAKY_RELU)
        return fail(SIR_EINVAL, fn, "act must be identity, relu or leaky_relu");
    if (B > 0 && (off == nullptr || X == nullptr || weight == nullptr || Y == nullptr || mean == nullptr ||
                  std_ == nullptr))
        return fail(SIR_EINVAL, fn, "NULL buffer");
    return finish(fn, sir::run_graph_norm_fwd(off, B, (int)F, X, ldx, weight, bias, mean_scale, eps, act, slope, R, ldr,
                                              Y, ldy, mean, std_, static_cast<hipStream_t>(stream)), nullptr);
}

int sir_graph_norm_bwd(const int64_t* off, int64_t B, int64_t F, const float* X, int64_t ldx,
                       const float* dY, int64_t ldg, const float* weight, const float* mean_scale,
                       const float* mean, const float* std_, float* dX, int64_t lddx,
                       float* dw_part, float* dms_part, float* db_part, void* stream) {
    const char* fn = "sir_graph_norm_bwd";
    if (B < 0 || F <= 0 || F > 65536) return fail(SIR_EINVAL, fn, "bad shape");
    if (ldx < F || ldg < F || lddx < F) return fail(SIR_EINVAL, fn, "leading dimensions must be >= F");
    if (B > 0 && (off == nullptr || X == nullptr || dY == nullptr || weight == nullptr || mean == nullptr ||
                  std_ == nullptr || dX == nullptr || dw_part == nullptr || db_part == nullptr))
        return fail(SIR_EINVAL, fn, "NULL buffer");
    if (mean_scale != nullptr && dms_part == nullptr && B > 0) return fail(SIR_EINVAL, fn, "dms_part needed");
    return finish(fn, sir::run_graph_norm_bwd(off, B, (int)F, X, ldx, dY, ldg, weight, nullptr, mean_scale, mean, std_,
                                              SIR_ACT_IDENTITY, 0.f, dX, lddx, dw_part, dms_part, db_part,
                                              static_cast<hipStream_t>(stream)), nullptr);
}

int sir_graph_norm_act_bwd(const int64_t* off, int64_t B, int64_t F, const float* X, int64_t ldx,
                           const float* dY, int64_t ldg, const float* weight, const float* bias,
                           const float* mean_scale, const float* mean, const float* std_, int act, float slope,
                           float* dX, int64_t lddx, float* dw_part, float* dms_part, float* db_part, void* stream) {
    const char* fn = "sir_graph_norm_act_bwd";
    if (B < 0 || F <= 0 || F > 65536) return fail(SIR_EINVAL, fn, "bad shape");
    if (ldx < F || ldg < F || lddx < F) return fail(SIR_EINVAL, fn, "leading dimensions must be >= F");
    if (act != SIR_ACT_IDENTITY && act != SIR_ACT_RELU && act != SIR_ACT_LEAKY_RELU)
        return fail(SIR_EINVAL, fn, "act must be identity, relu or leaky_relu");
    if (B > 0 && (off == nullptr || X == nullptr || dY == nullptr || weight == nullptr || mean == nullptr ||
                  std_ == nullptr || dX == nullptr || dw_part == nullptr || db_part == nullptr))
        return fail(SIR_EINVAL, fn, "NULL buffer");
    if (mean_scale != nullptr && dms_part == nullptr && B > 0) return fail(SIR_EINVAL, fn, "dms_part needed");
    return finish(fn, sir::run_graph_norm_bwd(off, B, (int)F, X, ldx, dY, ldg, weight, bias, mean_scale, mean, std_,
                                              act, slope, dX, lddx, dw_part, dms_part, db_part,
                                              static_cast<hipStream_t>(stream)), nullptr);
}

int64_t sir_csr_build_workspace(int64_t n_rows, int64_t E) {
    if (n_rows < 0 || E < 0 || E >= INT32_MAX || n_rows >= INT32_MAX) return -1;
    return sir::csr_build_workspace(n_rows, E);
}

int sir_csr_build(const int64_t* rows, const int64_t* cols, int64_t E, int64_t n_rows, int64_t n_cols,
                  int64_t chunk, int32_t* rowptr, int32_t* col, int64_t* eid, int32_t* items, int32_t* splits,
                  int64_t* counts, void* workspace, int64_t workspace_bytes, void* stream) {
    const char* fn = "sir_csr_build";
    if (n_rows < 0 || E < 0 || n_cols < 0) return fail(SIR_EINVAL, fn, "negative size");
    if (E >= INT32_MAX || n_rows >= INT32_MAX) return fail(SIR_EINVAL, fn, "int32 plan: E and n_rows must be < 2^31");
    if (chunk < 1 || chunk > (1 << 24)) return fail(SIR_EINVAL, fn, "chunk must be in [1, 2^24]");
    if (rowptr == nullptr || counts == nullptr) return fail(SIR_EINVAL, fn, "NULL rowptr/counts");
    if (E > 0 && (rows == nullptr || cols == nullptr || col == nullptr || eid == nullptr))
        return fail(SIR_EINVAL, fn, "NULL edge buffer");
    if (n_rows > 0 && (items == nullptr || splits == nullptr)) return fail(SIR_EINVAL, fn, "NULL items/splits");
    const int64_t need = sir::csr_build_workspace(n_rows, E);
    if (need < 0) return fail(SIR_ELAUNCH, fn, "workspace query failed");
    if (workspace == nullptr || workspace_bytes < need) return fail(SIR_EINVAL, fn, "workspace too small");
    return finish(fn, sir::run_csr_build(rows, cols, E, n_rows, n_cols, (int)chunk, rowptr, col, eid, items, splits,
                                         counts, workspace, workspace_bytes, static_cast<hipStream_t>(stream)),
                  "workspace too small");
}

int sir_csr_perm(const int64_t* eid_a, const int64_t* eid_b, int64_t E, int32_t* pos_ws, int32_t* perm,
                 void* stream) {
    const char* fn = "sir_csr_perm";
    if (E < 0 || E >= INT32_MAX) return fail(SIR_EINVAL, fn, "E must be in [0, 2^31)");
    if (E > 0 && (eid_a == nullptr || eid_b == nullptr || pos_ws == nullptr || perm == nullptr))
        return fail(SIR_EINVAL, fn, "NULL buffer");
    return finish(fn, sir::run_csr_perm(eid_a, eid_b, E, pos_ws, perm, static_cast<hipStream_t>(stream)), nullptr);
}

int64_t sir_gemm_pack_bytes(int64_t N, int64_t K) {
    if (N <= 0 || K <= 0 || N > 65536 || K > 65536) return 0;
    return sir::gemm_pack_bytes(N, K);
}

int sir_gemm_pack(const float* W, int64_t ldw, int64_t N, int64_t K, int trans, void* packed, void* stream) {
    const char* fn = "sir_gemm_pack";
    if (N <= 0 || K <= 0 || N > 65536 || K > 65536) return fail(SIR_EINVAL, fn, "N and K must be in [1, 65536]");
    if (W == nullptr || packed == nullptr) return fail(SIR_EINVAL, fn, "NULL buffer");
    if (ldw < (trans ? N : K)) return fail(SIR_EINVAL, fn, "ldw too small");
    if ((reinterpret_cast<uintptr_t>(packed) & 15u) != 0) return fail(SIR_EINVAL, fn, "packed must be 16-B aligned");
    hipError_t err = sir::run_gemm_pack(W, ldw, (int)N, (int)K, trans ? 1 : 0, packed, static_cast<hipStream_t>(stream));
    return finish(fn, err, nullptr);
}

int sir_gemm_nt(const float* A, int64_t lda, int64_t M, int64_t K, const void* packed, int64_t N,
                const float* bias, float* C, int64_t ldc, const sir_dropout_t* drop, void* stream) {
    const char* fn = "sir_gemm_nt";
    if (M < 0 || N <= 0 || K <= 0 || N > 65536 || K > 65536) return fail(SIR_EINVAL, fn, "bad shape");
    if ((M + 255) / 256 * ((N + 127) / 128) > (int64_t)INT_MAX) return fail(SIR_EINVAL, fn, "M too large");
    if (K % 4 != 0 || N % 4 != 0 || lda % 4 != 0 || ldc % 4 != 0 || lda < K || ldc < N)
        return fail(SIR_EINVAL, fn, "K, N, lda, ldc must be multiples of 4 (lda >= K, ldc >= N)");
    // a 256-row tile of A is addressed by one buffer resource with 32-bit signed byte offsets
    if (lda > SIR_GEMM_MAX_LD) return fail(SIR_EINVAL, fn, "lda too large (256 rows must span < 2^31 bytes)");
    if (M > 0 && (A == nullptr || C == nullptr || packed == nullptr)) return fail(SIR_EINVAL, fn, "NULL buffer");
    if (((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(C) | reinterpret_cast<uintptr_t>(bias) |
          reinterpret_cast<uintptr_t>(packed)) & 15u) != 0)
        return fail(SIR_EINVAL, fn, "A, C, bias and packed must be 16-B aligned");
    hipError_t err = sir::run_gemm_nt(A, lda, M, (int)K, packed, (int)N, bias, C, ldc, static_cast<hipStream_t>(stream),
                                      to_drop(drop, 0));
    return finish(fn, err, nullptr);
}

int sir_gemm_nt_dact(const float* A, int64_t lda, int64_t M, int64_t K, const void* packed, int64_t N,
                     const float* gate, const uint64_t* gate_mask, int act, float slope, float* C, int64_t ldc,
                     void* stream) {
    const char* fn = "sir_gemm_nt_dact";
    if (M < 0 || N <= 0 || K <= 0 || N > 65536 || K > 65536) return fail(SIR_EINVAL, fn, "bad shape");
    if ((M + 255) / 256 * ((N + 127) / 128) > (int64_t)INT_MAX) return fail(SIR_EINVAL, fn, "M too large");
    if (K % 4 != 0 || N % 4 != 0 || lda % 4 != 0 || ldc % 4 != 0 || lda < K || ldc < N)
        return fail(SIR_EINVAL, fn, "K, N, lda, ldc must be multiples of 4 (lda >= K, ldc >= N)");
    if (lda > SIR_GEMM_MAX_LD || ldc > SIR_GEMM_MAX_LD) return fail(SIR_EINVAL, fn, "lda / ldc too large");
    if (act != SIR_ACT_RELU && act != SIR_ACT_LEAKY_RELU) return fail(SIR_EINVAL, fn, "act must be ReLU or LeakyReLU");
    if (M > 0 && (A == nullptr || C == nullptr || packed == nullptr || (gate == nullptr && gate_mask == nullptr)))
        return fail(SIR_EINVAL, fn, "NULL buffer");
    if (gate_mask != nullptr && N != 256) return fail(SIR_EUNSUPPORTED, fn, "gate_mask needs N = 256");
    if (((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(C) | reinterpret_cast<uintptr_t>(gate) |
          reinterpret_cast<uintptr_t>(packed)) & 15u) != 0)
        return fail(SIR_EINVAL, fn, "A, C, gate and packed must be 16-B aligned");
    hipError_t err = sir::run_gemm_nt(A, lda, M, (int)K, packed, (int)N, nullptr, C, ldc, static_cast<hipStream_t>(stream),
                                      sir::Drop(), gate_mask != nullptr ? nullptr : gate, act == SIR_ACT_RELU ? 1 : 0,
                                      slope, gate_mask);
    return finish(fn, err, nullptr);
}

int sir_gemm_nt_direct(const float* A, int64_t lda, int64_t M, int64_t K, const float* W, int64_t ldw, int trans,
                       int64_t N, const float* bias, float* C, int64_t ldc, const sir_dropout_t* drop, void* stream) {
    const char* fn = "sir_gemm_nt_direct";
    if (M < 0 || N <= 0 || K <= 0 || N > 65536 || K > 65536) return fail(SIR_EINVAL, fn, "bad shape");
    if ((M + 31) / 32 * ((N + 31) / 32) > (int64_t)INT_MAX) return fail(SIR_EINVAL, fn, "M too large");
    if (K % 4 != 0 || N % 4 != 0 || lda % 4 != 0 || ldc % 4 != 0 || lda < K || ldc < N)
        return fail(SIR_EINVAL, fn, "K, N, lda, ldc must be multiples of 4 (lda >= K, ldc >= N)");
    if (trans != 0 && trans != 1) return fail(SIR_EINVAL, fn, "trans must be 0 or 1");
    if (ldw < (trans ? N : K)) return fail(SIR_EINVAL, fn, "ldw too small");
    if (lda > SIR_GEMM_MAX_LD || ldw > SIR_GEMM_MAX_LD) return fail(SIR_EINVAL, fn, "lda/ldw too large");
    if (M > 0 && (A == nullptr || C == nullptr || W == nullptr)) return fail(SIR_EINVAL, fn, "NULL buffer");
    if (((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(C) | reinterpret_cast<uintptr_t>(bias)) & 15u) != 0)
        return fail(SIR_EINVAL, fn, "A, C and bias must be 16-B aligned");
    if ((reinterpret_cast<uintptr_t>(W) & 3u) != 0) return fail(SIR_EINVAL, fn, "W must be 4-B aligned");
    hipError_t err = sir::run_gemm_nt_direct(A, lda, M, (int)K, W, ldw, trans, (int)N, bias, C, ldc,
                                             static_cast<hipStream_t>(stream), to_drop(drop, 0));
    return finish(fn, err, nullptr);
}

int sir_gemm_nt_direct2(const float* A, int64_t lda, int64_t M, int64_t K, const float* W, int64_t ldw,
                        const float* W2, int64_t ldw2, int64_t split, int trans, int64_t N, const float* bias,
                        int64_t bias_cols, float* C, int64_t ldc, const sir_dropout_t* drop, void* stream) {
    const char* fn = "sir_gemm_nt_direct2";
    if (M < 0 || N <= 0 || K <= 0 || N > 65536 || K > 65536) return fail(SIR_EINVAL, fn, "bad shape");
    if ((M + 31) / 32 * ((N + 31) / 32) > (int64_t)INT_MAX) return fail(SIR_EINVAL, fn, "M too large");
    if (K % 4 != 0 || N % 4 != 0 || lda % 4 != 0 || ldc % 4 != 0 || lda < K || ldc < N)
        return fail(SIR_EINVAL, fn, "K, N, lda, ldc must be multiples of 4 (lda >= K, ldc >= N)");
    if (trans != 0 && trans != 1) return fail(SIR_EINVAL, fn, "trans must be 0 or 1");
    const int64_t rows = trans ? K : N;           // weight rows: k (trans) or output features
    if (split <= 0 || split > rows) return fail(SIR_EINVAL, fn, "split must be in (0, weight rows]");
    if (bias_cols < 0 || bias_cols % 4 != 0) return fail(SIR_EINVAL, fn, "bias_cols must be a multiple of 4");
    if (ldw < (trans ? N : K) || ldw2 < (trans ? N : K)) return fail(SIR_EINVAL, fn, "ldw / ldw2 too small");
    if (lda > SIR_GEMM_MAX_LD || ldw > SIR_GEMM_MAX_LD || ldw2 > SIR_GEMM_MAX_LD)
        return fail(SIR_EINVAL, fn, "lda/ldw too large");
    if (M > 0 && (A == nullptr || C == nullptr || W == nullptr || (split < rows && W2 == nullptr)))
        return fail(SIR_EINVAL, fn, "NULL buffer");
    if (((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(C) | reinterpret_cast<uintptr_t>(bias) |
          reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(W2)) & 15u) != 0 || ldw % 4 != 0 || ldw2 % 4 != 0)
        return fail(SIR_EINVAL, fn, "A, C, bias, W, W2 must be 16-B aligned, ldw / ldw2 multiples of 4");
    hipError_t err = sir::run_gemm_nt_direct(A, lda, M, (int)K, W, ldw, trans, (int)N, bias, C, ldc,
                                             static_cast<hipStream_t>(stream), to_drop(drop, 0),
                                             split < rows ? W2 : nullptr, ldw2, split, bias_cols);
    return finish(fn, err, nullptr);
}

int64_t sir_gemm_tn_workspace(int64_t R, int64_t M, int64_t N) {
    if (R < 0 || M <= 0 || N <= 0 || M > 65536 || N > 65536) return 0;
    return sir::gemm_tn_workspace(R, M, N);
}

int sir_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t R, int64_t M, int64_t N,
                float* C, int64_t ldc, float* colsum_a, void* workspace, int64_t workspace_bytes, void* stream) {
    const char* fn = "sir_gemm_tn";
    if (R < 0 || M <= 0 || N <= 0 || M > 65536 || N > 65536) return fail(SIR_EINVAL, fn, "bad shape");
    if (lda < M || ldb < N || ldc < N) return fail(SIR_EINVAL, fn, "leading dimension too small");
    if (lda > SIR_GEMM_MAX_LD || ldb > SIR_GEMM_MAX_LD)
        return fail(SIR_EINVAL, fn, "lda/ldb too large (a 32-row chunk must span < 2^31 bytes)");
    if (C == nullptr || workspace == nullptr || (R > 0 && (A == nullptr || B == nullptr)))
        return fail(SIR_EINVAL, fn, "NULL buffer");
    if (workspace_bytes < sir::gemm_tn_workspace(R, M, N)) return fail(SIR_EINVAL, fn, "workspace too small");
    hipError_t err = sir::run_gemm_tn(A, lda, B, ldb, R, (int)M, (int)N, C, ldc, colsum_a, workspace,
                                      static_cast<hipStream_t>(stream));
    return finish(fn, err, nullptr);
}

int sir_gemm_tn16(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t R, int64_t M, int64_t N, int dtype,
                  float* C, int64_t ldc, float* colsum_a, void* workspace, int64_t workspace_bytes, void* stream) {
    const char* fn = "sir_gemm_tn16";
    if (dtype != SIR_DTYPE_BF16 && dtype != SIR_DTYPE_F16) return fail(SIR_EINVAL, fn, "dtype must be BF16 or F16");
    if (R < 0 || M <= 0 || N <= 0 || M > 65536 || N > 65536) return fail(SIR_EINVAL, fn, "bad shape");
    if (lda < M || ldb < N || ldc < N) return fail(SIR_EINVAL, fn, "leading dimension too small");
    if (M % 2 != 0 || N % 2 != 0 || lda % 2 != 0 || ldb % 2 != 0)
        return fail(SIR_EINVAL, fn, "M, N, lda, ldb must be even");
    if (lda > SIR_GEMM_MAX_LD || ldb > SIR_GEMM_MAX_LD)
        return fail(SIR_EINVAL, fn, "lda/ldb too large (a 32-row chunk must span < 2^31 bytes)");
    if (C == nullptr || workspace == nullptr || (R > 0 && (A == nullptr || B == nullptr)))
        return fail(SIR_EINVAL, fn, "NULL buffer");
    if (((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 3u) != 0)
        return fail(SIR_EINVAL, fn, "A and B must be 4-B aligned");
    if (workspace_bytes < sir::gemm_tn_workspace(R, M, N)) return fail(SIR_EINVAL, fn, "workspace too small");
    hipError_t err = sir::run_gemm_tn16(A, lda, B, ldb, R, (int)M, (int)N, dtype, C, ldc, colsum_a, workspace,
                                        static_cast<hipStream_t>(stream));
    return finish(fn, err, nullptr);
}

int64_t sir_gemm_pack16_bytes(int64_t N, int64_t K) {
    if (N <= 0 || K <= 0 || N > 65536 || K > 65536 || K % 16 != 0) return 0;
    return sir::gemm_pack16_bytes(N, K);
}

int sir_gemm_pack16(const float* W, int64_t ldw, int64_t N, int64_t K, int trans, int dtype, void* packed, void* stream) {
    const char* fn = "sir_gemm_pack16";
    if (dtype != SIR_DTYPE_BF16 && dtype != SIR_DTYPE_F16) return fail(SIR_EINVAL, fn, "dtype must be BF16 or F16");
    if (N <= 0 || K <= 0 || N > 65536 || K > 65536 || K % 16 != 0)
        return fail(SIR_EINVAL, fn, "N in [1, 65536], K in [16, 65536] and a multiple of 16");
    if (W == nullptr || packed == nullptr) return fail(SIR_EINVAL, fn, "NULL buffer");
    if (ldw < (trans ? N : K)) return fail(SIR_EINVAL, fn, "ldw too small");
    if ((reinterpret_cast<uintptr_t>(packed) & 15u) != 0) return fail(SIR_EINVAL, fn, "packed must be 16-B aligned");
    hipError_t err = sir::run_gemm_pack16(W, ldw, (int)N, (int)K, trans ? 1 : 0, dtype, packed, static_cast<hipStream_t>(stream));
    return finish(fn, err, nullptr);
}

int sir_gemm_nt16(const void* A, int64_t lda, int a_dtype, int64_t M, int64_t K, const void* packed, int64_t N,
                  int dtype, const float* bias, void* C, int64_t ldc, int c_dtype, void* Acopy, int64_t ldac,
                  const sir_dropout_t* drop, void* stream) {
    const char* fn = "sir_gemm_nt16";
    if (dtype != SIR_DTYPE_BF16 && dtype != SIR_DTYPE_F16) return fail(SIR_EINVAL, fn, "dtype must be BF16 or F16");
    if (a_dtype != dtype && a_dtype != SIR_DTYPE_F32) return fail(SIR_EINVAL, fn, "a_dtype must be dtype or F32");
    if (c_dtype != dtype && c_dtype != SIR_DTYPE_F32) return fail(SIR_EINVAL, fn, "c_dtype must be dtype or F32");
    if (M < 0 || N <= 0 || N > 512 || (K != 128 && K != 256 && K != 512)) return fail(SIR_EINVAL, fn, "bad shape");
    if ((M + 255) / 256 * ((N + 255) / 256) > (int64_t)INT_MAX) return fail(SIR_EINVAL, fn, "M too large");
    const int64_t av = a_dtype == SIR_DTYPE_F32 ? 4 : 8;     // elements per 16 B of A
    const int64_t cv = c_dtype == SIR_DTYPE_F32 ? 4 : 8;     // elements per 16 B of C
    if (N % cv != 0 || lda % av != 0 || lda < K || ldc < N || ldc % cv != 0)
        return fail(SIR_EINVAL, fn, "N, ldc multiples of 16 B of C, lda a multiple of 16 B, lda >= K, ldc >= N");
    if (lda > SIR_GEMM_MAX_LD || ldc > SIR_GEMM_MAX_LD) return fail(SIR_EINVAL, fn, "lda/ldc too large");
    if (Acopy != nullptr && (a_dtype != SIR_DTYPE_F32 || ldac < K || ldac % 8 != 0 || ldac > SIR_GEMM_MAX_LD))
        return fail(SIR_EINVAL, fn, "Acopy needs an fp32 A and ldac >= K, a multiple of 8");
    if (M > 0 && (A == nullptr || C == nullptr || packed == nullptr)) return fail(SIR_EINVAL, fn, "NULL buffer");
    if (((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(C) | reinterpret_cast<uintptr_t>(Acopy) |
          reinterpret_cast<uintptr_t>(packed)) & 15u) != 0)
        return fail(SIR_EINVAL, fn, "A, C, Acopy and packed must be 16-B aligned");
    hipError_t err = sir::run_gemm_nt16(A, lda, a_dtype, M, (int)K, packed, (int)N, dtype, bias, C, ldc, c_dtype, Acopy,
                                        ldac, static_cast<hipStream_t>(stream), to_drop(drop, 0));
    return finish(fn, err, nullptr);
}

int sir_dropout_apply(void* X, int64_t ldx, int64_t M, int64_t N, int dtype, int64_t col0,
                      const sir_dropout_t* drop, void* stream) {
    const char* fn = "sir_dropout_apply";
    if (dtype != SIR_DTYPE_F32 && dtype != SIR_DTYPE_BF16 && dtype != SIR_DTYPE_F16)
        return fail(SIR_EINVAL, fn, "dtype must be SIR_DTYPE_F32, _BF16 or _F16");
    if (M < 0 || N < 0 || N > (1 << 24) || M > INT32_MAX || ldx < N || col0 < 0 || col0 > (1 << 24))
        return fail(SIR_EINVAL, fn, "bad shape");
    if (M > 0 && N > 0 && X == nullptr) return fail(SIR_EINVAL, fn, "NULL X");
    return finish(fn, sir::run_dropout_apply(X, ldx, M, (int)N, dtype, to_drop(drop, col0), static_cast<hipStream_t>(stream)),
                  nullptr);
}

}  // extern "C"
