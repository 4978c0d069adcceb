/*
 * sirconv.h — C ABI of the MI355X (gfx950) SIRConv edge-aggregation kernels.
 *
 * This is the drop-in boundary for the hot path of briangodwinlim/SIR-GCN `SIRConv`
 * (models/conv.py:7-67).  In the reference the path is
 *     graph.update_all(self.message_func, self._agg_func('m', 'ft'))      conv.py:63
 * with the edge UDF  m = out_norm[u] * in_norm[v] * sigma(eq[v] + ek[u])   conv.py:43-45
 * which DGL 2.1.0 runs as index_select gathers + elementwise + GSpMM(copy_e, sum)
 * over the in-edge CSC (and, under autograd, gsddmm/index_add for the backward).
 * Entry points, by the reference code they replace (INTEGRATION.md §2 has the table):
 *  - the edge aggregation and its backward (conv.py:43-45,63): sir_edge_agg_fwd / _bwd_dst /
 *    _bwd_src / _bwd (one launch), with the sign mask of the ReLU family (sir_mask_words);
 *  - the degree norms (conv.py:51-57): sir_degree_norms;
 *  - the projections and their gradients (nn.Linear, conv.py:60-61,65): the split-fp16 MFMA
 *    GEMMs sir_gemm_nt / sir_gemm_nt_direct / sir_gemm_tn and the 16-bit (autocast) ones, the
 *    bias gradients sir_col_sum, the Q/K feature dropout sir_dropout_t (conv.py:35,60-61);
 *  - agg='max' and the per-edge Linear sigma (conv.py:46-47): sir_edge_mlp_* / sir_edge_max_*;
 *    the edge-materialised helpers (sir_edge_gather_add / _act, sir_segment_*);
 *  - GraphNorm (models/norm.py:7-29): sir_graph_norm_fwd / _bwd, with the stack's activation and
 *    residual fused: sir_graph_norm_act_fwd / _bwd;
 *  - the graph input (DGL's CSC build for batched graphs): sir_csr_build / sir_csr_perm.
 *
 * Conventions
 *  - All pointers are DEVICE pointers; all work is enqueued on `stream` (a hipStream_t,
 *    NULL = default stream); calls are asynchronous, stateless and reentrant.
 *  - The caller owns every buffer.  Outputs are fully overwritten (no pre-zeroing).
 *  - Row-major feature matrices with explicit leading dimensions (elements).
 *  - Graph structure is a "row CSR": rows are the nodes being reduced INTO, `col` holds the
 *    node at the other end of each edge, edges of a row are in ascending edge id
 *    (DGL's stable CSC order).  int32 indices (valid while E < 2^31).
 *  - Work plan: `items` = int32[n_items][4] {row, e_begin, e_end, slot}; every row appears
 *    in >= 1 item; a row longer than the plan's chunk is split over several items with
 *    slot >= 0 (partial-sum slot), unsplit rows have slot = -1.  `splits` =
 *    int32[n_splits][4] {row, slot_begin, n_slots, degree} for the split rows, combined in
 *    slot order (deterministic, no atomics).  `partial` = float[n_slots_total * H] scratch.
 *  - `col` (and `perm_s`) may be NULL when the graph has no edges.
 *  - Return 0 on success, otherwise an SIR_E* code; sir_last_error() gives the text
 *    (thread-local).
 */
#ifndef SIRCONV_H
#define SIRCONV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SIR_ABI_VERSION 16

/* aggregation: conv.py:41 (`sym` -> fn.sum with deg^-1/2 norms conv.py:54-57).  SIR_AGG_ACCUMULATE,
 * OR'd into the forward's `agg` (SUM / SYM): S[v] = S[v] + the sum over the given items' edges, rows
 * without items untouched — the segmented forward of the multi-GPU edge-cut (a row's edges in fixed
 * segments by source owner, each aggregated as its halo rows land; sirgcn/dist.py). */
enum { SIR_AGG_SUM = 0, SIR_AGG_MEAN = 1, SIR_AGG_SYM = 2, SIR_AGG_ACCUMULATE = 16 };
/* sigma: the `activation` callable of conv.py:32,45 (ReLU, LeakyReLU(slope), GELU erf / tanh) */
enum { SIR_ACT_IDENTITY = 0, SIR_ACT_RELU = 1, SIR_ACT_LEAKY_RELU = 2, SIR_ACT_GELU = 3, SIR_ACT_GELU_TANH = 4 };
/* Storage dtype of every feature matrix of an edge-pass call (Q, K, G, S, dQ, dK, Gm): fp32, or the
 * 16-bit types the reference's AMP path produces (torch.amp.autocast, heterophilous-datasets/train.py:75;
 * fp16 is autocast's CUDA default, bf16 is BASELINE config 2).  16-bit values are widened to fp32 on
 * load; sigma, sigma', the norm product and the accumulation run in fp32 (the reference promotes its
 * messages to fp32 before the reduction) and each output is rounded once (RNE).
 * Deviation from the reference's AMP dataflow (stated, not hidden): autocast forms eq + ek as a 16-bit
 * add and sigma's output in 16 bits before the norm multiply promotes it; here z = Q[v] + K[u] and
 * sigma(z) stay fp32 (no intermediate 16-bit rounding), and the autocast layer keeps dX and the weight
 * gradients in fp32 (the reference rounds them to the 16-bit type first).  The results are at least
 * as accurate; parity under autocast is tolerance-level (tests/test_amp_gpu.py), never bit-level, and a
 * GradScaler step that the reference would skip on a 16-bit overflow of dW is not skipped here.
 * 16-bit storage needs H % 4 == 0 and leading dimensions that are multiples of 4 (8-B aligned rows).
 * Norms and the `partial` workspace are fp32 in every mode. */
enum { SIR_DTYPE_F32 = 0, SIR_DTYPE_BF16 = 1, SIR_DTYPE_F16 = 2 };
/* error codes */
enum { SIR_OK = 0, SIR_EINVAL = 1, SIR_EUNSUPPORTED = 2, SIR_ELAUNCH = 3 };

int sir_abi_version(void);
/* First 16 hex digits of sha256 over the library's kernel and ABI sources (the .hip, .h and .cpp files
 * of csrc/ and the .h files of include/, concatenated in path order) at build time: lets a host detect a stale prebuilt library. */
const char* sir_source_hash(void);
const char* sir_last_error(void);

/*
 * Feature dropout on Q and K — conv.py:35,60-61: K = Dropout(p)(X W_K^T), Q = Dropout(p)(X W_Q^T + b_Q),
 * two independent nn.Dropout masks (the reference trains with p = 0.1-0.2, e.g. ogbn-arxiv/train.py:303).
 * Element (row, col) of QK = [Q | K] (col < H: Q, col >= H: K) is kept iff a counter-based hash of
 * (seed, row, col) is >= round(p * 2^32); kept elements are scaled by 1 / (1 - p) (fp32).  No mask
 * is stored: the QK GEMM applies it to its output (sir_gemm_nt / sir_gemm_nt16, C column = QK
 * column), the backward edge passes apply the same bits to dQ (columns 0..H-1) and dK (H..2H-1)
 * before storing them — the dropout's backward (grad * mask * scale).  16-bit outputs scale the value
 * rounded to the 16-bit type and round again (the reference's Dropout of a half-precision tensor).
 * A NULL pointer, or p <= 0, means no dropout; p >= 1 drops everything.  `seed_ptr` (may be NULL): a
 * DEVICE pointer to the 64-bit seed, read by each kernel when it starts, overriding `seed` — the
 * graph-safe form: a HIP graph that captured the launch together with the device op writing the
 * seed (the host's RNG draw on the stream) replays with a fresh mask each time, and the backward
 * passes given the same pointer read the same seed.
 */
typedef struct {
    uint64_t seed;
    double p;
    const uint64_t* seed_ptr;
} sir_dropout_t;

/* In place: X[m][n] = keep(m, col0 + n) ? X[m][n] * scale : 0 for an [M, N] block of QK (ldx
 * elements per row, dtype SIR_DTYPE_*) — the forward dropout of a QK computed by another GEMM. */
int sir_dropout_apply(void* X, int64_t ldx, int64_t M, int64_t N, int dtype, int64_t col0,
                      const sir_dropout_t* drop, void* stream);

/*
 * Per-edge sign-mask size (64-bit words) for hidden size H and activation `act`, or 0 when
 * the sign-mask backward is not available (needs act in {RELU, LEAKY_RELU}, H % 4 == 0,
 * H <= 1024, 16-B aligned rows).  Layout, edge e in destination-CSR order:
 *   128 < H (full-wave rows): word mask[e*NW + 4*j + w], bit l = (Q[v] + K[u])[4*(l + 64*j) + w] > 0;
 *   H <= 128 (rows of L = 4, 8, 16 or 32 lanes, L = the smallest holding H/4): a record of
 *   NW 64-bit words (NW = max(L/16, 1)) read as little-endian bits, bit (w*L + l) =
 *   (Q[v] + K[u])[4*l + w] > 0 (bits past H zero).
 */
int64_t sir_mask_words(int64_t H, int act);

/*
 * conv.py:51-57 degree normalisers: norm[i] = 1 / sqrt((float)max(deg_i, 1)) with
 * deg_i = rowptr[i+1] - rowptr[i] (IEEE sqrt and division: the bits CPU torch.pow(d, -0.5)
 * returns).  Computes in_norm from the destination CSR and (if non-NULL) out_norm from the
 * source CSR, n = number of nodes.
 */
int sir_degree_norms(const int32_t* rowptr_dst, float* in_norm,
                     const int32_t* rowptr_src, float* out_norm, int64_t n, void* stream);

/*
 * Column sums out[c] = sum_r X[r*ld + c] of a tall fp32 matrix — the bias gradients of the
 * layer's linears (db_R = sum_v dY[v], db_Q = sum_v dQ[v]; autograd of conv.py:61,65).
 * Deterministic (fixed two-level order).  n_cols % 4 == 0, ld % 4 == 0, X 16-B aligned;
 * workspace: SIR_COLSUM_BLOCKS * n_cols floats.
 */
#define SIR_COLSUM_BLOCKS 1024
int sir_col_sum(const float* X, int64_t ld, int64_t n_rows, int64_t n_cols, float* out,
                float* workspace, void* stream);

/*
 * Forward edge aggregation — replaces conv.py:63 (update_all with the sum/mean/sym UDF).
 *   S[v] = sum_{e in row v} c_e * sigma(Q[v] + K[col[e]]),  c_e = norm_col[u] * norm_row[v]
 *   (SYM only; SUM/MEAN use c_e = 1 exactly as ones*ones in conv.py:45), MEAN divides by
 *   max(degree, 1) afterwards (DGL fn.mean).  Rows with no edges get S = 0.
 *   rowptr/col: row CSR by destination (rows = dst nodes, col = src node ids).
 *   Q: [n_rows, H] (ldq) indexed by row;  K: [*, H] (ldk) indexed by col.
 *   norm_row / norm_col: fp32 (SYM only, else may be NULL).
 *   mask_out: NULL, or E * sir_mask_words(H, act) words receiving the sign of every z
 *   (input of the sign-mask backward).
 */
int sir_edge_agg_fwd(const int32_t* rowptr, const int32_t* col,
                     const int32_t* items, int64_t n_items,
                     const int32_t* splits, int64_t n_splits,
                     int64_t H, int dtype,
                     const void* Q, int64_t ldq, const void* K, int64_t ldk,
                     const float* norm_row, const float* norm_col,
                     int agg, int act, float slope,
                     void* S, int64_t lds, uint64_t* mask_out, float* partial, void* stream);

/*
 * Backward, destination pass — the Q half of autograd through conv.py:45,63.
 *   g = G[v] (MEAN: G[v] / max(deg v, 1)),  t_e = g * c_e (SYM) or g,
 *   dQ[v] = sum_{e in row v} sigma'(Q[v] + K[u]) * t_e   (sigma' as torch's backward).
 *   If MEAN and Gm != NULL, the divided rows g are also written to Gm (for the src pass).
 *   16-bit storage: g is rounded to the storage dtype before use (the values written to Gm), so
 *   both passes see the same g.
 *   mask != NULL selects the sign-mask mode: sigma'(z) is read from the forward's mask and
 *   Q, K are not touched (may be NULL); results are bit-identical to the recompute mode.
 */
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
                         float* partial, const sir_dropout_t* drop, void* stream);

/*
 * Backward, source pass — the K half (replaces the index_add of conv.py:45's src gather).
 *   Row CSR by SOURCE: rows = src nodes u, col = dst node ids v (ascending edge id).
 *   dK[u] = sum_{e in row u} sigma'(Q[v] + K[u]) * t_e,  t_e = Gd[v] * c_e (SYM) or Gd[v],
 *   where Gd is the already-divided gradient (MEAN: the Gm of the dst pass; else G).
 *   norm_row = out-norm of u, norm_col = in-norm of v (SYM only).
 *   mask != NULL: sign-mask mode (K, Q unused); perm_s[j] = destination-CSR position of the
 *   edge at source-CSR position j (indexes the mask).
 */
int sir_edge_agg_bwd_src(const int32_t* rowptr_s, const int32_t* col_s, const int32_t* perm_s,
                         const int32_t* items, int64_t n_items,
                         const int32_t* splits, int64_t n_splits,
                         int64_t H, int dtype,
                         const void* K, int64_t ldk, const void* Q, int64_t ldq,
                         const uint64_t* mask,
                         const void* Gd, int64_t ldg,
                         const float* norm_row, const float* norm_col,
                         int agg, int act, float slope,
                         void* dK, int64_t lddk, float* partial, const sir_dropout_t* drop, void* stream);

/*
 * Both backward passes in ONE launch — sign-mask mode, SUM or SYM (MEAN's source pass needs the
 * destination pass's Gm first: use the two calls above).  Same results, bit for bit, as
 * sir_edge_agg_bwd_dst followed by sir_edge_agg_bwd_src with the same arguments; the destination
 * pass (VALU-bound) and the source pass (HBM-bound) share the CUs instead of running one after the
 * other.  in_norm / out_norm: the SYM degree norms (NULL otherwise).  The two passes write their
 * split rows' partial sums to separate workspaces: partial (destination plan's slots * H floats)
 * and partial_s (source plan's slots * H floats).
 */
int sir_edge_agg_bwd(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                     const int32_t* splits, int64_t n_splits,
                     const int32_t* rowptr_s, const int32_t* col_s, const int32_t* perm_s,
                     const int32_t* items_s, int64_t n_items_s, const int32_t* splits_s, int64_t n_splits_s,
                     int64_t H, int dtype, const uint64_t* mask, const void* G, int64_t ldg,
                     const float* in_norm, const float* out_norm, int agg, int act, float slope,
                     void* dQ, int64_t lddq, void* dK, int64_t lddk, float* partial, float* partial_s,
                     const sir_dropout_t* drop, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Edge-materialised path: agg_type='max' (conv.py:46-47 + DGL max reduce) and sigma callables the
 * fused kernels do not cover (e.g. Sequential(ReLU, Linear, ReLU), dictionary-lookup/model.py:17).
 * Edge rows are in destination-CSR order (position e of the dst CSR).  F = feature width
 * (<= 1024).  Same work plan (items / splits) as above.
 * ------------------------------------------------------------------------------------------- */

/* Z[e] = Q[row(e)] + K[col[e]]  (the `edges.dst['eq'] + edges.src['ek']` of conv.py:45) */
int sir_edge_gather_add(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                        int64_t F, const float* Q, int64_t ldq, const float* K, int64_t ldk,
                        float* Z, int64_t ldz, void* stream);

/* A[e] = act(Q[row(e)] + K[col[e]]), act = SIR_ACT_IDENTITY / _RELU / _LEAKY_RELU (slope): the
 * materialised max backward's activations in one pass (conv.py:45-47; for the ReLU family sign(A)
 * = sign(z), so sigma' is taken from A and z is never stored).  sign_mask (optional, F = 256):
 * uint64[E][4], bit l of word x = A[e][4 l + x] > 0 — the gate of sir_gemm_nt_dact.  ABI 12. */
int sir_edge_gather_act(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                        int64_t F, const float* Q, int64_t ldq, const float* K, int64_t ldk, int act, float slope,
                        float* A, int64_t lda, uint64_t* sign_mask, void* stream);

/* out[row] = sum_{e in row} c_e * X[idx(e)],  idx(e) = perm ? perm[e] : e,
 * c_e = norm_col[col[e]] * norm_row[row] when norm_row != NULL (the sym norm product, conv.py:45),
 * mean != 0 divides by max(deg, 1) (fn.mean).  Rows without edges get 0.  Sequential in edge order
 * within a row (split rows: partial rows combined in slot order; partial = n_slots * F floats).
 * With the destination CSR this is update_all(copy_e, sum|mean); with the source CSR and perm it
 * is the index_add of the src gather's backward (dK). */
int sir_segment_sum(const int32_t* rowptr, const int32_t* col, const int32_t* perm,
                    const int32_t* items, int64_t n_items, const int32_t* splits, int64_t n_splits,
                    int64_t F, const float* X, int64_t ldx, const float* norm_row, const float* norm_col,
                    int mean, float* out, int64_t ldo, float* partial, void* stream);

/* Backward of sir_segment_sum over the destination CSR: dM[e] = c_e * g[row],
 * g = dS (mean: dS / max(deg, 1)). */
int sir_edge_broadcast(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                       int64_t F, const float* dS, int64_t lds, const float* norm_row, const float* norm_col,
                       int mean, float* dM, int64_t ldm, void* stream);

/* DGL max reduce: Y[row] = max_{e in row} M[e] elementwise, arg = the FIRST arg-max edge position
 * (ties keep the earlier edge), rows without edges: Y = 0, arg = -1.
 * pval/parg: n_slots * F workspace for split rows. */
int sir_segment_max(const int32_t* items, int64_t n_items, const int32_t* splits, int64_t n_splits,
                    int64_t F, const float* M, int64_t ldm, float* Y, int64_t ldy, int32_t* arg, int64_t lda,
                    float* pval, int32_t* parg, void* stream);

/* Backward of sir_segment_max: dM[e] = (arg[row] == e) ? dY[row] : 0 for every edge (dM fully written). */
int sir_segment_max_bwd(const int32_t* items, int64_t n_items, int64_t F, const int32_t* arg, int64_t lda,
                        const float* dY, int64_t ldy, float* dM, int64_t ldm, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fused per-edge dense layer.  For every edge u->v of a destination row:
 *   z = Q[v] + K[u],  a = act1(z),  h = W a + b,  m = act2(h)
 * reduced into out[v]: SUM / MEAN / SYM (c_e = norm_col[u] * norm_row[v]) as sir_edge_agg_fwd, or
 * SIR_AGG_MAX: elementwise max with the FIRST arg-max edge's destination-CSR position in arg
 * (rows without edges: 0 / -1) — DGL fn.max.  Covers conv.py:45 with sigma = Sequential(act1,
 * Linear(H, F), act2) (dictionary-lookup/model.py:17) and conv.py:46-47 (agg_type='max': W = W_R,
 * act2 = identity).  No per-edge tensor is written.  fp32 throughout (MFMA fp32 products).
 * W: [F, H] row-major (an nn.Linear weight), packed once by sir_edge_mlp_pack.  Limits: H % 4 == 0,
 * H <= 512, F <= 512, Q/K 16-B aligned rows.  act2 in {IDENTITY, RELU}.  Split rows: pval
 * (n_slots * F floats) and, for MAX, parg (n_slots * F ints).
 * ------------------------------------------------------------------------------------------- */
#define SIR_AGG_MAX 3
int64_t sir_edge_mlp_pack_bytes(int64_t H, int64_t F);
int sir_edge_mlp_pack(const float* W, int64_t H, int64_t F, void* packed, void* stream);
int sir_edge_mlp_fwd(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                     const int32_t* splits, int64_t n_splits, int64_t H, int64_t F,
                     const float* Q, int64_t ldq, const float* K, int64_t ldk,
                     const float* norm_row, const float* norm_col, int agg, int act1, float slope, int act2,
                     const void* packed, const float* bias, float* out, int64_t ldo, int32_t* arg, int64_t lda,
                     float* pval, int32_t* parg, void* stream);

/* The same forward over the dst-CSR edge STREAM (H = 256, F <= 256: the S1 / S2 max shape): 32-edge
 * MFMA tiles are consecutive windows of each block's edge range, so short rows share a tile.
 * erow[e] = destination row of dst-CSR edge e (n_edges entries); work = sir_edge_mlp_stream_work_bytes(F)
 * bytes (per-block boundary partials).  Same outputs as sir_edge_mlp_fwd (MAX: bit-identical values
 * and first arg-max edges; the sum family adds each row's terms in edge order).  ABI 12. */
int64_t sir_edge_mlp_stream_work_bytes(int64_t F);
int sir_edge_mlp_fwd_stream(const int32_t* rowptr, const int32_t* col, const int32_t* erow, int64_t n_rows,
                            int64_t n_edges, int64_t H, int64_t F, const float* Q, int64_t ldq, const float* K,
                            int64_t ldk, const float* norm_row, const float* norm_col, int agg, int act1, float slope,
                            int act2, const void* packed, const float* bias, float* out, int64_t ldo, int32_t* arg,
                            int64_t lda, void* work, void* stream);

/* agg='max' under autocast (heterophilous-datasets/train.py:75, ABI 15): Q / K rows stored in bf16 or fp16
 * (dtype SIR_DTYPE_BF16 / F16, rows 8-B aligned, ld % 4 == 0).  z = Q[v] + K[u] and act1 in fp32, a
 * rounded once to dtype, h = a W^T + b as ONE dtype MFMA per 16 k with fp32 accumulation on W and b
 * rounded to dtype (autocast's half-precision Linear), the max and the first arg-max edge over the fp32
 * h.  W packed by sir_edge_mlp_pack_st with the same dtype (sir_edge_mlp_pack_bytes bytes).  agg must be
 * SIR_AGG_MAX, act2 IDENTITY; otherwise the arguments, outputs (fp32 out) and limits of sir_edge_mlp_fwd /
 * sir_edge_mlp_fwd_stream. */
int sir_edge_mlp_pack_st(const float* W, int64_t H, int64_t F, int dtype, void* packed, void* stream);
int sir_edge_mlp_fwd_st(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                        const int32_t* splits, int64_t n_splits, int64_t H, int64_t F, const void* Q, int64_t ldq,
                        const void* K, int64_t ldk, int dtype, int agg, int act1, float slope, int act2,
                        const void* packed, const float* bias, float* out, int64_t ldo, int32_t* arg, int64_t lda,
                        float* pval, int32_t* parg, void* stream);
int sir_edge_mlp_fwd_stream_st(const int32_t* rowptr, const int32_t* col, const int32_t* erow, int64_t n_rows,
                               int64_t n_edges, int64_t H, int64_t F, const void* Q, int64_t ldq, const void* K,
                               int64_t ldk, int dtype, int agg, int act1, float slope, int act2, const void* packed,
                               const float* bias, float* out, int64_t ldo, int32_t* arg, int64_t lda, void* work,
                               void* stream);

/* Backward of the SUM / MEAN / SYM form (H, F <= 256): the destination pass writes dQ [rows, H] and one
 * partial [dW (FP x HP) | db (FP)] row per block into wpart (FP = F rounded up to 32, HP = H rounded up
 * to 8; sir_edge_mlp_bwd_parts(n_items, H, F) rows of FP*HP + FP floats: sum them in row order, e.g.
 * with sir_col_sum); MEAN also writes Gm = G / deg [rows, F] for the source pass.  The source pass
 * (rows = sources, col = destinations) writes dK [rows, H] from Gd (= Gm for MEAN, else G).
 * Split rows: partial = n_slots * H floats.  Deterministic (no atomics).  (ABI 9: replaces
 * sir_edge_mlp_bwd_waves(n_items), whose H, F <= 64 kernels these generalise.) */
int64_t sir_edge_mlp_bwd_parts(int64_t n_items, int64_t H, int64_t F);
int sir_edge_mlp_bwd_dst(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                         const int32_t* splits, int64_t n_splits, int64_t H, int64_t F,
                         const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* G, int64_t ldg,
                         const float* norm_row, const float* norm_col, int agg, int act1, float slope, int act2,
                         const void* packed, const float* W, const float* bias, float* dQ, int64_t lddq,
                         float* Gm, float* partial, float* wpart, void* stream);
int sir_edge_mlp_bwd_src(const int32_t* rowptr_s, const int32_t* col_s, const int32_t* items, int64_t n_items,
                         const int32_t* splits, int64_t n_splits, int64_t H, int64_t F,
                         const float* K, int64_t ldk, const float* Q, int64_t ldq, const float* Gd, int64_t ldg,
                         const float* norm_row, const float* norm_col, int agg, int act1, float slope, int act2,
                         const void* packed, const float* W, const float* bias, float* dK, int64_t lddk,
                         float* partial, void* stream);

/* Backward of the SIR_AGG_MAX form (conv.py:46-47, act2 = identity, W = W_R [O, H]) for H, O <= 256,
 * without any [E, *] tensor: dm_e[o] = dY[v][o] if edge e is the first arg-max edge of (v, o) (arg
 * from sir_edge_mlp_fwd: dst-CSR positions, -1 for empty rows), else 0; then, recomputing z and a
 * per edge, da = dm W, dz = act1'(z) da.  The destination pass writes dQ [rows, H] and one partial
 * [dW_R (OP x HP) | db_R (OP)] row per block into wpart (sir_edge_mlp_bwd_parts(n_items, H, O) rows,
 * OP = O rounded up to 32, HP = H rounded up to 8: sum them in row order).  The source pass (rows =
 * sources, col = destinations, perm = the source CSR's dst-CSR positions) writes dK [rows, H].
 * Split rows: partial = n_slots * H floats.  Deterministic (no atomics). */
int sir_edge_max_bwd_dst(const int32_t* rowptr, const int32_t* col, const int32_t* items, int64_t n_items,
                         const int32_t* splits, int64_t n_splits, int64_t H, int64_t O,
                         const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* dY, int64_t ldy,
                         const int32_t* arg, int64_t lda, int act1, float slope, const float* W,
                         float* dQ, int64_t lddq, float* partial, float* wpart, void* stream);
int sir_edge_max_bwd_src(const int32_t* rowptr_s, const int32_t* col_s, const int32_t* perm_s,
                         const int32_t* items, int64_t n_items, const int32_t* splits, int64_t n_splits,
                         int64_t H, int64_t O, const float* K, int64_t ldk, const float* Q, int64_t ldq,
                         const float* dY, int64_t ldy, const int32_t* arg, int64_t lda, int act1, float slope,
                         const float* W, float* dK, int64_t lddk, float* partial, void* stream);

/* agg_type='max' backward from the arg-max routing alone (conv.py:46-47; ABI 14): dY[v][o] reaches only
 * the first arg-max edge arg[v][o] (a dst-CSR position in [rowptr[v], rowptr[v+1]), else none), so
 *   dA_e = sum_{o : arg[v][o] = e} dY[v][o] W[o, :],  dz_e = act1'(Q[v] + K[u]) dA_e,
 *   dQ[v] = sum_e dz_e (dst CSR),  dK[u] = sum_e dz_e (src CSR),
 *   dW[o, :] = sum_v dY[v][o] act1(Q[v] + K[col[arg[v][o]]]),  db[o] = sum_v dY[v][o]
 * with V * O * H multiply-adds per product (not E * O * H) and no [E, H] / [E, O] buffer.  Workspace:
 * ent = 8 * V * O + 64 bytes (V * O < 2^31; ABI 16: the last 64 bytes hold the dQ / dK passes' work-queue
 * counters, zeroed by the call), ecnt_d / ecnt_s = 8 * E bytes each, partial = max(n_slots) * H
 * floats, dbpart = route_blocks * O4 floats (O4 = O rounded up to 4) and wpart = dw_ranges * O * H floats (the sizes from
 * sir_edge_max_bwd_sparse_parts; sum each over its rows in row order for db / dW, e.g. sir_col_sum;
 * wpart NULL skips the dW pass, for a caller that has A and uses sir_max_dw_rows).  With no work items
 * (n_items_d == 0) dbpart, and with V == 0 wpart, is written as zeros.
 * pinv[dst-CSR position] = src-CSR position (the inverse of the source CSR's perm).  H % 4 == 0,
 * H <= 512, O <= 256, Q / K / W rows 16-B aligned.  Deterministic (no atomics). */
int sir_edge_max_bwd_sparse_parts(int64_t n_items_d, int64_t V, int64_t* route_blocks, int64_t* dw_ranges);
int sir_edge_max_bwd_sparse(const int32_t* rowptr_d, const int32_t* col_d, const int32_t* items_d, int64_t n_items_d,
                            const int32_t* splits_d, int64_t n_splits_d, const int32_t* col_s,
                            const int32_t* items_s, int64_t n_items_s, const int32_t* splits_s, int64_t n_splits_s,
                            const int32_t* pinv, int64_t V, int64_t E, int64_t H, int64_t O,
                            const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* dY, int64_t ldy,
                            const int32_t* arg, int64_t lda, int act1, float slope, const float* W,
                            float* dQ, int64_t lddq, float* dK, int64_t lddk, float* partial, void* ent,
                            void* ecnt_d, void* ecnt_s, float* dbpart, float* wpart, void* stream);

/* dW_R / db_R of the edge-materialised max backward without dM [E, O] (ABI 14): A [E, H] = act1(z_e) in
 * dst-CSR order, dW[o, :] = sum_v dY[v][o] A[arg[v][o], :], db[o] = sum_v dY[v][o] (arg[v][o] in
 * [rowptr[v], rowptr[v+1]), else no term).  wpart: sir_max_dw_rows_parts(V, H) rows of ldw >= O * H + O4
 * floats (O4 = O rounded up to 4): [dW (O x H, row-major) | db (O4)] per row; sum them in row order (e.g.
 * sir_col_sum).  O <= 256, H % 4 == 0, A rows 16-B aligned.  Deterministic.  V == 0: the one row of
 * wpart (sir_max_dw_rows_parts(0, H) == 1) is written as zeros (wpart may then be NULL). */
int64_t sir_max_dw_rows_parts(int64_t V, int64_t H);
/* The same dW_R / db_R without A: a = act1(Q[v] + K[col[e]]) recomputed per row batch (dst CSR rowptr /
 * col), so with sir_edge_max_bwd_sparse (wpart NULL) the max backward holds no [E, *] buffer.  Same wpart
 * layout and sizes as sir_max_dw_rows; Q / K rows 16-B aligned. */
int sir_max_dw_qk(const int32_t* rowptr, const int32_t* col, int64_t V, const int32_t* arg, int64_t lda,
                  const float* dY, int64_t ldy, const float* Q, int64_t ldq, const float* K, int64_t ldk, int64_t O,
                  int64_t H, int act1, float slope, float* wpart, int64_t ldw, void* stream);
int sir_max_dw_rows(const int32_t* rowptr, int64_t V, const int32_t* arg, int64_t lda, const float* dY, int64_t ldy,
                    const float* A, int64_t ldA, int64_t O, int64_t H, float* wpart, int64_t ldw, void* stream);

/* ---------------------------------------------------------------------------------------------
 * GraphNorm (models/norm.py:7-29) on a batched graph: graph b owns node rows [off[b], off[b+1])
 * (off = int64 [B+1], the prefix sum of batch_num_nodes).  Per graph and feature:
 *   mean = sum x / n,  d = x - mean * mean_scale,  std = sqrt(sum d^2 / n + eps),
 *   y = (weight * d) / std + bias
 * Sums run in node order (the reference's scatter_add_ order).  bias / mean_scale may be NULL
 * (the reference's bias=False -> + 0, mean_scale=False -> * 1).  mean/std: [B, F] outputs kept
 * for the backward.  F <= 65536.
 * ------------------------------------------------------------------------------------------- */
int sir_graph_norm_fwd(const int64_t* off, int64_t B, int64_t F, const float* X, int64_t ldx,
                       const float* weight, const float* bias, const float* mean_scale, float eps,
                       float* Y, int64_t ldy, float* mean, float* std_, void* stream);

/* Backward: dX (fully written) and per-graph partials [B, F] of the parameter gradients
 * (dweight = sum_b dw_part, dmean_scale = sum_b dms_part, dbias = sum_b db_part; dms_part may be
 * NULL when mean_scale is NULL). */
int sir_graph_norm_bwd(const int64_t* off, int64_t B, int64_t F, const float* X, int64_t ldx,
                       const float* dY, int64_t ldg, const float* weight, const float* mean_scale,
                       const float* mean, const float* std_, float* dX, int64_t lddx,
                       float* dw_part, float* dms_part, float* db_part, void* stream);

/* The stack's residual and activation around a layer without a norm, one pass per direction
 * (zinc/model.py:53-56: order 0, out = act(Y + R); ogbn-arxiv/model.py:65-73 without its norm:
 * order 1, out = act(Y) + R).  Y [M, N] is the layer output in `dtype` (SIR_DTYPE_F32 / BF16 / F16:
 * the autocast layer's 16-bit output), R and out fp32; act = SIR_ACT_IDENTITY / _RELU /
 * _LEAKY_RELU (slope).  The same ops, types and order as torch's add, relu / leaky_relu and their
 * autograd (a 16-bit activation rounds to its type, a 16-bit gradient is rounded once from fp32):
 * bit-identical to the separate torch kernels.  Backward: D = dout (fp32); dY in `dtype`; order 0
 * also writes dR = act'(Y + R) D (order 1: dR is D itself, DR ignored).  D2 (optional; ABI 16): a
 * second fp32 gradient of out, added to D as it is read — the residual gradient of the next layer,
 * whose input out is (the sum autograd would otherwise form in its own pass); order 1 then writes that
 * sum D + D2 to dR (required).  N % 4 == 0; rows 16-B
 * aligned (leading dimensions multiples of 4 elements).  ABI 13. */
int sir_resid_act_fwd(const void* Y, int64_t ldy, int dtype, const float* R, int64_t ldr, float* out, int64_t ldo,
                      int64_t M, int64_t N, int act, float slope, int order, void* stream);
int sir_resid_act_bwd(const float* D, int64_t ldd, const float* D2, int64_t ldd2, const void* Y, int64_t ldy, int dtype,
                      const float* R, int64_t ldr, void* dY, int64_t lddy, float* dR, int64_t lddr, int64_t M, int64_t N,
                      int act, float slope, int order, void* stream);

/* GraphNorm with the stack's activation and residual after it, one kernel per direction — the
 * layer loop of ogbn-arxiv/model.py:65-73 / ogbg-molhiv/model.py:76-84 (h = act(norm(h)) + resid)
 * and, with R = NULL, zinc/model.py:54-55 (h = act(norm(h))).  Forward: Y = act(y) + R with y the
 * sir_graph_norm_fwd output and act = SIR_ACT_IDENTITY / _RELU / _LEAKY_RELU (slope): torch's
 * relu / leaky_relu and add, the same ops (bit-identical to the three separate calls).  Backward:
 * dY is the gradient of Y; the kernel takes act'(y) dY (y recomputed by the forward's own ops, so
 * on the same side of 0; leaky_relu_backward's y > 0 ? g : g * slope) into the GraphNorm backward;
 * R's gradient is dY itself (the caller's).  bias as in the forward (NULL: none).  ABI 13. */
int sir_graph_norm_act_fwd(const int64_t* off, int64_t B, int64_t F, const float* X, int64_t ldx,
                           const float* weight, const float* bias, const float* mean_scale, float eps, int act,
                           float slope, const float* R, int64_t ldr, float* Y, int64_t ldy, float* mean, float* std_,
                           void* stream);
int sir_graph_norm_act_bwd(const int64_t* off, int64_t B, int64_t F, const float* X, int64_t ldx,
                           const float* dY, int64_t ldg, const float* weight, const float* bias,
                           const float* mean_scale, const float* mean, const float* std_, int act, float slope,
                           float* dX, int64_t lddx, float* dw_part, float* dms_part, float* db_part, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Device-side graph plan build.  Replaces DGL's lazily built in-edge CSC
 * (the COO -> CSR counting sort DGL runs on the first update_all, conv.py:63) and this repo's
 * work-plan construction, for batched graphs / DropEdge re-builds (models/utils.py:96-102).
 *
 * rows, cols: int64 [E] device (for the in-edge CSR: rows = dst, cols = src); ids are checked
 * against [0, n_rows) / [0, n_cols) ON THE DEVICE: the count of bad ids lands in counts[4] and
 * the caller must check it (the plan is garbage when it is non-zero).  Outputs (device):
 *   rowptr int32 [n_rows+1]; col int32 [E]; eid int64 [E] (edge ids, ascending inside a row —
 *   a stable sort, DGL's order); items int32 [n_rows + E/chunk][4] and splits int32
 *   [min(n_rows, E/(chunk+1)) + 1][4] (capacities; the used counts are written to counts);
 *   counts int64 [5] = {n_items, n_splits, n_slots, max_degree, n_bad_ids}.
 * workspace: sir_csr_build_workspace(n_rows, E) bytes.  E < 2^31, 1 <= chunk.
 * ------------------------------------------------------------------------------------------- */
int64_t sir_csr_build_workspace(int64_t n_rows, int64_t E);

int sir_csr_build(const int64_t* rows, const int64_t* cols, int64_t E, int64_t n_rows, int64_t n_cols,
                  int64_t chunk, int32_t* rowptr, int32_t* col, int64_t* eid, int32_t* items, int32_t* splits,
                  int64_t* counts, void* workspace, int64_t workspace_bytes, void* stream);

/* perm[j] = position in CSR A of the edge at position j of CSR B (eid_a, eid_b: the two CSRs'
 * edge-id arrays over the same E edges).  pos_ws: int32 [E] scratch.  Used for the src-CSR ->
 * dst-CSR map of the sign-mask backward. */
int sir_csr_perm(const int64_t* eid_a, const int64_t* eid_b, int64_t E, int32_t* pos_ws, int32_t* perm,
                 void* stream);

/* ---------------------------------------------------------------------------------------------
 * Projection GEMMs of the layer: the nn.Linear calls conv.py:60-61 (Q, K), conv.py:65 (W_R) and
 * their autograd (G = dY W_R, dX, dW_R, dW_Q, dW_K).  fp32 in / fp32 out, computed on fp16 MFMA
 * with every operand split into two fp16 terms under a power-of-two scale per contraction row
 * (hi*hi + hi*lo + lo*hi, fp32 accumulation): the accuracy of an fp32 GEMM (tests hold it to
 * <= 2x torch fp32's error against fp64).  Not bit-identical to any fp32 BLAS (neither is one
 * BLAS to another).  Elements more than 2^29 below their row's maximum lose relative precision
 * (absolute error <= 2^-40 of that maximum).
 * ------------------------------------------------------------------------------------------- */

/* Largest leading dimension (elements) of a GEMM data operand: a 256-row tile is addressed with
 * 32-bit byte offsets.  Larger strides are rejected with SIR_EINVAL. */
#define SIR_GEMM_MAX_LD (1 << 20)

/* Weight operand B [N, K] for sir_gemm_nt: B[n][k] = W[n*ldw + k] (trans = 0, an nn.Linear
 * weight used as x W^T) or W[k*ldw + n] (trans = 1, x W).  packed: sir_gemm_pack_bytes(N, K)
 * bytes, 16-B aligned; re-pack whenever W changes. */
int64_t sir_gemm_pack_bytes(int64_t N, int64_t K);
int sir_gemm_pack(const float* W, int64_t ldw, int64_t N, int64_t K, int trans, void* packed, void* stream);

/* C[M, N] = A[M, K] B^T + bias  (bias [N] or NULL).  A, C row-major; K, N, lda, ldc multiples of
 * 4; A, C, bias 16-B aligned.  Replaces addmm(b, X, W^T) / mm(X, W). */
int sir_gemm_nt(const float* A, int64_t lda, int64_t M, int64_t K, const void* packed, int64_t N,
                const float* bias, float* C, int64_t ldc, const sir_dropout_t* drop, void* stream);

/* C = sigma'(gate) * (A B^T) with B packed as for sir_gemm_nt: gate [M, N] with C's leading dimension
 * (the activation's input z or output sigma(z): the same sign for the ReLU family); act =
 * SIR_ACT_RELU (gate > 0 ? x : 0) or SIR_ACT_LEAKY_RELU (gate > 0 ? x : x * slope) — torch's
 * threshold / leaky_relu backward fused into the GEMM's epilogue (the materialised max backward's
 * dZ = sigma'(z) * (dM W_R), conv.py:46-47).  gate_mask (instead of gate, N = 256): the sign
 * words of sir_edge_gather_act — 32 B per row read instead of the row's gate values.  ABI 12. */
int sir_gemm_nt_dact(const float* A, int64_t lda, int64_t M, int64_t K, const void* packed, int64_t N,
                     const float* gate, const uint64_t* gate_mask, int act, float slope, float* C, int64_t ldc,
                     void* stream);

/* Small batches (config 5's 1.6k-node molecule batches): C[M, N] = A[M, K] B^T + bias with the
 * weight read as fp32 straight from W (B[n][k] = W[n*ldw + k], trans = 0, or W[k*ldw + n], trans =
 * 1) — no packing pass per weight update; both operands split in the kernel, each with running
 * scales.  Same accuracy bar as sir_gemm_nt (fp32-equivalent); any M, but the small tiles (64 weight
 * lines x 32 rows, LDS-DMA staged; a 4-byte-aligned W takes a register-load kernel) and the
 * in-kernel weight split make it the route for M below ~16k rows only.  K, N, lda, ldc multiples of
 * 4; A, C, bias 16-B aligned; ldw <= SIR_GEMM_MAX_LD.  Replaces addmm(b, X, W^T) / mm(X, W). */
int sir_gemm_nt_direct(const float* A, int64_t lda, int64_t M, int64_t K, const float* W, int64_t ldw, int trans,
                       int64_t N, const float* bias, float* C, int64_t ldc, const sir_dropout_t* drop, void* stream);

/* sir_gemm_nt_direct with the weight in two parts and a partial bias: weight rows r < split come
 * from W, rows r >= split from W2 (row r - split; the rows are output features for trans = 0 and k
 * for trans = 1), and the bias covers the first bias_cols output columns (+ 0 on the rest) — the
 * layer's QK = X [W_Q; W_K]^T + [b_Q; 0] and dX = [dQ dK] [W_Q; W_K] (conv.py:60-61) without the
 * per-step torch.cat of the weights and the pad of the bias.  W, W2, bias 16-B aligned, ldw, ldw2
 * multiples of 4; 0 < split <= weight rows (split = rows: W alone); bias_cols % 4 == 0.  ABI 13. */
int sir_gemm_nt_direct2(const float* A, int64_t lda, int64_t M, int64_t K, const float* W, int64_t ldw,
                        const float* W2, int64_t ldw2, int64_t split, int trans, int64_t N, const float* bias,
                        int64_t bias_cols, float* C, int64_t ldc, const sir_dropout_t* drop, void* stream);

/* C[M, N] = A^T B with A [R, M] (lda), B [R, N] (ldb): the weight gradients (contraction over the
 * R node rows, split over row ranges; the partial products are added in a fixed order, so the
 * result is run-to-run deterministic).  colsum_a [M] or NULL: also the column sums of A
 * (sum_r A[r][m]) — the bias gradient of the same linear (db_R = sum dY with A = dY, db_Q with
 * A = dQ), read from the loads the GEMM does anyway; deterministic.
 * workspace: sir_gemm_tn_workspace(R, M, N) bytes. */
int64_t sir_gemm_tn_workspace(int64_t R, int64_t M, int64_t N);
int sir_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t R, int64_t M, int64_t N,
                float* C, int64_t ldc, float* colsum_a, void* workspace, int64_t workspace_bytes, void* stream);

/* The same contraction on 16-bit operands (the autocast path's weight gradients): A [R, M], B [R, N]
 * bf16 (dtype SIR_DTYPE_BF16) or fp16 (SIR_DTYPE_F16), C [M, N] and colsum_a [M] fp32.  Each 16-bit
 * product is exact in fp32, so one 16-bit MFMA per step with fp32 accumulation (no operand split,
 * no fp32 copies of A and B).  M, N, lda, ldb even; A, B 4-B aligned.  Replaces autograd's
 * mm(dY^T, S) / mm(dQK^T, X) of the half-precision nn.Linear (and their fp32 casts).
 * workspace: sir_gemm_tn_workspace(R, M, N) bytes. */
int sir_gemm_tn16(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t R, int64_t M, int64_t N, int dtype,
                  float* C, int64_t ldc, float* colsum_a, void* workspace, int64_t workspace_bytes, void* stream);

/* The forward projections and input gradients of the autocast path on 16-bit MFMA: the
 * half-precision nn.Linear (x W^T + b in bf16 / fp16, conv.py:60-61,65 under torch.autocast) and
 * its input gradient (dY W).  Weight operand packed by sir_gemm_pack16 (rounded to dtype, RNE;
 * re-pack whenever W changes; sir_gemm_pack16_bytes(N, K) bytes, 16-B aligned):
 *   C[M, N] = A[M, K] B^T + bias,  B[n][k] = W[n*ldw + k] (trans = 0) or W[k*ldw + n] (trans = 1).
 * dtype (SIR_DTYPE_BF16 / F16) is the MFMA type; a_dtype = dtype (A already 16-bit) or
 * SIR_DTYPE_F32 (A rounded to dtype on load: the autocast cast fused into the GEMM; with
 * Acopy != NULL the rounded A is also written to Acopy [M, K] (ldac)); c_dtype = dtype (RNE of the
 * fp32 accumulator) or SIR_DTYPE_F32.  bias [N] fp32 (the caller passes the dtype-rounded bias of
 * autocast) or NULL.  K in {128, 256, 512}; N <= 512; lda, N and ldc multiples of 16 bytes of
 * A / C (8 16-bit or 4 fp32 elements); ldc >= N; A, C, Acopy, packed 16-B aligned.  One 16-bit
 * MFMA per step, fp32 accumulation. */
int64_t sir_gemm_pack16_bytes(int64_t N, int64_t K);
int sir_gemm_pack16(const float* W, int64_t ldw, int64_t N, int64_t K, int trans, int dtype, void* packed, void* stream);
int sir_gemm_nt16(const void* A, int64_t lda, int a_dtype, int64_t M, int64_t K, const void* packed, int64_t N,
                  int dtype, const float* bias, void* C, int64_t ldc, int c_dtype, void* Acopy, int64_t ldac,
                  const sir_dropout_t* drop, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SIRCONV_H */
