// sirconv_maxbwd.hip — the agg_type='max' backward driven by the arg-max routing alone (SURVEY §8 f1;
// reference conv.py:46-47 with DGL fn.max): no [E, *] tensor and no edge-contracted dense GEMM.
//
//   Y[v][o] = max_e z_e[o],  z_e = W_R a_e + b_R,  a_e = act1(Q[v] + K[u]),  arg[v][o] = first arg-max edge
//
// dY[v][o] reaches only the arg edge of (v, o).  With L_e = {o : arg[v][o] = e} (e's routed outputs):
//   dA_e       = sum_{o in L_e} dY[v][o] W_R[o, :]        (|L_e| rows of W_R instead of all O)
//   dz_e       = act1'(Q[v] + K[u]) * dA_e,   dQ[v] = sum_e dz_e,   dK[u] = sum_e dz_e
//   dW_R[o, :] = sum_v dY[v][o] a_{arg[v][o]},   db_R[o] = sum_v dY[v][o]   (rows with an edge)
// Every product is V * O * H multiply-adds where the dense route's GEMMs are E * O * H (E / V = the mean
// degree: 20x fewer at S1), in true fp32 (fmaf), every sum in a fixed order (run-to-run deterministic).
//
//   k_maxb_route  one wave per destination work item: the item's (v, o) pairs grouped by arg edge, edges
//                 ascending, o ascending inside an edge -> entries {o, dY} (row v's block starts at v * O),
//                 per-edge {start, count} in dst-CSR and src-CSR order, per-block db_R partials.
//   k_maxb_dz     a 128-column slice of W_R resident in LDS; a 32-lane group per edge (4 columns a lane)
//                 reads the edge's entries and the W_R rows they name, dA -> dz -> summed per row: dQ on
//                 the destination CSR, dK on the source CSR (same kernel, the routing table in that
//                 CSR's order).  Split hub rows write partial rows, combined in slot order.
//   k_maxb_dw     a wave per (64 outputs x 32 columns) tile over a range of destination rows: 8 lanes per
//                 output o gather a_{arg[v][o]} (Q[v] + K[col[arg]], act1, 128 B a row) and accumulate
//                 dY[v][o] a; per-range partials summed in range order afterwards.
#include "sirconv_edge_impl.h"

#ifndef SIR_MAXB_QC
#define SIR_MAXB_QC 4           // items a work-queue claim of the dz passes
#endif

namespace sir {
namespace {

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// ------------------------------------------------------------------------------ routing table
// NK = ceil(O / 64) outputs per lane (o = 64 k + lane).  Items hold <= 256 edges in the standard plans;
// longer items are walked in 256-edge windows.
template <int NK>
__global__ void __launch_bounds__(256)
k_maxb_route(const int* __restrict__ rowptr, const int4* __restrict__ items, int64_t n_items,
             const int* __restrict__ arg, int64_t lda, const float* __restrict__ dY, int64_t ldy, int O,
             const int* __restrict__ pinv, int2* __restrict__ ent, int2* __restrict__ ecnt,
             int2* __restrict__ ecnt_s, float* __restrict__ dbpart) {
    __shared__ int s_st[4][256], s_cn[4][256];
    __shared__ unsigned s_occ[4][8];
    __shared__ float s_db[4][64 * NK];
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t below = (l == 0) ? 0ull : (~0ull >> (64 - l));     // lanes < l
    float db[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) db[k] = 0.f;
    for (int64_t wi = (int64_t)blockIdx.x * 4 + w; wi < n_items; wi += (int64_t)gridDim.x * 4) {
        const int4 it = uniform_item(items, wi);
        const int row = it.x, e0 = it.y, e1 = it.z;
        const int rs = rowptr[row], re = rowptr[row + 1];
        int a[NK];
        float y[NK];
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int o = 64 * k + l;
            a[k] = (o < O) ? arg[(int64_t)row * lda + o] : -1;
            y[k] = (o < O) ? dY[(int64_t)row * ldy + o] : 0.f;
            if (a[k] < rs || a[k] >= re) a[k] = -1;                  // no arg edge (empty row / NaN)
        }
        int cursor = 0;                                              // entries of this row before e0
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            cursor += __popcll(__ballot(a[k] >= 0 && a[k] < e0));
            if (a[k] >= e0 && a[k] < e1) db[k] += y[k];
        }
        int64_t cur = (int64_t)row * O + cursor;
        for (int w0 = e0; w0 < e1; w0 += 256) {
            const int n = (e1 - w0) < 256 ? (e1 - w0) : 256;
            for (int i = l; i < 256; i += 64) { s_st[w][i] = 0; s_cn[w][i] = 0; }
            if (l < 8) s_occ[w][l] = 0u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < NK; ++k)
                if (a[k] >= w0 && a[k] < w0 + n) atomicOr(&s_occ[w][(a[k] - w0) >> 5], 1u << ((a[k] - w0) & 31));
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (int wd = 0; wd < 8; ++wd) {
                unsigned bits = __builtin_amdgcn_readfirstlane(s_occ[w][wd]);
                while (bits) {
                    const int b = __builtin_ctz(bits);
                    bits &= bits - 1u;
                    const int e = w0 + 32 * wd + b;
                    int cnt = 0;
#pragma unroll
                    for (int k = 0; k < NK; ++k) {
                        const uint64_t m = __ballot(a[k] == e);
                        if (a[k] == e)
                            ent[cur + cnt + __popcll(m & below)] = make_int2(64 * k + l, __float_as_int(y[k]));
                        cnt += __popcll(m);
                    }
                    if (l == 0) { s_st[w][e - w0] = (int)cur; s_cn[w][e - w0] = cnt; }
                    cur += cnt;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (int i = l; i < n; i += 64) {
                const int2 r = make_int2(s_st[w][i], s_cn[w][i]);
                ecnt[w0 + i] = r;
                if (ecnt_s != nullptr) ecnt_s[pinv[w0 + i]] = r;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
    }
#pragma unroll
    for (int k = 0; k < NK; ++k) s_db[w][64 * k + l] = db[k];
    __syncthreads();
    const int OP4 = (O + 3) & ~3;                                    // row pitch (zero past O)
    for (int o = threadIdx.x; o < OP4; o += 256)
        dbpart[(int64_t)blockIdx.x * OP4 + o] = (o < O) ? ((s_db[0][o] + s_db[1][o]) + s_db[2][o]) + s_db[3][o] : 0.f;
}

// ------------------------------------------------------------------------------ dz passes (dQ / dK)
// 16 waves; W_R[:, c0 : c0 + 128] as [OPAD][32] float4 in LDS (c0 = 128 * (blockIdx.x % nsl)).  Each wave
// owns a work item of its CSR; its two 32-lane groups (4 columns a lane) take alternate edges, U each per
// batch.  The next batch's {start, count} and neighbour index (at an item's last batch: the next item's
// descriptor, own row and first batch) are in flight while the current batch's entries run; the entry
// loop is wave-uniform (both groups' counts, 4 entries a step: staged slots past a count hold {0, 0.f}).
// Items are handed out by a work queue (one counter per column slice, zeroed before the launch), QC at a
// time: an item's cost is its entry count, which on the source CSR ranges over 1-5,600 entries (S1), so a
// static item -> wave assignment left the pass waiting on its slowest waves (max / mean wave work 1.48 on
// S1, 1.22 on the destination CSR).  The next chunk is claimed one chunk ahead (its atomic's latency hidden
// under the current chunk); a wave stops at its first claim past the last item.
template <bool DST, int ACT1, int OPAD, int U>
__global__ void __launch_bounds__(1024)
k_maxb_dz(const int* __restrict__ col, const int4* __restrict__ items, int64_t n_items,
          const int2* __restrict__ ecnt, const int2* __restrict__ ent,
          const float* __restrict__ own, int64_t ldown, const float* __restrict__ oth, int64_t ldoth,
          const float* __restrict__ W, int H, int O, float slope, int nsl,
          float* __restrict__ out, int64_t ldo, float* __restrict__ partial, int* __restrict__ qctr) {
    constexpr int QC = SIR_MAXB_QC;
    __shared__ float4 sW[OPAD * 32];
    __shared__ int2 sE[16][2][32];
    const int t = threadIdx.x, l = t & 63, g = l >> 5, c = l & 31;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int s = blockIdx.x % nsl;
    const int c0 = 128 * s;
    for (int i = t; i < OPAD * 32; i += 1024) {
        const int o = i >> 5, cc = c0 + 4 * (i & 31);
        sW[i] = (o < O && cc < H) ? ld4(W + (int64_t)o * H + cc) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    const int cc = c0 + 4 * c;
    const bool colok = cc < H;
    const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
    int* const ctr = qctr + s;
    int pend = (l == 0) ? atomicAdd(ctr, QC) : 0;
    int64_t wi = __builtin_amdgcn_readfirstlane(pend);
    if (wi >= n_items) return;               // whole wave; no block barrier past this point
    pend = (l == 0) ? atomicAdd(ctr, QC) : 0;  // the next chunk, read when this one is done
    int qi = 0;                              // position of wi in its chunk
    int4 it = uniform_item(items, wi);
    float4 ov = colok ? ld4(own + (int64_t)it.x * ldown + cc) : zero4;
    int2 ec[U];
    int nb[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const int e = it.y + g + 2 * j;
        ec[j] = (e < it.z) ? ecnt[e] : make_int2(0, 0);
        nb[j] = (e < it.z) ? col[e] : 0;
    }
    while (true) {
        const int row = it.x, e1 = it.z, slot = it.w;
        int64_t wn;
        if (qi + 1 < QC) {
            wn = wi + 1;
        } else {                             // into the claimed chunk; claim the one after it
            wn = __builtin_amdgcn_readfirstlane(pend);
            if (wn < n_items) pend = (l == 0) ? atomicAdd(ctr, QC) : 0;
        }
        const bool more = wn < n_items;
        const int4 itn = more ? uniform_item(items, wn) : make_int4(0, 0, 0, 0);
        float4 ovn = zero4;
        float4 acc = zero4;
        for (int t0 = it.y; t0 < e1; t0 += 2 * U) {
            float4 xv[U];
            int2 en[U];
#pragma unroll
            for (int j = 0; j < U; ++j) {
                xv[j] = (ec[j].y > 0 && colok) ? ld4(oth + (int64_t)nb[j] * ldoth + cc) : zero4;
                en[j] = (c < ec[j].y) ? ent[ec[j].x + c] : make_int2(0, 0);
            }
            // the next batch: this item's, or the next item's first (with its own row)
            const bool last = t0 + 2 * U >= e1;
            const int nt0 = last ? itn.y : t0 + 2 * U;
            const int ne1 = last ? itn.z : e1;
            if (last && more && colok) ovn = ld4(own + (int64_t)itn.x * ldown + cc);
            int2 ec2[U];
            int nb2[U];
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int e = nt0 + g + 2 * j;
                const bool ok = e < ne1 && (!last || more);
                ec2[j] = ok ? ecnt[e] : make_int2(0, 0);
                nb2[j] = ok ? col[e] : 0;
            }
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int cnt = ec[j].y;
                const int oc = __shfl_xor(cnt, 32);          // unconditionally: a cross-lane read in one arm
                const int cntw = __builtin_amdgcn_readfirstlane(cnt > oc ? cnt : oc);   // of a ?: sees inactive lanes
                float4 da = zero4;
                for (int b0 = 0; b0 < cntw; b0 += 32) {                   // entries in batches of 32
                    const int2 mine = (b0 == 0) ? en[j] : ((b0 + c < cnt) ? ent[ec[j].x + b0 + c] : make_int2(0, 0));
                    __builtin_amdgcn_wave_barrier();
                    sE[w][g][c] = mine;
                    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    const int m = (cntw - b0) < 32 ? (cntw - b0) : 32;
                    for (int i = 0; i < m; i += 4) {
                        const int2 p0 = sE[w][g][i], p1 = sE[w][g][i + 1];
                        const int2 p2 = sE[w][g][i + 2], p3 = sE[w][g][i + 3];
                        const float4 w0 = sW[p0.x * 32 + c], w1 = sW[p1.x * 32 + c];
                        const float4 w2 = sW[p2.x * 32 + c], w3 = sW[p3.x * 32 + c];
                        const float y0 = __int_as_float(p0.y), y1 = __int_as_float(p1.y);
                        const float y2 = __int_as_float(p2.y), y3 = __int_as_float(p3.y);
                        da.x = fmaf(y0, w0.x, da.x); da.y = fmaf(y0, w0.y, da.y);
                        da.z = fmaf(y0, w0.z, da.z); da.w = fmaf(y0, w0.w, da.w);
                        da.x = fmaf(y1, w1.x, da.x); da.y = fmaf(y1, w1.y, da.y);
                        da.z = fmaf(y1, w1.z, da.z); da.w = fmaf(y1, w1.w, da.w);
                        da.x = fmaf(y2, w2.x, da.x); da.y = fmaf(y2, w2.y, da.y);
                        da.z = fmaf(y2, w2.z, da.z); da.w = fmaf(y2, w2.w, da.w);
                        da.x = fmaf(y3, w3.x, da.x); da.y = fmaf(y3, w3.y, da.y);
                        da.z = fmaf(y3, w3.z, da.z); da.w = fmaf(y3, w3.w, da.w);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
                if (cnt > 0) {
                    // z = Q[v] + K[u] in the reference's operand order on either pass
                    const float4 q4 = DST ? ov : xv[j];
                    const float4 k4 = DST ? xv[j] : ov;
                    acc.x += dsig<ACT1>(q4.x + k4.x, da.x, slope);
                    acc.y += dsig<ACT1>(q4.y + k4.y, da.y, slope);
                    acc.z += dsig<ACT1>(q4.z + k4.z, da.z, slope);
                    acc.w += dsig<ACT1>(q4.w + k4.w, da.w, slope);
                }
            }
#pragma unroll
            for (int j = 0; j < U; ++j) { ec[j] = ec2[j]; nb[j] = nb2[j]; }
        }
        if (it.y == e1) {                    // an empty row: this item's batch loop never ran
            if (more && colok) ovn = ld4(own + (int64_t)itn.x * ldown + cc);
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int e = itn.y + g + 2 * j;
                const bool ok = more && e < itn.z;
                ec[j] = ok ? ecnt[e] : make_int2(0, 0);
                nb[j] = ok ? col[e] : 0;
            }
        }
        // the two groups hold alternate edges of the same columns
        float4 r;
        r.x = acc.x + __shfl_xor(acc.x, 32);
        r.y = acc.y + __shfl_xor(acc.y, 32);
        r.z = acc.z + __shfl_xor(acc.z, 32);
        r.w = acc.w + __shfl_xor(acc.w, 32);
        if (g == 0 && colok) {
            float* dst = (slot < 0) ? out + (int64_t)row * ldo + cc : partial + (int64_t)slot * H + cc;
            *reinterpret_cast<float4*>(dst) = r;
        }
        if (!more) break;
        wi = wn;
        qi = (qi + 1 < QC) ? qi + 1 : 0;
        it = itn;
        ov = ovn;
    }
}

// split rows: out[row] = sum of the row's partial rows in slot order
__global__ void k_maxb_combine(const int4* __restrict__ splits, int H, const float* __restrict__ partial,
                               float* __restrict__ out, int64_t ldo) {
    const int4 sp = splits[blockIdx.x];
    for (int f = threadIdx.x; f < H; f += blockDim.x) {
        const float* p = partial + (int64_t)sp.y * H + f;
        float s = 0.f;
        int k = 0;
        for (; k + 8 <= sp.z; k += 8) {          // 8 loads in flight, added in slot order
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = p[(int64_t)(k + i) * H];
#pragma unroll
            for (int i = 0; i < 8; ++i) s += v[i];
        }
        for (; k < sp.z; ++k) s += p[(int64_t)k * H];
        out[(int64_t)sp.x * ldo + f] = s;
    }
}

// ------------------------------------------------------------------------------ dW_R
#ifndef SIR_MAXB_DW_ROWS
#define SIR_MAXB_DW_ROWS 1      // rows in flight per step (2: 142 VGPRs, 3 waves / SIMD)
#endif
// Block = 4 waves = 4 consecutive 32-column tiles of one 64-output tile; grid.y = destination-row ranges.
// Lane (i8 = lane / 8, q = lane % 8) holds outputs o = 64 ot + 8 i + i8 (i < 8) x columns c0 + 4 q .. + 3:
// per row the 64 outputs' arg rows K[col[arg]] are read 8 lanes to a row (128 contiguous bytes each),
// a = act1(Q[v] + K[u]) and dY[v][o] a accumulated.  Two rows in flight per step.
template <int ACT1>
__global__ void __launch_bounds__(256)
k_maxb_dw(const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ arg, int64_t lda,
          const float* __restrict__ dY, int64_t ldy, const float* __restrict__ Q, int64_t ldq,
          const float* __restrict__ K, int64_t ldk, int V, int O, int H, float slope, int nct, int rows_per,
          float* __restrict__ wpart) {
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nctb = (nct + 3) / 4;
    const int ot = blockIdx.x / nctb;
    const int ct = (blockIdx.x % nctb) * 4 + w;
    if (ct >= nct) return;                                   // whole wave; no block barrier below
    const int ol = 64 * ot + l;                              // the output this lane loads arg / dY for
    const bool olok = ol < O;
    const int i8 = l >> 3, q = l & 7;
    const int cq = 32 * ct + 4 * q;                          // this lane's 4 columns
    const bool cok = cq < H;
    const int r0 = blockIdx.y * rows_per;
    const int r1 = (r0 + rows_per) < V ? (r0 + rows_per) : V;
    float4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = r0; r < r1; r += SIR_MAXB_DW_ROWS) {
        const bool two = SIR_MAXB_DW_ROWS == 2 && r + 1 < r1;
        int u[SIR_MAXB_DW_ROWS];
        float y[SIR_MAXB_DW_ROWS];
#pragma unroll
        for (int h = 0; h < SIR_MAXB_DW_ROWS; ++h) {
            const int rr = two ? r + h : r;
            const int a = olok ? arg[(int64_t)rr * lda + ol] : -1;
            const bool v = a >= rowptr[rr] && a < rowptr[rr + 1] && (h == 0 || two);
            y[h] = (v && olok) ? dY[(int64_t)rr * ldy + ol] : 0.f;
            u[h] = v ? col[a] : -1;
        }
        float4 kv[SIR_MAXB_DW_ROWS][8];
#pragma unroll
        for (int h = 0; h < SIR_MAXB_DW_ROWS; ++h)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int ui = __shfl(u[h], 8 * i + i8);
                kv[h][i] = (ui >= 0 && cok) ? ld4(K + (int64_t)ui * ldk + cq) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
        for (int h = 0; h < SIR_MAXB_DW_ROWS; ++h) {
            const int rr = two ? r + h : r;
            const float4 q4 = cok ? ld4(Q + (int64_t)rr * ldq + cq) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float yi = __shfl(y[h], 8 * i + i8);
                acc[i].x = fmaf(yi, sig<ACT1>(q4.x + kv[h][i].x, slope), acc[i].x);
                acc[i].y = fmaf(yi, sig<ACT1>(q4.y + kv[h][i].y, slope), acc[i].y);
                acc[i].z = fmaf(yi, sig<ACT1>(q4.z + kv[h][i].z, slope), acc[i].z);
                acc[i].w = fmaf(yi, sig<ACT1>(q4.w + kv[h][i].w, slope), acc[i].w);
            }
        }
    }
    if (cok) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int o = 64 * ot + 8 * i + i8;
            if (o < O) *reinterpret_cast<float4*>(wpart + ((int64_t)blockIdx.y * O + o) * H + cq) = acc[i];
        }
    }
}

// ------------------------------------------------------------------------------ dW_R from materialised A
// The edge-materialised max backward's dW_R / db_R without dM [E, O] or the dense TN GEMM: A [E, H] holds
// a_e = act1(z_e) in dst-CSR order, so dW_R[o, :] = sum_v dY[v][o] A[arg[v][o], :] reads each row's A rows
// contiguously.  Block = 512 lanes, lane = (output o <= 256, 32-column half of the 64 columns c0 = 64 blockIdx.x); grid.y =
// destination-row ranges.  Consecutive rows are batched up to 4 rows / 64 edges: the batch's A columns (and
// its rows' arg / dY) are loaded one batch ahead into registers and staged in LDS; each lane adds dY[v][o] A[arg][cols] from
// LDS; a row longer than 64 edges is a batch of its own whose lanes read their arg rows from global memory.
// Partials [range][O * H (+ O: db_R on the first column block)], summed in range order afterwards.
constexpr int MDW_ROWS = 4, MDW_EDGES = 64, MDW_PITCH = 68, MDW_WIN = 1024;

__global__ void __launch_bounds__(512)
k_max_dw_rows(const int* __restrict__ rowptr, const int* __restrict__ arg, int64_t lda,
              const float* __restrict__ dY, int64_t ldy, const float* __restrict__ A, int64_t ldA,
              int V, int O, int H, int rows_per, float* __restrict__ wpart, int64_t ldw) {
    __shared__ float sA[MDW_EDGES * MDW_PITCH];
    __shared__ int sRp[MDW_WIN + 1];                          // rowptr[wb .. wb + MDW_WIN]
    const int t = threadIdx.x;
    const int o = t & 255, hc = t >> 8;                      // output, half of the 64-column block
    const bool ook = o < O;
    const int c0 = 64 * blockIdx.x;
    const int cl = 32 * hc;                                  // this lane's 32 columns: c0 + cl ..
    const int r0 = blockIdx.y * rows_per;
    const int r1 = (r0 + rows_per) < V ? (r0 + rows_per) : V;
    float4 acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    float db = 0.f;
    int wb = r0;
    auto fill = [&]() {                                      // the rowptr window (all threads, then a barrier)
        for (int i = t; i <= MDW_WIN && wb + i <= V; i += 512) sRp[i] = rowptr[wb + i];
        __syncthreads();
    };
    auto rp = [&](int r) { return sRp[r - wb]; };
    // batch = rows [br, be) with edges [rowptr[br], rowptr[be]); hub = one row over MDW_EDGES edges
    auto form = [&](int br, int& be, bool& hub) {
        const int base = rp(br);
        be = br + 1;
        hub = rp(br + 1) - base > MDW_EDGES;
        if (!hub)
            while (be < r1 && be - br < MDW_ROWS && rp(be + 1) - base <= MDW_EDGES) ++be;
    };
    float4 pre[MDW_EDGES / 32];
    int pa[MDW_ROWS];
    float py[MDW_ROWS];
    auto load = [&](int br, int be, bool hub) {
        const int base = rp(br);
        const int ne = rp(be) - base;
#pragma unroll
        for (int k = 0; k < MDW_EDGES / 32; ++k) {
            const int i = t + 512 * k;             // float4 index: edge i / 16, quad i % 16
            const int e = i >> 4, q = i & 15;
            pre[k] = (!hub && e < ne && c0 + 4 * q < H) ? ld4(A + (int64_t)(base + e) * ldA + c0 + 4 * q)
                                                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    int na[MDW_ROWS];
    float ny[MDW_ROWS];
    auto load_args = [&](int br, int be) {                   // into na / ny: one batch ahead
#pragma unroll
        for (int j = 0; j < MDW_ROWS; ++j) {
            const int r = br + j;
            na[j] = (ook && r < be) ? arg[(int64_t)r * lda + o] : -1;
            ny[j] = (ook && r < be) ? dY[(int64_t)r * ldy + o] : 0.f;
        }
    };
    int br = r0, be = r0;
    bool hub = false;
    if (br < r1) { fill(); form(br, be, hub); load(br, be, hub); load_args(br, be); }
    while (br < r1) {
#pragma unroll
        for (int j = 0; j < MDW_ROWS; ++j) { pa[j] = na[j]; py[j] = ny[j]; }
        // stage the current batch (and cache its row bounds), then put the next batch in flight
#pragma unroll
        for (int k = 0; k < MDW_EDGES / 32; ++k) {
            const int i = t + 512 * k;
            *reinterpret_cast<float4*>(&sA[(i >> 4) * MDW_PITCH + 4 * (i & 15)]) = pre[k];
        }
        const int cbr = br, cbe = be;
        const bool chub = hub;
        int crp[MDW_ROWS + 1];
#pragma unroll
        for (int j = 0; j <= MDW_ROWS; ++j) crp[j] = (cbr + j <= cbe) ? rp(cbr + j) : 0;
        __syncthreads();
        br = be;
        if (br < r1) {
            if (br + MDW_ROWS + 1 > wb + MDW_WIN) { wb = br; fill(); }
            form(br, be, hub);
            load(br, be, hub);
            load_args(br, be);
        }
        const int base = crp[0];
#pragma unroll
        for (int j = 0; j < MDW_ROWS; ++j) {
            if (cbr + j >= cbe) break;
            const int a = pa[j];
            if (a < crp[j] || a >= crp[j + 1]) continue;            // no arg edge (empty row)
            const float y = py[j];
            if (hc == 0) db += y;
            if (chub) {                                                 // hub row: arg rows from global memory
                const float* ap = A + (int64_t)a * ldA + c0 + cl;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const float4 v = (c0 + cl + 4 * q < H) ? ld4(ap + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
                    acc[q].x = fmaf(y, v.x, acc[q].x); acc[q].y = fmaf(y, v.y, acc[q].y);
                    acc[q].z = fmaf(y, v.z, acc[q].z); acc[q].w = fmaf(y, v.w, acc[q].w);
                }
            } else {
                const float* ap = &sA[(a - base) * MDW_PITCH + cl];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const float4 v = *reinterpret_cast<const float4*>(ap + 4 * q);
                    acc[q].x = fmaf(y, v.x, acc[q].x); acc[q].y = fmaf(y, v.y, acc[q].y);
                    acc[q].z = fmaf(y, v.z, acc[q].z); acc[q].w = fmaf(y, v.w, acc[q].w);
                }
            }
        }
        __syncthreads();
    }
    if (ook) {
        float* wp = wpart + (int64_t)blockIdx.y * ldw;
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (c0 + cl + 4 * q < H) *reinterpret_cast<float4*>(wp + (int64_t)o * H + c0 + cl + 4 * q) = acc[q];
        if (blockIdx.x == 0 && hc == 0) wp[(int64_t)O * H + o] = db;
    }
    if (blockIdx.x == 0 && hc == 0 && t >= O && t < ((O + 3) & ~3))
        wpart[(int64_t)blockIdx.y * ldw + (int64_t)O * H + t] = 0.f;
}

// dW_R / db_R with the activations recomputed in the batch staging instead of read from A [E, H]: each
// non-hub batch gathers K[col[e]] of its edges and Q of its rows, stages a = act1(Q[v] + K[u]) in LDS and
// accumulates as k_max_dw_rows does (hub rows: each lane gathers its arg edge's K row).  The batch's
// column ids are loaded two batches ahead, its K / Q columns one batch ahead (raw, activated at staging).
// With the routed dQ / dK passes this leaves the max backward without any [E, *] buffer.
template <int ACT1>
__global__ void __launch_bounds__(512)
k_max_dw_qk(const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ arg, int64_t lda,
            const float* __restrict__ dY, int64_t ldy, const float* __restrict__ Q, int64_t ldq,
            const float* __restrict__ K, int64_t ldk, int V, int O, int H, float slope, int rows_per,
            float* __restrict__ wpart, int64_t ldw) {
    __shared__ float sA[MDW_EDGES * MDW_PITCH];
    __shared__ int sRp[MDW_WIN + 1];                          // rowptr[wb .. wb + MDW_WIN]
    const int t = threadIdx.x;
    const int o = t & 255, hc = t >> 8;                      // output, half of the 64-column block
    const bool ook = o < O;
    const int c0 = 64 * blockIdx.x;
    const int cl = 32 * hc;                                  // this lane's 32 accumulated columns
    const int qq = t & 15;                                   // staging: this thread's quad of the 64 columns
    const bool qok = c0 + 4 * qq < H;
    const int r0 = blockIdx.y * rows_per;
    const int r1 = (r0 + rows_per) < V ? (r0 + rows_per) : V;
    const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = zero4;
    float db = 0.f;
    int wb = r0;
    auto fill = [&]() {
        for (int i = t; i <= MDW_WIN && wb + i <= V; i += 512) sRp[i] = rowptr[wb + i];
        __syncthreads();
    };
    auto rp = [&](int r) { return sRp[r - wb]; };
    auto form = [&](int br, int& be, bool& hub) {
        const int base = rp(br);
        be = br + 1;
        hub = rp(br + 1) - base > MDW_EDGES;
        if (!hub)
            while (be < r1 && be - br < MDW_ROWS && rp(be + 1) - base <= MDW_EDGES) ++be;
    };
    // staging edges of this thread: e_k = t / 16 + 32 k (k < 2), quad qq
    auto load_cols = [&](int br, int be, bool hub, int* cn) {
        const int base = rp(br), ne = rp(be) - base;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int e = (t >> 4) + 32 * k;
            cn[k] = (!hub && e < ne) ? col[base + e] : -1;
        }
    };
    auto load_qk = [&](int br, int be, const int* cn, float4* kq, float4* qq4) {
        const int base = rp(br);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int ge = base + (t >> 4) + 32 * k;        // global edge position
            int r = br;
#pragma unroll
            for (int j = 1; j < MDW_ROWS; ++j)
                if (br + j < be && ge >= rp(br + j)) r = br + j;
            const bool ok = cn[k] >= 0 && qok;
            kq[k] = ok ? ld4(K + (int64_t)cn[k] * ldk + c0 + 4 * qq) : zero4;
            qq4[k] = ok ? ld4(Q + (int64_t)r * ldq + c0 + 4 * qq) : zero4;
        }
    };
    int pa[MDW_ROWS], na[MDW_ROWS];
    float py[MDW_ROWS], ny[MDW_ROWS];
    auto load_args = [&](int br, int be) {
#pragma unroll
        for (int j = 0; j < MDW_ROWS; ++j) {
            const int r = br + j;
            na[j] = (ook && r < be) ? arg[(int64_t)r * lda + o] : -1;
            ny[j] = (ook && r < be) ? dY[(int64_t)r * ldy + o] : 0.f;
        }
    };
    if (r0 >= r1) goto done;
    {
        fill();
        // batch c (current, K / Q in kq / qv), n1 (next: columns in cn1)
        int br = r0, be, bn, ben;
        bool hub, hubn;
        int cn0[2], cn1[2];
        float4 kq[2], qv[2];
        form(br, be, hub);
        load_cols(br, be, hub, cn0);
        load_qk(br, be, cn0, kq, qv);
        load_args(br, be);
        bn = be;
        if (bn < r1) {
            if (bn + MDW_ROWS + 1 > wb + MDW_WIN) { __syncthreads(); wb = bn; fill(); }
            form(bn, ben, hubn);
            load_cols(bn, ben, hubn, cn1);
        }
        while (br < r1) {
            // stage batch c: a = act1(Q[v] + K[u])
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int e = (t >> 4) + 32 * k;
                float4 a;
                a.x = sig<ACT1>(qv[k].x + kq[k].x, slope); a.y = sig<ACT1>(qv[k].y + kq[k].y, slope);
                a.z = sig<ACT1>(qv[k].z + kq[k].z, slope); a.w = sig<ACT1>(qv[k].w + kq[k].w, slope);
                *reinterpret_cast<float4*>(&sA[e * MDW_PITCH + 4 * qq]) = a;
            }
#pragma unroll
            for (int j = 0; j < MDW_ROWS; ++j) { pa[j] = na[j]; py[j] = ny[j]; }
            const int cbr = br, cbe = be;
            const bool chub = hub;
            int crp[MDW_ROWS + 1];
#pragma unroll
            for (int j = 0; j <= MDW_ROWS; ++j) crp[j] = (cbr + j <= cbe) ? rp(cbr + j) : 0;
            __syncthreads();
            // next batch: its K / Q columns in flight; the one after: its column ids
            br = bn; be = ben; hub = hubn;
            if (br < r1) {
                load_qk(br, be, cn1, kq, qv);
                load_args(br, be);
                bn = be;
                if (bn < r1) {
                    if (bn + MDW_ROWS + 1 > wb + MDW_WIN) {
                        // the window moves to batch br (its bounds stay readable); every thread is past
                        // its reads of the old window first
                        __syncthreads();
                        wb = br; fill();
                    }
                    form(bn, ben, hubn);
                    load_cols(bn, ben, hubn, cn1);
                }
            }
            const int base = crp[0];
#pragma unroll
            for (int j = 0; j < MDW_ROWS; ++j) {
                if (cbr + j >= cbe) break;
                const int a = pa[j];
                if (a < crp[j] || a >= crp[j + 1]) continue;            // no arg edge (empty row)
                const float y = py[j];
                if (hc == 0) db += y;
                if (chub) {                                             // hub row: the arg edge's K row
                    const int u = col[a];
                    const float* kp = K + (int64_t)u * ldk + c0 + cl;
                    const float* qp = Q + (int64_t)(cbr + j) * ldq + c0 + cl;
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        if (c0 + cl + 4 * q < H) {
                            const float4 kv = ld4(kp + 4 * q), qv4 = ld4(qp + 4 * q);
                            acc[q].x = fmaf(y, sig<ACT1>(qv4.x + kv.x, slope), acc[q].x);
                            acc[q].y = fmaf(y, sig<ACT1>(qv4.y + kv.y, slope), acc[q].y);
                            acc[q].z = fmaf(y, sig<ACT1>(qv4.z + kv.z, slope), acc[q].z);
                            acc[q].w = fmaf(y, sig<ACT1>(qv4.w + kv.w, slope), acc[q].w);
                        }
                    }
                } else {
                    const float* ap = &sA[(a - base) * MDW_PITCH + cl];
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const float4 v = *reinterpret_cast<const float4*>(ap + 4 * q);
                        acc[q].x = fmaf(y, v.x, acc[q].x); acc[q].y = fmaf(y, v.y, acc[q].y);
                        acc[q].z = fmaf(y, v.z, acc[q].z); acc[q].w = fmaf(y, v.w, acc[q].w);
                    }
                }
            }
            __syncthreads();
        }
    }
done:
    if (ook) {
        float* wp = wpart + (int64_t)blockIdx.y * ldw;
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (c0 + cl + 4 * q < H) *reinterpret_cast<float4*>(wp + (int64_t)o * H + c0 + cl + 4 * q) = acc[q];
        if (blockIdx.x == 0 && hc == 0) wp[(int64_t)O * H + o] = db;
    }
    if (blockIdx.x == 0 && hc == 0 && t >= O && t < ((O + 3) & ~3))
        wpart[(int64_t)blockIdx.y * ldw + (int64_t)O * H + t] = 0.f;
}

// k_max_dw_qk with larger batches (round 6): up to MDW2_ROWS rows / MDW2_EDGES edges per batch (4 / 64
// above), the batch's arg / dY staged in LDS with its activations (registers: one batch of K / Q columns and
// arg / dY in flight), its row bounds in LDS (the rowptr window may move while it is summed).  k_max_dw_qk
// spent ~5.7 us a batch at S1 against ~0.5 us of arithmetic: each 4-row batch waited for its gathers behind
// two barriers.  Same per-lane order of terms (rows ascending, the arg edge's activation recomputed with the
// same operations): bit-identical to k_max_dw_qk.
constexpr int MDW2_ROWS = 16, MDW2_EDGES = 128, MDW2_WIN = 1024;
#ifndef SIR_MAXDW2_OCC
#define SIR_MAXDW2_OCC 2        // blocks per CU the register budget is held to (2: <= 128 VGPRs; LDS fits two)
#endif

// waves per SIMD the register budget is held to: two blocks a CU (<= 128 VGPRs) but for the GELU forms,
// whose erf code would spill there (one block, <= 256)
constexpr int mdw2_wpe(int act) { return (act == ACT_GELU || act == ACT_GELU_TANH) ? 2 : 2 * SIR_MAXDW2_OCC; }
template <int ACT1>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(mdw2_wpe(ACT1))))
k_max_dw_qk2(const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ arg, int64_t lda,
             const float* __restrict__ dY, int64_t ldy, const float* __restrict__ Q, int64_t ldq,
             const float* __restrict__ K, int64_t ldk, int V, int O, int H, float slope, int rows_per,
             float* __restrict__ wpart, int64_t ldw) {
    constexpr int NR = MDW2_ROWS, NE = MDW2_EDGES, WIN = MDW2_WIN, PITCH = MDW_PITCH;
    constexpr int EPT = NE * 16 / 512;                       // staged (edge, quad) float4s per thread
    constexpr int APT = NR * 256 / 512;                      // staged (row, output) pairs per thread
    static_assert(EPT * 512 == NE * 16 && APT * 512 == NR * 256, "staging map");
    __shared__ float sA[NE * PITCH];
    __shared__ int sArg[NR * 256];
    __shared__ float sY[NR * 256];
    __shared__ int sRp[WIN + 1];                             // rowptr[wb .. wb + WIN]
    __shared__ int sB[NR + 1];                               // the staged batch's row bounds
    __shared__ float sZ[64];                                 // a zero row: lanes without a term read it
    __shared__ float4 sQ[2][NR * 16];                        // Q quads of the staged batch's rows (by parity)
    const int t = threadIdx.x;
    const int o = t & 255, hc = t >> 8;                      // output, half of the 64-column block
    const bool ook = o < O;
    const int c0 = 64 * blockIdx.x;
    const int cl = 32 * hc;                                  // this lane's 32 accumulated columns
    const int qq = t & 15;                                   // staging: this thread's quad of the 64 columns
    const bool qok = c0 + 4 * qq < H;
    const int r0 = blockIdx.y * rows_per;
    const int r1 = (r0 + rows_per) < V ? (r0 + rows_per) : V;
    const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = zero4;
    float db = 0.f;
    int wb = r0;
    auto fill = [&]() {
        for (int i = t; i <= WIN && wb + i <= V; i += 512) sRp[i] = rowptr[wb + i];
        __syncthreads();
    };
    auto rp = [&](int r) { return sRp[r - wb]; };
    auto form = [&](int br, int& be, bool& hub) {
        const int base = rp(br);
        be = br + 1;
        hub = rp(br + 1) - base > NE;
        if (!hub)
            while (be < r1 && be - br < NR && rp(be + 1) - base <= NE) ++be;
    };
    // this thread's staging edges e_k = t / 16 + 32 k: column ids and rows (a merge walk over the bounds);
    // threads t < 16 NR also fetch quad t % 16 of the batch's row t / 16 of Q (staged in LDS one batch later)
    auto load_cols = [&](int br, int be, bool hub, int* cn, int* rn, float4& qn) {
        const int base = rp(br), ne = rp(be) - base;
        const int qr = br + (t >> 4);
        qn = (t < 16 * NR && !hub && qr < be && qok) ? ld4(Q + (int64_t)qr * ldq + c0 + 4 * qq) : zero4;
        int j = br;
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int e = (t >> 4) + 32 * k;
            const bool ok = !hub && e < ne;
            while (ok && j + 1 < be && base + e >= rp(j + 1)) ++j;
            cn[k] = ok ? col[base + e] : -1;
            rn[k] = j;
        }
    };
    auto load_k = [&](const int* cn, float4* kq) {
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const bool ok = cn[k] >= 0 && qok;
            kq[k] = ok ? ld4(K + (int64_t)cn[k] * ldk + c0 + 4 * qq) : zero4;
        }
    };
    // staged pairs of this thread: (row br + hc + 2 k, output o)
    auto load_args = [&](int br, int be, int* na, float* ny) {
#pragma unroll
        for (int k = 0; k < APT; ++k) {
            const int r = br + hc + 2 * k;
            na[k] = (ook && r < be) ? arg[(int64_t)r * lda + o] : -1;
            ny[k] = (ook && r < be) ? dY[(int64_t)r * ldy + o] : 0.f;
        }
    };
    if (r0 >= r1) goto done;
    if (t < 64) sZ[t] = 0.f;                                 // visible after fill()'s barrier
    {
        fill();
        int br = r0, be, bn, ben;
        bool hub, hubn;
        int cn[EPT], rn[EPT], rc[EPT], na[APT];
        float ny[APT];
        float4 kq[EPT], qn;
        int par = 0;                                         // parity of the batch being staged
        form(br, be, hub);
        load_cols(br, be, hub, cn, rn, qn);
        if (t < 16 * NR) sQ[0][t] = qn;
        __syncthreads();
        load_k(cn, kq);
#pragma unroll
        for (int k = 0; k < EPT; ++k) rc[k] = rn[k] - br;
        load_args(br, be, na, ny);
        bn = be;
        qn = zero4;
        if (bn < r1) {
            if (bn + NR + 1 > wb + WIN) { __syncthreads(); wb = bn; fill(); }
            form(bn, ben, hubn);
            load_cols(bn, ben, hubn, cn, rn, qn);
        }
        while (br < r1) {
            // stage batch (br, be): a = act1(Q[v] + K[u]), arg / dY, row bounds
#pragma unroll
            for (int k = 0; k < EPT; ++k) {
                const int e = (t >> 4) + 32 * k;
                const float4 qv = sQ[par][rc[k] * 16 + qq];
                float4 a;
                a.x = sig<ACT1>(qv.x + kq[k].x, slope); a.y = sig<ACT1>(qv.y + kq[k].y, slope);
                a.z = sig<ACT1>(qv.z + kq[k].z, slope); a.w = sig<ACT1>(qv.w + kq[k].w, slope);
                *reinterpret_cast<float4*>(&sA[e * PITCH + 4 * qq]) = a;
            }
            if (t < 16 * NR) sQ[par ^ 1][t] = qn;                // the next batch's Q rows
            par ^= 1;
#pragma unroll
            for (int k = 0; k < APT; ++k) {
                sArg[(hc + 2 * k) * 256 + o] = na[k];
                sY[(hc + 2 * k) * 256 + o] = ny[k];
            }
            if (t <= NR) sB[t] = (br + t <= be) ? rp(br + t) : 0;
            const int cbr = br, cbe = be;
            const bool chub = hub;
            __syncthreads();
            // next batch: its K / Q columns and arg / dY in flight; the one after: its column ids
            br = bn; be = ben; hub = hubn;
            if (br < r1) {
                load_k(cn, kq);
#pragma unroll
                for (int k = 0; k < EPT; ++k) rc[k] = rn[k] - br;
                load_args(br, be, na, ny);
                bn = be;
                if (bn < r1) {
                    if (bn + NR + 1 > wb + WIN) { __syncthreads(); wb = br; fill(); }
                    form(bn, ben, hubn);
                    load_cols(bn, ben, hubn, cn, rn, qn);
                }
            }
            const int base = sB[0];
            if (!chub) {
                // branch-free over the lanes: a lane without a term (empty row, o >= O) multiplies the
                // zero row by 0 (adds +0: the same values as skipping it, -0 sums aside)
                for (int j = 0; j < cbe - cbr; ++j) {
                    const int a = sArg[j * 256 + o];
                    const bool ok = ook && a >= sB[j] && a < sB[j + 1];
                    const float y = ok ? sY[j * 256 + o] : 0.f;
                    if (hc == 0) db += y;
                    const float* ap = ok ? &sA[(a - base) * PITCH + cl] : &sZ[cl];
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const float4 v = *reinterpret_cast<const float4*>(ap + 4 * q);
                        acc[q].x = fmaf(y, v.x, acc[q].x); acc[q].y = fmaf(y, v.y, acc[q].y);
                        acc[q].z = fmaf(y, v.z, acc[q].z); acc[q].w = fmaf(y, v.w, acc[q].w);
                    }
                }
            }
            for (int j = 0; chub && j < cbe - cbr; ++j) {
                const int a = sArg[j * 256 + o];
                if (!ook || a < sB[j] || a >= sB[j + 1]) continue;    // no arg edge (empty row)
                const float y = sY[j * 256 + o];
                if (hc == 0) db += y;
                {                                                     // hub row: the arg edge's K row
                    const int u = col[a];
                    const float* kp = K + (int64_t)u * ldk + c0 + cl;
                    const float* qp = Q + (int64_t)(cbr + j) * ldq + c0 + cl;
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        if (c0 + cl + 4 * q < H) {
                            const float4 kv = ld4(kp + 4 * q), qv4 = ld4(qp + 4 * q);
                            acc[q].x = fmaf(y, sig<ACT1>(qv4.x + kv.x, slope), acc[q].x);
                            acc[q].y = fmaf(y, sig<ACT1>(qv4.y + kv.y, slope), acc[q].y);
                            acc[q].z = fmaf(y, sig<ACT1>(qv4.z + kv.z, slope), acc[q].z);
                            acc[q].w = fmaf(y, sig<ACT1>(qv4.w + kv.w, slope), acc[q].w);
                        }
                    }
                }
            }
            __syncthreads();
        }
    }
done:
    if (ook) {
        float* wp = wpart + (int64_t)blockIdx.y * ldw;
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (c0 + cl + 4 * q < H) *reinterpret_cast<float4*>(wp + (int64_t)o * H + c0 + cl + 4 * q) = acc[q];
        if (blockIdx.x == 0 && hc == 0) wp[(int64_t)O * H + o] = db;
    }
    if (blockIdx.x == 0 && hc == 0 && t >= O && t < ((O + 3) & ~3))
        wpart[(int64_t)blockIdx.y * ldw + (int64_t)O * H + t] = 0.f;
}

#ifndef SIR_MAXB_U
#define SIR_MAXB_U 4
#endif
#ifndef SIR_MAXDW
#define SIR_MAXDW 2             // sir_max_dw_qk: 1 = k_max_dw_qk (4-row / 64-edge batches), 2 = k_max_dw_qk2
#endif

template <typename Fn>
hipError_t maxb_acts(int act1, Fn&& fn) {
    switch (act1) {
        case ACT_IDENTITY: return fn(std::integral_constant<int, ACT_IDENTITY>());
        case ACT_RELU: return fn(std::integral_constant<int, ACT_RELU>());
        case ACT_LEAKY: return fn(std::integral_constant<int, ACT_LEAKY>());
        case ACT_GELU: return fn(std::integral_constant<int, ACT_GELU>());
        case ACT_GELU_TANH: return fn(std::integral_constant<int, ACT_GELU_TANH>());
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

int64_t maxb_dw_ranges(int64_t V) {
    // ~2048 waves of dW tiles at O = H = 256 (32 tiles): 64 ranges; at least 16 rows a range
    int64_t r = 64;
    while (r > 1 && V / r < 16) r >>= 1;
    return r;
}

int64_t max_dw_rows_ranges(int64_t V, int H) {
    // two 512-thread blocks a CU (110 VGPRs): 512 / (H / 64) column blocks' worth of row ranges, at least
    // 64 rows a range
    const int64_t nc = (H + 63) / 64;
    int64_t r = 512 / (nc > 0 ? nc : 1);
    if (r < 1) r = 1;
    while (r > 1 && V / r < 64) r >>= 1;
    return r;
}

hipError_t run_max_dw_rows(const int* rowptr, int64_t V, const int* arg, int64_t lda, const float* dY, int64_t ldy,
                           const float* A, int64_t ldA, int O, int H, float* wpart, int64_t ldw, hipStream_t st) {
    // no rows: the one partial (max_dw_rows_ranges(0, H) == 1) is written as zeros, never left unset
    if (V == 0) return wpart != nullptr ? hipMemsetAsync(wpart, 0, (size_t)ldw * sizeof(float), st) : hipSuccess;
    const int64_t R = max_dw_rows_ranges(V, H);
    const int rows_per = (int)((V + R - 1) / R);
    hipLaunchKernelGGL(k_max_dw_rows, dim3((unsigned)((H + 63) / 64), (unsigned)R), dim3(512), 0, st, rowptr, arg,
                       lda, dY, ldy, A, ldA, (int)V, O, H, rows_per, wpart, ldw);
    return hipGetLastError();
}

hipError_t run_max_dw_qk(const int* rowptr, const int* col, int64_t V, const int* arg, int64_t lda, const float* dY,
                         int64_t ldy, const float* Q, int64_t ldq, const float* K, int64_t ldk, int O, int H, int act1,
                         float slope, float* wpart, int64_t ldw, hipStream_t st) {
    if (V == 0) return wpart != nullptr ? hipMemsetAsync(wpart, 0, (size_t)ldw * sizeof(float), st) : hipSuccess;
    const int64_t R = max_dw_rows_ranges(V, H);
    const int rows_per = (int)((V + R - 1) / R);
    const char* e = getenv("SIR_MAXDW");
    const int form = (e != nullptr && e[0] != 0) ? atoi(e) : SIR_MAXDW;
    return maxb_acts(act1, [&](auto A1) -> hipError_t {
        constexpr int X1 = decltype(A1)::value;
        if (form == 1)
            hipLaunchKernelGGL((k_max_dw_qk<X1>), dim3((unsigned)((H + 63) / 64), (unsigned)R), dim3(512), 0, st,
                               rowptr, col, arg, lda, dY, ldy, Q, ldq, K, ldk, (int)V, O, H, slope, rows_per, wpart,
                               ldw);
        else
            hipLaunchKernelGGL((k_max_dw_qk2<X1>), dim3((unsigned)((H + 63) / 64), (unsigned)R), dim3(512), 0, st,
                               rowptr, col, arg, lda, dY, ldy, Q, ldq, K, ldk, (int)V, O, H, slope, rows_per, wpart,
                               ldw);
        return hipGetLastError();
    });
}

hipError_t run_max_bwd_sparse(const MaxBwdArgs& a, hipStream_t st) {
    const int O = a.O, H = a.H;
    const int opad = O <= 64 ? 64 : (O <= 128 ? 128 : 256);
    const int nk = opad / 64;
    hipError_t err = hipSuccess;
    // nothing to route / no rows: the partials the caller sums are zeros, never left unset (one route
    // block, one dW range: maxb_route_blocks(0) == maxb_dw_ranges(0) == 1)
    if (a.n_items_d == 0 && a.dbpart != nullptr &&
        (err = hipMemsetAsync(a.dbpart, 0, (size_t)((O + 3) / 4 * 4) * sizeof(float), st)) != hipSuccess)
        return err;
    if (a.V == 0 && a.wpart != nullptr &&
        (err = hipMemsetAsync(a.wpart, 0, (size_t)O * H * sizeof(float), st)) != hipSuccess)
        return err;
    // the dz passes' work-queue counters: 16 ints after the entries (the dQ pass [0, nsl), the dK pass [8, 8 + nsl))
    int* const qctr = reinterpret_cast<int*>(static_cast<int2*>(a.ent) + a.V * O);
    if (a.ent != nullptr && (a.n_items_d > 0 || a.n_items_s > 0) &&
        (err = hipMemsetAsync(qctr, 0, 16 * sizeof(int), st)) != hipSuccess)
        return err;
    // 1. routing table + db partials
    if (a.n_items_d > 0) {
        const int nb = (int)(a.route_blocks);
#define SIR_MAXB_ROUTE(NKV)                                                                                        \
        hipLaunchKernelGGL((k_maxb_route<NKV>), dim3((unsigned)nb), dim3(256), 0, st, a.rowptr_d,                    \
                           reinterpret_cast<const int4*>(a.items_d), a.n_items_d, a.arg, a.lda, a.dY, a.ldy, O,       \
                           a.pinv, reinterpret_cast<int2*>(a.ent), reinterpret_cast<int2*>(a.ecnt_d),                  \
                           reinterpret_cast<int2*>(a.ecnt_s), a.dbpart)
        if (nk == 1) SIR_MAXB_ROUTE(1);
        else if (nk == 2) SIR_MAXB_ROUTE(2);
        else SIR_MAXB_ROUTE(4);
#undef SIR_MAXB_ROUTE
        if ((err = hipGetLastError()) != hipSuccess) return err;
    }
    const int nsl = (H + 127) / 128;
    const int ncu = device_cu_count();
    const int nbs = (ncu + nsl - 1) / nsl;
    err = maxb_acts(a.act1, [&](auto A1) -> hipError_t {
        constexpr int X1 = decltype(A1)::value;
        auto dz = [&](auto D, auto OP) -> hipError_t {
            constexpr bool DV = decltype(D)::value;
            constexpr int OPV = decltype(OP)::value;
            const int4* items = reinterpret_cast<const int4*>(DV ? a.items_d : a.items_s);
            const int64_t n_items = DV ? a.n_items_d : a.n_items_s;
            if (n_items == 0) return hipSuccess;
            hipLaunchKernelGGL((k_maxb_dz<DV, X1, OPV, SIR_MAXB_U>), dim3((unsigned)(nbs * nsl)), dim3(1024), 0, st,
                               DV ? a.col_d : a.col_s, items, n_items,
                               reinterpret_cast<const int2*>(DV ? a.ecnt_d : a.ecnt_s),
                               reinterpret_cast<const int2*>(a.ent), DV ? a.Q : a.K, DV ? a.ldq : a.ldk,
                               DV ? a.K : a.Q, DV ? a.ldk : a.ldq, a.W, H, O, a.slope, nsl,
                               DV ? a.dQ : a.dK, DV ? a.lddq : a.lddk, a.partial, qctr + (DV ? 0 : 8));
            hipError_t e2 = hipGetLastError();
            if (e2 != hipSuccess) return e2;
            const int64_t ns = DV ? a.n_splits_d : a.n_splits_s;
            if (ns > 0) {
                hipLaunchKernelGGL(k_maxb_combine, dim3((unsigned)ns), dim3(256), 0, st,
                                   reinterpret_cast<const int4*>(DV ? a.splits_d : a.splits_s), H, a.partial,
                                   DV ? a.dQ : a.dK, DV ? a.lddq : a.lddk);
                e2 = hipGetLastError();
            }
            return e2;
        };
        auto both = [&](auto OP) -> hipError_t {
            hipError_t e2 = dz(std::true_type(), OP);
            if (e2 != hipSuccess) return e2;
            return dz(std::false_type(), OP);
        };
        hipError_t e1;
        if (opad == 64) e1 = both(std::integral_constant<int, 64>());
        else if (opad == 128) e1 = both(std::integral_constant<int, 128>());
        else e1 = both(std::integral_constant<int, 256>());
        if (e1 != hipSuccess) return e1;
        // 3. dW_R partials (wpart NULL: the caller computes dW_R itself, e.g. sir_max_dw_rows)
        if (a.V > 0 && a.wpart != nullptr) {
            const int nct = (H + 31) / 32;
            const int not_ = (O + 63) / 64;
            const int64_t R = maxb_dw_ranges(a.V);
            const int rows_per = (int)((a.V + R - 1) / R);
            hipLaunchKernelGGL((k_maxb_dw<X1>), dim3((unsigned)(not_ * ((nct + 3) / 4)), (unsigned)R), dim3(256), 0, st,
                               a.rowptr_d, a.col_d, a.arg, a.lda, a.dY, a.ldy, a.Q, a.ldq, a.K, a.ldk, (int)a.V, O, H,
                               a.slope, nct, rows_per, a.wpart);
            return hipGetLastError();
        }
        return hipSuccess;
    });
    return err;
}

}  // namespace sir
