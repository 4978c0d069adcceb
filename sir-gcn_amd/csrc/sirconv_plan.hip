// sirconv_plan.hip — device-side COO -> row-CSR + work-plan build.
//
// DGL builds a graph's in-edge CSC lazily on the first update_all (conv.py:63) with a stable
// counting sort on the host; batched configs (zinc/train.py, ogbg-molhiv) and DropEdge
// (models/utils.py:96-102) rebuild it for every batch / layer.  Here the whole plan is built on
// the device in a few launches:
//   1. k_count     : per-edge validation, int32 sort keys/values, in-degree histogram
//   2. radix sort  : (row, edge id) pairs, stable  ->  edge ids ascending inside every row
//   3. k_gather    : col = cols[eid]
//   4. scan        : per-row {deg, n_items, is_split, n_slots} -> rowptr and plan offsets
//   5. k_rows      : rowptr, work items {row, e_begin, e_end, slot}, split rows
//                    {row, slot_begin, n_slots, degree}, totals
// Deterministic (integer atomics only in the histogram, stable sort).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "sirconv_internal.h"

namespace sir {
namespace {

struct RowAcc {
    int deg, items, split, slots;
};

struct RowAdd {
    __host__ __device__ RowAcc operator()(const RowAcc& a, const RowAcc& b) const {
        return RowAcc{a.deg + b.deg, a.items + b.items, a.split + b.split, a.slots + b.slots};
    }
};

__global__ void k_count(const int64_t* __restrict__ rows, const int64_t* __restrict__ cols, int64_t E,
                        int64_t n_rows, int64_t n_cols, int* __restrict__ deg, unsigned* __restrict__ keys,
                        int* __restrict__ vals, unsigned long long* __restrict__ bad) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    int64_t r = rows[e];
    const int64_t c = cols[e];
    if (r < 0 || r >= n_rows || c < 0 || c >= n_cols) {
        atomicAdd(bad, 1ull);
        r = 0;                                  // keep the sort in range; the host raises
    }
    atomicAdd(deg + r, 1);
    keys[e] = (unsigned)r;
    vals[e] = (int)e;
}

__global__ void k_gather(const int* __restrict__ eid32, const int64_t* __restrict__ cols, int64_t E, int64_t n_cols,
                         int* __restrict__ col, int64_t* __restrict__ eid) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= E) return;
    const int e = eid32[i];
    int64_t c = cols[e];
    if (c < 0 || c >= n_cols) c = 0;            // flagged by k_count
    col[i] = (int)c;
    eid[i] = e;
}

__global__ void k_row_acc(const int* __restrict__ deg, int64_t n_rows, int chunk, RowAcc* __restrict__ acc) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    const int d = deg[r];
    const int nch = d > chunk ? (d + chunk - 1) / chunk : 1;
    const int s = nch > 1;
    acc[r] = RowAcc{d, nch, s, s ? nch : 0};
}

__global__ void k_rows(const RowAcc* __restrict__ acc, const RowAcc* __restrict__ off, int64_t n_rows, int chunk,
                       int* __restrict__ rowptr, int4* __restrict__ items, int4* __restrict__ splits,
                       int64_t* __restrict__ counts) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    const RowAcc a = acc[r];
    const RowAcc o = off[r];
    const int rp = o.deg;
    rowptr[r] = rp;
    for (int k = 0; k < a.items; ++k) {
        const int eb = rp + k * chunk;
        const int ee = min(eb + chunk, rp + a.deg);
        items[o.items + k] = make_int4((int)r, eb, ee, a.split ? o.slots + k : -1);
    }
    if (a.split) splits[o.split] = make_int4((int)r, o.slots, a.items, a.deg);
    atomicMax(reinterpret_cast<unsigned long long*>(counts + 3), (unsigned long long)a.deg);
    if (r == n_rows - 1) {
        rowptr[n_rows] = rp + a.deg;
        counts[0] = o.items + a.items;
        counts[1] = o.split + a.split;
        counts[2] = o.slots + a.slots;
    }
}

__global__ void k_pos(const int64_t* __restrict__ eid_a, int64_t E, int* __restrict__ pos) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < E) pos[eid_a[i]] = (int)i;
}

__global__ void k_perm(const int64_t* __restrict__ eid_b, int64_t E, const int* __restrict__ pos,
                       int* __restrict__ perm) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < E) perm[i] = pos[eid_b[i]];
}

inline size_t up256(size_t x) { return (x + 255) & ~size_t(255); }

inline int key_bits(int64_t n_rows) {
    int b = 1;
    while (b < 31 && (int64_t(1) << b) < n_rows) ++b;
    return b;
}

// workspace: deg | acc | off | keys_in | keys_out | vals_in | vals_out | cub temp
struct Layout {
    size_t deg, acc, off, kin, kout, vin, vout, temp, temp_bytes, total;
};

hipError_t layout(int64_t n_rows, int64_t E, Layout& L) {
    size_t sort_bytes = 0, scan_bytes = 0;
    if (E > 0) {
        hipError_t err = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const unsigned*)nullptr, (unsigned*)nullptr,
                                                            (const int*)nullptr, (int*)nullptr, (int)E, 0,
                                                            key_bits(n_rows));
        if (err != hipSuccess) return err;
    }
    if (n_rows > 0) {
        hipError_t err = hipcub::DeviceScan::ExclusiveScan(nullptr, scan_bytes, (const RowAcc*)nullptr,
                                                           (RowAcc*)nullptr, RowAdd(), RowAcc{0, 0, 0, 0},
                                                           (int)n_rows);
        if (err != hipSuccess) return err;
    }
    size_t o = 0;
    L.deg = o;  o += up256(sizeof(int) * (size_t)(n_rows + 1));
    L.acc = o;  o += up256(sizeof(RowAcc) * (size_t)(n_rows + 1));
    L.off = o;  o += up256(sizeof(RowAcc) * (size_t)(n_rows + 1));
    L.kin = o;  o += up256(sizeof(int) * (size_t)(E + 1));
    L.kout = o; o += up256(sizeof(int) * (size_t)(E + 1));
    L.vin = o;  o += up256(sizeof(int) * (size_t)(E + 1));
    L.vout = o; o += up256(sizeof(int) * (size_t)(E + 1));
    L.temp = o;
    L.temp_bytes = up256(sort_bytes > scan_bytes ? sort_bytes : scan_bytes) + 256;
    o += L.temp_bytes;
    L.total = o;
    return hipSuccess;
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

int64_t csr_build_workspace(int64_t n_rows, int64_t E) {
    Layout L;
    if (layout(n_rows, E, L) != hipSuccess) return -1;
    return (int64_t)L.total;
}

hipError_t run_csr_build(const int64_t* rows, const int64_t* cols, int64_t E, int64_t n_rows, int64_t n_cols,
                         int chunk, int* rowptr, int* col, int64_t* eid, int32_t* items, int32_t* splits,
                         int64_t* counts, void* ws, int64_t ws_bytes, hipStream_t st) {
    Layout L;
    hipError_t err = layout(n_rows, E, L);
    if (err != hipSuccess) return err;
    if ((int64_t)L.total > ws_bytes) return hipErrorInvalidValue;
    char* w = static_cast<char*>(ws);
    int* deg = reinterpret_cast<int*>(w + L.deg);
    RowAcc* acc = reinterpret_cast<RowAcc*>(w + L.acc);
    RowAcc* off = reinterpret_cast<RowAcc*>(w + L.off);
    unsigned* kin = reinterpret_cast<unsigned*>(w + L.kin);
    unsigned* kout = reinterpret_cast<unsigned*>(w + L.kout);
    int* vin = reinterpret_cast<int*>(w + L.vin);
    int* vout = reinterpret_cast<int*>(w + L.vout);
    void* temp = w + L.temp;
    // counts: {n_items, n_splits, n_slots, max_degree, n_bad_ids}
    if ((err = hipMemsetAsync(counts, 0, 5 * sizeof(int64_t), st)) != hipSuccess) return err;
    if ((err = hipMemsetAsync(deg, 0, sizeof(int) * (size_t)(n_rows + 1), st)) != hipSuccess) return err;
    if (n_rows == 0) return hipMemsetAsync(rowptr, 0, sizeof(int), st);
    if (E > 0) {
        hipLaunchKernelGGL(k_count, dim3(nblk(E)), dim3(256), 0, st, rows, cols, E, n_rows, n_cols, deg, kin, vin,
                           reinterpret_cast<unsigned long long*>(counts + 4));
        if ((err = hipGetLastError()) != hipSuccess) return err;
        size_t tb = L.temp_bytes;
        err = hipcub::DeviceRadixSort::SortPairs(temp, tb, kin, kout, vin, vout, (int)E, 0, key_bits(n_rows), st);
        if (err != hipSuccess) return err;
        hipLaunchKernelGGL(k_gather, dim3(nblk(E)), dim3(256), 0, st, vout, cols, E, n_cols, col, eid);
        if ((err = hipGetLastError()) != hipSuccess) return err;
    }
    hipLaunchKernelGGL(k_row_acc, dim3(nblk(n_rows)), dim3(256), 0, st, deg, n_rows, chunk, acc);
    if ((err = hipGetLastError()) != hipSuccess) return err;
    size_t tb = L.temp_bytes;
    err = hipcub::DeviceScan::ExclusiveScan(temp, tb, acc, off, RowAdd(), RowAcc{0, 0, 0, 0}, (int)n_rows, st);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(k_rows, dim3(nblk(n_rows)), dim3(256), 0, st, acc, off, n_rows, chunk, rowptr,
                       reinterpret_cast<int4*>(items), reinterpret_cast<int4*>(splits), counts);
    return hipGetLastError();
}

hipError_t run_csr_perm(const int64_t* eid_a, const int64_t* eid_b, int64_t E, int* pos_ws, int* perm,
                        hipStream_t st) {
    if (E == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pos, dim3(nblk(E)), dim3(256), 0, st, eid_a, E, pos_ws);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(k_perm, dim3(nblk(E)), dim3(256), 0, st, eid_b, E, pos_ws, perm);
    return hipGetLastError();
}

}  // namespace sir
