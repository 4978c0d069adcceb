// sirconv_dropout.h — the layer's feature dropout on Q and K (conv.py:35,60-61: nn.Dropout(p) applied
// to X W_K^T and to X W_Q^T + b_Q), fused into the kernels that already touch those elements.
//
// The mask is never stored.  Element (row, col) of QK = [Q | K] (col < H: Q, col >= H: K) is kept
// iff a counter-based hash of (seed, row, col) is >= thr = round(p 2^32); a kept element is scaled
// by 1 / (1 - p) (nn.Dropout's scale, computed in fp32).  The QK GEMM's epilogue applies it to the
// forward values; the backward edge passes apply the SAME mask (the hash is recomputed from the
// row and column each of them writes) to dQ = dQK[:, :H] and dK = dQK[:, H:] before storing them,
// which is the backward of the dropout (grad * mask * scale).  Q and K draw independent bits, as
// the reference's two Dropout calls do.  The hash is murmur3's 32-bit finaliser, once per row and
// once per element.
//
// The seed is a kernel argument or, when `sptr` is set, a uint64 in device memory read when the
// kernel starts (drop_resolve, first thing in every kernel that takes a Drop): a forward captured in
// a HIP graph then draws a fresh mask on every replay, because the captured RNG op that writes the
// seed (torch.randint on the device, graph-safe philox) runs again; the backward reads the same word.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sir {

struct Drop {
    uint32_t s0 = 0, s1 = 0;   // seed words
    uint32_t thr_lo = 0;       // keep iff hash >= thr (thr = thr_hi * 2^32 + thr_lo, in [0, 2^32])
    uint32_t thr_hi = 0;
    float scale = 1.f;
    int col0 = 0;              // column of the first output feature in QK (0: Q / whole QK, H: K)
    const uint64_t* sptr = nullptr;   // device-resident seed (overrides s0 / s1 at kernel start)
    __host__ __device__ bool on() const { return (thr_lo | thr_hi) != 0; }
};

__host__ __device__ inline void drop_seed_words(Drop& d, uint64_t seed) {
    d.s0 = (uint32_t)seed;
    d.s1 = (uint32_t)(seed >> 32) ^ 0x6A09E667u;
}

// device: a Drop whose seed words come from `sptr` when set (one load per thread, at kernel start)
#ifndef SIR_DROP_DEVSEED
#define SIR_DROP_DEVSEED 1
#endif
__device__ __forceinline__ Drop drop_resolve(Drop d) {
    if (SIR_DROP_DEVSEED && d.on() && d.sptr != nullptr) drop_seed_words(d, *d.sptr);
    return d;
}

__host__ __device__ inline uint32_t drop_fmix(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
__host__ __device__ inline uint32_t drop_row_hash(const Drop& d, int64_t row) {
    return drop_fmix(((uint32_t)row * 0x9E3779B1u) ^ ((uint32_t)((uint64_t)row >> 32) * 0x7FEB352Du) ^ d.s0);
}
__host__ __device__ inline bool drop_keep(const Drop& d, uint32_t rh, int col) {
    const uint32_t h = drop_fmix(rh ^ ((uint32_t)col * 0xCC9E2D51u + d.s1));
    return d.thr_hi == 0 && h >= d.thr_lo;       // thr = 2^32 (p = 1) keeps nothing
}

// host: the Drop of a probability p and a 64-bit seed (p <= 0: off)
inline Drop make_drop(double p, uint64_t seed, int col0 = 0, const uint64_t* sptr = nullptr) {
    Drop d;
    if (!(p > 0.0)) return d;
    const double t = p >= 1.0 ? 4294967296.0 : p * 4294967296.0;
    uint64_t thr = (uint64_t)(t + 0.5);
    if (thr == 0) thr = 1;                       // a tiny p still drops something (never "off")
    d.thr_lo = (uint32_t)thr;
    d.thr_hi = (uint32_t)(thr >> 32);
    d.scale = p >= 1.0 ? 0.f : (float)(1.0 / (1.0 - p));
    drop_seed_words(d, seed);
    d.col0 = col0;
    d.sptr = sptr;
    return d;
}

}  // namespace sir
