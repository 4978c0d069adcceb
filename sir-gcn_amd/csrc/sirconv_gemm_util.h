// sirconv_gemm_util.h — helpers shared by the projection GEMM kernels (sirconv_gemm.hip,
// sirconv_gemm16.hip): the LDS fragment image order, raw buffer resources, the XCD-aware block remap.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sir {
namespace gemm {

// Fragment image of one LDS plane (and of the packed weights): the 16 halves of a row's k16
// step are two 16-byte pieces h = 0, 1; piece (row, h) sits at byte
//   (row / 32) * 1024 + h * 512 + (row % 32) * 16
// so the 64 lanes of an MFMA operand read (lane = h * 32 + row % 32) fetch 1 KiB in lane order:
// every 16-lane group of a ds_read_b128 covers 256 contiguous bytes (no bank conflict).
__host__ __device__ constexpr int fimg(int row, int h) { return ((row >> 5) << 10) + (h << 9) + ((row & 31) << 4); }

typedef __amdgpu_buffer_rsrc_t rsrc_t;
// raw buffer resource over [p, p + bytes): out-of-range loads return 0 (gfx9 word3 0x00020000)
__device__ inline rsrc_t mk_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// Bijective XCD-aware remap: consecutive wgids land on the same XCD (blocks are dispatched
// round-robin over the 8 XCDs).
__device__ inline int xcd_remap(int bid, int nblk) {
    const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

}  // namespace gemm
}  // namespace sir
