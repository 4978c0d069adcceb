// MFMA throughput probe (round 5): v_mfma_f32_32x32x16_f16 and v_mfma_f32_16x16x32_f16 back to back on
// independent accumulators, one block of W waves per CU on every CU, operands random in [-1, 1) or zero
// (DVFS: MI355X_MICROARCH.md).  Prints wall time per MFMA per SIMD and the chip's f16 TFLOP/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(512) k32(const h8* in, float* out, int iters) {
    const int l = threadIdx.x;
    h8 a = in[l & 255], b = in[(l + 7) & 255];
    f16v acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = (f16v){};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[i], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, acc[i], 0, 0, 0);
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i][l & 15];
    out[blockIdx.x * blockDim.x + l] = s;
}
__global__ void __launch_bounds__(512) k16(const h8* in, float* out, int iters) {     // same FLOPs per iteration
    const int l = threadIdx.x;
    h8 a = in[l & 255], b = in[(l + 7) & 255];
    f4v acc[32];
    for (int i = 0; i < 32; ++i) acc[i] = (f4v){};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 32; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[i], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 32; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, acc[i], 0, 0, 0);
    }
    float s = 0;
    for (int i = 0; i < 32; ++i) s += acc[i][l & 3];
    out[blockIdx.x * blockDim.x + l] = s;
}
int main() {
    std::vector<_Float16> h(256 * 8), z(256 * 8, (_Float16)0.f);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (_Float16)((float)((i * 2654435761u) % 2000) / 1000.f - 1.f);
    h8 *in, *zin; float* out;
    (void)hipMalloc(&in, h.size() * 2); (void)hipMalloc(&zin, h.size() * 2); (void)hipMalloc(&out, 256 * 512 * 4);
    (void)hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(zin, z.data(), z.size() * 2, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int iters = 4000;
    for (int shape = 0; shape < 2; ++shape)
        for (int data = 0; data < 2; ++data)
            for (int threads : {256, 512}) {
                float best = 1e30f;
                for (int rep = 0; rep < 3; ++rep) {
                    (void)hipEventRecord(e0);
                    if (shape == 0) hipLaunchKernelGGL(k32, dim3(256), dim3(threads), 0, 0, data ? zin : in, out, iters);
                    else hipLaunchKernelGGL(k16, dim3(256), dim3(threads), 0, 0, data ? zin : in, out, iters);
                    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
                    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
                    if (ms < best) best = ms;
                }
                const double flop = 256.0 * threads / 64 * iters * 16.0 * 32768;   // both shapes: 16 x 32 k-flop-units per iteration
                printf("%s %s waves/CU %d: %.3f ms, %.0f TFLOP/s f16 (%.0f %% of 2.5 PF)\n", shape ? "16x16x32" : "32x32x16",
                       data ? "zero  " : "random", threads / 64, best, flop / (best * 1e-3) / 1e12, flop / (best * 1e-3) / 2.5e15 * 100);
            }
    return 0;
}
