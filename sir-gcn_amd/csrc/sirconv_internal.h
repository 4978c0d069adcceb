// Internal declarations shared by the kernel TU and the C-ABI TU (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sir {

enum { AGG_SUM = 0, AGG_MEAN = 1, AGG_SYM = 2 };
enum { ACT_IDENTITY = 0, ACT_RELU = 1, ACT_LEAKY = 2, ACT_GELU = 3, ACT_GELU_TANH = 4 };
enum { MODE_FWD = 0, MODE_BWD_DST = 1, MODE_BWD_SRC = 2 };

struct EdgeArgs {
    const int* rowptr;
    const int* col;
    const int32_t* items;
    int64_t n_items;
    const float* R;  int64_t ldr;     // row-side features
    const float* C;  int64_t ldc;     // gathered (col-side) features
    const float* G;  int64_t ldg;     // gradient rows (row-side for BWD_DST, gathered for BWD_SRC)
    const float* norm_row;
    const float* norm_col;
    float slope;
    int H;
    float* out;  int64_t ldo;
    float* partial;
    float* Gm;  int64_t ldgm;
};

hipError_t run_edge(int mode, const EdgeArgs& a, int agg, int act,
                    const int32_t* splits, int64_t n_splits, float* out_final, int64_t ld_final,
                    bool mean_div, hipStream_t st, const char** why);

}  // namespace sir
