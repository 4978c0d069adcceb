// sirconv_bwd_src_f32.hip — instantiates the MODE_BWD_SRC edge kernels for f32 feature storage (one TU per
// pass and dtype: parallel builds).
#include "sirconv_edge_impl.h"

namespace sir {
template <>
hipError_t launch_edge_pass<ST_F32, MODE_BWD_SRC>(const EdgeArgs& a, int agg, int act, Shape s, hipStream_t st) {
    return launch_edge_mode<ST_F32, MODE_BWD_SRC>(a, agg, act, s, st);
}
}  // namespace sir
