// sirconv_bwd_dst_f16.hip — instantiates the MODE_BWD_DST edge kernels for f16 feature storage (one TU per
// pass and dtype: parallel builds).
#include "sirconv_edge_impl.h"

namespace sir {
template <>
hipError_t launch_edge_pass<ST_F16, MODE_BWD_DST>(const EdgeArgs& a, int agg, int act, Shape s, hipStream_t st) {
    return launch_edge_mode<ST_F16, MODE_BWD_DST>(a, agg, act, s, st);
}
}  // namespace sir
