// sirconv_bwd_dst.hip — instantiates the MODE_BWD_DST edge kernels (one TU per pass: parallel builds).
#include "sirconv_edge_impl.h"

namespace sir {
hipError_t launch_mode_bwd_dst(const EdgeArgs& a, int agg, int act, Shape s, hipStream_t st) {
    return launch_edge_mode<MODE_BWD_DST>(a, agg, act, s, st);
}
}  // namespace sir
