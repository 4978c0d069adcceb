// sirconv_bwd_src.hip — instantiates the MODE_BWD_SRC edge kernels (one TU per pass: parallel builds).
#include "sirconv_edge_impl.h"

namespace sir {
hipError_t launch_mode_bwd_src(const EdgeArgs& a, int agg, int act, Shape s, hipStream_t st) {
    return launch_edge_mode<MODE_BWD_SRC>(a, agg, act, s, st);
}
}  // namespace sir
