// sirconv_fwd.hip — instantiates the MODE_FWD edge kernels (one TU per pass: parallel builds).
#include "sirconv_edge_impl.h"

namespace sir {
hipError_t launch_mode_fwd(const EdgeArgs& a, int agg, int act, Shape s, hipStream_t st) {
    return launch_edge_mode<MODE_FWD>(a, agg, act, s, st);
}
}  // namespace sir
