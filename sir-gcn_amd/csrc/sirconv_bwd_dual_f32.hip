// sirconv_bwd_dual_f32.hip — instantiates the one-launch sign-mask backward (dQ pass || dK pass)
// for f32 feature storage.
#include "sirconv_edge_impl.h"

namespace sir {
template <>
hipError_t launch_edge_dual<ST_F32>(const EdgeArgs& a, const EdgeArgs& b, int agg, int act, Shape s, hipStream_t st) {
    return launch_edge_dual_st<ST_F32>(a, b, agg, act, s, st);
}
}  // namespace sir
