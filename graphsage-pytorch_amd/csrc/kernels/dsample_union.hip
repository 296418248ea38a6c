// Device sampler, hops before the last: models.py:282-286 (see dsample.hip).
#include "dsample.hpp"

namespace gs {
namespace ds {

void launch_hop_union(const DevGraph& g, Ctl* c, const HopBufs& hb, UnionBufs& ub, const HopBufs& next, int hop,
                      int k, int64_t nd_max, int64_t nd_next_max, int flags, int32_t* pack, hipStream_t st) {
    fail(GS_EINVAL, "device sampler: multi-hop union not built yet");
}

}  // namespace ds
}  // namespace gs
