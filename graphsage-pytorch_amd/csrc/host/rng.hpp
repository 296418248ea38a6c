// The opaque C-ABI rng handle (gs_rng in include/graphsage_amd.h): one CPython
// `random.Random` stream, shared by the sampler and UnsupervisedLoss.
#pragma once

#include "mt19937.hpp"

struct gs_rng {
    gs::MT19937 mt;
};
