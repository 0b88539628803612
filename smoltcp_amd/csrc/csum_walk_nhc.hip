// Instantiates the walk kernel (csum_walk.h) with the 6LoWPAN NHC UDP gates, for emit and verify
// over fixed-stride and descriptor batches.
#include "csum_walk.h"

namespace smolcsum {
template hipError_t launch_walk_nhc<MODE_EMIT, true>(int, int, const KParams&, uint32_t, hipStream_t);
template hipError_t launch_walk_nhc<MODE_EMIT, false>(int, int, const KParams&, uint32_t, hipStream_t);
template hipError_t launch_walk_nhc<MODE_VERIFY, true>(int, int, const KParams&, uint32_t, hipStream_t);
template hipError_t launch_walk_nhc<MODE_VERIFY, false>(int, int, const KParams&, uint32_t, hipStream_t);
}  // namespace smolcsum
