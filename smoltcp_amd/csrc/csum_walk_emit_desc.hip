// Instantiates the walk kernel (csum_walk.h) for MODE_EMIT, descriptor batches.
#include "csum_walk.h"

namespace smolcsum {
template hipError_t launch_walk<MODE_EMIT, false>(int, int, const KParams&, uint32_t, hipStream_t);
}  // namespace smolcsum
