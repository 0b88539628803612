// Dispatches a batched call to the walk kernel instantiation for its mode and batch form (and, in the
// experiments build, instantiates the walk kernel's MODE_COPY variants).
#include "csum_walk.h"

namespace smolcsum {

// instantiated in csum_walk_{data,emit,verify}_{fixed,desc}.hip and csum_walk_nhc.hip
extern template hipError_t launch_walk<MODE_DATA, true>(int, int, const KParams&, uint32_t, hipStream_t);
extern template hipError_t launch_walk<MODE_DATA, false>(int, int, const KParams&, uint32_t, hipStream_t);
extern template hipError_t launch_walk<MODE_EMIT, true>(int, int, const KParams&, uint32_t, hipStream_t);
extern template hipError_t launch_walk<MODE_EMIT, false>(int, int, const KParams&, uint32_t, hipStream_t);
extern template hipError_t launch_walk<MODE_VERIFY, true>(int, int, const KParams&, uint32_t, hipStream_t);
extern template hipError_t launch_walk<MODE_VERIFY, false>(int, int, const KParams&, uint32_t, hipStream_t);
extern template hipError_t launch_walk_nhc<MODE_EMIT, true>(int, int, const KParams&, uint32_t, hipStream_t);
extern template hipError_t launch_walk_nhc<MODE_EMIT, false>(int, int, const KParams&, uint32_t, hipStream_t);
extern template hipError_t launch_walk_nhc<MODE_VERIFY, true>(int, int, const KParams&, uint32_t, hipStream_t);
extern template hipError_t launch_walk_nhc<MODE_VERIFY, false>(int, int, const KParams&, uint32_t, hipStream_t);

hipError_t launch_csum(int mode, int shape, int var, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    const bool implicit = p.desc == nullptr;
    if (p.addrs) {  // 6LoWPAN NHC UDP
        if (mode == MODE_EMIT)
            return implicit ? launch_walk_nhc<MODE_EMIT, true>(shape, var, p, max_blocks, s)
                            : launch_walk_nhc<MODE_EMIT, false>(shape, var, p, max_blocks, s);
        if (mode == MODE_VERIFY)
            return implicit ? launch_walk_nhc<MODE_VERIFY, true>(shape, var, p, max_blocks, s)
                            : launch_walk_nhc<MODE_VERIFY, false>(shape, var, p, max_blocks, s);
        return hipErrorInvalidValue;
    }
    switch (mode) {
        case MODE_DATA:
            return implicit ? launch_walk<MODE_DATA, true>(shape, var, p, max_blocks, s)
                            : launch_walk<MODE_DATA, false>(shape, var, p, max_blocks, s);
        case MODE_EMIT:
            return implicit ? launch_walk<MODE_EMIT, true>(shape, var, p, max_blocks, s)
                            : launch_walk<MODE_EMIT, false>(shape, var, p, max_blocks, s);
        case MODE_COPY:
            return implicit ? launch_copy<true>(shape, var, p, max_blocks, s) : launch_copy<false>(shape, var, p, max_blocks, s);
        default:
            return implicit ? launch_walk<MODE_VERIFY, true>(shape, var, p, max_blocks, s)
                            : launch_walk<MODE_VERIFY, false>(shape, var, p, max_blocks, s);
    }
}

}  // namespace smolcsum
