// The block orders of the walk kernel (smoltcp_amd/csrc/csum_launch.h: xcd_block, xcd_chunk) must be
// bijections on [0, nwg): every record is visited exactly once whatever the grid.  Host-only check
// over grid sizes around multiples of 8 and of 8K, and the kernels' own grid sizes.
#include <cstdio>
#include <vector>

#include "../../smoltcp_amd/csrc/csum_launch.h"

using namespace smolcsum;

static bool bijective(uint64_t nwg, uint64_t K) {
    std::vector<unsigned char> seen(nwg, 0);
    for (uint64_t b = 0; b < nwg; ++b) {
        const uint64_t m = K == 1 ? xcd_block(b, nwg) : xcd_chunk(b, nwg, K);
        if (m >= nwg || seen[m]) return false;
        seen[m] = 1;
        // blocks that share an XCD (b % 8) keep the dispatch order among themselves
    }
    return true;
}

int main() {
    int bad = 0;
    const uint64_t Ks[] = {1, 2, 3, 4, 7, 16, 64, 256};
    for (uint64_t K : Ks) {
        for (uint64_t nwg = 1; nwg < 3000; ++nwg)
            if (!bijective(nwg, K)) {
                std::printf("not a bijection: nwg %llu K %llu\n", (unsigned long long)nwg, (unsigned long long)K);
                ++bad;
            }
        for (uint64_t nwg : {32768ull, 32769ull, 131072ull, 1048575ull, 4194304ull})
            if (!bijective(nwg, K)) ++bad;
    }
    // xcd_block: the blocks of one XCD (b % 8 equal) take one contiguous range, in dispatch order
    for (uint64_t nwg : {8ull, 9ull, 100ull, 32768ull, 32773ull}) {
        for (uint64_t x = 0; x < 8 && x < nwg; ++x) {
            uint64_t prev = ~0ull;
            for (uint64_t b = x; b < nwg; b += 8) {
                const uint64_t m = xcd_block(b, nwg);
                if (prev != ~0ull && m != prev + 1) ++bad;
                prev = m;
            }
        }
    }
    std::printf(bad ? "FAILED %d\n" : "grid orders ok\n", bad);
    return bad ? 1 : 0;
}
