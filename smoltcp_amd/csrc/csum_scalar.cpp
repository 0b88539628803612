// Scalar host mirrors of smoltcp::wire::checksum (include/smolcsum.h, group 1): plain C++, no
// HIP, so that the sanitizer build (tests/cpp/Makefile `sanitize`) can instrument them.
#include <cstdint>
#include <cstring>

#include "../../include/smolcsum.h"

namespace {

inline uint16_t fold_u32(uint32_t w) {  // propagate_carries, src/wire/ip.rs:767-770
    uint32_t s = (w >> 16) + (w & 0xffffu);
    return (uint16_t)(((s >> 16) + s) & 0xffffu);
}

inline uint16_t swap16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }

}  // namespace

extern "C" {

// checksum::data, src/wire/ip.rs:773-804.  Little-endian u16 words are summed exactly in 64 bits
// and truncated to 32 bits, which equals the reference's wrapping u32 accumulator.
uint16_t smol_csum_data(const uint8_t* d, size_t n) {
    uint64_t acc = 0;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t q;
        std::memcpy(&q, d + i, 8);
        acc += (q & 0xffffu) + ((q >> 16) & 0xffffu) + ((q >> 32) & 0xffffu) + (q >> 48);
    }
    for (; i + 2 <= n; i += 2) acc += (uint32_t)d[i] | ((uint32_t)d[i + 1] << 8);
    if (i < n) acc += d[i];
    return swap16(fold_u32((uint32_t)acc));
}

// checksum::combine, src/wire/ip.rs:807-813
uint16_t smol_csum_combine(const uint16_t* c, size_t n) {
    uint32_t acc = 0;
    for (size_t i = 0; i < n; i++) acc += c[i];
    return fold_u32(acc);
}

static uint16_t pseudo(const uint8_t* src, const uint8_t* dst, size_t alen, uint8_t nh,
                       uint32_t length) {
    const uint8_t pl[4] = {0, nh, (uint8_t)(length >> 8), (uint8_t)length};
    const uint16_t parts[3] = {smol_csum_data(src, alen), smol_csum_data(dst, alen),
                               smol_csum_data(pl, 4)};
    return smol_csum_combine(parts, 3);
}

// checksum::pseudo_header_v4, src/wire/ip.rs:816-831
uint16_t smol_csum_pseudo_header_v4(const uint8_t src[4], const uint8_t dst[4], uint8_t nh,
                                    uint32_t length) {
    return pseudo(src, dst, 4, nh, length);
}

// checksum::pseudo_header_v6, src/wire/ip.rs:834-849
uint16_t smol_csum_pseudo_header_v6(const uint8_t src[16], const uint8_t dst[16], uint8_t nh,
                                    uint32_t length) {
    return pseudo(src, dst, 16, nh, length);
}

// checksum::pseudo_header, src/wire/ip.rs:851-869
int smol_csum_pseudo_header(int src_family, const uint8_t* src, int dst_family,
                            const uint8_t* dst, uint8_t nh, uint32_t length, uint16_t* out) {
    if (!src || !dst || !out || src_family != dst_family) return SMOL_EINVAL;
    if (src_family == 4) { *out = smol_csum_pseudo_header_v4(src, dst, nh, length); return SMOL_OK; }
    if (src_family == 6) { *out = smol_csum_pseudo_header_v6(src, dst, nh, length); return SMOL_OK; }
    return SMOL_EINVAL;
}

}  // extern "C"
