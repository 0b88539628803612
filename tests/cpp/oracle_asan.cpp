// Sanitizer driver (tests/cpp/Makefile `sanitize`, run by tests/test_sanitize_cpu.py): the CPU
// oracle (oracle/csum_oracle.c) and the library's scalar host mirrors (csum_scalar.cpp), built with
// -fsanitize=address,undefined, over every truncation of the golden records and over random
// records.  Each truncated record lives in a heap block of exactly its length, so any read past
// the bytes the geometry checks allow is reported by AddressSanitizer; UBSan traps on shifts,
// overflow of signed arithmetic and misaligned accesses.
//
//   oracle_asan records <file>     lines "<kind> <hex>" (kind 1 = IP, 2 = Ethernet)
//   oracle_asan random <seed> <n>  n random records (plausible IPv4 / IPv6 / Ethernet headers)
//   oracle_asan frag <seed> <n>    n random IPv4 fragment groups through oracle_batch_emit_frag /
//                                  _verify_frag (every fragment in a heap block of exactly its length;
//                                  sound, overlapping, gapped and truncated layouts, offsets up to the
//                                  13-bit maximum 65528, invalid group ranges), and random frag.buffer
//                                  contents through oracle_emit_like_dispatch_ip
// Prints "ok <records>" and exits 0; a mismatch between the scalar mirror and the oracle exits 1.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/smolcsum.h"

extern "C" {
uint16_t oracle_data(const uint8_t* data, size_t len);
uint8_t oracle_record_verify(const uint8_t* rec, size_t len, int kind, const smol_checksum_caps_t* caps);
uint8_t oracle_record_emit(uint8_t* rec, size_t len, int kind, const smol_checksum_caps_t* caps);
uint8_t oracle_nhc_udp_verify(const uint8_t* rec, size_t len, const uint8_t* addrs, const smol_checksum_caps_t* caps);
uint8_t oracle_nhc_udp_emit(uint8_t* rec, size_t len, const uint8_t* addrs, const smol_checksum_caps_t* caps);
void oracle_batch_copy_emit(uint8_t* buf, const smol_csum_desc_t* desc, uint64_t n, uint64_t stride, uint32_t len,
                            uint32_t kind, const smol_checksum_caps_t* caps, const uint8_t* src,
                            const smol_csum_copy_t* copy, uint8_t* status);
void oracle_batch_emit_frag(uint8_t* buf, const smol_csum_desc_t* desc, uint64_t n, uint64_t stride, uint32_t len,
                            uint32_t kind, const smol_csum_frag_group_t* groups, uint64_t ngroups,
                            const smol_checksum_caps_t* caps, uint8_t* status);
void oracle_batch_verify_frag(uint8_t* buf, const smol_csum_desc_t* desc, uint64_t n, uint64_t stride, uint32_t len,
                              uint32_t kind, const smol_csum_frag_group_t* groups, uint64_t ngroups,
                              const smol_checksum_caps_t* caps, uint8_t* status);
int oracle_emit_like_dispatch_ip(uint8_t* fbuf, size_t fbuf_len, const smol_checksum_caps_t* caps);
}

static int failures = 0;

static const smol_checksum_caps_t kCaps[4] = {
    {0, 0, 0, 0, 0, {0, 0, 0}}, {3, 3, 3, 3, 3, {0, 0, 0}}, {1, 2, 1, 2, 1, {0, 0, 0}}, {2, 1, 2, 1, 2, {0, 0, 0}}};

// One record of exactly `len` heap bytes through every oracle entry point and the scalar mirror.
static void exercise(const uint8_t* bytes, size_t len, int kind) {
    uint8_t* r = static_cast<uint8_t*>(std::malloc(len ? len : 1));
    std::memcpy(r, bytes, len);
    if (smol_csum_data(r, len) != oracle_data(r, len)) {
        std::fprintf(stderr, "data mismatch at len %zu\n", len);
        ++failures;
    }
    static const uint8_t addrs[32] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16,
                                      17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32};
    for (const auto& c : kCaps) {
        (void)oracle_record_verify(r, len, kind, &c);
        uint8_t* e = static_cast<uint8_t*>(std::malloc(len ? len : 1));
        std::memcpy(e, r, len);
        (void)oracle_record_emit(e, len, kind, &c);
        const uint8_t st = oracle_record_verify(e, len, kind, &c);
        (void)st;
        std::memcpy(e, r, len);
        (void)oracle_nhc_udp_verify(e, len, addrs, &c);
        (void)oracle_nhc_udp_emit(e, len, addrs, &c);
        std::free(e);
    }
    // fused copy + emit: the second half of the record from a source block of exactly that size
    const uint32_t half = (uint32_t)(len / 2), plen = (uint32_t)(len - half);
    uint8_t* src = static_cast<uint8_t*>(std::malloc(plen ? plen : 1));
    for (uint32_t i = 0; i < plen; ++i) src[i] = uint8_t(i * 7 + 1);
    smol_csum_desc_t d = {0, (uint32_t)len, (uint8_t)kind, 0, 0};
    smol_csum_copy_t cp = {0, half, plen};
    uint8_t st = 0;
    oracle_batch_copy_emit(r, &d, 1, 0, 0, 0, &kCaps[0], src, &cp, &st);
    std::free(src);
    std::free(r);
}

static std::vector<uint8_t> unhex(const std::string& h) {
    std::vector<uint8_t> v;
    for (size_t i = 0; i + 1 < h.size(); i += 2) v.push_back(uint8_t(std::stoul(h.substr(i, 2), nullptr, 16)));
    return v;
}

static uint32_t xs(uint32_t& x) {  // xorshift32
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return x;
}

// One random fragment group: `count` fragments, each its own heap block, plus invalid group ranges.
static void exercise_frag(uint32_t& x) {
    const uint32_t count = 1 + xs(x) % ((xs(x) & 7) ? 6 : 40);
    const uint32_t mode = xs(x) % 6;  // 0-2 sound layouts, 3 near the maximum offset, 4 broken, 5 truncated
    const uint8_t proto = (const uint8_t[]){1, 2, 6, 17, 89}[xs(x) % 5];
    const uint32_t step = 8 * (1 + xs(x) % 40);
    std::vector<uint8_t*> blocks(count);
    std::vector<smol_csum_desc_t> desc(count);
    std::vector<size_t> lens(count);
    uint32_t base_off = mode == 3 ? 65528 - step * (count - 1) % 65528 : 0;
    base_off &= ~7u;
    for (uint32_t i = 0; i < count; ++i) {
        const bool last = i + 1 == count;
        uint32_t plen = last ? 1 + xs(x) % (step + 60) : step;
        if (mode == 3 && last) plen = 65535 - 20 - (base_off + step * i > 65515 ? 65515 : base_off + step * i) % 65516;
        if (plen > 65515) plen = 65515;
        const int eth = (xs(x) % 4) == 0;
        size_t len = (eth ? 14 : 0) + 20 + plen;
        if (mode == 5) len = xs(x) % (len + 1);
        lens[i] = len;
        uint8_t* b = static_cast<uint8_t*>(std::malloc(len ? len : 1));
        for (size_t k = 0; k < len; ++k) b[k] = uint8_t(xs(x));
        const size_t io = eth ? 14 : 0;
        if (eth && len >= 14) { b[12] = 0x08; b[13] = 0x00; }
        if (len >= io + 20) {
            uint8_t* ip = b + io;
            ip[0] = 0x45;
            const uint32_t tl = 20 + plen - (mode == 4 ? xs(x) % 3 : 0);
            ip[2] = uint8_t(tl >> 8); ip[3] = uint8_t(tl);
            ip[4] = 0x12; ip[5] = uint8_t(mode == 4 && (xs(x) & 1) ? xs(x) : 0x34);
            uint32_t off = (base_off + step * i) / 8;
            if (mode == 4 && (xs(x) & 1)) off = xs(x) & 0x1fff;
            if (off > 0x1fff) off = 0x1fff;
            const uint32_t mf = last ? (mode == 4 ? xs(x) & 1 : 0) : 1;
            ip[6] = uint8_t((mf << 5) | (off >> 8)); ip[7] = uint8_t(off);
            ip[9] = proto;
            for (int k = 12; k < 20; ++k) ip[k] = uint8_t(k);
        }
        blocks[i] = b;
    }
    // records live in separate heap blocks: offsets from the lowest one
    uintptr_t lo = (uintptr_t)blocks[0];
    for (auto* b : blocks) lo = (uintptr_t)b < lo ? (uintptr_t)b : lo;
    for (uint32_t i = 0; i < count; ++i)
        desc[i] = smol_csum_desc_t{(uint64_t)((uintptr_t)blocks[i] - lo), (uint32_t)lens[i],
                                   (uint8_t)(lens[i] >= 14 && blocks[i][12] == 0x08 && blocks[i][13] == 0 ? 2 : 1),
                                   (uint8_t)((xs(x) % 16) == 0 ? SMOL_REC_IPHDR_ONLY : 0), 0};
    const smol_csum_frag_group_t groups[5] = {{0, count, 0}, {count, 1, 0}, {count - 1, 2, 0}, {0, count, 7},
                                              {1, 0xffffffffu, 0}};
    std::vector<uint8_t> st(count);
    for (const auto& c : kCaps) {
        oracle_batch_verify_frag((uint8_t*)lo, desc.data(), count, 0, 0, 0, groups, 5, &c, st.data());
        oracle_batch_emit_frag((uint8_t*)lo, desc.data(), count, 0, 0, 0, groups, 5, &c, st.data());
        oracle_batch_verify_frag((uint8_t*)lo, desc.data(), count, 0, 0, 0, groups, 5, &c, st.data());
    }
    for (auto* b : blocks) std::free(b);
    // the reference's dispatch_ip route over a random frag.buffer
    const size_t fl = xs(x) % 5000;
    uint8_t* fb = static_cast<uint8_t*>(std::malloc(fl ? fl : 1));
    for (size_t k = 0; k < fl; ++k) fb[k] = uint8_t(xs(x));
    if (fl >= 20) {
        fb[0] = uint8_t(0x40 | (5 + xs(x) % 11));
        const size_t tl = xs(x) % (fl + 10);
        fb[2] = uint8_t(tl >> 8); fb[3] = uint8_t(tl);
        fb[9] = (const uint8_t[]){1, 2, 6, 17}[xs(x) % 4];
    }
    for (const auto& c : kCaps) (void)oracle_emit_like_dispatch_ip(fb, fl, &c);
    std::free(fb);
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const std::string mode = argv[1];
    size_t count = 0;
    if (mode == "records") {
        std::ifstream f(argv[2]);
        std::string line;
        while (std::getline(f, line)) {
            std::istringstream is(line);
            int kind;
            std::string h;
            if (!(is >> kind >> h)) continue;
            const auto b = unhex(h);
            for (size_t n = 0; n <= b.size(); ++n) exercise(b.data(), n, kind);  // every truncation
            ++count;
        }
    } else if (mode == "random" && argc >= 4) {
        uint32_t x = (uint32_t)std::strtoul(argv[2], nullptr, 0) | 1u;
        const size_t n = std::strtoull(argv[3], nullptr, 0);
        std::vector<uint8_t> b;
        for (size_t i = 0; i < n; ++i) {
            const size_t len = xs(x) % 400;
            b.assign(len, 0);
            for (auto& v : b) v = uint8_t(xs(x));
            const int kind = 1 + (int)(xs(x) % 2);
            const size_t ip = kind == 2 ? 14 : 0;
            if (kind == 2 && len >= 14) { b[12] = (xs(x) & 1) ? 0x08 : 0x86; b[13] = b[12] == 0x08 ? 0x00 : 0xdd; }
            if (len > ip) {
                const bool v6 = kind == 2 ? b[12] == 0x86 : (xs(x) & 1);
                b[ip] = v6 ? 0x60 : uint8_t(0x40 | (5 + xs(x) % 11));
                if (len > ip + 3 && !v6) { const size_t tl = len - ip - xs(x) % 3; b[ip + 2] = uint8_t(tl >> 8); b[ip + 3] = uint8_t(tl); }
                if (len > ip + 6 && v6) { const size_t pl = len - ip - 40 - xs(x) % 3; b[ip + 4] = uint8_t(pl >> 8); b[ip + 5] = uint8_t(pl); }
                if (len > ip + 9) {
                    static const uint8_t protos[] = {1, 2, 6, 17, 58, 0};
                    b[v6 ? ip + 6 : ip + 9] = protos[xs(x) % 6];
                    if (!v6) { b[ip + 6] = 0x40; b[ip + 7] = 0; }
                }
            }
            exercise(b.data(), len, kind);
            ++count;
        }
    } else if (mode == "frag" && argc >= 4) {
        uint32_t x = (uint32_t)std::strtoul(argv[2], nullptr, 0) | 1u;
        const size_t n = std::strtoull(argv[3], nullptr, 0);
        for (size_t i = 0; i < n; ++i, ++count) exercise_frag(x);
    } else {
        return 2;
    }
    std::printf("ok %zu\n", count);
    return failures ? 1 : 0;
}
