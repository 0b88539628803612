// C++ host-mirror test (smoltcp_amd/host/smoltcp_checksum.hpp), driven by tests/test_host_cpp.py.
//
//   test_host_mirror vectors <file>   scalar mirrors vs expected values computed by the oracle
//   test_host_mirror nodev            Engine() must throw SMOL_ENODEV without a GPU (no fallback)
//   test_host_mirror offload <n>      GPU: an offloading device's TX/RX path over n frames —
//                                     host frames -> HBM -> Engine::emit -> host, checked with the
//                                     scalar mirrors; then corrupt every 7th frame and compare
//                                     Engine::verify's verdicts with the scalar gates.
// Exit status 0 on success; failures print a line and exit 1.
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../smoltcp_amd/host/offload_ring.hpp"
#include "../../smoltcp_amd/host/smoltcp_checksum.hpp"

namespace ck = smoltcp::wire::checksum;
using smoltcp::phy::ChecksumCapabilities;

static int failures = 0;
#define EXPECT(c, ...)                                  \
    do {                                                \
        if (!(c)) {                                     \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);          \
            std::fprintf(stderr, "\n");                 \
            ++failures;                                 \
        }                                               \
    } while (0)

static std::vector<uint8_t> unhex(const std::string& h) {
    std::vector<uint8_t> v;
    if (h == "-") return v;
    for (size_t i = 0; i + 1 < h.size(); i += 2) v.push_back(uint8_t(std::stoul(h.substr(i, 2), nullptr, 16)));
    return v;
}

// Lines: "data <hex> <expect>" | "ph <srchex> <dsthex> <nh> <len> <expect>" | "comb <expect> <w>..."
static int run_vectors(const char* path) {
    std::ifstream f(path);
    std::string line;
    int n = 0;
    while (std::getline(f, line)) {
        std::istringstream is(line);
        std::string op;
        is >> op;
        if (op == "data") {
            std::string h;
            unsigned want;
            is >> h >> want;
            auto b = unhex(h);
            EXPECT(ck::data(b) == want, "data(len %zu) = %u, want %u", b.size(), ck::data(b), want);
        } else if (op == "ph") {
            std::string s, d;
            unsigned nh, want;
            unsigned long len;
            is >> s >> d >> nh >> len >> want;
            auto sb = unhex(s), db = unhex(d);
            if (want == 0x10000) {  // family mismatch: must throw (the reference panics)
                bool threw = false;
                try {
                    ck::pseudo_header(sb, db, uint8_t(nh), uint32_t(len));
                } catch (const smoltcp_amd::Error& e) {
                    threw = e.code() == SMOL_EINVAL;
                }
                EXPECT(threw, "pseudo_header family mismatch did not throw");
            } else {
                uint16_t got = ck::pseudo_header(sb, db, uint8_t(nh), uint32_t(len));
                EXPECT(got == want, "pseudo_header = %u, want %u", got, want);
                if (sb.size() == 4) {
                    uint8_t s4[4], d4[4];
                    std::copy(sb.begin(), sb.end(), s4);
                    std::copy(db.begin(), db.end(), d4);
                    EXPECT(ck::pseudo_header_v4(s4, d4, uint8_t(nh), uint32_t(len)) == want, "pseudo_header_v4");
                } else {
                    uint8_t s6[16], d6[16];
                    std::copy(sb.begin(), sb.end(), s6);
                    std::copy(db.begin(), db.end(), d6);
                    EXPECT(ck::pseudo_header_v6(s6, d6, uint8_t(nh), uint32_t(len)) == want, "pseudo_header_v6");
                }
            }
        } else if (op == "comb") {
            unsigned want, w;
            std::vector<uint16_t> ws;
            is >> want;
            while (is >> w) ws.push_back(uint16_t(w));
            EXPECT(ck::combine(ws) == want, "combine(%zu words) = %u, want %u", ws.size(), ck::combine(ws), want);
        } else {
            continue;
        }
        ++n;
    }
    // phy policy mirror (src/phy/mod.rs:188-233)
    using smoltcp::phy::Checksum;
    EXPECT(smoltcp::phy::rx(Checksum::Both) && smoltcp::phy::tx(Checksum::Both), "Both");
    EXPECT(smoltcp::phy::rx(Checksum::Rx) && !smoltcp::phy::tx(Checksum::Rx), "Rx");
    EXPECT(!smoltcp::phy::rx(Checksum::Tx) && smoltcp::phy::tx(Checksum::Tx), "Tx");
    EXPECT(!smoltcp::phy::rx(Checksum::None) && !smoltcp::phy::tx(Checksum::None), "None");
    auto ig = ChecksumCapabilities::ignored().c();
    EXPECT(ig.ipv4 == 3 && ig.udp == 3 && ig.tcp == 3 && ig.icmpv4 == 3 && ig.icmpv6 == 3, "ignored()");
    auto df = ChecksumCapabilities{}.c();
    EXPECT(df.ipv4 == 0 && df.icmpv6 == 0, "default caps");
    std::printf("vectors %d\n", n);
    return n > 0 ? 0 : 1;
}

static int run_nodev() {
    try {
        smoltcp_amd::Engine e(0);
    } catch (const smoltcp_amd::Error& e) {
        if (e.code() == SMOL_ENODEV) {
            std::printf("nodev ok\n");
            return 0;
        }
        std::fprintf(stderr, "unexpected error %d\n", e.code());
        return 1;
    }
    std::fprintf(stderr, "Engine created without a device\n");
    return 1;
}

// ---- a tiny IPv4 frame builder (header checksum and L4 checksum fields left 0) --------------
static std::vector<uint8_t> frame(uint32_t i, uint32_t stride) {
    uint32_t pay = 16 + (i * 131u) % (stride - 60);
    bool udp = i % 2;
    uint32_t l4 = (udp ? 8 : 20) + pay;
    uint32_t tot = 20 + l4;
    std::vector<uint8_t> b(tot, 0);
    b[0] = 0x45;
    b[2] = uint8_t(tot >> 8), b[3] = uint8_t(tot);
    b[8] = 64;
    b[9] = udp ? 17 : 6;
    const uint8_t src[4] = {10, 0, uint8_t(i >> 8), uint8_t(i)}, dst[4] = {10, 1, 2, 3};
    std::copy(src, src + 4, b.begin() + 12);
    std::copy(dst, dst + 4, b.begin() + 16);
    uint8_t* p = b.data() + 20;
    p[0] = 0x30, p[1] = 0x39, p[2] = 0x00, p[3] = 0x35;
    if (udp) {
        p[4] = uint8_t(l4 >> 8), p[5] = uint8_t(l4);
    } else {
        p[12] = 5 << 4;
        p[13] = 0x18;
    }
    uint32_t x = 0x9E3779B9u * (i + 1);
    for (uint32_t k = (udp ? 8 : 20); k < l4; ++k) {
        x ^= x << 13, x ^= x >> 17, x ^= x << 5;
        p[k] = uint8_t(x);
    }
    return b;
}

// The scalar gates a receiving stack applies (Ipv4Packet::verify_checksum, ipv4.rs:363-370;
// Udp/TcpPacket::verify_checksum, udp.rs:125-147 / tcp.rs:388-405), over the host mirrors.
static bool host_accepts(const uint8_t* b) {
    uint32_t tot = uint32_t(b[2]) << 8 | b[3];
    if (ck::data({b, 20}) != 0xffff) return false;
    uint8_t nh = b[9];
    const uint8_t* l4 = b + 20;
    uint32_t len = tot - 20;
    if (nh == 17) {
        if (l4[6] == 0 && l4[7] == 0) return true;  // UDP: no checksum (udp.rs:138-140)
        len = uint32_t(l4[4]) << 8 | l4[5];
    }
    uint16_t w[2] = {ck::pseudo_header({b + 12, 4}, {b + 16, 4}, nh, len), ck::data({l4, len})};
    return ck::combine(w) == 0xffff;
}

#define HIPCHECK(x)                                                          \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));     \
            return 1;                                                        \
        }                                                                    \
    } while (0)

static int run_offload(uint32_t n) {
    const uint32_t stride = 1536;
    std::vector<uint8_t> host(size_t(n) * stride, 0);
    for (uint32_t i = 0; i < n; ++i) {
        auto f = frame(i, stride);
        std::copy(f.begin(), f.end(), host.begin() + size_t(i) * stride);
    }
    uint8_t *d_buf = nullptr, *d_st = nullptr;
    hipStream_t s;
    HIPCHECK(hipMalloc(&d_buf, host.size()));
    HIPCHECK(hipMalloc(&d_st, n));
    HIPCHECK(hipStreamCreate(&s));
    smoltcp_amd::Engine eng(0);
    auto batch = smoltcp_amd::Batch::fixed(n, stride, stride);
    // TX: the device fills every checksum (the stack runs with ChecksumCapabilities::ignored())
    HIPCHECK(hipMemcpyAsync(d_buf, host.data(), host.size(), hipMemcpyHostToDevice, s));
    eng.emit(d_buf, batch, ChecksumCapabilities{}, nullptr, s);
    HIPCHECK(hipMemcpyAsync(host.data(), d_buf, host.size(), hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    uint32_t ok = 0;
    for (uint32_t i = 0; i < n; ++i) ok += host_accepts(host.data() + size_t(i) * stride);
    EXPECT(ok == n, "after emit %u of %u frames pass the host gates", ok, n);
    // RX: corrupt every 7th frame (one payload or header bit), verify on the device
    for (uint32_t i = 0; i < n; i += 7) {
        uint8_t* b = host.data() + size_t(i) * stride;
        uint32_t tot = uint32_t(b[2]) << 8 | b[3];
        b[(i * 977u) % tot] ^= uint8_t(1u << (i % 8));
    }
    std::vector<uint8_t> st(n);
    HIPCHECK(hipMemcpyAsync(d_buf, host.data(), host.size(), hipMemcpyHostToDevice, s));
    eng.verify(d_buf, batch, d_st, ChecksumCapabilities{}, s);
    HIPCHECK(hipMemcpyAsync(st.data(), d_st, n, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    uint32_t mismatch = 0, rejected = 0;
    for (uint32_t i = 0; i < n; ++i) {
        bool dev = smoltcp_amd::accepted(st[i]);
        rejected += !dev;
        mismatch += dev != host_accepts(host.data() + size_t(i) * stride);
    }
    EXPECT(mismatch == 0, "%u device verdicts differ from the host gates", mismatch);
    EXPECT(rejected > 0, "no corrupted frame was rejected");
    HIPCHECK(hipFree(d_buf));
    HIPCHECK(hipFree(d_st));
    HIPCHECK(hipStreamDestroy(s));
    std::printf("offload %u frames: emitted all valid, %u rejected after corruption\n", n, rejected);
    return 0;
}

// Raw-socket frames through OffloadRing (SMOL_REC_IPHDR_ONLY): every 5th slot
// carries a frame whose L4 checksum the user wrote (0xBEEF, wrong on purpose), marked raw.  After
// emit, raw frames keep their L4 bytes and get a valid IPv4 header; the others pass the host gates.
// Verify then accepts the raw frames on their IPv4 gate alone (status UNSUPPORTED: no L4 checksum
// on their path) and checks the others fully.  Chunks of 1000 slots: some hold no raw frame
// (fixed-stride batches), the others go through descriptors.
static int run_raw(uint32_t n) {
    const uint32_t stride = 1536;
    smoltcp_amd::OffloadRing ring(0, n, stride, smoltcp_amd::Medium::Ip, 1000);
    std::vector<std::vector<uint8_t>> want(n);
    for (uint32_t i = 0; i < n; ++i) {
        auto f = frame(i, stride);
        const bool raw = i % 5 == 0 && (i / 1000) % 3 != 1;  // chunk 1, 4, ...: no raw frame
        if (raw) {
            const uint32_t fo = f[9] == 17 ? 26 : 36;
            f[fo] = 0xBE, f[fo + 1] = 0xEF;
        }
        std::fill(ring.slot(i), ring.slot(i) + stride, 0);
        std::copy(f.begin(), f.end(), ring.slot(i));
        ring.mark_raw(i, raw);
        want[i] = f;
    }
    ring.emit(n);
    uint32_t bad = 0, raws = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* b = ring.slot(i);
        if (i % 5 == 0 && (i / 1000) % 3 != 1) {
            ++raws;
            const bool l4_same = std::equal(want[i].begin() + 20, want[i].end(), b + 20);
            bad += !(l4_same && ck::data({b, 20}) == 0xffff);
        } else {
            bad += !host_accepts(b);
        }
    }
    EXPECT(bad == 0, "%u frames wrong after emit", bad);
    ring.verify(n);
    uint32_t vbad = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t st = ring.status()[i];
        if (i % 5 == 0 && (i / 1000) % 3 != 1) vbad += !(smoltcp_amd::accepted(st) && (st & SMOL_ST_UNSUPPORTED));
        else vbad += smoltcp_amd::accepted(st) != host_accepts(ring.slot(i));
    }
    EXPECT(vbad == 0, "%u verify statuses wrong", vbad);
    std::printf("raw %u frames (%u raw): emit kept the user's L4 bytes, verify gated their IPv4 header only\n", n, raws);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    std::string mode = argv[1];
    int rc = 2;
    try {
        if (mode == "vectors" && argc > 2) rc = run_vectors(argv[2]);
        else if (mode == "nodev") rc = run_nodev();
        else if (mode == "offload") rc = run_offload(argc > 2 ? uint32_t(std::atoi(argv[2])) : 10000);
        else if (mode == "raw") rc = run_raw(argc > 2 ? uint32_t(std::atoi(argv[2])) : 10000);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 1;
    }
    return failures ? 1 : rc;
}
