// loopback_ring — the C1 analogue: smoltcp's examples/loopback_benchmark.rs
// moves TCP segments through a Loopback device; with checksums on, every segment is filled on TX
// and verified on RX.  Here the frames are Ethernet + IPv4 + TCP, sized like that benchmark
// (FaultInjector MTU 1536 -> ip_mtu 1522 -> MSS 1482 B of payload; src/phy/fault_injector.rs:18,
// src/phy/mod.rs:282-287), built by the host "stack" into a pinned ring with zero checksum
// fields (the stack runs with ChecksumCapabilities::ignored(), src/phy/mod.rs:223-233), then
//
//   GPU offload: OffloadRing::emit (H2D -> smol_csum_batch_emit -> D2H), loop the ring back,
//                OffloadRing::verify (H2D -> smol_csum_batch_verify -> status D2H);
//   CPU inline:  the same fill + verify per frame with the scalar mirrors on one host thread
//                (what smoltcp does in Ipv4Repr/TcpRepr::emit and ::parse with caps = Both).
//
//   loopback_ring [frames] [reps] [dump-prefix]      prints one JSON line
//
// With a dump prefix, every 97th frame of the last GPU pass is written out as built (zero checksum
// fields: PREFIX.before), after OffloadRing::emit (PREFIX.after) and its verify status byte
// (PREFIX.status), so that a test can compare them with the oracle byte for byte.
//
// Rates are frame bytes per second through the checksum stage (frame building excluded).
#include <chrono>
#include <cstdio>
#include <string>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../smoltcp_amd/host/offload_ring.hpp"

namespace ck = smoltcp::wire::checksum;
using Clock = std::chrono::steady_clock;

static constexpr uint32_t kFrame = 1536, kEth = 14, kMss = kFrame - kEth - 40;

static void build_frame(uint8_t* f, uint32_t seq, const uint8_t* payload) {
    std::memset(f, 0, kEth + 40);
    const uint8_t mac_a[6] = {2, 0, 0, 0, 0, 1}, mac_b[6] = {2, 0, 0, 0, 0, 2};
    std::memcpy(f, mac_b, 6);
    std::memcpy(f + 6, mac_a, 6);
    f[12] = 0x08, f[13] = 0x00;
    uint8_t* ip = f + kEth;
    const uint32_t tot = 40 + kMss;
    ip[0] = 0x45, ip[2] = uint8_t(tot >> 8), ip[3] = uint8_t(tot), ip[8] = 64, ip[9] = 6;
    const uint8_t a[4] = {127, 0, 0, 1};
    std::memcpy(ip + 12, a, 4);
    std::memcpy(ip + 16, a, 4);
    uint8_t* t = ip + 20;
    t[0] = 0x04, t[1] = 0xd2, t[2] = 0x04, t[3] = 0xd3;  // 1234 -> 1235
    t[4] = uint8_t(seq >> 24), t[5] = uint8_t(seq >> 16), t[6] = uint8_t(seq >> 8), t[7] = uint8_t(seq);
    t[12] = 5 << 4, t[13] = 0x10, t[14] = 0xff, t[15] = 0xff;
    std::memcpy(t + 20, payload, kMss);  // TcpRepr::emit copies the payload (tcp.rs:1087)
}

// Ipv4Repr::emit + TcpRepr::emit checksum fill (ipv4.rs:506-513, tcp.rs:616-626), host mirrors.
static void cpu_fill(uint8_t* f) {
    uint8_t* ip = f + kEth;
    ip[10] = ip[11] = 0;
    uint16_t c = uint16_t(~ck::data({ip, 20}));
    ip[10] = uint8_t(c >> 8), ip[11] = uint8_t(c);
    uint8_t* t = ip + 20;
    const uint32_t len = 20 + kMss;
    t[16] = t[17] = 0;
    uint16_t w[2] = {ck::pseudo_header({ip + 12, 4}, {ip + 16, 4}, 6, len), ck::data({t, len})};
    c = uint16_t(~ck::combine(w));
    t[16] = uint8_t(c >> 8), t[17] = uint8_t(c);
}

// Ipv4Repr::parse + TcpRepr::parse checksum gates (ipv4.rs:553, tcp.rs:917-919).
static bool cpu_verify(const uint8_t* f) {
    const uint8_t* ip = f + kEth;
    if (ck::data({ip, 20}) != 0xffff) return false;
    const uint8_t* t = ip + 20;
    const uint32_t len = 20 + kMss;
    uint16_t w[2] = {ck::pseudo_header({ip + 12, 4}, {ip + 16, 4}, 6, len), ck::data({t, len})};
    return ck::combine(w) == 0xffff;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? uint32_t(std::atoi(argv[1])) : (1u << 18);
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    std::vector<uint8_t> sockbuf(size_t(kMss) * 64);
    for (size_t i = 0; i < sockbuf.size(); ++i) sockbuf[i] = uint8_t(i * 2654435761u >> 24);
    try {
        smoltcp_amd::OffloadRing ring(0, n, kFrame, smoltcp_amd::Medium::Ethernet);
        auto build_all = [&] {
            for (uint32_t i = 0; i < n; ++i) build_frame(ring.slot(i), i * kMss, sockbuf.data() + (i % 64) * kMss);
        };
        const double bytes = double(n) * kFrame;
        // ---- GPU offload
        build_all();
        ring.emit(n);  // warm-up (also JIT-free first launch)
        ring.verify(n);
        double t_emit = 0, t_verify = 0;
        uint64_t accepted = 0;
        for (int r = 0; r < reps; ++r) {
            build_all();
            auto t0 = Clock::now();
            ring.emit(n);
            auto t1 = Clock::now();
            ring.verify(n);  // the TX ring looped back as the RX ring
            auto t2 = Clock::now();
            t_emit += std::chrono::duration<double>(t1 - t0).count();
            t_verify += std::chrono::duration<double>(t2 - t1).count();
        }
        for (uint32_t i = 0; i < n; ++i) accepted += smoltcp_amd::accepted(ring.status()[i]);
        if (argc > 3) {  // the sample the oracle checks: frames as built, as emitted, their status
            const std::string pre = argv[3];
            FILE* fb = std::fopen((pre + ".before").c_str(), "wb");
            FILE* fa = std::fopen((pre + ".after").c_str(), "wb");
            FILE* fs = std::fopen((pre + ".status").c_str(), "wb");
            if (!fb || !fa || !fs) throw std::runtime_error("cannot write the dump files");
            std::vector<uint8_t> f(kFrame);
            for (uint32_t i = 0; i < n; i += 97) {
                std::memset(f.data(), 0, kFrame);
                build_frame(f.data(), i * kMss, sockbuf.data() + (i % 64) * kMss);
                std::fwrite(f.data(), 1, kFrame, fb);
                std::fwrite(ring.slot(i), 1, kFrame, fa);
                std::fwrite(ring.status() + i, 1, 1, fs);
            }
            std::fclose(fb);
            std::fclose(fa);
            std::fclose(fs);
        }
        uint64_t cross = 0;  // the host gates agree with the GPU on the emitted frames
        for (uint32_t i = 0; i < n; i += 97) cross += cpu_verify(ring.slot(i));
        // ---- CPU inline (1 thread, scalar mirrors)
        double c_emit = 0, c_verify = 0;
        uint64_t c_acc = 0;
        const int creps = reps < 2 ? reps : 2;
        for (int r = 0; r < creps; ++r) {
            build_all();
            auto t0 = Clock::now();
            for (uint32_t i = 0; i < n; ++i) cpu_fill(ring.slot(i));
            auto t1 = Clock::now();
            c_acc = 0;
            for (uint32_t i = 0; i < n; ++i) c_acc += cpu_verify(ring.slot(i));
            auto t2 = Clock::now();
            c_emit += std::chrono::duration<double>(t1 - t0).count();
            c_verify += std::chrono::duration<double>(t2 - t1).count();
        }
        std::printf(
            "{\"workload\": \"C1 analogue: %u Ethernet+IPv4+TCP frames of %u B (MSS %u) in a pinned loopback ring\", "
            "\"frames\": %u, \"frame_bytes\": %u, "
            "\"gpu_offload\": {\"emit_GBs\": %.2f, \"verify_GBs\": %.2f, \"roundtrip_GBs\": %.2f, \"accepted\": %llu, "
            "\"host_gate_sample_accepted\": %llu, \"host_gate_sample\": %u}, "
            "\"cpu_inline_1thread\": {\"emit_GBs\": %.2f, \"verify_GBs\": %.2f, \"roundtrip_GBs\": %.2f, \"accepted\": %llu}}\n",
            n, kFrame, kMss, n, kFrame, bytes * reps / t_emit / 1e9, bytes * reps / t_verify / 1e9,
            bytes * reps / (t_emit + t_verify) / 1e9, (unsigned long long)accepted, (unsigned long long)cross,
            (n + 96) / 97, bytes * creps / c_emit / 1e9, bytes * creps / c_verify / 1e9,
            bytes * creps / (c_emit + c_verify) / 1e9, (unsigned long long)c_acc);
        return accepted == n && c_acc == n && cross == (n + 96) / 97 ? 0 : 1;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "loopback_ring: %s\n", e.what());
        return 1;
    }
}
