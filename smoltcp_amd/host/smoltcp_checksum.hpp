// smoltcp_checksum.hpp — C++ host-side mirror of the reference interface over the C ABI.
//
// The reference is Rust and this image has no Rust toolchain, so the host side above the C ABI
// (include/smolcsum.h) is this header: the same names, argument meanings and error behaviour as
//
//   smoltcp::wire::checksum::{data, combine, pseudo_header_v4, pseudo_header_v6, pseudo_header}
//                                                            (src/wire/ip.rs:762-869)
//   smoltcp::phy::{Checksum, ChecksumCapabilities}           (src/phy/mod.rs:173-234)
//
// plus the batched engine (`smoltcp_amd::Engine`, one device context) that a checksum-offloading
// `phy::Device` drives: `emit` for TxToken::consume, `verify` before an RxToken is handed out.
// Errors become `smoltcp_amd::Error` exceptions here, on the C++ side; none crosses the C ABI.
// `pseudo_header` throws where the reference panics (`unreachable!()`, ip.rs:866).
//
// Header-only; link with -lsmolcsum (smoltcp_amd/libsmolcsum.so).  Device pointers are plain
// `hipMalloc` pointers and streams are `hipStream_t` passed as `void*`, so this header needs no
// HIP include.
#pragma once

#include <cstddef>
#include <cstdint>
#include <span>
#include <stdexcept>
#include <string>

#include "../../include/smolcsum.h"

namespace smoltcp_amd {

class Error : public std::runtime_error {
public:
    Error(int code, const std::string& what) : std::runtime_error(what), code_(code) {}
    int code() const noexcept { return code_; }

private:
    int code_;
};

inline void check(int rc, const char* what) {
    if (rc == SMOL_OK) return;
    std::string msg = std::string(what) + " failed (" + std::to_string(rc) + ")";
    if (rc == SMOL_EHIP) msg += ": " + std::string(smol_csum_last_error());
    throw Error(rc, msg);
}

}  // namespace smoltcp_amd

namespace smoltcp {

// ---- wire::checksum (src/wire/ip.rs:762-869) --------------------------------------------------
namespace wire::checksum {

// checksum::data (ip.rs:773-804)
inline uint16_t data(std::span<const uint8_t> bytes) { return smol_csum_data(bytes.data(), bytes.size()); }

// checksum::combine (ip.rs:807-813)
inline uint16_t combine(std::span<const uint16_t> checksums) {
    return smol_csum_combine(checksums.data(), checksums.size());
}

// checksum::pseudo_header_v4 (ip.rs:816-831)
inline uint16_t pseudo_header_v4(const uint8_t (&src)[4], const uint8_t (&dst)[4], uint8_t next_header,
                                 uint32_t length) {
    return smol_csum_pseudo_header_v4(src, dst, next_header, length);
}

// checksum::pseudo_header_v6 (ip.rs:834-849)
inline uint16_t pseudo_header_v6(const uint8_t (&src)[16], const uint8_t (&dst)[16], uint8_t next_header,
                                 uint32_t length) {
    return smol_csum_pseudo_header_v6(src, dst, next_header, length);
}

// checksum::pseudo_header (ip.rs:851-869): an address is 4 (IPv4) or 16 (IPv6) bytes.
inline uint16_t pseudo_header(std::span<const uint8_t> src, std::span<const uint8_t> dst, uint8_t next_header,
                              uint32_t length) {
    auto fam = [](size_t n) { return n == 4 ? 4 : n == 16 ? 6 : 0; };
    uint16_t out = 0;
    int rc = smol_csum_pseudo_header(fam(src.size()), src.data(), fam(dst.size()), dst.data(), next_header,
                                     length, &out);
    if (rc == SMOL_EINVAL) throw smoltcp_amd::Error(rc, "pseudo_header: address family mismatch");
    smoltcp_amd::check(rc, "smol_csum_pseudo_header");
    return out;
}

// checksum::format_checksum (ip.rs:871-886): the annotation the packet pretty-printers append.
inline const char* format_checksum(bool correct, bool partially_correct) {
    if (correct) return "";
    return partially_correct ? " (partial checksum correct)" : " (checksum incorrect)";
}

// The annotations of one verify status byte (SMOL_ST_*): the IPv4 header line
// (Ipv4Packet pretty_print, ipv4.rs:698: format_checksum(verify_checksum(), false)) and the
// UDP / TCP line (pretty_print_ip_payload, ip.rs:930-962: verify_checksum() and
// verify_partial_checksum()).
inline const char* ipv4_annotation(uint8_t status) { return format_checksum(status & SMOL_ST_IP_VALID, false); }
inline const char* l4_annotation(uint8_t status) {
    return format_checksum(status & SMOL_ST_L4_VALID, status & SMOL_ST_L4_PARTIAL);
}

}  // namespace wire::checksum

// ---- phy::Checksum / phy::ChecksumCapabilities (src/phy/mod.rs:173-234) -------------------------
namespace phy {

enum class Checksum : uint8_t {
    Both = SMOL_CHECKSUM_BOTH,  // the default (mod.rs:178)
    Rx = SMOL_CHECKSUM_RX,
    Tx = SMOL_CHECKSUM_TX,
    None = SMOL_CHECKSUM_NONE,
};

// Checksum::rx / Checksum::tx (mod.rs:188-203)
constexpr bool rx(Checksum c) { return c == Checksum::Both || c == Checksum::Rx; }
constexpr bool tx(Checksum c) { return c == Checksum::Both || c == Checksum::Tx; }

struct ChecksumCapabilities {
    Checksum ipv4 = Checksum::Both;
    Checksum udp = Checksum::Both;
    Checksum tcp = Checksum::Both;
    Checksum icmpv4 = Checksum::Both;
    Checksum icmpv6 = Checksum::Both;

    // ChecksumCapabilities::ignored (mod.rs:223-233): the device does all checksum work.
    static constexpr ChecksumCapabilities ignored() {
        return {Checksum::None, Checksum::None, Checksum::None, Checksum::None, Checksum::None};
    }

    smol_checksum_caps_t c() const {
        smol_checksum_caps_t r{};
        r.ipv4 = uint8_t(ipv4);
        r.udp = uint8_t(udp);
        r.tcp = uint8_t(tcp);
        r.icmpv4 = uint8_t(icmpv4);
        r.icmpv6 = uint8_t(icmpv6);
        return r;
    }
};

}  // namespace phy
}  // namespace smoltcp

namespace smoltcp_amd {

enum class Medium : uint8_t { Raw = SMOL_KIND_RAW, Ip = SMOL_KIND_IP, Ethernet = SMOL_KIND_ETH };

// Record geometry of one batch: a fixed stride, or a device array of descriptors.
struct Batch {
    const smol_csum_desc_t* d_desc = nullptr;
    uint64_t n = 0;
    uint64_t stride = 0;
    uint32_t len = 0;
    Medium kind = Medium::Ip;
    uint8_t flags = 0;  // SMOL_REC_* of every record (fixed stride; descriptors carry their own)

    static Batch fixed(uint64_t n, uint64_t stride, uint32_t len, Medium kind = Medium::Ip, uint8_t flags = 0) {
        return Batch{nullptr, n, stride, len, kind, flags};
    }
    static Batch described(const smol_csum_desc_t* d_desc, uint64_t n) { return Batch{d_desc, n, 0, 0, Medium::Ip, 0}; }

    smol_csum_batch_t c() const {
        smol_csum_batch_t b{};
        b.desc = d_desc;
        b.n = n;
        b.stride = stride;
        b.len = len;
        b.kind = uint8_t(kind);
        b.flags = flags;
        return b;
    }
};

// One device context (not thread-safe: one Engine per host thread).  Every call is asynchronous
// on `stream`; buffers are device pointers owned by the caller.
class Engine {
public:
    explicit Engine(int device = 0) { check(smol_csum_ctx_create(device, &ctx_), "smol_csum_ctx_create"); }
    ~Engine() {
        if (ctx_) smol_csum_ctx_destroy(ctx_);
    }
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;
    Engine(Engine&& o) noexcept : ctx_(o.ctx_) { o.ctx_ = nullptr; }

    // Repr::emit checksum gates, in place (d_status nullable: MALFORMED / UNSUPPORTED bits).
    void emit(uint8_t* d_buf, const Batch& b, const smoltcp::phy::ChecksumCapabilities& caps = {},
              uint8_t* d_status = nullptr, void* stream = nullptr) {
        auto bc = b.c();
        auto cc = caps.c();
        check(smol_csum_batch_emit(ctx_, d_buf, &bc, &cc, d_status, stream), "smol_csum_batch_emit");
    }

    // TcpRepr/UdpRepr::emit's "copy the payload, then fill": d_copy[i] moves record i's payload
    // from d_src into the record, then the checksums are emitted, in one pass.
    void copy_emit(uint8_t* d_buf, const Batch& b, const uint8_t* d_src, const smol_csum_copy_t* d_copy,
                   const smoltcp::phy::ChecksumCapabilities& caps = {}, uint8_t* d_status = nullptr,
                   void* stream = nullptr) {
        auto bc = b.c();
        auto cc = caps.c();
        check(smol_csum_batch_copy_emit(ctx_, d_buf, &bc, d_src, d_copy, &cc, d_status, stream),
              "smol_csum_batch_copy_emit");
    }

    // Repr::parse checksum gates: d_status[i] = SMOL_ST_* bits.
    void verify(const uint8_t* d_buf, const Batch& b, uint8_t* d_status,
                const smoltcp::phy::ChecksumCapabilities& caps = {}, void* stream = nullptr) {
        auto bc = b.c();
        auto cc = caps.c();
        check(smol_csum_batch_verify(ctx_, d_buf, &bc, &cc, d_status, stream), "smol_csum_batch_verify");
    }

    // IPv4 fragment groups: d_groups[k] = one datagram's fragments (consecutive records).  Fills every
    // fragment header and each datagram's L4 checksum over its reassembled payload (the iface's
    // "emit whole, then fragment", src/iface/interface/mod.rs:1276-1331).
    void emit_frag(uint8_t* d_buf, const Batch& b, const smol_csum_frag_group_t* d_groups, uint64_t n_groups,
                   const smoltcp::phy::ChecksumCapabilities& caps = {}, uint8_t* d_status = nullptr,
                   void* stream = nullptr) {
        auto bc = b.c();
        auto cc = caps.c();
        check(smol_csum_batch_emit_frag(ctx_, d_buf, &bc, d_groups, n_groups, &cc, d_status, stream),
              "smol_csum_batch_emit_frag");
    }
    // Fragment headers + the reassembled datagram's L4 gate (src/iface/interface/ipv4.rs:103-146).
    void verify_frag(const uint8_t* d_buf, const Batch& b, const smol_csum_frag_group_t* d_groups,
                     uint64_t n_groups, uint8_t* d_status, const smoltcp::phy::ChecksumCapabilities& caps = {},
                     void* stream = nullptr) {
        auto bc = b.c();
        auto cc = caps.c();
        check(smol_csum_batch_verify_frag(ctx_, d_buf, &bc, d_groups, n_groups, &cc, d_status, stream),
              "smol_csum_batch_verify_frag");
    }

    // 6LoWPAN NHC UDP (sixlowpan::nhc::UdpNhcRepr::emit / ::parse): every record is a LOWPAN_NHC
    // UDP packet; d_addrs[i] holds record i's IPv6 addresses (IPHC-decompressed).
    void nhc_udp_emit(uint8_t* d_buf, const Batch& b, const smol_ipv6_addr_pair_t* d_addrs,
                      const smoltcp::phy::ChecksumCapabilities& caps = {}, uint8_t* d_status = nullptr,
                      void* stream = nullptr) {
        auto bc = b.c();
        auto cc = caps.c();
        check(smol_csum_batch_nhc_udp_emit(ctx_, d_buf, &bc, d_addrs, &cc, d_status, stream),
              "smol_csum_batch_nhc_udp_emit");
    }
    void nhc_udp_verify(const uint8_t* d_buf, const Batch& b, const smol_ipv6_addr_pair_t* d_addrs,
                        uint8_t* d_status, const smoltcp::phy::ChecksumCapabilities& caps = {},
                        void* stream = nullptr) {
        auto bc = b.c();
        auto cc = caps.c();
        check(smol_csum_batch_nhc_udp_verify(ctx_, d_buf, &bc, d_addrs, &cc, d_status, stream),
              "smol_csum_batch_nhc_udp_verify");
    }

    // checksum::data over every record span.
    void data(const uint8_t* d_buf, const Batch& b, uint16_t* d_out, void* stream = nullptr) {
        auto bc = b.c();
        check(smol_csum_batch_data(ctx_, d_buf, &bc, d_out, stream), "smol_csum_batch_data");
    }


    smol_csum_ctx_t* handle() const { return ctx_; }

private:
    smol_csum_ctx_t* ctx_ = nullptr;
};

constexpr bool accepted(uint8_t status) { return (status & SMOL_ST_ACCEPT) != 0; }

}  // namespace smoltcp_amd
