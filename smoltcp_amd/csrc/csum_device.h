// Device-side building blocks of the checksum engine (gfx950 / CDNA4).
//
// Arithmetic background (RFC 1071 and smoltcp's checksum::data, src/wire/ip.rs:773-804):
// data(b) sums native-endian (little-endian) u16 words into a u32 and folds twice, then
// byte-swaps.  For spans shorter than 131075 bytes the u32 never wraps, so data(b) is the unique
// value in [1, 0xffff] congruent to the big-endian word sum mod 0xffff, or 0 iff every byte is 0.
// Any association order therefore gives the reference's bit pattern, and a sum of aligned u16
// words taken from an ODD start address equals data() without the final byte swap (RFC 1071
// §2(B)).  The protocol kernels use exactly that: one v_sad_u16 per dword.  The raw data() kernel
// keeps separate even/odd byte sums (v_sad_u8) so that it is bit-exact even where the reference's
// u32 accumulator wraps (spans > 131074 bytes, release-mode semantics).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/smolcsum.h"
#include "csum_launch.h"

namespace smolcsum {

// propagate_carries, src/wire/ip.rs:767-770.  For any x < 2^32 the result is 0 iff x == 0 and
// otherwise the representative of x mod 0xffff in [1, 0xffff].
__device__ __forceinline__ uint32_t fold32(uint32_t w) {
    uint32_t s = (w >> 16) + (w & 0xffffu);
    return ((s >> 16) + s) & 0xffffu;
}

__device__ __forceinline__ uint32_t bswap16(uint32_t v) { return ((v >> 8) | (v << 8)) & 0xffffu; }

// Keep the bytes j (0..3) of dword w with lo <= j < hi.
__device__ __forceinline__ uint32_t mask_dword(uint32_t w, int lo, int hi) {
    lo = min(max(lo, 0), 4);
    hi = min(max(hi, 0), 4);
    if (hi <= lo) return 0u;
    uint64_t m = ((1ull << (8 * hi)) - 1ull) & ~((1ull << (8 * lo)) - 1ull);
    return w & (uint32_t)m;
}

// Sum of the two little-endian u16 halves of w, added to acc (one v_sad_u16).
__device__ __forceinline__ uint32_t add_words(uint32_t w, uint32_t acc) {
    return __builtin_amdgcn_sad_u16(w, 0u, acc);
}

// Sum of bytes 0 and 2 (even addresses of a 4-aligned dword) / bytes 1 and 3 (odd addresses).
__device__ __forceinline__ uint32_t add_even_bytes(uint32_t w, uint32_t acc) {
    return __builtin_amdgcn_sad_u8(w & 0x00ff00ffu, 0u, acc);
}
__device__ __forceinline__ uint32_t add_odd_bytes(uint32_t w, uint32_t acc) {
    return __builtin_amdgcn_sad_u8(w & 0xff00ff00u, 0u, acc);
}

__device__ __forceinline__ bool caps_rx(uint32_t c) {  // Checksum::rx, src/phy/mod.rs:188-194
    return c == SMOL_CHECKSUM_BOTH || c == SMOL_CHECKSUM_RX;
}
__device__ __forceinline__ bool caps_tx(uint32_t c) {  // Checksum::tx, src/phy/mod.rs:196-203
    return c == SMOL_CHECKSUM_BOTH || c == SMOL_CHECKSUM_TX;
}

enum : uint32_t { P_NONE = 0, P_ICMP4 = 1, P_IGMP = 2, P_TCP = 6, P_UDP = 17, P_ICMP6 = 58, P_NHC_UDP = 0x111 };

// Where the gates of one record look.  Offsets are relative to the record start.
struct Geom {
    uint32_t st;         // SMOL_ST_MALFORMED | SMOL_ST_UNSUPPORTED
    uint32_t fam;        // 0 (no IP header checked), 4, 6
    uint32_t ip_off;     // IP header offset (0, or 14 behind Ethernet)
    uint32_t ip_hl;      // IPv4 header length (IHL*4)
    uint32_t addr_off;   // pseudo-header source address; destination follows contiguously
    uint32_t addr_words; // u16 words of src+dst (4 for IPv4, 16 for IPv6)
    uint32_t proto;      // P_* of the L4 gate reached, P_NONE if none
    uint32_t l4_off;     // L4 buffer offset (the slice the reference wraps in the L4 Packet)
    uint32_t l4_len;     // L4 buffer length
    uint32_t span_end;   // end of the summed L4 span (UDP: l4_off + UDP length field)
    uint32_t fo;         // checksum field offset inside the L4 header (NHC UDP: in the record)
    uint32_t in_off;     // emit: the IPv4 header embedded in an ICMPv4 DstUnreachable /
    uint32_t in_hl;      // TimeExceeded message (record offset, length; 0 = none)
};

// Icmpv6Packet::check_len, src/wire/icmpv6.rs:274-338: the bytes a message of type t needs
// (max(HEADER_END, header_len()), :296 and header_len :397-418), or 0 when check_len rejects the
// type outright (Message::Unknown, and RplControl, whose proto-rpl feature is not in the default
// feature set, Cargo.toml:104-112).
__host__ __device__ __forceinline__ uint32_t icmpv6_min_len(uint32_t t) {
    switch (t) {
        case 0x01: case 0x02: case 0x03: case 0x04:  // DstUnreachable, PktTooBig, TimeExceeded, ParamProblem
        case 0x80: case 0x81:                        // EchoRequest, EchoReply
        case 0x85:                                   // RouterSolicit
        case 0x8f: return 8;                         // MldReport
        case 0x86: return 16;                        // RouterAdvert (RETRANS_TM.end)
        case 0x87: case 0x88: return 24;             // NeighborSolicit / NeighborAdvert (TARGET_ADDR.end)
        case 0x89: return 40;                        // Redirect (DEST_ADDR.end)
        case 0x82: return 28;                        // MldQuery (QUERY_NUM_SRCS.end)
        default: return 0;
    }
}

// Whether the iface drops a received packet on the options of its Hop-by-Hop header, record bytes
// [pos, end) (process_hopbyhop, src/iface/interface/ipv6.rs:282-313):
//   Ipv6HopByHopRepr::parse (ipv6hbh.rs:70-89) fails on an option that fails Ipv6Option::check_len
//   (ipv6option.rs:158-182: a lone non-Pad1 byte, or data past the end) or Repr::parse (:286-320:
//   RouterAlert whose data length is not 2); its Vec holds IPV6_HBH_MAX_OPTIONS = 4 options
//   (build.rs:19), so the 5th option is parsed and then ends the walk;
//   the iface drops on any of those 4 that is not Pad1 / PadN / RouterAlert and whose type's top two
//   bits ask for a discard (Ipv6OptionFailureType, ipv6option.rs:71-77; Rpl 0x63 is Unknown without
//   the proto-rpl feature).
// Receive only: emit never parses the options.  Rare (one leading Hop-by-Hop header): <= 5 options.
template <class RD>
__device__ __forceinline__ bool hbh_options_drop(const RD& rd, uint32_t pos, uint32_t end) {
    for (int i = 0; i < 5 && pos < end; ++i) {
        const uint32_t t = rd(pos);
        if (t == 0) {  // Pad1
            pos += 1;
            continue;
        }
        if (end - pos == 1) return true;
        const uint32_t dl = rd(pos + 1);
        if (end - pos < 2 + dl) return true;
        if (t == 5 && dl != 2) return true;
        if (i < 4 && t != 1 && t != 5 && (t & 0xc0u)) return true;
        pos += 2 + dl;
    }
    return false;
}

// Record geometry: how smoltcp's iface reaches the checksum gates.  Mirrors, check for check,
//   Ethernet  src/iface/interface/ethernet.rs:4-46
//   IPv4      Ipv4Packet::check_len src/wire/ipv4.rs:241-256, version gate :549-551, fragments
//             src/iface/interface/ipv4.rs:110-146
//   IPv6      Ipv6Packet::check_len src/wire/ipv6.rs:400-407, one leading Hop-by-Hop header
//             src/iface/interface/ipv6.rs:205-211,300-303 (Ipv6ExtHeader::check_len,
//             src/wire/ipv6ext_header.rs:55-69; verify: its options, hbh_options_drop), next header
//             dispatch :323-366
//   L4        UdpPacket::check_len udp.rs:57-69, TcpPacket::check_len tcp.rs:155-167 (verify: and the
//             port tests of UdpRepr::parse udp.rs:246-248 / TcpRepr::parse tcp.rs:910-915),
//             Icmpv4Packet::check_len icmpv4.rs:207-214, IgmpPacket::check_len igmp.rs:73-80,
//             Icmpv6Packet::check_len icmpv6.rs:274-338 (verify: the message-type lengths of
//             icmpv6_min_len; emit: the generic len >= 4 — Icmpv6Packet::fill_checksum fills any type).
//   ICMPv4 errors (emit): Icmpv4Repr::emit writes the embedded IPv4 header of DstUnreachable /
//             TimeExceeded with Ipv4Repr::emit under the same caps (icmpv4.rs:520-543), so its header
//             checksum is filled (or zeroed) before the ICMP checksum covers it.
//   6LoWPAN NHC UDP (KIND_NHC_UDP): UdpNhcPacket::check_len nhc.rs:486-500 and the dispatch test of
//             UdpNhcRepr::parse :701-703; the payload follows the inline checksum if any, and on
//             emit always an inline checksum (payload_mut :622-626).
// `rd(o)` returns the record byte at offset o (only called for o < len).
// NHC: the instantiation for the 6LoWPAN entry points (the IP path carries no NHC code).
template <bool NHC = false, class RD>
__device__ __forceinline__ Geom parse_geometry(const RD& rd, uint32_t len, uint32_t kind, bool emit = false) {
    Geom g = {};
    uint32_t ip_off = 0;
    // SMOL_REC_IPHDR_ONLY: a raw socket's frame, the IP header's gate only (src/socket/raw.rs:406-423,
    // src/iface/packet.rs:132-136 on TX; src/iface/interface/ipv4.rs:150-151 on RX)
    const bool hdr_only = (kind & KIND_IPHDR_ONLY) != 0;
    kind &= 0xffu;
    if (NHC && kind == KIND_NHC_UDP) {
        if (len < 1) { g.st = SMOL_ST_MALFORMED; return g; }
        const uint32_t b0 = rd(0);
        const uint32_t ps = (b0 & 3u) == 0 ? 4u : (b0 & 3u) == 3 ? 1u : 3u;  // ports_size :602-611
        const uint32_t cs = (emit || !(b0 & 4u)) ? 2u : 0u;                     // checksum_size :593-599
        if (1 + ps + cs > len || (b0 >> 3) != 0x1eu) { g.st = SMOL_ST_MALFORMED; return g; }
        // verify: destination port 0 (inline in ports modes 0b00 / 0b10) is dropped by UdpRepr::parse
        // of the decompressed header (src/iface/interface/sixlowpan.rs:745-775, udp.rs:246-248)
        if (!emit && ((b0 & 3u) == 0 || (b0 & 3u) == 2)) {
            const uint32_t dp = (b0 & 3u) == 0 ? (rd(3) << 8 | rd(4)) : (rd(2) << 8 | rd(3));
            if (dp == 0) { g.st = SMOL_ST_MALFORMED; return g; }
        }
        g.proto = P_NHC_UDP;
        g.l4_off = 1 + ps + cs;
        g.l4_len = len - g.l4_off;
        g.span_end = len;
        g.fo = 1 + ps;
        g.addr_words = 16;
        return g;
    }
    if (kind == SMOL_KIND_ETH) {
        if (len < 14) { g.st = SMOL_ST_MALFORMED; return g; }
        uint32_t et = (rd(12) << 8) | rd(13);
        if (et != 0x0800u && et != 0x86ddu) { g.st = SMOL_ST_UNSUPPORTED; return g; }
        ip_off = 14;
        if (len < 15) { g.st = SMOL_ST_MALFORMED; return g; }
        uint32_t ver = rd(14) >> 4;
        if ((et == 0x0800u && ver != 4) || (et == 0x86ddu && ver != 6)) {
            g.st = SMOL_ST_MALFORMED;
            return g;
        }
    } else if (kind != SMOL_KIND_IP) {
        g.st = SMOL_ST_UNSUPPORTED;
        return g;
    }
    const uint32_t lb = len - ip_off;
    if (lb < 1) { g.st = SMOL_ST_MALFORMED; return g; }
    const uint32_t b0 = rd(ip_off);
    const uint32_t version = b0 >> 4;
    if (version == 4) {
        if (lb < 20) { g.st = SMOL_ST_MALFORMED; return g; }
        const uint32_t hl = (b0 & 0x0fu) * 4;
        const uint32_t total = (rd(ip_off + 2) << 8) | rd(ip_off + 3);
        if (lb < hl || hl > total || lb < total || hl < 20) { g.st = SMOL_ST_MALFORMED; return g; }
        g.fam = 4;
        g.ip_off = ip_off;
        g.ip_hl = hl;
        g.addr_off = ip_off + 12;
        g.addr_words = 4;
        if (hdr_only) { g.st = SMOL_ST_UNSUPPORTED; return g; }
        const uint32_t b6 = rd(ip_off + 6);
        const uint32_t frag = ((b6 & 0x1fu) << 8) | rd(ip_off + 7);
        if ((b6 & 0x20u) || frag) { g.st = SMOL_ST_UNSUPPORTED; return g; }
        g.l4_off = ip_off + hl;
        g.l4_len = total - hl;
        const uint32_t p = rd(ip_off + 9);
        if (p != P_UDP && p != P_TCP && p != P_ICMP4 && p != P_IGMP) {
            g.st = SMOL_ST_UNSUPPORTED;
            return g;
        }
        g.proto = p;
    } else if (version == 6) {
        if (lb < 40) { g.st = SMOL_ST_MALFORMED; return g; }
        const uint32_t plen = (rd(ip_off + 4) << 8) | rd(ip_off + 5);
        if (lb < 40 + plen) { g.st = SMOL_ST_MALFORMED; return g; }
        g.fam = 6;
        g.ip_off = ip_off;
        g.addr_off = ip_off + 8;
        g.addr_words = 16;
        if (hdr_only) { g.st = SMOL_ST_UNSUPPORTED; return g; }
        uint32_t cur = ip_off + 40, rem = plen;
        uint32_t nh = rd(ip_off + 6);
        if (nh == 0) {  // Hop-by-Hop
            if (rem < 8) { g.st = SMOL_ST_MALFORMED; return g; }
            const uint32_t hbh = (rd(cur + 1) + 1) * 8;
            if (rem < hbh) { g.st = SMOL_ST_MALFORMED; return g; }
            if (!emit && hbh_options_drop(rd, cur + 2, cur + hbh)) { g.st = SMOL_ST_MALFORMED; return g; }
            nh = rd(cur);
            cur += hbh;
            rem -= hbh;
        }
        g.l4_off = cur;
        g.l4_len = rem;
        if (nh != P_UDP && nh != P_TCP && nh != P_ICMP6) { g.st = SMOL_ST_UNSUPPORTED; return g; }
        g.proto = nh;
    } else {
        g.st = SMOL_ST_MALFORMED;  // IpVersion::of_packet fails: dropped
        return g;
    }
    const uint32_t l4 = g.l4_off;
    switch (g.proto) {
        case P_UDP: {
            g.fo = 6;
            if (g.l4_len < 8) { g.st = SMOL_ST_MALFORMED; break; }
            const uint32_t ul = (rd(l4 + 4) << 8) | rd(l4 + 5);
            if (g.l4_len < ul || ul < 8) { g.st = SMOL_ST_MALFORMED; break; }
            g.span_end = l4 + ul;
            // UdpRepr::parse rejects destination port 0 before its checksum gate (udp.rs:246-248)
            if (!emit && (rd(l4 + 2) | rd(l4 + 3)) == 0) g.st = SMOL_ST_MALFORMED;
            break;
        }
        case P_TCP: {
            g.fo = 16;
            if (g.l4_len < 20) { g.st = SMOL_ST_MALFORMED; break; }
            const uint32_t thl = (rd(l4 + 12) >> 4) * 4;
            if (g.l4_len < thl || thl < 20) { g.st = SMOL_ST_MALFORMED; break; }
            g.span_end = l4 + g.l4_len;
            // TcpRepr::parse rejects source or destination port 0 first (tcp.rs:910-915)
            if (!emit && ((rd(l4) | rd(l4 + 1)) == 0 || (rd(l4 + 2) | rd(l4 + 3)) == 0)) g.st = SMOL_ST_MALFORMED;
            break;
        }
        case P_ICMP4:
        case P_IGMP:
            g.fo = 2;
            if (g.l4_len < 8) { g.st = SMOL_ST_MALFORMED; break; }
            g.span_end = l4 + g.l4_len;
            if (emit && g.proto == P_ICMP4) {
                const uint32_t t = rd(l4);
                if ((t == 3 || t == 11) && g.l4_len >= 28 && (rd(l4 + 8) >> 4) == 4) {
                    const uint32_t ihl = (rd(l4 + 8) & 0x0fu) * 4;  // Ipv4Packet::header_len, as fill_checksum
                    if (ihl >= 20 && 8 + ihl <= g.l4_len) {
                        g.in_off = l4 + 8;
                        g.in_hl = ihl;
                    }
                }
            }
            break;
        default: {  // P_ICMP6
            g.fo = 2;
            const uint32_t need = (emit || g.l4_len < 4) ? 4u : icmpv6_min_len(rd(l4));
            if (need == 0 || g.l4_len < need) { g.st = SMOL_ST_MALFORMED; break; }
            g.span_end = l4 + g.l4_len;
            break;
        }
    }
    return g;
}

}  // namespace smolcsum
