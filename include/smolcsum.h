/*
 * smolcsum.h — C ABI of the MI355X (gfx950) Internet-checksum engine.
 *
 * This is the drop-in boundary for the one hot path of smoltcp 0.13.1 that this repository
 * accelerates: the RFC 1071 one's-complement checksum of `smoltcp::wire::checksum` and the
 * per-protocol emit/verify gates built on it.  Every entry point below names the reference
 * interface it replaces (paths relative to the smoltcp source tree).
 *
 * Two groups of entry points:
 *
 *  1. Scalar host mirrors of `smoltcp::wire::checksum` (src/wire/ip.rs:762-869).  Bit-identical
 *     results, same argument meaning, host memory, synchronous.  A Rust `extern "C"` binding
 *      can route `checksum::data` & co. here unchanged.
 *
 *  2. Batched device entry points.  One contiguous DEVICE buffer holds many records (IP packets,
 *     Ethernet frames or raw spans); a record is either described by a descriptor array (device
 *     memory) or implied by a fixed stride.  Each call is asynchronous and stream-ordered on the
 *     HIP stream passed in; the caller owns every buffer.  The engine reads the IP header inside
 *     the record to find the protocol, the L4 span and the pseudo-header addresses, exactly as
 *     smoltcp's iface does before it calls the per-protocol gates:
 *       - smol_csum_batch_emit   == the checksum part of Ipv4Repr/UdpRepr/TcpRepr/Icmpv4Repr/
 *         Icmpv6Repr/IgmpRepr::emit under `caps` (fill when caps.X.tx(), else write 0);
 *       - smol_csum_batch_verify == the checksum gates of the matching Repr::parse under `caps`
 *         (verify when caps.X.rx()), reported as one status byte per record;
 *       - smol_csum_batch_data   == checksum::data() over each raw span.
 *     A device that offloads checksums (phy::Device with ChecksumCapabilities::ignored(),
 *     src/phy/mod.rs:223-233) runs emit in TxToken::consume and verify before yielding an
 *     RxToken, with the stack's default caps (Checksum::Both).
 *
 * Errors: every function returning int returns SMOL_OK (0) or a negative SMOL_E* code.  No C++
 * exception crosses this boundary.  There is no CPU fallback for the batched calls: with no
 * usable HIP device they return SMOL_ENODEV.
 *
 * Threading: a context belongs to one device and one host thread at a time (not thread-safe);
 * use one context per host thread.  Calls on the same stream are ordered.
 */
#ifndef SMOLCSUM_H
#define SMOLCSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMOLCSUM_ABI_VERSION 6

/* ---- error codes ------------------------------------------------------------------------ */
enum {
    SMOL_OK = 0,
    SMOL_EINVAL = -1,  /* bad argument: NULL pointer with n > 0, unknown kind, bad caps value   */
    SMOL_ENODEV = -2,  /* no HIP device, or the device ordinal is out of range                   */
    SMOL_EHIP = -3,    /* a HIP runtime call failed; smol_csum_last_error() gives the message    */
    SMOL_ERANGE = -4,  /* a size limit was exceeded (record longer than SMOL_MAX_RECORD_LEN)     */
    SMOL_ENOMEM = -5   /* host allocation failed                                                 */
};

/* Longest record the batched kernels accept.  Protocol records never exceed 65535 + 14 bytes
 * (u16 length fields); raw data() spans may be up to 1 GiB.  data() stays bit-exact with the
 * reference's release-mode u32 wrap-around for spans longer than 131074 bytes (src/wire/ip.rs:776). */
#define SMOL_MAX_RECORD_LEN (1u << 30)

/* ---- policy: mirrors phy::Checksum / phy::ChecksumCapabilities (src/phy/mod.rs:176-218) --- */
typedef enum {
    SMOL_CHECKSUM_BOTH = 0, /* Checksum::Both (the default, src/phy/mod.rs:178) */
    SMOL_CHECKSUM_RX = 1,   /* Checksum::Rx */
    SMOL_CHECKSUM_TX = 2,   /* Checksum::Tx */
    SMOL_CHECKSUM_NONE = 3  /* Checksum::None */
} smol_checksum_t;

/* Field order and meaning of ChecksumCapabilities {ipv4, udp, tcp, icmpv4, icmpv6}.  Each byte is
 * a smol_checksum_t.  IGMP has no entry in the reference: IgmpRepr::emit always fills
 * (src/wire/igmp.rs:293) and IgmpRepr::parse never verifies (src/wire/igmp.rs:204-248); the
 * batched calls do the same. */
typedef struct {
    uint8_t ipv4;
    uint8_t udp;
    uint8_t tcp;
    uint8_t icmpv4;
    uint8_t icmpv6;
    uint8_t reserved[3]; /* must be 0 */
} smol_checksum_caps_t;

/* ---- record kinds ----------------------------------------------------------------------- */
enum {
    SMOL_KIND_RAW = 0, /* a plain byte span: only smol_csum_batch_data is meaningful            */
    SMOL_KIND_IP = 1,  /* an IPv4 or IPv6 packet (Medium::Ip); version from the first nibble     */
    SMOL_KIND_ETH = 2  /* an Ethernet II frame (Medium::Ethernet) carrying IPv4 (0x0800) or IPv6
                          (0x86DD); other ethertypes are reported SMOL_ST_UNSUPPORTED           */
};

/* One record of a batch (16 bytes, device memory).  `len` is the number of bytes the device
 * buffer holds for this record (the Rx/Tx token buffer length); the IP length fields inside the
 * record decide the spans that are summed, exactly as in the reference. */
typedef struct {
    uint64_t offset; /* byte offset of the record from the batch base pointer (any alignment) */
    uint32_t len;    /* record length in bytes, <= SMOL_MAX_RECORD_LEN                         */
    uint8_t kind;    /* SMOL_KIND_*                                                            */
    uint8_t flags;   /* SMOL_REC_* (0 for an ordinary record); other bits must be 0            */
    uint16_t reserved;
} smol_csum_desc_t;

/* Record flags (smol_csum_desc_t.flags, or smol_csum_batch_t.flags for every record of a
 * fixed-stride batch).
 *
 * SMOL_REC_IPHDR_ONLY — a raw-socket frame.  A raw socket's L4 bytes go out as the user wrote
 * them: dispatch copies IpPayload::Raw verbatim (src/iface/packet.rs:132-136) and only the IPv4
 * header is emitted by the stack (Ipv4Repr::emit under caps.ipv4, src/socket/raw.rs:406-423).  On
 * receive the raw socket sees the packet after the IPv4 header gate and before any L4 gate
 * (src/iface/interface/ipv4.rs:150-151).  So for such a record emit fills (or zeroes) the IPv4
 * header checksum only and never touches a byte past the IP header; verify applies the IPv4
 * header gate only.  The record is reported SMOL_ST_UNSUPPORTED (no L4 checksum on its path), or
 * SMOL_ST_MALFORMED when its IP header fails check_len.  In a fragment group the flag on any of
 * the group's records makes the whole datagram raw. */
#define SMOL_REC_IPHDR_ONLY 0x01u

/* Batch flag (smol_csum_batch_t.flags, fixed-stride and descriptor batches alike; ABI 5).
 *
 * SMOL_BATCH_FIELD_STORES — emit writes the checksum fields only (2-byte stores), never a whole
 * 64-byte segment around them.  By default emit rewrites such segments, neighbouring records'
 * bytes included, with the values it read (smol_csum_batch_emit below): a caller that writes other
 * bytes of the batch's records from another stream while emit runs sets this flag.  Slower (one
 * partial-line write per field). */
#define SMOL_BATCH_FIELD_STORES 0x80u

/* Batch geometry (host memory).  If `desc` is non-NULL it is a DEVICE array of `n` descriptors
 * and `stride`/`len`/`kind` are ignored.  Otherwise record i starts at base + i*stride, has
 * length `len` and kind `kind` (the fixed-size case: no descriptor traffic at all). */
typedef struct {
    const smol_csum_desc_t* desc;
    uint64_t n;
    uint64_t stride;
    uint32_t len;
    uint8_t kind;
    uint8_t flags;       /* SMOL_REC_* for every record of a fixed-stride batch (ignored with desc) */
    uint8_t reserved[2]; /* must be 0 */
} smol_csum_batch_t;

/* ---- per-record status byte (verify; emit reports the MALFORMED/UNSUPPORTED bits) ------- */
enum {
    SMOL_ST_IP_OK = 0x01,      /* IPv4 header gate passed: verified under caps.ipv4.rx(), or not
                                  checked (caps, IPv6, non-IP).  Ipv4Repr::parse, ipv4.rs:553   */
    SMOL_ST_L4_OK = 0x02,      /* L4 gate passed: verified under caps.X.rx(), or not checked
                                  (caps, IGMP, fragment, unsupported protocol)                    */
    SMOL_ST_L4_PARTIAL = 0x04, /* UDP/TCP verify_partial_checksum(): field == pseudo-header sum
                                  (udp.rs:112-119, tcp.rs:376-385)                              */
    SMOL_ST_IP_VALID = 0x08,   /* Ipv4Packet::verify_checksum() regardless of caps (1 if no
                                  IPv4 header)                                                   */
    SMOL_ST_L4_VALID = 0x10,   /* the L4 verify_checksum() regardless of caps (1 if no L4 span)  */
    SMOL_ST_MALFORMED = 0x20,  /* the reference's parse drops the packet before any checksum is
                                  looked at: a check_len() on the path failed, or (verify only) a
                                  port Repr::parse rejects first — UDP destination port 0
                                  (udp.rs:246-248), TCP source or destination port 0
                                  (tcp.rs:910-915) — or (verify only, ABI 6) the iface drops an
                                  IPv6 packet on its Hop-by-Hop options: an option that fails to
                                  parse, or an unknown option whose type asks for a discard
                                  (process_hopbyhop, iface/interface/ipv6.rs:282-313).  The L4 bits
                                  are then not evaluated (set).  Emit never rejects ports or
                                  options: Repr::emit does not check them.                       */
    SMOL_ST_UNSUPPORTED = 0x40,/* no L4 checksum on this record's path: IPv4 fragment, protocol
                                  smoltcp does not checksum, IPv6 next header other than a
                                  leading Hop-by-Hop + TCP/UDP/ICMPv6, non-IP ethertype          */
    SMOL_ST_ACCEPT = 0x80      /* IP_OK && L4_OK && !MALFORMED: the checksum gates pass         */
};

/* ---- 1. scalar host mirrors of smoltcp::wire::checksum ---------------------------------- */

/* checksum::data — src/wire/ip.rs:773-804.  RFC 1071 sum without the final complement. */
uint16_t smol_csum_data(const uint8_t* data, size_t len);

/* checksum::combine — src/wire/ip.rs:807-813. */
uint16_t smol_csum_combine(const uint16_t* checksums, size_t n);

/* checksum::pseudo_header_v4 — src/wire/ip.rs:816-831.  `length` is truncated to u16 as in the
 * reference (NetworkEndian::write_u16(.., length as u16)). */
uint16_t smol_csum_pseudo_header_v4(const uint8_t src_addr[4], const uint8_t dst_addr[4],
                                    uint8_t next_header, uint32_t length);

/* checksum::pseudo_header_v6 — src/wire/ip.rs:834-849. */
uint16_t smol_csum_pseudo_header_v6(const uint8_t src_addr[16], const uint8_t dst_addr[16],
                                    uint8_t next_header, uint32_t length);

/* checksum::pseudo_header — src/wire/ip.rs:851-869.  `family` is 4 or 6 for each address; the
 * reference panics (unreachable!) on a family mismatch; this returns SMOL_EINVAL instead and
 * writes nothing. */
int smol_csum_pseudo_header(int src_family, const uint8_t* src_addr, int dst_family,
                            const uint8_t* dst_addr, uint8_t next_header, uint32_t length,
                            uint16_t* out);

/* ---- 2. batched device engine ----------------------------------------------------------- */

typedef struct smol_csum_ctx smol_csum_ctx_t;

/* Create a context bound to HIP device `device`.  Returns SMOL_ENODEV when no such device. */
int smol_csum_ctx_create(int device, smol_csum_ctx_t** out);
int smol_csum_ctx_destroy(smol_csum_ctx_t* ctx);

/* checksum::data() over every record span; d_out[i] = data(record i) (u16, numeric value as the
 * reference returns it).  Record kinds are ignored: every record is a raw span. */
int smol_csum_batch_data(smol_csum_ctx_t* ctx, const uint8_t* d_buf,
                         const smol_csum_batch_t* batch, uint16_t* d_out, void* stream);

/* In-place emit: for every record write the IPv4 header checksum and the L4 checksum the way the
 * reference's Repr::emit does under `caps` (fill when tx(), else 0; UDP 0 -> 0xffff; IGMP always
 * filled).  An ICMPv4 DstUnreachable / TimeExceeded message's embedded IPv4 header gets its header
 * checksum first, under caps.ipv4, as Icmpv4Repr::emit writes it with Ipv4Repr::emit
 * (src/wire/icmpv4.rs:520-543).  `d_status` (nullable) receives SMOL_ST_MALFORMED /
 * SMOL_ST_UNSUPPORTED per record.  Kernels on `stream` only; records must not overlap.  The kernels
 * write the 64-byte segment around a record's fields whole where that is race-free within the
 * call: the segment's other bytes, which may belong to the records just before and after it in
 * the batch (contiguous with it in memory, no field of theirs in the segment), are written back
 * with the values the kernels read.  Bytes outside the batch's records are never written.  So
 * nothing else may write the batch's records while the call runs, the same rule copy-emit states,
 * unless the batch sets SMOL_BATCH_FIELD_STORES (fields only).  Descriptor batches of records that
 * lie back to back take the staged form (one launch stages each record's field values in the
 * context's scratch, a second one writes the field segments, per 2^21 records): the context owns
 * ~17 MB of device scratch, allocated by smol_csum_ctx_create, and orders a staged emit issued on
 * another stream after the previous one (an event wait), so emits on one context may use several
 * streams.  No device memory is allocated by a batched call: the calls may be captured in a HIP
 * graph (a graph holding a staged emit uses the context's scratch when it replays: do not replay it
 * concurrently with another emit on the same context). */
int smol_csum_batch_emit(smol_csum_ctx_t* ctx, uint8_t* d_buf, const smol_csum_batch_t* batch,
                         const smol_checksum_caps_t* caps, uint8_t* d_status, void* stream);

/* Verify: d_status[i] = SMOL_ST_* bits for record i under `caps` (Repr::parse gates). */
int smol_csum_batch_verify(smol_csum_ctx_t* ctx, const uint8_t* d_buf,
                           const smol_csum_batch_t* batch, const smol_checksum_caps_t* caps,
                           uint8_t* d_status, void* stream);

/* Payload copy of one record for smol_csum_batch_copy_emit (16 bytes, device memory). */
typedef struct {
    uint64_t src_offset; /* payload position in the source buffer (any alignment)          */
    uint32_t dst_offset; /* where the payload goes inside the record                         */
    uint32_t len;        /* payload bytes (0: nothing to copy)                               */
} smol_csum_copy_t;

/* Fused payload copy + emit: the TcpRepr::emit / UdpRepr::emit sequence "copy the payload into
 * the packet, then fill the checksum" (src/wire/tcp.rs:1087-1095, src/wire/udp.rs:300-308) in one
 * pass.  For every record i: copy d_src[copy[i].src_offset ..][.. len] to record bytes
 * [dst_offset, dst_offset + len), then emit exactly as smol_csum_batch_emit does (the headers in
 * front of the payload were already written by the caller).  The payload is read once and
 * written once; nothing is read back.  The result is bit-identical to a memcpy followed by
 * smol_csum_batch_emit, including when the copied range covers a checksum field (the emitted
 * field wins).  A record whose copy range does not fit (dst_offset + len > record length) is
 * left untouched and reported SMOL_ST_MALFORMED.  `d_copy` is a 16-byte-aligned device array of
 * n entries; the source must not overlap the batch buffer, and records must not overlap one another
 * (the kernel rewrites every byte of a record — the bytes outside its copy range with their own
 * values — so that whole cache lines leave L2). */
int smol_csum_batch_copy_emit(smol_csum_ctx_t* ctx, uint8_t* d_buf, const smol_csum_batch_t* batch,
                              const uint8_t* d_src, const smol_csum_copy_t* d_copy,
                              const smol_checksum_caps_t* caps, uint8_t* d_status, void* stream);

/* ---- 3. IPv4 fragment groups ------------------------------------------------------------- */

/* One IPv4 datagram carried by `count` consecutive records of a batch, starting at record
 * `first` (16 bytes, device memory): its fragments, in any order.  A group of one unfragmented
 * packet is allowed.  Groups must not share records.  A group that does not lie inside the batch
 * (first >= n, or count > n - first), whose count is 0 or above SMOL_MAX_FRAGMENTS, or whose
 * reserved word is not 0 is invalid: none of its records is read or written, status included. */
typedef struct {
    uint64_t first;
    uint32_t count;    /* 1 .. SMOL_MAX_FRAGMENTS */
    uint32_t reserved; /* must be 0 */
} smol_csum_frag_group_t;

/* Fragments per group the kernels accept (smoltcp's default fragmentation and reassembly buffers
 * hold 1500 bytes, gen_config.py; 256 fragments of 8 bytes cover 2 KB, of 1480 bytes 370 KB). */
#define SMOL_MAX_FRAGMENTS 256u

/* Emit for IPv4 datagrams the stack fragmented under offloaded checksums.  The iface emits the
 * whole datagram with the device's caps (the L4 checksum written 0) and only then cuts it into
 * fragments that reach TxToken::consume one by one (src/iface/interface/mod.rs:1276-1331,
 * src/iface/interface/ipv4.rs:421-490), so the device, holding a datagram's fragments until the
 * last one, fills per group: every fragment's IPv4 header checksum (caps.ipv4, as
 * dispatch_ipv4_frag does) and the datagram's L4 checksum over the reassembled datagram — its
 * L4 length, its pseudo-header, ICMPv4 error messages' embedded header included — written into
 * the fragment that holds the field.  That is the RFC 1071 / 768 / 793 checksum a receiver
 * verifies, and the one smoltcp's own reassembling receive path accepts.
 *
 * Deliberate divergence from the reference's software route.  With its default caps the reference
 * emits a datagram it will fragment into the whole fixed-size frag.buffer
 * (FRAGMENTATION_BUFFER_SIZE bytes, mod.rs:1320; emit_payload gets &mut buffer[hl..],
 * mod.rs:1263-1267, packet.rs:80-83,166-171):
 *   - UDP: identical.  UdpPacket::fill_checksum covers the UDP length field's span (udp.rs:194-208).
 *   - TCP: differs whenever the datagram is shorter than the buffer.  TcpPacket::fill_checksum
 *     sums the whole buffer tail and puts its length in the pseudo-header (tcp.rs:616-626), so the
 *     reference's fragments carry a checksum its own reassembling receiver rejects.
 *   - ICMPv4 echo: identical only when the buffer tail past the datagram is zero;
 *     Icmpv4Packet::fill_checksum sums the whole tail, stale bytes of earlier datagrams included
 *     (icmpv4.rs:339-346, 502-503).  ICMPv4 error messages: the reference's emit panics on a tail
 *     (copy_from_slice of unequal lengths, icmpv4.rs:529-530, 543-544).
 * tests/test_frag_cpu.py restates that route (oracle_emit_like_dispatch_ip) and pins each case.
 *
 * A group is usable when every record is an IPv4 packet (Medium::Ip, or Ethernet with ethertype
 * 0x0800) passing Ipv4Packet::check_len, all share the reassembly key (ident, source, destination,
 * protocol: ipv4.rs get_key), the payloads cover [0, T) exactly once with exactly one last
 * fragment (MF clear) ending at T; otherwise its records are reported SMOL_ST_MALFORMED and only
 * their own headers are filled.  A group with SMOL_REC_IPHDR_ONLY on any record gets its headers
 * only (a raw socket's datagram).  `d_status` (nullable) receives SMOL_ST_MALFORMED /
 * SMOL_ST_UNSUPPORTED per record of every valid group. */
int smol_csum_batch_emit_frag(smol_csum_ctx_t* ctx, uint8_t* d_buf, const smol_csum_batch_t* batch,
                              const smol_csum_frag_group_t* d_groups, uint64_t n_groups,
                              const smol_checksum_caps_t* caps, uint8_t* d_status, void* stream);

/* Verify for fragmented IPv4 datagrams (src/iface/interface/ipv4.rs:103-146: every fragment
 * passes Ipv4Repr::parse, then the reassembled payload reaches the L4 gate).  Per record: its own
 * IPv4 bits, the datagram's L4 bits, and SMOL_ST_ACCEPT only when every fragment of the group
 * passes its IPv4 gate and the datagram its L4 gate (a dropped fragment never completes the
 * datagram).  Records outside every group are not written. */
int smol_csum_batch_verify_frag(smol_csum_ctx_t* ctx, const uint8_t* d_buf, const smol_csum_batch_t* batch,
                                const smol_csum_frag_group_t* d_groups, uint64_t n_groups,
                                const smol_checksum_caps_t* caps, uint8_t* d_status, void* stream);

/* ---- 4. 6LoWPAN next-header-compressed UDP (RFC 6282 §4.3) ------------------------------- */

/* The IPv6 source and destination addresses of one record (32 bytes, device memory): 6LoWPAN's
 * IPHC header compresses them (to nothing, when they derive from the link-layer addresses), so the
 * iface's decompression result travels beside the batch. */
typedef struct {
    uint8_t src[16];
    uint8_t dst[16];
} smol_ipv6_addr_pair_t;

/* UdpNhcRepr::emit's checksum (src/wire/sixlowpan/nhc.rs:746-776) over every record: each record
 * is a LOWPAN_NHC UDP packet, from its dispatch byte (0b11110CPP) to the end of the payload; the
 * payload follows an inline checksum (UdpNhcPacket::payload_mut, nhc.rs:622-626).  Under
 * caps.udp.tx() the checksum !combine([pseudo_header_v6(src, dst, Udp, n + 8), src_port,
 * dst_port, n + 8, data(payload)]) is written to the field and the C bit cleared (set_checksum,
 * nhc.rs:676-681; no 0 -> 0xffff mapping); otherwise nothing is written.  The ports are read back
 * from the packet in the encoding set_ports (nhc.rs:635-673) wrote them.  A record shorter than
 * its header or without the UDP dispatch is left untouched and reported SMOL_ST_MALFORMED.
 * `d_addrs` holds n address pairs (4-byte aligned); record kinds are ignored. */
int smol_csum_batch_nhc_udp_emit(smol_csum_ctx_t* ctx, uint8_t* d_buf, const smol_csum_batch_t* batch,
                                 const smol_ipv6_addr_pair_t* d_addrs, const smol_checksum_caps_t* caps,
                                 uint8_t* d_status, void* stream);

/* UdpNhcRepr::parse's checksum gate (src/wire/sixlowpan/nhc.rs:693-729): SMOL_ST_MALFORMED when
 * UdpNhcPacket::check_len (nhc.rs:486-500) or the dispatch test fails, or (ABI 5) when an inline
 * destination port (ports modes 0b00 / 0b10) is 0: the iface parses the decompressed header with
 * UdpRepr::parse, which drops it (src/iface/interface/sixlowpan.rs:745-775, udp.rs:246-248);
 * otherwise under
 * caps.udp.rx() an inline checksum must equal the one computed over the ports as the packet
 * accessors read them (nhc.rs:513-577); an elided checksum (C bit set) is not checked.  The IP
 * bits are always set (no IPv4 header). */
int smol_csum_batch_nhc_udp_verify(smol_csum_ctx_t* ctx, const uint8_t* d_buf,
                                   const smol_csum_batch_t* batch, const smol_ipv6_addr_pair_t* d_addrs,
                                   const smol_checksum_caps_t* caps, uint8_t* d_status, void* stream);

/* Message of the last SMOL_EHIP error on this thread ("" if none). */
const char* smol_csum_last_error(void);

/* ABI version compiled into the library (SMOLCSUM_ABI_VERSION). */
int smol_csum_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* SMOLCSUM_H */
