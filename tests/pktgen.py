"""Host-side packet builders for the parity tests (plain Python/numpy, no checksum logic: every
checksum field is written as given, usually 0)."""
from __future__ import annotations

import numpy as np

import oracle


def be16(v: int) -> bytes:
    return bytes([(v >> 8) & 0xFF, v & 0xFF])


def ipv4(src: bytes, dst: bytes, proto: int, payload: bytes, ihl: int = 5, ttl: int = 64,
         flags_frag: int = 0x4000, ident: int = 0, csum: int = 0, options: bytes | None = None,
         total_len: int | None = None) -> bytes:
    hl = ihl * 4
    opts = options if options is not None else bytes(hl - 20)
    assert len(opts) == hl - 20
    tl = hl + len(payload) if total_len is None else total_len
    h = bytes([0x40 | ihl, 0]) + be16(tl) + be16(ident) + be16(flags_frag) + bytes([ttl, proto]) \
        + be16(csum) + src + dst + opts
    return h + payload


def ipv6(src: bytes, dst: bytes, nh: int, payload: bytes, hop: int = 64,
         payload_len: int | None = None) -> bytes:
    pl = len(payload) if payload_len is None else payload_len
    return bytes([0x60, 0, 0, 0]) + be16(pl) + bytes([nh, hop]) + src + dst + payload


def hbh(next_header: int, length_units: int, rng) -> bytes:
    """IPv6 Hop-by-Hop header of (length_units+1)*8 bytes: PadN filler."""
    total = (length_units + 1) * 8
    body = bytearray(total - 2)  # Pad1 options (type 0) ...
    if total - 4 < 256:
        body[0] = 1  # ... or one PadN option when it fits
        body[1] = total - 4
    return bytes([next_header, length_units]) + bytes(body)


def hbh_opts(next_header: int, opts: bytes, pad: bool = True) -> bytes:
    """IPv6 Hop-by-Hop header carrying the option bytes `opts` as given (valid or not), padded with
    Pad1 options (zero bytes) to a multiple of 8 bytes (pad=False: `opts` must already fit)."""
    n = len(opts) + 2
    total = (n + 7) // 8 * 8
    body = bytes(opts) + bytes(total - n if pad else 0)
    assert (len(body) + 2) % 8 == 0
    return bytes([next_header, (len(body) + 2) // 8 - 1]) + body


def random_hbh_options(rng, max_opts: int = 7) -> bytes:
    """Random option TLVs for process_hopbyhop (src/iface/interface/ipv6.rs:282-313): Pad1, PadN,
    RouterAlert (right and wrong data length), unknown types of every failure action, Rpl (0x63),
    and now and then a truncated last option."""
    out = bytearray()
    unknown = [0x0F, 0x1E, 0x3F, 0x40, 0x7F, 0x80, 0xC2, 0x63, 0x3E]  # skip (00) and discard (01/10/11)
    for _ in range(int(rng.integers(0, max_opts + 1))):
        c = int(rng.integers(0, 6))
        if c == 0:
            out += b"\x00"  # Pad1
        elif c == 1:
            dl = int(rng.integers(0, 6))
            out += bytes([1, dl]) + bytes(dl)  # PadN
        elif c == 2:
            dl = 2 if rng.random() < 0.8 else int(rng.integers(0, 5))
            out += bytes([5, dl]) + rand_bytes(rng, dl)  # RouterAlert
        else:
            dl = int(rng.integers(0, 6))
            out += bytes([unknown[int(rng.integers(0, len(unknown)))], dl]) + rand_bytes(rng, dl)
    if rng.random() < 0.15 and out:
        out = out[:-int(rng.integers(1, min(3, len(out)) + 1))]  # a truncated last option
    return bytes(out)


def udp(sport: int, dport: int, payload: bytes, csum: int = 0, length: int | None = None) -> bytes:
    ln = 8 + len(payload) if length is None else length
    return be16(sport) + be16(dport) + be16(ln) + be16(csum) + payload


def tcp(sport: int, dport: int, payload: bytes, csum: int = 0, doff: int = 5, flags: int = 0x18,
        seq: int = 1, ack: int = 2) -> bytes:
    opts = bytes((doff - 5) * 4)
    return be16(sport) + be16(dport) + seq.to_bytes(4, "big") + ack.to_bytes(4, "big") + \
        bytes([doff << 4, flags]) + be16(8192) + be16(csum) + be16(0) + opts + payload


def icmp_echo(t: int, payload: bytes, csum: int = 0) -> bytes:
    return bytes([t, 0]) + be16(csum) + be16(0x1234) + be16(0xABCD) + payload


def icmp4_error(t: int, code: int, inner: bytes, csum: int = 0) -> bytes:
    """ICMPv4 DstUnreachable (3) / TimeExceeded (11) with `inner` (an IPv4 header + data) after the
    4 unused bytes, as Icmpv4Repr::emit lays it out (icmpv4.rs:520-543)."""
    return bytes([t, code]) + be16(csum) + bytes(4) + inner


def icmp6(t: int, body_len: int, rng, csum: int = 0) -> bytes:
    """ICMPv6 message of type t: 4-byte header + body_len random bytes (the check_len tests)."""
    return bytes([t, 0]) + be16(csum) + rand_bytes(rng, body_len)


def fragment_like_iface(dgram: bytes, ip_mtu: int, ident: int, fill_header: bool):
    """Cut an IPv4 datagram (20-byte header + the L4 bytes, as emit_ip left it in frag.buffer) the
    way smoltcp's iface sends it: dispatch_ip's first fragment (src/iface/interface/mod.rs:1276-1331)
    and dispatch_ipv4_frag's others (src/iface/interface/ipv4.rs:440-490).  Fragment data is
    max_ipv4_fragment_size (src/phy/mod.rs:297-300: the payload MTU rounded down to 8 bytes); each
    header is the datagram's with total length, ident, MF, DF = 0 and the offset rewritten, its
    checksum filled when caps.ipv4.tx() (`fill_header`), else left 0 as Ipv4Repr::emit wrote it."""
    from oracle import pyref

    hdr, data = bytearray(dgram[:20]), dgram[20:]
    step = (ip_mtu - 20) - (ip_mtu - 20) % 8
    frags = []
    for off in range(0, len(data), step):
        part = data[off: off + step]
        h = bytearray(hdr)
        h[2:4] = (20 + len(part)).to_bytes(2, "big")
        h[4:6] = ident.to_bytes(2, "big")
        more = off + step < len(data)
        h[6:8] = ((0x2000 if more else 0) | (off // 8)).to_bytes(2, "big")
        h[10:12] = b"\0\0"
        if fill_header:
            pyref.ipv4_fill(h)
        frags.append(bytes(h) + part)
    return frags


def eth(payload: bytes, ethertype: int = 0x0800) -> bytes:
    return bytes([0x02, 0, 0, 0, 0, 1, 0x02, 0, 0, 0, 0, 2]) + be16(ethertype) + payload


def rand_bytes(rng, n: int) -> bytes:
    return rng.integers(0, 256, n, dtype=np.uint8).tobytes()


NHC_PORTS_SIZE = {0: 4, 1: 3, 2: 3, 3: 1}  # UdpNhcPacket::ports_size, nhc.rs:602-611


def nhc_udp(rng, mode: int, elided: bool, plen: int, csum: int = 0) -> bytes:
    """A LOWPAN_NHC UDP packet (RFC 6282 §4.3): dispatch 0b11110CPP, ports in mode ``mode``
    (random inline bytes), an inline checksum unless ``elided``, ``plen`` random payload bytes."""
    head = bytes([0xF0 | (4 if elided else 0) | mode]) + rand_bytes(rng, NHC_PORTS_SIZE[mode])
    return head + (b"" if elided else be16(csum)) + rand_bytes(rng, plen)


def pack(records, align: int = 1, gap_rng=None, base_pad: int = 0):
    """Pack byte records into one host buffer; returns (buf, offsets, lengths).  ``gap_rng`` adds
    random 0..7 byte gaps (odd offsets)."""
    offs, lens, chunks, pos = [], [], [], base_pad
    if base_pad:
        chunks.append(bytes(base_pad))
    for r in records:
        gap = int(gap_rng.integers(0, 8)) if gap_rng is not None else 0
        if gap:
            chunks.append(bytes([0xA5]) * gap)
            pos += gap
        if align > 1 and pos % align:
            pad = align - pos % align
            chunks.append(bytes(pad))
            pos += pad
        offs.append(pos)
        lens.append(len(r))
        chunks.append(r)
        pos += len(r)
    chunks.append(bytes(16))  # tail slack
    buf = np.frombuffer(b"".join(chunks), dtype=np.uint8).copy()
    return buf, np.array(offs, dtype=np.uint64), np.array(lens, dtype=np.uint32)


def oracle_desc(offs, lens, kinds, flags=0):
    from smoltcp_amd.engine import make_descriptors

    return make_descriptors(offs, lens, kinds, flags)


def oracle_verify_records(buf, offs, lens, kinds, caps=(0, 0, 0, 0, 0)):
    d = oracle_desc(offs, lens, kinds)
    return oracle.batch_verify(buf, d, len(d), caps=caps)


def oracle_emit_records(buf, offs, lens, kinds, caps=(0, 0, 0, 0, 0)):
    d = oracle_desc(offs, lens, kinds)
    return oracle.batch_emit(buf, d, len(d), caps=caps)


def oracle_data_records(buf, offs, lens):
    d = oracle_desc(offs, lens, 0)
    return oracle.batch_data(buf, d, len(d))
