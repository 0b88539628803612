"""Pure-Python restatement of smoltcp's ``wire::checksum`` (test infrastructure only).

Independent of ``csum_oracle.c``: written from ``src/wire/ip.rs:762-869`` a second time so the two
restatements can check each other, and used by ``tests/golden/make_golden.py``.  Loops over
Python ints; use it for small inputs only.
"""
from __future__ import annotations


def propagate_carries(word: int) -> int:
    """src/wire/ip.rs:767-770 (u32 -> u16, two end-around-carry folds)."""
    s = (word >> 16) + (word & 0xFFFF)
    return ((s >> 16) + (s & 0xFFFF)) & 0xFFFF


def data(b: bytes) -> int:
    """checksum::data, src/wire/ip.rs:773-804, on a little-endian host (u32 wrap-around)."""
    accum = 0
    n4 = len(b) - len(b) % 4
    for i in range(0, n4, 4):  # :782-788
        accum = (accum + (b[i] | (b[i + 1] << 8))) & 0xFFFFFFFF
        accum = (accum + (b[i + 2] | (b[i + 3] << 8))) & 0xFFFFFFFF
    rem = b[n4:]
    if len(rem) >= 2:  # :791-795
        accum = (accum + (rem[0] | (rem[1] << 8))) & 0xFFFFFFFF
        rem = rem[2:]
    if rem:  # :798-800
        accum = (accum + rem[0]) & 0xFFFFFFFF
    c = propagate_carries(accum)
    return ((c >> 8) | (c << 8)) & 0xFFFF  # u16::to_be, :803


def combine(checksums) -> int:
    """checksum::combine, src/wire/ip.rs:807-813."""
    accum = 0
    for w in checksums:
        accum = (accum + w) & 0xFFFFFFFF
    return propagate_carries(accum)


def _proto_len(proto: int, length: int) -> bytes:
    return bytes([0, proto & 0xFF, (length >> 8) & 0xFF, length & 0xFF])


def pseudo_header_v4(src: bytes, dst: bytes, proto: int, length: int) -> int:
    """src/wire/ip.rs:816-831."""
    assert len(src) == 4 and len(dst) == 4
    return combine([data(src), data(dst), data(_proto_len(proto, length))])


def pseudo_header_v6(src: bytes, dst: bytes, proto: int, length: int) -> int:
    """src/wire/ip.rs:834-849 (length truncated to u16 at :842)."""
    assert len(src) == 16 and len(dst) == 16
    return combine([data(src), data(dst), data(_proto_len(proto, length))])


def pseudo_header(src: bytes, dst: bytes, proto: int, length: int) -> int:
    """src/wire/ip.rs:851-869; a family mismatch is unreachable!() in the reference."""
    if len(src) == 4 and len(dst) == 4:
        return pseudo_header_v4(src, dst, proto, length)
    if len(src) == 16 and len(dst) == 16:
        return pseudo_header_v6(src, dst, proto, length)
    raise ValueError("address family mismatch (reference: unreachable!())")


def fill_l4(buf: bytearray, field: int, value: int) -> None:
    buf[field] = (value >> 8) & 0xFF
    buf[field + 1] = value & 0xFF


def ipv4_verify(pkt: bytes) -> bool:
    """src/wire/ipv4.rs:363-370."""
    hl = (pkt[0] & 0x0F) * 4
    return data(pkt[:hl]) == 0xFFFF


def ipv4_fill(pkt: bytearray) -> None:
    """src/wire/ipv4.rs:506-513."""
    hl = (pkt[0] & 0x0F) * 4
    fill_l4(pkt, 10, 0)
    fill_l4(pkt, 10, ~data(bytes(pkt[:hl])) & 0xFFFF)


def udp_verify(udp: bytes, src: bytes, dst: bytes) -> bool:
    """src/wire/udp.rs:129-147."""
    if (udp[6] << 8 | udp[7]) == 0:
        return True
    ulen = udp[4] << 8 | udp[5]
    return combine([pseudo_header(src, dst, 17, ulen), data(udp[:ulen])]) == 0xFFFF


def udp_fill(udp: bytearray, src: bytes, dst: bytes) -> None:
    """src/wire/udp.rs:194-208."""
    fill_l4(udp, 6, 0)
    ulen = udp[4] << 8 | udp[5]
    c = ~combine([pseudo_header(src, dst, 17, ulen), data(bytes(udp[:ulen]))]) & 0xFFFF
    fill_l4(udp, 6, 0xFFFF if c == 0 else c)


def tcp_verify(tcp: bytes, src: bytes, dst: bytes) -> bool:
    """src/wire/tcp.rs:395-405."""
    return combine([pseudo_header(src, dst, 6, len(tcp)), data(tcp)]) == 0xFFFF


def tcp_verify_partial(tcp: bytes, src: bytes, dst: bytes) -> bool:
    """src/wire/tcp.rs:376-385."""
    return pseudo_header(src, dst, 6, len(tcp)) == (tcp[16] << 8 | tcp[17])


def tcp_fill(tcp: bytearray, src: bytes, dst: bytes) -> None:
    """src/wire/tcp.rs:616-626."""
    fill_l4(tcp, 16, 0)
    fill_l4(tcp, 16, ~combine([pseudo_header(src, dst, 6, len(tcp)), data(bytes(tcp))]) & 0xFFFF)


def icmpv4_verify(p: bytes) -> bool:
    """src/wire/icmpv4.rs:277-284 (and IGMP, src/wire/igmp.rs:122-129)."""
    return data(p) == 0xFFFF


def icmpv4_fill(p: bytearray) -> None:
    """src/wire/icmpv4.rs:339-346 (and IGMP, src/wire/igmp.rs:163-170)."""
    fill_l4(p, 2, 0)
    fill_l4(p, 2, ~data(bytes(p)) & 0xFFFF)


def icmpv6_verify(p: bytes, src: bytes, dst: bytes) -> bool:
    """src/wire/icmpv6.rs:424-434."""
    return combine([pseudo_header_v6(src, dst, 58, len(p)), data(p)]) == 0xFFFF


def icmpv6_fill(p: bytearray, src: bytes, dst: bytes) -> None:
    """src/wire/icmpv6.rs:538-553."""
    fill_l4(p, 2, 0)
    fill_l4(p, 2, ~combine([pseudo_header_v6(src, dst, 58, len(p)), data(bytes(p))]) & 0xFFFF)


# ---- 6LoWPAN NHC UDP (src/wire/sixlowpan/nhc.rs) -----------------------------------------------


def _nhc_sizes(b0: int):
    """UdpNhcPacket::ports_size / checksum_size, nhc.rs:593-611."""
    ports = {0: 4, 1: 3, 2: 3, 3: 1}[b0 & 3]
    return ports, (0 if b0 & 4 else 2)


def nhc_ports(p: bytes, emit: bool = False):
    """src_port / dst_port accessors (nhc.rs:513-577) as written; with ``emit`` the destination of
    mode 0b01 comes from byte 3, where set_ports (nhc.rs:655-662) put it."""
    m = p[0] & 3
    src = (p[1] << 8 | p[2]) if m in (0, 1) else (0xF000 + p[1]) if m == 2 else 0xF0B0 + (p[1] >> 4)
    if m == 0:
        dst = p[3] << 8 | p[4]
    elif m == 1:
        dst = 0xF000 + (p[3] if emit else p[1])
    elif m == 2:
        dst = p[2] << 8 | p[3]
    else:
        dst = 0xF0B0 + p[1]
    return src, dst


def nhc_udp_checksum(src: bytes, dst: bytes, sport: int, dport: int, payload: bytes) -> int:
    """nhc.rs:705-716 / :760-771."""
    n = len(payload)
    return ~combine([pseudo_header_v6(src, dst, 17, n + 8), sport, dport, (n + 8) & 0xFFFF,
                     data(payload)]) & 0xFFFF


def nhc_udp_verify(p: bytes, src: bytes, dst: bytes):
    """UdpNhcRepr::parse's checksum test (nhc.rs:697-723): None when the packet is dropped before
    it (check_len, dispatch, or the destination port 0 that the iface's UdpRepr::parse of the
    decompressed header drops), else whether the inline checksum (if any) matches."""
    if len(p) < 1:
        return None
    ports, cs = _nhc_sizes(p[0])
    if 1 + ports + cs > len(p) or (p[0] >> 3) != 0x1E:
        return None
    sport, dport = nhc_ports(p)
    if dport == 0:  # dropped by UdpRepr::parse after decompression (sixlowpan.rs:745-775, udp.rs:246-248)
        return None
    if cs == 0:
        return True
    return nhc_udp_checksum(src, dst, sport, dport, p[1 + ports + cs:]) == (p[1 + ports] << 8 | p[2 + ports])


def nhc_udp_fill(p: bytearray, src: bytes, dst: bytes) -> bool:
    """UdpNhcRepr::emit's checksum (nhc.rs:759-774): payload after an inline checksum, C bit
    cleared, field written.  False (untouched) when the header does not fit / no UDP dispatch."""
    if len(p) < 1:
        return False
    ports, _ = _nhc_sizes(p[0])
    if 1 + ports + 2 > len(p) or (p[0] >> 3) != 0x1E:
        return False
    sport, dport = nhc_ports(bytes(p), emit=True)
    c = nhc_udp_checksum(src, dst, sport, dport, bytes(p[1 + ports + 2:]))
    p[0] &= ~4 & 0xFF
    fill_l4(p, 1 + ports, c)
    return True


# ---- IPv6 Hop-by-Hop options on receive (an independent, literal restatement) -------------------

IPV6_HBH_MAX_OPTIONS = 4  # build.rs:19


def _hbh_options(opt: bytes):
    """Ipv6HopByHopRepr::parse (ipv6hbh.rs:70-89) over Ipv6OptionsIterator (ipv6option.rs:386-420):
    the option types it keeps, or None when an option fails to parse."""
    kept, pos = [], 0
    while pos < len(opt):
        rest = opt[pos:]
        t = rest[0]
        if t == 0:  # Pad1: check_len passes, buffer_len 1 (:172-174, :323)
            repr_, size = 0, 1
        else:
            if len(rest) == 1:  # check_len: no length byte (:176-178)
                return None
            dl = rest[1]
            if len(rest) < 2 + dl:  # check_len: data past the end (:180-184)
                return None
            if t == 5 and dl != 2:  # Repr::parse RouterAlert (:293-300)
                return None
            repr_, size = t, 2 + dl
        if len(kept) == IPV6_HBH_MAX_OPTIONS:  # Vec::push fails: `break` (ipv6hbh.rs:82-85)
            break
        kept.append(repr_)
        pos += size
    return kept


def hbh_options_drop(opt: bytes) -> bool:
    """process_hopbyhop (src/iface/interface/ipv6.rs:282-313): True when the packet is dropped."""
    kept = _hbh_options(bytes(opt))
    if kept is None:  # check!(Ipv6HopByHopRepr::parse(..))
        return True
    for t in kept:
        if t in (0, 1, 5):  # Pad1, PadN, RouterAlert
            continue
        if t & 0xC0:  # Ipv6OptionFailureType::from(type): Discard / DiscardSendAll / DiscardSendUnicast
            return True
    return False
