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
