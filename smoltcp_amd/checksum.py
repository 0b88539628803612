"""``smoltcp::wire::checksum`` (src/wire/ip.rs:762-869) through the C ABI's scalar host mirrors.

Same names and argument meaning as the reference module: ``data``, ``combine``,
``pseudo_header_v4``, ``pseudo_header_v6``, ``pseudo_header`` (which raises on an address-family
mismatch where the reference hits ``unreachable!()``).
"""
from __future__ import annotations

import ctypes

from ._lib import SMOL_OK, check, lib


def _buf(b: bytes):
    b = bytes(b)
    return ctypes.create_string_buffer(b, len(b)) if b else None, len(b)


def data(b: bytes) -> int:
    """checksum::data — RFC 1071 sum without the final complement (src/wire/ip.rs:773-804)."""
    p, n = _buf(b)
    return int(lib().smol_csum_data(p, n))


def combine(checksums) -> int:
    """checksum::combine (src/wire/ip.rs:807-813)."""
    ws = list(checksums)
    arr = (ctypes.c_uint16 * max(len(ws), 1))(*ws)
    return int(lib().smol_csum_combine(arr, len(ws)))


def pseudo_header_v4(src_addr: bytes, dst_addr: bytes, next_header: int, length: int) -> int:
    """checksum::pseudo_header_v4 (src/wire/ip.rs:816-831)."""
    assert len(src_addr) == 4 and len(dst_addr) == 4
    return int(lib().smol_csum_pseudo_header_v4(bytes(src_addr), bytes(dst_addr), next_header & 0xFF,
                                                length & 0xFFFFFFFF))


def pseudo_header_v6(src_addr: bytes, dst_addr: bytes, next_header: int, length: int) -> int:
    """checksum::pseudo_header_v6 (src/wire/ip.rs:834-849)."""
    assert len(src_addr) == 16 and len(dst_addr) == 16
    return int(lib().smol_csum_pseudo_header_v6(bytes(src_addr), bytes(dst_addr), next_header & 0xFF,
                                                length & 0xFFFFFFFF))


def format_checksum(correct: bool, partially_correct: bool) -> str:
    """checksum::format_checksum (src/wire/ip.rs:871-886): the annotation the pretty-printers
    append to a packet line."""
    if correct:
        return ""
    return " (partial checksum correct)" if partially_correct else " (checksum incorrect)"


def ipv4_annotation(status: int) -> str:
    """The IPv4 header line's annotation for a verify status byte (Ipv4Packet's pretty_print,
    src/wire/ipv4.rs:698: format_checksum(verify_checksum(), false))."""
    return format_checksum(bool(status & 0x08), False)  # SMOL_ST_IP_VALID


def l4_annotation(status: int) -> str:
    """The UDP / TCP line's annotation (pretty_print_ip_payload, src/wire/ip.rs:930-962:
    verify_checksum() and verify_partial_checksum())."""
    return format_checksum(bool(status & 0x10), bool(status & 0x04))  # L4_VALID, L4_PARTIAL


def pseudo_header(src_addr: bytes, dst_addr: bytes, next_header: int, length: int) -> int:
    """checksum::pseudo_header (src/wire/ip.rs:851-869): dispatch on the address family."""
    fam = {4: 4, 16: 6}
    out = ctypes.c_uint16(0)
    rc = lib().smol_csum_pseudo_header(fam.get(len(src_addr), 0), bytes(src_addr),
                                       fam.get(len(dst_addr), 0), bytes(dst_addr),
                                       next_header & 0xFF, length & 0xFFFFFFFF, ctypes.byref(out))
    if rc != SMOL_OK:
        raise ValueError("address family mismatch (the reference panics: unreachable!())")
    check(rc, "smol_csum_pseudo_header")
    return int(out.value)
