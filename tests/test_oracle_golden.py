"""Pin the CPU oracle to the reference's own known-answer vectors (CPU only).

Mirrors the reference's deconstruct/construct tests: e.g. src/wire/udp.rs test_deconstruct
(checksum()==0x124d, verify_checksum()) and test_construct (fill over a junk field reproduces the
bytes).  Both restatements — oracle/pyref.py (pure Python) and oracle/csum_oracle.c — are checked.
"""
import ctypes

import numpy as np
import pytest

import oracle
from oracle import pyref

ST_IP_OK, ST_L4_OK, ST_PARTIAL, ST_IP_VALID, ST_L4_VALID = 0x01, 0x02, 0x04, 0x08, 0x10
ST_MALFORMED, ST_UNSUPPORTED, ST_ACCEPT = 0x20, 0x40, 0x80


def _arr(b):
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


def _c_verify(k, b):
    L = oracle.lib()
    a = _arr(b)
    src = _arr(bytes.fromhex(k["src"])) if k["src"] else None
    dst = _arr(bytes.fromhex(k["dst"])) if k["dst"] else None
    p = a.ctypes.data
    proto = k["proto"]
    if proto == "ipv4":
        return bool(L.oracle_ipv4_verify(p))
    if proto == "udp":
        return bool(L.oracle_udp_verify(p, 4 if src.size == 4 else 6, src.ctypes.data, dst.ctypes.data))
    if proto == "tcp":
        return bool(L.oracle_tcp_verify(p, a.size, 4 if src.size == 4 else 6, src.ctypes.data,
                                        dst.ctypes.data))
    if proto in ("icmpv4", "igmp"):
        return bool(L.oracle_icmpv4_verify(p, a.size))
    if proto == "icmpv6":
        return bool(L.oracle_icmpv6_verify(p, a.size, src.ctypes.data, dst.ctypes.data))
    raise AssertionError(proto)


def _c_fill(k, b):
    L = oracle.lib()
    a = _arr(b)
    src = _arr(bytes.fromhex(k["src"])) if k["src"] else None
    dst = _arr(bytes.fromhex(k["dst"])) if k["dst"] else None
    p = a.ctypes.data
    proto = k["proto"]
    if proto == "ipv4":
        L.oracle_ipv4_fill(p)
    elif proto == "udp":
        L.oracle_udp_fill(p, 4 if src.size == 4 else 6, src.ctypes.data, dst.ctypes.data)
    elif proto == "tcp":
        L.oracle_tcp_fill(p, a.size, 4 if src.size == 4 else 6, src.ctypes.data, dst.ctypes.data)
    elif proto in ("icmpv4", "igmp"):
        L.oracle_icmpv4_fill(p, a.size)
    elif proto == "icmpv6":
        L.oracle_icmpv6_fill(p, a.size, src.ctypes.data, dst.ctypes.data)
    return a.tobytes()


def _py_verify(k, b):
    src = bytes.fromhex(k["src"]) if k["src"] else None
    dst = bytes.fromhex(k["dst"]) if k["dst"] else None
    proto = k["proto"]
    if proto == "ipv4":
        return pyref.ipv4_verify(b)
    if proto == "udp":
        return pyref.udp_verify(b, src, dst)
    if proto == "tcp":
        return pyref.tcp_verify(b, src, dst)
    if proto in ("icmpv4", "igmp"):
        return pyref.icmpv4_verify(b)
    return pyref.icmpv6_verify(b, src, dst)


def _py_fill(k, b):
    src = bytes.fromhex(k["src"]) if k["src"] else None
    dst = bytes.fromhex(k["dst"]) if k["dst"] else None
    buf = bytearray(b)
    proto = k["proto"]
    if proto == "ipv4":
        pyref.ipv4_fill(buf)
    elif proto == "udp":
        pyref.udp_fill(buf, src, dst)
    elif proto == "tcp":
        pyref.tcp_fill(buf, src, dst)
    elif proto in ("icmpv4", "igmp"):
        pyref.icmpv4_fill(buf)
    else:
        pyref.icmpv6_fill(buf, src, dst)
    return bytes(buf)


def _kats(golden):
    return golden["kat"]


def test_kat_count(golden):
    assert len(golden["kat"]) >= 15
    assert len(golden["iface_ipv6_packets"]) >= 7
    assert len(golden["fuzz_corpus_frames"]) == 10


@pytest.mark.parametrize("impl", ["c", "py"])
def test_kat_deconstruct(golden, impl):
    """checksum field == the asserted value and verify_checksum() holds (deconstruct tests)."""
    for k in _kats(golden):
        b = bytes.fromhex(k["bytes"])
        f = k["field"]
        assert (b[f] << 8 | b[f + 1]) == k["checksum"], k["name"]
        got = _c_verify(k, b) if impl == "c" else _py_verify(k, b)
        assert got == k["verify"], (k["name"], k["cite"])


@pytest.mark.parametrize("impl", ["c", "py"])
def test_kat_construct(golden, impl):
    """fill_checksum over the field value the reference test left there reproduces the bytes."""
    for k in _kats(golden):
        if k["pre_fill_field"] is None:
            continue
        b = bytearray.fromhex(k["bytes"])
        f = k["field"]
        b[f] = k["pre_fill_field"] >> 8
        b[f + 1] = k["pre_fill_field"] & 0xFF
        out = _c_fill(k, bytes(b)) if impl == "c" else _py_fill(k, bytes(b))
        assert out.hex() == k["bytes"], (k["name"], k["cite"])


def test_kat_negative_bitflip(golden):
    """Single-bit corruption (phy::FaultInjector's recipe, src/phy/fault_injector.rs:45-51) is
    caught — except on a UDP record whose field is 0 (no checksum)."""
    rng = np.random.default_rng(7)
    for k in _kats(golden):
        if k["proto"] == "udp" and k["checksum"] == 0:
            continue
        b = bytearray.fromhex(k["bytes"])
        for _ in range(16):
            c = bytearray(b)
            span = (c[0] & 0x0F) * 4 if k["proto"] == "ipv4" else len(c)  # IPv4: header only
            i = int(rng.integers(span))
            if k["proto"] == "udp" and i in (4, 5):
                continue  # the UDP length field moves the span instead
            c[i] ^= 1 << int(rng.integers(8))
            if k["proto"] == "udp" and c[6] == 0 and c[7] == 0:
                continue
            assert _c_verify(k, bytes(c)) is False, (k["name"], i)
            assert _py_verify(k, bytes(c)) is False


def test_iface_ipv6_packets(golden):
    """IPv6 packets from src/iface/interface/tests/ipv6.rs that parse_ipv6() accepts with default
    caps (ICMPv6 checksum verified), including an odd-length ICMPv6 payload."""
    L = oracle.lib()
    caps = oracle.caps_c()
    for p in golden["iface_ipv6_packets"]:
        a = _arr(bytes.fromhex(p["bytes"]))
        st = L.oracle_record_verify(a.ctypes.data, a.size, 1, ctypes.byref(caps))
        assert st & ST_ACCEPT and st & ST_L4_VALID, p["cite"]
        assert not st & (ST_MALFORMED | ST_UNSUPPORTED), p["cite"]
        # and the pure-Python restatement on the ICMPv6 part
        b = bytes.fromhex(p["bytes"])
        plen = b[4] << 8 | b[5]
        assert b[6] == 58
        assert pyref.icmpv6_verify(b[40:40 + plen], b[8:24], b[24:40]), p["cite"]


def test_iface_ipv6_hop_by_hop_packets(golden):
    """The four hop_by_hop_* packets of src/iface/interface/tests/ipv6.rs:151,200,232,290: the skip
    option's packet is accepted (its ICMPv6 echo request passes the checksum gate), the three whose
    options make process_hopbyhop drop the packet (ipv6.rs:282-313) are MALFORMED: dropped before any
    checksum is looked at.  Emit does not parse the options: it fills all four the same way."""
    L = oracle.lib()
    caps = oracle.caps_c()
    hbh = golden["iface_ipv6_hop_by_hop"]
    assert [p["dropped"] for p in hbh] == [False, True, True, True]
    for p in hbh:
        b = bytes.fromhex(p["bytes"])
        a = _arr(b)
        st = L.oracle_record_verify(a.ctypes.data, a.size, 1, ctypes.byref(caps))
        if p["dropped"]:
            assert st & ST_MALFORMED and not st & ST_ACCEPT, (p["cite"], hex(st))
        else:
            assert st & ST_ACCEPT and st & ST_L4_VALID and not st & ST_MALFORMED, (p["cite"], hex(st))
        hlen = (b[41] + 1) * 8
        assert pyref.hbh_options_drop(b[42:40 + hlen]) == p["dropped"], p["cite"]
        # emit: the ICMPv6 checksum behind the header is filled (the multicast packet reuses the
        # others' ICMPv6 bytes under another destination, so only a correct checksum is asserted)
        e = _arr(b)
        e[40 + hlen + 2:40 + hlen + 4] = 0
        L.oracle_record_emit(e.ctypes.data, e.size, 1, ctypes.byref(caps))
        plen = b[4] << 8 | b[5]
        assert pyref.icmpv6_verify(e.tobytes()[40 + hlen:40 + plen], b[8:24], b[24:40]), p["cite"]
        if b[24] != 0xFF:
            assert e.tobytes() == b, p["cite"]


@pytest.mark.parametrize("seed", [1, 2])
def test_hbh_options_c_matches_pyref(seed):
    """The C restatement of process_hopbyhop's option walk against pyref's literal one (iterator +
    4-entry Vec), on random option bytes biased towards Pad1 / PadN / RouterAlert / discard types."""
    L = oracle.lib()
    rng = np.random.default_rng(seed)
    types = np.array([0, 1, 5, 2, 0x0F, 0x40, 0x80, 0xC0, 0x63], dtype=np.uint8)
    for _ in range(20000):
        n = int(rng.integers(0, 40))
        a = rng.integers(0, 256, n).astype(np.uint8)
        m = rng.random(n) < 0.6
        a[m] = rng.choice(types, int(m.sum()))
        s = rng.random(n) < 0.5
        a[s] = rng.integers(0, 4, int(s.sum()))
        got = L.oracle_hbh_options_drop(a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), n)
        assert bool(got) == pyref.hbh_options_drop(a.tobytes()), a.tobytes().hex()


CORPUS_EXPECT = {
    # frame: (IP header valid, L4 fully valid, L4 partial (TX-offload) checksum, unsupported)
    "arp.bin": None,
    "icmpv4_reply.bin": (True, True, False),
    "icmpv4_request.bin": (True, True, False),
    "icmpv4_unreachable.bin": (True, True, False),
    "icmpv6_nbr_solicitation.bin": (True, True, False),
    "tcpv4_data.bin": (True, False, True),
    "tcpv4_fin.bin": (True, False, True),
    "tcpv4_rst.bin": (True, True, False),
    "tcpv4_syn.bin": (True, False, True),
    "udpv4.bin": (True, True, False),
}


def test_fuzz_corpus_frames(golden):
    """The 10 captured Ethernet frames of fuzz/corpus/packet_parser.  Their checksums were written
    by real senders; the three tcpv4 frames from a TX-offloading host carry only the pseudo-header
    partial sum (verify_partial_checksum true, verify_checksum false)."""
    L = oracle.lib()
    caps = oracle.caps_c()
    for fr in golden["fuzz_corpus_frames"]:
        a = _arr(bytes.fromhex(fr["bytes"]))
        st = L.oracle_record_verify(a.ctypes.data, a.size, 2, ctypes.byref(caps))
        exp = CORPUS_EXPECT[fr["name"]]
        if exp is None:
            assert st & ST_UNSUPPORTED and st & ST_ACCEPT
            continue
        ip_ok, l4_ok, partial = exp
        assert bool(st & ST_IP_VALID) == ip_ok, fr["name"]
        assert bool(st & ST_L4_VALID) == l4_ok, fr["name"]
        assert bool(st & ST_PARTIAL) == partial, fr["name"]
        assert bool(st & ST_ACCEPT) == (ip_ok and l4_ok), fr["name"]


def test_pyref_matches_c_oracle_random():
    """The two restatements agree on random spans, odd lengths, all-0x00/0xFF spans and spans
    long enough to wrap the reference's u32 accumulator (> 131074 bytes)."""
    rng = np.random.default_rng(0x5EED)
    cases = [b"", b"\x00", b"\xff", b"\x00" * 64, b"\xff" * 63, b"\xff" * 131074, b"\xff" * 131076,
             b"\xff" * 262150]
    for n in list(range(1, 70)) + [1499, 1500, 9000]:
        cases.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    for c in cases:
        assert oracle.data(c) == pyref.data(c), len(c)


def test_data_zero_iff_all_zero():
    for n in range(0, 40):
        assert oracle.data(b"\x00" * n) == 0
        if n:
            b = bytearray(n)
            b[n // 2] = 1
            assert oracle.data(bytes(b)) != 0


def test_pseudo_header_v4_v6():
    rng = np.random.default_rng(3)
    L = oracle.lib()
    for _ in range(200):
        s4, d4 = rng.integers(0, 256, 4, dtype=np.uint8), rng.integers(0, 256, 4, dtype=np.uint8)
        s6, d6 = rng.integers(0, 256, 16, dtype=np.uint8), rng.integers(0, 256, 16, dtype=np.uint8)
        proto = int(rng.integers(256))
        ln = int(rng.integers(0, 1 << 20))  # u16 truncation exercised
        assert L.oracle_pseudo_v4(s4.ctypes.data, d4.ctypes.data, proto, ln) == \
            pyref.pseudo_header_v4(s4.tobytes(), d4.tobytes(), proto, ln)
        assert L.oracle_pseudo_v6(s6.ctypes.data, d6.ctypes.data, proto, ln) == \
            pyref.pseudo_header_v6(s6.tobytes(), d6.tobytes(), proto, ln)
    with pytest.raises(ValueError):
        pyref.pseudo_header(b"\x00" * 4, b"\x00" * 16, 6, 0)


def test_icmpv6_check_len_table(golden):
    """oracle_icmpv6_min_len restates Icmpv6Packet::check_len's per-type rule: pinned to the table
    make_golden.py extracted from src/wire/icmpv6.rs (enum values, field ends, header_len arms,
    the check_len arm) for every type value; types the enum does not name are Message::Unknown."""
    tab = golden["icmpv6_check_len"]["min_len"]
    L = oracle.lib()
    for t in range(256):
        assert L.oracle_icmpv6_min_len(t) == tab.get(str(t), 0), t


def test_icmpv6_truncated_typed_messages_malformed(golden):
    """A typed ICMPv6 message shorter than its header is dropped by check_len before the
    checksum gate (SMOL_ST_MALFORMED, no ACCEPT) even with a correct checksum; at its minimum
    length it passes.  Emit keeps the generic len >= 4 rule (fill_checksum covers any type)."""
    from tests import pktgen as P

    rng = np.random.default_rng(6)
    a6, b6 = bytes(range(16)), bytes(range(16, 32))
    tab = {int(k): v for k, v in golden["icmpv6_check_len"]["min_len"].items()}
    for t in list(range(256)):
        need = tab.get(t, 0)
        for body in sorted({0, 3, 4, max(need - 5, 0), max(need - 4, 0), need, need + 3}):
            msg = P.icmp6(t, body, rng)
            rec = np.frombuffer(P.ipv6(a6, b6, 58, msg), np.uint8).copy()
            oracle.batch_emit(rec, None, 1, len(rec), len(rec), 1)  # fill (generic rule)
            st = int(oracle.batch_verify(rec, None, 1, len(rec), len(rec), 1)[0])
            ok = need != 0 and len(msg) >= need
            assert bool(st & ST_MALFORMED) == (not ok), (t, len(msg), st)
            assert bool(st & ST_ACCEPT) == ok, (t, len(msg), st)
            assert pyref.icmpv6_verify(bytes(rec[40:]), a6, b6)  # the fill itself is valid


def test_icmpv4_error_embedded_header_corpus(golden):
    """fuzz/corpus/packet_parser/icmpv4_unreachable.bin is a real DstUnreachable message whose
    embedded IPv4 header checksum (0xb0b4), ICMP checksum and outer header checksum were written by
    its sender.  Zero all three (what the stack writes under offloaded caps), emit with default
    caps: the frame must come back byte for byte.  With caps.ipv4 = None the inner (and outer)
    header field stays 0 and the ICMP checksum covers that."""
    fr = [f for f in golden["fuzz_corpus_frames"] if f["name"] == "icmpv4_unreachable.bin"][0]
    orig = _arr(bytes.fromhex(fr["bytes"]))
    ip = 14
    hl = (orig[ip] & 15) * 4
    icmp = ip + hl
    assert orig[icmp] == 3 and orig[icmp + 8] >> 4 == 4
    z = orig.copy()
    for off in (ip + 10, icmp + 2, icmp + 8 + 10):
        z[off:off + 2] = 0
    got = z.copy()
    st = oracle.batch_emit(got, None, 1, got.size, got.size, 2)
    assert st[0] == 0 and np.array_equal(got, orig)
    got = z.copy()
    oracle.batch_emit(got, None, 1, got.size, got.size, 2, caps=(3, 0, 0, 0, 0))
    assert got[icmp + 18] == 0 and got[icmp + 19] == 0 and got[ip + 10] == 0
    tot = int.from_bytes(bytes(orig[ip + 2:ip + 4]), "big")
    assert pyref.icmpv4_verify(bytes(got[icmp:ip + tot]))
