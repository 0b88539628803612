"""Status semantics on the CPU oracle: the port tests Repr::parse makes before its checksum gate,
and raw-socket records (SMOL_REC_IPHDR_ONLY).  The GPU side of both is tests/test_gpu_status.py.

* UdpRepr::parse rejects destination port 0 before it looks at the checksum
  (src/wire/udp.rs:246-248); TcpRepr::parse rejects source or destination port 0
  (src/wire/tcp.rs:910-915).  Verify reports such records SMOL_ST_MALFORMED, never ACCEPT; emit
  fills them (Repr::emit checks no ports).
* A raw socket's frame: dispatch copies the user's L4 bytes verbatim (src/iface/packet.rs:132-136)
  and only the IPv4 header is emitted (src/socket/raw.rs:406-423); on receive the raw socket sees
  the packet after the IPv4 gate, before any L4 gate (src/iface/interface/ipv4.rs:150-151).
"""
import numpy as np
import pytest

import oracle
from tests import pktgen as P

A4, B4 = bytes([192, 168, 1, 1]), bytes([192, 168, 1, 2])
A6, B6 = bytes([0xFE, 0x80] + [0] * 13 + [1]), bytes([0xFE, 0x80] + [0] * 13 + [2])
ST_IP_OK, ST_L4_OK, ST_IP_VALID, ST_L4_VALID = 0x01, 0x02, 0x08, 0x10
ST_MALFORMED, ST_UNSUPPORTED, ST_ACCEPT = 0x20, 0x40, 0x80
RAW = oracle.REC_IPHDR_ONLY


def port_records(rng):
    """(record, verify-MALFORMED expected) over UDP / TCP, IPv4 / IPv6, every port zero pattern."""
    out = []
    for fam in (4, 6):
        for proto in (17, 6):
            for sp, dp in ((0, 0), (0, 53), (53, 0), (1234, 53)):
                pay = P.rand_bytes(rng, int(rng.integers(0, 300)))
                l4 = P.udp(sp, dp, pay) if proto == 17 else P.tcp(sp, dp, pay)
                rec = P.ipv4(A4, B4, proto, l4) if fam == 4 else P.ipv6(A6, B6, proto, l4)
                bad = dp == 0 if proto == 17 else (sp == 0 or dp == 0)
                out.append((rec, bad))
    return out


def test_port_zero_verify_malformed_emit_fills():
    rng = np.random.default_rng(1)
    recs = port_records(rng)
    buf, offs, lens = P.pack([r for r, _ in recs], gap_rng=rng)
    est = P.oracle_emit_records(buf, offs, lens, 1)
    assert not est.any(), "emit does not reject ports"
    st = P.oracle_verify_records(buf, offs, lens, 1)
    for (rec, bad), s in zip(recs, st):
        if bad:
            assert s & ST_MALFORMED and not s & ST_ACCEPT
            # the L4 gate was never reached: its bits say "not checked"
            assert s & ST_L4_OK and s & ST_L4_VALID
        else:
            assert s & ST_ACCEPT and not s & ST_MALFORMED
    # the emitted checksum is still the reference's (a record with its ports fixed verifies)
    for i, (rec, bad) in enumerate(recs):
        if not bad:
            continue
        o, n = int(offs[i]), int(lens[i])
        r = buf[o:o + n].copy()
        l4 = 20 if r[0] >> 4 == 4 else 40
        assert oracle.lib().oracle_record_verify(r.ctypes.data, n, 1, oracle.caps_c()) & ST_MALFORMED
        if r[0] >> 4 == 4:
            is_udp = r[9] == 17
            ok = oracle.lib().oracle_udp_verify(r[l4:].ctypes.data, 4, r[12:].ctypes.data, r[16:].ctypes.data) \
                if is_udp else oracle.lib().oracle_tcp_verify(r[l4:].ctypes.data, n - l4, 4, r[12:].ctypes.data,
                                                               r[16:].ctypes.data)
            assert ok


def test_port_zero_caps_none_still_malformed():
    """The port test precedes the caps gate: with checksums off the record is still dropped."""
    rng = np.random.default_rng(2)
    recs = port_records(rng)
    buf, offs, lens = P.pack([r for r, _ in recs])
    P.oracle_emit_records(buf, offs, lens, 1)
    st = P.oracle_verify_records(buf, offs, lens, 1, caps=(3, 3, 3, 3, 3))
    for (_, bad), s in zip(recs, st):
        assert bool(s & ST_MALFORMED) == bad and bool(s & ST_ACCEPT) == (not bad)


def raw_records(rng):
    """Raw-socket frames: arbitrary L4 bytes (wrong or partial checksums, port 0, truncated),
    IPv4 (options too) and IPv6, Ethernet-framed or not."""
    out = []
    for i in range(24):
        pay = P.rand_bytes(rng, int(rng.integers(0, 200)))
        k = i % 6
        if k == 0:
            l4 = P.udp(0, 0, pay, csum=0xBEEF)
        elif k == 1:
            l4 = P.tcp(1, 2, pay, csum=0x1234)
        elif k == 2:
            l4 = pay[:3]  # shorter than any L4 header
        elif k == 3:
            l4 = P.icmp_echo(8, pay, csum=0xFFFF)
        else:
            l4 = pay
        proto = (17, 6, 17, 1, 253, 89)[k]
        if i % 4 == 3:
            rec = P.ipv6(A6, B6, proto if proto != 1 else 58, l4)
        else:
            rec = P.ipv4(A4, B4, proto, l4, ihl=5 + (i % 3), csum=0x5A5A)
        out.append(P.eth(rec, 0x86DD if rec[0] >> 4 == 6 else 0x0800) if i % 5 == 0 else rec)
    return out


@pytest.mark.parametrize("fixed", [False, True])
def test_iphdr_only_emit_header_only(fixed):
    rng = np.random.default_rng(3)
    recs = raw_records(rng)
    if fixed:
        recs = [r for r in recs if r[0] >> 4 in (4, 6)]
        L = max(len(r) for r in recs)
        recs = [r + bytes(L - len(r)) for r in recs]
        buf = np.frombuffer(b"".join(recs) + bytes(16), np.uint8).copy()
        before = buf.copy()
        st = oracle.batch_emit(buf, None, len(recs), L, L, oracle.kind_flags(1, RAW))
        offs, lens = np.arange(len(recs)) * L, np.full(len(recs), L)
        kinds = [1] * len(recs)
    else:
        buf, offs, lens = P.pack(recs, gap_rng=rng)
        before = buf.copy()
        kinds = [2 if r[0] == 0x02 else 1 for r in recs]
        desc = P.oracle_desc(offs, lens, kinds, RAW)
        st = oracle.batch_emit(buf, desc, len(desc))
    assert (st == ST_UNSUPPORTED).all()
    for o, n, k in zip(offs, lens, kinds):
        o, n = int(o), int(n)
        io = 14 if k == 2 else 0
        ip = before[o + io:o + n]
        after = buf[o + io:o + n]
        if ip[0] >> 4 == 4:
            hl = (ip[0] & 15) * 4
            assert np.array_equal(after[hl:], ip[hl:]), "L4 bytes are the user's"
            assert oracle.lib().oracle_ipv4_verify(after.ctypes.data)
            assert not np.array_equal(after[10:12], ip[10:12]) or oracle.lib().oracle_ipv4_verify(ip.ctypes.data)
        else:
            assert np.array_equal(after, ip), "IPv6: nothing to write"
    # ignored caps.ipv4: the header field written 0, the rest untouched
    if not fixed:
        b2 = before.copy()
        oracle.batch_emit(b2, desc, len(desc), caps=(3, 0, 0, 0, 0))
        for o, n, k in zip(offs, lens, kinds):
            ip = b2[int(o) + (14 if k == 2 else 0):int(o) + int(n)]
            if ip[0] >> 4 == 4:
                assert ip[10] == 0 and ip[11] == 0


def test_iphdr_only_verify_ip_gate_only():
    rng = np.random.default_rng(4)
    recs = raw_records(rng)
    buf, offs, lens = P.pack(recs, gap_rng=rng)
    kinds = [2 if r[0] == 0x02 else 1 for r in recs]
    desc = P.oracle_desc(offs, lens, kinds, RAW)
    oracle.batch_emit(buf, desc, len(desc))
    st = oracle.batch_verify(buf, desc, len(desc))
    # every raw frame passes: its IPv4 header was filled, its L4 bytes are not looked at
    assert ((st & 0xBF) == (ST_IP_OK | ST_L4_OK | ST_IP_VALID | ST_L4_VALID | ST_ACCEPT)).all()
    assert (st & ST_UNSUPPORTED).all()
    # a header bit flip is still caught by the IPv4 gate
    i = next(j for j, r in enumerate(recs) if kinds[j] == 1 and r[0] >> 4 == 4)
    buf[int(offs[i]) + 8] ^= 1
    st = oracle.batch_verify(buf, desc, len(desc))
    assert not st[i] & ST_ACCEPT and not st[i] & ST_IP_VALID
    # without the flag the same bytes reach the L4 gates (and most of them fail there)
    plain = P.oracle_desc(offs, lens, kinds)
    assert (oracle.batch_verify(buf, plain, len(plain)) & ST_ACCEPT).sum() < (st & ST_ACCEPT).sum()
