"""6LoWPAN NHC UDP (src/wire/sixlowpan/nhc.rs) on the CPU: the C oracle and the pure-Python
restatement against the reference's own datagram (tests/golden/kat.json ``sixlowpan_nhc_udp``:
the reassembled UDP datagram of ``sixlowpan_three_fragments``, inline checksum 0xb46b) and against
each other on random packets of every port mode, with and without an inline checksum."""
import numpy as np
import pytest

import oracle
from oracle import pyref
from tests import pktgen as P

ST_ACCEPT, ST_L4_VALID, ST_MALFORMED = 0x80, 0x10, 0x20


def _kat(golden):
    k = golden["sixlowpan_nhc_udp"][0]
    return k, bytes.fromhex(k["bytes"]), bytes.fromhex(k["src"]), bytes.fromhex(k["dst"])


def _one(pkt: bytes):
    return np.frombuffer(pkt, np.uint8).copy()


def test_kat_verifies(golden):
    k, pkt, src, dst = _kat(golden)
    assert pyref.nhc_ports(pkt) == (k["src_port"], k["dst_port"])
    assert pyref.nhc_udp_verify(pkt, src, dst) is True
    addrs = np.frombuffer(src + dst, np.uint8)
    st = oracle.batch_nhc_udp_verify(_one(pkt), None, 1, addrs, len(pkt), len(pkt))
    assert st[0] & ST_ACCEPT and st[0] & ST_L4_VALID
    bad = bytearray(pkt)
    bad[100] ^= 0x40
    assert pyref.nhc_udp_verify(bytes(bad), src, dst) is False
    st = oracle.batch_nhc_udp_verify(_one(bytes(bad)), None, 1, addrs, len(pkt), len(pkt))
    assert not st[0] & ST_ACCEPT
    # caps.udp = None: a wrong checksum is not looked at (L4_VALID still reports it)
    st = oracle.batch_nhc_udp_verify(_one(bytes(bad)), None, 1, addrs, len(pkt), len(pkt), caps=(0, 3, 0, 0, 0))
    assert st[0] & ST_ACCEPT and not st[0] & ST_L4_VALID


def test_kat_construct(golden):
    """Emit over the packet with its checksum zeroed — also with the C bit set, as a packet whose
    checksum was elided — reproduces the reference bytes."""
    k, pkt, src, dst = _kat(golden)
    addrs = np.frombuffer(src + dst, np.uint8)
    for c_bit in (0, 4):
        pre = bytearray(pkt)
        pre[0] |= c_bit
        pre[5] = pre[6] = 0
        py = bytearray(pre)
        assert pyref.nhc_udp_fill(py, src, dst)
        assert bytes(py) == pkt
        buf = _one(bytes(pre))
        st = oracle.batch_nhc_udp_emit(buf, None, 1, addrs, len(pkt), len(pkt))
        assert st[0] == 0 and buf.tobytes() == pkt
    # caps.udp without tx: nothing is written
    buf = _one(bytes(pre))
    oracle.batch_nhc_udp_emit(buf, None, 1, addrs, len(pkt), len(pkt), caps=(0, 1, 0, 0, 0))
    assert buf.tobytes() == bytes(pre)


def random_records(rng, n):
    """Every port mode, inline / elided checksum, payloads 0..199 B, some cut inside the header,
    some with another NHC dispatch."""
    recs = []
    for i in range(n):
        mode, elided = i % 4, bool((i >> 2) & 1)
        r = bytearray(P.nhc_udp(rng, mode, elided, int(rng.integers(0, 200))))
        if i % 23 == 0:
            r = r[: int(rng.integers(0, 1 + P.NHC_PORTS_SIZE[mode] + 2))]
        if i % 29 == 0 and r:
            r[0] = 0xE0 | (r[0] & 7)
        if i % 7 == 3 and mode in (0, 2) and len(r) >= 5:  # destination port 0 (inline)
            r[3 if mode == 0 else 2] = 0
            r[4 if mode == 0 else 3] = 0
        recs.append(bytes(r))
    return recs


def pyref_emit(r: bytes, addrs_row: np.ndarray, caps):
    """(bytes after emit, malformed) by the pure-Python restatement."""
    ok_header = bool(r) and (r[0] >> 3) == 0x1E and len(r) >= 1 + P.NHC_PORTS_SIZE[r[0] & 3] + 2
    py = bytearray(r)
    if ok_header and caps[1] in (0, 2):
        pyref.nhc_udp_fill(py, addrs_row[:16].tobytes(), addrs_row[16:].tobytes())
    return bytes(py), not ok_header


@pytest.mark.parametrize("caps", [(0, 0, 0, 0, 0), (0, 1, 0, 0, 0), (0, 2, 0, 0, 0), (0, 3, 0, 0, 0)])
def test_oracle_vs_pyref_random(caps):
    rng = np.random.default_rng(42 + caps[1])
    recs = random_records(rng, 400)
    addrs = rng.integers(0, 256, (len(recs), 32), dtype=np.uint8)
    buf, offs, lens = P.pack(recs, gap_rng=rng)
    desc = P.oracle_desc(offs, lens, 0)
    st = oracle.batch_nhc_udp_verify(buf.copy(), desc, len(recs), addrs, caps=caps)
    for i, r in enumerate(recs):
        v = pyref.nhc_udp_verify(r, addrs[i, :16].tobytes(), addrs[i, 16:].tobytes())
        if v is None:
            assert st[i] & ST_MALFORMED and not st[i] & ST_ACCEPT, i
            continue
        assert bool(st[i] & ST_L4_VALID) == v, i
        assert bool(st[i] & ST_ACCEPT) == (v or caps[1] in (2, 3)), i
    out = buf.copy()
    est = oracle.batch_nhc_udp_emit(out, desc, len(recs), addrs, caps=caps)
    for i, r in enumerate(recs):
        want, mal = pyref_emit(r, addrs[i], caps)
        assert out[int(offs[i]): int(offs[i]) + int(lens[i])].tobytes() == want, i
        assert bool(est[i] & ST_MALFORMED) == mal, i


def test_emitted_packets_verify():
    """emit -> verify round trip in port modes 0b00 and 0b10.  (Mode 0b01: the reference's parse
    reads the destination from byte 1, nhc.rs:553-559, where its set_ports put it in byte 3; mode
    0b11: set_ports encodes both ports as 0, nhc.rs:641-645.  Both are restated as written.)"""
    rng = np.random.default_rng(7)
    recs = [P.nhc_udp(rng, m, False, int(rng.integers(0, 100))) for m in (0, 2) * 50]
    addrs = rng.integers(0, 256, (len(recs), 32), dtype=np.uint8)
    buf, offs, lens = P.pack(recs, gap_rng=rng)
    desc = P.oracle_desc(offs, lens, 0)
    oracle.batch_nhc_udp_emit(buf, desc, len(recs), addrs)
    st = oracle.batch_nhc_udp_verify(buf, desc, len(recs), addrs)
    assert all(s & ST_ACCEPT for s in st)
