"""IPv4 fragment groups on the CPU oracle (the restated semantics of smol_csum_batch_emit_frag /
_verify_frag, include/smolcsum.h).

The route the drop-in boundary takes: under offloaded caps the iface emits a
datagram whole with its L4 checksum written 0 and then cuts it into fragments
(src/iface/interface/mod.rs:1276-1331, ipv4.rs:421-490); the device fills the group with the RFC
checksum of the reassembled datagram: the datagram emitted whole with its checksums, then
fragmented with every fragment header filled.  Receive: every fragment's header gate plus the
reassembled datagram's L4 gate (ipv4.rs:103-146).

The reference's OWN software route differs for TCP and ICMPv4: dispatch_ip emits into the whole
fixed-size frag.buffer, so those checksums cover the buffer's tail (mod.rs:1263-1267,1320;
packet.rs:80-83,166-171).  `test_reference_route_*` restate that route
(oracle_emit_like_dispatch_ip) and pin where the engine deliberately differs."""
import numpy as np
import pytest

import oracle
from tests import pktgen as P

A, B = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
DEFAULT, IGNORED = (0, 0, 0, 0, 0), (3, 3, 3, 3, 3)
ST_ACCEPT, ST_MALFORMED, ST_UNSUPPORTED, ST_L4_VALID, ST_IP_VALID = 0x80, 0x20, 0x40, 0x10, 0x08


def datagrams(rng, n, lo=600, hi=4000):
    out = []
    for i in range(n):
        pay = P.rand_bytes(rng, int(rng.integers(lo, hi)))
        k = i % 4
        if k == 0:
            out.append(P.ipv4(A, B, 17, P.udp(5000 + i, 53, pay), flags_frag=0x4000))
        elif k == 1:
            out.append(P.ipv4(A, B, 6, P.tcp(6000 + i, 80, pay), flags_frag=0x4000))
        elif k == 2:
            out.append(P.ipv4(A, B, 1, P.icmp_echo(8, pay), flags_frag=0x4000))
        else:  # an ICMPv4 error carrying an embedded header (filled by the group emit too)
            inner = P.ipv4(B, A, 17, P.udp(7, 9, pay[:200]))
            out.append(P.ipv4(A, B, 1, P.icmp4_error(3, 3, inner + pay[200:]), flags_frag=0x4000))
    return out


def emit_whole(d: bytes, caps) -> bytes:
    a = np.frombuffer(d, np.uint8).copy()
    oracle.batch_emit(a, None, 1, a.size, a.size, 1, caps)
    return a.tobytes()


def tx_pair(dgrams, mtu, eth=False, shuffle_rng=None):
    """(offloaded fragments, reference fragments, groups) for a list of datagrams."""
    off, ref, groups, first = [], [], [], 0
    for i, d in enumerate(dgrams):
        fo = P.fragment_like_iface(emit_whole(d, IGNORED), mtu, 0x4000 + i, fill_header=False)
        fr = P.fragment_like_iface(emit_whole(d, DEFAULT), mtu, 0x4000 + i, fill_header=True)
        order = list(range(len(fo)))
        if shuffle_rng is not None:
            shuffle_rng.shuffle(order)
        fo, fr = [fo[j] for j in order], [fr[j] for j in order]
        if eth:
            fo, fr = [P.eth(x) for x in fo], [P.eth(x) for x in fr]
        off += fo
        ref += fr
        groups.append((first, len(fo)))
        first += len(fo)
    return off, ref, groups


def pack(recs, groups, seed=0):
    buf, offs, lens = P.pack(recs, gap_rng=np.random.default_rng(seed))
    return buf, offs, lens, oracle.FRAG_GROUP_DTYPE, np.array([(f, c, 0) for f, c in groups], dtype=oracle.FRAG_GROUP_DTYPE)


@pytest.mark.parametrize("mtu,eth", [(576, False), (1280, True), (1500, False), (68, False)])
def test_group_emit_equals_emit_then_fragment(mtu, eth):
    rng = np.random.default_rng(mtu)
    dg = datagrams(rng, 16, 60 if mtu == 68 else 600, 900 if mtu == 68 else 4000)
    off, ref, groups = tx_pair(dg, mtu, eth, shuffle_rng=rng)
    buf, offs, lens, _, g = pack(off, groups, mtu)
    kind = 2 if eth else 1
    desc = P.oracle_desc(offs, lens, kind)
    st = oracle.batch_emit_frag(buf, desc, len(desc), g)
    for o, ln, want in zip(offs, lens, ref):
        assert buf[int(o):int(o) + int(ln)].tobytes() == want
    assert not st.any()
    vst = oracle.batch_verify_frag(buf, desc, len(desc), g)
    assert (vst & ST_ACCEPT).all() and (vst & ST_L4_VALID).all()


def test_group_of_one_equals_plain_emit_verify():
    rng = np.random.default_rng(1)
    recs = [emit_whole(d, IGNORED) for d in datagrams(rng, 12, 20, 1400)]
    buf, offs, lens, _, g = pack(recs, [(i, 1) for i in range(len(recs))])
    desc = P.oracle_desc(offs, lens, 1)
    a, b = buf.copy(), buf.copy()
    for caps in (DEFAULT, (2, 3, 0, 1, 0), (3, 2, 2, 3, 3)):
        s1 = oracle.batch_emit_frag(a, desc, len(desc), g, caps=caps)
        s2 = oracle.batch_emit(b, desc, len(desc), caps=caps)
        assert np.array_equal(a, b) and np.array_equal(s1, s2)
        assert np.array_equal(oracle.batch_verify_frag(a, desc, len(desc), g, caps=caps),
                              oracle.batch_verify(a, desc, len(desc), caps=caps))


def test_group_verify_rejections():
    rng = np.random.default_rng(7)
    dg = datagrams(rng, 4, 2000, 3000)
    _, ref, groups = tx_pair(dg, 576)
    base, offs, lens, _, g = pack(ref, groups)
    desc = P.oracle_desc(offs, lens, 1)
    assert (oracle.batch_verify_frag(base, desc, len(desc), g) & ST_ACCEPT).all()
    f0, c0 = groups[0]
    # a payload bit flip in the last fragment: L4 fails for the whole datagram, headers stay valid
    b = base.copy()
    o = int(offs[f0 + c0 - 1]) + 30
    b[o] ^= 0x10
    st = oracle.batch_verify_frag(b, desc, len(desc), g)
    assert not (st[f0:f0 + c0] & (ST_ACCEPT | ST_L4_VALID)).any() and (st[f0:f0 + c0] & ST_IP_VALID).all()
    assert (st[f0 + c0:] & ST_ACCEPT).all()
    # a header bit flip in fragment 1: that fragment's header is invalid, the datagram is dropped
    b = base.copy()
    b[int(offs[f0 + 1]) + 8] ^= 0x01  # TTL: not part of the reassembly key
    st = oracle.batch_verify_frag(b, desc, len(desc), g)
    assert not (st[f0:f0 + c0] & ST_ACCEPT).any() and not st[f0 + 1] & ST_IP_VALID and st[f0] & ST_IP_VALID
    # caps.ipv4 = Tx (no rx check): the same datagram is accepted
    st = oracle.batch_verify_frag(b, desc, len(desc), g, caps=(2, 0, 0, 0, 0))
    assert (st[f0:f0 + c0] & ST_ACCEPT).all()


def test_group_contract_violations_malformed():
    rng = np.random.default_rng(9)
    dg = datagrams(rng, 1, 2500, 2600)
    _, ref, _ = tx_pair(dg, 576)
    n = len(ref)
    cases = {
        "missing middle": [ref[i] for i in range(n) if i != 1],
        "missing last": ref[:-1],
        "duplicate": ref + [ref[1]],
        "other ident": ref[:1] + [ref[1][:4] + b"\x12\x34" + ref[1][6:]] + ref[2:],
        "two last": ref[:-1] + [ref[-1], ref[-1][:6] + bytes([ref[-1][6] & 0x1f]) + ref[-1][7:]],
    }
    for name, recs in cases.items():
        buf, offs, lens, _, g = pack(recs, [(0, len(recs))])
        desc = P.oracle_desc(offs, lens, 1)
        before = buf.copy()
        st = oracle.batch_emit_frag(buf, desc, len(desc), g)
        assert (st & ST_MALFORMED).all(), name
        vst = oracle.batch_verify_frag(before, desc, len(desc), g)
        assert (vst & ST_MALFORMED).all() and not (vst & ST_ACCEPT).any(), name


# ---- the reference's own route: dispatch_ip into the whole frag.buffer --------------------------

FRAG_BUFFER_SIZES = (1500, 4096)  # build.rs:15 default; lib.rs:156, the reference's test config


def reference_route(d: bytes, fbuf_size: int, tail: bytes, mtu: int, ident: int):
    """What the reference sends with its default caps for datagram `d` (checksum fields 0), emitted
    into a frag.buffer of `fbuf_size` bytes whose bytes past the datagram are `tail`: (rc,
    fragments)."""
    assert len(d) + len(tail) == fbuf_size
    fb = np.frombuffer(d + tail, np.uint8).copy()
    rc = oracle.emit_like_dispatch_ip(fb, DEFAULT)
    return rc, (P.fragment_like_iface(fb[:len(d)].tobytes(), mtu, ident, fill_header=True) if rc == 0 else None)


def engine_route(d: bytes, mtu: int, ident: int):
    """The offload route: fragments of the datagram emitted under ignored caps, then the group emit."""
    fo = P.fragment_like_iface(emit_whole(d, IGNORED), mtu, ident, fill_header=False)
    buf, offs, lens, _, g = pack(fo, [(0, len(fo))])
    desc = P.oracle_desc(offs, lens, 1)
    st = oracle.batch_emit_frag(buf, desc, len(desc), g)
    assert not st.any()
    return [buf[int(o):int(o) + int(n)].tobytes() for o, n in zip(offs, lens)]


def verify_group(frags):
    buf, offs, lens, _, g = pack(frags, [(0, len(frags))])
    desc = P.oracle_desc(offs, lens, 1)
    return oracle.batch_verify_frag(buf, desc, len(desc), g)


def route_datagram(rng, proto, size):
    pay = P.rand_bytes(rng, size)
    if proto == 17:
        return P.ipv4(A, B, 17, P.udp(5000, 53, pay[:size - 28]), flags_frag=0x4000)
    if proto == 6:
        return P.ipv4(A, B, 6, P.tcp(6000, 80, pay[:size - 40]), flags_frag=0x4000)
    return P.ipv4(A, B, 1, P.icmp_echo(8, pay[:size - 28]), flags_frag=0x4000)


@pytest.mark.parametrize("fbuf", FRAG_BUFFER_SIZES)
def test_reference_route_udp_identical(fbuf):
    """UDP: UdpPacket::fill_checksum covers the length field's span (udp.rs:194-208), so the
    reference's fragments equal the engine's whatever the buffer tail holds."""
    rng = np.random.default_rng(fbuf)
    mtu = 576 if fbuf == 1500 else 1500
    for size in (mtu + 1, (mtu + fbuf) // 2, fbuf):
        d = route_datagram(rng, 17, size)
        for tail in (bytes(fbuf - size), P.rand_bytes(rng, fbuf - size)):
            rc, ref = reference_route(d, fbuf, tail, mtu, 0x77)
            assert rc == 0 and ref == engine_route(d, mtu, 0x77)
            assert (verify_group(ref) & ST_ACCEPT).all()


@pytest.mark.parametrize("fbuf", FRAG_BUFFER_SIZES)
def test_reference_route_tcp_differs(fbuf):
    """TCP: TcpPacket::fill_checksum sums the whole buffer tail and puts its length in the
    pseudo-header (tcp.rs:616-626), so whenever the datagram is shorter than frag.buffer the
    reference's checksum differs from the engine's RFC checksum, and the reference's own
    reassembling receive path (the group verify) rejects it; the engine's is accepted.  A datagram
    that fills the buffer exactly is the one case where both agree."""
    rng = np.random.default_rng(fbuf + 1)
    mtu = 576 if fbuf == 1500 else 1500
    for size in (mtu + 1, (mtu + fbuf) // 2, fbuf - 1):
        d = route_datagram(rng, 6, size)
        eng = engine_route(d, mtu, 0x78)
        assert (verify_group(eng) & ST_ACCEPT).all()
        for tail in (bytes(fbuf - size), P.rand_bytes(rng, fbuf - size)):
            rc, ref = reference_route(d, fbuf, tail, mtu, 0x78)
            assert rc == 0 and ref != eng
            # only the TCP checksum field differs: same fragments, same headers, same payload bytes
            diff = [i for i, (x, y) in enumerate(zip(ref, eng)) if x != y]
            assert diff == [0] and len(ref) == len(eng)
            assert [k for k in range(len(ref[0])) if ref[0][k] != eng[0][k]] in ([36], [37], [36, 37])
            st = verify_group(ref)
            assert not (st & (ST_ACCEPT | ST_L4_VALID)).any() and (st & ST_IP_VALID).all()
    d = route_datagram(rng, 6, fbuf)
    rc, ref = reference_route(d, fbuf, b"", mtu, 0x79)
    assert rc == 0 and ref == engine_route(d, mtu, 0x79)


@pytest.mark.parametrize("fbuf", FRAG_BUFFER_SIZES)
def test_reference_route_icmpv4(fbuf):
    """ICMPv4 echo: Icmpv4Packet::fill_checksum sums the whole tail (icmpv4.rs:339-346, 502-503):
    identical to the engine when the tail is zero, different (and rejected by the reassembling
    receiver) when it holds stale bytes.  An error message with a tail makes the reference panic
    (copy_from_slice, icmpv4.rs:529-530)."""
    rng = np.random.default_rng(fbuf + 2)
    mtu = 576 if fbuf == 1500 else 1500
    for size in (mtu + 1, (mtu + fbuf) // 2, fbuf - 2):
        d = route_datagram(rng, 1, size)
        eng = engine_route(d, mtu, 0x7A)
        rc, ref = reference_route(d, fbuf, bytes(fbuf - size), mtu, 0x7A)
        assert rc == 0 and ref == eng
        tail = P.rand_bytes(rng, fbuf - size)
        if not any(tail[0::2]) and not any(tail[1::2]):
            continue
        rc, ref = reference_route(d, fbuf, tail, mtu, 0x7A)
        assert rc == 0 and ref != eng
        assert not (verify_group(ref) & ST_ACCEPT).any()
    inner = P.ipv4(B, A, 17, P.udp(7, 9, P.rand_bytes(rng, 600)))
    d = P.ipv4(A, B, 1, P.icmp4_error(3, 3, inner), flags_frag=0x4000)
    fb = np.frombuffer(d + bytes(fbuf - len(d)), np.uint8).copy()
    assert oracle.emit_like_dispatch_ip(fb, DEFAULT) == (0 if len(d) == fbuf else -2)


def test_reference_route_drops_oversize():
    """frag.buffer shorter than the datagram: dispatch_ip drops it (mod.rs:1293-1298)."""
    rng = np.random.default_rng(3)
    d = np.frombuffer(route_datagram(rng, 17, 1600), np.uint8).copy()
    assert oracle.emit_like_dispatch_ip(d[:1500].copy(), DEFAULT) == -1


# ---- group validity (include/smolcsum.h: invalid groups are not read or written) ---------------

def test_invalid_groups_untouched():
    rng = np.random.default_rng(11)
    dg = datagrams(rng, 2, 2000, 2500)
    off, _, groups = tx_pair(dg, 576)
    buf, offs, lens, _, g = pack(off, groups)
    n = len(offs)
    desc = P.oracle_desc(offs, lens, 1)
    f0, c0 = groups[0]
    bad = np.array([(n, 1, 0), (n - 1, 2, 0), (f0, c0, 1), (f0, 0, 0), (2**63, 3, 0), (1, 2**32 - 1, 0)],
                   dtype=oracle.FRAG_GROUP_DTYPE)
    before = buf.copy()
    for caps in (DEFAULT, IGNORED):
        st = oracle.batch_emit_frag(buf, desc, n, bad, caps=caps)
        assert np.array_equal(buf, before) and not st.any()
        assert not oracle.batch_verify_frag(buf, desc, n, bad, caps=caps).any()
    # a valid group next to the invalid ones is still served
    mixed = np.concatenate([bad[:2], g[:1]])
    st = oracle.batch_emit_frag(buf, desc, n, mixed)
    assert not np.array_equal(buf, before) and not st.any()
    assert (oracle.batch_verify_frag(buf, desc, n, mixed)[f0:f0 + c0] & ST_ACCEPT).all()


def test_raw_group_headers_only():
    """SMOL_REC_IPHDR_ONLY on any record of a group: a raw socket's datagram, headers only."""
    rng = np.random.default_rng(12)
    dg = datagrams(rng, 4, 1500, 2500)
    off, _, groups = tx_pair(dg, 576)
    buf, offs, lens, _, g = pack(off, groups)
    n = len(offs)
    flags = np.zeros(n, np.uint8)
    f1, c1 = groups[1]
    flags[f1 + c1 - 1] = oracle.REC_IPHDR_ONLY
    desc = P.oracle_desc(offs, lens, 1, flags)
    ref = buf.copy()
    st = oracle.batch_emit_frag(buf, desc, n, g)
    assert (st[f1:f1 + c1] == ST_UNSUPPORTED).all() and not np.delete(st, range(f1, f1 + c1)).any()
    for i in range(f1, f1 + c1):  # only the fragment headers changed, and they are valid
        o, ln = int(offs[i]), int(lens[i])
        assert np.array_equal(buf[o + 20:o + ln], ref[o + 20:o + ln])
        assert oracle.lib().oracle_ipv4_verify(buf[o:].ctypes.data)
    vst = oracle.batch_verify_frag(buf, desc, n, g)
    assert (vst[f1:f1 + c1] & ST_ACCEPT).all() and (vst[f1:f1 + c1] & ST_UNSUPPORTED).all()
