"""IPv4 fragment groups on the CPU oracle (the restated semantics of smol_csum_batch_emit_frag /
_verify_frag, include/smolcsum.h).

The route the drop-in boundary takes: under offloaded caps the iface emits a
datagram whole with its L4 checksum written 0 and then cuts it into fragments
(src/iface/interface/mod.rs:1276-1331, ipv4.rs:440-490); the device fills the group.  The result
must equal what the reference sends with its default caps: the datagram emitted whole with its
checksums, then fragmented with every fragment header filled.  Receive: every fragment's header
gate plus the reassembled datagram's L4 gate (ipv4.rs:103-146)."""
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
