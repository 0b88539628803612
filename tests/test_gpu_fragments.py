"""IPv4 fragmentation refill on the GPU: the iface fragments an IPv4
datagram that exceeds the MTU (src/iface/interface/mod.rs:1276-1331, src/iface/interface/ipv4.rs:
440-490).  The datagram is emitted whole first — its L4 checksum covers the whole payload — and
every fragment then gets its own IPv4 header (ident, MF, fragment offset) and
Ipv4Packet::fill_checksum under caps.ipv4.tx().

Here: UDP / TCP / ICMP datagrams of 3-9 KB are emitted whole on the device; the host cuts them into
MTU-sized fragments the way the iface does (8-byte-aligned fragment data, the header of the
datagram with total length, MF and offset rewritten, its checksum left stale); the device emits the
fragments (IPv4 header only: a fragment has no L4 gate) and verifies them; the host reassembles the
fragment payloads and the device verifies the reassembled datagram.  Every device result is
compared with the oracle bit for bit.
"""
import numpy as np
import pytest

import oracle
from tests import pktgen as P

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smoltcp_amd import engine as E  # noqa: E402
from tests.engines import VariantEngine  # noqa: E402


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    e = VariantEngine(0)
    yield e
    e.close()


def _device_emit(eng, recs, caps=(0, 0, 0, 0, 0), gap_seed=None):
    rng = np.random.default_rng(gap_seed) if gap_seed is not None else None
    buf, offs, lens = P.pack(recs, gap_rng=rng)
    batch = E.Batch.from_records(offs, lens, E.KIND_IP, "cuda:0")
    d = torch.from_numpy(buf.copy()).cuda()
    st = torch.zeros(len(recs), dtype=torch.uint8, device="cuda:0")
    eng.emit(d, batch, caps=caps, status=st)
    got = d.cpu().numpy()
    ref = buf.copy()
    ref_st = P.oracle_emit_records(ref, offs, lens, np.full(len(recs), E.KIND_IP, np.uint8), caps)
    assert np.array_equal(got, ref)
    assert np.array_equal(st.cpu().numpy(), ref_st)
    vst = eng.verify(d, batch, caps=caps).cpu().numpy()
    assert np.array_equal(vst, P.oracle_verify_records(got, offs, lens, np.full(len(recs), E.KIND_IP, np.uint8), caps))
    return [got[int(o): int(o) + int(n)].tobytes() for o, n in zip(offs, lens)], vst


def _fragment(dgram: bytes, mtu: int, ident: int):
    """Cut an IPv4 datagram (20-byte header) into fragments of at most `mtu` bytes: fragment data
    in multiples of 8 bytes (Ipv4 max_ipv4_fragment_size), the datagram's header with total length,
    ident, MF and offset rewritten; the header checksum is left as it was (stale)."""
    hdr, data = bytearray(dgram[:20]), dgram[20:]
    step = (mtu - 20) // 8 * 8
    frags = []
    for off in range(0, len(data), step):
        part = data[off: off + step]
        h = bytearray(hdr)
        h[2:4] = (20 + len(part)).to_bytes(2, "big")
        h[4:6] = ident.to_bytes(2, "big")
        more = off + step < len(data)
        h[6:8] = ((0x2000 if more else 0) | (off // 8)).to_bytes(2, "big")
        frags.append(bytes(h) + part)
    return frags


@pytest.mark.parametrize("mtu", [576, 1280, 1500])
def test_fragment_refill_and_reassembly(eng, mtu):
    rng = np.random.default_rng(mtu)
    a, b = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    dgrams = []
    for i in range(48):
        pay = P.rand_bytes(rng, int(rng.integers(3000, 9000)))
        kind = i % 3
        if kind == 0:
            dgrams.append(P.ipv4(a, b, 17, P.udp(5000 + i, 53, pay), flags_frag=0))
        elif kind == 1:
            dgrams.append(P.ipv4(a, b, 6, P.tcp(6000 + i, 80, pay), flags_frag=0))
        else:
            dgrams.append(P.ipv4(a, b, 1, P.icmp_echo(8, pay), flags_frag=0))
    # 1. the whole datagrams: IPv4 header + L4 checksum over the whole payload
    whole, vst = _device_emit(eng, dgrams, gap_seed=1)
    assert all(s & E.ST_ACCEPT and s & E.ST_L4_VALID for s in vst)
    # 2. the fragments: header refill only (a fragment has no L4 gate: UNSUPPORTED)
    frags, owner = [], []
    for i, d in enumerate(whole):
        f = _fragment(d, mtu, ident=0x1000 + i)
        frags += f
        owner += [i] * len(f)
    for caps in ((0, 0, 0, 0, 0), (3, 0, 0, 0, 0)):
        out, fst = _device_emit(eng, frags, caps=caps, gap_seed=2)
        if caps[0] == 0:
            assert all(s & E.ST_IP_VALID and s & E.ST_UNSUPPORTED and s & E.ST_ACCEPT for s in fst)
            refilled = out
    # 3. reassembly: the fragment payloads give back the datagram, whose checksums verify
    for i, d in enumerate(whole):
        parts = [f for f, o in zip(refilled, owner) if o == i]
        data = b"".join(f[20:] for f in parts)
        assert data == d[20:]
    _, rst = _device_emit(eng, [d for d in whole], gap_seed=3)
    assert all(s & E.ST_ACCEPT for s in rst)


# ---------------------------------------------------------------------------------------------
# Fragment groups through the drop-in route (smol_csum_batch_emit_frag / _verify_frag): the iface
# fragments first with the L4 field and every header checksum written 0 by the offloaded caps;
# the device fills each group; the bytes must equal the reference's "emit whole, then fragment".
# ---------------------------------------------------------------------------------------------

from tests import test_frag_cpu as F  # noqa: E402


def _groups_dev(groups):
    g = E.make_groups([f for f, _ in groups], [c for _, c in groups])
    return torch.from_numpy(g.view(np.uint8).copy()).cuda(), g


def _device_frag(eng, recs, groups, kind, caps=(0, 0, 0, 0, 0), seed=0):
    buf, offs, lens = P.pack(recs, gap_rng=np.random.default_rng(seed))
    batch = E.Batch.from_records(offs, lens, kind, "cuda:0")
    gd, gh = _groups_dev(groups)
    d = torch.from_numpy(buf.copy()).cuda()
    st = torch.zeros(len(recs), dtype=torch.uint8, device="cuda:0")
    eng.emit_frag(d, batch, gd, caps=caps, status=st)
    got = d.cpu().numpy()
    ref = buf.copy()
    desc = P.oracle_desc(offs, lens, kind)
    ref_st = oracle.batch_emit_frag(ref, desc, len(desc), gh, caps=caps)
    diff = np.nonzero(got != ref)[0]
    assert diff.size == 0, diff[:8]
    assert np.array_equal(st.cpu().numpy(), ref_st)
    vst = eng.verify_frag(d, batch, gd, caps=caps).cpu().numpy()
    assert np.array_equal(vst, oracle.batch_verify_frag(ref, desc, len(desc), gh, caps=caps))
    return got, offs, lens, vst


@pytest.mark.parametrize("mtu,eth", [(576, False), (1280, True), (1500, False), (68, True)])
def test_group_emit_drop_in_route(eng, mtu, eth):
    rng = np.random.default_rng(mtu + 1)
    small = mtu == 68
    dg = F.datagrams(rng, 40, 60 if small else 600, 900 if small else 8000)
    off, ref, groups = F.tx_pair(dg, mtu, eth, shuffle_rng=rng)
    got, offs, lens, vst = _device_frag(eng, off, groups, E.KIND_ETH if eth else E.KIND_IP, seed=mtu)
    for o, ln, want in zip(offs, lens, ref):
        assert got[int(o):int(o) + int(ln)].tobytes() == want
    assert (vst & E.ST_ACCEPT).all()


def test_group_caps_and_one_record_groups(eng):
    """Every caps row; groups of one unfragmented packet mixed with fragmented datagrams."""
    rng = np.random.default_rng(11)
    dg = F.datagrams(rng, 24, 300, 3000)
    off, _, groups = F.tx_pair(dg, 1280, shuffle_rng=rng)
    singles = [F.emit_whole(d, F.IGNORED) for d in F.datagrams(rng, 8, 20, 1200)]
    recs = off + singles
    groups = groups + [(len(off) + i, 1) for i in range(len(singles))]
    for caps in ((0, 0, 0, 0, 0), (3, 0, 0, 0, 0), (0, 3, 3, 3, 0), (2, 1, 2, 1, 3), (1, 2, 1, 2, 0)):
        _device_frag(eng, recs, groups, E.KIND_IP, caps=caps, seed=sum(caps))


def test_group_verify_rejects_corrupted_and_broken(eng):
    """RX: a corrupted reassembled datagram is rejected for every fragment, a corrupted header only
    drops its datagram, and groups that break the contract are MALFORMED — all as the oracle."""
    rng = np.random.default_rng(12)
    dg = F.datagrams(rng, 30, 1500, 6000)
    _, ref, groups = F.tx_pair(dg, 576, shuffle_rng=rng)
    recs = [bytearray(r) for r in ref]
    for gi, (f, c) in enumerate(groups):
        if gi % 3 == 0:  # payload flip somewhere in the datagram
            r = recs[f + int(rng.integers(c))]
            r[20 + int(rng.integers(len(r) - 20))] ^= 1 << int(rng.integers(8))
        elif gi % 3 == 1:  # header flip (TTL) in one fragment
            recs[f + int(rng.integers(c))][8] ^= 0x04
    recs = [bytes(r) for r in recs]
    # contract breakers appended: a missing fragment, a duplicate, an ident mismatch
    _, extra, eg = F.tx_pair(F.datagrams(rng, 3, 2500, 2600), 576)
    base = len(recs)
    (f0, c0), (f1, c1), (f2, c2) = eg
    broken = [extra[f0:f0 + c0 - 1], extra[f1:f1 + c1] + [extra[f1]],
              [extra[f2][:4] + b"\x55\x55" + extra[f2][6:]] + extra[f2 + 1:f2 + c2]]
    for b in broken:
        groups.append((base, len(b)))
        recs += b
        base += len(b)
    buf, offs, lens = P.pack(recs, gap_rng=np.random.default_rng(5))
    batch = E.Batch.from_records(offs, lens, E.KIND_IP, "cuda:0")
    gd, gh = _groups_dev(groups)
    d = torch.from_numpy(buf.copy()).cuda()
    for caps in ((0, 0, 0, 0, 0), (2, 0, 0, 0, 0), (0, 2, 2, 2, 0)):
        vst = eng.verify_frag(d, batch, gd, caps=caps).cpu().numpy()
        desc = P.oracle_desc(offs, lens, E.KIND_IP)
        assert np.array_equal(vst, oracle.batch_verify_frag(buf, desc, len(desc), gh, caps=caps)), caps
        if caps == (0, 0, 0, 0, 0):
            for gi, (f, c) in enumerate(groups[:30]):
                assert bool((vst[f:f + c] & E.ST_ACCEPT).all()) == (gi % 3 == 2), gi
            assert (vst[len(ref):] & E.ST_MALFORMED).all()


def test_group_fixed_stride(eng):
    """Fragment records at a fixed stride (a device RX ring), groups over them."""
    rng = np.random.default_rng(13)
    off, ref, groups = F.tx_pair(F.datagrams(rng, 20, 1000, 5000), 1500, shuffle_rng=rng)
    stride = 1501
    host = np.zeros(len(off) * stride + 64, np.uint8)
    for i, r in enumerate(off):
        host[i * stride:i * stride + len(r)] = np.frombuffer(r, np.uint8)
    # records shorter than the stride: the IP total length decides, the rest is slack
    d = torch.from_numpy(host.copy()).cuda()
    batch = E.Batch.fixed(len(off), stride, stride, E.KIND_IP)
    gd, gh = _groups_dev(groups)
    eng.emit_frag(d, batch, gd)
    got = d.cpu().numpy()
    want = host.copy()
    oracle.batch_emit_frag(want, None, len(off), gh, stride=stride, length=stride, kind=1)
    assert np.array_equal(got, want)
    for i, r in enumerate(ref):
        assert got[i * stride:i * stride + len(r)].tobytes() == r
    vst = eng.verify_frag(d, batch, gd).cpu().numpy()
    assert (vst & E.ST_ACCEPT).all()
