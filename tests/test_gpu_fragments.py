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


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    e = E.ChecksumEngine(0)
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
