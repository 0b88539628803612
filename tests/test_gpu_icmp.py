"""GPU parity for the ICMP rules added in round 2, against the CPU oracle.

* ICMPv4 DstUnreachable / TimeExceeded: Icmpv4Repr::emit writes the embedded IPv4 header with
  Ipv4Repr::emit under the same caps before the ICMP checksum covers it
  (src/wire/icmpv4.rs:520-543, src/wire/ipv4.rs:605-611).  Pinned by the fuzz-corpus frame
  icmpv4_unreachable.bin (all three checksums written by a real sender: zeroed, the emit must give
  the frame back), then random messages against the oracle, through every emit path: the walk
  kernel (fixed stride and descriptors, every load variant), the tile kernel and the fused
  copy + emit.
* ICMPv6 Icmpv6Packet::check_len (src/wire/icmpv6.rs:274-338): a typed message shorter than its
  header is MALFORMED on verify; every type value x lengths around its minimum, walk and tile
  kernels.
"""
import numpy as np
import pytest

import oracle
from tests import pktgen as P

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smoltcp_amd import engine as E  # noqa: E402
from tests.engines import VariantEngine  # noqa: E402

V4A, V4B = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
A6, B6 = bytes(range(16)), bytes(range(16, 32))
CAPS = [(0, 0, 0, 0, 0), (3, 0, 0, 0, 0), (2, 0, 0, 3, 0), (0, 0, 0, 1, 0), (1, 3, 3, 2, 3)]


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    e = VariantEngine(0)
    yield e
    e.close()


def _with(eng, variant=-1, shape=-1):
    eng.set_variant(variant)
    eng.set_shape(shape)


def _reset(eng):
    eng.set_variant(-1)
    eng.set_shape(-1)


def _emit_desc(eng, records, kind, caps, variant):
    buf, offs, lens = P.pack(records, gap_rng=np.random.default_rng(len(records)))
    batch = E.Batch.from_records(offs, lens, kind, "cuda:0")
    d = torch.from_numpy(buf.copy()).cuda()
    st = torch.zeros(len(records), dtype=torch.uint8, device="cuda:0")
    _with(eng, variant)
    try:
        eng.emit(d, batch, caps=caps, status=st)
        vst = eng.verify(d, batch, caps=caps).cpu().numpy()
    finally:
        _reset(eng)
    ref = buf.copy()
    ref_st = P.oracle_emit_records(ref, offs, lens, kind, caps)
    got = d.cpu().numpy()
    diff = np.nonzero(got != ref)[0]
    assert diff.size == 0, (variant, caps, diff[:8])
    assert np.array_equal(st.cpu().numpy(), ref_st), (variant, caps)
    assert np.array_equal(vst, P.oracle_verify_records(ref, offs, lens, kind, caps)), (variant, caps)
    return got, offs, lens


def _emit_fixed(eng, rec, n, stride, kind, caps, variant, off=0):
    host = np.zeros(off + n * stride + 64, np.uint8)
    for i in range(n):
        host[off + i * stride: off + i * stride + len(rec)] = np.frombuffer(rec, np.uint8)
    d = torch.from_numpy(host.copy()).cuda()
    _with(eng, variant)
    try:
        eng.emit(d[off:], E.Batch.fixed(n, stride, len(rec), kind), caps=caps)
    finally:
        _reset(eng)
    ref = host.copy()
    sub = ref[off:].copy()
    oracle.batch_emit(sub, None, n, stride, len(rec), kind, caps)
    ref[off:] = sub
    got = d.cpu().numpy()
    assert np.array_equal(got, ref), (variant, stride, off, np.nonzero(got != ref)[0][:8])
    return got


def _corpus_frame(golden):
    fr = [f for f in golden["fuzz_corpus_frames"] if f["name"] == "icmpv4_unreachable.bin"][0]
    orig = bytes.fromhex(fr["bytes"])
    icmp = 14 + (orig[14] & 15) * 4
    z = bytearray(orig)
    for o in (14 + 10, icmp + 2, icmp + 8 + 10):  # outer header, ICMP, embedded header checksums
        z[o:o + 2] = b"\0\0"
    return orig, bytes(z), icmp


def test_icmpv4_unreachable_corpus_frame_every_path(eng, golden):
    """The zeroed corpus frame comes back byte for byte from every emit path."""
    orig, z, _ = _corpus_frame(golden)
    for variant in eng.avail((-1, 7, 3, 4, 1, 5, 0, 6)):  # tile (default for descriptors) and walk
        got, offs, lens = _emit_desc(eng, [z] * 5, E.KIND_ETH, (0, 0, 0, 0, 0), variant)
        for o, ln in zip(offs, lens):
            assert got[int(o):int(o) + int(ln)].tobytes() == orig, variant
    for variant in eng.avail((-1, 9, 10, 6, 1, 0)):  # fixed stride: walk kernel (line grid default)
        for stride, off in ((len(z), 0), (601, 3), (640, 0)):
            got = _emit_fixed(eng, z, 37, stride, E.KIND_ETH, (0, 0, 0, 0, 0), variant, off)
            for i in range(37):
                assert got[off + i * stride: off + i * stride + len(z)].tobytes() == orig


def test_icmpv4_unreachable_corpus_frame_copy_emit(eng, golden):
    """Fused copy + emit with the ICMP message (embedded header included) copied from a source
    buffer that still holds the sender's checksums: the emitted fields win, as after memcpy +
    emit, and the frame comes back whole."""
    orig, z, icmp = _corpus_frame(golden)
    n = 9
    for start in (icmp, icmp + 8, icmp + 4):
        pay = orig[start:]  # the source keeps the real (non-zero) inner checksum
        recs = [z[:start] + bytes(len(pay)) for _ in range(n)]
        buf, offs, lens = P.pack(recs, gap_rng=np.random.default_rng(start))
        src = np.frombuffer(b"".join(bytes(5) + pay for _ in range(n)) + bytes(16), np.uint8).copy()
        src_off = np.array([i * (5 + len(pay)) + 5 for i in range(n)], np.uint64)
        cp = E.make_copies(src_off, start, len(pay))
        batch = E.Batch.from_records(offs, lens, E.KIND_ETH, "cuda:0")
        d = torch.from_numpy(buf.copy()).cuda()
        eng.copy_emit(d, batch, torch.from_numpy(src).cuda(), torch.from_numpy(cp.view(np.uint8).copy()).cuda())
        got = d.cpu().numpy()
        for o, ln in zip(offs, lens):
            assert got[int(o):int(o) + int(ln)].tobytes() == orig, start
        ref = buf.copy()
        oracle.batch_copy_emit(ref, P.oracle_desc(offs, lens, E.KIND_ETH), n, src, cp)
        assert np.array_equal(got, ref)


def _icmp4_errors(rng, n):
    """Random IPv4 packets carrying ICMPv4 messages around the rule's edges: error and non-error
    types, inner version 4 / 6 / garbage, IHL 0..15 with options, messages cut before, at and
    after the inner header."""
    recs = []
    for _ in range(n):
        t = int(rng.choice([3, 11, 3, 11, 0, 8, 12, 5]))
        ihl = int(rng.choice([5, 5, 5, 6, 15, 4, 0]))
        ver = int(rng.choice([4, 4, 4, 6, 0]))
        inner_hdr = bytearray(rng.integers(0, 256, max(ihl * 4, 20), dtype=np.uint8).tobytes())
        inner_hdr[0] = (ver << 4) | ihl
        inner = bytes(inner_hdr) + P.rand_bytes(rng, int(rng.integers(0, 40)))
        cut = int(rng.integers(0, len(inner) + 1)) if rng.random() < 0.3 else len(inner)
        recs.append(P.ipv4(V4A, V4B, 1, P.icmp4_error(t, int(rng.integers(0, 16)), inner[:cut])))
    return recs


def test_icmpv4_errors_random_vs_oracle(eng):
    rng = np.random.default_rng(2024)
    ip = _icmp4_errors(rng, 500)
    eth = [P.eth(r) for r in _icmp4_errors(rng, 200)]
    for caps in CAPS:
        for variant in eng.avail((-1, 3, 1, 5)):
            _emit_desc(eng, ip, E.KIND_IP, caps, variant)
            _emit_desc(eng, eth, E.KIND_ETH, caps, variant)


def test_icmpv4_error_fixed_stride_vs_oracle(eng):
    """The iface test's port-unreachable shape (src/iface/interface/tests/ipv4.rs:280-385: an
    IPv4/ICMPv4 DstUnreachable carrying the 20-byte header of the offending UDP datagram and its
    20 UDP bytes), emitted at fixed strides with every caps row."""
    udp = P.udp(67, 68, b"Hello, Wold!")
    inner = P.ipv4(bytes([127, 0, 0, 2]), bytes([127, 0, 0, 1]), 17, udp)
    pkt = P.ipv4(bytes([127, 0, 0, 1]), bytes([127, 0, 0, 2]), 1, P.icmp4_error(3, 3, inner))
    for caps in CAPS:
        for variant in eng.avail((-1, 9, 1)):
            for stride, off in ((len(pkt), 0), (len(pkt) + 1, 1), (256, 7)):
                _emit_fixed(eng, pkt, 301, stride, E.KIND_IP, caps, variant, off)


def test_icmpv6_check_len_every_type(eng, golden):
    """Every type value x lengths around its check_len minimum, IPv6 and Ethernet: verify status
    (MALFORMED / ACCEPT) and emit bytes equal the oracle's, walk and tile kernels."""
    rng = np.random.default_rng(58)
    tab = {int(k): v for k, v in golden["icmpv6_check_len"]["min_len"].items()}
    recs = []
    for t in range(256):
        need = tab.get(t, 0)
        for body in sorted({0, 3, 4, max(need - 5, 0), max(need - 4, 0), need, need + 9}):
            msg = bytearray(P.icmp6(t, body, rng))
            pkt = P.ipv6(A6, B6, 58, bytes(msg))
            recs.append(pkt)
    host = np.concatenate([np.frombuffer(r, np.uint8) for r in recs])
    # valid checksums first (oracle fill), so ACCEPT depends on check_len only
    buf, offs, lens = P.pack(recs)
    P.oracle_emit_records(buf, offs, lens, E.KIND_IP)
    filled = [buf[int(o):int(o) + int(ln)].tobytes() for o, ln in zip(offs, lens)]
    assert host.size == sum(len(r) for r in recs)
    for variant in eng.avail((-1, 3, 4, 7, 1, 0)):
        for rs, kind in ((filled, E.KIND_IP), ([P.eth(r, 0x86DD) for r in filled], E.KIND_ETH)):
            b2, o2, l2 = P.pack(rs, gap_rng=np.random.default_rng(variant + 5))
            batch = E.Batch.from_records(o2, l2, kind, "cuda:0")
            d = torch.from_numpy(b2.copy()).cuda()
            _with(eng, variant)
            try:
                st = eng.verify(d, batch).cpu().numpy()
            finally:
                _reset(eng)
            ref = P.oracle_verify_records(b2, o2, l2, kind)
            assert np.array_equal(st, ref), (variant, np.nonzero(st != ref)[0][:8])
            mal = (ref & E.ST_MALFORMED) != 0
            assert mal.any() and (~mal).any()
    _emit_desc(eng, recs, E.KIND_IP, (0, 0, 0, 0, 0), -1)
    _emit_desc(eng, recs, E.KIND_IP, (0, 0, 0, 0, 0), 1)
