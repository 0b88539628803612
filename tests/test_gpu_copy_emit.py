"""GPU parity of the fused payload copy + emit (smol_csum_batch_copy_emit) against the oracle's
literal restatement: memcpy of each payload, then the record emit (TcpRepr::emit
src/wire/tcp.rs:1087-1095, UdpRepr::emit src/wire/udp.rs:300-308).

Each case builds the intended packets, replaces the payload range of every record with garbage,
places the payloads at arbitrary (odd, unaligned) source offsets, and compares the device's
record bytes and status with the oracle bit for bit.  Covered: fixed-stride and packed descriptor
batches, every source/destination alignment, copy ranges that cover the checksum fields (the
emitted field must win) or that cover bytes emit never writes, zero-length copies, ranges that do
not fit (record untouched, MALFORMED), every launch shape, caps that zero the fields, records the
gates reject.
"""
import numpy as np
import pytest

import oracle
from tests import pktgen as P

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smoltcp_amd import engine as E  # noqa: E402
from tests.engines import VariantEngine  # noqa: E402

V4A, V4B = bytes([10, 1, 2, 3]), bytes([10, 4, 5, 6])
V6A = bytes(range(0x20, 0x30))
V6B = bytes(range(0x40, 0x50))


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    e = VariantEngine(0)
    yield e
    e.close()


def _packet(rng, i):
    kind = i % 6
    pay = P.rand_bytes(rng, int(rng.integers(0, 1500)))
    if kind == 0:
        return P.ipv4(V4A, V4B, 17, P.udp(1000 + i, 53, pay)), 28
    if kind == 1:
        return P.ipv4(V4A, V4B, 6, P.tcp(2000 + i, 80, pay, doff=5 + i % 3)), 20 + 20 + 4 * (i % 3)
    if kind == 2:
        return P.ipv6(V6A, V6B, 6, P.tcp(3000 + i, 443, pay)), 60
    if kind == 3:
        return P.ipv6(V6A, V6B, 17, P.udp(4000 + i, 53, pay)), 48
    if kind == 4:
        return P.ipv4(V4A, V4B, 1, P.icmp_echo(8, pay)), 28
    return P.ipv6(V6A, V6B, 58, P.icmp_echo(128, pay)), 48


def _run(eng, recs, copies_spec, caps=(0, 0, 0, 0, 0), shape=-1, fixed_stride=None, gap_seed=None, seed=0,
         fixed_len=None, variant=-1, blocks=0, base=0):
    """recs: list of full packets; copies_spec: list of (dst_offset, len) per record (payload taken
    from the packet itself).  Fixed-stride batches: record i at base + i * fixed_stride, fixed_len
    (default: the stride) bytes, random bytes in the gaps.  Returns (device statuses)."""
    rng = np.random.default_rng(seed)
    n = len(recs)
    if fixed_stride:
        L = fixed_len or fixed_stride
        buf = rng.integers(0, 256, base + n * fixed_stride + 16, dtype=np.uint8)
        offs = base + np.arange(n, dtype=np.uint64) * fixed_stride
        lens = np.full(n, L, np.uint32)
        for i, r in enumerate(recs):
            assert len(r) <= L
            buf[offs[i]:offs[i] + len(r)] = np.frombuffer(r, np.uint8)
    else:
        buf, offs, lens = P.pack(recs, gap_rng=np.random.default_rng(gap_seed) if gap_seed is not None else None)
    # source: each payload at a random (unaligned) offset, with random filler around it
    src_chunks, src_offs, pos = [], [], 0
    for i, r in enumerate(recs):
        d0, ln = copies_spec[i]
        gap = int(rng.integers(0, 37))
        src_chunks.append(P.rand_bytes(rng, gap))
        pos += gap
        src_offs.append(pos)
        full = np.frombuffer(r, np.uint8)
        body = full[d0:d0 + ln] if d0 + ln <= len(full) else np.concatenate([full[d0:], rng.integers(0, 256, d0 + ln - len(full), dtype=np.uint8)])
        src_chunks.append(bytes(body))
        pos += ln
    src_chunks.append(P.rand_bytes(rng, 16))
    src = np.frombuffer(b"".join(src_chunks), np.uint8).copy()
    # garbage where the payload will go
    for i in range(n):
        d0, ln = copies_spec[i]
        a = int(offs[i]) + d0
        end = min(a + ln, int(offs[i]) + int(lens[i]))
        if end > a:
            buf[a:end] = rng.integers(0, 256, end - a, dtype=np.uint8)
    copies = E.make_copies(src_offs, [c[0] for c in copies_spec], [c[1] for c in copies_spec])
    kinds = np.ones(n, np.uint8)
    desc = P.oracle_desc(offs, lens, kinds)

    ref = buf.copy()
    ref_st = oracle.batch_copy_emit(ref, desc, n, src, copies, caps=caps)

    eng.set_shape(shape)
    eng.set_variant(variant)
    eng.set_max_blocks(blocks)
    try:
        d = torch.from_numpy(buf.copy()).cuda()
        dsrc = torch.from_numpy(src).cuda()
        dcp = torch.from_numpy(copies.view(np.uint8).copy()).cuda()
        st = torch.zeros(n, dtype=torch.uint8, device="cuda")
        if fixed_stride:
            batch = E.Batch.fixed(n, fixed_stride, fixed_len or fixed_stride, E.KIND_IP)
            dv = d[base:]
        else:
            batch = E.Batch.from_records(offs, lens, kinds, "cuda:0")
            dv = d
        eng.copy_emit(dv, batch, dsrc, dcp, caps=caps, status=st)
        launched = eng.last_launch()
        got = d.cpu().numpy()
    finally:
        eng.set_shape(-1)
        eng.set_variant(-1)
        eng.set_max_blocks(0)
    if n:  # the forced variant ran its own kernel (default: copy_kernel variant 21)
        want = ("csum_kernel", variant) if variant in (1, 8, 11, 16) else \
            ("copy_kernel", variant if variant in (17, 22, 30, 98, 102) else 21)
        if variant in (49, 50, 55) and fixed_stride and 1024 <= (fixed_len or fixed_stride) <= 1921:
            want = ("copy_kernel", variant)  # the transposed layout (csum_xcopy.hip)
        assert (launched["kernel"], launched["variant"]) == want, (variant, launched)
    diff = np.nonzero(got != ref)[0]
    assert diff.size == 0, f"bytes differ at {diff[:8]} (got {got[diff[:8]]} want {ref[diff[:8]]})"
    assert np.array_equal(st.cpu().numpy(), ref_st)
    # the emitted records verify (where the gates reach a checksum)
    return ref_st, got, offs, lens


def test_copy_emit_fixed_stride_payloads(eng):
    rng = np.random.default_rng(1)
    recs, spec = [], []
    for i in range(3001):
        pay = P.rand_bytes(rng, 1472)
        recs.append(P.ipv4(V4A, V4B, 17, P.udp(1, 2, pay)))
        spec.append((28, 1472))
    st, got, offs, lens = _run(eng, recs, spec, fixed_stride=1500, seed=2)
    vst = oracle.batch_verify(got.copy(), None, len(recs), 1500, 1500, 1)
    assert ((vst & E.ST_ACCEPT) != 0).all()


def _fixed_case(rng, n, L):
    """Mixed packets that fit L bytes, with copy ranges of every kind (see
    test_copy_over_fields_and_edge_ranges)."""
    recs, spec = [], []
    for i in range(n):
        r, hdr = _packet(rng, i)
        r = r[:L] if len(r) > L else r
        if len(r) < hdr:
            r, hdr = P.ipv4(V4A, V4B, 17, P.udp(1, 2, P.rand_bytes(rng, L - 28))), 28
        # the IP / UDP length fields must match the cut packet: rebuild the common case
        if i % 6 == 0:
            r = P.ipv4(V4A, V4B, 17, P.udp(1000 + i, 53, P.rand_bytes(rng, min(L, 1500) - 28)))
            hdr = 28
        recs.append(r)
        m = i % 11
        if m == 0:
            spec.append((0, len(r)))
        elif m == 1:
            spec.append((hdr, 0))
        elif m == 2:
            spec.append((hdr, L - hdr + 1))      # does not fit the record: MALFORMED, untouched
        elif m == 3:
            spec.append((5, 30))
        elif m == 4:
            spec.append((1, L - 1))              # up to the record's last byte
        elif m == 5:
            spec.append((hdr, max(0, len(r) - hdr - 3)))  # ends short of the packet
        else:
            spec.append((hdr, L - hdr))          # payload to the end of the record
    return recs, spec


@pytest.mark.parametrize("stride,length", [(384, 384), (385, 385), (1500, 1500), (1514, 1514), (2048, 1500),
                                           (4001, 4001), (700, 400), (1921, 1921), (1030, 1024)])
def test_copy_emit_fixed_stride_mixed(eng, stride, length):
    """Fixed-stride batches of mixed records with every kind of copy range, at odd strides, gaps
    between records (random bytes that must survive), a batch base off the line grid, batch sizes
    around the 32-record workgroup, natural and capped grids."""
    rng = np.random.default_rng(stride + length)
    for n, base in ((1, 0), (2, 5), (33, 64), (1029, 3), (2048, 0)):
        recs, spec = _fixed_case(rng, n, length)
        # the default (17), a capped grid, the prefetch variant (1), the two-load variant (8), the
        # lane-shuffle variants (11, 16)
        for variant, blocks in ((-1, 0), (-1, 7), (1, 0), (11, 0), (11, 7), (8, 0), (8, 7), (16, 0), (16, 7), (17, 0),
                               (17, 7), (21, 0), (21, 7), (49, 0), (50, 0), (98, 0), (102, 0), (102, 7)):
            if not eng.has(variant):
                continue
            _run(eng, recs, spec, fixed_stride=stride, fixed_len=length, variant=variant, blocks=blocks,
                 base=base, seed=n + variant)


@pytest.mark.parametrize("variant", [49, 50, 55])
@pytest.mark.parametrize("stride,length", [(1500, 1500), (1505, 1500), (1024, 1024), (1921, 1921), (1337, 1337)])
def test_xcopy_fast_layout(eng, stride, length, variant):
    """Copy-emit variants 49 / 50 (the transposed layout, natural / persistent grid) where its fast layout applies: every record of a
    wavefront has its payload from inside the header window to the record's end (IPv4 / IPv6, UDP /
    TCP / ICMP, payloads at source offsets of every 4-byte phase); then the same batch with one record
    in 37 copying a shorter range, so that some wavefronts take the generic path.  Bit-exact
    against the oracle, statuses included."""
    eng.need(variant)
    rng = np.random.default_rng(stride * 7 + length)
    for n, base in ((1, 0), (9, 3), (1029, 0), (4099, 17)):
        recs, spec = [], []
        for i in range(n):
            k = i % 5
            if k == 0:
                recs.append(P.ipv4(V4A, V4B, 17, P.udp(7, 9, P.rand_bytes(rng, length - 28))))
                spec.append((28, length - 28))
            elif k == 1:
                recs.append(P.ipv4(V4A, V4B, 6, P.tcp(7, 9, P.rand_bytes(rng, length - 44), doff=6)))
                spec.append((44, length - 44))
            elif k == 2:
                recs.append(P.ipv6(V6A, V6B, 17, P.udp(7, 9, P.rand_bytes(rng, length - 48))))
                spec.append((48, length - 48))
            elif k == 3:
                recs.append(P.ipv6(V6A, V6B, 58, P.icmp_echo(128, P.rand_bytes(rng, length - 48))))
                spec.append((48, length - 48))
            else:
                recs.append(P.ipv4(V4A, V4B, 1, P.icmp_echo(8, P.rand_bytes(rng, length - 28))))
                spec.append((20, length - 20))  # the copy covers the ICMP header and its checksum field
        _run(eng, recs, spec, fixed_stride=stride, fixed_len=length, variant=variant, base=base, seed=n)
        mixed = [(c[0], c[1] - 5) if i % 37 == 5 else c for i, c in enumerate(spec)]
        _run(eng, recs, mixed, fixed_stride=stride, fixed_len=length, variant=variant, base=base, seed=n + 1)


COPY_VARIANTS = [-1, 1, 8, 11, 16, 17, 21, 22, 30]


@pytest.mark.parametrize("variant", COPY_VARIANTS)
@pytest.mark.parametrize("shape", [-1, 0, 1, 2, 3, 4, 5, 7])
def test_copy_emit_mixed_packed(eng, shape, variant):
    eng.need(variant)
    rng = np.random.default_rng(10 + shape)
    recs, spec = [], []
    for i in range(1200):
        r, hdr = _packet(rng, i)
        recs.append(r)
        spec.append((hdr, len(r) - hdr))
    st, got, offs, lens = _run(eng, recs, spec, shape=shape, gap_seed=3, seed=4, variant=variant)
    assert (st & E.ST_MALFORMED).sum() == 0


@pytest.mark.parametrize("variant", [-1, 16, 17, 21])
def test_copy_emit_packed_zero_gaps(eng, variant):
    """C3-style batch: TCP records of U[64, 9000] bytes packed back to back with no gap (odd
    offsets), so neighbouring records share cache lines.  Copy-emit rewrites every byte of a record
    (include/smolcsum.h); a neighbour's bytes must survive bit for bit."""
    eng.need(variant)
    rng = np.random.default_rng(17)
    recs, spec = [], []
    for i in range(1500):
        L = int(rng.integers(64, 9001))
        r = P.ipv4(V4A, V4B, 6, P.tcp(1000 + i % 5000, 80, P.rand_bytes(rng, L - 40)))
        recs.append(r)
        spec.append((40, L - 40) if i % 3 else (20 + int(rng.integers(0, 20)), L - 40))
    st, got, offs, lens = _run(eng, recs, spec, seed=18, variant=variant)
    assert (offs % 2 == 1).any() and not (st & E.ST_MALFORMED).any()
    vst = P.oracle_verify_records(got.copy(), offs, lens, np.ones(len(recs), np.uint8))
    assert (vst & E.ST_ACCEPT).all()


@pytest.mark.parametrize("variant", COPY_VARIANTS)
def test_copy_emit_all_alignments(eng, variant):
    """dst offsets and source offsets cover every residue mod 16."""
    eng.need(variant)
    rng = np.random.default_rng(7)
    recs, spec = [], []
    for i in range(512):
        pay = P.rand_bytes(rng, 100 + i % 200)
        r = P.ipv4(V4A, V4B, 6, P.tcp(5, 6, pay))
        recs.append(r)
        d0 = 40 - (i % 16)  # copy part of the header too: ranges start anywhere in the TCP header
        spec.append((d0, len(r) - d0 - (i % 5)))
    for shape in (-1, 0, 5):
        _run(eng, recs, spec, gap_seed=9, seed=11, variant=variant, shape=shape)


@pytest.mark.parametrize("variant", COPY_VARIANTS)
def test_copy_over_fields_and_edge_ranges(eng, variant):
    eng.need(variant)
    rng = np.random.default_rng(21)
    recs, spec = [], []
    for i in range(400):
        r, hdr = _packet(rng, i)
        recs.append(r)
        m = i % 8
        if m == 0:
            spec.append((0, len(r)))            # whole packet from the source: fields overwritten by emit
        elif m == 1:
            spec.append((hdr, 0))               # nothing to copy
        elif m == 2:
            spec.append((hdr, len(r) - hdr + 1))  # one byte too long: MALFORMED, untouched
        elif m == 3:
            spec.append((len(r), 0))            # empty range at the very end
        elif m == 4:
            spec.append((5, 30))                # IP header bytes incl. the IPv4 checksum field
        elif m == 5:
            spec.append((hdr - 3, 7))           # straddles header / payload
        elif m == 6:
            spec.append((1, len(r) - 1))
        else:
            spec.append((hdr, len(r) - hdr))
    st, got, _, _ = _run(eng, recs, spec, gap_seed=5, seed=6, variant=variant)
    assert ((st & E.ST_MALFORMED) != 0).sum() >= 50


def test_copy_emit_caps_and_rejected_records(eng):
    rng = np.random.default_rng(31)
    recs, spec = [], []
    for i in range(300):
        r, hdr = _packet(rng, i)
        if i % 10 == 0:  # an IPv4 fragment: no L4 field written, but the IP header is
            r = P.ipv4(V4A, V4B, 17, P.udp(1, 2, P.rand_bytes(rng, 40)), flags_frag=0x2000)
            hdr = 20
        if i % 10 == 1:  # an unsupported protocol: copy over where a field would be
            r = P.ipv4(V4A, V4B, 99, P.rand_bytes(rng, 64))
            hdr = 0
        recs.append(r)
        spec.append((hdr, len(r) - hdr))
    for caps in [(3, 3, 3, 3, 3), (1, 2, 1, 2, 1), (0, 0, 0, 0, 0)]:
        for variant in eng.avail((-1, 8, 11, 16, 17)):
            _run(eng, recs, spec, caps=caps, gap_seed=8, seed=12, variant=variant)


def test_copy_emit_errors(eng):
    d = torch.zeros(64, dtype=torch.uint8, device="cuda")
    cp = torch.zeros(32, dtype=torch.uint8, device="cuda")
    b = E.Batch.fixed(1, 64, 64, E.KIND_IP)
    with pytest.raises(Exception):
        eng.copy_emit(d, b, d, cp[1:17])  # copies array not 16-byte aligned
    eng.copy_emit(d, E.Batch.fixed(0, 64, 64, E.KIND_IP), d, cp)  # empty batch: no-op


@pytest.mark.parametrize("variant", COPY_VARIANTS)
def test_copy_emit_far_fields(eng, variant):
    """IPv6 records whose Hop-by-Hop header pushes the TCP / UDP checksum field past the 128-B
    header window (or across its edge): the field must still be the emitted value, whether the copy
    range covers it or not, at every record alignment."""
    eng.need(variant)
    rng = np.random.default_rng(21)
    recs, spec = [], []
    for i in range(600):
        units = int(rng.integers(6, 40))  # 56 .. 320 B of Hop-by-Hop header
        pay = P.rand_bytes(rng, int(rng.integers(0, 900)))
        if i % 2:
            l4 = P.udp(7 + i, 9, pay)
            nh, fo = 17, 6
        else:
            l4 = P.tcp(7 + i, 9, pay, doff=5 + i % 4)
            nh, fo = 6, 16
        hb = P.hbh(nh, units, rng)
        r = P.ipv6(V6A, V6B, 0, hb + l4)
        l4_off = 40 + len(hb)
        recs.append(r)
        m = i % 4
        if m == 0:
            spec.append((l4_off + (8 if nh == 17 else 4 * (5 + i % 4)), len(pay)))  # the payload
        elif m == 1:
            spec.append((l4_off + fo - 3, min(40, len(r) - (l4_off + fo - 3))))  # over the field
        elif m == 2:
            spec.append((40, len(r) - 40))  # everything after the IPv6 header
        else:
            spec.append((int(rng.integers(0, len(r))), 0))
    for shape in (-1, 1, 3):
        st, got, _, _ = _run(eng, recs, spec, gap_seed=13, seed=14 + shape, variant=variant, shape=shape)
        assert (st & E.ST_MALFORMED).sum() == 0


@pytest.mark.parametrize("variant", COPY_VARIANTS)
def test_copy_emit_tiny_records(eng, variant):
    """Records of 0 .. 47 bytes (shorter than the header window, than one 16-B chunk, or empty)
    packed at odd offsets, with copy ranges anywhere inside them (or not fitting)."""
    eng.need(variant)
    rng = np.random.default_rng(33)
    recs, spec = [], []
    for i in range(900):
        n = int(rng.integers(0, 48))
        if i % 3 == 0 and n >= 28:
            r = P.ipv4(V4A, V4B, 17, P.udp(i, 9, P.rand_bytes(rng, n - 28)))
        else:
            r = P.rand_bytes(rng, n)
        recs.append(r)
        d0 = int(rng.integers(0, n + 1))
        ln = int(rng.integers(0, n - d0 + 2))  # sometimes one byte too long: MALFORMED, untouched
        spec.append((d0, ln))
    for shape in (-1, 0, 1):
        _run(eng, recs, spec, gap_seed=17, seed=18 + shape, variant=variant, shape=shape)


@pytest.mark.parametrize("variant", [-1, 16, 17, 21])
def test_copy_emit_packed_fields_in_last_line(eng, variant):
    """Records packed back to back (no gaps) where some hold their L4 checksum field in their last
    128-B line (an IPv6 Hop-by-Hop header of 256-2000 B before a short TCP / UDP segment), between
    ordinary ones: the fields and the neighbours' bytes, which share those lines, must come out
    exactly as memcpy + emit leaves them."""
    eng.need(variant)
    rng = np.random.default_rng(41)
    recs, spec = [], []
    for i in range(1500):
        if i % 3 == 1:
            units = int(rng.integers(31, 250))
            pay = P.rand_bytes(rng, int(rng.integers(0, 120)))
            l4 = P.udp(7 + i, 9, pay) if i % 2 else P.tcp(7 + i, 9, pay)
            hb = P.hbh(17 if i % 2 else 6, units, rng)
            r = P.ipv6(V6A, V6B, 0, hb + l4)
            spec.append((40, len(r) - 40) if i % 4 else (len(r) - len(pay), len(pay)))
        else:
            r, hdr = _packet(rng, i)
            if len(r) < 256:
                r = P.ipv4(V4A, V4B, 17, P.udp(1000 + i, 53, P.rand_bytes(rng, 300 + i % 700)))
                hdr = 28
            spec.append((hdr, len(r) - hdr))
        recs.append(r)
    for shape in (-1, 2, 4, 7):
        st, got, offs, lens = _run(eng, recs, spec, seed=42 + shape, variant=variant, shape=shape)
        assert not (st & E.ST_MALFORMED).any()
        vst = P.oracle_verify_records(got.copy(), offs, lens, np.ones(len(recs), np.uint8))
        assert (vst & E.ST_ACCEPT).all()
