"""Whole-segment emit (csum_walk.h variants 19 and 23-27) against the oracle, and its write set.

Emit fills two 2-byte fields per IPv4 record (one per IPv6 record).  The whole-segment variants
instead write the 64-byte segment holding a record's fields whole, from the group's LDS window, where
that is race-free within the call: the segment's bytes outside the record must belong to the
neighbouring records r - 1 / r + 1, contiguous in memory, with none of their fields inside it
(their groups publish extents and field ranges in LDS; variant 23 / 26 read the whole workgroup's
entries after a barrier).  The reference path is `TcpRepr::emit` -> `TcpPacket::fill_checksum`
(/root/reference/src/wire/tcp.rs:1087-1095,616-626) and `UdpRepr::emit` (udp.rs:300-308); the
result must equal the oracle's 2-byte fills byte for byte over the whole buffer.

Descriptor batches (C3-like) cover: packed records sorted and shuffled (memory neighbours that are
not index neighbours), random gaps, short records (a segment spanning three records), fields in the
records' last bytes (IPv6 Hop-by-Hop) next to records whose field segments start in the previous
record, IPv4 options, Ethernet frames, raw-socket records, every shape, natural and 1 / 3 / 5-block
grids.  The write-set test runs emit while a second stream rewrites every byte outside the
records: a kernel that wrote a byte outside its records back with a stale value would leave a
value the other stream never wrote last (a race detector, not a proof)."""
import numpy as np
import pytest

import oracle
from tests import pktgen as P

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smoltcp_amd import engine as E  # noqa: E402
from tests.dispatch_table import fixed_launch
from tests.engines import VariantEngine  # noqa: E402

SEG_VARIANTS = (23, 24, 25, 26, 27, 28)
SHAPES = [0, 1, 2, 3, 4, 5, 6, 7, 8]
V4A, V4B = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
A6, B6 = bytes(range(16)), bytes(range(16, 32))


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    e = VariantEngine(0)
    yield e
    e.close()


def _record(rng, i, lo, hi):
    """One IP packet of about U[lo, hi) bytes: IPv4 UDP / TCP (options sometimes), IPv6 UDP / TCP /
    ICMPv6, IPv6 with a Hop-by-Hop header that pushes the L4 field to the record's end."""
    k = i % 6
    n = int(rng.integers(lo, hi))
    if k == 0:
        return P.ipv4(V4A, V4B, 17, P.udp(1000 + i, 53, P.rand_bytes(rng, max(0, n - 28))))
    if k == 1:
        ihl = 5 + int(rng.integers(0, 11)) if i % 12 == 1 else 5
        return P.ipv4(V4A, V4B, 6, P.tcp(7, 8, P.rand_bytes(rng, max(0, n - 20 - 4 * ihl))), ihl=ihl)
    if k == 2:
        return P.ipv6(A6, B6, 17, P.udp(5, 6, P.rand_bytes(rng, max(0, n - 48))))
    if k == 3:
        return P.ipv6(A6, B6, 6, P.tcp(9, 10, P.rand_bytes(rng, max(0, n - 60))))
    if k == 4:
        return P.ipv6(A6, B6, 58, P.icmp6(128, max(4, n - 44), rng))
    units = max(0, (n - 40 - 8 - 10) // 8 - 1)
    return P.ipv6(A6, B6, 0, P.hbh(17, min(units, 200), rng) + P.udp(5, 6, P.rand_bytes(rng, 2)))


def _desc_case(eng, host, offs, lens, kinds, flags=0, variants=SEG_VARIANTS, blocks_list=(0, 1, 3, 5),
               shapes=(-1,)):
    """Emit a descriptor batch in each variant / shape / grid and compare the whole buffer (bytes
    outside the records included) and the status with the oracle."""
    n = len(offs)
    batch = E.Batch.from_records(offs, lens, kinds, "cuda:0", flags=flags)
    desc = P.oracle_desc(offs, lens, kinds, flags)
    ref = host.copy()
    ref_st = oracle.batch_emit(ref, desc, n)
    for variant in eng.avail(variants):
        for shape in shapes:
            for blocks in blocks_list:
                d = torch.from_numpy(host.copy()).cuda()
                st = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
                eng.set_variant(variant)
                eng.set_shape(shape)
                eng.set_max_blocks(blocks)
                try:
                    eng.emit(d, batch, status=st)
                    launched = eng.last_launch()
                    got = d.cpu().numpy()
                finally:
                    eng.set_variant(-1)
                    eng.set_shape(-1)
                    eng.set_max_blocks(0)
                if variant >= 0:
                    assert (launched["kernel"], launched["variant"]) == ("csum_kernel", variant), launched
                diff = np.nonzero(got != ref)[0]
                assert diff.size == 0, (variant, shape, blocks, diff[:8])
                assert np.array_equal(st.cpu().numpy(), ref_st), (variant, shape, blocks)


def _layout(recs, order, gaps, rng, pad=64):
    """Place records in memory in `order` (a permutation), `gaps[j]` bytes after the j-th placed one;
    descriptors stay in index order.  Returns (host buffer, offsets, lengths)."""
    lens = np.array([len(r) for r in recs], dtype=np.uint32)
    offs = np.zeros(len(recs), dtype=np.uint64)
    pos = pad
    for j, i in enumerate(order):
        offs[i] = pos
        pos += int(lens[i]) + int(gaps[j])
    host = rng.integers(0, 256, pos + pad, dtype=np.uint8)
    for i, r in enumerate(recs):
        host[int(offs[i]): int(offs[i]) + len(r)] = np.frombuffer(r, np.uint8)
    return host, offs, lens


@pytest.mark.parametrize("lo,hi", [(64, 300), (200, 1600), (28, 90)])
def test_desc_packed_sorted(eng, lo, hi):
    """Records back to back in index order (C3's layout): most field segments start in the previous
    record and go out whole; short records make a segment span three records."""
    rng = np.random.default_rng(lo * 7 + hi)
    recs = [_record(rng, i, lo, hi) for i in range(1500)]
    host, offs, lens = _layout(recs, np.arange(len(recs)), np.zeros(len(recs), int), rng, pad=37)
    _desc_case(eng, host, offs, lens, E.KIND_IP)


def test_desc_every_shape(eng):
    rng = np.random.default_rng(3)
    recs = [_record(rng, i, 64, 700) for i in range(700)]
    host, offs, lens = _layout(recs, np.arange(len(recs)), np.zeros(len(recs), int), rng, pad=5)
    _desc_case(eng, host, offs, lens, E.KIND_IP, variants=(23, 26, 28), blocks_list=(0, 3), shapes=SHAPES)


def test_desc_shuffled_and_gapped(eng):
    """Memory order differs from descriptor order (whole runs shuffled, single records swapped),
    random 0..7-byte gaps between some records: a segment may go out whole only next to the index
    neighbours that are also the memory neighbours."""
    rng = np.random.default_rng(11)
    n = 1200
    recs = [_record(rng, i, 64, 400) for i in range(n)]
    # runs of 1..40 records in index order, the runs shuffled
    cuts = np.sort(rng.choice(np.arange(1, n), 60, replace=False))
    runs = np.split(np.arange(n), cuts)
    rng.shuffle(runs)
    order = np.concatenate(runs)
    swap = rng.choice(n, 100, replace=False)
    order[swap] = order[swap[::-1]]
    gaps = np.where(rng.random(n) < 0.2, rng.integers(1, 8, n), 0)
    host, offs, lens = _layout(recs, order, gaps, rng)
    _desc_case(eng, host, offs, lens, E.KIND_IP)
    # fully random order
    order = rng.permutation(n)
    host, offs, lens = _layout(recs, order, np.zeros(n, int), rng)
    _desc_case(eng, host, offs, lens, E.KIND_IP, blocks_list=(0, 3))


def test_desc_fields_at_record_ends(eng):
    """IPv6 records whose UDP field sits in their last 64 bytes (Hop-by-Hop) alternate with IPv4 /
    IPv6 records whose field segments start in the previous record's last bytes."""
    rng = np.random.default_rng(77)
    recs = []
    for i in range(900):
        L = int(rng.integers(120, 330))
        if i % 3 == 0:
            units = (L - 40 - 8 - 10) // 8 - 1
            h = P.hbh(17, units, rng)
            room = max(0, L - 40 - len(h) - 8)
            body = P.ipv6(A6, B6, 0, h + P.udp(5, 6, P.rand_bytes(rng, int(rng.integers(0, room + 1)))))
        elif i % 3 == 1:
            body = P.ipv4(V4A, V4B, 17, P.udp(1, 2, P.rand_bytes(rng, int(rng.integers(0, L - 28)))))
        else:
            body = P.ipv6(A6, B6, 6, P.tcp(7, 8, P.rand_bytes(rng, int(rng.integers(0, L - 60)))))
        recs.append(body)
    host, offs, lens = _layout(recs, np.arange(len(recs)), np.zeros(len(recs), int), rng, pad=63)
    _desc_case(eng, host, offs, lens, E.KIND_IP)


def test_desc_ethernet_raw_and_malformed(eng):
    """Ethernet frames, raw-socket records (IPv4 header only: their L4 bytes must stay as written)
    and malformed / unsupported records packed between ordinary ones."""
    rng = np.random.default_rng(21)
    recs, kinds, flags = [], [], []
    for i in range(800):
        r = _record(rng, i, 64, 500)
        if i % 4 == 0:
            r = P.eth(r, 0x0800 if r[0] >> 4 == 4 else 0x86DD)
            kinds.append(E.KIND_ETH)
        else:
            kinds.append(E.KIND_IP)
        if i % 9 == 0:
            r = r[: int(rng.integers(1, 30))]  # cut inside the headers
        if i % 7 == 3 and r[0] >> 4 == 4 and kinds[-1] == E.KIND_IP:
            flags.append(E.REC_IPHDR_ONLY)
        else:
            flags.append(0)
        recs.append(r)
    host, offs, lens = _layout(recs, np.arange(len(recs)), np.zeros(len(recs), int), rng)
    _desc_case(eng, host, offs, lens, np.array(kinds, np.uint8), flags=np.array(flags, np.uint8))


def test_c3_seed_segments(eng):
    """The C3 seed layout (TCP U[64, 9000], packed, odd offsets) synthesized on the device, 4000
    records, every whole-segment variant against the oracle."""
    rng = np.random.default_rng(0x5EED0002)
    n = 4000
    lens = rng.integers(64, 9001, n).astype(np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    buf = torch.zeros(int(offs[-1] + lens[-1]) + 16, dtype=torch.uint8, device="cuda:0")
    eng.synth(buf, E.Batch.from_records(offs, lens, E.KIND_IP, "cuda:0"), E.SYNTH_TCP4, seed=0x5EED0002)
    _desc_case(eng, buf.cpu().numpy().copy(), offs, lens, E.KIND_IP, blocks_list=(0, 5))


@pytest.mark.parametrize("gap,L", [(0, 1500), (24, 1500), (0, 2500), (24, 2500), (40, 9000)])
def test_emit_write_set_concurrent(eng, gap, L):
    """Emit never writes a byte outside its records: while emit runs on one stream, another stream
    rewrites every byte outside the records (before the batch, the gaps between records, after the
    batch) with 1, 2, ..., K.  Afterwards those bytes must all hold K and the records must equal the
    oracle's emit.  Fixed-stride (variant 19, the transposed walk 44 / 47 and the defaults: 2500 B
    and 9000 B run the transposed walk) and descriptor batches."""
    n = (1 << 15) if L < 5000 else (1 << 12)
    stride = L + gap
    pre, post = 4096, 4096
    total = pre + n * stride + post
    buf = torch.zeros(total, dtype=torch.uint8, device="cuda:0")
    fixed = E.Batch.fixed(n, stride, L, E.KIND_IP)
    eng.synth(buf[pre:], fixed, E.SYNTH_UDP4, seed=99 + gap)
    offs = np.arange(n, dtype=np.uint64) * stride
    desc_batch = E.Batch.from_records(offs, np.full(n, L, np.uint32), E.KIND_IP, "cuda:0")
    inside = torch.zeros(total, dtype=torch.bool, device="cuda:0")
    inside[pre: pre + n * stride].view(n, stride)[:, :L] = True
    outside_idx = torch.nonzero(~inside).flatten()
    host0 = buf.cpu().numpy().copy()
    rec0 = host0[pre: pre + n * stride].copy()
    ref = rec0.copy()
    oracle.batch_emit(ref, None, n, stride, L, E.KIND_IP)
    s_emit, s_write = torch.cuda.Stream(), torch.cuda.Stream()
    K = 120
    for variant, batch in ((19, fixed), (29, fixed), (-1, fixed), (23, fixed), (26, desc_batch), (28, desc_batch),
                           (-1, desc_batch), (37, fixed), (39, fixed), (44, fixed), (47, fixed), (12, fixed),
                           (61, desc_batch), (62, desc_batch), (97, desc_batch), (103, desc_batch), (104, desc_batch), (101, fixed)):
        if not eng.has(variant):
            continue
        d = torch.from_numpy(host0.copy()).cuda()
        torch.cuda.synchronize()
        eng.set_variant(variant)
        try:
            for k in range(1, K + 1):
                with torch.cuda.stream(s_write):
                    d.index_fill_(0, outside_idx, k)
                if k % 12 == 1:
                    eng.emit(d[pre:], batch, stream=s_emit)
            torch.cuda.synchronize()
        finally:
            eng.set_variant(-1)
        got = d.cpu().numpy()
        out = got[(~inside).cpu().numpy()]
        assert (out == K).all(), (variant, gap, np.nonzero(out != K)[0][:8])
        assert np.array_equal(got[pre: pre + n * stride].reshape(n, stride)[:, :L],
                              ref.reshape(n, stride)[:, :L]), (variant, gap)


def test_field_stores_flag(eng):
    """SMOL_BATCH_FIELD_STORES: emit stores the checksum fields only.  The output equals the
    oracle's (fixed-stride and descriptor batches, every whole-segment variant forced), and bytes
    of the records next to the fields that another stream rewrites while emit runs keep that
    stream's last value."""
    rng = np.random.default_rng(8)
    recs = [_record(rng, i, 64, 600) for i in range(900)]
    host, offs, lens = _layout(recs, np.arange(len(recs)), np.zeros(len(recs), int), rng, pad=21)
    n = len(recs)
    desc = P.oracle_desc(offs, lens, E.KIND_IP)
    ref = host.copy()
    oracle.batch_emit(ref, desc, n)
    batch = E.Batch.from_records(offs, lens, E.KIND_IP, "cuda:0", batch_flags=E.BATCH_FIELD_STORES)
    for variant in eng.avail((-1, 19, 23, 26, 27, 28, 29, 39, 7, 61, 62)):
        d = torch.from_numpy(host.copy()).cuda()
        eng.set_variant(variant)
        try:
            eng.emit(d, batch)
            got = d.cpu().numpy()
        finally:
            eng.set_variant(-1)
        assert np.array_equal(got, ref), (variant, np.nonzero(got != ref)[0][:8])
    # fixed-stride C2-like batches (1500 B, 2500 B: the transposed walk; 1600 B: the walk kernel): UDP
    # payload bytes 30..63 of every record (in the segment that holds the IPv4 header and UDP
    # checksums) rewritten from another stream while emit runs
    for n, L in ((1 << 15, 1500), (1 << 14, 2500), (1 << 15, 1600)):
        buf = torch.zeros(n * L + 64, dtype=torch.uint8, device="cuda:0")
        fixed = E.Batch.fixed(n, L, L, E.KIND_IP, flags=E.BATCH_FIELD_STORES)
        eng.synth(buf, fixed, E.SYNTH_UDP4, seed=5)
        payload = buf[: n * L].view(n, L)[:, 30:64]
        s_emit, s_write = torch.cuda.Stream(), torch.cuda.Stream()
        torch.cuda.synchronize()
        K = 120
        for k in range(1, K + 1):
            with torch.cuda.stream(s_write):
                payload.fill_(k)
            if k % 12 == 1:
                eng.emit(buf, fixed, stream=s_emit)
        torch.cuda.synchronize()
        assert bool((payload == K).all()), L
        ll = eng.last_launch()
        # SMOL_BATCH_FIELD_STORES: the table's kernel with 2-B field stores (the walk kernel's 5, the
        # transposed walk's 44)
        kern, _ = fixed_launch("emit", L, L)
        assert (ll["kernel"], ll["variant"]) == ((kern, 44) if kern == "xwalk_kernel" else (kern, 5)), (L, ll)


def test_staged_emit_tiny_neighbours_concurrent(eng):
    """The staged descriptor emit (97, and 103 / 94 from the experiments build) next to records that
    give its shared-segment rule trouble: long IPv4/TCP records back to back with tiny raw records
    (12-60 B, no fields) before them, and small gaps before some wavefronts' first records.  While
    emit runs, another stream rewrites every byte outside the records; those bytes must end with that
    stream's last value and the records must equal the oracle's emit (a segment may start in the
    record before only when that record is at least 64 B long and ends where this one begins)."""
    rng = np.random.default_rng(0x71)
    n = 8192
    lens = rng.integers(1100, 2400, n).astype(np.uint32)
    tiny = rng.random(n) < 0.2
    lens[tiny] = rng.integers(12, 61, int(tiny.sum()))
    gaps = np.where(rng.random(n) < 0.1, rng.integers(1, 40, n), 0).astype(np.uint64)
    pre, post = 4096, 4096
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[1:])
    total = pre + int(offs[-1] + lens[-1]) + post
    buf = torch.zeros(total, dtype=torch.uint8, device="cuda:0")
    batch = E.Batch.from_records(offs, lens, E.KIND_IP, "cuda:0")
    eng.synth(buf[pre:], batch, E.SYNTH_TCP4, seed=0x71)
    host0 = buf.cpu().numpy().copy()
    for j in np.nonzero(tiny)[0]:  # raw junk: no IP header the parse accepts
        a = pre + int(offs[j])
        host0[a: a + int(lens[j])] = 0
    inside = np.zeros(total, dtype=bool)
    for o, l in zip(offs, lens):
        inside[pre + int(o): pre + int(o) + int(l)] = True
    outside_idx = torch.from_numpy(np.nonzero(~inside)[0]).cuda()
    ref = host0[pre:].copy()
    oracle.batch_emit(ref, P.oracle_desc(offs, lens, E.KIND_IP), n, 0, 0, E.KIND_IP)
    s_emit, s_write = torch.cuda.Stream(), torch.cuda.Stream()
    K = 60
    ran = 0
    for variant in (-1, 97, 103, 104, 105, 94):
        if not eng.has(variant):
            continue
        ran += 1
        d = torch.from_numpy(host0.copy()).cuda()
        torch.cuda.synchronize()
        eng.set_variant(variant)
        try:
            for k in range(1, K + 1):
                with torch.cuda.stream(s_write):
                    d.index_fill_(0, outside_idx, k)
                if k % 6 == 1:
                    eng.emit(d[pre:], batch, stream=s_emit)
            torch.cuda.synchronize()
        finally:
            eng.set_variant(-1)
        got = d.cpu().numpy()
        assert (got[~inside] == K).all(), (variant, np.nonzero(got[~inside] != K)[0][:8])
        assert np.array_equal(got[pre:][inside[pre:]], ref[inside[pre:]]), variant
    assert ran >= 2
