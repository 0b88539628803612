"""Status semantics on the GPU against the oracle (the CPU side is tests/test_status_cpu.py):

* port-zero rejects of UdpRepr::parse (src/wire/udp.rs:246-248) / TcpRepr::parse
  (src/wire/tcp.rs:910-915): verify reports SMOL_ST_MALFORMED, emit fills as usual;
* raw-socket records (SMOL_REC_IPHDR_ONLY): emit fills the IPv4 header only and leaves the user's
  L4 bytes (wrong, partial or no checksums) untouched; verify applies the IPv4 gate only
  (src/socket/raw.rs:406-423, src/iface/packet.rs:132-136, src/iface/interface/ipv4.rs:150-151);
* fragment groups outside the batch (or otherwise invalid) are neither read nor written, and a
  group with a raw record is served headers only.

Every kernel that can serve the records runs: the walk kernel's variants, the tile kernel (emit
over descriptors) and copy-emit, on descriptor batches and at a fixed stride.  Bit-exact vs the
oracle."""
import numpy as np
import pytest

import oracle
from tests import pktgen as P
from tests import test_frag_cpu as F
from tests import test_status_cpu as S

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smoltcp_amd import engine as E  # noqa: E402
from tests.engines import VariantEngine  # noqa: E402

CAPS = [(0, 0, 0, 0, 0), (3, 3, 3, 3, 3), (2, 1, 2, 1, 0), (1, 2, 1, 2, 3)]
# descriptor batches: default (tile kernel for emit, 13 for verify), walk variants 0 / 1 / 5 / 13
DESC_VARIANTS = [-1, 0, 1, 5, 13]


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    e = VariantEngine(0)
    yield e
    e.close()


def _check_desc(eng, recs, kinds, flags, seed):
    rng = np.random.default_rng(seed)
    buf, offs, lens = P.pack(recs, gap_rng=rng)
    batch = E.Batch.from_records(offs, lens, kinds, "cuda:0", flags=flags)
    desc = P.oracle_desc(offs, lens, kinds, flags)
    for variant in eng.avail(DESC_VARIANTS):
        eng.set_variant(variant)
        try:
            for caps in CAPS:
                d = torch.from_numpy(buf.copy()).cuda()
                st = torch.zeros(len(recs), dtype=torch.uint8, device="cuda:0")
                eng.emit(d, batch, caps=caps, status=st)
                got = d.cpu().numpy()
                ref = buf.copy()
                ref_st = oracle.batch_emit(ref, desc, len(desc), caps=caps)
                diff = np.nonzero(got != ref)[0]
                assert diff.size == 0, (variant, caps, diff[:8])
                assert np.array_equal(st.cpu().numpy(), ref_st), (variant, caps)
                vst = eng.verify(d, batch, caps=caps).cpu().numpy()
                assert np.array_equal(vst, oracle.batch_verify(ref, desc, len(desc), caps=caps)), (variant, caps)
        finally:
            eng.set_variant(-1)


def test_port_zero_desc(eng):
    rng = np.random.default_rng(21)
    recs = [r for r, _ in S.port_records(rng)] * 3
    kinds = np.full(len(recs), E.KIND_IP, np.uint8)
    _check_desc(eng, recs, kinds, 0, seed=1)


def test_port_zero_fixed_stride(eng):
    """C2-shaped UDP records at a fixed stride, every 7th with destination port 0."""
    n, L = 700, 1500
    buf = torch.empty(n * L, dtype=torch.uint8, device="cuda:0")
    batch = E.Batch.fixed(n, L, kind=E.KIND_IP)
    eng.synth(buf, batch, E.SYNTH_UDP4, seed=77)
    h = buf.cpu().numpy().copy()
    for i in range(0, n, 7):
        h[i * L + 22:i * L + 24] = 0  # UDP destination port
    for variant in eng.avail((-1, 0, 1, 5, 6)):
        eng.set_variant(variant)
        try:
            d = torch.from_numpy(h.copy()).cuda()
            eng.emit(d, batch)
            ref = h.copy()
            oracle.batch_emit(ref, None, n, L, L, E.KIND_IP)
            assert np.array_equal(d.cpu().numpy(), ref), variant
            vst = eng.verify(d, batch).cpu().numpy()
            rst = oracle.batch_verify(ref, None, n, L, L, E.KIND_IP)
            assert np.array_equal(vst, rst), variant
            assert (rst[::7] & E.ST_MALFORMED).all() and not (rst[::7] & E.ST_ACCEPT).any()
        finally:
            eng.set_variant(-1)


def test_raw_records_desc(eng):
    """Raw-socket frames mixed with ordinary ones in one descriptor batch."""
    rng = np.random.default_rng(22)
    raw = S.raw_records(rng)
    normal = [F.emit_whole(d, F.IGNORED) for d in F.datagrams(rng, 12, 20, 1400)]
    recs = raw + normal + raw[::-1]
    kinds = np.array([E.KIND_ETH if r[0] == 0x02 else E.KIND_IP for r in recs], np.uint8)
    flags = np.array([E.REC_IPHDR_ONLY] * len(raw) + [0] * len(normal) + [E.REC_IPHDR_ONLY] * len(raw), np.uint8)
    _check_desc(eng, recs, kinds, flags, seed=2)


def test_raw_records_fixed_stride_and_copy_emit(eng):
    """A fixed-stride batch flagged raw (smol_csum_batch_t.flags): UDP datagrams whose user
    checksums must survive emit — and copy-emit, whose payload copy still happens.  1500 B (walk
    kernel emit, transposed-walk verify) and 2500 B (transposed walk for both)."""
    for n, L in ((512, 2500), (512, 1500)):
        buf = torch.empty(n * L, dtype=torch.uint8, device="cuda:0")
        plain = E.Batch.fixed(n, L, kind=E.KIND_IP)
        eng.synth(buf, plain, E.SYNTH_UDP4, seed=78)
        h = buf.cpu().numpy().copy()
        h.reshape(n, L)[:, 26:28] = np.array([0xBE, 0xEF], np.uint8)  # the user's UDP checksum
        batch = E.Batch.fixed(n, L, kind=E.KIND_IP, flags=E.REC_IPHDR_ONLY)
        for variant in eng.avail((-1, 0, 1, 5, 44, 47)):
            eng.set_variant(variant)
            try:
                d = torch.from_numpy(h.copy()).cuda()
                st = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
                eng.emit(d, batch, status=st)
                ref = h.copy()
                rst = oracle.batch_emit(ref, None, n, L, L, oracle.kind_flags(E.KIND_IP, E.REC_IPHDR_ONLY))
                got = d.cpu().numpy()
                assert np.array_equal(got, ref), (variant, L)
                assert np.array_equal(st.cpu().numpy(), rst) and (rst == E.ST_UNSUPPORTED).all()
                assert (got.reshape(n, L)[:, 26:28] == [0xBE, 0xEF]).all()
                vst = eng.verify(d, batch).cpu().numpy()
                assert np.array_equal(vst, oracle.batch_verify(ref, None, n, L, L,
                                                               oracle.kind_flags(E.KIND_IP, E.REC_IPHDR_ONLY)))
                assert (vst & E.ST_ACCEPT).all()
            finally:
                eng.set_variant(-1)
    src = np.random.default_rng(5).integers(0, 256, n * 1472 + 16, dtype=np.uint8)
    copies = E.make_copies(np.arange(n, dtype=np.uint64) * 1472, 28, 1472)
    ref = h.copy()
    oracle.batch_copy_emit(ref, None, n, src, copies, L, L, oracle.kind_flags(E.KIND_IP, E.REC_IPHDR_ONLY))
    for variant in eng.avail((-1, 1, 17, 49, 55)):
        eng.set_variant(variant)
        try:
            d = torch.from_numpy(h.copy()).cuda()
            eng.copy_emit(d, batch, torch.from_numpy(src).cuda(), torch.from_numpy(copies.view(np.uint8).copy()).cuda())
            assert np.array_equal(d.cpu().numpy(), ref), variant
        finally:
            eng.set_variant(-1)


def test_frag_invalid_and_raw_groups(eng):
    rng = np.random.default_rng(23)
    off, _, groups = F.tx_pair(F.datagrams(rng, 6, 1500, 4000), 576, shuffle_rng=rng)
    buf, offs, lens = P.pack(off, gap_rng=rng)
    n = len(offs)
    flags = np.zeros(n, np.uint8)
    f3, c3 = groups[3]
    flags[f3] = E.REC_IPHDR_ONLY
    f0, c0 = groups[0]
    bad = [(n, 1, 0), (n - 1, 2, 0), (f0, c0, 1), (f0, 0, 0), (2**63, 3, 0), (1, 2**32 - 1, 0), (0, 300, 0)]
    gh = np.array([(f, c, 0) for f, c in groups[1:]] + bad, dtype=E.FRAG_GROUP_DTYPE)
    gd = torch.from_numpy(gh.view(np.uint8).copy()).cuda()
    batch = E.Batch.from_records(offs, lens, E.KIND_IP, "cuda:0", flags=flags)
    desc = P.oracle_desc(offs, lens, E.KIND_IP, flags)
    for caps in ((0, 0, 0, 0, 0), (3, 0, 0, 0, 0)):
        d = torch.from_numpy(buf.copy()).cuda()
        st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda:0")
        eng.emit_frag(d, batch, gd, caps=caps, status=st)
        ref = buf.copy()
        rst = np.full(n, 0xEE, np.uint8)
        o_st = oracle.batch_emit_frag(ref, desc, n, gh, caps=caps)
        covered = np.zeros(n, bool)
        for f, c in groups[1:]:
            covered[f:f + c] = True
        rst[covered] = o_st[covered]
        assert np.array_equal(d.cpu().numpy(), ref), caps
        assert np.array_equal(st.cpu().numpy(), rst), caps
        # group 0 is only named by invalid groups: untouched, no status written
        o, e = int(offs[f0]), int(offs[f0 + c0 - 1] + lens[f0 + c0 - 1])
        assert np.array_equal(d.cpu().numpy()[o:e], buf[o:e])
        assert (st.cpu().numpy()[f0:f0 + c0] == 0xEE).all()
        assert (rst[f3:f3 + c3] == E.ST_UNSUPPORTED).all()
        vs = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda:0")
        eng.verify_frag(d, batch, gd, caps=caps, status=vs)
        o_v = oracle.batch_verify_frag(ref, desc, n, gh, caps=caps)
        want = np.full(n, 0xEE, np.uint8)
        want[covered] = o_v[covered]
        assert np.array_equal(vs.cpu().numpy(), want), caps
