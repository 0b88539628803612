"""The measurement tools of include/smolcsum_tools.h that experiments rely on: the field-scatter pass
(tools/exp_scatter.py) and the launched-kernel record (smol_csum_tool_last_launch) over every
kernel family."""
import numpy as np
import pytest
import torch

from smoltcp_amd import engine as E
from tests import pktgen as P
from tests.dispatch_table import fixed_launch
from tests.engines import VariantEngine

pytestmark = pytest.mark.gpu
CAPS = (0, 0, 0, 0, 0)


@pytest.fixture(scope="module")
def eng():
    e = VariantEngine(0)
    yield e
    e.close()


@pytest.mark.parametrize("nt", [False, True])
def test_field_scatter(eng, nt):
    """Every listed 2-B big-endian value lands at its offset (odd and even offsets, the buffer's
    last two bytes); every other byte is untouched; offsets past the buffer are skipped."""
    rng = np.random.default_rng(3 + nt)
    size = 1 << 16
    host = rng.integers(0, 256, size, dtype=np.uint8)
    offs = np.unique(rng.integers(0, size - 1, 3000)).astype(np.int64)
    offs = offs[np.concatenate([[True], np.diff(offs) >= 2])]  # no two stores overlap
    offs = np.concatenate([offs[offs < size - 3], [size - 2]])
    vals = rng.integers(0, 1 << 16, offs.size).astype(np.uint16)
    ref = host.copy()
    ref[offs] = (vals >> 8).astype(np.uint8)
    ref[offs + 1] = (vals & 0xFF).astype(np.uint8)
    d = torch.from_numpy(host.copy()).cuda()
    a = torch.from_numpy(np.concatenate([offs, [size - 1, size + 100]])).cuda()  # two past the end
    v = torch.from_numpy(np.concatenate([vals, [1, 2]]).astype(np.uint16).view(np.int16)).cuda()
    eng.field_scatter(d, a, v, nt=nt)
    got = d.cpu().numpy()
    assert np.array_equal(got, ref), np.nonzero(got != ref)[0][:8]


@pytest.mark.parametrize("flags,size", [(2, 64), (4, 32), (8, 128)])
def test_field_scatter_whole_shapes(eng, flags, size):
    """The timing shapes of the scatter probe: the aligned 64-B segment / 32-B sector / 128-B line
    holding each listed offset is overwritten whole with the value repeated; nothing else changes;
    a shape that would run past the buffer is skipped."""
    rng = np.random.default_rng(flags)
    nbytes = 1 << 14
    host = rng.integers(0, 256, nbytes, dtype=np.uint8)
    offs = np.array([0, 77, 1000, 4097, nbytes - 2], dtype=np.int64)
    vals = np.array([0x1234, 0xABCD, 0x0F0F, 0x5A5A, 0x7777], dtype=np.uint16)
    ref = host.copy()
    for o, v in zip(offs, vals):
        s0 = int(o) // size * size
        if s0 + size <= nbytes:
            ref[s0:s0 + size] = np.tile(np.array([v & 0xFF, v >> 8], np.uint8), size // 2)
    d = torch.from_numpy(host.copy()).cuda()
    eng.field_scatter(d, torch.from_numpy(offs).cuda(), torch.from_numpy(vals.view(np.int16)).cuda(), nt=flags)
    got = d.cpu().numpy()
    assert np.array_equal(got, ref), np.nonzero(got != ref)[0][:8]


def test_last_launch_families(eng):
    """The launched-kernel record names the kernel family and the variant each entry point ran."""
    n, L = 257, 1500
    buf = torch.zeros(n * L, dtype=torch.uint8, device="cuda:0")
    b = E.Batch.fixed(n, L, L, E.KIND_IP)
    eng.synth(buf, b, E.SYNTH_UDP4, seed=1)
    eng.emit(buf, b)
    ll = eng.last_launch()
    # packed fixed-stride emit of 1400-1580-B records (not multiples of 64 B): the transposed walk
    # with its field segments stored non-temporal
    assert (ll["kernel"], ll["variant"]) == fixed_launch("emit", L, L), ll
    eng.verify(buf, b)
    ll = eng.last_launch()
    # the dispatch table's choices (tests/dispatch_table.py reads smoltcp_amd/csrc/dispatch_table.inc)
    assert (ll["kernel"], ll["variant"]) == fixed_launch("verify", L, L), ll
    for LL, stride in ((1320, 1320), (1500, 1501), (2500, 2500), (1600, 1600), (1500, 1564), (9000, 9000),
                       (8000, 8000), (1536, 1536), (12000, 12000), (2500, 2564), (1700, 1764), (1024, 1024)):
        for op in ("emit", "verify"):
            bb = E.Batch.fixed(8, stride, LL, E.KIND_IP)
            t = torch.zeros(8 * stride + 64, dtype=torch.uint8, device="cuda:0")
            getattr(eng, op)(t, bb)
            ll = eng.last_launch()
            assert (ll["kernel"], ll["variant"]) == fixed_launch(op, LL, stride), (LL, stride, op, ll)
            if ll["kernel"] == "xwalk_kernel":  # 8 / 4 / 2 / 1 records per wavefront by length
                assert ll["G"] == 64 // (8 if LL <= 1921 else 4 if LL <= 3969 else 2 if LL <= 8065 else 1), (LL, ll)
    offs = np.arange(n, dtype=np.uint64) * L
    bd = E.Batch.from_records(offs, np.full(n, L, np.uint32), E.KIND_IP, "cuda:0")
    # descriptor batches: the per-group descriptor walk (csum_dwalk.hip, cached header windows),
    # 8 lanes x 4 chunks, both operations (emit staged on a fresh context: 97); the tile kernel when
    # forced (variant 7)
    e2 = VariantEngine(0)
    try:
        e2.emit(buf, bd)
        ll = e2.last_launch()
    finally:
        e2.close()
    assert (ll["kernel"], ll["variant"], ll["G"], ll["U"]) == ("dwalk_kernel", 97, 8, 4), ll
    eng.verify(buf, bd)
    ll = eng.last_launch()
    assert (ll["kernel"], ll["variant"], ll["G"], ll["U"]) == ("dwalk_kernel", 63, 8, 4), ll
    eng.set_variant(7)
    try:
        eng.emit(buf, bd)
        ll = eng.last_launch()
    finally:
        eng.set_variant(-1)
    assert (ll["kernel"], ll["variant"]) == ("csum_tile_kernel", 2), ll
    src = torch.zeros(n * 1472 + 16, dtype=torch.uint8, device="cuda:0")
    cp = torch.from_numpy(E.make_copies(np.arange(n, dtype=np.uint64) * 1472, 28, 1472).view(np.uint8).copy()).cuda()
    eng.copy_emit(buf, b, src, cp)
    ll = eng.last_launch()
    assert (ll["kernel"], ll["variant"], ll["G"], ll["U"]) == ("copy_kernel", 21, 16, 4), ll


def test_kernel_for_names_the_launch(eng):
    """smol_csum_tool_kernel_for (csum_api.cpp pick_kernel, the decision run() launches) names the kernel
    every fixed-stride length, descriptor batch and forced variant actually ran (last_launch)."""
    cases = [(LL, stride, op) for LL, stride in ((1320, 1320), (1500, 1500), (1500, 1564), (1600, 1600), (2500, 2500),
                                                 (9000, 9000), (12000, 12000), (1024, 1024), (1700, 1764))
             for op in ("emit", "verify", "data")]
    for LL, stride, op in cases:
        bb = E.Batch.fixed(8, stride, LL, E.KIND_IP)
        t = torch.zeros(8 * stride + 64, dtype=torch.uint8, device="cuda:0")
        want = eng.kernel_for(op, bb)
        getattr(eng, op)(t, bb)
        assert eng.last_launch()["kernel"] == want, (LL, stride, op, want, eng.last_launch())
    n, L = 64, 1500
    buf = torch.zeros(n * L, dtype=torch.uint8, device="cuda:0")
    bd = E.Batch.from_records(np.arange(n, dtype=np.uint64) * L, np.full(n, L, np.uint32), E.KIND_IP, "cuda:0")
    for v in (-1, 7, 13, 60, 63, 41):
        eng.set_variant(v)
        try:
            for op in ("emit", "verify"):
                want = eng.kernel_for(op, bd)
                getattr(eng, op)(buf, bd)
                assert eng.last_launch()["kernel"] == want, (v, op, want, eng.last_launch())
        finally:
            eng.set_variant(-1)


@pytest.mark.parametrize("v", [17, 21])
def test_forced_copy_variant_serves_other_ops(eng, v):
    """A copy-emit-only variant forced on the context (it used to fail emit / verify with
    SMOL_EHIP) runs copy-emit itself and leaves emit / verify on their default kernels, bit-exact."""
    import oracle

    n, L = 96, 1500
    b = E.Batch.fixed(n, L, L, E.KIND_IP)
    buf = torch.zeros(n * L, dtype=torch.uint8, device="cuda:0")
    eng.synth(buf, b, E.SYNTH_UDP4, seed=11)
    host = buf.cpu().numpy().copy()
    want_emit, want_verify = eng.kernel_for("emit", b), eng.kernel_for("verify", b)
    eng.set_variant(v)
    try:
        assert eng.kernel_for("emit", b) == want_emit and eng.kernel_for("verify", b) == want_verify
        eng.emit(buf, b)
        assert eng.last_launch()["kernel"] == want_emit
        st = eng.verify(buf, b)
        assert eng.last_launch()["kernel"] == want_verify
        src = torch.randint(0, 256, (n * 1472 + 16,), dtype=torch.uint8, device="cuda:0")
        cp = torch.from_numpy(E.make_copies(np.arange(n, dtype=np.uint64) * 1472, 28, 1472).view(np.uint8).copy()).cuda()
        eng.copy_emit(torch.zeros_like(buf), b, src, cp)
        ll = eng.last_launch()
        assert (ll["kernel"], ll["variant"]) == ("copy_kernel", v), ll
    finally:
        eng.set_variant(-1)
    ref = host.copy()
    oracle.batch_emit(ref, None, n, L, L, E.KIND_IP, (0, 0, 0, 0, 0))
    assert np.array_equal(buf.cpu().numpy(), ref)
    assert np.array_equal(st.cpu().numpy(), oracle.batch_verify(ref, None, n, L, L, E.KIND_IP, (0, 0, 0, 0, 0)))


@pytest.mark.parametrize("nt", [False, True])
def test_segment_probe_changes_nothing(eng, nt):
    """The segment-shape floor probe (bench.py roofline.floor) rewrites the field segments with their own
    bytes: the buffer is bit-identical afterwards, for C2-like field offsets and a partial last piece."""
    n, L = 3000, 1500
    nbytes = n * L + 5000  # a tail past the last whole 8-KiB piece
    host = np.random.default_rng(8).integers(0, 256, nbytes, dtype=np.uint8)
    d = torch.from_numpy(host.copy()).cuda()
    addrs = torch.from_numpy(np.sort(np.concatenate([np.arange(n) * L + 10, np.arange(n) * L + 26])).astype(np.int64)).cuda()
    bitmap, nseg = E.segment_bitmap(addrs, nbytes // 16 * 16)
    assert nseg == len({a >> 6 for a in addrs.cpu().tolist()} | {(a + 1) >> 6 for a in addrs.cpu().tolist()})
    eng.segment_probe(d, bitmap, nt=nt)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), host)


def test_descriptor_emit_choice_follows_the_records(eng):
    """Descriptor-batch emit picks the staged form (97) or the in-place one (41) from the previous staged
    call's sample of wavefront flags (csum_api.cpp update_desc_choice): short records (no wavefront
    stages) switch a fresh context to 41 after one call, long back-to-back records keep 97; both
    forms write the oracle's bytes."""
    import oracle

    rng = np.random.default_rng(97)
    e = VariantEngine(0)
    try:
        def batch_of(lo, hi, n):
            lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
            offs = np.zeros(n, dtype=np.uint64)
            offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
            total = int(offs[-1] + lens[-1]) + 16
            buf = torch.zeros(total, dtype=torch.uint8, device="cuda:0")
            b = E.Batch.from_records(offs, lens, E.KIND_IP, "cuda:0")
            e.synth(buf, b, E.SYNTH_TCP4, seed=int(lo))
            return buf, b, offs, lens

        def run(buf, b, offs, lens):
            host = buf.cpu().numpy().copy()
            e.emit(buf, b)
            torch.cuda.synchronize()
            ll = e.last_launch()
            ref = host.copy()
            oracle.batch_emit(ref, P.oracle_desc(offs, lens, E.KIND_IP), len(offs), 0, 0, E.KIND_IP, CAPS)
            assert np.array_equal(buf.cpu().numpy(), ref)
            return ll["variant"]

        short = batch_of(64, 300, 20000)
        assert run(*short) == 97  # a fresh context stages (no sample yet)
        assert run(*short) == 41  # nothing staged in the sample: in place
        assert e.kernel_for("emit", short[1]) == "dwalk_kernel"
        long_ = batch_of(3000, 9000, 4000)
        assert run(*long_) == 41  # (the decision of the last sample)
        for _ in range(70):  # the staged probe every 64 in-place calls, which then sticks
            v = run(*long_)
            if v == 97:
                break
        assert v == 97
        assert run(*long_) == 97
    finally:
        e.close()
