"""The sharded (N > 1) path with world size 2 over gloo.

Each rank takes its record range of one global batch (smoltcp_amd.shard), copies the byte range
it needs, checksums its shard, and the gathered per-rank results must equal one pass over the
whole batch.  On CPU the shard is processed by the oracle (these tests check the partitioning and
the reporting collectives, not the kernels); the `gpu` variant runs the HIP engine in both ranks
on cuda:0.  Rendezvous on 127.0.0.1.
"""
import os
import socket

import numpy as np
import pytest

import oracle
from smoltcp_amd import shard as S
from tests import pktgen as P

torch = pytest.importorskip("torch")
mp = pytest.importorskip("torch.multiprocessing")

WORLD = 2
V4A, V4B = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _records(n, seed):
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        pay = P.rand_bytes(rng, int(rng.integers(0, 1400)))
        l4 = P.udp(1000 + i, 53, pay) if i % 2 else P.tcp(2000 + i, 80, pay)
        recs.append(P.ipv4(V4A, V4B, 17 if i % 2 else 6, l4))
    return recs


def _fixed_global(n, stride, seed):
    recs = _records(n, seed)
    buf = np.zeros(n * stride + 16, dtype=np.uint8)
    for i, r in enumerate(recs):
        buf[i * stride:i * stride + len(r)] = np.frombuffer(r, dtype=np.uint8)
    return buf


def _init(rank, port):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(WORLD),
                      RANK=str(rank), LOCAL_RANK="0")
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    return dist


def _oracle_shard(buf, sh, kind=1):
    """Emit then verify the shard's byte range on the oracle: (bytes, emit status, verify status)."""
    local = buf[sh.byte_lo:sh.byte_hi].copy()
    local = np.concatenate([local, np.zeros(16, dtype=np.uint8)])
    if sh.desc is not None:
        est = oracle.batch_emit(local, sh.desc, sh.n)
        vst = oracle.batch_verify(local, sh.desc, sh.n)
    else:
        est = oracle.batch_emit(local, None, sh.n, sh.stride, sh.length, kind)
        vst = oracle.batch_verify(local, None, sh.n, sh.stride, sh.length, kind)
    return local[:sh.byte_hi - sh.byte_lo], est, vst


def _worker_cpu(rank, port):
    dist = _init(rank, port)
    try:
        # fixed stride: 37 records of 1500 B (odd count: ranks get 19 and 18)
        n, stride = 37, 1500
        g = _fixed_global(n, stride, seed=7)
        sh = S.shard_fixed(n, stride, stride, rank, WORLD)
        part = _oracle_shard(g, sh)
        parts = [None] * WORLD
        dist.all_gather_object(parts, (sh.lo, sh.hi, sh.byte_lo, part))
        if rank == 0:
            whole = g.copy()
            est = oracle.batch_emit(whole, None, n, stride, stride, 1)
            vst = oracle.batch_verify(whole, None, n, stride, stride, 1)
            assert sum(p[1] - p[0] for p in parts) == n
            for lo, hi, b0, (bytes_, e, v) in parts:
                assert np.array_equal(bytes_, whole[b0:b0 + len(bytes_)])
                assert np.array_equal(e, est[lo:hi]) and np.array_equal(v, vst[lo:hi])
            assert (vst & 0x80).all()  # emitted records verify

        # packed odd offsets + descriptors (rebased per shard)
        rng = np.random.default_rng(11)
        buf, offs, lens = P.pack(_records(25, seed=12), gap_rng=rng)
        desc = P.oracle_desc(offs, lens, 1)
        sh = S.shard_records(desc, rank, WORLD)
        part = _oracle_shard(buf, sh)
        dist.all_gather_object(parts, (sh.lo, sh.hi, sh.byte_lo, part))
        if rank == 0:
            whole = buf.copy()
            est = oracle.batch_emit(whole, desc, len(desc))
            vst = oracle.batch_verify(whole, desc, len(desc))
            for lo, hi, b0, (bytes_, e, v) in parts:
                assert np.array_equal(bytes_, whole[b0:b0 + len(bytes_)])
                assert np.array_equal(e, est[lo:hi]) and np.array_equal(v, vst[lo:hi])

        # reporting collectives: max over ranks, whole-job aggregate
        m = S.max_over_ranks(1.5 + rank)
        assert m == 2.5
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _worker_gpu(rank, port):
    dist = _init(rank, port)
    try:
        from smoltcp_amd import engine as E

        eng = E.ChecksumEngine(0)
        n, stride = 4099, 1500
        g = _fixed_global(n, stride, seed=21)
        sh = S.shard_fixed(n, stride, stride, rank, WORLD)
        d = torch.from_numpy(np.concatenate([g[sh.byte_lo:sh.byte_hi], np.zeros(16, np.uint8)])).to("cuda:0")
        b = E.Batch.fixed(sh.n, stride, stride, E.KIND_IP)
        est = torch.zeros(sh.n, dtype=torch.uint8, device="cuda:0")
        eng.emit(d, b, status=est)
        vst = eng.verify(d, b)
        part = (d.cpu().numpy()[:sh.byte_hi - sh.byte_lo], est.cpu().numpy(), vst.cpu().numpy())
        parts = [None] * WORLD
        dist.all_gather_object(parts, (sh.lo, sh.hi, sh.byte_lo, part))
        if rank == 0:
            whole = g.copy()
            e_ref = oracle.batch_emit(whole, None, n, stride, stride, 1)
            v_ref = oracle.batch_verify(whole, None, n, stride, stride, 1)
            for lo, hi, b0, (bytes_, e, v) in parts:
                assert np.array_equal(bytes_, whole[b0:b0 + len(bytes_)])
                assert np.array_equal(e, e_ref[lo:hi]) and np.array_equal(v, v_ref[lo:hi])
        eng.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_shard_ranges_cover_and_balance():
    for n in (0, 1, 2, 7, 1 << 20, (1 << 20) + 3):
        for w in (1, 2, 3, 8):
            rs = [S.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            sizes = [hi - lo for lo, hi in rs]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        S.shard_range(4, 2, 2)


def test_shard_geometry():
    sh = S.shard_fixed(10, 1500, 1400, 1, 2)
    assert (sh.lo, sh.hi, sh.byte_lo, sh.byte_hi) == (5, 10, 7500, 9 * 1500 + 1400)
    desc = P.oracle_desc(np.array([3, 100, 7, 50], np.uint64), np.array([10, 20, 30, 5], np.uint32), 1)
    sh = S.shard_records(desc, 1, 2)
    assert (sh.byte_lo, sh.byte_hi) == (7, 55)
    assert list(sh.desc["offset"]) == [0, 43]
    assert S.rank_seed(5, 0) != S.rank_seed(5, 1)
    assert S.aggregate_rate(1 << 30, 2, 4, 2.0) == 4.0
    assert S.max_over_ranks(3.25) == 3.25  # no process group: identity


def test_sharded_batch_gloo_world2():
    mp.spawn(_worker_cpu, args=(_free_port(),), nprocs=WORLD, join=True)


@pytest.mark.gpu
def test_sharded_batch_gpu_world2():
    """Both ranks on the box's one GPU, each running the HIP engine on its shard."""
    assert torch.cuda.is_available()
    mp.spawn(_worker_gpu, args=(_free_port(),), nprocs=WORLD, join=True)
