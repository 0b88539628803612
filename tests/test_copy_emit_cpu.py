"""CPU checks of the copy + emit contract: the oracle's fused restatement equals memcpy followed
by the record emit, and the C ABI validates its arguments without a device."""
import ctypes

import numpy as np

import oracle
import smoltcp_amd
from smoltcp_amd import _lib
from smoltcp_amd.engine import COPY_DTYPE, make_copies
from tests import pktgen as P


def test_copy_dtype_matches_header():
    assert COPY_DTYPE.itemsize == 16 and oracle.COPY_DTYPE == COPY_DTYPE


def test_oracle_copy_emit_is_memcpy_then_emit():
    rng = np.random.default_rng(3)
    recs = []
    for i in range(64):
        pay = P.rand_bytes(rng, int(rng.integers(0, 300)))
        recs.append(P.ipv4(bytes(4), bytes([1, 2, 3, 4]), 17 if i % 2 else 6,
                           P.udp(1, 2, pay) if i % 2 else P.tcp(3, 4, pay)))
    buf, offs, lens = P.pack(recs, gap_rng=rng)
    hdr = np.array([28 if i % 2 else 40 for i in range(len(recs))], np.uint32)
    plen = lens - hdr
    plen[5] = lens[5] + 1 - hdr[5]  # does not fit
    src = rng.integers(0, 256, int(plen.sum()) + 64, dtype=np.uint8)
    soff = np.concatenate([[0], np.cumsum(plen[:-1].astype(np.uint64))]).astype(np.uint64) + 3
    copies = make_copies(soff, hdr, plen)
    desc = P.oracle_desc(offs, lens, 1)
    got = buf.copy()
    st = oracle.batch_copy_emit(got, desc, len(recs), src, copies)
    want = buf.copy()
    for i in range(len(recs)):
        if i == 5:
            continue
        a = int(offs[i]) + int(hdr[i])
        want[a:a + int(plen[i])] = src[int(soff[i]):int(soff[i]) + int(plen[i])]
    keep = np.ones(len(recs), bool)
    keep[5] = False
    ref_st = oracle.batch_emit(want, desc[keep], int(keep.sum()))
    assert np.array_equal(got, want)
    assert st[5] == 0x20 and np.array_equal(st[keep], ref_st)


def test_copy_emit_abi_argument_checks():
    L = smoltcp_amd.lib()
    b = _lib.BatchC()
    b.n = 1
    caps = _lib.Caps()
    assert L.smol_csum_batch_copy_emit(None, None, ctypes.byref(b), None, None, ctypes.byref(caps), None,
                                       None) == _lib.SMOL_EINVAL
