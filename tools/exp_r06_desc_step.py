#!/usr/bin/env python3
"""Experiment (round 6): descriptor-batch emit variants in bench.py's step order, over record-length
mixes and layouts: R = 4 TX / RX batch pairs in turn, each step = emit of TX batch i (the variant under
test) + verify of RX batch i (the library's default), HIP events around each kernel; K timed steps
after 3R untimed ones, interleaved over rounds.  Synthetic IPv4/TCP; layouts: packed (C3), random
0-7-byte gaps, shuffled descriptors, short records (64-1500 B) packed and gapped.
Usage: SMOLCSUM_LIB=.../libsmolcsum_exp.so [VARS=41,94] [CASES=c3_packed,...] [K=12] exp_r06_desc_step.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from smoltcp_amd import engine as E  # noqa: E402

CASES = [("c3_packed", 64, 9000, False, False), ("c3_gapped", 64, 9000, True, False),
         ("c3_shuffled", 64, 9000, False, True), ("short_packed", 64, 1500, False, False),
         ("short_gapped", 64, 1500, True, False), ("mid_packed", 500, 3000, False, False)]


def main():
    eng = E.ChecksumEngine(0)
    K, R = int(os.environ.get("K", "12")), 4
    vars_ = [int(x) for x in os.environ.get("VARS", "41,94").split(",")]
    only = os.environ.get("CASES")
    rng = np.random.default_rng(6)
    for name, lo, hi, gapped, shuffled in CASES:
        if only and name not in only.split(","):
            continue
        n = 1 << 20
        lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
        gaps = rng.integers(0, 8, n).astype(np.uint64) if gapped else np.zeros(n, np.uint64)
        offs = np.zeros(n, dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[1:])
        total = int(offs[-1] + lens[-1]) + 16
        if shuffled:
            p = rng.permutation(n)
            offs, lens = offs[p], lens[p]
        batch = E.Batch.from_records(offs, lens, E.KIND_IP, "cuda:0")
        txs, rxs = [], []
        for j in range(R):
            t = torch.zeros(total, dtype=torch.uint8, device="cuda:0")
            eng.synth(t, batch, E.SYNTH_TCP4, seed=7 + j)
            r = t.clone()
            eng.emit(r, batch)
            eng.corrupt(r, batch, every=64, seed=j)
            txs.append(t)
            rxs.append(r)
        st = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        # the variants write the same bytes
        ref = None
        for v in vars_:
            eng.set_variant(v)
            t = txs[0].clone()
            eng.emit(t, batch)
            ref = t if ref is None else ref
            assert torch.equal(ref, t), (name, v)
            del t
        eng.set_variant(-1)
        del ref
        res = {}
        for _ in range(3):
            for v in vars_:
                ev = []
                for i in range(K + 3 * R):
                    j = i % R
                    a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                    eng.set_variant(v)
                    a.record()
                    eng.emit(txs[j], batch)
                    b.record()
                    eng.set_variant(-1)
                    eng.verify(rxs[j], batch, status=st)
                    c.record()
                    if i >= 3 * R:
                        ev.append((a, b, c))
                torch.cuda.synchronize()
                res.setdefault(f"emit{v}", []).append(sum(a.elapsed_time(b) for a, b, _ in ev) / K)
                res.setdefault(f"verify_after{v}", []).append(sum(b.elapsed_time(c) for _, b, c in ev) / K)
                res.setdefault(f"step{v}", []).append(sum(a.elapsed_time(c) for a, _, c in ev) / K)
        eng.set_variant(-1)
        print(json.dumps({"case": name, "n": n, "bytes": int(lens.astype(np.uint64).sum()),
                          **{k: round(min(t), 4) for k, t in res.items()}}), flush=True)
        del txs, rxs


if __name__ == "__main__":
    main()
