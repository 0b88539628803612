#!/usr/bin/env python3
"""Experiment (round 5): verify / emit over descriptor batches, the default kernels against the
transposed walk over descriptor batches (variant 56, experiments build), for record-length mixes and
layouts: packed (C3), random 0-7-byte gaps between records, descriptors in shuffled order; ~2-4.7 GB
per batch of synthetic IPv4/TCP.  Interleaved rounds, K launches each, one JSON line per case.
fixed1320 / fixed1500: fixed-length records given as descriptors, beside the fixed-stride batch's default.
Usage: SMOLCSUM_LIB=.../libsmolcsum_exp.so [VARS=-1,56] [CASES=c3_packed,...] [K=16] exp_r05_desc.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from smoltcp_amd import engine as E  # noqa: E402


def main():
    eng = E.ChecksumEngine(0)
    K = int(os.environ.get("K", "16"))
    vars_ = [int(x) for x in os.environ.get("VARS", "-1,56").split(",")]
    rng = np.random.default_rng(5)
    cases = [("c3_packed", 64, 9000, False, False), ("c3_gapped", 64, 9000, True, False),
             ("c3_shuffled", 64, 9000, False, True), ("short_packed", 64, 1500, False, False),
             ("short_gapped", 64, 1500, True, False), ("fixed1320", 1320, 1320, False, False),
             ("fixed1500", 1500, 1500, False, False)]
    only = os.environ.get("CASES")
    for name, lo, hi, gapped, shuffled in cases:
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
        buf = torch.zeros(total, dtype=torch.uint8, device="cuda:0")
        batch = E.Batch.from_records(offs, lens, E.KIND_IP, "cuda:0")
        eng.synth(buf, batch, E.SYNTH_TCP4, seed=7)
        eng.emit(buf, batch)
        st = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        res = {}
        for rnd in range(3):
            for v in vars_:
                eng.set_variant(v)
                for op in ("verify", "emit"):
                    fn = (lambda: eng.verify(buf, batch, status=st)) if op == "verify" else (lambda: eng.emit(buf, batch))
                    for _ in range(3):
                        fn()
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(K):
                        fn()
                    b.record()
                    torch.cuda.synchronize()
                    res.setdefault(f"{op}{v}", []).append(a.elapsed_time(b) / K)
        eng.set_variant(-1)
        if lo == hi:  # the same records as a fixed-stride batch, the library's default for it
            fb = E.Batch.fixed(n, lo, lo, E.KIND_IP)
            for rnd in range(3):
                for _ in range(3):
                    eng.verify(buf, fb, status=st)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(K):
                    eng.verify(buf, fb, status=st)
                b.record()
                torch.cuda.synchronize()
                res.setdefault("verify_fixed_default", []).append(a.elapsed_time(b) / K)
        print(json.dumps({"case": name, "n": n, "bytes": int(lens.astype(np.uint64).sum()),
                          **{k: round(min(t), 4) for k, t in res.items()}}), flush=True)
        del buf


if __name__ == "__main__":
    main()
