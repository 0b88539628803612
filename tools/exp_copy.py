#!/usr/bin/env python3
"""Time the fused copy + emit (C2copy workload) per launch shape and kernel variant: one JSON line each.

Usage: [XCD=K] exp_copy.py [shapes, e.g. 0,1,3,5] [variants, e.g. 8,11,12]   (XCD: the block order, see
smol_csum_tool_set_xcd_remap)"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smoltcp_amd import engine as E  # noqa: E402


def main():
    n, L = 1 << 20, 1500
    eng = E.ChecksumEngine(0)
    eng.set_xcd_remap(int(os.environ.get("XCD", "-1")))
    dev = torch.device("cuda:0")
    tx = torch.empty(n * L, dtype=torch.uint8, device=dev)
    b = E.Batch.fixed(n, L, L, E.KIND_IP)
    eng.synth(tx, b, E.SYNTH_UDP4, 0x5EED0006)
    src = torch.randint(0, 256, (n * 1472 + 16,), dtype=torch.uint8, device=dev)
    cp = torch.from_numpy(E.make_copies(np.arange(n, dtype=np.uint64) * 1472, 28, 1472).view(np.uint8).copy()).to(dev)
    variants = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "-1").split(",")]
    import time
    t0 = time.perf_counter()  # clock ramp (bench.py --ramp-ms)
    while time.perf_counter() - t0 < 0.3:
        for _ in range(8):
            eng.copy_emit(tx, b, src, cp)
        torch.cuda.synchronize()
    shapes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,3,5").split(",")]
    K = int(os.environ.get("K", "20"))
    ref = None
    for rnd, shape, var in [(r, s, v) for r in range(int(os.environ.get("ROUNDS", "3"))) for s in shapes for v in variants]:
        eng.set_shape(shape)
        eng.set_variant(var)
        for _ in range(3):
            eng.copy_emit(tx, b, src, cp)
        if rnd == 0:  # every (shape, variant) leaves the same bytes
            torch.cuda.synchronize()
            if ref is None:
                ref = tx.clone()
            elif not torch.equal(ref, tx) and str(var) not in os.environ.get("NOCHECK", "").split(","):
                raise SystemExit(f"shape {shape} variant {var}: copy-emit output differs from the first one's")
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(K):
            eng.copy_emit(tx, b, src, cp)
        z.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(z) / K
        moved = n * (28 + 1472 + 1472 + 4)
        print(json.dumps({"round": rnd, "shape": shape, "variant": var, "ms": round(ms, 4), "GBs_rw": round(moved / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
