#!/usr/bin/env python3
"""Launch-shape sweep for the checksum kernels (tuning tool): times emit and verify for every
shape x {nt, plain} x grid cap on one workload, interleaved in one process.

    python tools/sweep.py [--config c2|c3|c4] [--n N] [--reps R]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from smoltcp_amd import engine as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--shapes", default="0,1,2,3,4,5,6,7,8")
    ap.add_argument("--blocks", default="0")
    ap.add_argument("--var", default="0,1,2")
    ap.add_argument("--tile", default="32")
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = E.ChecksumEngine(0)
    wl = bench.Workload(E, eng, args.config, args.n, 0, dev)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(dev)
    rows = []
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    import time
    t0 = time.perf_counter()  # clock ramp (bench.py --ramp-ms): 0.3 s of steps before timing
    while time.perf_counter() - t0 < 0.3:
        for _ in range(8):
            eng.emit(wl.tx, wl.batch, stream=s)
            eng.verify(wl.rx, wl.batch, status=wl.status, stream=s)
        torch.cuda.synchronize()
    for rnd in range(args.rounds):
        for shape in [int(x) for x in args.shapes.split(",")]:
            for var, bpc, tile in [(a, b, d) for a in [int(x) for x in args.var.split(",")]
                                   for b in [int(x) for x in args.blocks.split(",")]
                                   for d in [int(x) for x in args.tile.split(",")]]:
                if True:
                    eng.set_shape(shape)
                    eng.set_variant(var)
                    eng.set_tile(tile)
                    eng.set_max_blocks(bpc * cus)
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                    for _ in range(2):
                        eng.emit(wl.tx, wl.batch, stream=s)
                        eng.verify(wl.rx, wl.batch, status=wl.status, stream=s)
                    ev[0].record(s)
                    for _ in range(args.reps):
                        eng.emit(wl.tx, wl.batch, stream=s)
                    ev[1].record(s)
                    for _ in range(args.reps):
                        eng.verify(wl.rx, wl.batch, status=wl.status, stream=s)
                    ev[2].record(s)
                    torch.cuda.synchronize()
                    em = ev[0].elapsed_time(ev[1]) / args.reps
                    vm = ev[1].elapsed_time(ev[2]) / args.reps
                    row = {"round": rnd, "shape": shape, "var": var, "blocks_per_cu": bpc, "tile": tile,
                           "emit_ms": round(em, 4), "verify_ms": round(vm, 4),
                           "emit_GBs": round(wl.read_bytes / em / 1e6, 1),
                           "verify_GBs": round(wl.read_bytes / vm / 1e6, 1)}
                    rows.append(row)
                    print(json.dumps(row), flush=True)
    eng.set_shape(-1)
    eng.set_variant(-1)
    eng.set_max_blocks(0)


if __name__ == "__main__":
    main()
