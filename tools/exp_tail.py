#!/usr/bin/env python3
"""Experiment: how much a kernel boundary (the last workgroups draining, the next launch filling
the chip) costs in the C2 step.  Emit and verify over batches of 2^19, 2^20 and 2^21 C2 records,
timed per launch at steady clocks: if a launch over twice the records takes twice the time, the
boundary is free.  One JSON line per (records, op)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from smoltcp_amd import engine as E  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    eng = E.ChecksumEngine(0)
    wls = {n: bench.Workload(E, eng, "c2", n, 0, dev) for n in (1 << 19, 1 << 20, 1 << 21)}
    torch.cuda.synchronize()
    big = wls[1 << 21]
    t0 = time.perf_counter()  # clock ramp
    while time.perf_counter() - t0 < 0.3:
        for _ in range(4):
            eng.emit(big.tx, big.batch)
            eng.verify(big.rx, big.batch, status=big.status)
        torch.cuda.synchronize()
    K = 40
    for rnd in range(3):
        for n, wl in wls.items():
            for op in ("emit", "verify", "step"):
                def one():
                    if op in ("emit", "step"):
                        eng.emit(wl.tx, wl.batch)
                    if op in ("verify", "step"):
                        eng.verify(wl.rx, wl.batch, status=wl.status)
                for _ in range(3):
                    one()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(K):
                    one()
                b.record()
                torch.cuda.synchronize()
                ms = a.elapsed_time(b) / K
                if rnd:
                    print(json.dumps({"round": rnd, "records": n, "op": op, "ms": round(ms, 4),
                                      "ms_per_2^20": round(ms * (1 << 20) / n, 4)}), flush=True)


if __name__ == "__main__":
    main()
