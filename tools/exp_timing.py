#!/usr/bin/env python3
"""Experiment: what the bench's timing instrumentation costs.  One step = emit(tx) + verify(rx);
K steps timed (a) on torch's current (null) stream vs a created stream, (b) with per-kernel timing
events between the kernels vs only around the K steps."""
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
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    K = 50
    dev = torch.device("cuda", 0)
    eng = E.ChecksumEngine(0)
    wl = bench.Workload(E, eng, cfg, 0, 0, dev)
    torch.cuda.synchronize()
    for rnd in range(2):
        for sname, s in (("current", torch.cuda.current_stream(dev)), ("created", torch.cuda.Stream(dev))):
            for per_kernel in (False, True):
                for blocking in (False,):
                    def step(ev=None):
                        if ev is not None:
                            ev[0].record(s)
                        eng.emit(wl.tx, wl.batch, stream=s)
                        if ev is not None:
                            ev[1].record(s)
                        eng.verify(wl.rx, wl.batch, status=wl.status, stream=s)
                        if ev is not None:
                            ev[2].record(s)
                    for _ in range(5):
                        step()
                    torch.cuda.synchronize()
                    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)] if per_kernel else None
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    a.record(s)
                    for i in range(K):
                        step(evs[i] if evs else None)
                    b.record(s)
                    torch.cuda.synchronize()
                    wall = (time.perf_counter() - t0) / K * 1e3
                    row = {"round": rnd, "stream": sname, "per_kernel_events": per_kernel,
                           "ms_per_step_events": round(a.elapsed_time(b) / K, 4), "ms_per_step_wall": round(wall, 4)}
                    if evs:
                        row["emit_ms"] = round(sum(e[0].elapsed_time(e[1]) for e in evs) / K, 4)
                        row["verify_ms"] = round(sum(e[1].elapsed_time(e[2]) for e in evs) / K, 4)
                    if rnd:
                        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
