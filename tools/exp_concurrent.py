#!/usr/bin/env python3
"""Experiment: one bench step (emit over the TX batch + verify over the RX batch) issued
(a) serially on one stream, (b) on two streams (TX and RX concurrently), (c) captured in a HIP
graph (serial), (d) a graph with a TX / RX fork-join.  Times steps with HIP events."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from smoltcp_amd import engine as E  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    reps = 50
    dev = torch.device("cuda", 0)
    eng = E.ChecksumEngine(0)
    wl = bench.Workload(E, eng, cfg, 0, 0, dev)
    s0 = torch.cuda.Stream(dev)
    s1 = torch.cuda.Stream(dev)
    torch.cuda.synchronize()

    def serial():
        eng.emit(wl.tx, wl.batch, stream=s0)
        eng.verify(wl.rx, wl.batch, status=wl.status, stream=s0)

    def forked(main=s0, side=s1):
        ev = torch.cuda.Event()
        ev.record(main)
        side.wait_event(ev)
        eng.emit(wl.tx, wl.batch, stream=main)
        eng.verify(wl.rx, wl.batch, status=wl.status, stream=side)
        ev2 = torch.cuda.Event()
        ev2.record(side)
        main.wait_event(ev2)

    def rev():
        eng.verify(wl.rx, wl.batch, status=wl.status, stream=s0)
        eng.emit(wl.tx, wl.batch, stream=s0)

    def timeit(name, fn, steps_per_call=1):
        # everything (including graph replays, which launch on the current stream) runs on s0
        with torch.cuda.stream(s0):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s0)
            for _ in range(reps):
                fn()
            b.record(s0)
            torch.cuda.synchronize()
        ms = a.elapsed_time(b) / reps / steps_per_call
        gib = 2 * wl.span_bytes / (ms * 1e-3) / 2**30
        print(json.dumps({"cfg": cfg, "case": name, "ms_per_step": round(ms, 4), "GiB/s": round(gib, 1)}), flush=True)

    for rnd in range(2):
        timeit("serial, one stream", serial)
        timeit("verify then emit, one stream", rev)
        timeit("tx / rx on two streams", forked)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s0):
            for _ in range(10):
                serial()
        timeit("graph of 10 serial steps (per step)", lambda: g.replay(), 10)
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2, stream=s0):
            for _ in range(10):
                forked()
        timeit("graph of 10 forked steps (per step)", lambda: g2.replay(), 10)


if __name__ == "__main__":
    main()
