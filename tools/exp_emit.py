#!/usr/bin/env python3
"""Experiment: is emit slower than verify because of the kernel or because of the buffer state
(dirty lines left by the previous emit)?  Times emit/verify on both C2 buffers in several orders."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from smoltcp_amd import engine as E  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    eng = E.ChecksumEngine(0)
    wl = bench.Workload(E, eng, "c2", 0, 0, dev)
    s = torch.cuda.current_stream(dev)
    st = wl.status

    def t(name, fn, reps=10):
        for _ in range(2):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            fn()
        b.record(s)
        torch.cuda.synchronize()
        print(json.dumps({"case": name, "ms": round(a.elapsed_time(b) / reps, 4)}), flush=True)

    for var in (0, 1):
        eng.set_variant(var)
        print("variant", var)
        t("emit(tx)", lambda: eng.emit(wl.tx, wl.batch, stream=s))
        t("verify(tx) after emits", lambda: eng.verify(wl.tx, wl.batch, status=st, stream=s))
        t("verify(rx)", lambda: eng.verify(wl.rx, wl.batch, status=st, stream=s))
        t("emit(tx) caps=ignored", lambda: eng.emit(wl.tx, wl.batch, caps=(3, 3, 3, 3, 3), stream=s))
        t("emit(tx)+verify(rx)", lambda: (eng.emit(wl.tx, wl.batch, stream=s), eng.verify(wl.rx, wl.batch, status=st, stream=s)))
        t("verify(tx)+verify(rx)", lambda: (eng.verify(wl.tx, wl.batch, status=st, stream=s), eng.verify(wl.rx, wl.batch, status=st, stream=s)))
        sink = torch.zeros(1, dtype=torch.int32, device=dev)
        t("stream_read(tx)", lambda: eng.stream_read(wl.tx, sink, stream=s))


if __name__ == "__main__":
    main()
