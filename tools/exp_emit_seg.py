#!/usr/bin/env python3
"""Experiment: emit with the fields' 64-B segments written whole (variant 19) against variant 5,
on C2 and C4 at steady clocks, interleaved; both must leave the same bytes.
Usage: exp_emit_seg.py [c2,c4]"""
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
    cfgs = (sys.argv[1] if len(sys.argv) > 1 else "c2,c4").split(",")
    dev = torch.device("cuda", 0)
    eng = E.ChecksumEngine(0)
    wls = {c: bench.Workload(E, eng, c, 0, 0, dev) for c in cfgs}
    torch.cuda.synchronize()
    for c, wl in wls.items():  # same bytes from both variants
        outs = []
        for v in (5, 19):
            t = wl.tx.clone()
            eng.set_variant(v)
            eng.emit(t, wl.batch)
            torch.cuda.synchronize()
            outs.append(t)
        print(json.dumps({"cfg": c, "identical": bool(torch.equal(outs[0], outs[1]))}), flush=True)
        del outs
    eng.set_variant(-1)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for wl in wls.values():
            eng.emit(wl.tx, wl.batch)
        torch.cuda.synchronize()
    K = int(os.environ.get("K", "30"))
    VARS = [int(x) for x in os.environ.get("VARS", "5,19").split(",")]
    for rnd in range(4):
        for c, wl in wls.items():
            for v in VARS:
                eng.set_variant(v)
                for _ in range(3):
                    eng.emit(wl.tx, wl.batch)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(K):
                    eng.emit(wl.tx, wl.batch)
                b.record()
                torch.cuda.synchronize()
                if rnd:
                    print(json.dumps({"round": rnd, "cfg": c, "variant": v, "emit_ms": round(a.elapsed_time(b) / K, 4)}),
                          flush=True)
    eng.set_variant(-1)


if __name__ == "__main__":
    main()
