#!/usr/bin/env python3
"""Experiment: emit variants (whole 64-B field segments: 19, 23-27; 2-B stores: 5, 13; the tile
kernel: 7) on C2 / C3 / C4 at steady clocks, interleaved rounds on one box; every variant must leave
the same bytes as the first one listed.
Usage: [VARS=5,19,23] [VARS_c3=7,26,27] [K=30] [NOCHECK=34 (variants allowed to differ)] exp_emit_seg.py [c2,c4,c3]"""
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
    eng.set_xcd_remap(int(os.environ.get("XCD", "-1")))
    wls = {c: bench.Workload(E, eng, c, 0, 0, dev) for c in cfgs}
    torch.cuda.synchronize()
    def vars_of(c):
        return [int(x) for x in os.environ.get(f"VARS_{c}", os.environ.get("VARS", "5,19")).split(",")]

    for c, wl in wls.items():  # the same bytes from every variant
        ref = None
        for v in vars_of(c):
            t = wl.tx.clone()
            eng.set_variant(v)
            eng.emit(t, wl.batch)
            torch.cuda.synchronize()
            if ref is None:
                ref = t
            else:
                same = bool(torch.equal(ref, t))
                print(json.dumps({"cfg": c, "variant": v, "identical_to_first": same}), flush=True)
                if not same and str(v) not in os.environ.get("NOCHECK", "").split(","):
                    raise SystemExit(f"{c}: variant {v} differs from variant {vars_of(c)[0]}")
                del t
        del ref
    eng.set_variant(-1)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for wl in wls.values():
            eng.emit(wl.tx, wl.batch)
        torch.cuda.synchronize()
    K = int(os.environ.get("K", "30"))
    for rnd in range(4):
        for c, wl in wls.items():
            for v in vars_of(c):
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
