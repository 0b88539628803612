#!/usr/bin/env python3
"""Experiment (round 5): fixed-stride emit variants on C2 / C4 at steady clocks, over R = 4 TX
batches in turn (every emit a batch its previous pass did not just write, as the bench's timed steps
do since round 5), interleaved rounds on one box.  Verify of the RX batch is timed in the same
rounds as the reference.  Store variants must leave the bytes of the first variant listed; `| 64`
variants (experiments: stores compiled out) are timing only.
XCDS=-1,1,16: the emit variants under each XCD block mapping in turn (smol_csum_set_xcd_remap; -1 the
default), reported as `<variant>x<remap>`.
Usage: [VARS=29,5,31,32] [VVARS=-1,13 (verify variants)] [XCDS=-1] [K=32] [ROUNDS=4] exp_r05_emit.py [c2,c4]"""
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
    R = int(os.environ.get("R", "4"))
    wls = {c: bench.Workload(E, eng, c, 0, 0, dev, R) for c in cfgs}
    torch.cuda.synchronize()
    vars_ = [int(x) for x in os.environ.get("VARS", "29,5,31,32").split(",")]

    for c, wl in wls.items():  # the same bytes from every store variant
        ref = None
        for v in vars_:
            if v >= 64:
                continue
            t = wl.tx.clone()
            eng.set_variant(v)
            eng.emit(t, wl.batch)
            torch.cuda.synchronize()
            if ref is None:
                ref = t
            else:
                same = bool(torch.equal(ref, t))
                print(json.dumps({"cfg": c, "variant": v, "identical_to_first": same}), flush=True)
                if not same:
                    raise SystemExit(f"{c}: variant {v} differs from variant {vars_[0]}")
            del t
        del ref
    eng.set_variant(-1)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for wl in wls.values():
            for j in range(R):
                eng.emit(wl.txs[j], wl.batch)
                eng.verify(wl.rxs[j], wl.batch, status=wl.status)
        torch.cuda.synchronize()
    K = int(os.environ.get("K", "32"))

    def timed(fn):
        for j in range(R):
            fn(j)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(K):
            fn(i % R)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / K

    for rnd in range(int(os.environ.get("ROUNDS", "4"))):
        for c, wl in wls.items():
            for vv in [int(x) for x in os.environ.get("VVARS", "-1").split(",")]:
                eng.set_variant(vv)
                ver = timed(lambda j: eng.verify(wl.rxs[j], wl.batch, status=wl.status))
                name = "verify" if vv < 0 else f"verify{vv}"
                print(json.dumps({"round": rnd, "cfg": c, "variant": name, "ms": round(ver, 4)}), flush=True)
            for x in [int(y) for y in os.environ.get("XCDS", "-1").split(",")]:
                eng.set_xcd_remap(x)
                for v in vars_:
                    eng.set_variant(v)
                    fresh = timed(lambda j: eng.emit(wl.txs[j], wl.batch))
                    same = timed(lambda j: eng.emit(wl.txs[0], wl.batch))
                    print(json.dumps({"round": rnd, "cfg": c, "variant": v if x < 0 else f"{v}x{x}",
                                      "emit_fresh_ms": round(fresh, 4), "emit_same_ms": round(same, 4)}), flush=True)
                eng.set_xcd_remap(-1)
    eng.set_variant(-1)


if __name__ == "__main__":
    main()
