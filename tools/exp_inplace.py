#!/usr/bin/env python3
"""Experiment: why is the in-place step (C5: emit then verify of ONE buffer) slower per record than
C2's step (emit of the TX buffer, verify of a separate RX buffer) at the same size?

Two C2-sized buffers A and B (2^20 x 1500 B IPv4/UDP, emitted, so emit rewrites the same values).
Sequences, each timed per kernel with HIP events on one stream, interleaved rounds on one box:
  c2      emit A, verify B      (the C2 step)
  inplace emit A, verify A      (the C5 step)
  emit    emit A, emit A        (emit only)
  verify  verify A, verify A    (verify only)
  vv      verify A, verify B    (two read-only passes over different buffers)
  ev_swap emit A, verify B, emit B, verify A  (emit's buffer verified one kernel later)
Usage: exp_inplace.py [n_records] [seq,seq,...]   (SIZES="17,18,..." runs log2 sizes in turn;
XCD_EMIT / XCD_VERIFY = 1: that kernel with the XCD-contiguous block order)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from smoltcp_amd import engine as E  # noqa: E402


def main():
    sizes = [1 << int(x) for x in os.environ["SIZES"].split(",")] if os.environ.get("SIZES") else \
        [int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20]
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    for n in sizes:
        run(n, only)
        torch.cuda.empty_cache()


def run(n, only):
    L = 1500
    eng = E.ChecksumEngine(0)
    dev = torch.device("cuda", 0)
    b = E.Batch.fixed(n, L, L, E.KIND_IP)
    bufs = {}
    need_b = only is None or any(k in ("c2", "vv", "ev_swap") for k in only)
    for name, seed in (("A", 1), ("B", 2)) if need_b else (("A", 1),):
        t = torch.empty(n * L, dtype=torch.uint8, device=dev)
        eng.synth(t, b, E.SYNTH_UDP4, seed)
        eng.emit(t, b)
        bufs[name] = t
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    xe, xv = int(os.environ.get("XCD_EMIT", "-1")), int(os.environ.get("XCD_VERIFY", "-1"))

    def emit(x):
        eng.set_xcd_remap(xe)
        eng.emit(bufs[x], b)

    def verify(x):
        eng.set_xcd_remap(xv)
        eng.verify(bufs[x], b, status=st)

    seqs = {
        "c2": [("emit", emit, "A"), ("verify", verify, "B")],
        "inplace": [("emit", emit, "A"), ("verify", verify, "A")],
        "emit": [("emit", emit, "A"), ("emit", emit, "A")],
        "verify": [("verify", verify, "A"), ("verify", verify, "A")],
        "vv": [("verify", verify, "A"), ("verify", verify, "B")],
        "ev_swap": [("emit", emit, "A"), ("verify", verify, "B"), ("emit", emit, "B"), ("verify", verify, "A")],
    }
    if only:
        seqs = {k: v for k, v in seqs.items() if k in only}
    t0 = time.perf_counter()  # clock ramp
    while time.perf_counter() - t0 < 0.3:
        for _ in range(8):
            emit("A")
            verify("B" if need_b else "A")
        torch.cuda.synchronize()
    K = int(os.environ.get("K", "20"))
    for rnd in range(int(os.environ.get("ROUNDS", "4"))):
        for name, seq in seqs.items():
            for _ in range(2):
                for _, fn, x in seq:
                    fn(x)
            evs = []
            for _ in range(K):
                for kind, fn, x in seq:
                    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    fn(x)
                    z.record()
                    evs.append((kind, a, z))
            torch.cuda.synchronize()
            per = {}
            for kind, a, z in evs:
                per.setdefault(kind, []).append(a.elapsed_time(z))
            if rnd:
                print(json.dumps({"round": rnd, "seq": name, "n": n, "xcd_emit": xe, "xcd_verify": xv,
                                  **{f"{k}_ms": round(sum(v) / len(v), 4) for k, v in per.items()}}), flush=True)


if __name__ == "__main__":
    main()
