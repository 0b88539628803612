#!/usr/bin/env python3
"""Experiment: is the read stream slower over a very large buffer (C5: 201 GB in one allocation)
because of the span (address translation) or because of where the pages sit?

stream_read_kernel (the bench's read-only probe) over 1.5-GB windows at the start, middle and end
of one big allocation, over the whole allocation, and over a separate 1.5-GB allocation; then emit
of C5's 1500-B records over the same windows and over the whole buffer.
Usage: exp_bigbuf.py [GB]   (default 201)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from smoltcp_amd import engine as E  # noqa: E402


def timed(fn, reps):
    for _ in range(2):
        fn()
    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    z.record()
    torch.cuda.synchronize()
    return a.elapsed_time(z) / reps


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 201.0
    L = 1500
    eng = E.ChecksumEngine(0)
    dev = torch.device("cuda", 0)
    n_all = int(gb * 1e9) // L
    big = torch.empty(n_all * L, dtype=torch.uint8, device=dev)
    eng.synth(big, E.Batch.fixed(n_all, L, L, E.KIND_IP), E.SYNTH_UDP4, 7)
    eng.emit(big, E.Batch.fixed(n_all, L, L, E.KIND_IP))
    n_win = 1 << 20
    small = torch.empty(n_win * L, dtype=torch.uint8, device=dev)
    eng.synth(small, E.Batch.fixed(n_win, L, L, E.KIND_IP), E.SYNTH_UDP4, 8)
    eng.emit(small, E.Batch.fixed(n_win, L, L, E.KIND_IP))
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()  # clock ramp
    while time.perf_counter() - t0 < 0.3:
        eng.stream_read(small, sink)
        torch.cuda.synchronize()
    wins = {"start": 0, "middle": (n_all // 2) * L, "end": (n_all - n_win) * L}
    b_win = E.Batch.fixed(n_win, L, L, E.KIND_IP)
    for rnd in range(3):
        out = {"round": rnd}
        out["separate_read_TBs"] = round(small.numel() / timed(lambda: eng.stream_read(small, sink), 20) / 1e9, 3)
        out["separate_emit_ms"] = round(timed(lambda: eng.emit(small, b_win), 20), 4)
        for name, off in wins.items():
            v = big[off: off + n_win * L]
            out[f"{name}_read_TBs"] = round(v.numel() / timed(lambda: eng.stream_read(v, sink), 20) / 1e9, 3)
            out[f"{name}_emit_ms"] = round(timed(lambda: eng.emit(v, b_win), 20), 4)
        nb = big.numel() // 16 * 16
        out["whole_read_TBs"] = round(nb / timed(lambda: eng.stream_read(big, sink), 2) / 1e9, 3)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
