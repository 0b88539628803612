#!/usr/bin/env python3
"""C3 emit tax vs record alignment (tuning experiment): the C3 lengths (U[64,9000], 2^20 TCP/IPv4
records) laid out with every record start rounded up to A bytes (A = 1 is C3 itself: packed, odd
offsets).  Times emit and verify per kernel variant, interleaved, one JSON line each.

    python tools/exp_c3align.py [aligns, e.g. 1,2,4,16,128] [variants, e.g. 7,13]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smoltcp_amd import engine as E  # noqa: E402


def main():
    aligns = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4,16,128").split(",")]
    variants = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "7,13").split(",")]
    n = 1 << 20
    dev = torch.device("cuda:0")
    eng = E.ChecksumEngine(0)
    rng = np.random.default_rng(0x5EED0002)
    lens = rng.integers(64, 9001, n).astype(np.uint64)
    wls = {}
    for A in aligns:
        slot = (lens + (A - 1)) // A * A
        offs = np.zeros(n, dtype=np.uint64)
        offs[1:] = np.cumsum(slot[:-1])
        b = E.Batch.from_records(offs, lens.astype(np.uint32), E.KIND_IP, dev)
        tot = int(offs[-1] + lens[-1]) + 256
        tx = torch.zeros(tot, dtype=torch.uint8, device=dev)
        eng.synth(tx, b, E.SYNTH_TCP4, 0x5EED0002)
        rx = tx.clone()
        eng.emit(rx, b)
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        wls[A] = (b, tx, rx, st, int(lens.sum()))
    s = torch.cuda.current_stream(dev)
    for rnd in range(3):
        for A in aligns:
            b, tx, rx, st, nbytes = wls[A]
            for var in variants:
                eng.set_variant(var)
                eng.set_shape(8 if var == 13 else -1)
                for _ in range(2):
                    eng.emit(tx, b, stream=s)
                    eng.verify(rx, b, status=st, stream=s)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record(s)
                for _ in range(10):
                    eng.emit(tx, b, stream=s)
                ev[1].record(s)
                for _ in range(10):
                    eng.verify(rx, b, status=st, stream=s)
                ev[2].record(s)
                torch.cuda.synchronize()
                em, vm = ev[0].elapsed_time(ev[1]) / 10, ev[1].elapsed_time(ev[2]) / 10
                print(json.dumps({"round": rnd, "align": A, "var": var, "emit_ms": round(em, 4),
                                  "verify_ms": round(vm, 4), "tax_ms": round(em - vm, 4),
                                  "accept": int(((st & E.ST_ACCEPT) != 0).sum())}), flush=True)
    eng.set_variant(-1)
    eng.set_shape(-1)


if __name__ == "__main__":
    main()
