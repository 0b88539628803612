#!/usr/bin/env python3
"""A/B: fixed-stride emit with whole-line field writes on / off (C2 and C4 geometry)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smoltcp_amd import engine as E  # noqa: E402


def main():
    eng = E.ChecksumEngine(0)
    dev = torch.device("cuda:0")
    for name, L, prof in [("c2", 1500, E.SYNTH_UDP4), ("c4", 1320, E.SYNTH_V6MIX), ("eth1514", 1514, E.SYNTH_ETH_TCP4)]:
        n = 1 << 20
        buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
        b = E.Batch.fixed(n, L, L, E.KIND_ETH if prof == E.SYNTH_ETH_TCP4 else E.KIND_IP)
        eng.synth(buf, b, prof, 0x5EED0001)
        for rnd in range(2):
            for lw in (False, True):
                eng.set_line_writes(lw)
                for _ in range(3):
                    eng.emit(buf, b)
                a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(30):
                    eng.emit(buf, b)
                z.record()
                torch.cuda.synchronize()
                if rnd:
                    print(json.dumps({"cfg": name, "line_writes": lw, "emit_ms": round(a.elapsed_time(z) / 30, 4)}), flush=True)


if __name__ == "__main__":
    main()
