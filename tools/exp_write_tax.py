#!/usr/bin/env python3
"""Experiment (round 5): what one scattered field write costs HBM, against the spacing of the written
lines and the order they are written in.

For each spacing S (256 B .. 8 KB) the same 2^21 writes (2-B fields at byte 10 of each S-byte slot,
or the whole 64-B segment holding that byte) go into one of R = 4 regions of 2^21 * S bytes, in
address order, shuffled within windows of 8192 writes (about what the tile kernel's resident
workgroups have in flight), or fully shuffled.  Passes take the regions in turn, so that a pass
never rewrites lines the Infinity Cache still holds dirty from the previous one (as a TX path
that fills new frames), and the steady state includes the DRAM write-back of earlier passes.
Timed, interleaved on one box:
  alone     K write passes back to back, per pass;
  in_read   K (write pass + a read-only stream over a 4.7-GB buffer) minus K read streams, per pass:
            what the writes cost when their write-back lands inside a read stream (emit).
FORMS: field2 (2-B fields), seg32 / seg64 / seg128 (the aligned 32-B sector / 64-B segment / 128-B
line holding the field, written whole).
Usage: [SPACINGS=256,512,...] [FORMS=field2,seg64] [ORDERS=address,window8k,random] [N=2097152] [ROUNDS=3]
       exp_write_tax.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from smoltcp_amd import engine as E  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    eng = E.ChecksumEngine(0)
    N = int(os.environ.get("N", str(1 << 21)))
    spacings = [int(x) for x in os.environ.get("SPACINGS", "256,512,1024,1536,2048,4608,8192").split(",")]
    rounds = int(os.environ.get("ROUNDS", "3"))
    R = 4
    buf = torch.zeros(R * N * max(spacings) + 64, dtype=torch.uint8, device=dev)
    rd = torch.zeros(4_700_000_000 // 16 * 16, dtype=torch.uint8, device=dev)  # the read stream (C3's size)
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    vals = torch.full((N,), 0x1234, dtype=torch.int16, device=dev)
    g = torch.Generator(device="cpu").manual_seed(5)
    W = 8192
    K = 16

    def orders(S):
        a = torch.arange(N, dtype=torch.int64) * S + 10
        win = a.view(-1, W)
        perm = torch.argsort(torch.rand(win.shape, generator=g), dim=1)
        for name, x in (("address", a), ("window8k", torch.gather(win, 1, perm).reshape(-1)),
                        ("random", a[torch.randperm(N, generator=g)])):
            yield name, [(x + k * N * S).to(dev) for k in range(R)]

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def timed(fn):
        for k in range(R):
            fn(k)
        a, b = ev(), ev()
        a.record()
        for k in range(K):
            fn(k % R)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / K

    def t_alone(addrs, flags):
        return timed(lambda k: eng.field_scatter(buf, addrs[k], vals, nt=flags))

    def t_read(addrs, flags):
        r0 = min(timed(lambda k: eng.stream_read(rd, sink)) for _ in range(2))
        r1 = min(timed(lambda k: (eng.field_scatter(buf, addrs[k], vals, nt=flags), eng.stream_read(rd, sink)))
                 for _ in range(2))
        return r0, r1

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        eng.stream_read(rd, sink)
        torch.cuda.synchronize()
    for rnd in range(rounds):
        for S in spacings:
            for oname, addrs in orders(S):
                if oname not in os.environ.get("ORDERS", "address,window8k,random").split(","):
                    continue
                forms = {"field2": 0, "seg32": 4, "seg64": 2, "seg128": 8}
                for form in os.environ.get("FORMS", "field2,seg64").split(","):
                    flags = forms[form]
                    alone = t_alone(addrs, flags)
                    r0, r1 = t_read(addrs, flags)
                    print(json.dumps({"round": rnd, "spacing": S, "order": oname, "form": form, "writes": N,
                                      "alone_ms": round(alone, 4), "read_ms": round(r0, 4),
                                      "read_plus_writes_ms": round(r1, 4), "in_read_ms": round(r1 - r0, 4),
                                      "ns_per_write_in_read": round((r1 - r0) * 1e6 / N, 4)}), flush=True)


if __name__ == "__main__":
    main()
