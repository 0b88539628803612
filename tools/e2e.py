#!/usr/bin/env python3
"""End-to-end (host memory -> HBM -> checksum -> host memory) rate of the C2 workload.

The reference path starts and ends in host memory (the phy device buffer / loopback ring), so
BASELINE.json asks for the rate including pinned hipMemcpyAsync both ways.  Pipeline per chunk,
three HIP streams, `--buffers` device chunks in rotation (default 2: double-buffered):

    TX:  H2D(frames) -> smol_csum_batch_emit -> D2H(frames with checksums)
    RX:  H2D(frames) -> smol_csum_batch_verify -> D2H(status bytes)

Reported: record bytes per second through the whole pipeline, next to the bare PCIe copy rates
measured in the same process.

    python tools/e2e.py [--records N] [--chunk M] [--buffers B]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n_records: int = 1 << 20, chunk: int = 1 << 17, L: int = 1500, reps: int = 3, device: int = 0, nbuf: int = 2):
    import torch

    from smoltcp_amd import engine as E

    dev = torch.device("cuda", device)
    eng = E.ChecksumEngine(device)
    nchunks = (n_records + chunk - 1) // chunk
    # host frames: generated on the device once, copied to pinned host memory
    host_in = torch.empty(n_records * L, dtype=torch.uint8, pin_memory=True)
    host_out = torch.empty(n_records * L, dtype=torch.uint8, pin_memory=True)
    host_st = torch.empty(n_records, dtype=torch.uint8, pin_memory=True)
    tmp = torch.empty(chunk * L, dtype=torch.uint8, device=dev)
    for c in range(nchunks):
        m = min(chunk, n_records - c * chunk)
        b = E.Batch.fixed(m, L, L, E.KIND_IP)
        eng.synth(tmp, b, E.SYNTH_UDP4, seed=0x5EED0001 + c)
        host_in[c * chunk * L:(c * chunk + m) * L].copy_(tmp[:m * L])
    torch.cuda.synchronize()
    dbuf = [torch.empty(chunk * L, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    dst = [torch.empty(chunk, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    s_h2d, s_cmp, s_d2h = (torch.cuda.Stream(dev) for _ in range(3))

    def pipeline(mode: str):
        e_h2d = [torch.cuda.Event() for _ in range(nchunks)]
        e_cmp = [torch.cuda.Event() for _ in range(nchunks)]
        e_d2h = [torch.cuda.Event() for _ in range(nchunks)]
        for c in range(nchunks):
            m = min(chunk, n_records - c * chunk)
            k = c % nbuf
            lo, hi = c * chunk * L, (c * chunk + m) * L
            with torch.cuda.stream(s_h2d):
                if c >= nbuf:
                    s_h2d.wait_event(e_d2h[c - nbuf])  # the device chunk is free again
                dbuf[k][:m * L].copy_(host_in[lo:hi], non_blocking=True)
                e_h2d[c].record(s_h2d)
            with torch.cuda.stream(s_cmp):
                s_cmp.wait_event(e_h2d[c])
                b = E.Batch.fixed(m, L, L, E.KIND_IP)
                if mode == "tx":
                    eng.emit(dbuf[k], b, stream=s_cmp)
                else:
                    eng.verify(dbuf[k], b, status=dst[k], stream=s_cmp)
                e_cmp[c].record(s_cmp)
            with torch.cuda.stream(s_d2h):
                s_d2h.wait_event(e_cmp[c])
                if mode == "tx":
                    host_out[lo:hi].copy_(dbuf[k][:m * L], non_blocking=True)
                else:
                    host_st[c * chunk:c * chunk + m].copy_(dst[k][:m], non_blocking=True)
                e_d2h[c].record(s_d2h)
        torch.cuda.synchronize()

    def timed(fn):
        fn()  # warm-up
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return (time.perf_counter() - t0) / reps

    total = n_records * L
    res = {"records": n_records, "record_bytes": L, "chunk_records": chunk, "device_buffers": nbuf}
    # bare copy rates over the same bytes
    def h2d():
        for c in range(nchunks):
            m = min(chunk, n_records - c * chunk)
            dbuf[c % nbuf][:m * L].copy_(host_in[c * chunk * L:(c * chunk + m) * L], non_blocking=True)
        torch.cuda.synchronize()

    def d2h():
        for c in range(nchunks):
            m = min(chunk, n_records - c * chunk)
            host_out[c * chunk * L:(c * chunk + m) * L].copy_(dbuf[c % nbuf][:m * L], non_blocking=True)
        torch.cuda.synchronize()

    def duplex():  # H2D and D2H of the same bytes at once, on two streams (what TX needs)
        for c in range(nchunks):
            m = min(chunk, n_records - c * chunk)
            with torch.cuda.stream(s_h2d):
                dbuf[c % nbuf][:m * L].copy_(host_in[c * chunk * L:(c * chunk + m) * L], non_blocking=True)
            with torch.cuda.stream(s_d2h):
                host_out[c * chunk * L:(c * chunk + m) * L].copy_(dbuf[(c + 1) % nbuf][:m * L], non_blocking=True)
        torch.cuda.synchronize()

    res["h2d_GBs"] = round(total / timed(h2d) / 1e9, 2)
    res["d2h_GBs"] = round(total / timed(d2h) / 1e9, 2)
    res["duplex_each_way_GBs"] = round(total / timed(duplex) / 1e9, 2)
    t_tx = timed(lambda: pipeline("tx"))
    t_rx = timed(lambda: pipeline("rx"))
    res["tx_emit_e2e_GBs"] = round(total / t_tx / 1e9, 2)
    res["rx_verify_e2e_GBs"] = round(total / t_rx / 1e9, 2)
    res["tx_emit_e2e_GiBs"] = round(total / t_tx / 2**30, 2)
    res["rx_verify_e2e_GiBs"] = round(total / t_rx / 2**30, 2)
    # the RX input still carries the zero checksum fields of synthesis: the UDP gate accepts a
    # zero field but an IPv4 header with a zero checksum fails unless its other words happen to
    # sum to 0xffff (about 1 in 65535 headers), so only a handful of records may be accepted
    res["rx_accepted"] = int(((host_st & E.ST_ACCEPT) != 0).sum())
    # the TX output is the emitted batch: verifying it on the device must accept every record
    chk = torch.empty(chunk * L, dtype=torch.uint8, device=dev)
    acc = 0
    for c in range(nchunks):
        m = min(chunk, n_records - c * chunk)
        chk[:m * L].copy_(host_out[c * chunk * L:(c * chunk + m) * L])
        st = eng.verify(chk, E.Batch.fixed(m, L, L, E.KIND_IP))
        acc += int(((st & E.ST_ACCEPT) != 0).sum())
    res["tx_output_accepted"] = acc
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--chunk", type=int, default=1 << 17)
    ap.add_argument("--buffers", type=int, default=2)
    args = ap.parse_args()
    print(json.dumps(run(args.records, args.chunk, nbuf=args.buffers)))


if __name__ == "__main__":
    main()
