#!/usr/bin/env python3
"""Experiment: is emit's tax the field stores themselves (DRAM partial-line writes) or their place
inside the read stream?  Per config (C2 / C3 / C4 of bench.py), interleaved rounds on one box:
  emit      the library's emit of tx
  verify    the library's verify of tx (status out: same reads, no field stores)
  scatter   the field values written at their offsets by torch index_put (two byte scatters;
            an upper bound on a separate store pass: it also reads 8-B indices)
  v+s       verify then scatter, back to back (a deferred-store emit's cost)
  seg64 / v+seg64, seg128 / v+seg128: the same with the whole aligned 64-B / 128-B blocks holding
            the fields written (torch row index_put of their own bytes) instead of the 2-B fields
  v+sc / v+sc_nt: verify then the library's scatter kernel (smol_csum_tool_field_scatter), plain /
            non-temporal stores (what a two-pass emit would cost; round 4 also timed emit without its
            field stores, an experiment tile variant since removed:
            profiles/r04_experiments/c3_write_cost.jsonl "e34")
Usage: exp_scatter.py [c3,c2,c4]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from smoltcp_amd import engine as E  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    z.record()
    torch.cuda.synchronize()
    return a.elapsed_time(z) / reps


def main():
    cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["c3", "c2", "c4"]
    eng = E.ChecksumEngine(0)
    dev = torch.device("cuda", 0)
    for cfg in cfgs:
        wl = bench.Workload(E, eng, cfg, 0, 0, dev)
        eng.emit(wl.tx, wl.batch)
        addrs = bench.field_addrs(wl)
        hi, lo = wl.tx[addrs].clone(), wl.tx[addrs + 1].clone()
        a1 = addrs + 1
        v16 = ((hi.to(torch.int32) << 8) | lo.to(torch.int32))
        v16 = (((v16 + 32768) % 65536) - 32768).to(torch.int16)
        st = torch.empty(wl.n, dtype=torch.uint8, device=dev)
        blk = {}
        for w in (64, 128):
            rows = torch.unique(torch.cat([addrs // w, (addrs + 1) // w]))
            rows = rows[(rows + 1) * w <= wl.tx.numel()]
            view = wl.tx[: wl.tx.numel() // w * w].view(-1, w)
            blk[w] = (view, rows, view[rows].clone())

        def emit():
            eng.emit(wl.tx, wl.batch)

        def verify():
            eng.verify(wl.tx, wl.batch, status=st)

        def scatter():
            wl.tx[addrs] = hi
            wl.tx[a1] = lo

        def vs():
            verify()
            scatter()

        def sc(nt):
            eng.field_scatter(wl.tx, addrs, v16, nt=nt)

        def seg(w):
            view, rows, data = blk[w]
            view[rows] = data

        torch.cuda.synchronize()
        for rnd in range(int(os.environ.get("ROUNDS", "3"))):
            out = {"cfg": cfg, "round": rnd, "fields": int(addrs.numel()),
                   "seg64": int(blk[64][1].numel()), "seg128": int(blk[128][1].numel())}
            for name, fn in (("emit", emit), ("verify", verify), ("scatter", scatter), ("v+s", vs),
                             ("seg64", lambda: seg(64)), ("v+seg64", lambda: (verify(), seg(64))),
                             ("seg128", lambda: seg(128)), ("v+seg128", lambda: (verify(), seg(128))),
                             ("sc", lambda: sc(False)), ("v+sc", lambda: (verify(), sc(False))),
                             ("v+sc_nt", lambda: (verify(), sc(True)))):
                out[f"{name}_ms"] = round(timed(fn), 4)
            print(json.dumps(out), flush=True)
        del wl
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
