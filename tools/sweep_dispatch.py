#!/usr/bin/env python3
"""Round 6: the measured length sweep behind the fixed-stride dispatch table (csum_api.cpp
xwalk_table).

For record lengths L = 1024 + 64 k (k = 0 .. 124: "aligned", a multiple of 64) and L = 1024 + 64 k + 28
("unaligned": C2's 1500 B is k = 7), packed (stride = L), and for the unaligned lengths also with
64-B gaps (stride = L + 64), synthetic IPv4/UDP records in ~1.5-GB batches, R = 4 TX / RX batch pairs
in turn (every 64th RX record corrupted):
  verify   the walk kernel (variant 5), the transposed walk (47) and the transposed walk with the
           first-load hint (89), timed over the RX batches in turn;
  emit     in bench.py's step order (emit of TX batch i, then the library's default verify of RX batch
           i, HIP events around each emit, after 3R untimed steps of the same variant): the walk kernel
           (39), the transposed walk with whole segments (47) and with non-temporal segments (57).
Every variant's verify statuses and emitted bytes are checked equal to the walk kernel's (a checksum
of the buffer), so a faster kernel that computes something else fails the sweep.
One JSON line per (length, stride): the best of ROUNDS passes per kernel, in ms.
PROFILE=v6mix: C4's IPv6 TCP / UDP / ICMPv6 mix instead of IPv4/UDP (one field per record).
Late round 6: VERIFY / EMIT (comma lists) replace the variant sets, e.g. EMIT=39,47,57,101 VERIFY=5 for
the emit table with the write-through segment form (101).
Usage: [KS=0-124] [ROUNDS=3] [K=12] [FORMS=aligned,unaligned,gapped] [PROFILE=udp4|v6mix] [VERIFY=..] [EMIT=..]
       SMOLCSUM_LIB=.../libsmolcsum_exp.so python tools/sweep_dispatch.py > profiles/r06_dispatch_sweep_<box>.jsonl"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from smoltcp_amd import engine as E  # noqa: E402

VERIFY = tuple(int(v) for v in os.environ.get("VERIFY", "5,47,89").split(","))
EMIT = tuple(int(v) for v in os.environ.get("EMIT", "39,47,57").split(","))


def ks():
    spec = os.environ.get("KS", "0-124")
    out = []
    for part in spec.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def main():
    eng = E.ChecksumEngine(0)
    R, K, rounds = 4, int(os.environ.get("K", "12")), int(os.environ.get("ROUNDS", "3"))
    forms = os.environ.get("FORMS", "aligned,unaligned,gapped").split(",")
    cases = []
    for k in ks():
        if "aligned" in forms:
            cases.append((1024 + 64 * k, 0))
        if "unaligned" in forms:
            cases.append((1024 + 64 * k + 28, 0))
        if "gapped" in forms:
            cases.append((1024 + 64 * k + 28, 64))
    st = None
    t_start = time.time()
    pname = os.environ.get("PROFILE", "udp4")
    prof = {"udp4": E.SYNTH_UDP4, "v6mix": E.SYNTH_V6MIX}[pname]
    for L, gap in cases:
        S = L + gap
        n = (1536 << 20) // S
        batch = E.Batch.fixed(n, S, L, E.KIND_IP)
        rxs, txs = [], []
        for j in range(R):
            b = torch.empty(n * S + 64, dtype=torch.uint8, device="cuda:0")
            eng.synth(b, batch, prof, seed=L * 7 + j)
            txs.append(b.clone())
            eng.emit(b, batch)
            eng.corrupt(b, batch, every=64, seed=j)
            rxs.append(b)
        st = torch.empty(n, dtype=torch.uint8, device="cuda:0")

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

        def step_emit(v):
            # 3R untimed steps first: the previous variant's dirty field segments (its store policy)
            # must have left the Infinity Cache before this variant's steady state is timed
            evs = []
            for i in range(K + 3 * R):
                j = i % R
                eng.set_variant(v)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                eng.emit(txs[j], batch)
                b.record()
                eng.set_variant(-1)
                eng.verify(rxs[j], batch, status=st)
                if i >= 3 * R:
                    evs.append((a, b))
            torch.cuda.synchronize()
            return sum(a.elapsed_time(b) for a, b in evs) / len(evs)

        # correctness: every variant's verify statuses and emitted bytes equal the walk kernel's
        ref_st, ref_tx = None, None
        for v in VERIFY:
            eng.set_variant(v)
            s = eng.verify(rxs[0], batch, status=st).clone()
            ref_st = s if ref_st is None else ref_st
            assert torch.equal(ref_st, s), (L, S, "verify", v)
        for v in EMIT:
            eng.set_variant(v)
            t = txs[0].clone()
            eng.emit(t, batch)
            h = int(t[: t.numel() // 8 * 8].view(torch.int64).sum().item())
            ref_tx = h if ref_tx is None else ref_tx
            assert h == ref_tx, (L, S, "emit", v)
            del t
        eng.set_variant(-1)
        res = {}
        for _ in range(rounds):
            for v in VERIFY:
                eng.set_variant(v)
                res.setdefault(f"verify{v}", []).append(timed(lambda j: eng.verify(rxs[j], batch, status=st)))
            for v in EMIT:
                res.setdefault(f"emit{v}", []).append(step_emit(v))
        eng.set_variant(-1)
        line = {"len": L, "stride": S, "n": n, "profile": pname, **{k: round(min(t), 4) for k, t in res.items()}}
        line["fastest_verify"] = min(VERIFY, key=lambda v: line[f"verify{v}"])
        line["fastest_emit"] = min(EMIT, key=lambda v: line[f"emit{v}"])
        line["elapsed_s"] = round(time.time() - t_start, 1)
        print(json.dumps(line), flush=True)
        del rxs, txs


if __name__ == "__main__":
    main()
