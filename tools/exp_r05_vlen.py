#!/usr/bin/env python3
"""Experiment (round 5): fixed-stride verify and emit, the walk kernel (default) against the
transposed walk (variants 44 / 47) over record lengths, ~1.5 GB per batch, R = 4 batches in turn
(synthetic IPv4/UDP, every 64th record corrupted; emit timed after verify on the same batches).
Needs the experiments build (SMOLCSUM_LIB=.../libsmolcsum_exp.so).
GAP=g: stride = length + g (default 0, packed).
STEP=1: emit timed as in bench.py's step instead: emit of TX batch i mod R (its own buffers, HIP
events around each emit), then the default verify of RX batch i mod R.
PROFILE=v6mix: the IPv6 TCP / UDP / ICMPv6 mix (C4's) instead of IPv4/UDP.
Usage: [LENS=1024,1320,1500] [VVARS=-1,44] [EVARS=-1,44,47] [GAP=0] [K=24] exp_r05_vlen.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from smoltcp_amd import engine as E  # noqa: E402


def main():
    eng = E.ChecksumEngine(0)
    R, K = 4, int(os.environ.get("K", "24"))
    lens = [int(x) for x in os.environ.get("LENS", "1024,1320,1500,1760,1921,2500,3969,5000,8065,9000,12000,16257").split(",")]
    vv = [int(x) for x in os.environ.get("VVARS", "-1,44").split(",")]
    ev = [int(x) for x in os.environ.get("EVARS", "-1,44,47").split(",") if x]
    for L in lens:
        S = L + int(os.environ.get("GAP", "0"))
        n = (1536 << 20) // S
        batch = E.Batch.fixed(n, S, L, E.KIND_IP)
        rxs = []
        for j in range(R):
            b = torch.empty(n * S + 64, dtype=torch.uint8, device="cuda:0")
            prof = E.SYNTH_V6MIX if os.environ.get("PROFILE") == "v6mix" else E.SYNTH_UDP4
            eng.synth(b, batch, prof, seed=L + j)
            eng.emit(b, batch)
            eng.corrupt(b, batch, every=64, seed=j)
            rxs.append(b)
        st = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        ref = None
        for v in vv:  # identical statuses
            eng.set_variant(v)
            s = eng.verify(rxs[0], batch, status=st).clone()
            ref = s if ref is None else ref
            assert torch.equal(ref, s), (L, v)
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

        txs = [b.clone() for b in rxs] if os.environ.get("STEP") else None

        def step_emit(v):
            ev_ = []
            for i in range(K + R):
                j = i % R
                eng.set_variant(v)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                eng.emit(txs[j], batch)
                b.record()
                eng.set_variant(-1)
                eng.verify(rxs[j], batch, status=st)
                if i >= R:
                    ev_.append((a, b))
            torch.cuda.synchronize()
            return sum(a.elapsed_time(b) for a, b in ev_) / len(ev_)

        res = {}
        for rnd in range(3):
            if txs is not None:
                for v in ev:
                    res.setdefault(f"step_emit{v}", []).append(step_emit(v))
                continue
            for v in vv:
                eng.set_variant(v)
                res.setdefault(f"verify{v}", []).append(timed(lambda j: eng.verify(rxs[j], batch, status=st)))
            for v in ev:
                eng.set_variant(v)
                res.setdefault(f"emit{v}", []).append(timed(lambda j: eng.emit(rxs[j], batch)))
        eng.set_variant(-1)
        print(json.dumps({"len": L, "stride": S, "n": n, **{k: round(min(t), 4) for k, t in res.items()},
                          **{f"TBps_{k}": round(n * L / min(t) / 1e9, 2) for k, t in res.items()}}), flush=True)
        del rxs


if __name__ == "__main__":
    main()
