#!/usr/bin/env python3
"""Summary of an exp_r05_emit.py log: per (config, variant) the fresh-batch / same-batch emit times
over the rounds after the first, and the verify reference.  Usage: summ_emit.py LOG"""
import collections
import json
import sys

rows = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")]
agg = collections.defaultdict(list)
for r in rows:
    if r.get("round", 0) > 0:
        k = (r["cfg"], str(r["variant"]))
        agg[k].append((r["ms"],) if str(r["variant"]).startswith("verify") else (r["emit_fresh_ms"], r["emit_same_ms"]))
for (c, v), xs in sorted(agg.items()):
    cols = list(zip(*xs))
    print(c, v.rjust(6), "  ".join("%s %.4f-%.4f" % (n, min(col), max(col)) for n, col in zip(("fresh", "same"), cols)))
for r in rows:
    if "identical_to_first" in r and not r["identical_to_first"]:
        print("DIFFERS", r)
