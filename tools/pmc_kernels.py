#!/usr/bin/env python3
"""Mean of each counter per kernel over a rocprofv3 counter-collection CSV (any --pmc pass).

    python tools/pmc_kernels.py DIR [name-substring]

FETCH_SIZE is also shown doubled (the gfx950 correction of MI355X_MICROARCH.md, HBM / rocprofv3).
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    paths = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))
    if not paths:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if sub in name:
                    acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, cs in acc.items():
        parts = []
        for c, v in sorted(cs.items()):
            m = sum(v) / len(v)
            parts.append(f"{c}={m:.6g} (n={len(v)})" + (f" [x2: {2 * m:.6g}]" if c == "FETCH_SIZE" else ""))
        print(name[:90], "|", "; ".join(parts))


if __name__ == "__main__":
    main()
