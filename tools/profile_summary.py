#!/usr/bin/env python3
"""Summarise rocprofv3 output of `bench.py` runs into the files committed under profiles/.

    python tools/profile_summary.py --config c2 --kt DIR --fetch DIR --write DIR --out profiles/r01

Reads the kernel-trace stats CSV (`--kernel-trace --stats`) and the counter-collection CSVs of two
separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes, and writes
  <out>_kernel_stats_<cfg>.csv    (the stats CSV as rocprofv3 wrote it)
  <out>_pmc_{fetch,write}_<cfg>.csv
  <out>_traffic.json              (merged per config: HBM bytes per launch of emit / verify)

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes x1024): FETCH_SIZE is doubled per
/opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section: on gfx950 it counts half of a
streaming read of 16 B per lane).  Means over every dispatch of the kernel in the run.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import shutil

MODES = {"0": "data", "1": "emit", "2": "verify", "3": "copy_emit"}


def _find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    if not hits:
        raise SystemExit(f"no {pattern} under {d}")
    return hits[0]


def kernel_role(name: str):
    """'emit' / 'verify' / 'data' for the checksum kernels, else None."""
    if re.search(r"copy_kernel<", name):  # csum_copy.hip: <G, U, IMPLICIT>, copy-emit only
        return "copy_emit"
    if re.search(r"seg_pass\d*_kernel", name):  # csum_dwalk.hip: the staged emit's second launch
        return "emit_seg_pass"
    m = re.search(r"[xd]walk_kernel<([^>]*)>", name)  # csum_xwalk.hip <MODE, R, ...>, csum_dwalk.hip <MODE, ...>
    if m:
        return MODES.get(m.group(1).split(",")[0].strip())
    m = re.search(r"(csum_kernel|csum_tile_kernel)<([^>]*)>", name)
    if not m:
        return None
    args = [a.strip() for a in m.group(2).split(",")]
    return MODES.get(args[2])  # <G, U, MODE, IMPLICIT, VAR[, TILE]>


def pmc_means(path: str, counter: str):
    acc = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            role = kernel_role(row["Kernel_Name"])
            if role is None:
                continue
            e = acc.setdefault(role, {"kernel": row["Kernel_Name"], "vals": []})
            e["vals"].append(float(row["Counter_Value"]))
    return {k: (v["kernel"], sum(v["vals"]) / len(v["vals"]), len(v["vals"])) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--kt", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True, help="path prefix, e.g. profiles/r01")
    a = ap.parse_args()

    stats = _find(a.kt, "*kernel_stats.csv")
    fetch = _find(a.fetch, "*counter_collection.csv")
    write = _find(a.write, "*counter_collection.csv")
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    shutil.copy(stats, f"{a.out}_kernel_stats_{a.config}.csv")
    shutil.copy(fetch, f"{a.out}_pmc_fetch_{a.config}.csv")
    shutil.copy(write, f"{a.out}_pmc_write_{a.config}.csv")

    avg_ns = {}
    with open(stats) as f:
        for row in csv.DictReader(f):
            role = kernel_role(row["Name"])
            if role:
                avg_ns[role] = (row["Name"], float(row["AverageNs"]), int(row["Calls"]))

    fm, wm = pmc_means(fetch, "FETCH_SIZE"), pmc_means(write, "WRITE_SIZE")
    path = f"{a.out}_traffic.json"
    doc = {}
    if os.path.exists(path):
        with open(path) as f:
            doc = json.load(f)
    cfg = {}
    for role in sorted(set(fm) & set(wm)):
        rd = 2 * fm[role][1] * 1024
        wr = wm[role][1] * 1024
        cfg[role] = {"kernel": fm[role][0], "hbm_bytes_per_launch": int(rd + wr),
                     "read_bytes_corrected": int(rd), "write_bytes": int(wr),
                     "FETCH_SIZE_KB_mean": fm[role][1], "FETCH_SIZE_dispatches": fm[role][2],
                     "WRITE_SIZE_KB_mean": wm[role][1], "WRITE_SIZE_dispatches": wm[role][2]}
        if role in avg_ns:
            cfg[role]["kernel_trace_avg_ns"] = avg_ns[role][1]
            cfg[role]["kernel_trace_calls"] = avg_ns[role][2]
    if "emit" in cfg and "emit_seg_pass" in cfg:
        # staged emit (round 6): one emit call = the staging launch + the segment pass; "emit" is their
        # sum (what bench.py's HIP events around the call time), the parts stay beside it
        st, sp = cfg["emit"], cfg["emit_seg_pass"]
        cfg["emit_staging"] = st
        cfg["emit"] = {"kernel": st["kernel"] + " + " + sp["kernel"],
                       **{k: st[k] + sp[k] for k in ("hbm_bytes_per_launch", "read_bytes_corrected", "write_bytes")}}
        if "kernel_trace_avg_ns" in st and "kernel_trace_avg_ns" in sp:
            cfg["emit"]["kernel_trace_avg_ns"] = st["kernel_trace_avg_ns"] + sp["kernel_trace_avg_ns"]
    doc[a.config] = cfg
    doc["method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     "`python3 bench.py --config <cfg> --steps 5 --warmup 1 --ramp-ms 0 --cpu-seconds 0`; counters in KB "
                     "(x1024); FETCH_SIZE doubled per MI355X_MICROARCH.md (HBM / rocprofv3: gfx950 counts half "
                     "of a 16-B/lane streaming read); mean over dispatches. kernel_trace_avg_ns from "
                     "`rocprofv3 --kernel-trace --stats` of `bench.py --config <cfg> --steps 20 --warmup 5` (clock ramp included).")
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps({a.config: cfg}, indent=1))


if __name__ == "__main__":
    main()
