#!/usr/bin/env python3
"""Per-step timeline of a `bench.py` run from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 bench.py --steps K --warmup W --cpu-seconds 0
    python tools/step_trace.py DIR --steps K --warmup W [--out profiles/r03_step_trace_c2.json]

bench.py launches, after the workload set-up, the clock-ramp steps, W warm-up steps, the K timed
steps and K more steps with HIP events (the kernel-duration pass), each step = one emit (or
copy-emit) + one verify; then the probes (stream_read_kernel first) and one more emit.  The last 4K
checksum launches before the first probe kernel are therefore the timed and the event pass, and
the 2W before them the warm-up.  For every step this prints the emit and verify durations and the gaps
(emit start - previous verify end, verify start - emit end), and sums up the timed region: the
kernel sum, the gaps and the span from the first timed kernel's start to the last one's end.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from profile_summary import kernel_role  # noqa: E402


def load(d):
    hits = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    if not hits:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows, probes = [], []
    with open(hits[0]) as f:
        for r in csv.DictReader(f):
            role = kernel_role(r["Kernel_Name"])
            if role in ("emit", "verify", "copy_emit"):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), role))
            elif "stream_read_kernel" in r["Kernel_Name"]:
                probes.append(int(r["Start_Timestamp"]))
    rows.sort()
    if probes:  # drop what bench.py runs after the event pass (the probes and the re-emit)
        rows = [x for x in rows if x[0] < min(probes)]
    return rows


def steps_of(rows, first, count):
    out = []
    for s in range(count):
        e, v = rows[first + 2 * s], rows[first + 2 * s + 1]
        out.append({"emit_us": (e[1] - e[0]) / 1e3, "verify_us": (v[1] - v[0]) / 1e3,
                    "gap_ev_us": (v[0] - e[1]) / 1e3,
                    "start": e[0], "end": v[1]})
    for i in range(1, len(out)):
        out[i]["gap_ve_us"] = (out[i]["start"] - out[i - 1]["end"]) / 1e3
    if out:
        out[0]["gap_ve_us"] = None
    return out


def summarize(st):
    k = sum(s["emit_us"] + s["verify_us"] for s in st)
    span = (st[-1]["end"] - st[0]["start"]) / 1e3
    gaps = sum(s["gap_ev_us"] for s in st) + sum(s["gap_ve_us"] or 0 for s in st)
    return {"steps": len(st), "span_us": round(span, 2), "kernel_sum_us": round(k, 2),
            "gap_sum_us": round(gaps, 2), "span_per_step_us": round(span / len(st), 2),
            "kernel_per_step_us": round(k / len(st), 2),
            "emit_mean_us": round(sum(s["emit_us"] for s in st) / len(st), 2),
            "verify_mean_us": round(sum(s["verify_us"] for s in st) / len(st), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = load(a.dir)
    K, W = a.steps, a.warmup
    need = 2 * (W + 2 * K)
    if len(rows) < need:
        raise SystemExit(f"{len(rows)} checksum launches in the trace, need >= {need}")
    base = len(rows) - need
    warm = steps_of(rows, base, W)
    timed = steps_of(rows, base + 2 * W, K)
    evpass = steps_of(rows, base + 2 * W + 2 * K, K)
    res = {"warmup": summarize(warm) if W else None, "timed": summarize(timed), "event_pass": summarize(evpass),
           "timed_steps": [{k: (round(v, 2) if isinstance(v, float) else v) for k, v in s.items()
                            if k not in ("start", "end")} for s in timed],
           "setup_to_first_timed_us": round((timed[0]["start"] - (warm[-1]["end"] if warm else rows[0][1])) / 1e3, 2)}
    for name in ("warmup", "timed", "event_pass"):
        print(name, json.dumps(res[name]))
    for i, s in enumerate(res["timed_steps"]):
        print(f"  step {i:3d} emit {s['emit_us']:8.2f} verify {s['verify_us']:8.2f} "
              f"gap(e->v) {s['gap_ev_us']:6.2f} gap(v->e) {s['gap_ve_us'] if s['gap_ve_us'] is not None else '-'}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
