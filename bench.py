#!/usr/bin/env python3
"""Benchmark: device-resident batched Internet checksum (emit + verify) on MI355X.

Workload (BASELINE.json configs[1], "C2"): per GPU 2^20 IPv4/UDP datagrams of 1500 bytes in HBM
at a fixed 1500-byte stride.  One step = smol_csum_batch_emit over the TX batch (fill the IPv4
header and UDP checksums) + smol_csum_batch_verify over the RX batch (the same kind of datagrams,
already emitted, with 1/64 of them single-bit corrupted as phy::FaultInjector does).  The steps take
four TX / RX batch pairs in turn (--batches), so that every emit fills a batch whose field lines the
previous pass did not just write, as a TX path does.  Metric: GiB/s
checksummed = bytes covered by checksum::data spans (IPv4 header + UDP length) of both passes ÷
wall time, summed over GPUs (weak scaling: every rank owns its own batch; no collective on the
data path — only barrier + a max-reduction of the elapsed time for reporting).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5|c2copy]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

`--gpus N` without a torch.distributed.run environment starts the N rank processes itself (one per
GPU, before anything in this process touches a GPU); under torch.distributed.run the world size
must equal N.  `--dry-run` runs the same launch, rendezvous and reporting on CPU (gloo) with an
empty step: it checks the multi-rank plumbing, it measures nothing.

Prints ONE JSON line on rank 0 (see the contract in the task description / DESIGN.md §6).
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from smoltcp_amd import shard as S  # noqa: E402

METRIC = "GiB/s checksummed (device-resident), batched 1500B segments, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
GIB = float(1 << 30)
CPU_SAMPLE_BYTES = 1_600_000_000  # per buffer: larger than any host LLC (EPYC L3 <= 1.1 GB)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5", "c2copy"])
    ap.add_argument("--n", type=int, default=0, help="records per GPU (default: the config's)")
    ap.add_argument("--ramp-ms", type=float, default=300.0,
                    help="untimed steps for at least this long before the W warm-up steps, so that the "
                         "GPU's clocks have ramped up (0: none; profiles/r03_steps/)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0,
                    help="CPU-baseline budget, split between 1 thread and all threads (0: skip)")
    ap.add_argument("--shape", type=int, default=-1, help="force a launch shape (tuning)")
    ap.add_argument("--variant", type=int, default=-1, help="force a kernel variant (tuning)")
    ap.add_argument("--emit-variant", type=int, default=-1, help="force a kernel variant for emit only (tuning)")
    ap.add_argument("--verify-variant", type=int, default=-1, help="force a kernel variant for verify only (tuning)")
    ap.add_argument("--xcd-remap", type=int, default=-1, help="1/0: force the XCD-contiguous block order (tuning; "
                                                               "-1: the library's choice)")
    ap.add_argument("--launch-records", type=int, default=-1, help="records per kernel launch (tuning; 0: all)")
    ap.add_argument("--src-stride", type=int, default=1472,
                    help="c2copy: bytes between consecutive payloads in the source buffer (1472: packed; an "
                         "experiment knob: 1536 puts every payload on its own 128-B lines)")
    ap.add_argument("--batches", type=int, default=4,
                    help="TX / RX batch pairs the steps take in turn (1: re-emit one batch; C5 always 1: its one "
                         "201-GB buffer is emitted and verified in place)")
    ap.add_argument("--probe", action="store_true", help="(kept for old scripts: the probes always run)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch + rendezvous + reporting only, on CPU (gloo), no checksum work")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------------------------
# Launcher: --gpus N without torch.distributed.run
# ---------------------------------------------------------------------------------------------


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """Start `args.gpus` copies of this script, one per GPU (RANK = LOCAL_RANK = i), rendezvous on
    127.0.0.1, and wait for them.  Rank 0 prints the JSON line; this process prints nothing.  No
    GPU is initialised here: torch.cuda.device_count() only counts the devices.  If one rank
    fails, the others are stopped (they would wait at a barrier) and its exit code is returned."""
    n = args.gpus
    if not args.dry_run:
        import torch

        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) are visible", file=sys.stderr)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SMOLCSUM_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc, failed_at = 0, None
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad and failed_at is None:
            rc, failed_at = bad[0], time.monotonic()
        if all(c is not None for c in codes):
            break
        if failed_at is not None and time.monotonic() - failed_at > 20:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(0.1)
    return rc


# ---------------------------------------------------------------------------------------------
# Workloads
# ---------------------------------------------------------------------------------------------


class Workload:
    """Two HBM batches (tx, rx) of one config, generated on the device."""

    def __init__(self, E, eng, cfg: str, n: int, rank: int, dev, batches: int = 1, src_stride: int = 1472):
        import torch

        self.cfg = cfg
        self.E = E
        seed = S.rank_seed({"c2": 0x5EED0001, "c3": 0x5EED0002, "c4": 0x5EED0003, "c5": 0x5EED0005,
                            "c2copy": 0x5EED0006}[cfg], rank)
        self.seed = seed
        self.copy = None
        if cfg in ("c2", "c5", "c2copy"):
            self.n = n or (128 << 20 if cfg == "c5" else 1 << 20)
            L = 1500
            self.kind, self.profile = E.KIND_IP, E.SYNTH_UDP4
            self.batch = E.Batch.fixed(self.n, L, L, E.KIND_IP)
            self.total = self.n * L
            self.span_bytes = self.n * 1500  # IPv4 header (20) + UDP length (1480)
            self.read_bytes = self.n * L
            self.desc_bytes = 0
            self.workload = (f"C2: {self.n} x 1500 B IPv4/UDP datagrams, fixed stride, emit (tx) + "
                             f"verify (rx, 1/64 single-bit corrupted)") if cfg == "c2" else \
                (f"C5: {self.n} x 1500 B IPv4/UDP per GPU, in-place emit + verify of one batch") if cfg == "c5" else \
                (f"C2copy: C2 with the TX payloads (1472 B each) copied from a separate socket buffer by the "
                 f"fused copy + emit (UdpRepr::emit), + verify (rx)")
        elif cfg == "c3":
            self.n = n or (1 << 20)
            rng = np.random.default_rng(seed)
            lens = rng.integers(64, 9001, self.n).astype(np.uint32)
            offs = np.zeros(self.n, dtype=np.uint64)
            offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
            self.kind, self.profile = E.KIND_IP, E.SYNTH_TCP4
            self.batch = E.Batch.from_records(offs, lens, E.KIND_IP, dev)
            self.total = int(offs[-1] + lens[-1]) + 16
            self.span_bytes = int(lens.astype(np.uint64).sum())  # header + TCP segment = whole record
            self.read_bytes = self.span_bytes
            self.desc_bytes = 16 * self.n
            self.workload = f"C3: {self.n} IPv4/TCP segments, length U[64,9000], packed (odd offsets) + descriptors"
        else:  # c4
            self.n = n or (1 << 20)
            L = 1320
            self.kind, self.profile = E.KIND_IP, E.SYNTH_V6MIX
            self.batch = E.Batch.fixed(self.n, L, L, E.KIND_IP)
            self.total = self.n * L
            self.span_bytes = self.n * 1280  # L4 only (IPv6 has no header checksum)
            self.read_bytes = self.n * L
            self.desc_bytes = 0
            self.workload = f"C4: {self.n} IPv6 packets (40 B header + 1280 B TCP/UDP/ICMPv6 round-robin)"
        self.tx = torch.empty(self.total, dtype=torch.uint8, device=dev)
        eng.synth(self.tx, self.batch, self.profile, seed)
        if cfg == "c2copy":
            # payloads live in a socket-buffer-like source, back to back; headers are in the records
            self.src = torch.randint(0, 256, (self.n * src_stride + 16,), dtype=torch.uint8, device=dev)
            cp = E.make_copies(np.arange(self.n, dtype=np.uint64) * src_stride, 28, 1472)
            self.copy = torch.from_numpy(cp.view(np.uint8).copy()).to(dev)
            self.read_bytes = self.n * (28 + 1472)   # headers from the record, payload from the source
            self.write_bytes_tx = self.n * (1472 + 4)
        if cfg == "c5":
            self.rx = self.tx
        else:
            self.rx = torch.empty(self.total, dtype=torch.uint8, device=dev)
            eng.synth(self.rx, self.batch, self.profile, seed ^ 0xABCDEF)
            eng.emit(self.rx, self.batch)
            eng.corrupt(self.rx, self.batch, every=64, seed=seed)
        self.status = torch.empty(self.n, dtype=torch.uint8, device=dev)
        self.est = None
        # Batch pairs the steps take in turn.  A TX path fills new frames every time (udp.rs:300-308,
        # tcp.rs:1087-1095): re-emitting one batch lets the ~80 MB of field segments a C2 pass writes
        # sit dirty in the 256-MB Infinity Cache, where the next pass rewrites them without a DRAM
        # write (emit 4-9 % faster).  With R pairs, each step emits a batch R steps old.
        self.txs, self.rxs = [self.tx], [self.rx]
        if cfg != "c5":
            for _ in range(max(1, batches) - 1):
                self.txs.append(self.tx.clone())
                self.rxs.append(self.rx.clone())
        # emit's floor probe on fixed-stride IPv4 batches: (record stride, field offsets) — the IPv4
        # header checksum and the UDP checksum; C3 / C4 list their fields from the headers (field_addrs)
        self.probe_fields = (1500, 10, 26)


def field_addrs(wl):
    """Ascending byte offsets (int64, on the device) of the checksum fields emit fills in wl.tx: the
    IPv4 header checksum and the L4 checksum of each record (KIND_IP records without extension
    headers, as the synthetic profiles make them).  For emit's floor probe."""
    import torch

    b = wl.tx
    if wl.batch.desc is None:
        offs = torch.arange(wl.n, device=b.device, dtype=torch.int64) * wl.batch.stride
    else:
        offs = wl.batch.desc.view(torch.int64).view(wl.n, 2)[:, 0].clone()
    b0 = b[offs].to(torch.int64)
    v4 = (b0 >> 4) == 4
    ihl = (b0 & 15) * 4
    proto = torch.where(v4, b[offs + 9].to(torch.int64), b[offs + 6].to(torch.int64))
    l4 = torch.where(v4, offs + ihl, offs + 40)
    fo = torch.full_like(offs, -1)
    fo = torch.where(proto == 17, 6, fo)
    fo = torch.where(proto == 6, 16, fo)
    fo = torch.where((proto == 1) | (proto == 58), 2, fo)
    ip = offs[v4] + 10
    l4f = (l4 + fo)[fo >= 0]
    a, _ = torch.sort(torch.cat([ip, l4f]))
    return a


# ---------------------------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1): the oracle on the host cores this process may use
# ---------------------------------------------------------------------------------------------


def host_cpu_share() -> dict:
    """The host threads this process can actually run: the affinity mask, capped by a cgroup CPU
    quota when one is set (a container's share of a large host; `nproc` shows the whole host)."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(period)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                period = int(f.read())
            if q > 0:
                quota = q / period
        except (OSError, ValueError):
            pass
    threads = aff if quota is None else max(1, min(aff, int(math.floor(quota))))
    if os.environ.get("SMOL_CPU_THREADS"):
        threads = max(1, int(os.environ["SMOL_CPU_THREADS"]))
    return {"nproc": nproc, "affinity": aff, "cgroup_cpu_quota": quota, "threads": threads}


def _cpulist(text: str):
    out = []
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out += list(range(int(a), int(b or a) + 1))
    return out


def cgroup_cpu_stat() -> dict:
    """The cgroup's CPU accounting (cgroup v2 cpu.stat): usage and CFS bandwidth throttling. A job
    whose threads exceed its CPU quota within a period is stopped until the next one; the CPU
    baseline reports how often that happened while it ran."""
    out = {}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, _, v = line.partition(" ")
                if k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
                    out[k] = int(v)
    except (OSError, ValueError):
        pass
    return out


def cgroup_delta(a: dict, b: dict) -> dict:
    return {k: b[k] - a[k] for k in b if k in a}


def pick_cpus(threads: int):
    """`threads` CPUs of this process's affinity set for the CPU baseline: one hardware thread per
    core (SMT siblings only once every core has one), taken round-robin over the NUMA nodes so that
    every node's memory controllers serve the threads placed on it.  Returns (cpus, node of each)."""
    aff = set(os.sched_getaffinity(0))
    nodes = {}
    for path in glob.glob("/sys/devices/system/node/node[0-9]*/cpulist"):
        try:
            with open(path) as f:
                cs = [c for c in _cpulist(f.read()) if c in aff]
            if cs:
                nodes[int(path.split("node")[-1].split("/")[0])] = cs
        except (OSError, ValueError):
            pass
    if not nodes:
        nodes = {0: sorted(aff)}

    def core(c):
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/core_id") as f:
                cid = int(f.read())
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id") as f:
                return int(f.read()), cid
        except (OSError, ValueError):
            return c, c

    per_node = {}
    for n, cs in nodes.items():  # first hardware thread of each core, then the siblings
        seen, firsts, rest = set(), [], []
        for c in cs:
            (rest if core(c) in seen else firsts).append(c)
            seen.add(core(c))
        per_node[n] = firsts + rest
    order, i = [], 0
    while len(order) < threads and any(per_node.values()):
        for n in sorted(per_node):
            if per_node[n] and len(order) < threads:
                order.append((per_node[n].pop(0), n))
        i += 1
    order = order or [(c, 0) for c in sorted(aff)[:threads]]
    return [c for c, _ in order], [n for _, n in order]


class PinnedTeam:
    """`len(cpus)` host threads, thread i pinned to cpus[i] (Linux: sched_setaffinity(0) sets the
    calling thread's mask), running one job at a time: run(fn) calls fn(i) on every thread i and
    returns the results.  Memory a thread allocates and touches first lives on its NUMA node."""

    def __init__(self, cpus):
        import threading

        self.n = len(cpus)
        self.fn, self.out, self.stop = None, [None] * self.n, False
        self.go = threading.Barrier(self.n + 1)
        self.done = threading.Barrier(self.n + 1)
        self.threads = [threading.Thread(target=self._loop, args=(i, c), daemon=True) for i, c in enumerate(cpus)]
        for t in self.threads:
            t.start()

    def _loop(self, i, cpu):
        try:
            os.sched_setaffinity(0, {cpu})
        except OSError:
            pass
        while True:
            self.go.wait()
            if self.stop:
                return
            try:
                self.out[i] = self.fn(i)
            except BaseException as e:  # re-raised by run()
                self.out[i] = e
            self.done.wait()

    def run(self, fn):
        self.fn = fn
        self.go.wait()
        self.done.wait()
        for r in self.out:
            if isinstance(r, BaseException):
                raise r
        return list(self.out)

    def close(self):
        self.stop = True
        self.go.wait()
        for t in self.threads:
            t.join()


def cpu_baseline(E, wl, seconds: float):
    """cpu_baseline leg: the oracle (a C restatement of smoltcp's scalar checksum + gates), built on
    this host with ROCm clang -O3 -march=native, timed over a sample of the same workload larger
    than the host's last-level cache, on 1 thread and on every host thread this process may use;
    the value is the median of >= 10 passes.  The oracle is also the checker here: its emit of the
    sample (emit is idempotent) must reproduce the device's emitted bytes and its verify the
    device's status bytes, bit for bit."""
    import torch

    import oracle

    if seconds <= 0:
        return None, None
    share = host_cpu_share()
    threads = share["threads"]
    # one thread per core, spread over the NUMA nodes; every thread works on its own copy of its
    # records, first touched by itself (so it lives on the thread's node)
    pin, pin_nodes = pick_cpus(threads)
    if wl.batch.desc is None:
        L = wl.batch.length
        m = min(wl.n, max(1, CPU_SAMPLE_BYTES // L))
        end = (m - 1) * L + L
        desc, stride = None, L
        span = wl.span_bytes * m // wl.n
    else:
        d_all = wl.batch.desc.cpu().numpy().view(E.DESC_DTYPE)
        ends = d_all["offset"] + d_all["len"].astype(np.uint64)
        m = max(1, int(np.searchsorted(ends, np.uint64(CPU_SAMPLE_BYTES), side="right")))
        d = d_all[:m].copy()
        end = int(ends[m - 1])
        desc, stride, L = d, 0, 0
        span = int(d["len"].astype(np.uint64).sum())
    dev_tx = wl.tx[:end].cpu().numpy()
    dev_st = wl.status[:m].cpu().numpy()
    dev_rx = wl.rx[:end].cpu().numpy()
    caps = (0, 0, 0, 0, 0)
    build = oracle.use_native()
    bounds = [S.shard_range(m, t, threads) for t in range(threads)]

    def records_of(lo, hi):
        """(tx, rx, desc) copies of records [lo, hi), made by the calling thread."""
        if hi == lo:
            return None
        if desc is None:
            a, b, d = lo * stride, (hi - 1) * stride + L, None
        else:
            a = int(desc["offset"][lo])
            b = int(desc["offset"][hi - 1]) + int(desc["len"][hi - 1])
            d = desc[lo:hi].copy()
            d["offset"] -= np.uint64(a)
        return dev_tx[a:b].copy(), dev_rx[a:b].copy(), d, hi - lo, a

    def one_pass(part):  # emit tx + verify rx over one thread's records
        if part is None:
            return np.zeros(0, np.uint8)
        tx, rx, d, k, _ = part
        oracle.batch_emit(tx, d, k, stride, L, wl.kind, caps)
        return oracle.batch_verify(rx, d, k, stride, L, wl.kind, caps)

    def timed_passes(run_once, budget):
        run_once()  # warm
        times, t0 = [], time.perf_counter()
        out = None
        while len(times) < 10 or (time.perf_counter() - t0 < budget and len(times) < 200):
            a = time.perf_counter()
            out = run_once()
            times.append(time.perf_counter() - a)
        med, best = float(np.median(times)), float(min(times))
        p10, p90 = (float(x) for x in np.percentile(times, [10, 90]))
        return out, {"GiB/s": 2 * span / med / GIB, "best_GiB/s": 2 * span / best / GIB, "reps": len(times),
                     "median_s": med, "spread": float((max(times) - min(times)) / med),
                     "p10_p50_p90_GiB/s": [round(2 * span / x / GIB, 2) for x in (p90, med, p10)],
                     "spread_p10_p90": float((p90 - p10) / med)}

    res, cg = {}, {}
    team = PinnedTeam(pin)
    try:
        # all threads, each over its own records
        parts = team.run(lambda i: records_of(*bounds[i]))
        c0 = cgroup_cpu_stat()
        sts, res[threads] = timed_passes(lambda: team.run(lambda i: one_pass(parts[i])), seconds / 2)
        cg[threads] = cgroup_delta(c0, cgroup_cpu_stat())
        # one thread over the whole sample (thread 0's copy)
        if threads > 1:
            whole = team.run(lambda i: records_of(0, m) if i == 0 else None)[0]
            c0 = cgroup_cpu_stat()
            st1, res[1] = timed_passes(lambda: team.run(lambda i: one_pass(whole) if i == 0 else None)[0], seconds / 2)
            cg[1] = cgroup_delta(c0, cgroup_cpu_stat())
            del whole
        else:
            res[1] = res[threads]
    finally:
        team.close()
    torch.cuda.synchronize()
    st = np.concatenate(sts)
    emit_ok = all(p is None or np.array_equal(p[0], dev_tx[p[4]:p[4] + p[0].size]) for p in parts)
    tx = None
    parity = {"records": m, "emit_bitexact": bool(emit_ok),
              "verify_bitexact": bool(np.array_equal(st, dev_st)),
              "checker": "oracle/csum_oracle.c on the cpu_baseline sample"}
    r = res[threads]
    out = {"value": round(r["GiB/s"], 3), "unit": "GiB/s", "cores": threads, "kind": "port",
           "single_core_value": round(res[1]["GiB/s"], 3),
           "best_value": round(r["best_GiB/s"], 3), "single_core_best_value": round(res[1]["best_GiB/s"], 3),
           "spread": round(r["spread"], 3),
           "spread_p10_p90": round(r["spread_p10_p90"], 3),
           "pass_rate_p10_p50_p90": r["p10_p50_p90_GiB/s"],
           "single_core_pass_rate_p10_p50_p90": res[1]["p10_p50_p90_GiB/s"],
           "pinned_cpus": pin, "numa_nodes": sorted(set(pin_nodes)),
           "host": share,
           "cgroup_cpu_stat_delta": {"all_threads": cg.get(threads, {}), "one_thread": cg.get(1, {}),
                                     "what": "cgroup v2 cpu.stat over the timed passes: CPU time used and "
                                             "CFS quota throttling (periods the job was stopped)"},
           "sample": f"{m} records of the same workload ({end / 1e9:.2f} GB per buffer, > host LLC): emit tx + "
                     f"verify rx; median of {r['reps']} passes on {threads} threads ({res[1]['reps']} on 1; the "
                     f"host is shared: the fastest pass is beside it); "
                     f"oracle/csum_oracle.c built {build}; records split evenly over the threads, one thread "
                     f"per core spread over the NUMA nodes, each on its own first-touched copy of its records "
                     f"(the 1-thread value: one thread over the whole sample)"}
    return out, parity


def parity_spread(E, wl, records: int = 65536, windows: int = 64) -> dict:
    """The oracle check without timing, over `records` records sampled across the WHOLE batch (`windows`
    runs of consecutive records, evenly spaced from the first record to the last): the oracle's emit of
    each run (emit is idempotent) must reproduce the device's emitted TX bytes, and its verify of the
    RX bytes the device's status bytes, bit for bit.  Runs on every config, with or without the CPU
    baseline (whose sample is the batch's first 1.6 GB).  C2copy: the TX bytes are the fused
    copy-emit's; the oracle's copy + emit of each run (the payload copied from the source, then the
    fields) must reproduce them, so a wrong payload byte or field fails it (header bytes other than
    the fields are the oracle's input, not checked)."""
    import oracle

    n = wl.n
    per = max(1, min(n, records) // windows)
    starts = sorted({int(x) for x in np.linspace(0, max(0, n - per), windows)})
    desc_all = wl.batch.desc.cpu().numpy().view(E.DESC_DTYPE) if wl.batch.desc is not None else None
    stride, L = (wl.batch.stride, wl.batch.length) if desc_all is None else (0, 0)
    st_all = wl.status.cpu().numpy()
    copy_all = wl.copy.cpu().numpy().view(E.COPY_DTYPE) if wl.copy is not None else None
    checked, emit_ok, verify_ok = 0, True, True
    for lo in starts:
        hi = min(n, lo + per)
        if desc_all is None:
            a, b, d = lo * stride, (hi - 1) * stride + L, None
        else:
            d = desc_all[lo:hi].copy()
            a = int(d["offset"].min())
            b = int((d["offset"] + d["len"].astype(np.uint64)).max())
            d["offset"] -= np.uint64(a)
        tx = wl.tx[a:b].cpu().numpy()
        rx = wl.rx[a:b].cpu().numpy()
        ref = tx.copy()
        if copy_all is None:
            oracle.batch_emit(ref, d, hi - lo, stride, L, wl.kind, (0, 0, 0, 0, 0))
        else:
            cp = copy_all[lo:hi].copy()
            s0 = int(cp["src_offset"].min())
            s1 = int((cp["src_offset"] + cp["len"].astype(np.uint64)).max())
            cp["src_offset"] -= np.uint64(s0)
            src = wl.src[s0:s1].cpu().numpy()
            oracle.batch_copy_emit(ref, d, hi - lo, src, cp, stride, L, wl.kind, (0, 0, 0, 0, 0))
        emit_ok &= bool(np.array_equal(ref, tx))
        st = oracle.batch_verify(rx.copy(), d, hi - lo, stride, L, wl.kind, (0, 0, 0, 0, 0))
        verify_ok &= bool(np.array_equal(st, st_all[lo:hi]))
        checked += hi - lo
    return {"records": checked, "windows": len(starts), "emit_bitexact": emit_ok, "verify_bitexact": verify_ok,
            "checker": "oracle/csum_oracle.c",
            "sample": f"{len(starts)} runs of {per} consecutive records evenly spaced over all {n} records "
                      f"(first run at record 0, last ending at record {n - 1}): "
                      + ("the fused copy-emit's TX bytes" if copy_all is not None else "emit of TX batch 0")
                      + ", verify of RX batch 0 (the last verify's status)"}


def _launch_name(ll):
    """'xwalk_kernel v47 G8 U2' from an engine.last_launch() record."""
    return "?" if not ll else f"{ll['kernel']} v{ll['variant']} G{ll['G']} U{ll['U']}"


def load_traffic(cfg: str, kernel: str):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary (profiles/*traffic*.json)."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json")), reverse=True):
        try:
            with open(path) as f:
                t = json.load(f)
        except Exception:
            continue
        ent = t.get(cfg, {}).get(kernel)
        if ent and "hbm_bytes_per_launch" in ent:
            return ent["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


# ---------------------------------------------------------------------------------------------
# One rank
# ---------------------------------------------------------------------------------------------


def gather_floats(vals, device=None):
    """all_gather of a few floats per rank -> list (one list per rank); identity at world 1."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return [list(vals)]
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[float(x) for x in o.cpu().tolist()] for o in out]


def run_dry(args, world, rank, local):
    """--dry-run: the launch, rendezvous and reporting of a multi-rank run, on CPU, no work."""
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    if world > 1:
        dist.barrier()
    mine = time.perf_counter() - t0
    per = gather_floats([rank, local, mine])
    elapsed = S.max_over_ranks(mine)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(elapsed / max(args.steps, 1) * 1e3, 6),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
                          "data": "dry run: no checksum work", "dry_run": True,
                          "config": {"workload": f"dry run of --config {args.config}",
                                     "parallelism": f"shard x{world} (no collective)"},
                          "per_rank": [{"rank": int(p[0]), "local_rank": int(p[1]), "elapsed_s": p[2]} for p in per]}),
              flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    world, rank, local = S.dist_env()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, argv)
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if args.dry_run:
        run_dry(args, world, rank, local)
        return 0

    import torch
    import torch.distributed as dist

    from smoltcp_amd import engine as E

    if torch.cuda.device_count() <= local:
        print(f"bench.py: rank {rank} needs cuda:{local}, {torch.cuda.device_count()} GPU(s) visible",
              file=sys.stderr)
        return 2
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # one process group per job over RCCL, for the barriers and the max-over-ranks reduction only
    # (no collective on the data path); under a launcher (WORLD_SIZE set) also at world size 1, so
    # that a one-GPU box runs the same RCCL calls as the 8-GPU node
    pg = world > 1 or "WORLD_SIZE" in os.environ
    if pg:
        dist.init_process_group("nccl", device_id=dev)

    eng = E.ChecksumEngine(local)
    if args.shape >= 0:
        eng.set_shape(args.shape)
    if args.variant >= 0:
        eng.set_variant(args.variant)
    eng.set_xcd_remap(args.xcd_remap)
    if args.launch_records >= 0:
        eng.set_launch_records(args.launch_records)
    wl = Workload(E, eng, args.config, args.n, rank, dev, args.batches, args.src_stride)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)
    split_variants = args.emit_variant >= 0 or args.verify_variant >= 0  # (set per operation, host-side)
    R = len(wl.txs)
    nstep = [0]
    launched = {}  # the kernel each op ran (smol_csum_tool_last_launch), recorded at instrumented steps

    def step(ev=None, same=False):
        # step i emits TX batch i mod R and verifies RX batch i mod R (same: batch 0 every time)
        j = 0 if same else nstep[0] % R
        nstep[0] += 1
        if ev is not None:
            ev[0].record(stream)
        if split_variants:
            eng.set_variant(args.emit_variant if args.emit_variant >= 0 else args.variant)
        if wl.copy is not None:
            eng.copy_emit(wl.txs[j], wl.batch, wl.src, wl.copy, stream=stream)
        else:
            eng.emit(wl.txs[j], wl.batch, stream=stream)
        if ev is not None:
            launched["copy_emit" if wl.copy is not None else "emit"] = eng.last_launch()
            ev[1].record(stream)
        if split_variants:
            eng.set_variant(args.verify_variant if args.verify_variant >= 0 else args.variant)
        eng.verify(wl.rxs[j], wl.batch, status=wl.status, stream=stream)
        if ev is not None:
            launched["verify"] = eng.last_launch()
            ev[2].record(stream)

    # Clock ramp: a freshly idle MI355X takes ~15 ms of sustained load before its kernels run at
    # their steady-state speed (profiles/r03_steps/step_trace_c2_w5.json: verify 273 -> 245 us
    # over the 20 timed steps after 5 warm-up steps; 234 us after 100).  Untimed steps for
    # --ramp-ms of wall time come first, then the W warm-up steps the contract names.
    ramp_steps, r0 = 0, time.perf_counter()
    while (time.perf_counter() - r0) * 1e3 < args.ramp_ms:
        for _ in range(8):
            step()
        ramp_steps += 8
        torch.cuda.synchronize()
    ramp_ms = (time.perf_counter() - r0) * 1e3
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # The timed region: K steps with nothing between the kernels (timing events at the kernel
    # boundaries cost ~2 % of a step, tools/exp_timing.py).
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    torch.cuda.synchronize()
    mine = time.perf_counter() - t0
    if pg:
        dist.barrier()
    elapsed = S.max_over_ranks(mine, device=dev)

    # Kernel durations for the roofline: K more steps with HIP events at the kernel boundaries, on
    # the stream the kernels are launched on.
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize()

    emit_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    verify_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))

    # Side figure (not the value): the same K instrumented steps re-emitting ONE batch, as the bench
    # did through round 4.  Its field segments stay dirty in the Infinity Cache between passes, so
    # its emit is faster than a TX path's.
    same_batch = None
    if R > 1:
        evs1 = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
        for i in range(args.steps):
            step(evs1[i], same=True)
        torch.cuda.synchronize()
        e1 = float(np.mean([e[0].elapsed_time(e[1]) for e in evs1]))
        v1 = float(np.mean([e[1].elapsed_time(e[2]) for e in evs1]))
        same_batch = {"emit_ms": round(e1, 4), "verify_ms": round(v1, 4),
                      "emit_fresh_over_same": round(emit_ms / e1, 4),
                      "what": "K instrumented steps over batch pair 0 only (the round-1..4 bench form), right after "
                              "the rotating pass: the field segments the previous pass wrote are still dirty in "
                              "the Infinity Cache"}

    # the expected rejections of the last verify (1/64 single-bit flips, or none for C5)
    st = wl.status.cpu().numpy()
    rejected = int(((st & E.ST_ACCEPT) == 0).sum())
    per = gather_floats([rank, local, mine, emit_ms, verify_ms, rejected], device=dev)

    # Emit's floor (rank 0): the read-only stream probe over the TX buffer, and the same stream plus
    # emit's writes in emit's own shape (smol_csum_tool_segment_probe: every 64-B segment holding a
    # checksum field written back whole, with its own bytes, by the lanes that just read it; plain and
    # non-temporal stores, the faster is the floor).  floor_2b: the same stream plus a 2-B store at
    # every field instead (smol_csum_tool_field_probe / _list, the floor of a 2-B-store emit).
    probe = floor = None
    if rank == 0 and wl.copy is None:
        sink = torch.zeros(1, dtype=torch.int32, device=dev)

        def timed(fn, reps=10):
            for _ in range(3):
                fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(reps):
                fn()
            b.record(stream)
            torch.cuda.synchronize()
            return a.elapsed_time(b) / reps

        ro_ms = timed(lambda: eng.stream_read(wl.tx, sink, stream=stream))
        addrs = field_addrs(wl)
        nb = wl.tx.numel() // 16 * 16
        bitmap, nseg = E.segment_bitmap(addrs, nb)
        seg_ms = {nt: timed(lambda: eng.segment_probe(wl.tx, bitmap, nt=nt, stream=stream)) for nt in (False, True)}
        del bitmap
        # the 2-B probe stores into wl.tx: the bytes it overwrites are saved first and put back after it
        # (emit is not a restore: on C3 / C4 the probe's offsets are not all checksum fields)
        pieces = torch.arange(0, (nb + 8191) // 8192 + 1, device=dev, dtype=torch.int64) * 8192
        first = torch.searchsorted(addrs, pieces).to(torch.int32)
        del pieces
        saved = torch.stack([wl.tx[addrs], wl.tx[addrs + 1]])
        if wl.batch.desc is None and wl.cfg != "c4":
            stride, f1, f2 = wl.probe_fields
            fp_ms = timed(lambda: eng.field_probe(wl.tx, stride, f1, f2, stream=stream))
            where = (f"a 2-B store at offsets {f1}" + (f" and {f2}" if f2 != 0xFFFFFFFF else "")
                     + f" of every {stride}-B record")
        else:
            fp_ms = timed(lambda: eng.field_probe_list(wl.tx, addrs, first, stream=stream))
            where = f"a 2-B store at each of the {addrs.numel()} checksum fields of the records (from their headers)"
        wl.tx[addrs] = saved[0]
        wl.tx[addrs + 1] = saved[1]
        del saved
        del addrs, first
        torch.cuda.synchronize()
        probe = {"kernel": "stream_read_kernel", "bytes": nb, "ms": round(ro_ms, 4),
                 "GB/s": round(nb / ro_ms / 1e6, 1)}
        best_nt = seg_ms[True] <= seg_ms[False]
        floor = {"kernel": "segment_probe_kernel", "ms": round(min(seg_ms.values()), 4),
                 "stores": "non-temporal" if best_nt else "plain",
                 "ms_plain_stores": round(seg_ms[False], 4), "ms_nt_stores": round(seg_ms[True], 4),
                 "segments": nseg, "read_only_ms": round(ro_ms, 4),
                 "what": f"emit's floor in its store shape: the TX buffer streamed once (the stream-read probe's "
                         f"pattern) + the {nseg} 64-B segments holding its checksum fields written back whole with "
                         f"their own bytes by the lanes that just read them (no parse / gates); the faster of plain "
                         f"and non-temporal stores"}
        floor_2b = {"kernel": "field_probe_kernel", "ms": round(fp_ms, 4),
                    "what": "the 2-B-store reference: the same stream + " + where
                            + " (emit's store events as 2-B writes); the bytes the probe overwrote are restored"}

    unfused = None
    if wl.copy is not None and rank == 0:
        # the unfused TX path for comparison: payload copy (strided device copy) then emit
        dst = wl.tx.view(wl.n, 1500)[:, 28:]
        sst = args.src_stride
        srcv = wl.src[: wl.n * sst].view(wl.n, sst)[:, :1472]
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(2):
            dst.copy_(srcv)
            eng.emit(wl.tx, wl.batch, stream=stream)
        a.record(stream)
        for _ in range(args.steps):
            dst.copy_(srcv)
            eng.emit(wl.tx, wl.batch, stream=stream)
        b.record(stream)
        torch.cuda.synchronize()
        unfused = {"tx_ms": round(a.elapsed_time(b) / args.steps, 4),
                   "what": "payload copy (torch strided copy_) + smol_csum_batch_emit, same batch"}
        eng.copy_emit(wl.tx, wl.batch, wl.src, wl.copy, stream=stream)  # leave the fused result in place
        torch.cuda.synchronize()

    cpu, parity = None, None
    if rank == 0 and world == 1 and wl.copy is None:
        cpu, parity = cpu_baseline(E, wl, args.cpu_seconds)
    if rank == 0:
        spread = parity_spread(E, wl)
        parity = dict(parity or {}, spread=spread) if parity else {"spread": spread}

    if rank == 0:
        value = S.aggregate_rate(2 * wl.span_bytes, world, args.steps, elapsed)
        # roofline of the dominant kernel: algorithmic bytes per launch / its mean launch time
        kernels = {
            "emit": {"ms": emit_ms, "bytes": wl.read_bytes + wl.desc_bytes + 4 * wl.n},
            "verify": {"ms": verify_ms, "bytes": wl.read_bytes + wl.desc_bytes + wl.n},
        }
        if wl.copy is not None:  # fused copy + emit: headers + payload read once, payload written once
            kernels["emit"]["bytes"] = wl.read_bytes + wl.write_bytes_tx
            kernels["verify"]["bytes"] = wl.n * 1500 + wl.n
        dom = max(kernels, key=lambda k: kernels[k]["ms"])
        kd = kernels[dom]
        achieved = kd["bytes"] / (kd["ms"] * 1e-3) / 1e9
        dop = "copy_emit" if (wl.copy is not None and dom == "emit") else dom
        traffic, tsrc = load_traffic(args.config, dop)
        per_rank = [{"rank": int(p[0]), "local_rank": int(p[1]), "elapsed_s": round(p[2], 6),
                     "value": round(2 * wl.span_bytes * args.steps / p[2] / GIB, 2),
                     "ms_per_step": round(p[2] / args.steps * 1e3, 4), "emit_ms": round(p[3], 4),
                     "verify_ms": round(p[4], 4), "verify_rejected": int(p[5])} for p in per]
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: device-generated packets (splitmix64 payload, seeded), HBM-resident",
            "config": {"workload": wl.workload, "records_per_gpu": wl.n, "parallelism": f"shard x{world} (no collective)",
                       "checksummed_bytes_per_step_per_gpu": 2 * wl.span_bytes,
                       "process_group": dist.get_backend() if pg else None},
            "roofline": {"bound": "hbm", "kernel": f"{_launch_name(launched.get(dop))} ({dop})", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": tsrc,
                         "algorithmic_bytes_per_launch": kd["bytes"], "launch_ms": round(kd["ms"], 4)},
            "kernels_ms": {k: round(v["ms"], 4) for k, v in kernels.items()},
            "kernels_launched": {k: _launch_name(v) for k, v in launched.items()},
            "kernels_roofline": {k: {"algorithmic_bytes_per_launch": v["bytes"], "launch_ms": round(v["ms"], 4),
                                     "achieved_GBs": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1),
                                     "frac": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                                 for k, v in kernels.items()},
            "kernel_timing": "HIP events at the kernel boundaries on the launch stream, over a second pass of "
                             "K steps after the timed region (the timed region has no events between kernels)",
            "ramp": {"steps": ramp_steps, "ms": round(ramp_ms, 1),
                     "what": "untimed steps before the W warm-up steps until the GPU clocks have ramped "
                             "(steady state: profiles/r03_steps/)"},
            "verify_rejected": rejected,
            "batches": {"pairs": R, "what": (f"step i emits TX batch i mod {R} and verifies RX batch i mod {R} "
                                             "(timed steps and kernel timings alike)") if R > 1 else
                        "one batch (C5: emit and verify in place over one 201-GB buffer)"},
            "emit_same_batch": same_batch,
            "per_rank": per_rank,
            "cpu_baseline": cpu,
            "parity_sample": parity,
        }
        if probe:
            out["stream_read_probe"] = probe
        if floor and dom == "emit":
            out["roofline"]["floor"] = floor
            out["roofline"]["floor_frac"] = round(floor["ms"] / kd["ms"], 4)
            out["roofline"]["floor_2b"] = floor_2b
            out["roofline"]["floor_2b_frac"] = round(floor_2b["ms"] / kd["ms"], 4)
        if probe and dom in ("emit", "verify"):
            # the dominant kernel against the read-only stream over the same bytes (1.0 = it runs at
            # the speed of reading its input once at the best pattern)
            out["roofline"]["read_only_frac"] = round(probe["ms"] / kd["ms"], 4)
        # the whole step against the HBM peak: algorithmic bytes of both kernels / wall time per step
        step_bytes = sum(v["bytes"] for v in kernels.values())
        out["roofline"]["step_frac"] = round(step_bytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4)
        out["roofline"]["step_algorithmic_bytes"] = step_bytes
        if unfused:
            out["unfused_tx"] = unfused
        print(json.dumps(out), flush=True)
    if pg:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
