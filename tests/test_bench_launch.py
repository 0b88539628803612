"""bench.py's multi-rank launch: `--gpus N` starts N rank processes itself (before any GPU call),
rendezvous on 127.0.0.1 and rank 0 reports every rank.  `--dry-run` runs that launch,
rendezvous (gloo) and reporting on CPU with an empty step, so the N > 1 path of the driver's
scaling run is exercised here without a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout,
                          env=env, cwd=ROOT)


def _json_line(out: str):
    lines = [ln for ln in out.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_dry_run_launches_n_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr
    d = _json_line(r.stdout)
    assert d["n_gpus"] == n and d["dry_run"] is True
    assert sorted(p["rank"] for p in d["per_rank"]) == list(range(n))
    assert sorted(p["local_rank"] for p in d["per_rank"]) == list(range(n))  # one GPU per rank
    assert d["steps"] == 3 and d["warmup"] == 1


def test_dry_run_c5_config():
    r = _run(["--gpus", "2", "--dry-run", "--config", "c5", "--steps", "2"])
    assert r.returncode == 0, r.stderr
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and "c5" in d["config"]["workload"]


def test_world_size_must_match_gpus():
    """Under torch.distributed.run (WORLD_SIZE set) a mismatching --gpus is refused."""
    r = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr


def test_too_few_gpus_fails_loudly():
    """Without --dry-run the launcher counts the GPUs first (none in this container)."""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has GPUs")
    r = _run(["--gpus", "2", "--steps", "1"])
    assert r.returncode == 2
    assert "GPU(s) are visible" in r.stderr


def test_host_cpu_share():
    sys.path.insert(0, ROOT)
    import bench

    s = bench.host_cpu_share()
    assert s["threads"] >= 1 and s["nproc"] >= 1 and s["threads"] <= s["affinity"]


@pytest.mark.gpu
def test_bench_gpu_contract():
    """The real GPU path of the launcher: `--gpus 1` on the box, the JSON contract of the line
    (BASELINE.json's metric, n_gpus, per_rank, roofline with the emit floor, the clock ramp)."""
    r = _run(["--gpus", "1", "--config", "c2", "--steps", "3", "--warmup", "1", "--cpu-seconds", "0",
              "--ramp-ms", "50"], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert d["metric"] == base["metric"] and d["unit"] == "GiB/s" and d["higher_is_better"] is True
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["dtype"] == "u8"
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["scaling"] == "weak"
    assert [p["rank"] for p in d["per_rank"]] == [0]
    rl = d["roofline"]
    assert rl["bound"] == "hbm" and rl["unit"] == "GB/s" and rl["peak"] == 8000.0
    assert 0 < rl["frac"] < 1 and abs(rl["achieved"] / rl["peak"] - rl["frac"]) < 1e-3
    assert rl["floor"]["kernel"] == "segment_probe_kernel" and 0 < rl["floor_frac"]
    assert rl["floor"]["segments"] == 1310720 * d["config"]["records_per_gpu"] // (1 << 20)  # C2: 1.25 per record
    assert rl["floor_2b"]["kernel"] == "field_probe_kernel" and 0 < rl["floor_2b_frac"]
    sp = d["parity_sample"]["spread"]  # the oracle over runs of records spread across the whole batch
    assert sp["emit_bitexact"] and sp["verify_bitexact"] and sp["records"] >= 65536
    assert 0 < rl["read_only_frac"] and 0 < rl["step_frac"] < 1
    assert rl["step_algorithmic_bytes"] == sum(k["algorithmic_bytes_per_launch"] for k in d["kernels_roofline"].values())
    n64 = d["config"]["records_per_gpu"] // 64  # 1/64 single-bit flips (a few the gates cannot see)
    assert d["ramp"]["steps"] >= 8 and n64 - 16 <= d["verify_rejected"] <= n64
    assert d["cpu_baseline"] is None  # --cpu-seconds 0


@pytest.mark.gpu
def test_bench_c2copy_parity_spread():
    """C2copy's line carries the oracle check too: the fused copy-emit's TX bytes (payload and
    fields) over runs of records spread across the whole batch."""
    r = _run(["--gpus", "1", "--config", "c2copy", "--steps", "3", "--warmup", "1", "--cpu-seconds", "0",
              "--ramp-ms", "50"], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    sp = d["parity_sample"]["spread"]
    assert sp["emit_bitexact"] and sp["verify_bitexact"] and sp["records"] >= 65536
    assert "copy-emit" in sp["sample"]
    assert d["kernels_launched"]["copy_emit"].startswith("copy_kernel")


@pytest.mark.gpu
def test_bench_under_torchrun_rccl():
    """The driver's N > 1 launch (torch.distributed.run, one rank per GPU) at the size a one-GPU
    box allows: one rank, with the RCCL process group, barriers, max-over-ranks all_reduce and
    per-rank all_gather that every rank of the 8-GPU run makes."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "1", "--config", "c2",
           "--steps", "3", "--warmup", "1", "--cpu-seconds", "0", "--ramp-ms", "50"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 1 and d["config"]["process_group"] == "nccl"
    assert [p["rank"] for p in d["per_rank"]] == [0] and d["value"] > 0


def test_cpu_baseline_team_pinning():
    """The CPU baseline's threads: distinct CPUs of this process's affinity set, one per core
    first, spread over the NUMA nodes; each team thread runs pinned to its own CPU."""
    sys.path.insert(0, ROOT)
    import bench

    aff = os.sched_getaffinity(0)
    n = min(4, len(aff))
    cpus, nodes = bench.pick_cpus(n)
    assert len(cpus) == n == len(nodes) and len(set(cpus)) == n and set(cpus) <= aff
    team = bench.PinnedTeam(cpus)
    try:
        got = team.run(lambda i: (i, sorted(os.sched_getaffinity(0))))
        assert [g[0] for g in got] == list(range(n))
        assert all(g[1] == [cpus[g[0]]] for g in got)
        with pytest.raises(ZeroDivisionError):
            team.run(lambda i: 1 // (i - 1))  # an exception in one thread reaches the caller
        assert team.run(lambda i: i * i) == [i * i for i in range(n)]
    finally:
        team.close()
    assert os.sched_getaffinity(0) == aff  # the caller's own mask is untouched
