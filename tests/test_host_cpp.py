"""The C++ host-side mirror (smoltcp_amd/host/smoltcp_checksum.hpp) through tests/cpp/test_host_mirror.

CPU: the scalar mirrors against oracle-computed values (data / combine / pseudo_header incl. the
family-mismatch error), the phy policy mirror, and Engine() failing with SMOL_ENODEV (no CPU
fallback).  GPU: an offloading device's TX (emit) and RX (verify) over host frames, checked with the
scalar gates on the host.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import pyref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")
BIN = os.path.join(CPP, "test_host_mirror")


@pytest.fixture(scope="module")
def binary():
    # one make at a time: pytest-xdist workers may each build this module's binary
    import fcntl

    with open(os.path.join(CPP, ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", CPP], check=True)
    return BIN


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def test_cpp_scalar_mirrors(binary, tmp_path, golden):
    rng = np.random.default_rng(5)
    lines = []
    spans = [b"", b"\x00", b"\xff", bytes(131074), b"\xff" * 131075]
    spans += [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 3000, 200)]
    spans += [bytes.fromhex(k["bytes"]) for k in golden["kat"]]
    for s in spans:
        lines.append(f"data {s.hex() or '-'} {pyref.data(s)}")
    for _ in range(100):
        ws = [int(x) for x in rng.integers(0, 65536, int(rng.integers(0, 9)))]
        lines.append(f"comb {pyref.combine(ws)} " + " ".join(map(str, ws)))
    for _ in range(100):
        for n in (4, 16):
            a = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            nh, ln = int(rng.integers(256)), int(rng.integers(0, 1 << 32))
            lines.append(f"ph {a.hex()} {b.hex()} {nh} {ln} {pyref.pseudo_header(a, b, nh, ln)}")
    lines.append(f"ph {bytes(4).hex()} {bytes(16).hex()} 6 0 65536")  # mismatch -> error
    p = tmp_path / "vectors.txt"
    p.write_text("\n".join(lines) + "\n")
    r = subprocess.run([binary, "vectors", str(p)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert f"vectors {len(lines)}" in r.stdout


def test_grid_orders_bijective(binary):
    """The walk kernel's XCD block orders (csum_launch.h xcd_block / xcd_chunk) visit every block
    once for every grid size (host build of the same header)."""
    r = subprocess.run([os.path.join(CPP, "test_grid_order")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "grid orders ok" in r.stdout, r.stdout + r.stderr


def test_cpp_engine_fails_loudly_without_device(binary):
    if _has_gpu():
        pytest.skip("a GPU is present")
    r = subprocess.run([binary, "nodev"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_cpp_offload_device_roundtrip(binary):
    assert _has_gpu()
    r = subprocess.run([binary, "offload", "20011"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "emitted all valid" in r.stdout


@pytest.mark.gpu
def test_cpp_offload_ring_raw_frames(binary):
    """OffloadRing with raw-socket slots (SMOL_REC_IPHDR_ONLY through per-chunk descriptors):
    the user's L4 bytes survive emit, verify gates their IPv4 header only."""
    assert _has_gpu()
    r = subprocess.run([binary, "raw", "7003"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "kept the user's L4 bytes" in r.stdout


@pytest.mark.gpu
def test_loopback_ring_c1_analogue():
    """tools/loopback_ring (OffloadRing: pinned ring -> HBM -> emit / verify -> host): every
    emitted frame passes both the GPU verify and the host scalar gates, and a sample of the ring's
    frames matches the oracle's emit and verify bit for bit."""
    import json

    assert _has_gpu()
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools"), "loopback_ring"], check=True)
    import tempfile

    import numpy as np

    import oracle

    with tempfile.TemporaryDirectory() as td:
        pre = os.path.join(td, "c1")
        r = subprocess.run([os.path.join(ROOT, "tools", "loopback_ring"), "70001", "1", pre], capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        out = json.loads(r.stdout.strip().splitlines()[-1])
        assert out["gpu_offload"]["accepted"] == 70001
        assert out["cpu_inline_1thread"]["accepted"] == 70001
        before = np.fromfile(pre + ".before", np.uint8)
        after = np.fromfile(pre + ".after", np.uint8)
        status = np.fromfile(pre + ".status", np.uint8)
    # the sampled ring frames (every 97th) against the oracle, byte for byte: emit of the frames as
    # the host built them (Ethernet kind, default caps) is what OffloadRing::emit left in the ring,
    # and verify of those bytes gives the status the device reported
    frame = out["frame_bytes"]
    m = (70001 + 96) // 97
    assert before.size == after.size == m * frame and status.size == m
    ref = before.copy()
    oracle.batch_emit(ref, None, m, frame, frame, 2)
    assert np.array_equal(ref, after), np.nonzero(ref != after)[0][:8]
    assert np.array_equal(oracle.batch_verify(after.copy(), None, m, frame, frame, 2), status)
