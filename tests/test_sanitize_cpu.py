"""Host-side sanitizer run (ASan/UBSan on the C/C++ host code).

`make -C tests/cpp sanitize` builds
* oracle_asan: oracle/csum_oracle.c + the library's scalar mirrors (smoltcp_amd/csrc/csum_scalar.cpp)
  with -fsanitize=address,undefined, driven over every truncation of the golden records (KATs
  wrapped in IP packets, the iface IPv6 packets, the fuzz-corpus frames, the ICMP rule records) and
  over random records; each truncated record sits in a heap block of exactly its length;
* test_host_mirror_asan: the C++ host mirror driver (smoltcp_amd/host/smoltcp_checksum.hpp) with
  the same flags, over the scalar vectors and the no-device path.
Any report aborts the binary (-fno-sanitize-recover=all), which fails the test."""
import os
import subprocess

import numpy as np
import pytest

from oracle import pyref
from tests import pktgen as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")


@pytest.fixture(scope="module")
def built():
    # one build at a time: under pytest-xdist every worker runs this fixture, and a make that
    # relinks a binary while another worker executes it fails that worker's test
    import fcntl

    with open(os.path.join(CPP, ".sanitize.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", CPP, "sanitize"], check=True, timeout=600)
    return CPP


def _records(golden):
    out = []
    for f in golden["fuzz_corpus_frames"]:
        out.append((2, bytes.fromhex(f["bytes"])))
    for p in golden["iface_ipv6_packets"]:
        out.append((1, bytes.fromhex(p["bytes"])))
    v4a, v4b = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    for k in golden["kat"]:
        b = bytes.fromhex(k["bytes"])
        if k["proto"] == "ipv4":
            out.append((1, b))
        elif k["proto"] in ("icmpv6",) or (k["src"] and len(bytes.fromhex(k["src"])) == 16):
            nh = {"icmpv6": 58, "udp": 17, "tcp": 6}[k["proto"]]
            out.append((1, P.ipv6(bytes.fromhex(k["src"]), bytes.fromhex(k["dst"]), nh, b)))
        else:
            nh = {"udp": 17, "tcp": 6, "icmpv4": 1, "igmp": 2}[k["proto"]]
            out.append((1, P.ipv4(v4a, v4b, nh, b)))
    rng = np.random.default_rng(3)
    inner = P.ipv4(v4b, v4a, 17, P.udp(1, 2, b"x" * 12))
    out.append((1, P.ipv4(v4a, v4b, 1, P.icmp4_error(3, 3, inner))))
    out.append((1, P.ipv4(v4a, v4b, 1, P.icmp4_error(11, 0, P.ipv4(v4b, v4a, 6, b"", ihl=15)))))
    for t in (1, 128, 130, 134, 135, 137, 155, 200):
        out.append((1, P.ipv6(bytes(16), bytes(range(16)), 58, P.icmp6(t, 44, rng))))
    out.append((1, P.ipv6(bytes(16), bytes(16), 0, P.hbh(17, 3, rng) + P.udp(5, 6, b"abc"))))
    return out


def test_oracle_and_scalar_mirrors_asan_golden(built, golden, tmp_path):
    recs = _records(golden)
    f = tmp_path / "records.txt"
    f.write_text("".join(f"{k} {b.hex()}\n" for k, b in recs))
    r = subprocess.run([os.path.join(built, "oracle_asan"), "records", str(f)], capture_output=True, text=True,
                       timeout=600, env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.strip() == f"ok {len(recs)}"


@pytest.mark.parametrize("seed", [1, 0xC0FFEE])
def test_oracle_and_scalar_mirrors_asan_random(built, seed):
    r = subprocess.run([os.path.join(built, "oracle_asan"), "random", str(seed), "20000"], capture_output=True,
                       text=True, timeout=600, env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.strip() == "ok 20000"


@pytest.mark.parametrize("seed", [3, 0xF4A6])
def test_oracle_frag_groups_asan(built, seed):
    """The fragment-group oracle (group_copy into its 128 KiB reassembly buffer, offsets up to
    65528) and the dispatch_ip restatement under ASan/UBSan."""
    r = subprocess.run([os.path.join(built, "oracle_asan"), "frag", str(seed), "3000"], capture_output=True,
                       text=True, timeout=600, env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.strip() == "ok 3000"


def test_host_mirror_asan(built, tmp_path, golden):
    rng = np.random.default_rng(9)
    lines = []
    spans = [b"", b"\x00", b"\xff", bytes(131074), b"\xff" * 131075]
    spans += [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 3000, 100)]
    for s in spans:
        lines.append(f"data {s.hex() or '-'} {pyref.data(s)}")
    for _ in range(50):
        ws = [int(x) for x in rng.integers(0, 65536, int(rng.integers(0, 9)))]
        lines.append(f"comb {pyref.combine(ws)} " + " ".join(map(str, ws)))
        for n in (4, 16):
            a = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            nh, ln = int(rng.integers(256)), int(rng.integers(0, 1 << 32))
            lines.append(f"ph {a.hex()} {b.hex()} {nh} {ln} {pyref.pseudo_header(a, b, nh, ln)}")
    lines.append(f"ph {bytes(4).hex()} {bytes(16).hex()} 6 0 65536")
    p = tmp_path / "vectors.txt"
    p.write_text("\n".join(lines) + "\n")
    binary = os.path.join(built, "test_host_mirror_asan")
    r = subprocess.run([binary, "vectors", str(p)], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, r.stderr[-4000:]
    assert f"vectors {len(lines)}" in r.stdout
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if not has_gpu:
        r = subprocess.run([binary, "nodev"], capture_output=True, text=True, timeout=120, env=ENV)
        assert r.returncode == 0, r.stderr[-4000:]
