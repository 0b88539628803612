"""CPU-side checks of the C-ABI library: it loads, exports every symbol the headers declare, the
scalar host mirrors are bit-exact against the oracle, and the batched entry points fail loudly
(no CPU fallback) without a GPU.  No kernel is launched here."""
import ctypes
import os
import re
import sys

import numpy as np
import pytest

import oracle
from oracle import pyref
import smoltcp_amd
from smoltcp_amd import _lib, checksum

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    with open(os.path.join(ROOT, "include", header)) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(smol_csum_\w+)\s*\(", text)))


def test_library_loads_and_exports_all_declared_symbols():
    L = smoltcp_amd.lib()
    decl = _declared("smolcsum.h") + _declared("smolcsum_tools.h")
    assert len(decl) >= 17
    for name in decl:
        assert hasattr(L, name), f"{name} declared in include/ but not exported"
    assert sorted(_lib.ABI_SYMBOLS) == _declared("smolcsum.h")
    assert sorted(_lib.TOOL_SYMBOLS) == _declared("smolcsum_tools.h")
    assert L.smol_csum_abi_version() == 6


def test_library_is_a_gfx950_code_object():
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob, "libsmolcsum.so must embed gfx950 device code"


def test_scalar_data_matches_oracle():
    rng = np.random.default_rng(1)
    cases = [b"", b"\x01", b"\xff\xff", bytes(131074), b"\xff" * 131075, b"\xff" * 300001]
    cases += [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in range(0, 200)]
    cases += [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (1500, 9000, 65535)]
    for c in cases:
        assert checksum.data(c) == oracle.data(c), len(c)


def test_scalar_combine_and_pseudo_headers():
    rng = np.random.default_rng(2)
    for _ in range(300):
        ws = [int(x) for x in rng.integers(0, 65536, int(rng.integers(0, 8)))]
        assert checksum.combine(ws) == pyref.combine(ws)
        s4, d4 = rng.integers(0, 256, 4, dtype=np.uint8).tobytes(), rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
        s6, d6 = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        p, ln = int(rng.integers(256)), int(rng.integers(0, 1 << 32))
        assert checksum.pseudo_header_v4(s4, d4, p, ln) == pyref.pseudo_header_v4(s4, d4, p, ln)
        assert checksum.pseudo_header_v6(s6, d6, p, ln) == pyref.pseudo_header_v6(s6, d6, p, ln)
        assert checksum.pseudo_header(s4, d4, p, ln) == pyref.pseudo_header(s4, d4, p, ln)
        assert checksum.pseudo_header(s6, d6, p, ln) == pyref.pseudo_header(s6, d6, p, ln)
    with pytest.raises(ValueError):
        checksum.pseudo_header(bytes(4), bytes(16), 6, 0)


def test_scalar_mirrors_on_kats(golden):
    """data() of each KAT span (with its pseudo-header) reproduces the reference verdict."""
    for k in golden["kat"]:
        b = bytes.fromhex(k["bytes"])
        if k["proto"] == "ipv4":
            assert checksum.data(b[: (b[0] & 15) * 4]) == 0xFFFF
        elif k["proto"] in ("icmpv4", "igmp"):
            assert checksum.data(b) == 0xFFFF
        elif k["proto"] == "udp" and k["checksum"] == 0:
            continue
        else:
            src, dst = bytes.fromhex(k["src"]), bytes.fromhex(k["dst"])
            pnum = {"udp": 17, "tcp": 6, "icmpv6": 58}[k["proto"]]
            ln = (b[4] << 8 | b[5]) if k["proto"] == "udp" else len(b)
            span = b[:ln]
            if k["name"] == "udp4_zero_checksum":
                continue
            assert checksum.combine([checksum.pseudo_header(src, dst, pnum, ln), checksum.data(span)]) == 0xFFFF, k["name"]


def test_batched_calls_fail_loudly_without_a_device():
    L = smoltcp_amd.lib()
    h = ctypes.c_void_p()
    rc = L.smol_csum_ctx_create(0, ctypes.byref(h))
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if not has_gpu:
        assert rc == _lib.SMOL_ENODEV
    else:
        assert rc == _lib.SMOL_OK
        L.smol_csum_ctx_destroy(h)
    b = _lib.BatchC()
    b.n = 1
    caps = _lib.Caps()
    st = ctypes.c_uint8()
    assert L.smol_csum_batch_verify(None, None, ctypes.byref(b), ctypes.byref(caps), ctypes.byref(st), None) == _lib.SMOL_EINVAL
    assert L.smol_csum_batch_emit(None, None, ctypes.byref(b), ctypes.byref(caps), None, None) == _lib.SMOL_EINVAL
    assert L.smol_csum_batch_data(None, None, ctypes.byref(b), None, None) == _lib.SMOL_EINVAL
    with pytest.raises(Exception):
        from smoltcp_amd.engine import ChecksumEngine

        if not has_gpu:
            ChecksumEngine(0)
        else:
            raise RuntimeError("skip: GPU present")


def test_auto_shape():
    from smoltcp_amd.engine import auto_shape

    assert auto_shape(64) == 0      # 8 lanes x 6 chunks
    assert auto_shape(1500) == 7    # 8 x 7: eight 1500-byte records per wavefront, two steps each
    assert auto_shape(1900) == 4    # 32 x 4 (line grid: up to 2048 - 127 bytes)
    assert auto_shape(9000) == 6    # 64 x 4
    assert auto_shape(1500, True) == 8  # descriptors: 16 x 4 (verify: line grid, no prefetch)


def test_phy_policy_mirror():
    from smoltcp_amd.phy import Checksum, ChecksumCapabilities

    assert Checksum.Both.rx() and Checksum.Both.tx()
    assert Checksum.Rx.rx() and not Checksum.Rx.tx()
    assert Checksum.Tx.tx() and not Checksum.Tx.rx()
    assert not Checksum.None_.rx() and not Checksum.None_.tx()
    assert ChecksumCapabilities().as_tuple() == (0, 0, 0, 0, 0)
    assert ChecksumCapabilities.ignored().as_tuple() == (3, 3, 3, 3, 3)


def test_variant_lists():
    """The product library runs the defaults and one fallback per operation; the experiments build
    (when it has been built) every measured variant besides (csum_api.cpp variant_built)."""
    from smoltcp_amd import _lib

    L = _lib.lib()
    built = [v for v in range(-1, 128) if L.smol_csum_tool_variant_built(v)]
    assert built == [-1, 5, 7, 13, 17, 21, 39, 41, 44, 47, 57, 60, 63, 89, 97, 101], built
    if os.path.exists(_lib.EXP_LIB_PATH):
        X = _lib.lib(_lib.EXP_LIB_PATH)
        exp = {v for v in range(-1, 128) if X.smol_csum_tool_variant_built(v)}
        assert set(built) < exp and {0, 1, 3, 4, 16, 19, 23, 28, 29, 31, 37, 38, 42, 56, 80, 81, 82, 83, 64 + 37, 64 + 44, 64 + 47} <= exp


def test_dispatch_table_matches_sweeps():
    """smoltcp_amd/csrc/dispatch_table.inc (the fixed-stride dispatch, csum_api.cpp xwalk_auto) is what
    tools/gen_dispatch_table.py makes from the committed length sweeps (profiles/r06_dispatch_sweep_*),
    and C2's 1500-B records take the transposed walk with the first-load hint (verify) and with
    non-temporal write-through segments (emit, 101: the sweep's 57 with write-through stores)."""
    import subprocess

    from tests.dispatch_table import fixed_launch

    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_dispatch_table.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert fixed_launch("verify", 1500, 1500) == ("xwalk_kernel", 89)
    assert fixed_launch("emit", 1500, 1500) == ("xwalk_kernel", 101)
    assert fixed_launch("verify", 1000, 1000) == ("csum_kernel", 5)
