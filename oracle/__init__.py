"""CPU ORACLE — test infrastructure only.

Two independent restatements of smoltcp 0.13.1's Internet checksum:

* ``pyref`` — pure-Python loops over ``src/wire/ip.rs:762-869`` (small inputs only), used to
  cross-check the C restatement and to generate golden vectors;
* ``lib()`` — ctypes handle to ``liboracle.so`` built from ``csum_oracle.c`` (the per-protocol
  gates and the record/batch contract of ``include/smolcsum.h``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker or the timed CPU baseline.  The product
(``smoltcp_amd``) never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from . import pyref  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class CapsC(ctypes.Structure):
    """smol_checksum_caps_t (include/smolcsum.h)."""

    _fields_ = [
        ("ipv4", ctypes.c_uint8),
        ("udp", ctypes.c_uint8),
        ("tcp", ctypes.c_uint8),
        ("icmpv4", ctypes.c_uint8),
        ("icmpv6", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8 * 3),
    ]


def build() -> str:
    """Compile liboracle.so with the committed Makefile; returns its path."""
    import fcntl

    with open(os.path.join(_HERE, ".make.lock"), "w") as lk:  # one make at a time (pytest-xdist workers)
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "liboracle.so")


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    path = os.path.join(_HERE, "liboracle.so")
    if not os.path.exists(path):
        build()
    _LIB = _bind(ctypes.CDLL(path))
    return _LIB


NATIVE_CC = "/opt/rocm/lib/llvm/bin/clang"


def use_native() -> str:
    """bench.py's cpu_baseline: rebuild this restatement for the host it runs on (ROCm clang -O3
    -march=native) into a temporary directory and use it from now on.  Falls back
    to the committed recipe's build (gcc -O3 -march=x86-64-v3) if the compiler is missing.
    Returns a description of the build in use."""
    global _LIB
    import tempfile

    out = os.path.join(tempfile.mkdtemp(prefix="smol_oracle_"), "liboracle_native.so")
    cmd = [NATIVE_CC, "-O3", "-march=native", "-fPIC", "-shared", "-std=c11", "-o", out,
           os.path.join(_HERE, "csum_oracle.c")]
    try:
        subprocess.run(cmd, check=True, capture_output=True, timeout=120)
        _LIB = _bind(ctypes.CDLL(out))
        return "with ROCm clang -O3 -march=native on this host"
    except (OSError, subprocess.SubprocessError):
        lib()
        return "with gcc -O3 -march=x86-64-v3 (oracle/Makefile; ROCm clang unavailable)"


def _bind(L: ctypes.CDLL) -> ctypes.CDLL:
    u8p = ctypes.c_void_p
    L.oracle_data.argtypes = [u8p, ctypes.c_size_t]
    L.oracle_data.restype = ctypes.c_uint16
    L.oracle_combine.argtypes = [u8p, ctypes.c_size_t]
    L.oracle_combine.restype = ctypes.c_uint16
    for name in ("oracle_pseudo_v4", "oracle_pseudo_v6"):
        f = getattr(L, name)
        f.argtypes = [u8p, u8p, ctypes.c_uint8, ctypes.c_uint32]
        f.restype = ctypes.c_uint16
    L.oracle_ipv4_verify.argtypes = [u8p]
    L.oracle_ipv4_verify.restype = ctypes.c_int
    L.oracle_ipv4_fill.argtypes = [u8p]
    L.oracle_ipv4_fill.restype = None
    for name in ("oracle_udp_verify", "oracle_udp_verify_partial"):
        f = getattr(L, name)
        f.argtypes = [u8p, ctypes.c_int, u8p, u8p]
        f.restype = ctypes.c_int
    L.oracle_udp_fill.argtypes = [u8p, ctypes.c_int, u8p, u8p]
    L.oracle_udp_fill.restype = None
    for name in ("oracle_tcp_verify", "oracle_tcp_verify_partial"):
        f = getattr(L, name)
        f.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, u8p, u8p]
        f.restype = ctypes.c_int
    L.oracle_tcp_fill.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, u8p, u8p]
    L.oracle_tcp_fill.restype = None
    for name in ("oracle_icmpv4_verify", "oracle_igmp_verify"):
        f = getattr(L, name)
        f.argtypes = [u8p, ctypes.c_size_t]
        f.restype = ctypes.c_int
    for name in ("oracle_icmpv4_fill", "oracle_igmp_fill"):
        f = getattr(L, name)
        f.argtypes = [u8p, ctypes.c_size_t]
        f.restype = None
    L.oracle_icmpv6_verify.argtypes = [u8p, ctypes.c_size_t, u8p, u8p]
    L.oracle_icmpv6_verify.restype = ctypes.c_int
    L.oracle_icmpv6_fill.argtypes = [u8p, ctypes.c_size_t, u8p, u8p]
    L.oracle_icmpv6_fill.restype = None
    L.oracle_icmpv6_min_len.argtypes = [ctypes.c_uint8]
    L.oracle_icmpv6_min_len.restype = ctypes.c_size_t
    L.oracle_hbh_options_drop.argtypes = [u8p, ctypes.c_size_t]
    L.oracle_hbh_options_drop.restype = ctypes.c_int
    L.oracle_record_verify.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(CapsC)]
    L.oracle_record_verify.restype = ctypes.c_uint8
    L.oracle_record_emit.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(CapsC)]
    L.oracle_record_emit.restype = ctypes.c_uint8
    L.oracle_batch_data.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, u8p]
    L.oracle_batch_data.restype = None
    L.oracle_batch_emit.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                    ctypes.c_uint32, ctypes.POINTER(CapsC), u8p]
    L.oracle_batch_emit.restype = None
    L.oracle_batch_verify.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.POINTER(CapsC), u8p]
    L.oracle_batch_verify.restype = None
    L.oracle_batch_copy_emit.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.POINTER(CapsC), u8p, u8p, u8p]
    L.oracle_batch_copy_emit.restype = None
    L.oracle_nhc_udp_verify.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.POINTER(CapsC)]
    L.oracle_nhc_udp_verify.restype = ctypes.c_uint8
    L.oracle_nhc_udp_emit.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.POINTER(CapsC)]
    L.oracle_nhc_udp_emit.restype = ctypes.c_uint8
    for name in ("oracle_batch_emit_frag", "oracle_batch_verify_frag"):
        f = getattr(L, name)
        f.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, u8p,
                      ctypes.c_uint64, ctypes.POINTER(CapsC), u8p]
        f.restype = None
    for name in ("oracle_batch_nhc_udp_emit", "oracle_batch_nhc_udp_verify"):
        f = getattr(L, name)
        f.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, u8p,
                      ctypes.POINTER(CapsC), u8p]
        f.restype = None
    L.oracle_emit_like_dispatch_ip.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(CapsC)]
    L.oracle_emit_like_dispatch_ip.restype = ctypes.c_int
    return L


# SMOL_REC_IPHDR_ONLY (include/smolcsum.h): a raw-socket record; the oracle's batch functions take
# a record's flags in bits 8..15 of `kind` (descriptor batches: smol_csum_desc_t.flags).
REC_IPHDR_ONLY = 0x01


def kind_flags(kind: int, flags: int = 0) -> int:
    return int(kind) | (int(flags) << 8)


def emit_like_dispatch_ip(frag_buffer: np.ndarray, caps=(0, 0, 0, 0, 0)) -> int:
    """The reference's own route for a datagram it fragments (csum_oracle.c): the L4 checksum filled
    over frag.buffer[hl..] (the datagram's L4 bytes + the stale tail), in place.  Returns 0, -1
    (dropped / not IPv4) or -2 (the reference panics)."""
    c = caps_c(caps)
    return int(lib().oracle_emit_like_dispatch_ip(_ptr(frag_buffer), frag_buffer.size, ctypes.byref(c)))


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def caps_c(caps=(0, 0, 0, 0, 0)) -> CapsC:
    c = CapsC()
    c.ipv4, c.udp, c.tcp, c.icmpv4, c.icmpv6 = (int(x) for x in caps)
    return c


# ---- thin numpy wrappers ------------------------------------------------------------------


def data(b) -> int:
    a = np.frombuffer(bytes(b), dtype=np.uint8)
    return int(lib().oracle_data(_ptr(a) if a.size else None, a.size))


def batch_data(buf: np.ndarray, desc: np.ndarray | None, n: int, stride: int = 0, length: int = 0):
    out = np.zeros(n, dtype=np.uint16)
    lib().oracle_batch_data(_ptr(buf), _ptr(desc) if desc is not None else None, n, stride, length,
                            _ptr(out))
    return out


def batch_emit(buf: np.ndarray, desc, n: int, stride: int = 0, length: int = 0, kind: int = 1,
               caps=(0, 0, 0, 0, 0)):
    """In place on ``buf`` (host numpy uint8); returns the status array."""
    st = np.zeros(n, dtype=np.uint8)
    c = caps_c(caps)
    lib().oracle_batch_emit(_ptr(buf), _ptr(desc) if desc is not None else None, n, stride, length,
                            kind, ctypes.byref(c), _ptr(st))
    return st


COPY_DTYPE = np.dtype([("src_offset", "<u8"), ("dst_offset", "<u4"), ("len", "<u4")])


def batch_copy_emit(buf: np.ndarray, desc, n: int, src: np.ndarray, copy: np.ndarray, stride: int = 0,
                    length: int = 0, kind: int = 1, caps=(0, 0, 0, 0, 0)):
    """memcpy of each record's payload from ``src`` (``copy``: COPY_DTYPE array), then the record
    emit; in place on ``buf``.  Returns the status array."""
    st = np.zeros(n, dtype=np.uint8)
    c = caps_c(caps)
    copy = np.ascontiguousarray(copy, dtype=COPY_DTYPE)
    lib().oracle_batch_copy_emit(_ptr(buf), _ptr(desc) if desc is not None else None, n, stride, length,
                                 kind, ctypes.byref(c), _ptr(src) if src.size else None, _ptr(copy), _ptr(st))
    return st


def batch_verify(buf: np.ndarray, desc, n: int, stride: int = 0, length: int = 0, kind: int = 1,
                 caps=(0, 0, 0, 0, 0)):
    st = np.zeros(n, dtype=np.uint8)
    c = caps_c(caps)
    lib().oracle_batch_verify(_ptr(buf), _ptr(desc) if desc is not None else None, n, stride,
                              length, kind, ctypes.byref(c), _ptr(st))
    return st


FRAG_GROUP_DTYPE = np.dtype([("first", "<u8"), ("count", "<u4"), ("reserved", "<u4")])


def batch_emit_frag(buf: np.ndarray, desc, n: int, groups: np.ndarray, stride: int = 0, length: int = 0,
                    kind: int = 1, caps=(0, 0, 0, 0, 0)):
    """IPv4 fragment groups, emit (see csum_oracle.c): in place on ``buf``; returns the status
    array (records outside the groups: 0)."""
    st = np.zeros(n, dtype=np.uint8)
    c = caps_c(caps)
    g = np.ascontiguousarray(groups, dtype=FRAG_GROUP_DTYPE)
    lib().oracle_batch_emit_frag(_ptr(buf), _ptr(desc) if desc is not None else None, n, stride, length, kind,
                                 _ptr(g) if g.size else None, g.size, ctypes.byref(c), _ptr(st))
    return st


def batch_verify_frag(buf: np.ndarray, desc, n: int, groups: np.ndarray, stride: int = 0, length: int = 0,
                      kind: int = 1, caps=(0, 0, 0, 0, 0)):
    """IPv4 fragment groups, verify; returns the status array (records outside the groups: 0)."""
    st = np.zeros(n, dtype=np.uint8)
    c = caps_c(caps)
    g = np.ascontiguousarray(groups, dtype=FRAG_GROUP_DTYPE)
    lib().oracle_batch_verify_frag(_ptr(buf), _ptr(desc) if desc is not None else None, n, stride, length, kind,
                                   _ptr(g) if g.size else None, g.size, ctypes.byref(c), _ptr(st))
    return st


def batch_nhc_udp_emit(buf: np.ndarray, desc, n: int, addrs: np.ndarray, stride: int = 0, length: int = 0,
                       caps=(0, 0, 0, 0, 0)):
    """6LoWPAN NHC UDP emit (nhc.rs:746-776) in place on ``buf``; ``addrs``: n x 32 bytes (src, dst).
    Returns the status array."""
    st = np.zeros(n, dtype=np.uint8)
    c = caps_c(caps)
    addrs = np.ascontiguousarray(addrs, dtype=np.uint8)
    assert addrs.size >= 32 * n
    lib().oracle_batch_nhc_udp_emit(_ptr(buf), _ptr(desc) if desc is not None else None, n, stride, length,
                                    _ptr(addrs), ctypes.byref(c), _ptr(st))
    return st


def batch_nhc_udp_verify(buf: np.ndarray, desc, n: int, addrs: np.ndarray, stride: int = 0, length: int = 0,
                         caps=(0, 0, 0, 0, 0)):
    """6LoWPAN NHC UDP parse gate (nhc.rs:693-729); returns the status array."""
    st = np.zeros(n, dtype=np.uint8)
    c = caps_c(caps)
    addrs = np.ascontiguousarray(addrs, dtype=np.uint8)
    assert addrs.size >= 32 * n
    lib().oracle_batch_nhc_udp_verify(_ptr(buf), _ptr(desc) if desc is not None else None, n, stride, length,
                                      _ptr(addrs), ctypes.byref(c), _ptr(st))
    return st
