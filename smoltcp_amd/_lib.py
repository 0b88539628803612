"""ctypes binding of libsmolcsum.so (the C ABI declared in include/smolcsum.h).

The shared library is built in-tree (``smoltcp_amd/libsmolcsum.so``, see ``__graft_entry__.build``)
and travels with the repository snapshot to the GPU box.  There is no fallback: if the library is
missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SMOLCSUM_LIB: an alternative build of the same library (A/B experiments only)
LIB_PATH = os.environ.get("SMOLCSUM_LIB") or os.path.join(_HERE, "libsmolcsum.so")
# The experiments build (`make -C smoltcp_amd/csrc EXP=1`): the product library plus the measured
# kernel variants that are not defaults (tools/ and the variant tests load it when it exists).
EXP_LIB_PATH = os.path.join(_HERE, "libsmolcsum_exp.so")

SMOL_OK, SMOL_EINVAL, SMOL_ENODEV, SMOL_EHIP, SMOL_ERANGE, SMOL_ENOMEM = 0, -1, -2, -3, -4, -5
ERROR_NAMES = {
    SMOL_EINVAL: "SMOL_EINVAL",
    SMOL_ENODEV: "SMOL_ENODEV",
    SMOL_EHIP: "SMOL_EHIP",
    SMOL_ERANGE: "SMOL_ERANGE",
    SMOL_ENOMEM: "SMOL_ENOMEM",
}

# Every symbol include/smolcsum.h and include/smolcsum_tools.h declare.
ABI_SYMBOLS = [
    "smol_csum_data", "smol_csum_combine", "smol_csum_pseudo_header_v4",
    "smol_csum_pseudo_header_v6", "smol_csum_pseudo_header", "smol_csum_ctx_create",
    "smol_csum_ctx_destroy", "smol_csum_batch_data", "smol_csum_batch_emit",
    "smol_csum_batch_verify", "smol_csum_batch_copy_emit", "smol_csum_batch_emit_frag",
    "smol_csum_batch_verify_frag", "smol_csum_batch_nhc_udp_emit",
    "smol_csum_batch_nhc_udp_verify", "smol_csum_last_error", "smol_csum_abi_version",
]
TOOL_SYMBOLS = [
    "smol_csum_tool_synth", "smol_csum_tool_corrupt", "smol_csum_tool_set_shape",
    "smol_csum_tool_set_variant", "smol_csum_tool_set_tile",
    "smol_csum_tool_set_max_blocks", "smol_csum_tool_auto_shape", "smol_csum_tool_stream_read",
    "smol_csum_tool_set_xcd_remap", "smol_csum_tool_set_launch_records",
    "smol_csum_tool_field_probe",
    "smol_csum_tool_field_probe_list", "smol_csum_tool_segment_probe", "smol_csum_tool_field_scatter",
    "smol_csum_tool_variant_built",
    "smol_csum_tool_kernel_name", "smol_csum_tool_kernel_for", "smol_csum_tool_last_launch",
]
# Tool symbols added in later rounds: bound only when the loaded build has them (SMOLCSUM_LIB may name
# an older build for an A/B run), and a call to a missing one raises AttributeError naming it.
OPTIONAL_TOOL_SYMBOLS = ("smol_csum_tool_variant_built", "smol_csum_tool_kernel_for", "smol_csum_tool_segment_probe")


class SmolError(RuntimeError):
    def __init__(self, rc: int, what: str, detail: str = ""):
        name = ERROR_NAMES.get(rc, str(rc))
        super().__init__(f"{what} failed: {name}" + (f" ({detail})" if detail else ""))
        self.rc = rc


class Caps(ctypes.Structure):
    """smol_checksum_caps_t — phy::ChecksumCapabilities {ipv4, udp, tcp, icmpv4, icmpv6}."""

    _fields_ = [
        ("ipv4", ctypes.c_uint8),
        ("udp", ctypes.c_uint8),
        ("tcp", ctypes.c_uint8),
        ("icmpv4", ctypes.c_uint8),
        ("icmpv6", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8 * 3),
    ]


class BatchC(ctypes.Structure):
    """smol_csum_batch_t."""

    _fields_ = [
        ("desc", ctypes.c_void_p),
        ("n", ctypes.c_uint64),
        ("stride", ctypes.c_uint64),
        ("len", ctypes.c_uint32),
        ("kind", ctypes.c_uint8),
        ("flags", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8 * 2),
    ]


_LIBS = {}


def lib(path: str | None = None) -> ctypes.CDLL:
    """Load libsmolcsum.so, or the build at `path` (raises if it is absent: there is no CPU
    fallback)."""
    path = path or LIB_PATH
    if path in _LIBS:
        return _LIBS[path]
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    L = ctypes.CDLL(path)
    vp, u8, u16, u32, u64 = ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64
    sz, i32 = ctypes.c_size_t, ctypes.c_int
    L.smol_csum_data.argtypes = [vp, sz]
    L.smol_csum_data.restype = u16
    L.smol_csum_combine.argtypes = [vp, sz]
    L.smol_csum_combine.restype = u16
    L.smol_csum_pseudo_header_v4.argtypes = [vp, vp, u8, u32]
    L.smol_csum_pseudo_header_v4.restype = u16
    L.smol_csum_pseudo_header_v6.argtypes = [vp, vp, u8, u32]
    L.smol_csum_pseudo_header_v6.restype = u16
    L.smol_csum_pseudo_header.argtypes = [i32, vp, i32, vp, u8, u32, ctypes.POINTER(u16)]
    L.smol_csum_pseudo_header.restype = i32
    L.smol_csum_ctx_create.argtypes = [i32, ctypes.POINTER(vp)]
    L.smol_csum_ctx_create.restype = i32
    L.smol_csum_ctx_destroy.argtypes = [vp]
    L.smol_csum_ctx_destroy.restype = i32
    L.smol_csum_batch_data.argtypes = [vp, vp, ctypes.POINTER(BatchC), vp, vp]
    L.smol_csum_batch_data.restype = i32
    L.smol_csum_batch_emit.argtypes = [vp, vp, ctypes.POINTER(BatchC), ctypes.POINTER(Caps), vp, vp]
    L.smol_csum_batch_emit.restype = i32
    L.smol_csum_batch_verify.argtypes = [vp, vp, ctypes.POINTER(BatchC), ctypes.POINTER(Caps), vp, vp]
    L.smol_csum_batch_verify.restype = i32
    L.smol_csum_batch_copy_emit.argtypes = [vp, vp, ctypes.POINTER(BatchC), vp, vp, ctypes.POINTER(Caps), vp, vp]
    L.smol_csum_batch_copy_emit.restype = i32
    for name in ("smol_csum_batch_emit_frag", "smol_csum_batch_verify_frag"):
        f = getattr(L, name)
        f.argtypes = [vp, vp, ctypes.POINTER(BatchC), vp, u64, ctypes.POINTER(Caps), vp, vp]
        f.restype = i32
    for name in ("smol_csum_batch_nhc_udp_emit", "smol_csum_batch_nhc_udp_verify"):
        f = getattr(L, name)
        f.argtypes = [vp, vp, ctypes.POINTER(BatchC), vp, ctypes.POINTER(Caps), vp, vp]
        f.restype = i32
    L.smol_csum_last_error.argtypes = []
    L.smol_csum_last_error.restype = ctypes.c_char_p
    L.smol_csum_abi_version.argtypes = []
    L.smol_csum_abi_version.restype = i32
    L.smol_csum_tool_synth.argtypes = [vp, vp, ctypes.POINTER(BatchC), i32, u64, vp]
    L.smol_csum_tool_synth.restype = i32
    L.smol_csum_tool_corrupt.argtypes = [vp, vp, ctypes.POINTER(BatchC), u32, u64, vp]
    L.smol_csum_tool_corrupt.restype = i32
    L.smol_csum_tool_set_shape.argtypes = [vp, i32]
    L.smol_csum_tool_set_shape.restype = i32
    L.smol_csum_tool_set_variant.argtypes = [vp, i32]
    L.smol_csum_tool_set_variant.restype = i32
    L.smol_csum_tool_set_tile.argtypes = [vp, i32]
    L.smol_csum_tool_set_tile.restype = i32
    L.smol_csum_tool_set_max_blocks.argtypes = [vp, u32]
    L.smol_csum_tool_set_max_blocks.restype = i32
    L.smol_csum_tool_set_xcd_remap.argtypes = [vp, ctypes.c_int]
    L.smol_csum_tool_set_xcd_remap.restype = i32
    L.smol_csum_tool_set_launch_records.argtypes = [vp, u64]
    L.smol_csum_tool_set_launch_records.restype = i32
    L.smol_csum_tool_stream_read.argtypes = [vp, vp, u64, vp, vp]
    L.smol_csum_tool_stream_read.restype = i32
    L.smol_csum_tool_field_probe.argtypes = [vp, vp, u64, u64, ctypes.c_uint32, ctypes.c_uint32, vp]
    L.smol_csum_tool_field_probe.restype = i32
    L.smol_csum_tool_field_probe_list.argtypes = [vp, vp, u64, vp, vp, ctypes.c_int, vp]
    L.smol_csum_tool_field_probe_list.restype = i32
    L.smol_csum_tool_field_scatter.argtypes = [vp, vp, u64, vp, vp, u64, ctypes.c_int, vp]
    L.smol_csum_tool_field_scatter.restype = i32
    L.smol_csum_tool_auto_shape.argtypes = [u32, i32]
    L.smol_csum_tool_auto_shape.restype = i32
    L.smol_csum_tool_kernel_name.argtypes = [vp, i32, i32]
    L.smol_csum_tool_kernel_name.restype = ctypes.c_char_p
    L.smol_csum_tool_last_launch.argtypes = []
    L.smol_csum_tool_last_launch.restype = u32
    if hasattr(L, "smol_csum_tool_variant_built"):
        L.smol_csum_tool_variant_built.argtypes = [i32]
        L.smol_csum_tool_variant_built.restype = i32
    if hasattr(L, "smol_csum_tool_segment_probe"):
        L.smol_csum_tool_segment_probe.argtypes = [vp, vp, u64, vp, ctypes.c_int, vp]
        L.smol_csum_tool_segment_probe.restype = i32
    if hasattr(L, "smol_csum_tool_kernel_for"):
        L.smol_csum_tool_kernel_for.argtypes = [vp, i32, vp]
        L.smol_csum_tool_kernel_for.restype = ctypes.c_char_p
    _LIBS[path] = L
    return L


def check(rc: int, what: str, L: ctypes.CDLL | None = None) -> None:
    if rc != SMOL_OK:
        detail = (L or lib()).smol_csum_last_error().decode(errors="replace") if rc == SMOL_EHIP else ""
        raise SmolError(rc, what, detail)
