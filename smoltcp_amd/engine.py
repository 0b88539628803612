"""Batched device checksum engine over torch device tensors (HBM-resident batches).

``ChecksumEngine`` wraps one ``smol_csum_ctx_t`` (include/smolcsum.h).  Buffers are plain
``torch.uint8`` CUDA(HIP) tensors holding packed records; ``Batch`` describes where the records
are — a fixed stride (no descriptor traffic) or a device array of 16-byte descriptors.  Every
call is asynchronous on the given stream (default: torch's current stream on the engine's
device).  PyTorch is only the allocator/stream provider here; all checksum work runs in the HIP
kernels of libsmolcsum.so.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from ._lib import BatchC, Caps, check, lib
from .phy import ChecksumCapabilities

KIND_RAW, KIND_IP, KIND_ETH = 0, 1, 2
REC_IPHDR_ONLY = 0x01  # SMOL_REC_IPHDR_ONLY: a raw socket's frame (the IP header's gate only)
BATCH_FIELD_STORES = 0x80  # SMOL_BATCH_FIELD_STORES: emit stores the checksum fields only (no whole segments)

ST_IP_OK = 0x01
ST_L4_OK = 0x02
ST_L4_PARTIAL = 0x04
ST_IP_VALID = 0x08
ST_L4_VALID = 0x10
ST_MALFORMED = 0x20
ST_UNSUPPORTED = 0x40
ST_ACCEPT = 0x80

SYNTH_UDP4, SYNTH_TCP4, SYNTH_V6MIX, SYNTH_ETH_TCP4, SYNTH_RANDOM = 0, 1, 2, 3, 4

DESC_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("kind", "u1"), ("flags", "u1"),
                       ("reserved", "<u2")])
assert DESC_DTYPE.itemsize == 16

# smol_csum_copy_t: one payload copy per record (smol_csum_batch_copy_emit)
COPY_DTYPE = np.dtype([("src_offset", "<u8"), ("dst_offset", "<u4"), ("len", "<u4")])
assert COPY_DTYPE.itemsize == 16


# smol_csum_frag_group_t: one IPv4 datagram = `count` consecutive records from `first`
FRAG_GROUP_DTYPE = np.dtype([("first", "<u8"), ("count", "<u4"), ("reserved", "<u4")])
assert FRAG_GROUP_DTYPE.itemsize == 16
MAX_FRAGMENTS = 256


def make_groups(firsts, counts) -> np.ndarray:
    """Host array of smol_csum_frag_group_t (view it as uint8 and copy it to the device)."""
    g = np.zeros(len(firsts), dtype=FRAG_GROUP_DTYPE)
    g["first"] = np.asarray(firsts, dtype=np.uint64)
    g["count"] = np.asarray(counts, dtype=np.uint32)
    return g


def make_copies(src_offsets, dst_offsets, lengths) -> np.ndarray:
    """Host array of smol_csum_copy_t (view it as uint8 and copy it to the device)."""
    n = len(src_offsets)
    c = np.zeros(n, dtype=COPY_DTYPE)
    c["src_offset"] = np.asarray(src_offsets, dtype=np.uint64)
    c["dst_offset"] = np.broadcast_to(np.asarray(dst_offsets, dtype=np.uint32), (n,))
    c["len"] = np.broadcast_to(np.asarray(lengths, dtype=np.uint32), (n,))
    return c


def make_descriptors(offsets, lengths, kinds, flags=0) -> np.ndarray:
    """Host array of smol_csum_desc_t (view it as uint8 and copy it to the device)."""
    n = len(offsets)
    d = np.zeros(n, dtype=DESC_DTYPE)
    d["offset"] = np.asarray(offsets, dtype=np.uint64)
    d["len"] = np.asarray(lengths, dtype=np.uint32)
    d["kind"] = np.broadcast_to(np.asarray(kinds, dtype=np.uint8), (n,))
    d["flags"] = np.broadcast_to(np.asarray(flags, dtype=np.uint8), (n,))
    return d


@dataclass
class Batch:
    """smol_csum_batch_t: ``desc`` is a device tensor of n*16 bytes, or None for a fixed stride."""

    n: int
    stride: int = 0
    length: int = 0
    kind: int = KIND_IP
    desc: Optional[object] = None  # torch.Tensor (uint8, device) holding n descriptors
    flags: int = 0                 # SMOL_REC_* of every record of a fixed-stride batch, | SMOL_BATCH_*

    def c(self) -> BatchC:
        b = BatchC()
        b.desc = self.desc.data_ptr() if self.desc is not None else None
        b.n = self.n
        b.stride = self.stride
        b.len = self.length
        b.kind = self.kind
        b.flags = self.flags
        return b

    @staticmethod
    def fixed(n: int, stride: int, length: Optional[int] = None, kind: int = KIND_IP, flags: int = 0) -> "Batch":
        return Batch(n=n, stride=stride, length=stride if length is None else length, kind=kind, flags=flags)

    @staticmethod
    def from_records(offsets, lengths, kinds, device, flags=0, batch_flags: int = 0) -> "Batch":
        """`flags`: SMOL_REC_* per record (descriptor flags); `batch_flags`: SMOL_BATCH_* of the batch."""
        import torch

        d = make_descriptors(offsets, lengths, kinds, flags)
        t = torch.from_numpy(d.view(np.uint8).copy()).to(device)
        return Batch(n=len(d), desc=t, flags=batch_flags)


def _caps(caps) -> Caps:
    if caps is None:
        caps = ChecksumCapabilities()
    tup = caps.as_tuple() if isinstance(caps, ChecksumCapabilities) else tuple(int(x) for x in caps)
    c = Caps()
    c.ipv4, c.udp, c.tcp, c.icmpv4, c.icmpv6 = tup
    return c


def segment_bitmap(addrs, nbytes: int):
    """The segment probe's bitmap for 2-byte fields at the byte offsets `addrs` (device int64 tensor) of
    an `nbytes` buffer: bit s set for every 64-B segment s holding a field byte, ceil(nbytes / 8192) * 4
    int32 words (whole 8-KiB pieces of 128 segments)."""
    import torch

    nseg = (nbytes + 8191) // 8192 * 128
    flags = torch.zeros(nseg, dtype=torch.int64, device=addrs.device)
    flags[addrs >> 6] = 1
    flags[(addrs + 1) >> 6] = 1
    words = (flags.view(-1, 32) << torch.arange(32, device=addrs.device, dtype=torch.int64)).sum(dim=1)
    words = torch.where(words >= 1 << 31, words - (1 << 32), words)
    return words.to(torch.int32).contiguous(), int(flags.sum().item())


class ChecksumEngine:
    """One device context.  Not thread-safe: use one engine per host thread."""

    def __init__(self, device: int = 0, lib_path: Optional[str] = None):
        """`lib_path`: another build of the library (the experiments build, `_lib.EXP_LIB_PATH`)."""
        self.device = int(device)
        self._L = lib(lib_path)
        h = ctypes.c_void_p()
        check(self._L.smol_csum_ctx_create(self.device, ctypes.byref(h)), "smol_csum_ctx_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.smol_csum_ctx_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- helpers ----
    def _stream(self, stream):
        import torch

        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        return ctypes.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream))

    @staticmethod
    def _check_buf(buf, batch: Batch):
        assert buf.is_cuda and buf.dtype.itemsize == 1, "buffer must be a uint8 device tensor"
        assert buf.is_contiguous()
        if batch.desc is None and batch.n:
            need = (batch.n - 1) * batch.stride + batch.length
            assert need <= buf.numel(), f"batch needs {need} bytes, buffer has {buf.numel()}"

    # ---- reference surface ----
    def data(self, buf, batch: Batch, out=None, stream=None):
        """out[i] = checksum::data(record i) (int16 tensor holding the u16 bit pattern)."""
        import torch

        self._check_buf(buf, batch)
        if out is None:
            out = torch.empty(batch.n, dtype=torch.int16, device=buf.device)
        b = batch.c()
        check(self._L.smol_csum_batch_data(self._h, buf.data_ptr(), ctypes.byref(b), out.data_ptr(),
                                         self._stream(stream)), "smol_csum_batch_data")
        return out

    def emit(self, buf, batch: Batch, caps=None, status=None, stream=None):
        """In-place fill (Repr::emit gates under ``caps``); returns ``status`` (may be None)."""
        self._check_buf(buf, batch)
        b = batch.c()
        c = _caps(caps)
        check(self._L.smol_csum_batch_emit(self._h, buf.data_ptr(), ctypes.byref(b), ctypes.byref(c),
                                         status.data_ptr() if status is not None else None,
                                         self._stream(stream)), "smol_csum_batch_emit")
        return status

    def copy_emit(self, buf, batch: Batch, src, copies, caps=None, status=None, stream=None):
        """Fused payload copy + emit (smol_csum_batch_copy_emit): ``copies`` is a device uint8
        tensor of n smol_csum_copy_t (see make_copies), ``src`` the payload source tensor."""
        self._check_buf(buf, batch)
        assert src.is_cuda and copies.is_cuda and copies.numel() >= 16 * batch.n
        b = batch.c()
        c = _caps(caps)
        check(self._L.smol_csum_batch_copy_emit(self._h, buf.data_ptr(), ctypes.byref(b), src.data_ptr(),
                                              copies.data_ptr(), ctypes.byref(c),
                                              status.data_ptr() if status is not None else None,
                                              self._stream(stream)), "smol_csum_batch_copy_emit")
        return status

    def emit_frag(self, buf, batch: Batch, groups, caps=None, status=None, stream=None):
        """IPv4 fragment groups (smol_csum_batch_emit_frag): ``groups`` is a device uint8 tensor of
        smol_csum_frag_group_t (see make_groups).  Fills every fragment's header and each
        datagram's L4 checksum; returns ``status`` (may be None)."""
        self._check_buf(buf, batch)
        assert groups.is_cuda and groups.numel() % 16 == 0
        b = batch.c()
        c = _caps(caps)
        check(self._L.smol_csum_batch_emit_frag(self._h, buf.data_ptr(), ctypes.byref(b), groups.data_ptr(),
                                              groups.numel() // 16, ctypes.byref(c),
                                              status.data_ptr() if status is not None else None,
                                              self._stream(stream)), "smol_csum_batch_emit_frag")
        return status

    def verify_frag(self, buf, batch: Batch, groups, caps=None, status=None, stream=None):
        """IPv4 fragment groups (smol_csum_batch_verify_frag): status bytes of every grouped record
        (records outside the groups keep their value; a fresh status tensor starts zeroed)."""
        import torch

        self._check_buf(buf, batch)
        assert groups.is_cuda and groups.numel() % 16 == 0
        if status is None:
            status = torch.zeros(batch.n, dtype=torch.uint8, device=buf.device)
        b = batch.c()
        c = _caps(caps)
        check(self._L.smol_csum_batch_verify_frag(self._h, buf.data_ptr(), ctypes.byref(b), groups.data_ptr(),
                                                groups.numel() // 16, ctypes.byref(c), status.data_ptr(),
                                                self._stream(stream)), "smol_csum_batch_verify_frag")
        return status

    def nhc_udp_emit(self, buf, batch: Batch, addrs, caps=None, status=None, stream=None):
        """6LoWPAN NHC UDP emit (smol_csum_batch_nhc_udp_emit): ``addrs`` is a device uint8 tensor of
        n x 32 bytes (IPv6 source, destination per record)."""
        self._check_buf(buf, batch)
        assert addrs.is_cuda and addrs.numel() >= 32 * batch.n
        b = batch.c()
        c = _caps(caps)
        check(self._L.smol_csum_batch_nhc_udp_emit(self._h, buf.data_ptr(), ctypes.byref(b), addrs.data_ptr(),
                                                 ctypes.byref(c), status.data_ptr() if status is not None else None,
                                                 self._stream(stream)), "smol_csum_batch_nhc_udp_emit")
        return status

    def nhc_udp_verify(self, buf, batch: Batch, addrs, caps=None, status=None, stream=None):
        """6LoWPAN NHC UDP parse gate (smol_csum_batch_nhc_udp_verify); returns the status tensor."""
        import torch

        self._check_buf(buf, batch)
        assert addrs.is_cuda and addrs.numel() >= 32 * batch.n
        if status is None:
            status = torch.empty(batch.n, dtype=torch.uint8, device=buf.device)
        b = batch.c()
        c = _caps(caps)
        check(self._L.smol_csum_batch_nhc_udp_verify(self._h, buf.data_ptr(), ctypes.byref(b), addrs.data_ptr(),
                                                   ctypes.byref(c), status.data_ptr(), self._stream(stream)),
              "smol_csum_batch_nhc_udp_verify")
        return status

    def verify(self, buf, batch: Batch, caps=None, status=None, stream=None):
        """status[i] = SMOL_ST_* bits (Repr::parse gates under ``caps``)."""
        import torch

        self._check_buf(buf, batch)
        if status is None:
            status = torch.empty(batch.n, dtype=torch.uint8, device=buf.device)
        b = batch.c()
        c = _caps(caps)
        check(self._L.smol_csum_batch_verify(self._h, buf.data_ptr(), ctypes.byref(b), ctypes.byref(c),
                                           status.data_ptr(), self._stream(stream)),
              "smol_csum_batch_verify")
        return status

    # ---- tooling ----
    def synth(self, buf, batch: Batch, profile: int, seed: int, stream=None):
        self._check_buf(buf, batch)
        b = batch.c()
        check(self._L.smol_csum_tool_synth(self._h, buf.data_ptr(), ctypes.byref(b), int(profile),
                                         int(seed) & (2**64 - 1), self._stream(stream)),
              "smol_csum_tool_synth")

    def corrupt(self, buf, batch: Batch, every: int, seed: int, stream=None):
        self._check_buf(buf, batch)
        b = batch.c()
        check(self._L.smol_csum_tool_corrupt(self._h, buf.data_ptr(), ctypes.byref(b), int(every),
                                           int(seed) & (2**64 - 1), self._stream(stream)),
              "smol_csum_tool_corrupt")

    def stream_read(self, buf, sink, stream=None):
        """Read-only HBM streaming probe over the whole buffer (tooling)."""
        nbytes = buf.numel() // 16 * 16
        check(self._L.smol_csum_tool_stream_read(self._h, buf.data_ptr(), nbytes, sink.data_ptr(),
                                               self._stream(stream)), "smol_csum_tool_stream_read")

    def field_probe(self, buf, stride: int, f1: int, f2: int = 0xFFFFFFFF, stream=None):
        """Emit's floor probe (tooling, smol_csum_tool_field_probe): stream-read the buffer and store
        2 bytes at offsets f1 / f2 of every `stride`-byte record.  Overwrites those bytes."""
        nbytes = buf.numel() // 16 * 16
        check(self._L.smol_csum_tool_field_probe(self._h, buf.data_ptr(), nbytes, int(stride), int(f1), int(f2),
                                               self._stream(stream)), "smol_csum_tool_field_probe")

    def field_probe_list(self, buf, addrs, piece_first, seg64: bool = False, stream=None):
        """Emit's floor probe with listed store addresses (tooling, smol_csum_tool_field_probe_list):
        `addrs` a device u64 tensor of ascending byte offsets, `piece_first` a device u32 tensor with
        the index of the first address at or after each 8-KiB piece (ceil(bytes / 8192) + 1
        entries).  Overwrites the bytes at those offsets; with `seg64` rewrites the 64-B segments
        holding them whole, with their own values, instead."""
        nbytes = buf.numel() // 16 * 16
        check(self._L.smol_csum_tool_field_probe_list(self._h, buf.data_ptr(), nbytes, addrs.data_ptr(),
                                                    piece_first.data_ptr(), int(bool(seg64)),
                                                    self._stream(stream)),
              "smol_csum_tool_field_probe_list")

    def segment_probe(self, buf, bitmap, nt: bool = False, stream=None):
        """Emit's floor in its store shape (tooling, smol_csum_tool_segment_probe): the read stream over
        `buf` plus every 64-B segment whose bit is set in `bitmap` (device int32 tensor, one bit per
        segment, see segment_bitmap) rewritten whole with its own bytes; `nt`: non-temporal stores."""
        nbytes = buf.numel() // 16 * 16
        check(self._L.smol_csum_tool_segment_probe(self._h, buf.data_ptr(), nbytes, bitmap.data_ptr(), int(bool(nt)),
                                                 self._stream(stream)),
              "smol_csum_tool_segment_probe")

    def field_scatter(self, buf, addrs, vals, nt: int = 0, stream=None):
        """A separate store pass (tooling, smol_csum_tool_field_scatter): the big-endian u16 `vals[i]`
        at byte offset `addrs[i]` (device int64 / uint16-as-int16 tensors) of `buf`.  `nt`: the flags
        (bit 0 non-temporal stores; bits 1 / 2 / 3 the whole 64-B segment / 32-B sector / 128-B line
        instead)."""
        check(self._L.smol_csum_tool_field_scatter(self._h, buf.data_ptr(), buf.numel(), addrs.data_ptr(),
                                                 vals.data_ptr(), int(addrs.numel()), int(nt),
                                                 self._stream(stream)), "smol_csum_tool_field_scatter")

    def set_shape(self, shape: int):
        check(self._L.smol_csum_tool_set_shape(self._h, int(shape)), "smol_csum_tool_set_shape")

    def set_variant(self, variant: int):
        check(self._L.smol_csum_tool_set_variant(self._h, int(variant)), "smol_csum_tool_set_variant")

    def set_tile(self, records: int):
        check(self._L.smol_csum_tool_set_tile(self._h, int(records)), "smol_csum_tool_set_tile")

    def kernel_name(self, op: str, has_desc: bool = False) -> str:
        """Deprecated: the kernel an IP-path `op` launches for a batch of short records (no record
        length is passed; see kernel_for)."""
        code = {"data": 0, "emit": 1, "verify": 2, "copy_emit": 3}[op]
        return self._L.smol_csum_tool_kernel_name(self._h, code, int(bool(has_desc))).decode()

    def kernel_for(self, op: str, batch: Batch) -> str:
        """The kernel (rocprofv3 name prefix) an IP-path `op` ("data", "emit", "verify", "copy_emit")
        launches for `batch` with this engine's settings: the library's own dispatch decision."""
        code = {"data": 0, "emit": 1, "verify": 2, "copy_emit": 3}[op]
        b = batch.c()
        return self._L.smol_csum_tool_kernel_for(self._h, code, ctypes.byref(b)).decode()

    def variant_built(self, variant: int) -> bool:
        """Whether this build of the library runs `variant` (the product library: the defaults and
        one fallback per operation; the experiments build: every measured variant)."""
        return bool(self._L.smol_csum_tool_variant_built(int(variant)))

    def last_launch(self) -> dict:
        """The kernel instantiation of the process's last checksum launch: {"kernel": "csum_kernel" |
        "csum_tile_kernel" | "copy_kernel" | "csum_kernel_nhc" | "xwalk_kernel" | "dwalk_kernel", "variant": VAR, "G":
        lanes per record, "U": chunks per lane per step (xwalk_kernel: 1-KiB loads per record)} (None
        before the first launch)."""
        w = int(self._L.smol_csum_tool_last_launch())
        names = {1: "csum_kernel", 2: "csum_tile_kernel", 3: "copy_kernel", 4: "csum_kernel_nhc", 5: "xwalk_kernel",
                 6: "dwalk_kernel"}
        if not w >> 24:
            return None
        return {"kernel": names.get(w >> 24, "?"), "variant": (w >> 16) & 0xff, "G": (w >> 8) & 0xff, "U": w & 0xff}

    def set_xcd_remap(self, on: int):
        """1 / 0: force the XCD-contiguous block order on / off; K >= 2: runs of K workgroups per XCD
        turn; -1: the library's choice."""
        check(self._L.smol_csum_tool_set_xcd_remap(self._h, int(on)), "smol_csum_tool_set_xcd_remap")

    def set_launch_records(self, records: int):
        check(self._L.smol_csum_tool_set_launch_records(self._h, int(records)), "smol_csum_tool_set_launch_records")

    def set_max_blocks(self, max_blocks: int):
        check(self._L.smol_csum_tool_set_max_blocks(self._h, int(max_blocks)),
              "smol_csum_tool_set_max_blocks")


def auto_shape(length: int, has_desc: bool = False) -> int:
    return int(_lib.lib().smol_csum_tool_auto_shape(int(length), int(bool(has_desc))))
