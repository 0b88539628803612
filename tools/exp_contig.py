#!/usr/bin/env python3
"""Experiment: does C5's span cost (the read stream over one 201-GB allocation runs 6.5 % slower than
over a 1.5-GB window of it) depend on how the allocation is mapped?  The same
buffer allocated with hipExtMallocWithFlags(hipDeviceMallocDefault) and with
hipDeviceMallocContiguous (physically contiguous: the driver can map it with its largest
fragments), then per allocation: the read-only stream probe over the whole buffer and over a
1.5-GB window, and C5's emit / verify (2^27 x 1500 B, the library's defaults).
Usage: exp_contig.py [GB]   (default 201)"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from smoltcp_amd import engine as E  # noqa: E402
from smoltcp_amd._lib import BatchC, check, lib  # noqa: E402


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 201.0
    L = 1500
    n = int(gb * 1e9) // L
    nbytes = n * L
    eng = E.ChecksumEngine(0)
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    L_ = lib()
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    status = torch.empty(n, dtype=torch.uint8, device="cuda")
    caps = E._caps(None)

    def batch(count):
        b = BatchC()
        b.desc, b.n, b.stride, b.len, b.kind, b.flags = None, count, L, L, E.KIND_IP, 0
        return b

    def timed(fn, reps):
        fn()
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        z.record()
        torch.cuda.synchronize()
        return a.elapsed_time(z) / reps

    for flags, name in ((0, "default"), (4, "contiguous"), (0, "default"), (4, "contiguous")):
        ptr = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(ptr), nbytes + 4096, flags)
        if rc != 0:
            print(json.dumps({"alloc": name, "GB": gb, "hip_error": rc}), flush=True)
            continue
        try:
            bf = batch(n)
            check(L_.smol_csum_tool_synth(eng._h, ptr, ctypes.byref(bf), E.SYNTH_UDP4, 5, sp), "synth")
            check(L_.smol_csum_batch_emit(eng._h, ptr, ctypes.byref(bf), ctypes.byref(caps), None, sp), "emit")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.3:  # clock ramp
                L_.smol_csum_tool_stream_read(eng._h, ptr, (1 << 20) * L, sink.data_ptr(), sp)
                torch.cuda.synchronize()
            win = (1 << 20) * L
            out = {"alloc": name, "GB": round(nbytes / 1e9, 1)}
            out["window_read_TBs"] = round(win / timed(
                lambda: L_.smol_csum_tool_stream_read(eng._h, ptr, win, sink.data_ptr(), sp), 20) / 1e9, 3)
            whole = nbytes // 16 * 16
            out["whole_read_TBs"] = round(whole / timed(
                lambda: L_.smol_csum_tool_stream_read(eng._h, ptr, whole, sink.data_ptr(), sp), 2) / 1e9, 3)
            per = n / (1 << 20)
            out["emit_ms_per_2^20"] = round(timed(
                lambda: L_.smol_csum_batch_emit(eng._h, ptr, ctypes.byref(bf), ctypes.byref(caps), None, sp), 2)
                / per, 4)
            out["verify_ms_per_2^20"] = round(timed(
                lambda: L_.smol_csum_batch_verify(eng._h, ptr, ctypes.byref(bf), ctypes.byref(caps),
                                                  ctypes.c_void_p(status.data_ptr()), sp), 2) / per, 4)
            print(json.dumps(out), flush=True)
        finally:
            torch.cuda.synchronize()
            hip.hipFree(ptr)


if __name__ == "__main__":
    main()
