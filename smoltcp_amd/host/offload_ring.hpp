// offload_ring.hpp — pinned host ring + HBM staging for a checksum-offloading phy::Device.
//
// The C++ form of the `Mi355xOffload` wrapper sketched in INTEGRATION.md §4: frames live in a
// pinned host ring of `slots` fixed-size slots (like the reference's Loopback / QueueDevice
// rings, src/phy/loopback.rs, tests/netsim.rs:549-555); `emit(n)` and `verify(n)` move a burst
// through the GPU in chunks, pipelined over three HIP streams (H2D / checksum / D2H) with two
// device chunk buffers:
//
//   emit:   H2D(frames) -> smol_csum_batch_emit   -> D2H(frames)       (TxToken::consume)
//   verify: H2D(frames) -> smol_csum_batch_verify -> D2H(status bytes) (before an RxToken)
//
// Frames a raw socket produced are marked with mark_raw(): their L4 bytes are the user's
// (src/iface/packet.rs:132-136, src/socket/raw.rs:406-423), so a chunk holding one goes to the
// device with a descriptor array whose flags carry SMOL_REC_IPHDR_ONLY for those slots (the IPv4
// header is emitted, the L4 bytes are left alone); other chunks stay fixed-stride batches.
//
// Header-only; needs the HIP runtime (hip/hip_runtime_api.h, -lamdhip64) and libsmolcsum.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstring>
#include <string>

#include "smoltcp_checksum.hpp"

namespace smoltcp_amd {

inline void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw Error(SMOL_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

class OffloadRing {
public:
    OffloadRing(int device, uint32_t slots, uint32_t slot_bytes, Medium medium = Medium::Ethernet,
                uint32_t chunk = 65536)
        : eng_(device), slots_(slots), slot_(slot_bytes), chunk_(chunk < slots ? chunk : slots), medium_(medium) {
        hip_check(hipSetDevice(device), "hipSetDevice");
        hip_check(hipHostMalloc(reinterpret_cast<void**>(&host_), size_t(slots_) * slot_, hipHostMallocDefault),
                  "hipHostMalloc(ring)");
        hip_check(hipHostMalloc(reinterpret_cast<void**>(&status_), slots_, hipHostMallocDefault),
                  "hipHostMalloc(status)");
        hip_check(hipHostMalloc(reinterpret_cast<void**>(&raw_), slots_, hipHostMallocDefault), "hipHostMalloc(raw)");
        std::memset(raw_, 0, slots_);
        for (int k = 0; k < 2; ++k) {
            hip_check(hipMalloc(&dbuf_[k], size_t(chunk_) * slot_), "hipMalloc(chunk)");
            hip_check(hipMalloc(&dst_[k], chunk_), "hipMalloc(status)");
            hip_check(hipMalloc(reinterpret_cast<void**>(&ddesc_[k]), size_t(chunk_) * sizeof(smol_csum_desc_t)),
                      "hipMalloc(desc)");
            hip_check(hipHostMalloc(reinterpret_cast<void**>(&hdesc_[k]), size_t(chunk_) * sizeof(smol_csum_desc_t),
                                    hipHostMallocDefault), "hipHostMalloc(desc)");
        }
        for (auto& s : s_) hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    }
    ~OffloadRing() {
        for (auto& s : s_) (void)hipStreamDestroy(s);
        for (int k = 0; k < 2; ++k) {
            (void)hipFree(dbuf_[k]);
            (void)hipFree(dst_[k]);
            (void)hipFree(ddesc_[k]);
            (void)hipHostFree(hdesc_[k]);
        }
        (void)hipHostFree(host_);
        (void)hipHostFree(status_);
        (void)hipHostFree(raw_);
    }
    OffloadRing(const OffloadRing&) = delete;
    OffloadRing& operator=(const OffloadRing&) = delete;

    uint8_t* slot(uint32_t i) { return host_ + size_t(i) * slot_; }
    const uint8_t* status() const { return status_; }
    uint32_t slots() const { return slots_; }
    uint32_t slot_bytes() const { return slot_; }

    // Slot i holds a raw socket's frame (true) or a frame the stack built (false, the default).
    void mark_raw(uint32_t i, bool raw = true) {
        if (i >= slots_) throw Error(SMOL_ERANGE, "slot out of range");
        raw_[i] = raw ? 1 : 0;
    }

    // Fill the checksums of frames [0, n) in place (caps: the stack's, default Checksum::Both).
    void emit(uint32_t n, const smoltcp::phy::ChecksumCapabilities& caps = {}) { run(n, true, caps); }

    // status()[i] = SMOL_ST_* of frame i, for i < n.
    void verify(uint32_t n, const smoltcp::phy::ChecksumCapabilities& caps = {}) { run(n, false, caps); }

private:
    void run(uint32_t n, bool emit, const smoltcp::phy::ChecksumCapabilities& caps) {
        if (n > slots_) throw Error(SMOL_ERANGE, "burst larger than the ring");
        const uint32_t nch = (n + chunk_ - 1) / chunk_;
        hipEvent_t ev[3][2];
        for (auto& e : ev)
            for (auto& x : e) hip_check(hipEventCreateWithFlags(&x, hipEventDisableTiming), "hipEventCreate");
        for (uint32_t c = 0; c < nch; ++c) {
            const uint32_t k = c & 1, lo = c * chunk_, m = (n - lo < chunk_) ? n - lo : chunk_;
            const size_t bytes = size_t(m) * slot_;
            if (c >= 2) hip_check(hipStreamWaitEvent(s_[0], ev[2][k], 0), "wait d2h");  // chunk buffer free
            hip_check(hipMemcpyAsync(dbuf_[k], slot(lo), bytes, hipMemcpyHostToDevice, s_[0]), "H2D");
            bool any_raw = false;
            for (uint32_t j = 0; j < m && !any_raw; ++j) any_raw = raw_[lo + j] != 0;
            if (any_raw) {  // the chunk's descriptors, raw slots flagged (hdesc_[k] is free: c-2 finished)
                if (c >= 2) hip_check(hipEventSynchronize(ev[0][k]), "wait desc buffer");
                for (uint32_t j = 0; j < m; ++j)
                    hdesc_[k][j] = smol_csum_desc_t{uint64_t(j) * slot_, slot_, uint8_t(medium_),
                                                    uint8_t(raw_[lo + j] ? SMOL_REC_IPHDR_ONLY : 0u), 0};
                hip_check(hipMemcpyAsync(ddesc_[k], hdesc_[k], size_t(m) * sizeof(smol_csum_desc_t),
                                         hipMemcpyHostToDevice, s_[0]), "H2D(desc)");
            }
            hip_check(hipEventRecord(ev[0][k], s_[0]), "record");
            hip_check(hipStreamWaitEvent(s_[1], ev[0][k], 0), "wait h2d");
            Batch b = any_raw ? Batch::described(ddesc_[k], m) : Batch::fixed(m, slot_, slot_, medium_);
            if (emit) eng_.emit(dbuf_[k], b, caps, nullptr, s_[1]);
            else eng_.verify(dbuf_[k], b, dst_[k], caps, s_[1]);
            hip_check(hipEventRecord(ev[1][k], s_[1]), "record");
            hip_check(hipStreamWaitEvent(s_[2], ev[1][k], 0), "wait kernel");
            if (emit) hip_check(hipMemcpyAsync(slot(lo), dbuf_[k], bytes, hipMemcpyDeviceToHost, s_[2]), "D2H");
            else hip_check(hipMemcpyAsync(status_ + lo, dst_[k], m, hipMemcpyDeviceToHost, s_[2]), "D2H");
            hip_check(hipEventRecord(ev[2][k], s_[2]), "record");
        }
        hip_check(hipStreamSynchronize(s_[2]), "hipStreamSynchronize");
        for (auto& e : ev)
            for (auto& x : e) (void)hipEventDestroy(x);
    }

    Engine eng_;
    uint32_t slots_, slot_, chunk_;
    Medium medium_;
    uint8_t* host_ = nullptr;
    uint8_t* status_ = nullptr;
    uint8_t* raw_ = nullptr;  // per slot: a raw socket's frame
    uint8_t* dbuf_[2] = {nullptr, nullptr};
    uint8_t* dst_[2] = {nullptr, nullptr};
    smol_csum_desc_t* ddesc_[2] = {nullptr, nullptr};
    smol_csum_desc_t* hdesc_[2] = {nullptr, nullptr};
    hipStream_t s_[3] = {};
};

}  // namespace smoltcp_amd
