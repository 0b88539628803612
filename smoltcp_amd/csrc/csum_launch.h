// Host <-> kernel interface of the checksum engine (internal; the public ABI is
// include/smolcsum.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "../../include/smolcsum.h"

namespace smolcsum {

enum { MODE_DATA = 0, MODE_EMIT = 1, MODE_VERIFY = 2, MODE_COPY = 3 };  // COPY: fused copy + emit

// Internal record kind of the 6LoWPAN NHC UDP entry points (never in a descriptor).
constexpr uint32_t KIND_NHC_UDP = 0x10;
// Internal kind bit: SMOL_REC_IPHDR_ONLY (a raw socket's frame: the IP header's gate only).
constexpr uint32_t KIND_IPHDR_ONLY = 0x200;
// The kernels' view of a descriptor's kind byte + flags byte (the desc dword at offset 12).
__host__ __device__ __forceinline__ uint32_t desc_kind(uint32_t w) {
    return (w & 0xffu) | (((w >> 8) & SMOL_REC_IPHDR_ONLY) ? KIND_IPHDR_ONLY : 0u);
}

// Launch shapes: lanes per record (G) x 16-byte chunks per lane per step (U).
enum {
    CFG_G8U6 = 0,
    CFG_G16U3 = 1,
    CFG_G16U6 = 2,
    CFG_G32U3 = 3,
    CFG_G32U4 = 4,
    CFG_G64U2 = 5,
    CFG_G64U4 = 6,
    CFG_G8U7 = 7,
    CFG_G16U4 = 8,
    CFG_COUNT = 9
};

struct KParams {
    uint8_t* buf;
    const smol_csum_desc_t* desc;  // nullptr: implicit fixed-stride batch
    uint64_t n;
    uint64_t stride;
    uint32_t len;
    uint32_t kind;
    uint32_t caps_ipv4, caps_udp, caps_tcp, caps_icmpv4, caps_icmpv6;
    uint16_t* out16;  // MODE_DATA
    uint8_t* status;  // MODE_VERIFY (required), MODE_EMIT (optional)
    const uint8_t* dummy;  // 16-byte-aligned device line read by loads that have nothing to read
    uint32_t num_cu;       // compute units of the device (grid sizing)
    const uint8_t* src;             // MODE_COPY: payload source buffer
    const smol_csum_copy_t* copy;   // MODE_COPY: one payload copy per record (16-B aligned)
    const uint8_t* addrs;  // 6LoWPAN NHC UDP batches: 32 B (IPv6 src, dst) per record, else nullptr
    uint32_t xcd_remap;    // walk kernel: 0 dispatch order; 1 block b takes the records of block
                           // xcd_block(b); K >= 2: those of xcd_chunk(b, K) (see below)
    uint64_t* stage;       // staged emit (csum_walk.h stage_entry): one 8-B field entry per record
    uint32_t* stage_flags; // staged emit: one flag per 8 records (1: their entries are this call's)
};

// The 8 XCDs of an MI355X are dealt workgroups round-robin (MI355X_MICROARCH.md, workgroup dispatch:
// observed, not promised): blocks b, b + 8, ... share an XCD.  This bijection on [0, nwg) gives the
// blocks of one XCD a contiguous range of logical blocks, so that each XCD streams its own part of
// the batch (its L2 and address-translation caches see one region instead of every region).
__host__ __device__ inline uint64_t xcd_block(uint64_t b, uint64_t nwg) {
    const uint64_t q = nwg / 8, r = nwg % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// The same at a finer grain: the XCDs take turns over runs of K consecutive logical blocks (K = 1 is
// the dispatch order).  A bijection: the first nwg rounded down to 8K blocks are permuted, the rest
// keep their index.
__host__ __device__ inline uint64_t xcd_chunk(uint64_t b, uint64_t nwg, uint64_t K) {
    const uint64_t full = nwg / (8 * K) * (8 * K);
    if (b >= full) return b;
    const uint64_t x = b % 8, j = b / 8;
    return ((j / K) * 8 + x) * K + (j % K);
}

#ifdef __HIPCC__
// The logical block this workgroup works as (KParams::xcd_remap).
__device__ inline uint64_t logical_block(uint32_t xcd_remap) {
    return xcd_remap == 0 ? (uint64_t)blockIdx.x
           : xcd_remap == 1 ? xcd_block(blockIdx.x, gridDim.x)
                            : xcd_chunk(blockIdx.x, gridDim.x, xcd_remap);
}
#endif

// The kernel instantiation of the process's last checksum launch, packed kernel << 24 | variant << 16
// | G << 8 | U (smol_csum_tool_last_launch): tests check that a forced variant runs the kernel it
// names rather than a dispatch fallback.
enum { KERN_WALK = 1, KERN_TILE = 2, KERN_COPY = 3, KERN_WALK_NHC = 4, KERN_XWALK = 5, KERN_DWALK = 6 };
inline std::atomic<uint32_t> g_last_launch{0};
inline void note_launch(uint32_t kern, uint32_t var, uint32_t g, uint32_t u) {
    g_last_launch.store(kern << 24 | (var & 0xffu) << 16 | (g & 0xffu) << 8 | (u & 0xffu),
                        std::memory_order_relaxed);
}

// A dispatch may hold at most 2^32 - 1 work-items: 256-thread grids are capped at 2^24 - 1 blocks
// (every kernel loops with a grid stride, so a capped grid still covers the whole batch; C5's 2^27
// records per GPU need it).
constexpr uint64_t kMaxGridBlocks = 0xFFFFFFull;
__host__ __device__ inline uint32_t grid_blocks(uint64_t want, uint64_t cap) {
    uint64_t b = want < cap ? want : cap;
    b = b < kMaxGridBlocks ? b : kMaxGridBlocks;
    return (uint32_t)(b ? b : 1);
}

// Workgroups of `kernel` (256 threads) resident on the whole device, capped at max_blocks.
uint32_t resident_blocks(const void* kernel, uint32_t num_cu, uint32_t max_blocks);

hipError_t launch_csum(int mode, int shape, int var, const KParams& p, uint32_t max_blocks, hipStream_t s);
// Walk kernel for one (mode, batch form): csum_walk.h, instantiated in csum_walk_*.hip.
template <int MODE, bool IMPLICIT>
hipError_t launch_walk(int shape, int var, const KParams& p, uint32_t max_blocks, hipStream_t s);
// The same for 6LoWPAN NHC UDP batches (p.addrs set), csum_walk_nhc.hip.
template <int MODE, bool IMPLICIT>
hipError_t launch_walk_nhc(int shape, int var, const KParams& p, uint32_t max_blocks, hipStream_t s);
// Tile kernel (csum_tile.hip), emit / verify only; var 0 = non-temporal loads, 1 = plain loads.
hipError_t launch_tile(int mode, int shape, int var, int tile_records, const KParams& p, uint32_t max_blocks,
                       hipStream_t s);

// Stripe kernel (csum_tile.hip, variant 42): fixed-stride packed records of 1024-1520 bytes.
bool stripe_fits(const KParams& p);
hipError_t launch_stripe(int mode, const KParams& p, hipStream_t s);
// Transposed walk (csum_xwalk.hip, variants 44 / 47 = whole field segments): fixed-stride packed
// records of 1024-16257 bytes.
bool xwalk_fits(const KParams& p);
// Copy-emit on the transposed walk's layout (csum_xcopy.hip, variants 49 / 50 = persistent grid,
// experiments build): fixed-stride records of 1024-1921 bytes.
bool xcopy_fits(const KParams& p);
// Descriptor-batch walks (csum_dwalk.hip): variant 60 = verify default; 56 / 60 emit: experiments.
hipError_t launch_dwalk(int mode, int variant, const KParams& p, hipStream_t s);
hipError_t launch_xcopy(int variant, const KParams& p, hipStream_t s);
hipError_t launch_xwalk(int mode, int variant, const KParams& p, hipStream_t s);
// Staged emit (variants 80 / 81): the transposed walk writes each record's field entry to p.stage, then
// the segment pass writes the field segments whole (csum_xwalk.hip).  Records per launch pair:
constexpr uint64_t kStageChunk = 1ull << 21;
inline bool staged_variant(int v) { return v == 80 || v == 81; }
inline bool staged_desc_variant(int v) { return (v >= 94 && v <= 97) || (v >= 103 && v <= 105) || v == 109; }  // csum_dwalk.hip
// The segment pass of the staged emit (csum_dwalk.hip seg_pass4_kernel), after the staging launch.
hipError_t launch_seg_pass(const KParams& p, hipStream_t s, int form = 0);

// Synthetic batches and fault injection (tools; include/smolcsum_tools.h).
struct SynthParams {
    uint8_t* buf;
    const smol_csum_desc_t* desc;
    uint64_t n;
    uint64_t stride;
    uint32_t len;
    uint32_t profile;
    uint64_t seed;
};
hipError_t launch_synth(const SynthParams& p, uint32_t max_blocks, hipStream_t s);
hipError_t launch_corrupt(const SynthParams& p, uint32_t every, hipStream_t s);
// IPv4 fragment groups (csum_frag.hip): MODE_EMIT / MODE_VERIFY, one wavefront per group.
hipError_t launch_frag(int mode, const KParams& p, const smol_csum_frag_group_t* groups, uint64_t ngroups,
                       hipStream_t s);
hipError_t launch_stream_read(const uint8_t* buf, uint64_t bytes, uint32_t* sink, uint32_t max_blocks,
                              hipStream_t s);
hipError_t launch_field_probe(uint8_t* buf, uint64_t bytes, uint64_t stride, uint32_t f1, uint32_t f2,
                              uint32_t max_blocks, hipStream_t s);
hipError_t launch_field_scatter(uint8_t* buf, uint64_t bytes, const uint64_t* addrs, const uint16_t* vals, uint64_t n,
                                int nt, hipStream_t s);
hipError_t launch_field_probe_list(uint8_t* buf, uint64_t bytes, const uint64_t* addrs, const uint32_t* first,
                                   int seg64, uint32_t max_blocks, hipStream_t s);
hipError_t launch_segment_probe(uint8_t* buf, uint64_t bytes, const uint32_t* bitmap, int nt, uint32_t max_blocks,
                                hipStream_t s);

}  // namespace smolcsum
