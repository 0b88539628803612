// C ABI of the checksum engine: scalar host mirrors of smoltcp::wire::checksum and the batched
// device entry points (include/smolcsum.h), plus the tooling entry points
// (include/smolcsum_tools.h).  No exception crosses this boundary; every batched call either
// launches HIP kernels or returns an error — there is no CPU fallback.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <new>
#include <string>

#include "../../include/smolcsum.h"
#include "../../include/smolcsum_tools.h"
#include "csum_launch.h"

using namespace smolcsum;

struct smol_csum_ctx {
    int device;
    int num_cu;
    uint32_t max_blocks;  // grid cap (kNaturalGrid: one work item per group)
    int shape;            // -1 automatic, else CFG_*
    int variant;          // kernel variant (-1 automatic; csum_walk.h VarT, 3/4 tile kernel)
    uint8_t* dummy;       // 256 zero bytes on the device (target of loads with nothing to read)
    int tile_records;     // tile kernel: records per wavefront tile (32 or 64)
    bool max_blocks_set;  // grid cap given explicitly (tooling)
    int xcd_remap;        // walk kernel: each XCD's blocks take a contiguous range of records
                          // (-1: automatic, xcd_remap_auto; 0 / 1: forced, tooling)
    uint64_t launch_records;  // records per kernel launch (0: the whole batch in one launch)
    // staged emit (variant 94; 80 / 81 experiments): the field entries and per-8-record flags of one
    // chunk of kStageChunk records, allocated with the context (no allocation in a batched call);
    // stage_stream / stage_done order a staged emit on another stream after the previous one
    uint64_t* stage;
    uint32_t* stage_flags;
    void* stage_stream;
    bool stage_recorded;
    hipEvent_t stage_done;
    // descriptor-batch emit chooses between the staged form (97) and the in-place one (41) from the
    // previous staged call's wavefront flags (a sample of the first kSample copied to host memory):
    // staged while at least half of the sampled wavefronts staged, else in place, probing with the
    // staged form again every kReprobe calls
    uint32_t* sample_host;    // pinned
    hipEvent_t sample_ev;
    bool sample_pending;
    int desc_staged;          // 1: the staged form (also before any sample), 0: in place
    uint32_t since_probe;
};

namespace {
constexpr uint32_t kSample = 256;   // wavefront flags (8 records each) sampled per staged call
constexpr uint32_t kReprobe = 64;   // in-place calls between two staged probes
}

namespace smolcsum {

uint32_t resident_blocks(const void* kernel, uint32_t num_cu, uint32_t max_blocks) {
    if (num_cu == 0) return max_blocks;  // explicit grid cap (smol_csum_tool_set_max_blocks)
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const uint64_t cap = (uint64_t)per_cu * num_cu;
    return (uint32_t)(cap < max_blocks ? cap : max_blocks);
}

}  // namespace smolcsum

namespace {

thread_local std::string g_last_error;

int hip_fail(hipError_t e, const char* what) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return SMOL_EHIP;
}

struct DeviceGuard {  // run on ctx->device, restore the caller's current device afterwards
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        int now = -1;
        if (prev >= 0 && hipGetDevice(&now) == hipSuccess && now != prev) (void)hipSetDevice(prev);
    }
};

bool caps_valid(const smol_checksum_caps_t* c) {
    if (!c) return false;
    const uint8_t v[5] = {c->ipv4, c->udp, c->tcp, c->icmpv4, c->icmpv6};
    for (uint8_t x : v)
        if (x > SMOL_CHECKSUM_NONE) return false;
    return c->reserved[0] == 0 && c->reserved[1] == 0 && c->reserved[2] == 0;
}

// Grid cap meaning "one work item per group" (no persistent loop): on MI355X many small
// workgroups dispatched by the hardware beat a persistent grid (tools/sweep.py, C2: verify
// 0.244 ms vs 0.27 ms at 8 blocks per CU).
constexpr uint32_t kNaturalGrid = 0x7fffffffu;

// Kernel variant when none is forced (tools/sweep.py on MI355X, C2 / C3 / C4): the 128-byte line
// grid with non-temporal loads (verify: C2 0.2415 -> 0.2327 ms, C4 0.2158 -> 0.2083 ms, C3 0.826 ->
// 0.815 ms; fixed-stride emit with shared boundary lines, csum_walk.h shared_from: C2 0.3155 ->
// 0.304 ms, C4 0.2727 -> 0.263 ms), except emit over descriptor batches: the tile kernel on the
// line grid (variant 7, C3 0.9285 ms vs the walk kernel's best 0.9945 ms at the same shape; its
// verify is slower, 1.08 ms vs 0.83 ms).  walk_variant is the walk kernel's own choice, for the
// entry points the tile kernel does not serve (NHC, data, copy-emit): cached loads on the 16-byte
// grid for emit over descriptors (C3 0.9705 ms vs 0.9722 ms), the line grid otherwise.
// Verify over descriptor batches (C3) runs the line grid without the register prefetch (variant
// 13) at 16 x 4: with the record geometry in LDS that kernel holds 63 VGPRs (8 waves/SIMD), and the
// waves hide the latency the prefetch hid before: C3 verify 0.7998 ms (variant 5, 16 x 3) ->
// 0.7425 ms (tools/gpu_ab.sh, MI355X).  Fixed-stride verify keeps the prefetch (C2 8 x 7: 0.2378
// vs 0.2519 ms without).
int walk_variant(int mode, bool has_desc) {
    // fixed-stride emit: variant 5 with the fields' 64-B segments written whole where no neighbour's
    // field shares them (C2 emit 0.305 -> 0.294 ms, tools/exp_emit_seg.py), skipped on wavefronts
    // without an IPv4 record (variant 29: C2 0.2891-0.2894 vs 19's 0.2907-0.2913 ms, C4 0.2649-0.2658
    // vs 0.2654-0.2666 ms, interleaved on one box, profiles/r04_experiments/).  Round 5: variant 39
    // = 29, and on a wavefront without an IPv4 record whole segments for IPv6 records too, decided
    // by one ballot (bench lines over rotating batches, interleaved on one box,
    // profiles/r05_experiments/emit_variants_bench.txt: C4 5151-5157 -> 5237-5253 GiB/s, C2 equal)
    if (!has_desc) return mode == MODE_EMIT ? 39 : 5;
    return mode == MODE_EMIT ? 1 : mode == MODE_VERIFY ? 13 : 5;
}
// Round 5: verify over descriptor batches runs dwalk_kernel's per-group walk (csum_dwalk.hip: 8
// records per wavefront, parse first, 8 lanes x 4 chunks per step on the line grid, 7 waves / SIMD):
// C3 0.793 -> 0.742 ms, 64-1500-B records 0.343 -> 0.185 ms with non-temporal header windows
// (variant 60, tools/exp_r05_desc.py, profiles/r05_experiments/dwalk_layouts.jsonl).  Variant 63
// loads the header windows with the default cache policy, so that the stream's second read of those
// lines and emit's field stores hit the L2: C3 bench (4 batch pairs in turn, one box, interleaved)
// verify 0.742 -> 0.731 ms and emit 0.942 (tile 7) -> 0.896 ms, 5269 -> 5457 GiB/s
// (profiles/r05_experiments/dwalk_cached_windows.txt); its emit beats the tile kernel on every
// descriptor layout measured, 64-1500-B records 0.223 -> 0.184 ms.  The tile kernel stays the
// descriptor-emit fallback (NHC emit runs the walk kernel).
// Its emit form 41 sums the 16 window chunks from LDS and streams from chunk 16 (the window lines not
// read a second time): C3 emit 0.894 -> 0.881 ms, shuffled descriptors 0.922 -> 0.912, 64-1500-B
// records 0.186 -> 0.183; its verify measured 0.4 % slower, so verify stays on 63
// (profiles/r05_experiments/dwalk_cached_windows.txt).
int auto_variant(int mode, bool has_desc) {
    if (mode == MODE_EMIT && has_desc) return 41;
    if (mode == MODE_VERIFY && has_desc) return 63;
    return walk_variant(mode, has_desc);
}

// The transposed walk (csum_xwalk.hip) for fixed-stride records where it beats the walk kernel, from a
// measured table (round 6; VERDICT r05 item 7 replaced round 5's fitted length windows): one length
// sweep, tools/sweep_dispatch.py, over 1024 .. 9023 B in steps of 64 B (multiples of 64, + 28, and + 28
// with 64-B gaps), verify and emit (emit in bench.py's step order), on three boxes
// (profiles/r06_dispatch_sweep_box{1,2,3}.jsonl), turned into dispatch_table.inc by
// tools/gen_dispatch_table.py (the least summed time per entry).  Verify: the walk kernel (5), the
// transposed walk (47) or 47 with the first-load hint (89: lanes 0-3 of each record's first instruction
// with the default cache policy; C2 verify 0.2342 -> 0.2259 ms); emit: the walk kernel (39), 47, 57 (47
// with non-temporal field segments) or 101 (57's segments stored write-through), from a second emit
// sweep that ran all four (late round 6, profiles/r06_dispatch_sweep_wt_*.jsonl: two IPv4 boxes, two
// IPv6-mix boxes; C2's and C4's rows take 101).  Outside 1024 .. 9023 B the walk kernel
// (round 5: past 9000 B the two trade places by length, within 2 %).
// Returns the transposed-walk variant to run (0: the walk kernel).
#include "dispatch_table.inc"

int xwalk_auto(int mode, const smol_csum_batch_t* b) {
    if (b->desc || b->stride < b->len || (mode != MODE_VERIFY && mode != MODE_EMIT)) return 0;
    if (b->len < 1024 || b->len >= 1024 + 64 * 125) return 0;
    const uint32_t k = (b->len - 1024) / 64;
    const int col = b->stride != b->len ? 2 : (b->len % 64 == 0 ? 0 : 1);
    const char c = (mode == MODE_VERIFY ? kVerifyTable : kEmitTable)[k][col];
    if (mode == MODE_VERIFY) return c == 'h' ? 89 : c == 'x' ? 47 : 0;
    return c == 't' ? 101 : c == 'n' ? 57 : c == 'x' ? 47 : 0;
}

// The XCD block order (csum_launch.h xcd_block / xcd_chunk) when none is forced: the contiguous order
// for fixed-stride emit over at least 4 GiB.  Measured per 2^20 C2 records (tools/exp_inplace.py, one box,
// profiles/r04_experiments/xcd_remap.jsonl): emit 0.327 -> 0.298 ms at 2^22 records (6.3 GB),
// 0.332 -> 0.320 at 2^24, 0.338 -> 0.303 at 2^26, and C5's 2^27: 0.334 -> 0.300; at 2^20 records
// 0.297 -> 0.2995 (no gain).  Verify runs 4-6 % slower with it at every size, so it keeps the
// dispatch order.
// Verify over at least 64 GiB takes runs of 256 workgroups per XCD turn: C5's in-place verify 31.38-
// 31.46 -> 30.96-30.99 ms (profiles/r04_experiments/c5_verify_grain.jsonl); at 25 GB it was +1 %,
// at 100 GB -0.6 % (xcd_grain.jsonl), so smaller batches keep the dispatch order.
int xcd_remap_auto(int mode, const smol_csum_batch_t* b) {
    if (b->desc) return 0;
    const uint64_t bytes = b->n * b->stride;
    if (mode == MODE_EMIT) return bytes >= (4ull << 30) ? 1 : 0;
    if (mode == MODE_VERIFY) return bytes >= (64ull << 30) ? 256 : 0;
    return 0;
}

// SMOL_BATCH_FIELD_STORES: the same kernel without the whole-segment writes (2-B field stores only).
int field_store_variant(int variant, bool has_desc) {
    if (variant == 19 || variant == 23 || variant == 24 || variant == 25 || variant == 29 || variant == 39) return 5;
    if (variant == 47 || variant == 57 || variant == 45 || (variant >= 80 && variant <= 93) || variant == 99 || variant == 100 ||
        variant == 101)
        return 44;
    if (variant == 61) return 60;  // the descriptor walk's emit: 2-B stores (62: cached windows, 63)
    if (variant == 62 || variant == 18) return 63;  // (63 stores 2-B fields only)
    if (variant == 20) return 60;
    if (variant == 41 || (variant >= 94 && variant <= 97) || (variant >= 103 && variant <= 105) || variant == 109) return 41;
    if (variant == 26 || variant == 27 || variant == 28) return 13;
    return variant;
}

// The kernel variants this build runs (smol_csum_tool_variant_built).  The product library: the
// defaults (walk 5 / 39, transposed walk 47 / 57, descriptor walk 63 (verify) / 41 (emit), copy 21)
// and one fallback each (descriptor walk 60, tile 7, copy 17; walk 13 for NHC / data over
// descriptors and for forced variants; 44 = 47 / 57 with 2-B field stores, SMOL_BATCH_FIELD_STORES).  The experiments build (SMOL_EXP, libsmolcsum_exp.so): every measured variant.
bool variant_built(int v) {
    switch (v) {
        case -1: case 5: case 7: case 13: case 17: case 21: case 39: case 41: case 44: case 47: case 57: case 60: case 63:
        case 89: case 97: case 101: return true;
        default: break;
    }
#ifdef SMOL_EXP
    if ((v >= 80 && v <= 96 && v != 89) || (v >= 98 && v <= 100) || (v >= 102 && v <= 110) || v == 112 || v == 113) return true;
    const int b = v >= 64 ? v - 64 : v;
    if (v >= 64) return b == 5 || b == 29 || (b >= 31 && b <= 39) || b == 44 || b == 47 || b == 56 || b == 61;
    return (v >= 0 && v <= 4) || v == 6 || (v >= 8 && v <= 11) || v == 16 || v == 19 || (v >= 23 && v <= 29) ||
           (v >= 31 && v <= 38) || v == 40 || v == 12 || v == 14 || v == 42 || v == 43 || v == 45 || v == 46 || v == 15 || v == 18 || v == 20 || v == 22 || v == 30 || v == 41 || v == 48 || (v >= 49 && v <= 59) || v == 61 || v == 62;
#else
    return false;
#endif
}

bool line_grid(int variant) {
    if (variant >= 64) variant -= 64;  // experiment variants without stores
    if ((variant >= 31 && variant <= 40) || variant == 12 || variant == 14) return true;
    return variant == 5 || variant == 6 || variant == 9 || variant == 10 || variant == 13 || variant == 19 ||
           (variant >= 23 && variant <= 29);
}

int auto_shape(uint32_t len, bool has_desc, bool line = false, int variant = -1) {
    if (has_desc) return (variant == 13 || variant == 26 || variant == 27 || variant == 28) ? CFG_G16U4 : CFG_G16U3;
    const uint64_t need = (uint64_t)len + (line ? 127 : 15);  // bytes of aligned chunks a record can touch
    // eight records per wavefront in two steps, with as few idle lanes as possible (C4's 1320-B
    // records on the line grid: 8 x 6 0.2083 ms, 8 x 7 0.2188 ms; C2's 1500 B: 8 x 7 0.2327 ms)
    if (need <= 16 * 8 * 6 * 2) return CFG_G8U6;
    if (line && need <= 16 * 8 * 7 * 2) return CFG_G8U7;
    if (need <= 16 * 16 * 6) return CFG_G16U6;
    if (need <= 16 * 32 * 4) return CFG_G32U4;
    return CFG_G64U4;
}

int check_batch(const smol_csum_batch_t* b, const void* d_buf) {
    if (!b) return SMOL_EINVAL;
    if (b->n == 0) return SMOL_OK;
    if (!d_buf) return SMOL_EINVAL;
    if ((b->flags & ~(SMOL_REC_IPHDR_ONLY | SMOL_BATCH_FIELD_STORES)) != 0 || b->reserved[0] != 0 ||
        b->reserved[1] != 0)
        return SMOL_EINVAL;
    if (b->desc) {
        if (((uintptr_t)b->desc & 15u) != 0) return SMOL_EINVAL;
    } else if (b->len > SMOL_MAX_RECORD_LEN) {
        return SMOL_ERANGE;
    }
    return SMOL_OK;
}

// The kernel a batched call runs: its family, variant and (walk / tile / copy kernels) launch shape.
// One pure function, so that smol_csum_tool_kernel_for names exactly what run() launches.
enum Family { F_WALK, F_TILE, F_XWALK, F_DWALK, F_STRIPE, F_COPY, F_XCOPY };
struct Pick {
    int family;
    int variant;
    int shape;
};

// Variants that serve copy-emit only: copy_kernel (17, 21; 22 / 30 experiments), the transposed
// layout (49-55, experiments) and the walk kernel's MODE_COPY forms 8 / 11 / 16 (experiments).  Forced
// on a context, they leave emit / verify / data to the library's choice (the automatic dispatch).
bool copy_only(int v) { return v == 8 || v == 11 || v == 16 || v == 17 || v == 21 || v == 22 || v == 30 || v == 98 || v == 102 || (v >= 49 && v <= 55); }

Pick pick_kernel(const smol_csum_ctx_t* ctx, int mode, const smol_csum_batch_t* b, const KParams& p) {
    const bool has_desc = b->desc != nullptr;
    const bool nhc = p.addrs != nullptr;
    if (mode == MODE_COPY) {  // one fused pass (no tile / deferred variants)
        // default: variant 21 (csum_copy.hip: variant 17's body chunks = one source load + shift +
        // sum + store, with the first body round's loads issued ahead of round 1's stores) at its
        // default shape (16 x 4): C2copy 0.772-0.853 ms (variant 16) -> 0.692 ms (17) -> 0.678 ms
        // (21; tools/exp_copy.py, MI355X).  Variants 1 / 8 / 11 / 16 / 17 stay selectable.
        const int cv = ctx->variant;
        if (cv >= 49 && cv <= 55 && xcopy_fits(p)) return {F_XCOPY, cv, -1};
        const int var = (cv == 1 || cv == 8 || cv == 11 || cv == 16 || cv == 17 || cv == 22 || cv == 30 || cv == 98 || cv == 102) ? cv : 21;
        const bool ck = var == 17 || var == 21 || var == 22 || var == 30 || var == 98 || var == 102;
        const int gv = cv >= 0 ? cv : walk_variant(mode, has_desc);
        const int shape = ctx->shape >= 0 ? ctx->shape : ck ? (int)CFG_G16U4 : auto_shape(b->len, has_desc, line_grid(gv), gv);
        return {ck ? F_COPY : F_WALK, var, shape};
    }
    int variant = copy_only(ctx->variant) ? -1 : ctx->variant;
    if (variant < 0) {
        const int xv = nhc ? 0 : xwalk_auto(mode, b);
        variant = xv ? xv : auto_variant(mode, has_desc);
        // descriptor-batch emit: the staged form while the records stage (see smol_csum_ctx)
        if (variant == 41 && ctx->desc_staged) variant = 97;
    }
    if (mode == MODE_EMIT && (b->flags & SMOL_BATCH_FIELD_STORES)) variant = field_store_variant(variant, has_desc);
    // a kernel that does not serve the batch falls back to the default of its kind (descriptor emit:
    // the tile kernel; otherwise the walk kernel)
    const int fallback = (mode == MODE_EMIT && has_desc && !nhc) ? 7 : walk_variant(mode, has_desc);
    // the stripe kernel (variant 42, experiments): emit / verify of packed fixed-stride 1024-1520-B records
    if (variant == 42) {
        if ((mode == MODE_EMIT || mode == MODE_VERIFY) && !nhc && stripe_fits(p)) return {F_STRIPE, 42, -1};
        variant = fallback;
    }
    // the transposed walk (44 / 47 / 57 product, the others experiments): fixed-stride records of
    // 1024 - 16257 B
    const int v64 = variant % 64;
    const bool xw_var = (variant < 64 && (variant == 44 || variant == 47 || variant == 43 || variant == 45 || variant == 46 ||
                                          variant == 15 || variant == 48 || variant == 57 || variant == 58 || variant == 59)) ||
                        (variant >= 64 && (v64 == 44 || v64 == 47)) || staged_variant(variant) || (variant >= 82 && variant <= 93) ||
                        variant == 99 || variant == 100 || variant == 101 || variant == 106 || variant == 107 || variant == 108 || variant == 110 || variant == 112 || variant == 113;
    if (xw_var) {
        if ((mode == MODE_EMIT || mode == MODE_VERIFY) && !nhc && xwalk_fits(p)) return {F_XWALK, variant, -1};
        variant = fallback;
    }
    // descriptor-batch walks: 63 = verify default (cached header windows), 41 = emit default (its emit
    // form), 60 = the non-temporal-window verify; 56, 60's emit, 61 / 62 (whole field segments) and
    // 18 / 20 (non-temporal 2-B fields) in the experiments build, which also runs them forced over
    // fixed-stride batches
    if (mode == MODE_VERIFY) {
        if (variant == 41 || variant == 18 || variant == 62 || (variant >= 94 && variant <= 97) || (variant >= 103 && variant <= 105) || variant == 109) variant = 63;  // emit forms of 63
        if (variant == 20 || variant % 64 == 61) variant = 60;              // emit forms of 60
    }
#ifdef SMOL_EXP
    const bool dw_var = variant % 64 == 56 || variant == 60 || variant % 64 == 61 || variant == 62 || variant == 63 ||
                        variant == 18 || variant == 20 || variant == 41 || (variant >= 94 && variant <= 97) || (variant >= 103 && variant <= 105) || variant == 109;
    const bool dw_ok = (mode == MODE_EMIT || mode == MODE_VERIFY) && !nhc;
#else
    const bool dw_var = variant == 60 || variant == 63 || variant == 41 || variant == 97;
    const bool dw_ok = (mode == MODE_VERIFY || (mode == MODE_EMIT && variant != 60)) && has_desc && !nhc;
#endif
    if (dw_var) {
        if (dw_ok) return {F_DWALK, variant, -1};
        variant = fallback;
    }
    // the tile kernel (3 / 4 / 7: nt / plain / nt on the line grid): IP emit and verify only
    const bool tile_var = variant == 3 || variant == 4 || variant == 7;
    if (tile_var && (mode == MODE_DATA || nhc)) variant = walk_variant(mode, has_desc);
    const int shape = ctx->shape >= 0 ? ctx->shape : auto_shape(b->len, has_desc, line_grid(variant), variant);
    if (variant == 3 || variant == 4 || variant == 7) return {F_TILE, variant, shape};
    return {F_WALK, variant, shape};
}

const char* family_kernel(const Pick& k) {
    switch (k.family) {
        case F_TILE: case F_STRIPE: return "csum_tile_kernel";
        case F_XWALK: return "xwalk_kernel";
        case F_DWALK: return "dwalk_kernel";
        case F_COPY: return "copy_kernel";
        case F_XCOPY: return "xcopy_kernel";
        default: return "csum_kernel";
    }
}

// The automatic descriptor-batch emit (nothing forced, IP records, 2-B-field mode not asked).
bool has_desc_auto(const smol_csum_ctx_t* ctx, const smol_csum_batch_t* b, const uint8_t* d_addrs) {
    return b->desc && !d_addrs && ctx->variant < 0 && !(b->flags & SMOL_BATCH_FIELD_STORES);
}

bool capturing(hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

// Before a descriptor-batch emit: take the last staged call's sample when it has arrived (a
// non-blocking event query), and probe with the staged form every kReprobe in-place calls.
void update_desc_choice(smol_csum_ctx_t* ctx, hipStream_t s) {
    if (capturing(s)) return;  // a captured graph keeps the choice it was captured with
    if (ctx->sample_pending && hipEventQuery(ctx->sample_ev) == hipSuccess) {
        ctx->sample_pending = false;
        uint32_t n = ctx->sample_host[kSample], staged = 0;
        for (uint32_t i = 0; i < n && i < kSample; ++i) staged += ctx->sample_host[i] != 0u;
        ctx->desc_staged = n == 0 || 2 * staged >= n ? 1 : 0;
        ctx->since_probe = 0;
    }
    if (!ctx->desc_staged && !ctx->sample_pending && ++ctx->since_probe >= kReprobe) ctx->desc_staged = 1;
}

// After a staged descriptor-batch emit of n records: copy the first wavefront flags to host memory.
void sample_desc_choice(smol_csum_ctx_t* ctx, uint64_t n, hipStream_t s) {
    if (capturing(s) || ctx->sample_pending) return;
    const uint32_t waves = (uint32_t)((n + 7) / 8 < kSample ? (n + 7) / 8 : kSample);
    ctx->sample_host[kSample] = waves;
    if (hipMemcpyAsync(ctx->sample_host, ctx->stage_flags, waves * sizeof(uint32_t), hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipEventRecord(ctx->sample_ev, s) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    ctx->sample_pending = true;
}

int run(smol_csum_ctx_t* ctx, int mode, uint8_t* d_buf, const smol_csum_batch_t* b,
        const smol_checksum_caps_t* caps, uint16_t* d_out, uint8_t* d_status, void* stream,
        const uint8_t* d_src = nullptr, const smol_csum_copy_t* d_copy = nullptr,
        const uint8_t* d_addrs = nullptr) {
    KParams p;
    std::memset(&p, 0, sizeof p);
    p.src = d_src;
    p.copy = d_copy;
    p.buf = d_buf;
    p.desc = b->desc;
    p.n = b->n;
    p.stride = b->stride;
    p.len = b->len;
    p.kind = d_addrs ? KIND_NHC_UDP : (b->kind | ((b->flags & SMOL_REC_IPHDR_ONLY) ? KIND_IPHDR_ONLY : 0u));
    p.addrs = d_addrs;
    if (caps) {
        p.caps_ipv4 = caps->ipv4;
        p.caps_udp = caps->udp;
        p.caps_tcp = caps->tcp;
        p.caps_icmpv4 = caps->icmpv4;
        p.caps_icmpv6 = caps->icmpv6;
    }
    p.out16 = d_out;
    p.status = d_status;
    p.dummy = ctx->dummy;
    p.num_cu = ctx->max_blocks_set ? 0u : (uint32_t)(ctx->num_cu > 0 ? ctx->num_cu : 256);
    p.xcd_remap = ctx->xcd_remap >= 0 ? (uint32_t)ctx->xcd_remap : (uint32_t)xcd_remap_auto(mode, b);
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return hip_fail(hipErrorInvalidDevice, "hipSetDevice");
    const hipStream_t s = (hipStream_t)stream;
    // A batch larger than launch_records records goes out as consecutive launches on the stream,
    // each over the next launch_records records (the per-record arrays advance with them).
    const uint64_t per = ctx->launch_records ? ctx->launch_records : b->n;
    if (per < b->n) {
        for (uint64_t i0 = 0; i0 < b->n; i0 += per) {
            smol_csum_batch_t sub = *b;
            sub.n = b->n - i0 < per ? b->n - i0 : per;
            uint8_t* buf = d_buf;
            if (b->desc) sub.desc = b->desc + i0;
            else buf = d_buf + i0 * b->stride;
            const uint64_t keep = ctx->launch_records;
            ctx->launch_records = 0;
            const int rc = run(ctx, mode, buf, &sub, caps, d_out ? d_out + i0 : nullptr, d_status ? d_status + i0 : nullptr,
                               stream, d_src, d_copy ? d_copy + i0 : nullptr, d_addrs ? d_addrs + 32 * i0 : nullptr);
            ctx->launch_records = keep;
            if (rc != SMOL_OK) return rc;
        }
        return SMOL_OK;
    }
    const bool desc_auto = mode == MODE_EMIT && has_desc_auto(ctx, b, d_addrs);
    if (desc_auto) update_desc_choice(ctx, s);
    const Pick k = pick_kernel(ctx, mode, b, p);
    if (mode == MODE_EMIT && ((k.family == F_XWALK && staged_variant(k.variant)) ||
                              (k.family == F_DWALK && staged_desc_variant(k.variant)))) {
        // staged emit: kStageChunk records at a time through the context's entries, each chunk's staging
        // launch followed by its segment pass.  A call on another stream than the previous staged emit
        // first waits for that one (the entries are the context's).
        if (ctx->stage_recorded && ctx->stage_stream != stream) {
            hipError_t ew = hipStreamWaitEvent(s, ctx->stage_done, 0);
            if (ew != hipSuccess) return hip_fail(ew, "hipStreamWaitEvent (staged emit)");
        }
        for (uint64_t i0 = 0; i0 < b->n; i0 += kStageChunk) {
            KParams q = p;
            q.n = b->n - i0 < kStageChunk ? b->n - i0 : kStageChunk;
            if (b->desc) q.desc = b->desc + i0;
            else q.buf = d_buf + i0 * b->stride;
            if (d_status) q.status = d_status + i0;
            q.stage = ctx->stage;
            q.stage_flags = ctx->stage_flags;
            const hipError_t e = k.family == F_DWALK ? launch_dwalk(mode, k.variant, q, s) : launch_xwalk(mode, k.variant, q, s);
            if (e != hipSuccess) return hip_fail(e, "checksum kernel launch");
        }
        if (desc_auto) sample_desc_choice(ctx, b->n < kStageChunk ? b->n : kStageChunk, s);
        hipError_t er = hipEventRecord(ctx->stage_done, s);  // (after the sample's copy: it reads the flags)
        if (er != hipSuccess) return hip_fail(er, "hipEventRecord (staged emit)");
        ctx->stage_stream = stream;
        ctx->stage_recorded = true;
        return SMOL_OK;
    }
    hipError_t e = hipSuccess;
    switch (k.family) {
        case F_XCOPY: e = launch_xcopy(k.variant, p, s); break;
        case F_DWALK: e = launch_dwalk(mode, k.variant, p, s); break;
        case F_XWALK: e = launch_xwalk(mode, k.variant, p, s); break;
        case F_STRIPE: e = launch_stripe(mode, p, s); break;
        case F_TILE:
            e = launch_tile(mode, k.shape, k.variant == 7 ? 2 : k.variant - 3, ctx->tile_records, p, ctx->max_blocks, s);
            break;
        default: e = launch_csum(mode, k.shape, k.variant, p, ctx->max_blocks, s); break;  // walk / copy kernels
    }
    if (e != hipSuccess) return hip_fail(e, mode == MODE_COPY ? "copy-emit kernel launch" : "checksum kernel launch");
    return SMOL_OK;
}

}  // namespace

extern "C" {

// The scalar host mirrors (smol_csum_data, _combine, _pseudo_header*) are in csum_scalar.cpp.

// ---- context ---------------------------------------------------------------------------------

int smol_csum_ctx_create(int device, smol_csum_ctx_t** out) {
    if (!out) return SMOL_EINVAL;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        g_last_error = "no HIP device";
        return SMOL_ENODEV;
    }
    if (device < 0 || device >= count) return SMOL_ENODEV;
    int cus = 0;
    hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) return hip_fail(e, "hipDeviceGetAttribute");
    DeviceGuard guard(device);
    if (!guard.ok) return hip_fail(hipErrorInvalidDevice, "hipSetDevice");
    uint8_t* dummy = nullptr;
    e = hipMalloc(&dummy, 256);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc");
    e = hipMemset(dummy, 0, 256);
    if (e != hipSuccess) {
        (void)hipFree(dummy);
        return hip_fail(e, "hipMemset");
    }
    uint64_t* stage = nullptr;
    uint32_t* flags = nullptr;
    hipEvent_t done = nullptr;
    e = hipMalloc(&stage, kStageChunk * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc(&flags, (kStageChunk / 8 + 64) * sizeof(uint32_t));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
    uint32_t* sample = nullptr;
    hipEvent_t sev = nullptr;
    if (e == hipSuccess) e = hipHostMalloc(&sample, (kSample + 1) * sizeof(uint32_t), hipHostMallocDefault);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&sev, hipEventDisableTiming);
    if (e != hipSuccess) {
        (void)hipFree(dummy);
        if (stage) (void)hipFree(stage);
        if (flags) (void)hipFree(flags);
        if (sample) (void)hipHostFree(sample);
        return hip_fail(e, "context allocation");
    }
    auto* c = new (std::nothrow) smol_csum_ctx;
    if (!c) {
        (void)hipFree(dummy);
        (void)hipFree(stage);
        (void)hipFree(flags);
        (void)hipEventDestroy(done);
        (void)hipHostFree(sample);
        (void)hipEventDestroy(sev);
        return SMOL_ENOMEM;
    }
    c->dummy = dummy;
    c->stage = stage;
    c->stage_flags = flags;
    c->stage_stream = nullptr;
    c->stage_recorded = false;
    c->stage_done = done;
    c->sample_host = sample;
    c->sample_ev = sev;
    c->sample_pending = false;
    c->desc_staged = 1;
    c->since_probe = 0;
    c->tile_records = 32;
    c->max_blocks_set = false;
    c->xcd_remap = -1;
    c->launch_records = 0;
    c->device = device;
    c->num_cu = cus;
    c->max_blocks = kNaturalGrid;
    c->shape = -1;
    c->variant = -1;
    *out = c;
    return SMOL_OK;
}

int smol_csum_ctx_destroy(smol_csum_ctx_t* ctx) {
    if (!ctx) return SMOL_OK;
    {
        DeviceGuard guard(ctx->device);
        (void)hipFree(ctx->dummy);
        (void)hipFree(ctx->stage);
        (void)hipFree(ctx->stage_flags);
        (void)hipEventDestroy(ctx->stage_done);
        if (ctx->sample_pending) (void)hipEventSynchronize(ctx->sample_ev);
        (void)hipHostFree(ctx->sample_host);
        (void)hipEventDestroy(ctx->sample_ev);
    }
    delete ctx;
    return SMOL_OK;
}

// ---- batched device entry points -------------------------------------------------------------

int smol_csum_batch_data(smol_csum_ctx_t* ctx, const uint8_t* d_buf, const smol_csum_batch_t* b,
                         uint16_t* d_out, void* stream) {
    if (!ctx) return SMOL_EINVAL;
    int rc = check_batch(b, d_buf);
    if (rc != SMOL_OK || b->n == 0) return rc;
    if (!d_out) return SMOL_EINVAL;
    return run(ctx, MODE_DATA, const_cast<uint8_t*>(d_buf), b, nullptr, d_out, nullptr, stream);
}

int smol_csum_batch_emit(smol_csum_ctx_t* ctx, uint8_t* d_buf, const smol_csum_batch_t* b,
                         const smol_checksum_caps_t* caps, uint8_t* d_status, void* stream) {
    if (!ctx || !caps_valid(caps)) return SMOL_EINVAL;
    int rc = check_batch(b, d_buf);
    if (rc != SMOL_OK || b->n == 0) return rc;
    return run(ctx, MODE_EMIT, d_buf, b, caps, nullptr, d_status, stream);
}

int smol_csum_batch_verify(smol_csum_ctx_t* ctx, const uint8_t* d_buf, const smol_csum_batch_t* b,
                           const smol_checksum_caps_t* caps, uint8_t* d_status, void* stream) {
    if (!ctx || !caps_valid(caps)) return SMOL_EINVAL;
    int rc = check_batch(b, d_buf);
    if (rc != SMOL_OK || b->n == 0) return rc;
    if (!d_status) return SMOL_EINVAL;
    return run(ctx, MODE_VERIFY, const_cast<uint8_t*>(d_buf), b, caps, nullptr, d_status, stream);
}

int smol_csum_batch_copy_emit(smol_csum_ctx_t* ctx, uint8_t* d_buf, const smol_csum_batch_t* b,
                              const uint8_t* d_src, const smol_csum_copy_t* d_copy,
                              const smol_checksum_caps_t* caps, uint8_t* d_status, void* stream) {
    if (!ctx || !caps_valid(caps)) return SMOL_EINVAL;
    int rc = check_batch(b, d_buf);
    if (rc != SMOL_OK || b->n == 0) return rc;
    if (!d_src || !d_copy || ((uintptr_t)d_copy & 15u) != 0) return SMOL_EINVAL;
    return run(ctx, MODE_COPY, d_buf, b, caps, nullptr, d_status, stream, d_src, d_copy);
}

// ---- IPv4 fragment groups ---------------------------------------------------------------------

static int run_frag(smol_csum_ctx_t* ctx, int mode, uint8_t* d_buf, const smol_csum_batch_t* b,
                    const smol_csum_frag_group_t* d_groups, uint64_t n_groups, const smol_checksum_caps_t* caps,
                    uint8_t* d_status, void* stream) {
    if (!ctx || !caps_valid(caps)) return SMOL_EINVAL;
    int rc = check_batch(b, d_buf);
    if (rc != SMOL_OK) return rc;
    if (n_groups == 0) return SMOL_OK;
    if (b->n == 0 || !d_groups || ((uintptr_t)d_groups & 15u) != 0) return SMOL_EINVAL;
    if (mode == MODE_VERIFY && !d_status) return SMOL_EINVAL;
    KParams p;
    std::memset(&p, 0, sizeof p);
    p.buf = d_buf;
    p.desc = b->desc;
    p.n = b->n;
    p.stride = b->stride;
    p.len = b->len;
    p.kind = b->kind | ((b->flags & SMOL_REC_IPHDR_ONLY) ? KIND_IPHDR_ONLY : 0u);
    p.caps_ipv4 = caps->ipv4;
    p.caps_udp = caps->udp;
    p.caps_tcp = caps->tcp;
    p.caps_icmpv4 = caps->icmpv4;
    p.caps_icmpv6 = caps->icmpv6;
    p.status = d_status;
    p.dummy = ctx->dummy;
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return hip_fail(hipErrorInvalidDevice, "hipSetDevice");
    hipError_t e = launch_frag(mode, p, d_groups, n_groups, (hipStream_t)stream);
    return e == hipSuccess ? SMOL_OK : hip_fail(e, "fragment kernel launch");
}

int smol_csum_batch_emit_frag(smol_csum_ctx_t* ctx, uint8_t* d_buf, const smol_csum_batch_t* b,
                              const smol_csum_frag_group_t* d_groups, uint64_t n_groups,
                              const smol_checksum_caps_t* caps, uint8_t* d_status, void* stream) {
    return run_frag(ctx, MODE_EMIT, d_buf, b, d_groups, n_groups, caps, d_status, stream);
}

int smol_csum_batch_verify_frag(smol_csum_ctx_t* ctx, const uint8_t* d_buf, const smol_csum_batch_t* b,
                                const smol_csum_frag_group_t* d_groups, uint64_t n_groups,
                                const smol_checksum_caps_t* caps, uint8_t* d_status, void* stream) {
    return run_frag(ctx, MODE_VERIFY, const_cast<uint8_t*>(d_buf), b, d_groups, n_groups, caps, d_status, stream);
}

// ---- 6LoWPAN NHC UDP --------------------------------------------------------------------------

int smol_csum_batch_nhc_udp_emit(smol_csum_ctx_t* ctx, uint8_t* d_buf, const smol_csum_batch_t* b,
                                 const smol_ipv6_addr_pair_t* d_addrs, const smol_checksum_caps_t* caps,
                                 uint8_t* d_status, void* stream) {
    if (!ctx || !caps_valid(caps)) return SMOL_EINVAL;
    int rc = check_batch(b, d_buf);
    if (rc != SMOL_OK || b->n == 0) return rc;
    if (!d_addrs || ((uintptr_t)d_addrs & 3u) != 0) return SMOL_EINVAL;
    return run(ctx, MODE_EMIT, d_buf, b, caps, nullptr, d_status, stream, nullptr, nullptr,
               reinterpret_cast<const uint8_t*>(d_addrs));
}

int smol_csum_batch_nhc_udp_verify(smol_csum_ctx_t* ctx, const uint8_t* d_buf, const smol_csum_batch_t* b,
                                   const smol_ipv6_addr_pair_t* d_addrs, const smol_checksum_caps_t* caps,
                                   uint8_t* d_status, void* stream) {
    if (!ctx || !caps_valid(caps)) return SMOL_EINVAL;
    int rc = check_batch(b, d_buf);
    if (rc != SMOL_OK || b->n == 0) return rc;
    if (!d_status || !d_addrs || ((uintptr_t)d_addrs & 3u) != 0) return SMOL_EINVAL;
    return run(ctx, MODE_VERIFY, const_cast<uint8_t*>(d_buf), b, caps, nullptr, d_status, stream, nullptr,
               nullptr, reinterpret_cast<const uint8_t*>(d_addrs));
}

const char* smol_csum_last_error(void) { return g_last_error.c_str(); }

int smol_csum_abi_version(void) { return SMOLCSUM_ABI_VERSION; }

// ---- tooling (include/smolcsum_tools.h) -------------------------------------------------------

int smol_csum_tool_synth(smol_csum_ctx_t* ctx, uint8_t* d_buf, const smol_csum_batch_t* b,
                         int profile, uint64_t seed, void* stream) {
    if (!ctx || profile < 0 || profile > SMOL_SYNTH_RANDOM) return SMOL_EINVAL;
    int rc = check_batch(b, d_buf);
    if (rc != SMOL_OK || b->n == 0) return rc;
    SynthParams p{d_buf, b->desc, b->n, b->stride, b->len, (uint32_t)profile, seed};
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return hip_fail(hipErrorInvalidDevice, "hipSetDevice");
    hipError_t e = launch_synth(p, ctx->max_blocks, (hipStream_t)stream);
    return e == hipSuccess ? SMOL_OK : hip_fail(e, "synth kernel launch");
}

int smol_csum_tool_corrupt(smol_csum_ctx_t* ctx, uint8_t* d_buf, const smol_csum_batch_t* b,
                           uint32_t every, uint64_t seed, void* stream) {
    if (!ctx || every == 0) return SMOL_EINVAL;
    int rc = check_batch(b, d_buf);
    if (rc != SMOL_OK || b->n == 0) return rc;
    SynthParams p{d_buf, b->desc, b->n, b->stride, b->len, 0u, seed};
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return hip_fail(hipErrorInvalidDevice, "hipSetDevice");
    hipError_t e = launch_corrupt(p, every, (hipStream_t)stream);
    return e == hipSuccess ? SMOL_OK : hip_fail(e, "corrupt kernel launch");
}

int smol_csum_tool_set_shape(smol_csum_ctx_t* ctx, int shape) {
    if (!ctx || shape < -1 || shape >= CFG_COUNT) return SMOL_EINVAL;
    ctx->shape = shape;
    return SMOL_OK;
}

int smol_csum_tool_variant_built(int variant) { return variant_built(variant) ? 1 : 0; }

int smol_csum_tool_set_variant(smol_csum_ctx_t* ctx, int variant) {
    if (!ctx || !variant_built(variant)) return SMOL_EINVAL;
    ctx->variant = variant;
    return SMOL_OK;
}

int smol_csum_tool_set_tile(smol_csum_ctx_t* ctx, int records) {
    if (!ctx || (records != 32 && records != 64)) return SMOL_EINVAL;
    ctx->tile_records = records;
    return SMOL_OK;
}

int smol_csum_tool_set_max_blocks(smol_csum_ctx_t* ctx, uint32_t max_blocks) {
    if (!ctx) return SMOL_EINVAL;
    ctx->max_blocks = max_blocks ? max_blocks : kNaturalGrid;
    ctx->max_blocks_set = max_blocks != 0;
    return SMOL_OK;
}

int smol_csum_tool_set_xcd_remap(smol_csum_ctx_t* ctx, int on) {
    if (!ctx || on < -1) return SMOL_EINVAL;
    ctx->xcd_remap = on;
    return SMOL_OK;
}

int smol_csum_tool_set_launch_records(smol_csum_ctx_t* ctx, uint64_t records) {
    if (!ctx) return SMOL_EINVAL;
    ctx->launch_records = records;
    return SMOL_OK;
}

int smol_csum_tool_stream_read(smol_csum_ctx_t* ctx, const uint8_t* d_buf, uint64_t bytes,
                               uint32_t* d_sink, void* stream) {
    if (!ctx || !d_buf || !d_sink || (bytes & 15u) || ((uintptr_t)d_buf & 15u)) return SMOL_EINVAL;
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return hip_fail(hipErrorInvalidDevice, "hipSetDevice");
    hipError_t e = launch_stream_read(d_buf, bytes, d_sink, (uint32_t)(ctx->num_cu > 0 ? ctx->num_cu : 256) * 8u,
                                      (hipStream_t)stream);
    return e == hipSuccess ? SMOL_OK : hip_fail(e, "stream-read kernel launch");
}

int smol_csum_tool_field_probe(smol_csum_ctx_t* ctx, uint8_t* d_buf, uint64_t bytes, uint64_t stride,
                               uint32_t f1, uint32_t f2, void* stream) {
    if (!ctx || !d_buf || (bytes & 15u) || ((uintptr_t)d_buf & 15u) || stride == 0 || f1 == ~0u) return SMOL_EINVAL;
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return hip_fail(hipErrorInvalidDevice, "hipSetDevice");
    hipError_t e = launch_field_probe(d_buf, bytes, stride, f1, f2, (uint32_t)(ctx->num_cu > 0 ? ctx->num_cu : 256) * 8u,
                                      (hipStream_t)stream);
    return e == hipSuccess ? SMOL_OK : hip_fail(e, "field-probe kernel launch");
}

int smol_csum_tool_field_probe_list(smol_csum_ctx_t* ctx, uint8_t* d_buf, uint64_t bytes, const uint64_t* d_addrs,
                                    const uint32_t* d_piece_first, int flags, void* stream) {
    if (!ctx || !d_buf || !d_addrs || !d_piece_first || (bytes & 15u) || ((uintptr_t)d_buf & 15u) || (flags & ~1))
        return SMOL_EINVAL;
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return hip_fail(hipErrorInvalidDevice, "hipSetDevice");
    hipError_t e = launch_field_probe_list(d_buf, bytes, d_addrs, d_piece_first, flags & 1,
                                           (uint32_t)(ctx->num_cu > 0 ? ctx->num_cu : 256) * 8u, (hipStream_t)stream);
    return e == hipSuccess ? SMOL_OK : hip_fail(e, "field-probe kernel launch");
}

int smol_csum_tool_segment_probe(smol_csum_ctx_t* ctx, uint8_t* d_buf, uint64_t bytes, const uint32_t* d_bitmap, int flags,
                                 void* stream) {
    if (!ctx || !d_buf || !d_bitmap || (bytes & 15u) || ((uintptr_t)d_buf & 15u) || ((uintptr_t)d_bitmap & 15u) ||
        (flags & ~1))
        return SMOL_EINVAL;
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return hip_fail(hipErrorInvalidDevice, "hipSetDevice");
    hipError_t e = launch_segment_probe(d_buf, bytes, d_bitmap, flags & 1, (uint32_t)(ctx->num_cu > 0 ? ctx->num_cu : 256) * 8u,
                                        (hipStream_t)stream);
    return e == hipSuccess ? SMOL_OK : hip_fail(e, "segment-probe kernel launch");
}

int smol_csum_tool_field_scatter(smol_csum_ctx_t* ctx, uint8_t* d_buf, uint64_t bytes, const uint64_t* d_addrs,
                                 const uint16_t* d_vals, uint64_t n, int flags, void* stream) {
    if (!ctx || !d_buf || (n && (!d_addrs || !d_vals)) || (flags & ~15) || n > (0xFFFFFFull << 8)) return SMOL_EINVAL;
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return hip_fail(hipErrorInvalidDevice, "hipSetDevice");
    hipError_t e = launch_field_scatter(d_buf, bytes, d_addrs, d_vals, n, flags & 15, (hipStream_t)stream);
    return e == hipSuccess ? SMOL_OK : hip_fail(e, "field-scatter kernel launch");
}

int smol_csum_tool_auto_shape(uint32_t len, int has_desc) {
    // the walk kernel's verify shape (descriptor batches: its variant 13, which serves them when the
    // descriptor walk does not: NHC, data, forced variants)
    const int v = has_desc ? walk_variant(MODE_VERIFY, true) : auto_variant(MODE_VERIFY, false);
    return auto_shape(len, has_desc != 0, line_grid(v), v);
}

const char* smol_csum_tool_kernel_name(const smol_csum_ctx_t* ctx, int op, int has_desc) {
    // Without the batch this cannot see its record length: it answers for a batch that no
    // length-dependent kernel serves (descriptor batches exactly; fixed-stride batches the walk kernel's
    // lengths).  smol_csum_tool_kernel_for takes the batch.
    if (!ctx || op < MODE_DATA || op > MODE_COPY) return "";
    smol_csum_batch_t b;
    std::memset(&b, 0, sizeof b);
    b.n = 1;
    b.len = b.stride = 64;
    b.desc = has_desc ? reinterpret_cast<const smol_csum_desc_t*>(ctx->dummy) : nullptr;
    return smol_csum_tool_kernel_for(ctx, op, &b);
}

const char* smol_csum_tool_kernel_for(const smol_csum_ctx_t* ctx, int op, const smol_csum_batch_t* b) {
    if (!ctx || !b || op < MODE_DATA || op > MODE_COPY) return "";
    KParams p;
    std::memset(&p, 0, sizeof p);
    p.desc = b->desc;
    p.n = b->n;
    p.stride = b->stride;
    p.len = b->len;
    return family_kernel(pick_kernel(ctx, op, b, p));
}

uint32_t smol_csum_tool_last_launch(void) { return g_last_launch.load(std::memory_order_relaxed); }

}  // extern "C"
