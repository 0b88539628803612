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
    int defer_emit;       // -1 automatic, 0 field stores in the read pass, 1 two-pass emit
    uint64_t* patch;      // two-pass emit workspace: one meta word per record of a chunk
    uint8_t* lines;       // two-pass emit workspace: one 128-B line slot per record of a chunk
    uint64_t patch_cap;   // records the workspace holds
    int tile_records;     // tile kernel: records per wavefront tile (32 or 64)
    bool max_blocks_set;  // grid cap given explicitly (tooling)
};

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

inline uint16_t fold_u32(uint32_t w) {  // propagate_carries, src/wire/ip.rs:767-770
    uint32_t s = (w >> 16) + (w & 0xffffu);
    return (uint16_t)(((s >> 16) + s) & 0xffffu);
}

inline uint16_t swap16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }

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
int walk_variant(int mode, bool has_desc) { return mode == MODE_EMIT && has_desc ? 1 : 5; }
int auto_variant(int mode, bool has_desc) { return mode == MODE_EMIT && has_desc ? 7 : 5; }

bool line_grid(int variant) { return variant == 5 || variant == 6 || variant == 9 || variant == 10; }

int auto_shape(uint32_t len, bool has_desc, bool line = false) {
    if (has_desc) return CFG_G16U3;
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
    if (b->desc) {
        if (((uintptr_t)b->desc & 15u) != 0) return SMOL_EINVAL;
    } else if (b->len > SMOL_MAX_RECORD_LEN) {
        return SMOL_ERANGE;
    }
    return SMOL_OK;
}

// Two-pass emit workspace: records per chunk (8-B meta word + 128-B line slot each: 136 MiB).
constexpr uint64_t SMOL_EMIT_CHUNK = 1ull << 20;
constexpr uint64_t kLineSlot = 128;

int reserve_patch(smol_csum_ctx_t* ctx, uint64_t n) {
    if (n <= ctx->patch_cap) return SMOL_OK;
    DeviceGuard guard(ctx->device);
    if (ctx->patch) (void)hipFree(ctx->patch);
    if (ctx->lines) (void)hipFree(ctx->lines);
    ctx->patch = nullptr;
    ctx->lines = nullptr;
    ctx->patch_cap = 0;
    hipError_t e = hipMalloc(&ctx->patch, n * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc(&ctx->lines, n * kLineSlot);
    if (e != hipSuccess) {
        if (ctx->patch) (void)hipFree(ctx->patch);
        ctx->patch = nullptr;
        ctx->lines = nullptr;
        return hip_fail(e, "hipMalloc (emit workspace)");
    }
    ctx->patch_cap = n;
    return SMOL_OK;
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
    p.kind = d_addrs ? KIND_NHC_UDP : b->kind;
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
    DeviceGuard guard(ctx->device);
    if (!guard.ok) return hip_fail(hipErrorInvalidDevice, "hipSetDevice");
    // Variants: 0-2, 5-6 = walk kernel (csum_walk.h VarT: load policy, prefetch, chunk
    // grid), 3-4, 7 = tile kernel (csum_tile.hip: nt / plain loads, nt on the line grid), IP emit
    // and verify only; 8 = walk kernel without prefetch, copy-emit only (its default; other modes
    // run variant 0 for it).
    int variant = ctx->variant;
    const bool has_desc = b->desc != nullptr;
    if (variant < 0) variant = auto_variant(mode, has_desc);
    const bool tile_var = variant == 3 || variant == 4 || variant == 7;  // tile kernel: nt / plain / nt line grid
    if (tile_var && (mode == MODE_DATA || mode == MODE_COPY || d_addrs)) variant = walk_variant(mode, has_desc);
    const bool use_tile = variant == 3 || variant == 4 || variant == 7;
    int shape = ctx->shape >= 0 ? ctx->shape : auto_shape(b->len, has_desc, line_grid(variant));
    // Two-pass emit only on request: it trades the in-pass 2-byte stores for a meta word + line
    // slot per record and a scatter pass, and measured slower (C2: read pass 0.301 ms + scatter
    // 0.047 ms against 0.315 ms in one pass; the slot writes alone cost 0.049 ms).
    const bool two_pass = ctx->defer_emit == 1 && !d_addrs;
    const hipStream_t s = (hipStream_t)stream;
    if (mode == MODE_COPY) {  // one fused pass; the walk kernel only (no tile / deferred variants)
        hipError_t e = launch_csum(MODE_COPY, shape, ctx->variant == 1 ? 1 : 8, p, ctx->max_blocks, s);
        if (e != hipSuccess) return hip_fail(e, "copy-emit kernel launch");
        return SMOL_OK;
    }
    if (use_tile && !(mode == MODE_EMIT && two_pass)) {
        hipError_t e = launch_tile(mode, shape, variant == 7 ? 2 : variant - 3, ctx->tile_records, p, ctx->max_blocks, s);
        if (e != hipSuccess) return hip_fail(e, "checksum kernel launch");
        return SMOL_OK;
    }
    if (use_tile) variant = 0;
    if (mode != MODE_EMIT || !two_pass) {
        hipError_t e = launch_csum(mode, shape, variant, p, ctx->max_blocks, s);
        if (e != hipSuccess) return hip_fail(e, "checksum kernel launch");
        return SMOL_OK;
    }
    // Two-pass emit: read pass -> meta words (+ line slots), then the scatter pass, in chunks of at
    // most SMOL_EMIT_CHUNK records (the workspace is reserved once per context).  The first record
    // of a chunk hands over lines only when they lie inside it (the scatter pass cannot see the
    // previous chunk's meta words).
    const uint64_t cap = b->n < SMOL_EMIT_CHUNK ? b->n : SMOL_EMIT_CHUNK;
    int rc = reserve_patch(ctx, cap);
    if (rc != SMOL_OK) return rc;
    for (uint64_t start = 0; start < b->n; start += cap) {
        KParams q = p;
        q.n = (b->n - start) < cap ? (b->n - start) : cap;
        if (b->desc) q.desc = b->desc + start;
        else q.buf = d_buf + start * b->stride;
        if (d_status) q.status = d_status + start;
        q.patch = ctx->patch;
        q.lines = ctx->lines;
        hipError_t e = launch_csum(MODE_EMIT, shape, variant, q, ctx->max_blocks, s);
        if (e != hipSuccess) return hip_fail(e, "checksum kernel launch");
        e = launch_scatter(q, ctx->max_blocks, s);
        if (e != hipSuccess) return hip_fail(e, "scatter kernel launch");
    }
    return SMOL_OK;
}

}  // namespace

extern "C" {

// ---- scalar host mirrors --------------------------------------------------------------------

// checksum::data, src/wire/ip.rs:773-804.  Little-endian u16 words are summed exactly in 64 bits
// and truncated to 32 bits, which equals the reference's wrapping u32 accumulator.
uint16_t smol_csum_data(const uint8_t* d, size_t n) {
    uint64_t acc = 0;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t q;
        std::memcpy(&q, d + i, 8);
        acc += (q & 0xffffu) + ((q >> 16) & 0xffffu) + ((q >> 32) & 0xffffu) + (q >> 48);
    }
    for (; i + 2 <= n; i += 2) acc += (uint32_t)d[i] | ((uint32_t)d[i + 1] << 8);
    if (i < n) acc += d[i];
    return swap16(fold_u32((uint32_t)acc));
}

// checksum::combine, src/wire/ip.rs:807-813
uint16_t smol_csum_combine(const uint16_t* c, size_t n) {
    uint32_t acc = 0;
    for (size_t i = 0; i < n; i++) acc += c[i];
    return fold_u32(acc);
}

static uint16_t pseudo(const uint8_t* src, const uint8_t* dst, size_t alen, uint8_t nh,
                       uint32_t length) {
    const uint8_t pl[4] = {0, nh, (uint8_t)(length >> 8), (uint8_t)length};
    const uint16_t parts[3] = {smol_csum_data(src, alen), smol_csum_data(dst, alen),
                               smol_csum_data(pl, 4)};
    return smol_csum_combine(parts, 3);
}

// checksum::pseudo_header_v4, src/wire/ip.rs:816-831
uint16_t smol_csum_pseudo_header_v4(const uint8_t src[4], const uint8_t dst[4], uint8_t nh,
                                    uint32_t length) {
    return pseudo(src, dst, 4, nh, length);
}

// checksum::pseudo_header_v6, src/wire/ip.rs:834-849
uint16_t smol_csum_pseudo_header_v6(const uint8_t src[16], const uint8_t dst[16], uint8_t nh,
                                    uint32_t length) {
    return pseudo(src, dst, 16, nh, length);
}

// checksum::pseudo_header, src/wire/ip.rs:851-869
int smol_csum_pseudo_header(int src_family, const uint8_t* src, int dst_family,
                            const uint8_t* dst, uint8_t nh, uint32_t length, uint16_t* out) {
    if (!src || !dst || !out || src_family != dst_family) return SMOL_EINVAL;
    if (src_family == 4) { *out = smol_csum_pseudo_header_v4(src, dst, nh, length); return SMOL_OK; }
    if (src_family == 6) { *out = smol_csum_pseudo_header_v6(src, dst, nh, length); return SMOL_OK; }
    return SMOL_EINVAL;
}

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
    auto* c = new (std::nothrow) smol_csum_ctx;
    if (!c) {
        (void)hipFree(dummy);
        return SMOL_ENOMEM;
    }
    c->dummy = dummy;
    c->defer_emit = -1;
    c->tile_records = 32;
    c->max_blocks_set = false;
    c->lines = nullptr;
    c->patch = nullptr;
    c->patch_cap = 0;
    c->device = device;
    c->num_cu = cus;
    c->max_blocks = kNaturalGrid;
    c->shape = -1;
    c->variant = -1;
    *out = c;
    return SMOL_OK;
}

int smol_csum_ctx_reserve(smol_csum_ctx_t* ctx, uint64_t max_records) {
    if (!ctx) return SMOL_EINVAL;
    return reserve_patch(ctx, max_records < SMOL_EMIT_CHUNK ? max_records : SMOL_EMIT_CHUNK);
}

int smol_csum_ctx_destroy(smol_csum_ctx_t* ctx) {
    if (!ctx) return SMOL_OK;
    {
        DeviceGuard guard(ctx->device);
        (void)hipFree(ctx->dummy);
        if (ctx->patch) (void)hipFree(ctx->patch);
        if (ctx->lines) (void)hipFree(ctx->lines);
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

int smol_csum_tool_set_variant(smol_csum_ctx_t* ctx, int variant) {
    if (!ctx || variant < -1 || variant > 10) return SMOL_EINVAL;
    ctx->variant = variant;
    return SMOL_OK;
}

int smol_csum_tool_set_tile(smol_csum_ctx_t* ctx, int records) {
    if (!ctx || (records != 32 && records != 64)) return SMOL_EINVAL;
    ctx->tile_records = records;
    return SMOL_OK;
}

int smol_csum_tool_set_deferred_emit(smol_csum_ctx_t* ctx, int mode) {
    if (!ctx || mode < -1 || mode > 1) return SMOL_EINVAL;
    ctx->defer_emit = mode;
    return SMOL_OK;
}

int smol_csum_tool_set_max_blocks(smol_csum_ctx_t* ctx, uint32_t max_blocks) {
    if (!ctx) return SMOL_EINVAL;
    ctx->max_blocks = max_blocks ? max_blocks : kNaturalGrid;
    ctx->max_blocks_set = max_blocks != 0;
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

int smol_csum_tool_auto_shape(uint32_t len, int has_desc) {
    return auto_shape(len, has_desc != 0, line_grid(auto_variant(MODE_VERIFY, has_desc != 0)));
}

const char* smol_csum_tool_kernel_name(const smol_csum_ctx_t* ctx, int op, int has_desc) {
    if (!ctx || op < MODE_DATA || op > MODE_COPY) return "";
    const int v = ctx->variant >= 0 ? ctx->variant : auto_variant(op, has_desc != 0);
    const bool tile = (v == 3 || v == 4 || v == 7) && (op == MODE_EMIT || op == MODE_VERIFY) &&
                      !(op == MODE_EMIT && ctx->defer_emit == 1);
    return tile ? "csum_tile_kernel" : "csum_kernel";
}

}  // extern "C"
