/*
 * smolcsum_tools.h — benchmark / test tooling exported by libsmolcsum.so.  NOT part of the
 * drop-in boundary (that is include/smolcsum.h): synthetic packet batches generated on the
 * device (the 8 x 128 M x 1500 B configuration needs ~190 GB per GPU, which only the device can
 * produce in reasonable time), single-bit fault injection following phy::FaultInjector's recipe
 * (src/phy/fault_injector.rs:8-16,45-51), and a launch-shape override for tuning.
 */
#ifndef SMOLCSUM_TOOLS_H
#define SMOLCSUM_TOOLS_H

#include "smolcsum.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
    SMOL_SYNTH_UDP4 = 0,     /* IPv4 (IHL 5, DF, TTL 64) + UDP (length = record - 20) + payload */
    SMOL_SYNTH_TCP4 = 1,     /* IPv4 + TCP (20-byte header, ACK|PSH) + payload                  */
    SMOL_SYNTH_V6MIX = 2,    /* IPv6 + TCP / UDP / ICMPv6 echo, round-robin by record index     */
    SMOL_SYNTH_ETH_TCP4 = 3, /* Ethernet II + IPv4 + TCP (Medium::Ethernet frames)              */
    SMOL_SYNTH_RANDOM = 4    /* random bytes only                                               */
};

/* Fill every record of `batch` (device buffer) with a synthetic packet of the given profile;
 * all checksum fields are written as 0 (what Repr::emit writes when the device offloads).
 * Payload bytes are splitmix64(seed, position).  Deterministic for a given (batch, seed). */
int smol_csum_tool_synth(smol_csum_ctx_t* ctx, uint8_t* d_buf, const smol_csum_batch_t* batch,
                         int profile, uint64_t seed, void* stream);

/* Flip one bit in every `every`-th record (records i with i % every == 0), at a byte index and
 * bit drawn from xorshift32 seeded by (seed, i) — FaultInjector::corrupt's recipe. */
int smol_csum_tool_corrupt(smol_csum_ctx_t* ctx, uint8_t* d_buf, const smol_csum_batch_t* batch,
                           uint32_t every, uint64_t seed, void* stream);

/* Force a launch shape for the next batched calls on this context (-1 = automatic).  A shape is
 * (lanes per record) x (16-byte chunks per lane per step):
 * 0: 8 x 6, 1: 16 x 3, 2: 16 x 6, 3: 32 x 3, 4: 32 x 4, 5: 64 x 2, 6: 64 x 4, 7: 8 x 7, 8: 16 x 4. */
int smol_csum_tool_set_shape(smol_csum_ctx_t* ctx, int shape);

/* Kernel variant (-1 = automatic; since round 5: 63 for verify over descriptor batches, the
 * descriptor walk with cached header windows (csum_dwalk.hip; 60 = its non-temporal-window verify),
 * 41 for emit over them (63 with the window's chunks summed from LDS); for fixed-stride batches 57 (emit of packed 1400-1580-B records not multiples of 64 B:
 * the transposed walk with its field segments stored non-temporal), 47 (the transposed walk with
 * whole field segments: verify of packed 1473-1665-B records not multiples of 128 B, verify / emit
 * of 1666-8065-B records), 39 (other fixed-stride emit: variant 5 with whole field segments), 44
 * (47 / 57 under SMOL_BATCH_FIELD_STORES), 5 otherwise; 13 for NHC / data over descriptors; 21 for
 * copy-emit.  The product library runs these and 7 / 17; libsmolcsum_exp.so every variant below
 * (csum_api.cpp variant_built).  Round 1-4 meanings: 7 was emit over descriptor batches, 13 verify
 * over them, 29 fixed-stride emit.)  The
 * "walk" kernel (a group parses and finishes its own record) reads 16-byte chunks on a grid that
 * starts at the record's 16-byte boundary: 0 = non-temporal loads + register prefetch of the next
 * step, 1 = plain (cached) loads + prefetch, 2 = non-temporal loads without prefetch; or at its
 * 128-byte line boundary: 5 = non-temporal loads + prefetch, 6 = plain loads + prefetch.
 * 3 / 4 = the "tile" kernel (groups only stream and sum, lanes finish 64 records at once) with
 * non-temporal / plain loads on the 16-byte grid, 7 = the tile kernel with non-temporal loads on
 * the line grid — emit and verify only (data() uses the walk kernel).  8 = the walk kernel on the
 * 16-byte grid with plain loads and no prefetch.  9 / 10 = variant 5 with the first two / the first
 * 16-byte chunk of every lane's step loaded cached, so that the lines holding the fields are
 * resident in L2 when emit stores them (fixed-stride emit only; elsewhere 5).  13 = variant 5
 * without the prefetch.  19 = variant 5 whose emit writes the 64-byte segments holding an IPv4
 * record's fields whole where no neighbouring record's field shares them (fixed-stride emit;
 * elsewhere 5); 29 = 19 behind a wavefront ballot that skips the segment logic for steps without
 * an IPv4 record (the default for fixed-stride emit).  23-28 = whole-segment emit generalised to
 * any record extents (descriptor batches; csum_walk.h).  Copy-emit: 1 / 8 / 11 / 16 = the walk
 * kernel in its copy mode (prefetch / two aligned source chunks / one chunk + the next lane's /
 * dword-aligned source + one dword from the next lane); 17 = copy_kernel (csum_copy.hip), whose
 * shapes are 16 x 4 with 32 body chunks in round 1 (default, shape 8), 16 x 3 (1), 8 x 6 (0),
 * 8 x 4 (7), 16 x 5 (2), 16 x 4 with the body chunks of round 1 built the generic way (3),
 * 32 x 2 (4), 64 x 2 (5, 6); 21 (default) = 17 with the first body round's loads issued ahead of
 * round 1's stores (16 x 4 with 32 body chunks in round 1; shape 2: 16 x 5 with 16). */
int smol_csum_tool_set_variant(smol_csum_ctx_t* ctx, int variant);

/* Tile kernel: records per wavefront tile, 32 (default) or 64. */
int smol_csum_tool_set_tile(smol_csum_ctx_t* ctx, int records);

/* Cap the number of workgroups per launch (0 = automatic: CUs x 8). */
int smol_csum_tool_set_max_blocks(smol_csum_ctx_t* ctx, uint32_t max_blocks);

/* Walk-, tile- and copy-kernel launches with on = 1 map workgroup b to the records of workgroup xcd_block(b)
 * (csum_launch.h): the workgroups that share an XCD take one contiguous range of the batch.  on = K
 * >= 2: the XCDs take turns over runs of K workgroups (xcd_chunk).  0: the natural order.  -1 (the
 * default): the library's choice (contiguous for fixed-stride emit over >= 4 GiB, runs of 256 for
 * fixed-stride verify over >= 64 GiB, the dispatch order otherwise). */
int smol_csum_tool_set_xcd_remap(smol_csum_ctx_t* ctx, int on);

/* Batched calls over more than `records` records (0: no limit, the default) go out as consecutive
 * kernel launches of at most `records` records each, on the same stream. */
int smol_csum_tool_set_launch_records(smol_csum_ctx_t* ctx, uint64_t records);

/* Read-only HBM streaming probe over `bytes` (multiple of 16, 16-byte aligned `d_buf`): the
 * achievable read ceiling that the checksum kernels are compared with.  Each wavefront streams
 * contiguous 8-KiB pieces with eight non-temporal 16-byte loads per lane in flight (the fastest
 * pattern of tools/probe_bw.hip), 8 workgroups per CU.  `d_sink` is one u32. */
int smol_csum_tool_stream_read(smol_csum_ctx_t* ctx, const uint8_t* d_buf, uint64_t bytes,
                               uint32_t* d_sink, void* stream);

/* Emit's floor probe: the stream-read probe over `bytes` plus emit's store events — a big-endian
 * 2-byte store at record offsets f1 and f2 (f2 = 0xFFFFFFFF: none) of every record starting at a
 * multiple of `stride`, issued right after the 8-KiB piece holding the record's first byte has
 * been read.  Overwrites those bytes.  The floor of an emit that stores its fields as 2-byte
 * writes (fixed-stride emit writes whole 64-byte field segments where it can, and runs under it). */
int smol_csum_tool_field_probe(smol_csum_ctx_t* ctx, uint8_t* d_buf, uint64_t bytes, uint64_t stride,
                               uint32_t f1, uint32_t f2, void* stream);
/* The same probe with the store addresses listed (descriptor batches): `d_addrs` holds ascending
 * byte offsets into the buffer of 2-byte stores, and `d_piece_first[j]` the index of the first of them
 * at or after byte 8192 * j, for j = 0 .. ceil(bytes / 8192) (that many + 1 entries).  Overwrites
 * the bytes at those offsets.  `flags` bit 0: instead rewrite the whole 64-byte segment holding each
 * offset with the values it holds (the store shape of whole-segment emit; nothing changes). */
int smol_csum_tool_field_probe_list(smol_csum_ctx_t* ctx, uint8_t* d_buf, uint64_t bytes, const uint64_t* d_addrs,
                                    const uint32_t* d_piece_first, int flags, void* stream);
/* Emit's floor in emit's store shape: the stream-read probe over `bytes`, and every 64-byte segment
 * whose bit is set in `d_bitmap` (one bit per 64-byte segment of the buffer: bit s % 32 of word s / 32;
 * ceil(bytes / 8192) * 4 words, 16-byte aligned) written back whole with the bytes just read, by the
 * lanes that loaded it, right after the 8-KiB piece holding it has been read (nothing changes).
 * `flags` bit 0: the segments stored non-temporal.  Segments in the tail past the last whole 8-KiB
 * piece are read, not written. */
int smol_csum_tool_segment_probe(smol_csum_ctx_t* ctx, uint8_t* d_buf, uint64_t bytes, const uint32_t* d_bitmap, int flags,
                                 void* stream);
/* A separate store pass (experiments: what emit's field stores cost outside the read stream):
 * for i < n, the big-endian 2-byte value d_vals[i] at byte offset d_addrs[i] of the buffer, one
 * thread per store.  `flags` bit 0: non-temporal stores; bits 1 / 2 / 3: instead write the whole
 * aligned 64-byte segment / 32-byte sector / 128-byte line holding the offset (the value repeated: a
 * timing probe, the bytes change). */
int smol_csum_tool_field_scatter(smol_csum_ctx_t* ctx, uint8_t* d_buf, uint64_t bytes, const uint64_t* d_addrs,
                                 const uint16_t* d_vals, uint64_t n, int flags, void* stream);
/* The launch shape the library picks for a verify over an implicit batch of `len`-byte records. */
int smol_csum_tool_auto_shape(uint32_t len, int has_desc);

/* The kernel (the rocprofv3 name prefix: "csum_kernel", "csum_tile_kernel", "xwalk_kernel",
 * "dwalk_kernel", "copy_kernel" or "xcopy_kernel") that an IP-path operation on `batch` runs with this
 * context's variant setting: op 0 data, 1 emit, 2 verify, 3 copy-emit.  The same choice as the
 * batched entry points make (one dispatch function, csum_api.cpp pick_kernel). */
const char* smol_csum_tool_kernel_for(const smol_csum_ctx_t* ctx, int op, const smol_csum_batch_t* batch);
/* Deprecated (kept for old scripts): smol_csum_tool_kernel_for without the batch, so without its record
 * length — exact for descriptor batches; for fixed-stride batches it names the kernel of short records,
 * not the transposed walk that serves 1400-8065-B ones.  Use smol_csum_tool_kernel_for or
 * smol_csum_tool_last_launch. */
const char* smol_csum_tool_kernel_name(const smol_csum_ctx_t* ctx, int op, int has_desc);

/* The kernel instantiation of this process's last checksum launch (any context), packed as
 * kernel << 24 | variant << 16 | G << 8 | U; kernel 1 = csum_kernel, 2 = csum_tile_kernel,
 * 3 = copy_kernel, 4 = csum_kernel with the 6LoWPAN NHC gates, 5 = xwalk_kernel, 6 = dwalk_kernel;
 * 0 before the first launch. */
uint32_t smol_csum_tool_last_launch(void);

/* 1 when this build of the library runs kernel variant `variant` (smol_csum_tool_set_variant), else
 * 0.  The product library carries the defaults and one fallback per operation; the experiments
 * build (`make -C smoltcp_amd/csrc EXP=1`, libsmolcsum_exp.so) every measured variant. */
int smol_csum_tool_variant_built(int variant);

#ifdef __cplusplus
}
#endif

#endif /* SMOLCSUM_TOOLS_H */
