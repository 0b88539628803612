// Batched Internet-checksum kernels for MI355X (gfx950).
//
// One GROUP of G lanes (G = 8, 16, 32 or 64; a group never spans two wavefronts) owns one record
// at a time and walks the batch with a grid stride (with the default natural grid every group
// owns exactly one record).  The record's bytes are read as ALIGNED 16-byte chunks with
// global_load_dwordx4 (lane-contiguous, fully coalesced), U chunks per lane per step, so a step
// moves G*U*16 bytes.  The chunk grid starts either at the record's 16-byte boundary or at its
// 128-byte cache-line boundary (LINE variants): with non-temporal loads a record's first and last
// lines must be requested whole, or the neighbouring group's request for the rest of the line
// fetches it from HBM a second time (tools/probe_bw.hip `rec_walk`: 16-B grid + nt 5.8 TB/s,
// line grid + nt 7.3 TB/s).  The next step — or the next record's first step — is issued before
// the current one is summed, into a second register set: the loop body is written once and
// instantiated twice with the two sets' roles swapped (no register copies, so the compiler's
// counted s_waitcnt vmcnt leaves the prefetch in flight).  Every load instruction is issued
// unconditionally (out-of-range chunks read a 16-byte dummy line) for the same reason: a load
// inside a branch makes hipcc fall back to vmcnt(0).  Bytes of a chunk outside the summed span are
// masked; an aligned chunk never crosses a page, so reading the bytes around a record is safe.
//
// Small groups amortise the per-record work (header parse, reductions, the finishing lane) over
// several records per wavefront: at 1500-byte records a G=8 wave finishes eight records per step.
//
// The first WIN bytes of the chunk grid (128, or 256 on the line grid: at least the record's
// first 128 bytes, already in registers) are copied to a per-group LDS window, from which every
// lane reads the IP/L4 header fields the gates need; L4 header bytes past the window (behind a
// long IPv6 Hop-by-Hop header) are read from global memory.  Per lane the protocol kernels add
// aligned u16 words (v_sad_u16); DPP row reductions combine the group; one lane finishes the
// record: fold, byte-swap for an odd record start (RFC 1071 §2(B)), pseudo-header, gate, write.
//
// Emit writes two 2-byte fields per record (three for an ICMPv4 error message: the embedded IPv4
// header's too).  In place, each is a partial-line write that HBM merges with a read-modify-write,
// interleaved with the read stream (tools/probe_wr.hip: ~0.1 ms per 2^20 records at 1.5 KB).
//
// See csum_device.h for the arithmetic and the reference lines each rule follows.
//
// This header holds the kernel templates; the csum_walk_*.hip translation units instantiate them
// per (mode, batch form) so that the build compiles them in parallel.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csum_device.h"
#include "csum_launch.h"

namespace smolcsum {

// Kernel variants: load cache policy, register prefetch, chunk-grid alignment.
// 0 = nt + prefetch, 1 = plain + prefetch, 2 = nt without prefetch, 8 = plain without prefetch
// (16-byte grid); 5 = nt + prefetch, 6 = plain + prefetch (128-byte line grid).  3 / 4 / 7 are the
// tile kernel.
// 9 / 10 = variant 5 with the first two / the first chunk of every lane's step loaded cached
// (fixed-stride emit only: the 128-B line(s) holding the two fields stay resident in L2 when the
// field stores arrive; measured in DESIGN.md §5).
// 13 = variant 5 without the register prefetch.
// MODE_COPY (16-byte grid, plain loads, no register prefetch): 8 = two aligned source chunks per
// destination chunk; 11 = one, the second taken from the next lane of the group (DPP /
// ds_bpermute); 16 (the default) = variant 11 with dword-aligned source loads — a lane loads the 16
// source bytes from its chunk's first source byte rounded down to 4 (an unaligned 16-byte load), so
// the funnel is four v_alignbyte and only ONE dword comes from the next lane — and every byte of
// the record written (WHOLE, see walk_step).  Measured variants that lost are in DESIGN.md §6.
// Experiment variants (the experiments build, SMOL_EXP, only): emit walks shaped like verify's.
// 31 = 5 with the geometry in LDS and no shared_from; 32 = 29 with both; 33 = 29 with the geometry
// in LDS; 34 = 29 without shared_from; 35 = 5 without shared_from; 36 = 5 with the geometry in LDS.
// VAR | 64 (experiments): the same kernel with every global store of emit compiled out (the values
// computed and kept live, nothing written; wrong bytes, timing only).
template <int VAR_>
struct VarT {
    static constexpr int VAR = VAR_ & 63;
    static constexpr bool NOSTORE = (VAR_ & 64) != 0;
    static constexpr bool GLDS = VAR == 31 || VAR == 32 || VAR == 33 || VAR == 36;
    // 37 / 38: variant 5 with whole field segments decided by one ballot (BSEG; 38 also IPv6 records)
    // 39: variant 29 on a wavefront that holds an IPv4 record, 38's ballot decision on one that holds
    // none (BSEG_NO4: IPv6 records get whole segments too)
    // 12 / 14 (experiments build): 39 with the header lines (chunks u < 2 of a step: the LDS window)
    // loaded with the default cache policy, at a group's first load only (12) or at every step (14),
    // so that the field stores hit lines the L2 holds
    static constexpr bool BSEG = VAR == 37 || VAR == 38 || VAR == 39 || VAR == 40 || VAR == 12 || VAR == 14;
    static constexpr bool BSEG6 = VAR == 38 || VAR == 39 || VAR == 40 || VAR == 12 || VAR == 14;
    static constexpr bool BSEG_NO4 = VAR == 39 || VAR == 40 || VAR == 12 || VAR == 14;
    static constexpr int CU0 = VAR == 12 ? 2 : 0;
    // 40 (experiments build): 39 with the whole segments stored non-temporal (round 5: plain nt, lost;
    // since late round 6 write-through, sc1 nt, as the transposed walk's variant 101)
    static constexpr bool NTSEG = VAR == 40;
    static constexpr bool NOSHARE = VAR == 31 || VAR == 32 || VAR == 34 || VAR == 35;
    static constexpr int BASE = (VAR == 31 || VAR == 35 || VAR == 36 || VAR == 37 || VAR == 38) ? 5
                                : ((VAR >= 32 && VAR <= 34) || VAR == 39 || VAR == 40 || VAR == 12 || VAR == 14) ? 29 : VAR;
    static constexpr bool NT = VAR == 0 || VAR == 2 || VAR == 5 || VAR == 9 || VAR == 10 || VAR == 13 || VAR == 19 ||
                               (VAR >= 23 && VAR <= 29) || (VAR >= 31 && VAR <= 40) || VAR == 12 || VAR == 14;
    static constexpr bool PF = VAR != 2 && VAR != 8 && VAR != 11 && VAR != 13 && VAR != 16 && VAR != 26 && VAR != 27 &&
                               VAR != 28;
    static constexpr bool LINE = VAR == 5 || VAR == 6 || VAR == 9 || VAR == 10 || VAR == 13 || VAR == 19 ||
                                 (VAR >= 23 && VAR <= 29) || (VAR >= 31 && VAR <= 40) || VAR == 12 || VAR == 14;
    static constexpr int CACHED_U = (VAR == 9 || VAR == 14) ? 2 : VAR == 10 ? 1 : 0;
    static constexpr bool SHUF = VAR == 11 || VAR == 16;
    static constexpr bool WHOLE = VAR == 16;
    static constexpr bool SHUF2 = VAR == 16;
    static constexpr bool SEGW = VAR == 19 || BASE == 29;  // variant 5 + whole 64-B field segments (fixed-stride emit, walk_step)
    // SEGOPT bit 0 (29): the segment machinery skipped on wavefronts that hold no IPv4 record (a
    // ballot after the parse: IPv6 records have one field and keep the 2-B store).  (Round 4 also
    // measured the segments stored non-temporal: C2 emit 0.303 against 0.296 ms; removed.)
    static constexpr int SEGOPT = BASE == 29 ? 1 : 0;
    // 23-27 (emit): whole 64-B field segments with the neighbours' record extents published too, so
    // that they serve descriptor batches as well as fixed strides (SEGG); SEGB: the neighbours of the
    // whole workgroup, not only of the wavefront (a workgroup barrier after the parse, natural grid);
    // SEG6: IPv6 records too.  23 = 5 + SEGG + SEGB + SEG6, 24 = 23 without SEGB, 25 = 23 without
    // SEG6, 26 = 13 (no prefetch) + SEGG + SEGB + SEG6, 27 = 26 without SEGB, 28 = 27 compiled for
    // variant 13's occupancy (MinWaves).
    static constexpr bool SEGG = VAR >= 23 && VAR <= 28;
    static constexpr bool SEGB = VAR == 23 || VAR == 25 || VAR == 26;
    static constexpr bool SEG6 = VAR == 23 || VAR == 24 || VAR == 26 || VAR == 27 || VAR == 28;
};

template <bool LINE>
struct Grid {
    static constexpr uint64_t ALIGN = LINE ? 128 : 16;  // chunk-grid origin: record start rounded down
    static constexpr int WIN = LINE ? 256 : 128;        // LDS window bytes (from the grid origin)
    static constexpr int WIN_CH = WIN / 16;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Every device-memory access goes through an address_space(1) pointer so that hipcc emits
// global_load / global_store.  Record addresses are computed as integers; a plain (generic)
// pointer made from them would become flat_load_*, which counts on both vmcnt and lgkmcnt and
// makes the compiler drain every load with vmcnt(0) lgkmcnt(0) — no load pipelining at all.
#define GMEM __attribute__((address_space(1)))
typedef const GMEM u32x4* gcv4;
typedef const GMEM uint8_t* gcu8;
typedef GMEM uint8_t* gu8;
typedef GMEM uint16_t* gu16;

struct RecRef {
    uint64_t a0;  // absolute address of the record's first byte
    uint32_t len;
    uint32_t kind;  // SMOL_KIND_*; MODE_COPY adds KIND_BAD_COPY for a copy range that does not fit
    // MODE_COPY only: the record's payload [p0, p1) comes from sb + offset (sb = source address of
    // record offset 0, i.e. src + src_offset - dst_offset)
    uint64_t sb;
    uint32_t p0, p1;
};

constexpr uint32_t KIND_BAD_COPY = 0x100;

template <bool IMPLICIT, bool COPY, bool NHC = false>
__device__ __forceinline__ RecRef rec_at(const KParams& p, uint64_t r) {
    RecRef rr;
    if (IMPLICIT) {
        rr.a0 = (uint64_t)p.buf + r * p.stride;
        rr.len = p.len;
        rr.kind = p.kind;
    } else {
        const u32x4 d = *(gcv4)((uint64_t)p.desc + 16 * r);
        rr.a0 = (uint64_t)p.buf + ((uint64_t)d.x | ((uint64_t)d.y << 32));
        rr.len = d.z;
        rr.kind = NHC ? KIND_NHC_UDP : desc_kind(d.w);  // NHC UDP entry points: every record
    }
    rr.sb = 0;
    rr.p0 = rr.p1 = 0;
    if (COPY) {
        const u32x4 c = *(gcv4)((uint64_t)p.copy + 16 * r);
        const uint64_t so = (uint64_t)c.x | ((uint64_t)c.y << 32);
        if ((uint64_t)c.z + c.w <= rr.len) {
            rr.p0 = c.z;
            rr.p1 = c.z + c.w;
            rr.sb = (uint64_t)p.src + so - c.z;
        } else {
            rr.kind |= KIND_BAD_COPY;
        }
    }
    return rr;
}

// Aligned chunks of the record's grid (from the grid origin to the chunk holding the last byte).
template <bool LINE>
__device__ __forceinline__ uint32_t n_chunks(const RecRef& rr) {
    if (rr.len == 0) return 0;
    return (uint32_t)(((rr.a0 + rr.len + 15) >> 4) - ((rr.a0 & ~(Grid<LINE>::ALIGN - 1)) >> 4));
}

template <bool NT>
__device__ __forceinline__ u32x4 ld16(gcv4 q) {
    if (NT) return __builtin_nontemporal_load(q);
    return *q;
}

// The registers of one step: U record chunks; MODE_COPY adds the two aligned source chunks that
// cover each destination chunk's payload bytes.
template <int U, bool COPY>
struct Regs {
    u32x4 v[U];
};
template <int U>
struct Regs<U, true> {
    u32x4 v[U], s0[U], s1[U];
    u32x4 sx;  // SHUF: lane 0's source chunk for the chunk after the step (the group's last lane needs it)
    uint32_t sx1;  // SHUF2: lane 0's first source dword of the chunk after the step
};

// Issue the U loads of one step.  Unconditional: chunks past the record (or a step that does
// not exist) read the dummy line instead.  MODE_COPY: chunks entirely inside the payload are not
// read from the record (they are replaced), and the source chunks are read only where they hold
// payload bytes (so no load ever leaves the source range's aligned chunks).
// Chunks at addresses >= lim are not loaded (they come from the next record's LDS window, see
// shared_from).
// SHUF (MODE_COPY): each lane loads the aligned source chunk under its chunk's first byte whenever it
// lies in the source range's aligned chunks, payload or not (its left neighbour may need it), and
// lane 0 also loads the one under the chunk after the step (sx).
// SHUF2 (MODE_COPY): the source load of chunk k starts at A = (its first source byte) & ~3 when
// [A, A + 16) lies inside the source range's aligned chunks [first, last + 16); otherwise (the
// payload's first / last chunk) at first / last, and the merge shifts it there.  Lane 0 also loads
// the dword at A of the chunk after the step (sx1), for the group's last lane.
template <int G, int U, bool NT, bool COPY, bool LINE, int CACHED_U = 0, bool SHUF = false, bool SHUF2 = false>
__device__ __forceinline__ void load_step(Regs<U, COPY>& R, const RecRef& rr, uint32_t nch,
                                          uint32_t step, int lane, bool valid, uint64_t dummy,
                                          uint64_t lim = ~0ull) {
    static_assert(!(COPY && LINE), "MODE_COPY uses the 16-byte grid");
    const uint64_t base = rr.a0 & ~(Grid<LINE>::ALIGN - 1);
    if constexpr (COPY && SHUF2) {
        const bool pay = valid && rr.p1 > rr.p0;
        const uint64_t first = (rr.sb + rr.p0) & ~15ull, last = (rr.sb + rr.p1 - 1) & ~15ull;
        const uint64_t sk = rr.sb - (rr.a0 - base);  // source address of chunk 0's byte 0
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = step * (G * U) + u * G + lane;
            const bool in = valid && k < nch;
            const int64_t pos = (int64_t)(16u * k) - (int64_t)(rr.a0 - base);
            const bool full = pos >= (int64_t)rr.p0 && pos + 16 <= (int64_t)rr.p1;
            R.v[u] = ld16<NT>((gcv4)(in && !full ? base + 16ull * k : dummy));
            const uint64_t sa = sk + 16ull * k, A = sa & ~3ull;
            const uint64_t la = A < first ? first : A > last ? last : A;
            R.s0[u] = ld16<NT>((gcv4)(pay && sa + 16 > first && A <= last + 12 ? la : dummy));
        }
        const uint64_t AX = (sk + 16ull * ((step + 1) * (G * U))) & ~3ull;
        R.sx1 = *(const GMEM uint32_t*)(pay && lane == 0 && AX >= first && AX <= last + 12 ? AX : dummy);
        return;
    }
    if constexpr (COPY && SHUF) {
        const bool pay = valid && rr.p1 > rr.p0;
        const uint64_t first = (rr.sb + rr.p0) & ~15ull, last = (rr.sb + rr.p1 - 1) & ~15ull;
        const uint64_t sk = rr.sb - (rr.a0 - base);  // source address of chunk 0's byte 0
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = step * (G * U) + u * G + lane;
            const bool in = valid && k < nch;
            const int64_t pos = (int64_t)(16u * k) - (int64_t)(rr.a0 - base);
            const bool full = pos >= (int64_t)rr.p0 && pos + 16 <= (int64_t)rr.p1;
            R.v[u] = ld16<NT>((gcv4)(in && !full ? base + 16ull * k : dummy));
            const uint64_t sA = (sk + 16ull * k) & ~15ull;
            R.s0[u] = ld16<NT>((gcv4)(pay && sA >= first && sA <= last ? sA : dummy));
        }
        const uint64_t sX = (sk + 16ull * ((step + 1) * (G * U))) & ~15ull;
        R.sx = ld16<NT>((gcv4)(pay && lane == 0 && (sk & 15u) && sX >= first && sX <= last ? sX : dummy));
        return;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t k = step * (G * U) + u * G + lane;
        const bool in = valid && k < nch && base + 16ull * k < lim;
        if constexpr (!COPY) {
            const gcv4 q = (gcv4)(in ? base + 16ull * k : dummy);
            R.v[u] = u < CACHED_U ? ld16<false>(q) : ld16<NT>(q);  // folds per unrolled u
        } else {
            const int64_t pos = (int64_t)(16u * k) - (int64_t)(rr.a0 & 15u);  // record offset of the chunk
            const bool full = pos >= (int64_t)rr.p0 && pos + 16 <= (int64_t)rr.p1;
            const bool pay = rr.p1 > rr.p0 && pos < (int64_t)rr.p1 && pos + 16 > (int64_t)rr.p0;
            R.v[u] = ld16<NT>((gcv4)(in && !full ? base + 16ull * k : dummy));
            const uint64_t sa = rr.sb + (uint64_t)pos;                 // source of the chunk's byte 0
            const uint64_t sA = sa & ~15ull;
            const uint64_t first = (rr.sb + rr.p0) & ~15ull;           // first / last aligned source
            const uint64_t last = (rr.sb + rr.p1 - 1) & ~15ull;        // chunks holding payload
            R.s0[u] = ld16<NT>((gcv4)(in && pay && sA >= first ? sA : dummy));
            R.s1[u] = ld16<NT>((gcv4)(in && pay && (sa & 15u) && sA + 16 <= last ? sA + 16 : dummy));
        }
    }
}

// Bytes sh .. sh+15 of the 32-byte pair (lo, hi), sh in [0, 16).
__device__ __forceinline__ u32x4 funnel16(const u32x4& lo, const u32x4& hi, uint32_t sh) {
    const uint32_t q = sh >> 2, b = sh & 3u;
    auto pick = [&](uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
        return q == 0 ? a0 : q == 1 ? a1 : q == 2 ? a2 : a3;
    };
    const uint32_t x0 = pick(lo.x, lo.y, lo.z, lo.w);
    const uint32_t x1 = pick(lo.y, lo.z, lo.w, hi.x);
    const uint32_t x2 = pick(lo.z, lo.w, hi.x, hi.y);
    const uint32_t x3 = pick(lo.w, hi.x, hi.y, hi.z);
    const uint32_t x4 = pick(hi.x, hi.y, hi.z, hi.w);
    u32x4 r;
    r.x = __builtin_amdgcn_alignbyte(x1, x0, b);
    r.y = __builtin_amdgcn_alignbyte(x2, x1, b);
    r.z = __builtin_amdgcn_alignbyte(x3, x2, b);
    r.w = __builtin_amdgcn_alignbyte(x4, x3, b);
    return r;
}

// Byte mask of dword i (bytes 4i .. 4i+3 of a chunk) for chunk-relative byte range [lo, hi).
__device__ __forceinline__ uint32_t byte_mask(int lo, int hi, int i) { return mask_dword(0xffffffffu, lo - 4 * i, hi - 4 * i); }

// One byte from global memory, waited for inside the asm statement.  Used only for header bytes
// outside the LDS window (behind a long IPv6 Hop-by-Hop header).  Hidden from the compiler on
// purpose: a compiler-visible conditional load here makes hipcc's wait insertion drain the
// prefetched steps with vmcnt(0) at the loop head for every record.
__device__ __forceinline__ uint32_t ld_byte_sync(uint64_t a) {
    uint32_t x;
    asm volatile("global_load_ubyte %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(a) : "memory");
    return x;
}

// The same for one aligned dword (the IPv6 addresses of 6LoWPAN NHC UDP records).
__device__ __forceinline__ uint32_t ld_u32_sync(uint64_t a) {
    uint32_t x;
    asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(a) : "memory");
    return x;
}

// Sum over the G lanes of a group (all of them active).  Rows of 16 lanes reduce with DPP
// (quad_perm xor1 / xor2, row_half_mirror, row_mirror), wider groups add ds_swizzle / bpermute.
template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, true);  // row_half_mirror
    if (G >= 16) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, true);  // row_mirror
    if (G >= 32) v += (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);  // lane ^ 16 within 32
    if (G >= 64) v += (uint32_t)__shfl_xor((int)v, 32, 64);
    return v;
}

// The value x of lane (lane + 1) mod G of the caller's group (every lane of the group active).
template <int G>
__device__ __forceinline__ uint32_t group_next(uint32_t x, int lane) {
    if constexpr (G == 8) {
        const uint32_t a = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x101, 0xF, 0xF, false);  // row_shl:1
        const uint32_t b = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x117, 0xF, 0xF, false);  // row_shr:7
        return lane == G - 1 ? b : a;
    } else if constexpr (G == 16) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x12F, 0xF, 0xF, false);  // row_ror:15
    } else {
        const int src = (int)(threadIdx.x & 63u) - lane + ((lane + 1) & (G - 1));
        return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)x);
    }
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Store a big-endian u16 at any byte alignment.  NOSTORE (experiment variants only): the value
// computed and kept live, nothing stored.  NT (experiment variants only): non-temporal stores.
template <bool NOSTORE = false, bool NT = false>
__device__ __forceinline__ void store_be16(gu8 q, uint32_t v) {
    if constexpr (NOSTORE) {
        asm volatile("" ::"v"(v), "v"(q));
        return;
    }
    if constexpr (NT) {
        if (((uint64_t)q & 1u) == 0) {
            __builtin_nontemporal_store((uint16_t)bswap16(v), (gu16)q);
        } else {
            __builtin_nontemporal_store((uint8_t)(v >> 8), q);
            __builtin_nontemporal_store((uint8_t)v, q + 1);
        }
        return;
    }
    if (((uint64_t)q & 1u) == 0) {
        *(gu16)q = (uint16_t)bswap16(v);
    } else {
        q[0] = (uint8_t)(v >> 8);
        q[1] = (uint8_t)v;
    }
}

// Sum of the chunk's bytes inside [lo, hi) (chunk-relative byte positions), as aligned u16 words.
__device__ __forceinline__ uint32_t sum_masked_words(const u32x4& c, int lo, int hi, uint32_t acc) {
    acc = add_words(mask_dword(c.x, lo, hi), acc);
    acc = add_words(mask_dword(c.y, lo - 4, hi - 4), acc);
    acc = add_words(mask_dword(c.z, lo - 8, hi - 8), acc);
    return add_words(mask_dword(c.w, lo - 12, hi - 12), acc);
}


// Per-group walk state.
struct Walk {
    uint64_t r;      // current record
    RecRef cur, nxt; // current record, the group's next record (descriptor prefetched)
    uint32_t nch;    // aligned chunks of cur
    uint32_t step;   // step within cur
    Geom* g;         // cur's geometry (protocol modes) in LDS: 13 VGPRs less across the walk
    Geom gr;         // ... or in registers (MODE_EMIT: measured faster there, see csum_kernel)
    int s1;          // end of the summed span, relative to the record start
    uint32_t acc, acc2;
    uint32_t fip, fl4, fin;  // MODE_COPY: record offsets of the fields emit writes (NO_FIELD if none)
    int32_t segA, segB;      // SEGW: record-relative starts of the 64-B segments written whole (SEG_NONE: none)
    bool far;                // MODE_COPY, WHOLE: a field lies (partly) past the LDS window
};

constexpr uint32_t NO_FIELD = 0x3fffffffu;
constexpr int32_t SEG_NONE = -(1 << 30);
constexpr uint32_t MF_NONE = 0x3fffu;  // no field (finish_gates)

// SEGW (fixed-stride emit): the record a group is on (tag = low 32 bits of its index) and the
// record-offset range [lo, hi) of the fields emit may write there (lo = NO_FIELD, hi = 0: none),
// published in LDS after the parse for the neighbouring groups of the wavefront.  The tag is stored
// twice so that each neighbour reads its pair with one 8-byte LDS load.
struct SegInfo {
    uint32_t tag, hi;   // read by the next group
    uint32_t tag2, lo;  // read by the previous group
};

// SEGG: the same with the record's extent, so that a neighbour can tell whether the bytes of a
// segment outside its own record belong to this record (descriptor batches: records anywhere).
// All addresses absolute; [flo, fhi) = the fields' byte range (flo = ~0, fhi = 0: none).
// Record start `beg` (absolute), length, and [flo, fhi) relative to beg (flo = NO_FIELD, fhi = 0:
// none).  The group's own decision (record-relative segment starts, SEG_NONE: none) rides in the
// same entry, so that it costs no registers across the walk.
struct SegInfoG {
    uint32_t tag;
    int32_t segA, segB;
    uint32_t len;
    uint64_t beg;
    uint32_t flo, fhi;
};

// The record offsets of the fields emit may write (NO_FIELD: none): a superset of finish_gates'.
__device__ __forceinline__ void emit_fields(const Geom& g, uint32_t f[3]) {
    f[0] = g.fam == 4 ? g.ip_off + 10 : NO_FIELD;
    f[1] = (g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED)) ? g.l4_off + g.fo : NO_FIELD;
    f[2] = g.in_off ? g.in_off + 10 : NO_FIELD;
}

// Staged emit (round 6; csum_dwalk.hip variants 94-97, csum_xwalk.hip variants 80 / 81): a record whose
// field segments go out whole in the segment pass stages one 8-B entry: its two field offsets (< 256:
// the fields lie in its LDS window; 0xff: none) and the two big-endian field values; every other
// record of a staging wavefront writes ~0.  Each group of 8 consecutive records (one wavefront of the
// segment pass) has a flag word: 1 when its entries were written by this call, 0 when none was (the
// pass skips the group), so no entry of an earlier call is ever read.
__device__ __forceinline__ uint64_t stage_entry(uint32_t f0, uint32_t v0, uint32_t f1, uint32_t v1) {
    return (uint64_t)(f0 & 0xffu) | ((uint64_t)(f1 & 0xffu) << 8) | ((uint64_t)(v0 & 0xffffu) << 32) |
           ((uint64_t)(v1 & 0xffffu) << 48);
}
// The entry of record r (its fields from the LDS window, where finish_gates patched them in), or ~0
// when it is not staged; written by one lane.
__device__ __forceinline__ void stage_record(const KParams& p, uint64_t r, bool staged, const Geom& g,
                                             const uint8_t* winb, uint32_t hd) {
    uint64_t e = ~0ull;
    if (staged) {
        uint32_t f[3];
        emit_fields(g, f);
        auto val = [&](uint32_t fo) { return fo == NO_FIELD ? 0u : (uint32_t)((winb[hd + fo] << 8) | winb[hd + fo + 1]); };
        e = stage_entry(f[0] == NO_FIELD ? 0xffu : f[0], val(f[0]), f[1] == NO_FIELD ? 0xffu : f[1], val(f[1]));
    }
    __builtin_nontemporal_store(e, (GMEM uint64_t*)(p.stage + r));
}

// The gates of one record (MODE_EMIT / MODE_VERIFY / MODE_COPY), run by its whole group once every
// lane holds its part `acc` of the aligned-word sum over [0, span_end): the header bytes the lanes
// summed are taken out again, the IPv4 header sum and the pseudo-header address words are read from
// the LDS window (`winb`, record byte o at head + o), and lane 0 finishes and writes the record.
// WINB > 0 (MODE_COPY, WHOLE): field bytes inside the first WINB bytes of the chunk grid go into the
// LDS window (`winw`), whose chunks the caller stores afterwards, instead of to global memory.
// SEGP (fixed-stride emit, SEGW): the 64-B segments wsA / wsB (~0: none) go out whole from the
// window afterwards; a field is patched into the window, and stored to global memory unless both
// of its bytes lie in those segments.
// STG (staged emit, csum_dwalk.hip variants 96 / 97): `stg` 1 writes the record's field values to its staged
// entry instead of the record (the caller has decided its segments go out whole in the segment pass:
// no third field, both fields inside the LDS window); 2 stores the fields here and writes the entry
// ~0; 0 stores them here (a wavefront that stages nothing).
template <int G, int MODE, bool NHC, class RD, int WINB = 0, bool SEGP = false, bool NOSTORE = false,
          bool NTST = false, bool STG = false>
__device__ __forceinline__ void finish_gates(const KParams& p, const Geom& g, uint32_t acc, const RD& rd,
                                             const uint8_t* winb, uint32_t head, uint64_t a0, uint64_t r,
                                             int lane, uint8_t* winw = nullptr, uint64_t wsA = ~0ull,
                                             uint64_t wsB = ~0ull, int stg = 0) {
    constexpr bool EMITS = MODE == MODE_EMIT || MODE == MODE_COPY;
    const bool odd = (a0 & 1u) != 0;
    // Header bytes [0, l4_off) that the lanes summed (taken out of the L4 sum), the IPv4
    // header's big-endian word sum and the pseudo-header address words.  All of them sit in
    // the LDS window except behind a long Hop-by-Hop header (then read from global memory).
    const bool l4 = g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED);
    const uint32_t l4_off = l4 ? g.l4_off : 0u;
    uint32_t pre = 0;  // aligned-word sum contribution of the bytes [0, l4_off)
    for (uint32_t i = lane; NHC ? 2 * i + 1 < l4_off : 2 * i < l4_off; i += G) {
        // record offset 2i is the low byte of an aligned little-endian word for an even record
        // start, the high byte for an odd one (l4_off is even on the IP path)
        const uint32_t e = rd(2 * i), o = rd(2 * i + 1);
        pre += odd ? ((e << 8) + o) : (e + (o << 8));
    }
    // an odd l4_off (6LoWPAN NHC UDP payloads) leaves one byte, weighted by its address parity
    if (NHC && (l4_off & 1u) && lane == 0) pre += rd(l4_off - 1) << (8u * (uint32_t)((a0 + l4_off - 1) & 1u));
    uint32_t hsum = 0, psum = 0;
    if (g.fam == 4) {
        for (uint32_t i = lane; i < g.ip_hl / 2; i += G) {
            const uint32_t o = head + g.ip_off + 2 * i;
            if (!(EMITS && i == 5)) hsum += (winb[o] << 8) | winb[o + 1];
        }
    }
    if (l4 && (g.proto == P_UDP || g.proto == P_TCP || g.proto == P_ICMP6)) {
        for (uint32_t i = lane; i < g.addr_words; i += G) {
            const uint32_t o = head + g.addr_off + 2 * i;
            psum += (winb[o] << 8) | winb[o + 1];
        }
    }
    if (NHC && l4 && g.proto == P_NHC_UDP && lane < 8) {
        // the IPv6 addresses come with the batch (the IPHC header compresses them): 32 B per record
        const uint32_t v = ld_u32_sync((uint64_t)p.addrs + 32ull * r + 4u * (uint32_t)lane);
        psum = ((v & 0xffu) << 8 | ((v >> 8) & 0xffu)) + (((v >> 16) & 0xffu) << 8 | (v >> 24));
    }
    const uint32_t tot = group_sum<G>(acc);
    pre = group_sum<G>(pre);
    hsum = group_sum<G>(hsum);
    psum = group_sum<G>(psum);
    const gu8 wrec = (gu8)a0;
    if (lane == 0) {
        uint32_t st = g.st;
        uint32_t fip = MF_NONE, fl4 = MF_NONE, fin = MF_NONE, vip = 0, vl4 = 0, vin = 0;  // emit: the field writes
        // IPv4 header: data(header) (canonical fold of the big-endian word sum)
        uint32_t ip_valid = 1, ip_ok = 1;
        if (g.fam == 4) {
            const uint32_t hdr = fold32(hsum);
            if (EMITS) {
                fip = g.ip_off + 10;
                vip = caps_tx(p.caps_ipv4) ? (~hdr & 0xffffu) : 0u;
            } else {
                ip_valid = hdr == 0xffffu;
                ip_ok = caps_rx(p.caps_ipv4) ? ip_valid : 1u;
            }
        }
        uint32_t l4_valid = 1, l4_ok = 1, partial = 0;
        uint32_t nb0 = NO_FIELD;  // emit: new dispatch byte (NHC UDP: the C bit cleared)
        if (NHC && l4 && g.proto == P_NHC_UDP) {
            // 6LoWPAN NHC UDP: !combine([pseudo_header_v6(src, dst, Udp, n + 8), sport, dport,
            // n + 8, data(payload)]) — nhc.rs:705-716 (parse), :760-771 (emit).  Ports as the
            // accessors read them (nhc.rs:513-577, quirks included); on emit the mode-0b01
            // destination comes from byte 3, where set_ports put it (:655-662).
            const uint32_t b0 = rd(0), m = b0 & 3u;
            const uint32_t sport = m <= 1 ? (rd(1) << 8 | rd(2)) : m == 2 ? 0xf000u + rd(1) : 0xf0b0u + (rd(1) >> 4);
            uint32_t dport = m == 0 ? (rd(3) << 8 | rd(4)) : m == 1 ? 0xf000u + rd(1) : m == 2 ? (rd(2) << 8 | rd(3))
                                                                                          : 0xf0b0u + rd(1);
            if (EMITS && m == 1) dport = 0xf000u + rd(3);
            const uint32_t n8 = (g.l4_len + 8) & 0xffffu;
            const uint32_t f = fold32(tot - pre);
            const uint32_t dat = ((a0 + g.l4_off) & 1u) ? f : bswap16(f);  // == checksum::data(payload)
            const uint32_t ph = fold32(psum + P_UDP + n8);
            const uint32_t chk = ~fold32(ph + sport + dport + n8 + dat) & 0xffffu;
            if (EMITS) {
                if (caps_tx(p.caps_udp)) {  // set_checksum, nhc.rs:676-681 (no 0 -> 0xffff)
                    fl4 = g.fo;
                    vl4 = chk;
                    if (b0 & 4u) nb0 = b0 & ~4u;
                }
            } else {
                const bool present = !(b0 & 4u);
                l4_valid = present ? (chk == ((rd(g.fo) << 8) | rd(g.fo + 1))) : 1u;
                l4_ok = caps_rx(p.caps_udp) ? l4_valid : 1u;
            }
        } else if (l4) {
            const uint32_t fpos = g.l4_off + g.fo;
            const uint32_t field = (rd(fpos) << 8) | rd(fpos + 1);
            // aligned-word sum of the L4 span = lanes' sum of [0, span_end) minus the
            // header bytes [0, l4_off) (exact: no u32 wrap below 131072 bytes)
            uint32_t s = tot - pre;
            // aligned-word contribution of a big-endian u16 at an even record offset
            auto word = [&](uint32_t v) { return odd ? v : bswap16(v); };
            if (EMITS) {
                // the reference zeroes the field before summing: remove its bytes (the
                // field offset is even: its parity is the record start's)
                s -= word(field);
                if (g.in_off) {
                    // ICMPv4 DstUnreachable / TimeExceeded: Ipv4Repr::emit of the embedded header
                    // under the same caps (icmpv4.rs:526-528, 540-542; ipv4.rs:605-611) before the
                    // ICMP checksum covers it.  Rare: lane 0 alone.
                    uint32_t hin = 0;
                    for (uint32_t i = 0; i < g.in_hl / 2; ++i)
                        if (i != 5) hin += (rd(g.in_off + 2 * i) << 8) | rd(g.in_off + 2 * i + 1);
                    fin = g.in_off + 10;
                    vin = caps_tx(p.caps_ipv4) ? (~fold32(hin) & 0xffffu) : 0u;
                    s = s - word((rd(fin) << 8) | rd(fin + 1)) + word(vin);
                }
            }
            const uint32_t f = fold32(s);
            const uint32_t dat = odd ? f : bswap16(f);  // == checksum::data(span)
            uint32_t ph = 0, gate_caps = SMOL_CHECKSUM_NONE;
            const bool pseudo = g.proto == P_UDP || g.proto == P_TCP || g.proto == P_ICMP6;
            if (pseudo) {
                const uint32_t plen = g.proto == P_UDP ? (g.span_end - g.l4_off) : g.l4_len;
                ph = fold32(psum + g.proto + (plen & 0xffffu));  // pseudo_header()
            }
            const uint32_t comb = pseudo ? fold32(ph + dat) : dat;  // combine()
            switch (g.proto) {
                case P_UDP: gate_caps = p.caps_udp; break;
                case P_TCP: gate_caps = p.caps_tcp; break;
                case P_ICMP4: gate_caps = p.caps_icmpv4; break;
                case P_ICMP6: gate_caps = p.caps_icmpv6; break;
                default: gate_caps = SMOL_CHECKSUM_NONE; break;  // IGMP
            }
            if (EMITS) {
                const bool fill = g.proto == P_IGMP ? true : caps_tx(gate_caps);
                uint32_t c = ~comb & 0xffffu;
                if (g.proto == P_UDP && c == 0) c = 0xffffu;  // udp.rs:207
                fl4 = fpos;
                vl4 = fill ? c : 0u;
            } else {
                l4_valid = comb == 0xffffu;
                if (g.proto == P_UDP && field == 0) l4_valid = 1;  // udp.rs:138-140
                if (g.proto == P_UDP || g.proto == P_TCP) partial = ph == field;
                l4_ok = caps_rx(gate_caps) ? l4_valid : 1u;
            }
        }
        if (EMITS && SEGP) {
            auto put = [&](uint32_t f, uint32_t v) {
                const uint64_t x0 = (a0 + f) & ~63ull, x1 = (a0 + f + 1) & ~63ull;
                const bool cov = (x0 == wsA || x0 == wsB) && (x1 == wsA || x1 == wsB);
                for (uint32_t i = 0; i < 2; ++i)
                    if (head + f + i < (uint32_t)WINB) winw[head + f + i] = (uint8_t)(i ? v : v >> 8);
                if (!cov) store_be16<NOSTORE>(wrec + f, v);
            };
            if (fip != MF_NONE) put(fip, vip);
            if (fin != MF_NONE) put(fin, vin);
            if (fl4 != MF_NONE) put(fl4, vl4);
            if (p.status) ((gu8)p.status)[r] = (uint8_t)st;
        } else if (EMITS && WINB > 0) {
            auto put = [&](uint32_t f, uint32_t v) {
                for (uint32_t i = 0; i < 2; ++i) {
                    const uint8_t b = (uint8_t)(i ? v : v >> 8);
                    if (head + f + i < (uint32_t)WINB) winw[head + f + i] = b;
                    else wrec[f + i] = b;
                }
            };
            if (fip != MF_NONE) put(fip, vip);
            if (fin != MF_NONE) put(fin, vin);
            if (fl4 != MF_NONE) put(fl4, vl4);
            if (p.status) ((gu8)p.status)[r] = (uint8_t)st;
        } else if (EMITS) {
            if (STG && stg == 1) {
                const uint64_t e = stage_entry(fip == MF_NONE ? 0xffu : fip, vip, fl4 == MF_NONE ? 0xffu : fl4, vl4);
                if constexpr (NTST) {  // (experiments, dwalk variant 109) write-through non-temporal vector store
                    const uint64_t a = (uint64_t)(p.stage + r);
                    asm volatile("global_store_dwordx2 %0, %1, off sc1 nt" ::"v"(a), "v"(e) : "memory");
                } else {
                    __builtin_nontemporal_store(e, (GMEM uint64_t*)(p.stage + r));
                }
            } else {
                if (fip != MF_NONE) store_be16<NOSTORE, NTST>(wrec + fip, vip);
                if (fin != MF_NONE) store_be16<NOSTORE, NTST>(wrec + fin, vin);
                if (fl4 != MF_NONE) store_be16<NOSTORE, NTST>(wrec + fl4, vl4);
                if (NHC && nb0 != NO_FIELD) wrec[0] = (uint8_t)nb0;
                if (STG && stg == 2) __builtin_nontemporal_store(~0ull, (GMEM uint64_t*)(p.stage + r));
            }
            if (p.status) ((gu8)p.status)[r] = (uint8_t)st;
        } else {
            const bool mal = (st & SMOL_ST_MALFORMED) != 0;
            st |= (ip_ok ? SMOL_ST_IP_OK : 0u) | (l4_ok ? SMOL_ST_L4_OK : 0u) |
                  (partial ? SMOL_ST_L4_PARTIAL : 0u) | (ip_valid ? SMOL_ST_IP_VALID : 0u) |
                  (l4_valid ? SMOL_ST_L4_VALID : 0u) |
                  ((ip_ok && l4_ok && !mal) ? SMOL_ST_ACCEPT : 0u);
            if constexpr (NOSTORE) asm volatile("" ::"v"(st));  // (timing only: no status byte)
            else if constexpr (NTST) __builtin_nontemporal_store((uint8_t)st, (gu8)p.status + r);  // (verify: experiments)
            else ((gu8)p.status)[r] = (uint8_t)st;
        }
    }
}

// Fixed-stride emit on the line grid: the 128-B line holding record r+1's first byte also holds
// record r's last bytes, and with non-temporal loads two groups requesting it fetch it from HBM
// twice (C2: 5.6 % more HBM reads than the records' bytes).  When the group of record r+1 is this
// group's neighbour in the same wavefront, only that group loads the line — it is the first line of
// its LDS window — and this group reads its tail chunks there.  Measured (tools/sweep.py): emit
// 0.331 -> 0.304 ms on C2, 0.281 -> 0.263 ms on C4; verify got slower with it (C2 0.2377 -> 0.2434
// ms, C4 0.2101 -> 0.2217 ms, although its HBM reads fell to the records' bytes), so verify keeps
// loading both.  Returns the address
// from which record r's chunks come from the neighbour's window (~0: none).  Records take 2 or 3
// steps depending on their offset in the line, so groups are not in lockstep: the neighbour's
// window is used only when record r+1 is the neighbour's one and only record (the natural grid),
// so that it is filled at the start and never overwritten.  Stride >= 384 keeps that line out of
// record r's own window.
template <int G, int MODE, bool IMPLICIT, bool LINE, bool NOSHARE = false>
__device__ __forceinline__ uint64_t shared_from(const KParams& p, uint64_t r, uint64_t a0, int gib, uint64_t ngroups) {
    constexpr bool SHARE = IMPLICIT && LINE && MODE == MODE_EMIT && !NOSHARE;
    constexpr int GPW = 64 / G;  // groups per wavefront
    if (!SHARE || p.stride < 384 || (gib % GPW) == GPW - 1 || r + 1 >= p.n || r + 1 >= ngroups ||
        r + 1 + ngroups < p.n)
        return ~0ull;
    return (a0 + p.stride) & ~127ull;
}

// One step of the walk: prefetch the following step into `nx`, then sum `cv` (the current step)
// and finish the record on its last step.  Returns false when the group has no more work.
template <int G, int U, int MODE, bool IMPLICIT, bool NT, bool PF, bool SKIPD, bool LINE, bool NHC, int CU = 0,
          bool SHUF = false, bool WHOLE = false, bool SHUF2 = false, bool SEGW = false, bool SEGG = false,
          bool SEGB = false, bool SEG6 = false, int SEGOPT = 0, int VAR = 0>
__device__ __forceinline__ bool walk_step(const KParams& p, Walk& w, Regs<U, MODE == MODE_COPY>& cv,
                                          Regs<U, MODE == MODE_COPY>& nx, int lane, uint64_t ngroups, u32x4* win,
                                          int gib, SegInfo* si = nullptr, SegInfoG* sg = nullptr,
                                          bool blockwide = false) {
    constexpr bool COPY = MODE == MODE_COPY;
    // where the record geometry lives (Walk::g / Walk::gr): registers for emit with the register
    // prefetch, LDS otherwise
    constexpr bool GREG = MODE == MODE_EMIT && PF && !VarT<VAR>::GLDS;
    constexpr bool NOSHARE = VarT<VAR>::NOSHARE;
    constexpr bool NOSTORE = VarT<VAR>::NOSTORE;
    constexpr bool BSEG = VarT<VAR>::BSEG && MODE == MODE_EMIT && IMPLICIT && LINE && !NHC;
    constexpr bool SEGF = SEGW || BSEG;  // the finish writes the decided segments whole
    constexpr int WIN = Grid<LINE>::WIN;
    constexpr int WIN_CH = Grid<LINE>::WIN_CH;
    static_assert(G * U >= WIN_CH, "step 0 must cover the LDS window");
    const uint8_t* winb = reinterpret_cast<const uint8_t*>(win);
    const uint32_t nsteps = w.nch == 0 ? 1u : (w.nch + (G * U) - 1) / (G * U);
    const bool last = w.step + 1 >= nsteps;
    const uint64_t r2 = last ? w.r + ngroups : w.r;
    const bool have2 = r2 < p.n;
    const RecRef rec2 = last ? w.nxt : w.cur;
    const uint32_t nch2 = last ? n_chunks<LINE>(w.nxt) : w.nch;
    const uint32_t step2 = last ? 0u : w.step + 1;
    // SKIPD: no prefetch when the group has nothing left (one record per group in a natural grid:
    // every record's last step would otherwise issue U loads of the dummy line)
    if (PF && (!SKIPD || have2))
        load_step<G, U, NT, COPY, LINE, CU, SHUF, SHUF2>(nx, rec2, nch2, step2, lane, have2, (uint64_t)p.dummy,
                                            shared_from<G, MODE, IMPLICIT, LINE, NOSHARE>(p, r2, rec2.a0, gib, ngroups));
    // descriptor of the record after next (clamped index: an unconditional load)
    RecRef nxt2 = w.nxt;
    {
        const uint64_t r3 = r2 + ngroups < p.n ? r2 + ngroups : p.n - 1;
        const RecRef t = rec_at<IMPLICIT, COPY, NHC>(p, r3);
        if (last) nxt2 = t;
    }

    const uint64_t base = w.cur.a0 & ~(Grid<LINE>::ALIGN - 1);
    const uint32_t head = (uint32_t)(w.cur.a0 - base);
    // record byte o: LDS window when inside it, else global memory (long IPv6 extension chains)
    auto rd = [&](uint32_t o) -> uint32_t {
        const uint32_t x = head + o;
        if (x < (uint32_t)WIN) return (uint32_t)winb[x];
        if (COPY && o >= w.cur.p0 && o < w.cur.p1) return ld_byte_sync(w.cur.sb + o);
        return ld_byte_sync(w.cur.a0 + o);
    };
    // MODE_COPY: this step's chunks with the payload merged in (and stored once the fields are known)
    u32x4 cm[U];
#pragma unroll
    for (int u = 0; u < U; ++u) cm[u] = cv.v[u];
    if constexpr (COPY && SHUF2) {
        const uint64_t first = (w.cur.sb + w.cur.p0) & ~15ull, last = (w.cur.sb + w.cur.p1 - 1) & ~15ull;
        const uint64_t sk = w.cur.sb - head;  // source address of chunk 0's byte 0
        const uint32_t b = (uint32_t)(sk & 3u);
        // the dword at A of each lane's chunk (the next lane's funnel needs it): s0.x, or for a
        // chunk loaded at `last`, the dword (A - last) / 4 of it
        uint32_t xo[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = w.step * (G * U) + u * G + lane;
            const uint64_t A = (sk + 16ull * k) & ~3ull;
            const u32x4 c = cv.s0[u];
            xo[u] = c.x;
            if (A > last) {
                const uint32_t q = (uint32_t)(A - last) >> 2;
                xo[u] = q == 1 ? c.y : q == 2 ? c.z : c.w;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t nxd = group_next<G>(lane == 0 ? (u + 1 < U ? xo[u + 1 < U ? u + 1 : u] : cv.sx1) : xo[u], lane);
            const uint32_t k = w.step * (G * U) + u * G + lane;
            const int pos = (int)(16u * k) - (int)head;
            const int lo = (int)w.cur.p0 - pos, hi = (int)w.cur.p1 - pos;
            if (k < w.nch && w.cur.p1 > w.cur.p0 && hi > 0 && lo < 16) {
                const uint64_t sa = sk + 16ull * k, A = sa & ~3ull;
                const u32x4 c = cv.s0[u];
                u32x4 src;
                if (A >= first && A <= last) {
                    src.x = __builtin_amdgcn_alignbyte(c.y, c.x, b);
                    src.y = __builtin_amdgcn_alignbyte(c.z, c.y, b);
                    src.z = __builtin_amdgcn_alignbyte(c.w, c.z, b);
                    src.w = __builtin_amdgcn_alignbyte(nxd, c.w, b);
                } else {  // loaded at first (shift the bytes up) or at last (down)
                    const u32x4 z = {0u, 0u, 0u, 0u};
                    src = A < first ? funnel16(z, c, (uint32_t)(16 - (first - sa))) : funnel16(c, z, (uint32_t)(sa - last));
                }
                if (lo <= 0 && hi >= 16) {
                    cm[u] = src;
                } else {
                    const uint32_t m0 = byte_mask(lo, hi, 0), m1 = byte_mask(lo, hi, 1);
                    const uint32_t m2 = byte_mask(lo, hi, 2), m3 = byte_mask(lo, hi, 3);
                    cm[u].x = (src.x & m0) | (cm[u].x & ~m0);
                    cm[u].y = (src.y & m1) | (cm[u].y & ~m1);
                    cm[u].z = (src.z & m2) | (cm[u].z & ~m2);
                    cm[u].w = (src.w & m3) | (cm[u].w & ~m3);
                }
            }
        }
    } else if constexpr (COPY) {
        if constexpr (SHUF) {
            // the second source chunk of lane i's funnel is lane i+1's first (the group's last lane:
            // lane 0's next one), taken with all lanes of the group active
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u32x4 x = lane == 0 ? (u + 1 < U ? cv.s0[u + 1 < U ? u + 1 : u] : cv.sx) : cv.s0[u];
                cv.s1[u].x = group_next<G>(x.x, lane);
                cv.s1[u].y = group_next<G>(x.y, lane);
                cv.s1[u].z = group_next<G>(x.z, lane);
                cv.s1[u].w = group_next<G>(x.w, lane);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = w.step * (G * U) + u * G + lane;
            const int pos = (int)(16u * k) - (int)head;
            const int lo = (int)w.cur.p0 - pos, hi = (int)w.cur.p1 - pos;
            if (k < w.nch && w.cur.p1 > w.cur.p0 && hi > 0 && lo < 16) {
                const uint64_t sa = w.cur.sb + (uint64_t)(int64_t)pos;
                const u32x4 src = funnel16(cv.s0[u], cv.s1[u], (uint32_t)(sa & 15u));
                const uint32_t m0 = byte_mask(lo, hi, 0), m1 = byte_mask(lo, hi, 1);
                const uint32_t m2 = byte_mask(lo, hi, 2), m3 = byte_mask(lo, hi, 3);
                cm[u].x = (src.x & m0) | (cm[u].x & ~m0);
                cm[u].y = (src.y & m1) | (cm[u].y & ~m1);
                cm[u].z = (src.z & m2) | (cm[u].z & ~m2);
                cm[u].w = (src.w & m3) | (cm[u].w & ~m3);
            }
        }
    }
    if (w.step == 0) {
        w.acc = 0;
        w.acc2 = 0;
        if (MODE == MODE_DATA) {
            w.s1 = (int)w.cur.len;
        } else {
            // the window: chunks 0 .. WIN_CH-1 of the grid (chunk k = u * G + lane at step 0)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (u * G >= WIN_CH) break;
                const uint32_t k = (uint32_t)(u * G + lane);
                if (k < (uint32_t)WIN_CH && k < w.nch) win[k] = cm[u];
            }
            wave_lds_sync();
            if (COPY && (w.cur.kind & KIND_BAD_COPY)) {
                Geom g0 = Geom{};
                g0.st = SMOL_ST_MALFORMED;  // copy range does not fit: record left untouched
                if (lane == 0) *w.g = g0;
            } else if constexpr (GREG) {
                w.gr = parse_geometry<NHC>(rd, w.cur.len, w.cur.kind, true);
            } else {
                const Geom g0 = parse_geometry<NHC>(rd, w.cur.len, w.cur.kind, MODE == MODE_EMIT || MODE == MODE_COPY);
                if (lane == 0) *w.g = g0;
            }
            if (!GREG) wave_lds_sync();
            const Geom& g = GREG ? w.gr : *w.g;
            // the lanes sum [0, span_end): the header part is subtracted at the end
            w.s1 = (g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED)) ? (int)g.span_end : 0;
            if constexpr (SEGF) w.segA = w.segB = SEG_NONE;
            // SEGOPT / BSEG_NO4: whether the wavefront holds an IPv4 record (one ballot)
            const bool any4 = (SEGW && (SEGOPT & 1)) ? __any(g.fam == 4) : true;
            if (BSEG && (!VarT<VAR>::BSEG_NO4 || !any4)) {
                // Whole field segments, decided by one ballot.  A segment that starts before the
                // record also holds record r-1's last bytes; it goes out whole only when r-1 has no
                // field in its last 64 bytes (then no store of r-1's group can fall into it).  Each
                // group says so for its own record (ok_tail); with the natural grid every group of
                // the wavefront is on its one record at step 0, and group gib-1 holds record r-1.
                // A record whose fields end 64 bytes or more before its end never reaches into r+1
                // with its own segments.  The first group of a wavefront, a gapped stride and r = 0
                // keep the 2-B store for a segment that starts before the record.
                uint32_t f[3], lo = NO_FIELD, hi = 0;
                emit_fields(g, f);
                for (int j = 0; j < 3; ++j)
                    if (f[j] != NO_FIELD) {
                        lo = f[j] < lo ? f[j] : lo;
                        hi = f[j] + 2 > hi ? f[j] + 2 : hi;
                    }
                const bool ok_tail = hi == 0 || hi + 64 <= w.cur.len;
                const uint64_t okm = __ballot(lane == 0 && ok_tail);
                constexpr int GPW = 64 / G;
                const bool natural = ngroups >= p.n;
                const bool fam_ok = g.fam == 4 || (VarT<VAR>::BSEG6 && g.fam == 6);
                if (natural && fam_ok && hi != 0 && ok_tail && w.cur.len < (1u << 29)) {
                    const uint32_t wl = (uint32_t)(threadIdx.x & 63u);
                    const bool prev_ok = (gib % GPW) != 0 && w.r > 0 && p.len == p.stride &&
                                         ((okm >> (wl - (uint32_t)lane - G)) & 1ull);
                    const int32_t ph = (int32_t)(w.cur.a0 & 63u);
                    const int32_t rA = ((ph + (int32_t)lo) & ~63) - ph, rB = ((ph + (int32_t)hi - 1) & ~63) - ph;
                    const int32_t wend = 16 * (int32_t)(w.nch < (uint32_t)WIN_CH ? w.nch : (uint32_t)WIN_CH) - (int32_t)head;
                    auto whole = [&](int32_t rel) { return rB <= rA + 64 && rel + 64 <= wend && (rel >= 0 || prev_ok); };
                    if (whole(rA)) w.segA = rA;
                    if (rB != rA && whole(rB)) w.segB = rB;
                }
            }
            if (SEGW && any4) {
                // publish every field finish_gates may write (a superset is safe), then decide which
                // of this record's field segments go out whole (see the finish below)
                uint32_t f[3], lo = NO_FIELD, hi = 0;
                emit_fields(g, f);
                for (int j = 0; j < 3; ++j)
                    if (f[j] != NO_FIELD) {
                        lo = f[j] < lo ? f[j] : lo;
                        hi = f[j] + 2 > hi ? f[j] + 2 : hi;
                    }
                if (lane == 0) {
                    SegInfo e;
                    e.tag = e.tag2 = (uint32_t)w.r;
                    e.lo = lo;
                    e.hi = hi;
                    si[gib] = e;
                }
                w.segA = w.segB = SEG_NONE;
                // IPv4 records only (an IPv4 header and an L4 field: two store events per record);
                // the neighbours' field bounds, record-relative: the previous record's end by pend,
                // the next one's start at nbeg (another wavefront or another record: unknown)
                if (g.fam == 4 && p.stride >= 64 && p.n < 0xFFFFFFFFull && w.cur.len < (1u << 29)) {
                    wave_lds_sync();  // the neighbours' entries
                    constexpr int GPW = 64 / G;
                    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                    const uint64_t r = w.r;
                    int32_t pend = 1 << 30, nbeg = -(1 << 30);
                    const int32_t st = (int32_t)(p.stride < (1ull << 29) ? p.stride : (1ull << 29));
                    if ((gib % GPW) != 0) {
                        const u32x2 q = *reinterpret_cast<const u32x2*>(&si[gib - 1].tag);
                        if (r > 0 && q.x == (uint32_t)(r - 1)) pend = (int32_t)(q.y < (1u << 29) ? q.y : (1u << 29)) - st;
                    }
                    if ((gib % GPW) != GPW - 1) {
                        const u32x2 q = *reinterpret_cast<const u32x2*>(&si[gib + 1].tag2);
                        if (q.x == (uint32_t)(r + 1)) nbeg = st + (int32_t)(q.y < (1u << 29) ? q.y : (1u << 29));
                    }
                    // record-relative starts of the segments holding the first and the last field byte
                    const int32_t ph = (int32_t)(w.cur.a0 & 63u);
                    const int32_t rA = ((ph + (int32_t)lo) & ~63) - ph, rB = ((ph + (int32_t)hi - 1) & ~63) - ph;
                    const int32_t len = (int32_t)w.cur.len;
                    const bool packed = p.len == p.stride;
                    const bool lastrec = r + 1 >= p.n;
                    // the window holds the record's chunks only (past its last one: the dummy line)
                    const int32_t wend = 16 * (int32_t)(w.nch < (uint32_t)WIN_CH ? w.nch : (uint32_t)WIN_CH) - (int32_t)head;
                    auto whole = [&](int32_t rel) {
                        return rB <= rA + 64 && rel + 64 <= wend &&
                               (rel >= 0 || (packed && r > 0 && pend <= rel)) &&
                               (rel + 64 <= len || (packed && !lastrec && nbeg >= rel + 64));
                    };
                    if (whole(rA)) w.segA = rA;
                    if (rB != rA && whole(rB)) w.segB = rB;
                }
            }
        }
    }
    // MODE_COPY: store the payload bytes of this step (all of them, summed or not).  WHOLE: store
    // every byte of the record instead (the bytes outside the payload unchanged), so that no cache
    // line of the batch leaves L2 partially written — a partial line costs HBM a read-modify-write
    // (tools/probe_copy.hip: 0.818 ms with partial edge lines, 0.565 ms with whole lines) — and
    // store the window chunks (which hold the fields) at the end of the record, fields included.
    if constexpr (COPY) {
        const gu8 cbase = (gu8)base;
        // the fields to leave out (finish writes them).  WHOLE: the window holds every field but a
        // far one (a long IPv6 Hop-by-Hop header), so the offsets come from LDS only then
        int f0b = (int)w.fip, f1b = (int)w.fl4, f2b = (int)w.fin;
        if constexpr (WHOLE) {
            f0b = f1b = f2b = -(1 << 20);
            if (w.far) {
                const Geom& g = *w.g;
                f0b = g.fam == 4 ? (int)g.ip_off + 10 : -(1 << 20);
                f1b = (g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED)) ? (int)(g.l4_off + g.fo) : -(1 << 20);
                f2b = g.in_off ? (int)g.in_off + 10 : -(1 << 20);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = w.step * (G * U) + u * G + lane;
            const int pos = (int)(16u * k) - (int)head;
            const int lo = WHOLE ? -pos : (int)w.cur.p0 - pos;
            const int hi = WHOLE ? (int)w.cur.len - pos : (int)w.cur.p1 - pos;
            if (k < w.nch && (WHOLE ? (k >= (uint32_t)WIN_CH) : (w.cur.p1 > w.cur.p0 && hi > 0 && lo < 16))) {
                const int f0 = f0b - pos, f1 = f1b - pos, f2 = f2b - pos;
                const bool field = (f0 > -2 && f0 < 16) || (f1 > -2 && f1 < 16) || (f2 > -2 && f2 < 16);
                const gu8 dst = cbase + 16u * k;
                if (lo <= 0 && hi >= 16 && !field) {
                    *(GMEM u32x4*)dst = cm[u];
                } else {
                    const uint32_t cw[4] = {cm[u].x, cm[u].y, cm[u].z, cm[u].w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        uint32_t keep = byte_mask(lo, hi, i);
                        keep &= ~byte_mask(f0, f0 + 2, i);
                        keep &= ~byte_mask(f1, f1 + 2, i);
                        keep &= ~byte_mask(f2, f2 + 2, i);
                        if (keep == 0xffffffffu) {
                            *(GMEM uint32_t*)(dst + 4 * i) = cw[i];
                        } else if (keep) {
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                if (keep & (0xffu << (8 * j))) dst[4 * i + j] = (uint8_t)(cw[i] >> (8 * j));
                        }
                    }
                }
            }
        }
    }

    // ---- sum this step's chunks over [0, s1) (data: [0, len)) ----
    const int s1 = w.s1;
    const uint64_t lim = shared_from<G, MODE, IMPLICIT, LINE, NOSHARE>(p, w.r, w.cur.a0, gib, ngroups);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t k = w.step * (G * U) + u * G + lane;
        const int pos = (int)(16u * k) - (int)head;  // chunk start relative to the record
        if (k < w.nch && pos < s1 && pos + 16 > 0) {
            const uint64_t ca = base + 16ull * k;
            const u32x4 c = ca >= lim ? win[WIN_CH + ((ca - lim) >> 4)] : cm[u];  // neighbour's window
            if (pos < 0 || pos + 16 > s1) {  // first chunk (bytes before the record) / tail
                if (MODE == MODE_DATA) {
                    const int lo = -pos, hi = s1 - pos;
                    const uint32_t w0 = mask_dword(c.x, lo, hi), w1 = mask_dword(c.y, lo - 4, hi - 4);
                    const uint32_t w2 = mask_dword(c.z, lo - 8, hi - 8), w3 = mask_dword(c.w, lo - 12, hi - 12);
                    w.acc = add_even_bytes(w0, add_even_bytes(w1, add_even_bytes(w2, add_even_bytes(w3, w.acc))));
                    w.acc2 = add_odd_bytes(w0, add_odd_bytes(w1, add_odd_bytes(w2, add_odd_bytes(w3, w.acc2))));
                } else {
                    w.acc = sum_masked_words(c, -pos, s1 - pos, w.acc);
                }
            } else {
                if (MODE == MODE_DATA) {
                    w.acc = add_even_bytes(c.x, add_even_bytes(c.y, add_even_bytes(c.z, add_even_bytes(c.w, w.acc))));
                    w.acc2 = add_odd_bytes(c.x, add_odd_bytes(c.y, add_odd_bytes(c.z, add_odd_bytes(c.w, w.acc2))));
                } else {
                    w.acc = add_words(c.x, add_words(c.y, add_words(c.z, add_words(c.w, w.acc))));
                }
            }
        }
    }

    if constexpr (SEGG) {
        if (w.step == 0) {
            // After step 0's sum (fewer registers live than at the parse): publish the record's
            // extent and every field finish_gates may write (a superset is safe), then decide which
            // of this record's field segments go out whole.
            const Geom& g = GREG ? w.gr : *w.g;
            const uint64_t a0 = w.cur.a0;
            const int32_t len = (int32_t)w.cur.len;
            uint32_t lo = NO_FIELD, hi = 0;
            {
                uint32_t f[3];
                emit_fields(g, f);
                for (int j = 0; j < 3; ++j)
                    if (f[j] != NO_FIELD) {
                        lo = f[j] < lo ? f[j] : lo;
                        hi = f[j] + 2 > hi ? f[j] + 2 : hi;
                    }
            }
            if (lane == 0) {
                SegInfoG& e = sg[gib];
                e.tag = (uint32_t)w.r;
                e.segA = e.segB = SEG_NONE;
                e.len = w.cur.len;
                e.beg = a0;
                e.flo = lo;
                e.fhi = hi;
            }
            // SEGB: every group of the workgroup is on its first (and only) record here, so one
            // barrier makes every neighbour's entry visible (blockwide is uniform over the
            // workgroup: a natural grid and a full workgroup, see csum_kernel)
            if (SEGB && blockwide) __syncthreads();
            else wave_lds_sync();
            const bool fam_ok = g.fam == 4 || (SEG6 && g.fam == 6);
            if (fam_ok && lo != NO_FIELD && p.n < 0xFFFFFFFFull && w.cur.len < (1u << 29)) {
                constexpr int GPW = 64 / G;
                const uint64_t r = w.r;
                const bool have_prev = (SEGB && blockwide) ? gib > 0 : (gib % GPW) != 0;
                const bool have_next = (SEGB && blockwide) ? gib + 1 < 256 / G : (gib % GPW) != GPW - 1;
                // Everything relative to this record's start (int32: records are < 2^29 bytes).
                // The previous record ends here and its last field byte is before pfhi; the next one
                // starts at len and ends at nend, its first field byte at nflo (valid only when the
                // neighbour's group holds record r -/+ 1 right now: the tag check, and adjacent in
                // memory: the extent check)
                int32_t pbeg = 1 << 30, pfhi = 1 << 30, nend = -(1 << 30), nflo = -(1 << 30);
                if (have_prev && r > 0) {
                    const SegInfoG& q = sg[gib - 1];
                    const uint32_t ql = q.len < (1u << 29) ? q.len : (1u << 29);
                    if (q.tag == (uint32_t)(r - 1) && q.beg + q.len == a0) {
                        pbeg = -(int32_t)ql;
                        pfhi = q.fhi ? (int32_t)q.fhi - (int32_t)ql : pbeg;
                    }
                }
                if (have_next && r + 1 < p.n) {
                    const SegInfoG& q = sg[gib + 1];
                    const uint32_t ql = q.len < (1u << 29) ? q.len : (1u << 29);
                    if (q.tag == (uint32_t)(r + 1) && q.beg == a0 + (uint64_t)len) {
                        nend = len + (int32_t)ql;
                        nflo = q.flo != NO_FIELD ? len + (int32_t)q.flo : nend;
                    }
                }
                // record-relative starts of the segments holding the first and the last field byte
                const int32_t ph = (int32_t)(a0 & 63u);
                const int32_t SA = ((ph + (int32_t)lo) & ~63) - ph, SB = ((ph + (int32_t)hi - 1) & ~63) - ph;
                // the window holds the record's chunks only (past its last one: the dummy line)
                const int32_t head0 = (int32_t)(a0 & (Grid<LINE>::ALIGN - 1));
                const int32_t wend = 16 * (int32_t)(w.nch < (uint32_t)WIN_CH ? w.nch : (uint32_t)WIN_CH) - head0;
                auto whole = [&](int32_t S) {
                    return SB <= SA + 64 && S + 64 <= wend && (S >= 0 || (pbeg <= S && pfhi <= S)) &&
                           (S + 64 <= len || (nend >= S + 64 && nflo >= S + 64));
                };
                const int32_t sa = whole(SA) ? SA : SEG_NONE;
                const int32_t sb = (SB != SA && whole(SB)) ? SB : SEG_NONE;
                if (lane == 0) {
                    sg[gib].segA = sa;
                    sg[gib].segB = sb;
                }
            }
            wave_lds_sync();  // the decision, read back at the finish
        }
    }

    if (last) {
        const bool odd = (w.cur.a0 & 1u) != 0;
        const uint64_t r = w.r;
        if (MODE == MODE_DATA) {
            // exact little-endian word sum relative to the span start, modulo 2^32
            const uint32_t s_rel = odd ? (w.acc2 + (w.acc << 8)) : (w.acc + (w.acc2 << 8));
            const uint32_t tot = group_sum<G>(s_rel);
            if (lane == 0) ((gu16)p.out16)[r] = (uint16_t)bswap16(fold32(tot));
        } else {
            // SEGW: the 64-B segments that hold the fields go out whole from the LDS window, the
            // fields patched in: a whole segment costs HBM a plain write where a 2-B store costs a
            // read-modify-write (measured: C2 emit 0.305 -> 0.285 ms when every segment goes out
            // whole).  A segment also holds bytes of the neighbouring records; it is written whole
            // only when none of their fields lies in it (the field ranges their groups of this
            // wavefront publish after the parse say so), it holds no byte outside the batch's
            // records and the window holds all of it.  Fields outside such segments are stored as
            // 2-B fields.
            uint64_t wsA = ~0ull, wsB = ~0ull;
            if constexpr (SEGF) {  // the segments decided after the parse (step 0)
                if (w.segA != SEG_NONE) wsA = w.cur.a0 + (int64_t)w.segA;
                if (w.segB != SEG_NONE) wsB = w.cur.a0 + (int64_t)w.segB;
            }
            if constexpr (SEGG) {  // the segments decided after step 0's sum
                const int32_t sa = sg[gib].segA, sb = sg[gib].segB;
                if (sa != SEG_NONE) wsA = w.cur.a0 + (int64_t)sa;
                if (sb != SEG_NONE) wsB = w.cur.a0 + (int64_t)sb;
            }
            finish_gates<G, MODE, NHC, decltype(rd), ((COPY && WHOLE) || SEGF || SEGG) ? WIN : 0, SEGF || SEGG, NOSTORE>(
                p, GREG ? w.gr : *w.g, w.acc, rd, winb, head, w.cur.a0, r, lane, reinterpret_cast<uint8_t*>(win),
                wsA, wsB);
            if constexpr (SEGF || SEGG) {
                if (wsA != ~0ull || wsB != ~0ull) {
                    wave_lds_sync();
                    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                    auto seg_store = [&](uint64_t d) {
                        const u32x2 x = *reinterpret_cast<const u32x2*>(winb + (d - base));
                        if constexpr (NOSTORE) asm volatile("" ::"v"(x), "v"(d));
                        else if constexpr (VarT<VAR>::NTSEG)  // write-through non-temporal vector store
                            asm volatile("global_store_dwordx2 %0, %1, off sc1 nt" ::"v"(d), "v"(x) : "memory");
                        else *(GMEM u32x2*)d = x;
                    };
                    if (wsA != ~0ull && lane < 8) seg_store(wsA + 8u * (uint32_t)lane);
                    if (wsB != ~0ull && lane < 8) seg_store(wsB + 8u * (uint32_t)lane);
                    wave_lds_sync();  // the window is rewritten by the group's next record
                }
            }
            if constexpr (COPY && WHOLE) {  // the window chunks, fields patched in
                wave_lds_sync();
                for (uint32_t k = (uint32_t)lane; k < (uint32_t)WIN_CH && k < w.nch; k += G) {
                    const int pos = (int)(16u * k) - (int)head;
                    const u32x4 c = win[k];
                    const gu8 dst = (gu8)base + 16u * k;
                    const int lo = -pos, hi = (int)w.cur.len - pos;
                    if (lo <= 0 && hi >= 16) {
                        *(GMEM u32x4*)dst = c;
                    } else {
                        const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const uint32_t keep = byte_mask(lo, hi, i);
                            if (keep == 0xffffffffu) {
                                *(GMEM uint32_t*)(dst + 4 * i) = cw[i];
                            } else if (keep) {
#pragma unroll
                                for (int j = 0; j < 4; ++j)
                                    if (keep & (0xffu << (8 * j))) dst[4 * i + j] = (uint8_t)(cw[i] >> (8 * j));
                            }
                        }
                    }
                }
            }
        }
    }

    if (last) {
        w.cur = w.nxt;
        w.nxt = nxt2;
        w.nch = nch2;
        w.r = r2;
    }
    w.step = step2;
    return have2;
}

// MODE_DATA: checksum::data over [0, len).  MODE_EMIT / MODE_VERIFY: the protocol gates.
// MODE_COPY: payload copy + emit in one pass.  VAR: see VarT.
// Occupancy floor (waves per SIMD): variant 28 is 27 held to 7 waves, the occupancy of variant 13 at
// 16 x 4 (descriptor batches); the segment decision's registers otherwise cost it two waves.
template <int VAR, int MODE>
struct MinWaves {
    static constexpr int value = (MODE == MODE_EMIT && VAR == 28) ? 7 : 1;
};

template <int G, int U, int MODE, bool IMPLICIT, int VAR, bool NHC = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MinWaves<VAR, MODE>::value))) void csum_kernel(KParams p) {
    constexpr bool NT = VarT<VAR>::NT;
    constexpr bool PF = VarT<VAR>::PF;
    constexpr bool LINE = VarT<VAR>::LINE;
    constexpr int CU = VarT<VAR>::CACHED_U;
    constexpr bool SHUF = VarT<VAR>::SHUF;
    constexpr bool WHOLE = VarT<VAR>::WHOLE;
    constexpr bool SHUF2 = VarT<VAR>::SHUF2;
    // Fixed-stride batches: no prefetch once the group has nothing left (one record per group in
    // a natural grid), measured 1-1.5 % faster (C2 verify 0.2444 -> 0.2422 ms, C4 0.2219 -> 0.2189
    // ms).  Descriptor batches keep the unconditional prefetch: there the conditional load made
    // C3 verify 25 % slower (0.810 -> 0.989 ms).
    constexpr bool SKIPD = IMPLICIT;
    constexpr bool COPY = MODE == MODE_COPY;
    constexpr int GPB = 256 / G;
    static_assert(G >= 8 && G <= 64 && (G & (G - 1)) == 0, "group size");
    __shared__ u32x4 win[GPB][Grid<LINE>::WIN_CH];
    __shared__ Geom geo[GPB];
    constexpr bool SEGW = VarT<VAR>::SEGW && MODE == MODE_EMIT && IMPLICIT && LINE && !NHC;
    constexpr bool SEGG = VarT<VAR>::SEGG && MODE == MODE_EMIT && LINE && !NHC;
    constexpr bool SEGB = SEGG && VarT<VAR>::SEGB;
    constexpr bool SEG6 = SEGG && VarT<VAR>::SEG6;
    __shared__ SegInfo segi[SEGW ? GPB : 1];
    __shared__ SegInfoG segg[SEGG ? GPB : 1];

    const int lane = (int)(threadIdx.x % G);
    const int gib = (int)(threadIdx.x / G);
    const uint64_t ngroups = (uint64_t)gridDim.x * GPB;
    if constexpr (SEGW) {
        if (lane == 0) segi[gib].tag = segi[gib].tag2 = ~0u;  // no record yet (read by the neighbours)
    }
    if constexpr (SEGG) {
        if (lane == 0) segg[gib].tag = ~0u;
    }
    // SEGB: a natural grid (one record per group) and a full workgroup, the same for every wave of
    // the workgroup, so that each of them reaches the barrier after the parse exactly once
    const uint64_t bid = logical_block(p.xcd_remap);
    const bool blockwide = SEGB && ngroups >= p.n && bid * GPB + GPB <= p.n;
    Walk w;
    w.r = bid * GPB + gib;
    if (w.r >= p.n) return;
    w.cur = rec_at<IMPLICIT, COPY, NHC>(p, w.r);
    w.nxt = rec_at<IMPLICIT, COPY, NHC>(p, w.r + ngroups < p.n ? w.r + ngroups : p.n - 1);
    w.nch = n_chunks<LINE>(w.cur);
    w.step = 0;
    // The record geometry: in LDS, except for emit.  Measured (tools/gpu_ab.sh, MI355X): in LDS,
    // C4 verify 0.2167 -> 0.2044 ms (8 x 6: 113 -> 95 VGPRs, 4 -> 5 waves/SIMD) but C4 emit
    // 0.2656 -> 0.2738 ms; C2 (8 x 7) unchanged either way.
    w.g = &geo[gib];
    w.gr = Geom{};
    w.s1 = 0;
    w.acc = w.acc2 = 0;
    w.fip = w.fl4 = w.fin = NO_FIELD;
    w.far = false;
    w.segA = w.segB = SEG_NONE;

    Regs<U, COPY> va;
    if (PF) {
        Regs<U, COPY> vb;
        load_step<G, U, NT, COPY, LINE, (VarT<VAR>::CU0 ? VarT<VAR>::CU0 : CU), SHUF>(va, w.cur, w.nch, 0, lane, true, (uint64_t)p.dummy,
                                                  shared_from<G, MODE, IMPLICIT, LINE, VarT<VAR>::NOSHARE>(p, w.r, w.cur.a0, gib, ngroups));
        // the body is instantiated twice with the register sets' roles swapped
        while (true) {
            if (!walk_step<G, U, MODE, IMPLICIT, NT, PF, SKIPD, LINE, NHC, CU, SHUF, false, false, SEGW, SEGG, SEGB, SEG6,
                           VarT<VAR>::SEGOPT, VAR>(p, w, va, vb, lane, ngroups, &win[gib][0], gib, segi, segg, blockwide)) break;
            if (!walk_step<G, U, MODE, IMPLICIT, NT, PF, SKIPD, LINE, NHC, CU, SHUF, false, false, SEGW, SEGG, SEGB, SEG6,
                           VarT<VAR>::SEGOPT, VAR>(p, w, vb, va, lane, ngroups, &win[gib][0], gib, segi, segg, blockwide)) break;
        }
    } else {
        while (true) {
            load_step<G, U, NT, COPY, LINE, 0, SHUF, SHUF2>(va, w.cur, w.nch, w.step, lane, true, (uint64_t)p.dummy,
                                                            shared_from<G, MODE, IMPLICIT, LINE, VarT<VAR>::NOSHARE>(p, w.r, w.cur.a0, gib, ngroups));
            if (!walk_step<G, U, MODE, IMPLICIT, NT, PF, SKIPD, LINE, NHC, 0, SHUF, WHOLE, SHUF2, false, SEGG, SEGB, SEG6, 0, VAR>(
                    p, w, va, va, lane, ngroups, &win[gib][0], gib, nullptr, segg, blockwide)) break;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Launch table
// ---------------------------------------------------------------------------------------------

template <int G, int U, int MODE, bool IMPLICIT, int VAR, bool NHC = false>
hipError_t launch_one(const KParams& p, uint32_t max_blocks, hipStream_t s) {
    constexpr uint32_t GPB = 256 / G;
    const uint64_t want = (p.n + GPB - 1) / GPB;
    const uint32_t blocks = grid_blocks(want, max_blocks);
    note_launch(NHC ? KERN_WALK_NHC : KERN_WALK, VAR, G, U);
    hipLaunchKernelGGL((csum_kernel<G, U, MODE, IMPLICIT, VAR, NHC>), dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

template <int MODE, bool IMPLICIT, int VAR>
hipError_t launch_shape(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    switch (shape) {
        case CFG_G8U6: return launch_one<8, 6, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G8U7: return launch_one<8, 7, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G16U3: return launch_one<16, 3, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G16U4: return launch_one<16, 4, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G16U6: return launch_one<16, 6, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G32U3: return launch_one<32, 3, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G32U4: return launch_one<32, 4, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G64U2: return launch_one<64, 2, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        default: return launch_one<64, 4, MODE, IMPLICIT, VAR>(p, max_blocks, s);
    }
}

// The whole-segment emit variants (23-27) are built for the shapes emit picks (8 x 6 / 8 x 7 at a
// fixed stride, 16 x 3 / 16 x 4 over descriptors) and 32 x 4 / 64 x 4 for long records; the other
// shapes map to the one with the same group size.
template <bool IMPLICIT, int VAR>
hipError_t launch_seg_shape(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    switch (shape) {
        case CFG_G8U6: return launch_one<8, 6, MODE_EMIT, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G8U7: return launch_one<8, 7, MODE_EMIT, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G16U3: return launch_one<16, 3, MODE_EMIT, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G16U4:
        case CFG_G16U6: return launch_one<16, 4, MODE_EMIT, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G32U3:
        case CFG_G32U4: return launch_one<32, 4, MODE_EMIT, IMPLICIT, VAR>(p, max_blocks, s);
        default: return launch_one<64, 4, MODE_EMIT, IMPLICIT, VAR>(p, max_blocks, s);
    }
}

#ifdef SMOL_EXP
// Experiment variants of fixed-stride emit (31-38, and | 64 without stores): the two fixed-stride
// shapes only (other shapes map to the one with the same group size).
template <int VAR>
hipError_t launch_emit_exp(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    if (shape == CFG_G8U6) return launch_one<8, 6, MODE_EMIT, true, VAR>(p, max_blocks, s);
    return launch_one<8, 7, MODE_EMIT, true, VAR>(p, max_blocks, s);
}

// The experiments build (SMOL_EXP): every walk variant that was measured and is not a default.
template <int MODE, bool IMPLICIT>
hipError_t launch_walk_exp(int shape, int var, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    if constexpr (MODE == MODE_EMIT && IMPLICIT) {
        switch (var) {
            case 31: return launch_emit_exp<31>(shape, p, max_blocks, s);
            case 32: return launch_emit_exp<32>(shape, p, max_blocks, s);
            case 33: return launch_emit_exp<33>(shape, p, max_blocks, s);
            case 34: return launch_emit_exp<34>(shape, p, max_blocks, s);
            case 35: return launch_emit_exp<35>(shape, p, max_blocks, s);
            case 36: return launch_emit_exp<36>(shape, p, max_blocks, s);
            case 37: return launch_emit_exp<37>(shape, p, max_blocks, s);
            case 38: return launch_emit_exp<38>(shape, p, max_blocks, s);
            case 40: return launch_emit_exp<40>(shape, p, max_blocks, s);
            case 12: return launch_emit_exp<12>(shape, p, max_blocks, s);
            case 14: return launch_emit_exp<14>(shape, p, max_blocks, s);
            case 64 + 39: return launch_emit_exp<64 + 39>(shape, p, max_blocks, s);
            case 64 + 5: return launch_emit_exp<64 + 5>(shape, p, max_blocks, s);
            case 64 + 29: return launch_emit_exp<64 + 29>(shape, p, max_blocks, s);
            case 64 + 31: return launch_emit_exp<64 + 31>(shape, p, max_blocks, s);
            case 64 + 32: return launch_emit_exp<64 + 32>(shape, p, max_blocks, s);
            case 64 + 33: return launch_emit_exp<64 + 33>(shape, p, max_blocks, s);
            case 64 + 34: return launch_emit_exp<64 + 34>(shape, p, max_blocks, s);
            case 64 + 35: return launch_emit_exp<64 + 35>(shape, p, max_blocks, s);
            case 64 + 36: return launch_emit_exp<64 + 36>(shape, p, max_blocks, s);
            case 64 + 37: return launch_emit_exp<64 + 37>(shape, p, max_blocks, s);
            case 64 + 38: return launch_emit_exp<64 + 38>(shape, p, max_blocks, s);
            default: break;
        }
    }
    switch (var) {
        case 1: return launch_shape<MODE, IMPLICIT, 1>(shape, p, max_blocks, s);
        case 2: return launch_shape<MODE, IMPLICIT, 2>(shape, p, max_blocks, s);
        case 6: return launch_shape<MODE, IMPLICIT, 6>(shape, p, max_blocks, s);
        case 19: return launch_shape<MODE, IMPLICIT, 19>(shape, p, max_blocks, s);
        case 29:  // round 4's fixed-stride emit default
            if constexpr (MODE == MODE_EMIT && IMPLICIT) return launch_seg_shape<IMPLICIT, 29>(shape, p, max_blocks, s);
            return launch_shape<MODE, IMPLICIT, 5>(shape, p, max_blocks, s);
        case 23:
        case 24:
        case 25:
        case 26:
        case 27:
        case 28:
            if constexpr (MODE == MODE_EMIT) {
                switch (var) {
                    case 23: return launch_seg_shape<IMPLICIT, 23>(shape, p, max_blocks, s);
                    case 24: return launch_seg_shape<IMPLICIT, 24>(shape, p, max_blocks, s);
                    case 25: return launch_seg_shape<IMPLICIT, 25>(shape, p, max_blocks, s);
                    case 26: return launch_seg_shape<IMPLICIT, 26>(shape, p, max_blocks, s);
                    case 27: return launch_seg_shape<IMPLICIT, 27>(shape, p, max_blocks, s);
                    default: return launch_seg_shape<IMPLICIT, 28>(shape, p, max_blocks, s);
                }
            }
            return var >= 26 ? launch_shape<MODE, IMPLICIT, 13>(shape, p, max_blocks, s)
                             : launch_shape<MODE, IMPLICIT, 5>(shape, p, max_blocks, s);
        case 9:
        case 10:
            if constexpr (MODE == MODE_EMIT && IMPLICIT) {
                return var == 9 ? launch_shape<MODE, IMPLICIT, 9>(shape, p, max_blocks, s)
                                : launch_shape<MODE, IMPLICIT, 10>(shape, p, max_blocks, s);
            }
            return launch_shape<MODE, IMPLICIT, 5>(shape, p, max_blocks, s);
        case 0: return launch_shape<MODE, IMPLICIT, 0>(shape, p, max_blocks, s);
        case 31: case 32: case 33: case 34: case 35: case 36: case 37: case 38: case 40: case 12: case 14:
            return launch_shape<MODE, IMPLICIT, 5>(shape, p, max_blocks, s);  // emit variants: 5 elsewhere
        default: return hipErrorInvalidValue;
    }
}
#endif

// The product variants (csum_api.cpp variant_built): 5 (line grid, nt loads, register prefetch),
// 13 (5 without the prefetch) and, for fixed-stride emit, 39 (5 with whole field segments: 29's
// LDS-published decision on wavefronts with an IPv4 record, one ballot on the others).  Other
// variants: the experiments build.
template <int MODE, bool IMPLICIT>
hipError_t launch_walk(int shape, int var, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    switch (var) {
        case 5: return launch_shape<MODE, IMPLICIT, 5>(shape, p, max_blocks, s);
        case 13: return launch_shape<MODE, IMPLICIT, 13>(shape, p, max_blocks, s);
        case 39:
            if constexpr (MODE == MODE_EMIT && IMPLICIT) return launch_seg_shape<IMPLICIT, 39>(shape, p, max_blocks, s);
            return launch_shape<MODE, IMPLICIT, 5>(shape, p, max_blocks, s);
        default:
#ifdef SMOL_EXP
            return launch_walk_exp<MODE, IMPLICIT>(shape, var, p, max_blocks, s);
#else
            return hipErrorInvalidValue;
#endif
    }
}

// 6LoWPAN NHC UDP batches: the walk kernel instantiated with the NHC gates, on the two default
// variants (1: 16-B grid, cached loads; 5: line grid, nt loads) and three shapes (other shapes map
// to the one with the same group size or the nearest).
template <int MODE, bool IMPLICIT>
hipError_t launch_walk_nhc(int shape, int var, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    const int g = (shape == CFG_G8U6 || shape == CFG_G8U7) ? shape : CFG_G16U3;
    // the line-grid variants (the descriptor-verify default 13 included) run variant 5 here
    if (var == 5 || var == 6 || var == 9 || var == 10 || var == 13 || var == 19 || (var >= 23 && var <= 29)) {
        if (g == CFG_G8U6) return launch_one<8, 6, MODE, IMPLICIT, 5, true>(p, max_blocks, s);
        if (g == CFG_G8U7) return launch_one<8, 7, MODE, IMPLICIT, 5, true>(p, max_blocks, s);
        return launch_one<16, 3, MODE, IMPLICIT, 5, true>(p, max_blocks, s);
    }
    if (g == CFG_G8U6) return launch_one<8, 6, MODE, IMPLICIT, 1, true>(p, max_blocks, s);
    if (g == CFG_G8U7) return launch_one<8, 7, MODE, IMPLICIT, 1, true>(p, max_blocks, s);
    return launch_one<16, 3, MODE, IMPLICIT, 1, true>(p, max_blocks, s);
}

// MODE_COPY keeps three chunks per lane and step (record + two source chunks), so it is built for
// the U <= 3 shapes only (wider shapes map to the same group size with fewer chunks) and for the
// plain-load variants on the 16-byte grid.  (Copy-emit's default is now variant 17, copy_kernel in
// csum_copy.hip.)  Without the register prefetch (variant 8, round 1's default)
// the kernel needs fewer VGPRs and runs more waves per SIMD: C2 copy-emit 0.95 -> 0.85 ms on
// MI355X (tools/gpu_exp.sh sweep, profiles/r01_kernel_stats_c2copy.csv); variant 1 keeps the
// prefetch for comparison.
template <bool IMPLICIT, int VAR>
hipError_t launch_copy_var(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    switch (shape) {
        case CFG_G8U6:
        case CFG_G8U7: return launch_one<8, 3, MODE_COPY, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G32U3:
        case CFG_G32U4: return launch_one<32, 3, MODE_COPY, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G64U2:
        case CFG_G64U4: return launch_one<64, 2, MODE_COPY, IMPLICIT, VAR>(p, max_blocks, s);
        default: return launch_one<16, 3, MODE_COPY, IMPLICIT, VAR>(p, max_blocks, s);
    }
}

// variant 17: the class-split copy-emit kernel (csum_copy.hip)
hipError_t launch_copy_v17(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s);
// variant 21: variant 17 with the first body round's loads ahead of round 1's stores (csum_copy.hip)
hipError_t launch_copy_v21(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s);
#ifdef SMOL_EXP
// variants 30 / 22: 21 with non-temporal body stores / and source loads (csum_copy.hip)
hipError_t launch_copy_nt(int var, const KParams& p, uint32_t max_blocks, hipStream_t s);
#endif

// 17 / 21 (copy_kernel) are the product's; the walk kernel's MODE_COPY variants (1, 8, 11, 16: the
// round-1 / 2 designs) are in the experiments build only.
template <bool IMPLICIT>
hipError_t launch_copy(int shape, int var, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    switch (var) {
        case 17: return launch_copy_v17(shape, p, max_blocks, s);
        case 21: return launch_copy_v21(shape, p, max_blocks, s);
#ifdef SMOL_EXP
        case 30:
        case 98:
        case 102:
        case 22: return launch_copy_nt(var, p, max_blocks, s);
        case 1: return launch_copy_var<IMPLICIT, 1>(shape, p, max_blocks, s);
        case 11: return launch_copy_var<IMPLICIT, 11>(shape, p, max_blocks, s);
        case 8: return launch_copy_var<IMPLICIT, 8>(shape, p, max_blocks, s);
        case 16: return launch_copy_var<IMPLICIT, 16>(shape, p, max_blocks, s);
#endif
        default: return hipErrorInvalidValue;
    }
}

}  // namespace smolcsum
