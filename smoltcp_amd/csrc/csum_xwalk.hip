// Transposed walk (variants 44 / 47): fixed-stride emit / verify of records of 1024 .. 16257 bytes
// (packed or with gaps) over a natural grid, with the walk kernel's per-record work (a group
// of G lanes parses and finishes one record, R = 64 / G records per wavefront) and a different load
// mapping.
//
// The walk kernel's load instruction covers one 128-B line in each of the wavefront's 8 records
// (8 lanes per record); here load instruction (s, j) covers 1 KiB of ONE record: chunks
// 64 s .. 64 s + 63 of record j, one per lane, NS = 16 / R instructions per record.  A read-only probe
// of the two patterns over C2's 1.5 GB (tools/probe_pol.hip, profiles/r05_experiments/
// read_shape_probe.txt): 6.5 TB/s for the walk's (8 lanes, 2 steps), 7.2 TB/s for a whole wavefront
// per record in one step.  All 16 loads of a wavefront are issued at once, as buffer loads: one
// resource per wavefront based at its first record's line, record j's line offset as the scalar
// offset, the chunk as the lane's offset; a chunk past the record's loads gets an offset past the
// resource's range, which returns 0 without a memory access.  R by record length: 8 up to 1921 B,
// 4 up to 3969 B, 2 up to 8065 B, 1 up to 16257 B.
//
// Sums.  A lane adds its chunk of record j to its accumulator j (j is a compile-time index), and a
// reduce-scatter over the wavefront (exchanges across 32, 16, .., G lanes, then the group's own
// reduction) leaves record j's sum in group j.  Chunks are summed whole, up to the one holding the
// span's end (whose bytes past it its lane takes out again), and corrected from the LDS windows:
//  - the bytes of a record's first line before its start belong to the previous record:
//    subtracted (hs_j, from record j's window) and, for packed records whose previous record is in
//    this wavefront, added to that record, which does not load the line (the line holding record
//    j + 1's first byte is loaded once, as record j + 1's first chunk: csum_walk.h shared_from).
//
// Measured (profiles/r05_experiments/xwalk_*.jsonl): the other forms tried, a
// 64-bit-address load from the dummy line for out-of-range chunks, a persistent grid (one wavefront
// steps over the batch 8 records at a time, with or without the next step's loads issued ahead:
// PERSIST, variant 48) and 5 wavefronts per SIMD (96 VGPRs), were all slower.  The library uses it
// where it beats the walk kernel (csum_api.cpp xwalk_auto): verify of packed records from 1473 B
// (not multiples of 128 B below 1666 B), verify of gapped records and emit from 1666 B, up to 8065 B.
#include "csum_walk.h"

namespace smolcsum {

namespace xwalk {

constexpr int WIN_CH = 16;  // the LDS window: 256 B from the record's 128-B line
constexpr int WAVES = 4;    // wavefronts per workgroup

// The value of lane ^ H (H = 32 / 16 / 8 / ..: across the wavefront, a 32-lane half, a row)
template <int H>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
    if constexpr (H == 32) return (uint32_t)__shfl_xor((int)v, 32, 64);
    else if constexpr (H == 16) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);
    else return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
}

// Reduce-scatter of acc[0 .. N) over the lanes of bit H and below down to G: record j's partial sums
// end in the lanes with (lane / G) % (N) == j.
template <int N, int H>
__device__ __forceinline__ uint32_t reduce_scatter(const uint32_t* acc, int wl) {
    if constexpr (N == 1) {
        return acc[0];
    } else {
        const bool up = (wl & H) != 0;
        uint32_t a[N / 2];
#pragma unroll
        for (int i = 0; i < N / 2; ++i) {
            const uint32_t keep = up ? acc[i + N / 2] : acc[i];
            const uint32_t send = up ? acc[i] : acc[i + N / 2];
            a[i] = keep + lane_xor<H>(send);
        }
        return reduce_scatter<N / 2, H / 2>(a, wl);
    }
}

}  // namespace xwalk

// SEG (variant 47; emit): the 64-B segments that hold a record's fields go out whole from its LDS
// window, the fields patched in (csum_walk.h variant 38's decision, the wavefront's groups all on
// their one record): a whole segment costs HBM a plain write where a 2-B store costs a
// read-modify-write.  NOSTORE (variant 64 + v): emit computes every field value and stores none.
// PERSIST (variant 48, experiments build): a grid of the resident workgroups whose wavefronts step
// over the batch, issuing the next step's loads as soon as this step's sums are taken (before its
// finish and stores), so that no wavefront ends while its stores drain.
// NTS: the segments stored non-temporal, always (variant 57, the product's emit of packed
// 1400-1580-B records, csum_api.cpp xwalk_auto) or on a wavefront that holds an IPv4 record (58,
// experiments build).  NTS = 4 (variant 45, experiments build): each record's first load
// instruction (its first KiB, header lines included) with the default cache policy instead of
// non-temporal, so that the field stores hit lines the L2 holds (the descriptor walk's variant 63
// finding).  NTS = 8 (variant 43,
// experiments build): every load with the default cache policy; NTS = 16 (variant 46, experiments
// build): only the record's two header lines (lanes 0-15 of its first instruction) cached; NTS = 5
// (variant 15, experiments build): 45 with the segments stored non-temporal.
// HALF (variant 59, experiments build; R = 8, records of at most 1409 B, whose line-grid span fits
// 96 chunks): a record's second KiB is half an instruction, two records per instruction, so a
// wavefront issues 12 loads instead of 16.
// NTS = 65 (variant 101, the product's emit where the dispatch table says 'n', since late round 6): the
// segments stored with sc1 nt, write-through and non-temporal (the staged emit's segment-pass policy,
// here inside the stream), as a vector store written as the instruction; NTS = 64 (variant 100,
// experiments build): sc0 sc1 nt.
// STAGE (variants 80 / 81, round 6; emit): the field segments are not written here.  A record whose
// fields the whole segments cover (47's rule, all or nothing) stages one 8-B entry (its two field
// offsets and values, csum_walk.h stage_entry) in p.stage, and the segment pass (csum_dwalk.hip
// seg_pass4_kernel) writes the segments after this launch; any other
// record writes its fields here as 2-B stores and stages nothing.  NTS = 32 (variant 80): the
// lanes of a record's first instruction that hold the segments of record offsets [10, 28) (an IPv4
// record's two fields) load with the default cache policy, so that the segment pass finds those lines
// on chip; 81: every load non-temporal.  Why (tools/probe_wtax.hip): field
// writes that land while a read stream runs cost 65-77 ps each, the same writes in a pass of their own
// ~20 ps.
template <int MODE, int R, bool NOSTORE, bool SEG, bool PERSIST = false, int NTS = 0, bool HALF = false,
          bool STAGE = false, int HINT = 0, int WPE = 0, int WV = xwalk::WAVES, int STEPS = 1>
__global__ __launch_bounds__(64 * WV) __attribute__((amdgpu_waves_per_eu(WPE > 0 ? WPE : 1))) void xwalk_kernel(KParams p) {
    using namespace xwalk;
    constexpr bool EMIT = MODE == MODE_EMIT;
    constexpr int G = 64 / R;    // lanes per record
    constexpr int NS = 16 / R;   // load instructions (1 KiB each) per record
    constexpr int GPB = WV * R;  // WV: wavefronts per workgroup (8 in variant 107: a workgroup's 64 status bytes fill one segment)
    __shared__ u32x4 win[GPB][WIN_CH];
    __shared__ uint32_t spanbuf[GPB];
    const int wl = (int)(threadIdx.x & 63);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // uniform: scalar offsets
    const int lane = wl & (G - 1);
    const int gw = wl / G;  // the group (record) within the wavefront
    const int gib = wv * R + gw;
    const uint32_t len = p.len;
    const uint64_t stride = p.stride;
    // packed records share lines with their neighbours (each line is loaded once); with a gap every
    // record loads all its lines and sums them masked to its span
    const bool packed = stride == (uint64_t)len;
    // STEPS (variant 113, experiments build): a workgroup takes STEPS consecutive tiles of WV wavefronts
    // (wavefront w: tiles w, w + WV, ...), so that its records' status bytes fill whole segments
    const uint64_t nwaves = PERSIST ? (uint64_t)gridDim.x * WV : (uint64_t)(STEPS > 1 ? WV : 0);
    uint64_t tw = logical_block(p.xcd_remap) * WV * STEPS + (uint64_t)wv;  // the wavefront's step
    int step = 0;
    if (tw * R >= p.n) return;

    // ---- all loads of a step's records (record j: chunks below nload_j of its line grid) ----
    static_assert(!HALF || R == 8, "HALF: 8 records per wavefront");
    u32x4 v[NS][R];
    u32x4 vq[R / 2 > 0 ? R / 2 : 1];  // HALF: instruction q, lanes 0-31 / 32-63: chunks 64 .. 95 of records 2q / 2q + 1
    uint32_t head[R], nload[R];
    auto issue = [&](uint64_t t) {
        const uint64_t r0 = t * R;
        const uint32_t c = (uint32_t)(p.n - r0 < (uint64_t)R ? p.n - r0 : (uint64_t)R);
        const uint64_t wbase = ((uint64_t)p.buf + r0 * stride) & ~127ull;
        const uint32_t whi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(wbase >> 32));
        const uint32_t wlo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)wbase);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)whi << 32) | wlo), 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint64_t a0 = (uint64_t)p.buf + (r0 + (uint64_t)j) * stride;
            const uint64_t b = a0 & ~127ull;
            head[j] = (uint32_t)(a0 - b);
            const uint32_t nch = (uint32_t)j < c ? (uint32_t)(((a0 + len + 15) >> 4) - (b >> 4)) : 0u;
            // packed: the line holding record j + 1's first byte is record j + 1's to load
            const bool shared = packed && (uint32_t)j + 1 < c;
            nload[j] = shared ? (uint32_t)((((a0 + stride) & ~127ull) - b) >> 4) : nch;
            const int soff = __builtin_amdgcn_readfirstlane((int)(uint32_t)(b - wbase));
#pragma unroll
            for (int s = 0; s < (HALF ? 1 : NS); ++s) {
                const uint32_t k = (uint32_t)(64 * s + wl);
                const uint32_t o = k < nload[j] ? 16u * k : 0x80000000u;
                if ((NTS == 32 || (HINT >= 1 && HINT <= 7)) && s == 0) {  // some header lanes with the default cache policy
                    // HINT 1 (and NTS 32): the segments of record offsets [10, 28) (an IPv4 record's fields);
                    // 2: those of [0, 64); 3: the whole 256-B window; 4: the segment of offset 10 only;
                    // 5: the 16-B chunk of offset 10 only; 6: the segment of the record's first byte;
                    // 7: the line's first segment (lanes 0-3)
                    const uint32_t sg = (uint32_t)wl >> 2, h = head[j];
                    const bool c = (HINT == 0 || HINT == 1) ? (sg == (h + 10u) >> 6 || sg == (h + 27u) >> 6)
                                   : HINT == 2 ? (sg == h >> 6 || sg == (h + 63u) >> 6)
                                   : HINT == 3 ? wl < 16
                                   : HINT == 4 ? sg == (h + 10u) >> 6
                                   : HINT == 5 ? (uint32_t)wl == (h + 10u) >> 4
                                   : HINT == 6 ? sg == h >> 6
                                               : wl < 4;
                    if (c) v[s][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, 0);
                    else v[s][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, 2);
                } else if ((HINT == 8 && s == 0) || (HINT == 9 && s == 1) || HINT == 10) {
                    // 8: instruction 0 split in two (lanes 0-3 / the rest), both non-temporal; 9: lanes 0-3 of
                    // instruction 1 with the default policy; 10: lanes 0-3 of every instruction
                    if (wl < 4) v[s][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, HINT == 8 ? 2 : 0);
                    else v[s][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, 2);
                } else if (((NTS == 4 || NTS == 5) && s == 0) || NTS == 8) v[s][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, 0);
                else if (NTS == 16 && s == 0) {  // the header lines cached, the rest of the KiB nt
                    if (wl < 16) v[s][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, 0);
                    else v[s][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, 2);
                } else v[s][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, 2 /* nt */);
            }
        }
        if constexpr (HALF) {
#pragma unroll
            for (int q = 0; q < R / 2; ++q) {
                const bool hi = wl >= 32;
                const uint32_t k = 64u + (uint32_t)(wl & 31);
                const uint64_t bA = ((uint64_t)p.buf + (r0 + 2ull * q) * stride) & ~127ull;
                const uint64_t bB = ((uint64_t)p.buf + (r0 + 2ull * q + 1) * stride) & ~127ull;
                const uint32_t off = (uint32_t)((hi ? bB : bA) - wbase);
                const uint32_t nl = hi ? nload[2 * q + 1] : nload[2 * q];
                vq[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, k < nl ? off + 16u * k : 0x80000000u, 0, 2 /* nt */);
            }
        }
    };
    issue(tw);
    for (;;) {
    const uint64_t rw0 = tw * R;  // the wavefront's first record
    const uint32_t cnt = (uint32_t)(p.n - rw0 < (uint64_t)R ? p.n - rw0 : (uint64_t)R);
    // ---- the windows: chunks 0 .. 15 of record j are lanes 0 .. 15 of load (0, j) ----
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (wl < WIN_CH && (uint32_t)j < cnt) win[wv * R + j][wl] = v[0][j];
    wave_lds_sync();

    const bool mine = (uint32_t)gw < cnt;
    const uint64_t r = rw0 + (uint64_t)gw;
    const uint64_t a0 = (uint64_t)p.buf + r * stride;
    const uint32_t hd = (uint32_t)(a0 & 127u);
    const uint8_t* winb = reinterpret_cast<const uint8_t*>(&win[gib][0]);
    auto rd = [&](uint32_t o) -> uint32_t {
        const uint32_t x = hd + o;
        if (x < 16u * WIN_CH) return (uint32_t)winb[x];
        return ld_byte_sync(a0 + o);
    };
    Geom g = Geom{};
    if (mine) g = parse_geometry<false>(rd, len, p.kind, EMIT);
    const bool l4 = g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED);
    const int s1 = mine && l4 ? (int)g.span_end : 0;
    // hs: the bytes of this record's first line before its start (window bytes [0, hd)), as
    // aligned words; lane i takes window chunks i, i + G, ..
    uint32_t hs = 0;
#pragma unroll
    for (int c = 0; c < WIN_CH; c += G)
        if (c + lane < WIN_CH) hs = sum_masked_words(win[gib][c + lane], 0, (int)hd - 16 * (c + lane), hs);
    hs = group_sum<G>(hs);
    if (lane == 0) spanbuf[gib] = (uint32_t)s1;
    wave_lds_sync();
    int span[R];
#pragma unroll
    for (int j = 0; j < R; ++j) span[j] = (int)spanbuf[wv * R + j];

    // ---- sums: accumulator j of every lane holds its chunks of record j ----
    // Chunks below kend_j (the loaded chunks up to the span's end) are summed whole; the lane whose
    // chunk holds the span's end takes the bytes past it out again.  The bytes before the record in
    // its first line (hs) come out after the reduction.
    uint32_t acc[R], kend[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
        acc[j] = 0;
        const int hj = (int)head[j], sj = span[j];
        kend[j] = min(nload[j], (uint32_t)(hj + sj + 15) >> 4);
#pragma unroll
        for (int s = 0; s < (HALF ? 1 : NS); ++s) {
            const uint32_t k = (uint32_t)(64 * s + wl);
            const u32x4 c = v[s][j];
            const int pos = 16 * (int)k - hj;
            uint32_t x = k < kend[j] ? add_words(c.x, add_words(c.y, add_words(c.z, add_words(c.w, 0u)))) : 0u;
            if (k < kend[j] && pos + 16 > sj) x -= sum_masked_words(c, sj - pos, 16, 0u);
            acc[j] += x;
        }
    }
    if constexpr (HALF) {
#pragma unroll
        for (int q = 0; q < R / 2; ++q) {
            const bool hi = wl >= 32;
            const uint32_t k = 64u + (uint32_t)(wl & 31);
            const int hj = (int)(hi ? head[2 * q + 1] : head[2 * q]);
            const int sj = hi ? span[2 * q + 1] : span[2 * q];
            const uint32_t ke = hi ? kend[2 * q + 1] : kend[2 * q];
            const u32x4 c = vq[q];
            const int pos = 16 * (int)k - hj;
            uint32_t x = k < ke ? add_words(c.x, add_words(c.y, add_words(c.z, add_words(c.w, 0u)))) : 0u;
            if (k < ke && pos + 16 > sj) x -= sum_masked_words(c, sj - pos, 16, 0u);
            acc[2 * q] += hi ? 0u : x;
            acc[2 * q + 1] += hi ? x : 0u;
        }
    }
    // the next step's loads, ahead of this step's finish and stores
    const uint64_t tn = tw + nwaves;
    const bool more = (PERSIST || step + 1 < STEPS) && tn * R < p.n;
    if (more) issue(tn);
    // ---- reduce-scatter: record j's sum to group j ----
    uint32_t tot = group_sum<G>(reduce_scatter<R, 32>(acc, wl)) - hs;
    // packed: the bytes of this record's last line, which record j + 1 loaded, are record offsets
    // [len - hdn, len) = record j + 1's window bytes [0, hdn) (its hs when the span runs to the end)
    const uint32_t hs_next = (uint32_t)__shfl_down((int)hs, G, 64);
    if (packed && (uint32_t)gw + 1 < cnt) {
        if (s1 == (int)len) {
            tot += hs_next;
        } else {
            const uint32_t hdn = (uint32_t)((a0 + stride) & 127u);
            const int lim = min((int)hdn, s1 - ((int)len - (int)hdn));
            uint32_t t = 0;
#pragma unroll
            for (int c = 0; c < WIN_CH; c += G)
                if (c + lane < WIN_CH) t = sum_masked_words(win[gib + 1][c + lane], 0, lim - 16 * (c + lane), t);
            tot += group_sum<G>(t);
        }
    }
    // ---- finish: the walk kernel's gates (lane 0 writes) ----
    if constexpr (EMIT && SEG) {
        // A segment that starts before the record also holds record r-1's last bytes: whole only
        // for packed records, when r-1 has no field in its last 64 bytes (its group says so:
        // ok_tail) and r-1 is in this wavefront.  A record whose fields end 64 bytes or more before
        // its end never reaches into r+1 with its own segments, and r-1's segments then end before
        // this record, so no two groups write one segment.
        uint32_t f[3], lo = NO_FIELD, hi = 0;
        emit_fields(g, f);
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if (f[i] != NO_FIELD) {
                lo = f[i] < lo ? f[i] : lo;
                hi = f[i] + 2 > hi ? f[i] + 2 : hi;
            }
        const bool ok_tail = hi == 0 || hi + 64 <= len;
        const uint64_t okm = __ballot(lane == 0 && mine && ok_tail);
        uint64_t wsA = ~0ull, wsB = ~0ull;
        if (mine && (g.fam == 4 || g.fam == 6) && hi != 0 && ok_tail) {
            // gapped strides: the record's own bytes only (a gap is never written)
            const bool prev_ok = packed && gw != 0 && ((okm >> (wl - lane - G)) & 1ull);
            const int32_t ph = (int32_t)(a0 & 63u);
            const int32_t rA = ((ph + (int32_t)lo) & ~63) - ph, rB = ((ph + (int32_t)hi - 1) & ~63) - ph;
            const int32_t wend = 16 * WIN_CH - (int32_t)hd;
            auto whole_seg = [&](int32_t rel) { return rB <= rA + 64 && rel + 64 <= wend && (rel >= 0 || prev_ok); };
            if (whole_seg(rA)) wsA = a0 + (int64_t)rA;
            if (rB != rA && whole_seg(rB)) wsB = a0 + (int64_t)rB;
        }
        bool staged = false;
        if constexpr (STAGE) {
            // all or nothing: staged when the whole segments cover both bytes of every field (and the
            // record has no third field); otherwise every field goes out here as a 2-B store
            auto cov = [&](uint32_t fo) {
                const uint64_t x0 = (a0 + fo) & ~63ull, x1 = (a0 + fo + 1) & ~63ull;
                return (x0 == wsA || x0 == wsB) && (x1 == wsA || x1 == wsB);
            };
            staged = wsA != ~0ull && f[2] == NO_FIELD && (f[0] == NO_FIELD || cov(f[0])) && (f[1] == NO_FIELD || cov(f[1]));
            if (!staged) wsA = wsB = ~0ull;
        }
        uint8_t* winw = reinterpret_cast<uint8_t*>(&win[gib][0]);
        if (mine)
            finish_gates<G, MODE, false, decltype(rd), 16 * WIN_CH, true, NOSTORE>(
                p, g, lane == 0 ? tot : 0u, rd, winb, hd, a0, r, lane, winw, wsA, wsB);
        const bool nts = NTS == 1 || NTS == 5 || (NTS == 2 && __any(mine && g.fam == 4));
        wave_lds_sync();
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        const uint64_t wb = a0 & ~127ull;
        auto seg_store = [&](uint64_t d) {
            const u32x2 x = *reinterpret_cast<const u32x2*>(winb + (d - wb));
            if constexpr (NOSTORE) asm volatile("" ::"v"(x), "v"(d));
            else if constexpr (NTS == 64)  // (variant 100) write-through non-temporal vector store
                asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1 nt" ::"v"(d), "v"(x) : "memory");
            else if constexpr (NTS == 65)  // (variant 101) sc1 nt
                asm volatile("global_store_dwordx2 %0, %1, off sc1 nt" ::"v"(d), "v"(x) : "memory");
            else if (nts) __builtin_nontemporal_store(x, (GMEM u32x2*)d);
            else *(GMEM u32x2*)d = x;
        };
        if constexpr (STAGE) {
            if (mine && lane == 0) stage_record(p, r, staged, g, winb, hd);
            if (mine && lane == 0 && r % 8 == 0) p.stage_flags[r / 8] = 1u;  // every entry is written
        } else {
            if (wsA != ~0ull && lane < 8) seg_store(wsA + 8u * (uint32_t)lane);
            if (wsB != ~0ull && lane < 8) seg_store(wsB + 8u * (uint32_t)lane);
        }
    } else {
        if (mine)
            finish_gates<G, MODE, false, decltype(rd), 0, false, NOSTORE, (NTS & 128) != 0>(p, g, lane == 0 ? tot : 0u, rd,
                                                                                           winb, hd, a0, r, lane);
    }
    if (!more) break;
    wave_lds_sync();  // the windows are rewritten by the next step
    tw = tn;
    ++step;
    }
}

// records per wavefront for a record length (0: not served)
static int xwalk_records(uint32_t len) {
    if (len < 1024) return 0;
    for (int R = 8; R >= 1; R /= 2)
        if (len <= 1024u * (16 / R) - 127u) return R;
    return 0;
}

template <int R>
static void launch_xwalk_r(int mode, int variant, uint32_t blocks, const KParams& p, hipStream_t s) {
#ifdef SMOL_EXP
    if (mode == MODE_EMIT && staged_variant(variant)) {  // the staging launch (the segment pass follows)
        if (variant == 80) hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 32, false, true>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 0, false, true>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if (variant == 82 || variant == 83) {  // round 6: the field-segment lines loaded cached (HINT); 82 verify / 47's
                                          // emit, 83 = 57 (nt segment stores) + the hint
        if (mode == MODE_VERIFY) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 1>), dim3(blocks), dim3(256), 0, s, p);
        else if (variant == 83) hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 1, false, false, 1>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 0, false, false, 1>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if (variant == 113 && mode == MODE_VERIFY) {  // 89 with two tiles per workgroup (64 records at R = 8)
        hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 7, 0, xwalk::WAVES, 2>), dim3((blocks + 1) / 2),
                           dim3(256), 0, s, p);
        return;
    }
    if (variant == 113 && mode == MODE_EMIT) {  // 101 with two tiles per workgroup
        hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 65, false, false, 0, 0, xwalk::WAVES, 2>), dim3((blocks + 1) / 2),
                           dim3(256), 0, s, p);
        return;
    }
    if (variant == 108 && mode == MODE_VERIFY) {  // 89 with the status bytes stored non-temporal (NTS 128)
        hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 128, false, false, 7>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if (variant == 107 && mode == MODE_VERIFY && R == 8) {  // 89 in 512-thread workgroups (64 records, 64 status bytes)
        hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 7, 0, 8>), dim3((blocks + 1) / 2),
                           dim3(512), 0, s, p);
        return;
    }
    if ((variant == 110 || variant == 112) && mode == MODE_EMIT) {  // 101 + first-load hint 7 (110) / 1 (112); verify: 89
        if (variant == 110) hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 65, false, false, 7>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 65, false, false, 1>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if ((variant == 110 || variant == 112) && mode == MODE_VERIFY) {
        hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 7>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if ((variant == 107 || variant == 108) && mode == MODE_EMIT) {  // (107's / 108's emit: 101)
        hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 65>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if (variant == 106 && mode == MODE_VERIFY) {  // 89 without its status stores (timing only, experiments build)
        hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, true, false, false, 0, false, false, 7>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if (variant == 100) {  // round 6: 57 with the segments stored sc0 sc1 nt (101: sc1 nt, the product's); verify: 89
        if (mode == MODE_VERIFY) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 7>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 64>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if (variant == 93 || variant == 99) {  // round 6: 89 / 57 held to 5 (93) or 6 (99) wavefronts per SIMD
        if (variant == 93) {
            if (mode == MODE_VERIFY) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 7, 5>), dim3(blocks), dim3(256), 0, s, p);
            else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 1, false, false, 0, 5>), dim3(blocks), dim3(256), 0, s, p);
        } else {
            if (mode == MODE_VERIFY) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 7, 6>), dim3(blocks), dim3(256), 0, s, p);
            else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 1, false, false, 0, 6>), dim3(blocks), dim3(256), 0, s, p);
        }
        return;
    }
    if (variant >= 90 && variant <= 92) {  // verify hint forms 8-10 (emit: 57)
        if (mode == MODE_VERIFY) {
            if (variant == 90) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 8>), dim3(blocks), dim3(256), 0, s, p);
            else if (variant == 91) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 9>), dim3(blocks), dim3(256), 0, s, p);
            else hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 10>), dim3(blocks), dim3(256), 0, s, p);
        } else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 1>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if (variant >= 84 && variant <= 88) {  // verify hint forms 2-6 (emit: 57 with the same hint)
        if (mode == MODE_VERIFY) {
            switch (variant) {
                case 84: hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 2>), dim3(blocks), dim3(256), 0, s, p); break;
                case 85: hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 3>), dim3(blocks), dim3(256), 0, s, p); break;
                case 86: hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 4>), dim3(blocks), dim3(256), 0, s, p); break;
                case 87: hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 5>), dim3(blocks), dim3(256), 0, s, p); break;
                default: hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 6>), dim3(blocks), dim3(256), 0, s, p); break;
            }
        } else {
            switch (variant) {
                case 86: hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 1, false, false, 4>), dim3(blocks), dim3(256), 0, s, p); break;
                case 87: hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 1, false, false, 5>), dim3(blocks), dim3(256), 0, s, p); break;
                default: hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 1, false, false, 1>), dim3(blocks), dim3(256), 0, s, p); break;
            }
        }
        return;
    }
    if constexpr (R == 8) {
        if (variant == 59 && p.len <= 1409) {
            if (mode == MODE_VERIFY)
                hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, 8, false, false, false, 0, true>), dim3(blocks), dim3(256), 0, s, p);
            else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, 8, false, true, false, 0, true>), dim3(blocks), dim3(256), 0, s, p);
            return;
        }
    }
    if (variant == 15) {
        if (mode == MODE_VERIFY) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 5>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if (variant == 46) {
        if (mode == MODE_VERIFY) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 16>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if (variant == 43) {
        if (mode == MODE_VERIFY) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 8>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 8>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if (variant == 58) {
        if (mode == MODE_VERIFY) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 2>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if (variant == 45) {
        if (mode == MODE_VERIFY) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 4>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
    if (variant == 48) {  // persistent, next step's loads ahead (the resident workgroups)
        const uint32_t cap = mode == MODE_VERIFY
                                 ? resident_blocks((const void*)xwalk_kernel<MODE_VERIFY, R, false, false, true>,
                                                   p.num_cu ? p.num_cu : 256u, blocks)
                                 : resident_blocks((const void*)xwalk_kernel<MODE_EMIT, R, false, true, true>,
                                                   p.num_cu ? p.num_cu : 256u, blocks);
        const uint32_t b = blocks < cap ? blocks : cap;
        if (mode == MODE_VERIFY) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, true>), dim3(b), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, true>), dim3(b), dim3(256), 0, s, p);
        return;
    }
#endif
    const bool seg = variant % 64 == 47 || variant == 57 || variant == 89 || variant == 101;
    if (mode == MODE_VERIFY) {  // (57: 47's verify; 101: 89's)
        // 89 (round 6): lanes 0-3 of each record's first instruction (the first 64 B of its first line)
        // load with the default cache policy, the rest non-temporal: C2 verify 0.2342 -> 0.2259 ms
        // (bench lines interleaved on one box, profiles/r06_experiments/verify_hint_ab.txt); the split
        // itself without the policy change (90) gains nothing
        if (variant == 89 || variant == 101) hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false, false, 0, false, false, 7>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((xwalk_kernel<MODE_VERIFY, R, false, false>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
#ifdef SMOL_EXP
    // 64 + 44 / 64 + 47: stores compiled out (timing only); the numbers from 80 up are round-6 forms
    if (variant == 64 + 44 || variant == 64 + 47) {
        if (seg) hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, true, true>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, true, false>), dim3(blocks), dim3(256), 0, s, p);
        return;
    }
#endif
    // 101 (late round 6): 57's segments stored write-through (sc1 nt): C2 emit 0.3089-0.3102 ->
    // 0.3061-0.3064 ms, C4 0.2728-0.2739 -> 0.2682-0.2689 ms (bench lines interleaved on one box,
    // profiles/r06_experiments/writethrough_segments_ab.txt)
    if (variant == 101) hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 65>), dim3(blocks), dim3(256), 0, s, p);
    else if (variant == 57 || variant == 89) hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true, false, 1>), dim3(blocks), dim3(256), 0, s, p);
    else if (seg) hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, true>), dim3(blocks), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((xwalk_kernel<MODE_EMIT, R, false, false>), dim3(blocks), dim3(256), 0, s, p);
}

bool xwalk_fits(const KParams& p) {
    // the buffer offsets of a wavefront's records stay below 2^31
    return p.desc == nullptr && p.stride >= p.len && p.stride <= (1ull << 26) && xwalk_records(p.len) > 0;
}

hipError_t launch_xwalk(int mode, int variant, const KParams& p, hipStream_t s) {
    const int R = xwalk_records(p.len);
    if (R == 0) return hipErrorInvalidValue;
    const uint64_t per = (uint64_t)xwalk::WAVES * R;
    note_launch(KERN_XWALK, (uint32_t)variant, 64 / R, 16 / R);
    // one workgroup per 4R records and no grid-stride loop: a batch past kMaxGridBlocks workgroups
    // (more records than 288 GB of HBM holds at these lengths) goes out as several launches
    const uint64_t span = kMaxGridBlocks * per;
    for (uint64_t i0 = 0; i0 < p.n; i0 += span) {
        KParams q = p;
        q.n = p.n - i0 < span ? p.n - i0 : span;
        q.buf = p.buf + i0 * p.stride;
        if (p.status) q.status = p.status + i0;
        const uint32_t b = grid_blocks((q.n + per - 1) / per, kMaxGridBlocks);
        switch (R) {
            case 8: launch_xwalk_r<8>(mode, variant, b, q, s); break;
            case 4: launch_xwalk_r<4>(mode, variant, b, q, s); break;
            case 2: launch_xwalk_r<2>(mode, variant, b, q, s); break;
            default: launch_xwalk_r<1>(mode, variant, b, q, s); break;
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
#ifdef SMOL_EXP
        if (mode == MODE_EMIT && staged_variant(variant)) {
            if (!q.stage || !q.stage_flags || q.n > kStageChunk) return hipErrorInvalidValue;
            e = launch_seg_pass(q, s);
            if (e != hipSuccess) return e;
        }
#endif
    }
    return hipSuccess;
}

}  // namespace smolcsum
