// Descriptor-batch walks (dwalk_kernel): verify / emit of records of any length and layout, with
// the walk kernel's per-record parse and gates, 8 records per wavefront.
//
// Variant 63 (the product's descriptor-batch verify and emit since round 5) is variant 60 with the
// header windows loaded with the default cache policy: the stream below reads those lines again
// (non-temporal loads, line grid from the record's first line) and emit's field stores write them;
// with the windows cached both hit the L2.  Measured (bench.py --config c3, 4 batch pairs in turn,
// interleaved on one box): verify 0.742 -> 0.731 ms, emit 0.942 (tile kernel) -> 0.896 ms.
//
// Variant 60 (the descriptor-batch verify before variant 63): each group of 8 lanes streams
// its own record on the record's 128-B line grid, U = 4 chunks per lane per step, after its header
// window (two load instructions for the wavefront's 8 records) has been parsed, so that every chunk
// is summed against the record's known span end.  64 VGPRs, 7 wavefronts per SIMD.  Measured
// against the walk kernel's variant 13 (16 x 4, tools/exp_r05_desc.py,
// profiles/r05_experiments/dwalk_layouts.jsonl): C3 verify 0.742 against 0.793 ms, gapped 0.742 /
// 0.798, shuffled 0.760 / 0.815, records of 64-1500 B 0.185 / 0.343 ms.
//
// Variant 56 (experiments build):
// a wavefront owns 8 consecutive descriptors, a group of 8 lanes per record for the parse and the
// gates.  When the 8 records lie back to back in memory (C3: packed records), the wavefront streams
// their whole span [first record's 128-B line, last record's end) with wave-contiguous loads: load
// instruction i covers bytes 1024 i .. 1024 i + 1023 of the span, one 16-B chunk per lane, U = 4
// instructions in flight.  A lane adds its chunk to accumulator j of every record j the
// instruction overlaps (a wave-uniform test against record j's precomputed instruction range),
// whole when the chunk lies inside the record's checksummed span, masked otherwise; a
// reduce-scatter over the wavefront then leaves record j's sum in group j (csum_xwalk.hip).  A
// wavefront whose records do not lie back to back streams them the walk kernel's way: each group
// its own record, 8 lanes x U chunks per step.  The headers come from a 256-B LDS window
// per record, loaded (two instructions for the 8 records) and parsed before the sums, whose masks
// need each record's span end.
#include "csum_walk.h"

namespace smolcsum {

namespace dwalk {

constexpr int R = 8;       // records per wavefront
constexpr int G = 8;       // lanes per record (parse, gates)
constexpr int WAVES = 4;
constexpr int GPB = WAVES * R;
constexpr int WIN_CH = 16;  // the LDS window: 256 B from the record's 128-B line
constexpr int U = 4;        // load instructions in flight per wavefront
constexpr uint32_t kStageMinBytes = 1024;  // STAGE: the wavefront's mean record length to stage at

}  // namespace dwalk

// GROUPS (variant 60): every wavefront streams its records the per-group way (the product's form).
// SEG (variant 61, emit): the 64-B segments that hold a record's fields go out whole from its LDS
// window, the fields patched in, as the walk kernel's variant 39 does for fixed strides (§5 of
// a whole segment is a plain write at the memory side, a 2-B store a read-modify-write).
// SEGF bit 0: whole segments (variant 61); bit 1: the header windows loaded with the default cache
// policy instead of non-temporal (62 = both, 63 = bit 1 alone); bit 2: the 2-B fields stored
// non-temporal (experiments: 18 = 63 + bit 2, 20 = 60's emit + bit 2); bit 3: the window's 16
// chunks summed from LDS, the stream starting at chunk 16 (41 = 63 + bit 3: the product's
// descriptor-batch emit since late round 5); bit 4: staged (variant 94 = 61 + bits 1, 3 and 4, round 6):
// a record whose fields the whole segments cover (bit 0's rule, all or nothing) writes nothing here and
// stages one 8-B entry (its two field offsets and values) in p.stage for the segment pass
// (seg_pass_desc_kernel); any other record stores its fields here as 2-B writes and stages ~0.
// tools/probe_wtax.hip: field writes that land while a read stream runs cost 65-90 ps each, the same
// segments loaded again and written in a pass of their own ~40 ps.
template <int MODE, bool NOSTORE, bool GROUPS = false, int SEGF = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((SEGF & 160) ? 8 : 1))) void dwalk_kernel(KParams p) {
    using namespace dwalk;
    constexpr bool EMIT = MODE == MODE_EMIT;
    __shared__ u32x4 win[GPB][WIN_CH];
    __shared__ uint32_t spanbuf[GPB];
    const int wl = (int)(threadIdx.x & 63);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = wl & (G - 1);
    const int gw = wl / G;
    const int gib = wv * R + gw;
    const uint64_t rw0 = (logical_block(p.xcd_remap) * WAVES + (uint64_t)wv) * R;
    if (rw0 >= p.n) return;
    const uint32_t cnt = (uint32_t)(p.n - rw0 < (uint64_t)R ? p.n - rw0 : (uint64_t)R);
    const uint64_t dummy = (uint64_t)p.dummy;

    // ---- descriptors: lane j holds record j's ----
    // (a fixed-stride batch, experiments build: the descriptors it implies)
    u32x4 d = u32x4{0, 0, 0, 0};
    if (p.desc) {
        if ((uint32_t)wl < cnt) d = *(gcv4)((uint64_t)p.desc + 16 * (rw0 + (uint64_t)wl));
    } else {
        const uint64_t off = (rw0 + (uint64_t)wl) * p.stride;
        d = u32x4{(uint32_t)off, (uint32_t)(off >> 32), (uint32_t)wl < cnt ? p.len : 0u, 0u};
    }
    constexpr bool LITE = (SEGF & 64) != 0 && MODE == MODE_EMIT;
    constexpr bool STAGE_ANY = (SEGF & 16) != 0 || LITE;
    bool stage_wave = false;
    // GAPS (bit 512, LITE, late round 6): a wavefront stages whatever its records' layout (gaps,
    // shuffled descriptors) when their mean length is >= kStageMinBytes; each record's segment may
    // start in the record before it only when that one (the batch's record r - 1) ends where it begins
    constexpr bool GAPS = (SEGF & 512) != 0 && (SEGF & 64) != 0 && MODE == MODE_EMIT;
    uint64_t cmask = ~0ull;  // GAPS: lane j set when record j - 1 of the wavefront ends where j begins (>= 64 B)
    if constexpr (STAGE_ANY) {
        // from the descriptors in lanes 0 .. cnt - 1 (not the uniform arrays: they would stay live
        // in SGPRs, 87 against 58, one wavefront per SIMD fewer): back to back, and their span
        const uint64_t off = (uint64_t)d.x | ((uint64_t)d.y << 32), end = off + d.z;
        const uint64_t pend = (uint64_t)(uint32_t)__shfl_up((int)(uint32_t)end, 1, 64) |
                              ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(end >> 32), 1, 64) << 32);
        const bool gap = (uint32_t)wl < cnt && wl != 0 && pend != off;
        const uint64_t first = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)d.x) |
                               ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)d.y) << 32);
        const uint64_t last = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)end, (int)cnt - 1) |
                              ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(end >> 32), (int)cnt - 1) << 32);
        if constexpr (GAPS) {
            uint32_t lz = (uint32_t)wl < cnt ? d.z : 0u;
#pragma unroll
            for (int m = 1; m < R; m <<= 1) lz += (uint32_t)__shfl_xor((int)lz, m, 64);
            const uint32_t plen = (uint32_t)__shfl_up((int)d.z, 1, 64);
            cmask = __ballot((uint32_t)wl < cnt && wl != 0 && pend == off && plen >= 64u);
            stage_wave = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)lz) >= (uint64_t)cnt * dwalk::kStageMinBytes;
        } else {
            stage_wave = __ballot(gap) == 0 && last - first >= (uint64_t)cnt * dwalk::kStageMinBytes;
        }
    }
    // LITE: the record before the wavefront's first one ends where it begins (the batch's record r - 1,
    // loaded with the descriptors), so that record 0's field segment may start in it (below)
    bool prev_contig = false;
    if constexpr (LITE && (SEGF & 256) != 0) {
        if (rw0 > 0) {
            uint64_t pend;
            if (p.desc) {
                const u32x4 pd = *(gcv4)((uint64_t)p.desc + 16 * (rw0 - 1));
                pend = pd.z >= 64 ? ((uint64_t)pd.x | ((uint64_t)pd.y << 32)) + pd.z : ~0ull;  // (>= 64 B: as ok_tail)
            } else {
                pend = p.len >= 64 ? (rw0 - 1) * p.stride + p.len : ~0ull;
            }
            const uint64_t off0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)d.x) |
                                  ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)d.y) << 32);
            prev_contig = __builtin_amdgcn_readfirstlane((int)(pend == off0)) != 0;
        }
    }
    // wave-uniform record extents
    uint64_t A[R];
    uint32_t L[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const uint64_t off = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)d.x, j) |
                             ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)d.y, j) << 32);
        A[j] = (uint64_t)p.buf + off;
        L[j] = (uint32_t)j < cnt ? (uint32_t)__builtin_amdgcn_readlane((int)d.z, j) : 0u;
    }
    bool contig = true;  // the records lie back to back (and their span stays below 2 GiB)
#pragma unroll
    for (int j = 1; j < R; ++j)
        if ((uint32_t)j < cnt) contig = contig && A[j] == A[j - 1] + L[j - 1];
    const uint64_t span_lo = A[0] & ~127ull;
    contig = contig && A[cnt - 1] + L[cnt - 1] - span_lo < (1ull << 31);

    // ---- the windows: instruction w, lane l: record 4 w + l / 16, chunk l % 16 ----
    constexpr bool SEG = (SEGF & 1) != 0 && MODE == MODE_EMIT;
    constexpr bool STAGE = (SEGF & 16) != 0 && SEG;
    // LITE (bit 6, variant 96): staged like STAGE, but the decision (just before the finish) keeps
    // only its outcome and the field values go to the entry from finish_gates' registers (no window
    // patch, no whole-segment addresses): variant 41's finish otherwise
    constexpr bool WNT = (SEGF & 2) == 0;
    const bool mine = (uint32_t)gw < cnt;
    const uint64_t r = rw0 + (uint64_t)gw;
    const uint64_t a0 = (uint64_t)p.buf + ((uint64_t)(uint32_t)__shfl((int)d.x, gw, 64) |
                                           ((uint64_t)(uint32_t)__shfl((int)d.y, gw, 64) << 32));
    const uint32_t len = (uint32_t)__shfl((int)d.z, gw, 64);
    const uint32_t kind = p.desc ? desc_kind((uint32_t)__shfl((int)d.w, gw, 64)) : p.kind;
    const uint32_t hd = (uint32_t)(a0 & 127u);
    {
        u32x4 wc[2];
#pragma unroll
        for (int w = 0; w < 2; ++w) {
            const int rec = 4 * w + wl / 16, c = wl % 16;
            const uint64_t ra = (uint64_t)p.buf + ((uint64_t)(uint32_t)__shfl((int)d.x, rec, 64) |
                                                   ((uint64_t)(uint32_t)__shfl((int)d.y, rec, 64) << 32));
            const uint32_t rl = (uint32_t)__shfl((int)d.z, rec, 64);
            const uint64_t rb = ra & ~127ull;
            const bool in = (uint32_t)rec < cnt && rb + 16ull * (uint32_t)c < ra + rl;
            wc[w] = ld16<WNT>((gcv4)(in ? rb + 16ull * (uint32_t)c : dummy));
        }
#pragma unroll
        for (int w = 0; w < 2; ++w) {
            const int rec = 4 * w + wl / 16;
            if ((uint32_t)rec < cnt) win[wv * R + rec][wl % 16] = wc[w];
        }
    }
    wave_lds_sync();
    const uint8_t* winb = reinterpret_cast<const uint8_t*>(&win[gib][0]);
    auto rd = [&](uint32_t o) -> uint32_t {
        const uint32_t x = hd + o;
        if (x < 16u * WIN_CH) return (uint32_t)winb[x];
        return ld_byte_sync(a0 + o);
    };
    Geom g = Geom{};
    if (mine) g = parse_geometry<false>(rd, len, kind, EMIT);
    const bool l4 = g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED);
    if (lane == 0) spanbuf[gib] = mine && l4 ? g.span_end : 0u;
    // SEG: which of the record's field segments go out whole.  A segment that starts before the
    // record also holds the previous record's last bytes: whole only when that record lies right
    // before this one in the same wavefront (contig) and has no field in its last 64 bytes (then it
    // is longer than 64 bytes, and no store of its group falls into the segment).  A record whose
    // fields end 64 bytes or more before its end keeps its segments inside itself; the window must
    // hold the whole segment.  The rest are stored as 2-B fields.
    uint64_t wsA = ~0ull, wsB = ~0ull;
    // STAGE: a wavefront stages its records only when they lie back to back and average at least
    // kStageMinBytes each (wave-uniform); otherwise it runs variant 41's finish, 2-B field stores.
    // Measured in bench.py's step order (tools/exp_r06_desc_step.py, profiles/r06_experiments/
    // desc_layouts_step_41_94.jsonl), staging every record: C3 packed step 1.598 -> 1.503 ms and
    // 500-3000-B records 0.703 -> 0.685, but 64-1500-B records 0.389 -> 0.467 and gapped / shuffled C3
    // +1 / +1.6 % (not back to back: few segments may go out whole)
    if constexpr (SEG) {
      if (!STAGE || stage_wave) {
        uint32_t f[3], flo = NO_FIELD, fhi = 0;
        emit_fields(g, f);
        for (int j = 0; j < 3; ++j)
            if (f[j] != NO_FIELD) {
                flo = f[j] < flo ? f[j] : flo;
                fhi = f[j] + 2 > fhi ? f[j] + 2 : fhi;
            }
        const bool ok_tail = mine && len >= 64 && (fhi == 0 || fhi + 64 <= len);  // (len: a segment that
        // starts before the next record then holds only bytes of this one)
        const uint64_t okm = __ballot(lane == 0 && ok_tail);
        if (mine && (g.fam == 4 || g.fam == 6) && fhi != 0 && ok_tail) {
            const bool prev_ok = contig && gw != 0 && ((okm >> (uint32_t)(G * (gw - 1))) & 1ull);
            const int32_t ph = (int32_t)(a0 & 63u);
            const int32_t rA = ((ph + (int32_t)flo) & ~63) - ph, rB = ((ph + (int32_t)fhi - 1) & ~63) - ph;
            const int32_t wend = 16 * WIN_CH - (int32_t)hd;
            auto whole = [&](int32_t rel) { return rB <= rA + 64 && rel + 64 <= wend && (rel >= 0 || prev_ok); };
            if (whole(rA)) wsA = a0 + (int64_t)rA;
            if (rB != rA && whole(rB)) wsB = a0 + (int64_t)rB;
        }
        if constexpr (STAGE) {  // all or nothing: staged when the segments cover every field byte
            auto cov = [&](uint32_t fo) {
                const uint64_t x0 = (a0 + fo) & ~63ull, x1 = (a0 + fo + 1) & ~63ull;
                return (x0 == wsA || x0 == wsB) && (x1 == wsA || x1 == wsB);
            };
            const bool staged = wsA != ~0ull && f[2] == NO_FIELD && (f[0] == NO_FIELD || cov(f[0])) &&
                                (f[1] == NO_FIELD || cov(f[1]));
            if (!staged) wsA = wsB = ~0ull;
        }
      }
    }
    wave_lds_sync();
    uint32_t S1[R];
#pragma unroll
    for (int j = 0; j < R; ++j) S1[j] = (uint32_t)__builtin_amdgcn_readfirstlane((int)spanbuf[wv * R + j]);

    uint32_t a1 = 0;  // this lane's part of its group's record sum
    if (contig && !GROUPS) {
        // ---- stream the span, summing each chunk into the records it overlaps ----
        uint32_t acc[R];
#pragma unroll
        for (int j = 0; j < R; ++j) acc[j] = 0;
        // span base (128-B line) and end, relative record bounds [lo_j, lo_j + S1_j)
        const uint64_t sb = span_lo, se = A[cnt - 1] + L[cnt - 1];
        const uint32_t bytes = (uint32_t)(se - sb);
        int32_t lo[R];
        int32_t ifst[R], ilst[R];  // the load instructions that overlap record j's sum (empty: 0, -1)
#pragma unroll
        for (int j = 0; j < R; ++j) {
            lo[j] = (int32_t)(A[j] - sb);
            ifst[j] = S1[j] > 0 ? lo[j] >> 10 : 0;
            ilst[j] = S1[j] > 0 ? (lo[j] + (int32_t)S1[j] - 1) >> 10 : -1;
        }
        const uint32_t whi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(sb >> 32));
        const uint32_t wlo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sb);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)whi << 32) | wlo), 0, 0x7fffffff, 0x00020000);
        const uint32_t ni = (bytes + 1023u) >> 10;
        // U loads in flight, then their sums (measured: two sets in turn were slower, 0.90 against
        // 0.835 ms for C3 verify: hipcc waits for every outstanding load at the loop head)
        for (uint32_t i0 = 0; i0 < ni; i0 += U) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t P = 1024u * (i0 + (uint32_t)u) + 16u * (uint32_t)wl;
                v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, P < bytes ? P : 0x80000000u, 0, 2 /* nt */);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int32_t ii = (int32_t)(i0 + (uint32_t)u);
                if (ii >= (int32_t)ni) break;
                const int pos0 = 1024 * ii + 16 * wl;
                const u32x4 c = v[u];
                const uint32_t whole = add_words(c.x, add_words(c.y, add_words(c.z, add_words(c.w, 0u))));
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    if (ii >= ifst[j] && ii <= ilst[j]) {  // wave-uniform
                        const int pos = pos0 - lo[j];  // the chunk's start relative to record j
                        uint32_t x = 0;
                        if (pos >= 0 && pos + 16 <= (int)S1[j]) x = whole;
                        else if (pos + 16 > 0 && pos < (int)S1[j]) x = sum_masked_words(c, -pos, (int)S1[j] - pos, 0u);
                        acc[j] += x;
                    }
                }
            }
        }
        // ---- reduce-scatter: record j's sum to group j ----
        uint32_t a4[4], a2[2];
        const bool up32 = (wl & 32) != 0, up16 = (wl & 16) != 0, up8 = (wl & 8) != 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            a4[i] = (up32 ? acc[i + 4] : acc[i]) + (uint32_t)__shfl_xor((int)(up32 ? acc[i] : acc[i + 4]), 32, 64);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            a2[i] = (up16 ? a4[i + 2] : a4[i]) + (uint32_t)__builtin_amdgcn_ds_swizzle((int)(up16 ? a4[i] : a4[i + 2]), 0x401F);
        a1 = (up8 ? a2[1] : a2[0]) +
             (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(up8 ? a2[0] : a2[1]), 0x128, 0xF, 0xF, false);
    } else {
        // ---- records not back to back: each group streams its own record on its line grid,
        //      8 lanes x U chunks per step (the walk kernel's layout) ----
        const int s1 = mine && l4 ? (int)g.span_end : 0;
        const uint64_t base = a0 & ~127ull;
        const uint32_t nch = (uint32_t)((int)hd + s1 + 15) >> 4;  // chunks up to the span's end
        uint32_t cstart = 0;
        if constexpr ((SEGF & 8) != 0) {  // the window's chunks from LDS, the stream from chunk 16
#pragma unroll
            for (int h = 0; h < WIN_CH / G; ++h) {
                const uint32_t c = (uint32_t)(G * h + lane);
                const int pos = 16 * (int)c - (int)hd;
                if (c < nch) {
                    const u32x4 x = win[gib][c];
                    if (pos >= 0 && pos + 16 <= s1) a1 = add_words(x.x, add_words(x.y, add_words(x.z, add_words(x.w, a1))));
                    else a1 = sum_masked_words(x, -pos, s1 - pos, a1);
                }
            }
            cstart = WIN_CH;
        }
        for (uint32_t c0 = cstart; c0 < nch; c0 += (uint32_t)(G * U)) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = c0 + (uint32_t)(G * u + lane);
                v[u] = ld16<true>((gcv4)(c < nch ? base + 16ull * c : dummy));
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = c0 + (uint32_t)(G * u + lane);
                const int pos = 16 * (int)c - (int)hd;
                if (c < nch) {
                    if (pos >= 0 && pos + 16 <= s1) a1 = add_words(v[u].x, add_words(v[u].y, add_words(v[u].z, add_words(v[u].w, a1))));
                    else a1 = sum_masked_words(v[u], -pos, s1 - pos, a1);
                }
            }
        }
    }
    bool lite_staged = false;
    if constexpr (LITE) {
        if (stage_wave) {
            // 61's whole-segment rule (below), all or nothing over the record's fields
            uint32_t f[3], flo = NO_FIELD, fhi = 0;
            emit_fields(g, f);
            for (int j = 0; j < 3; ++j)
                if (f[j] != NO_FIELD) {
                    flo = f[j] < flo ? f[j] : flo;
                    fhi = f[j] + 2 > fhi ? f[j] + 2 : fhi;
                }
            const bool ok_tail = mine && len >= 64 && (fhi == 0 || fhi + 64 <= len);  // (len: a segment that
            // starts before the next record then holds only bytes of this one)
            const uint64_t okm = __ballot(lane == 0 && ok_tail);
            if (mine && (g.fam == 4 || g.fam == 6) && fhi != 0 && ok_tail && f[2] == NO_FIELD) {
                // a segment that starts before the record holds only bytes of the record before it: in the
                // wavefront, that record passed ok_tail; for the wavefront's first record (late round 6) it
                // only has to end where this one begins, since a staged record's field segments end at
                // least 64 B before its end (ok_tail) and an unstaged one's 2-B fields are written in this
                // launch, before the segment pass loads the segment
                const bool prev_ok = gw != 0 ? (((okm >> (uint32_t)(G * (gw - 1))) & 1ull) != 0 && ((cmask >> gw) & 1ull) != 0)
                                             : prev_contig;
                const int32_t ph = (int32_t)(a0 & 63u);
                const int32_t rA = ((ph + (int32_t)flo) & ~63) - ph, rB = ((ph + (int32_t)fhi - 1) & ~63) - ph;
                const int32_t wend = 16 * WIN_CH - (int32_t)hd;
                auto whole = [&](int32_t rel) { return rel + 64 <= wend && (rel >= 0 || prev_ok); };
                lite_staged = rB <= rA + 64 && whole(rA) && (rB == rA || whole(rB));
            }
        }
    }
    // ---- finish: the walk kernel's gates ----
    if constexpr (LITE) {
        if (mine) finish_gates<G, MODE, false, decltype(rd), 0, false, NOSTORE, (SEGF & 1024) != 0, true>(p, g, a1, rd, winb, hd, a0, r, lane,
                                                                                            nullptr, ~0ull, ~0ull,
                                                                                            !stage_wave ? 0 : lite_staged ? 1 : 2);
        if (wl == 0) p.stage_flags[rw0 / R] = stage_wave ? 1u : 0u;
    } else if (STAGE && !stage_wave) {  // (wave-uniform) variant 41's finish, nothing staged
        if (mine) finish_gates<G, MODE, false, decltype(rd), 0, false, NOSTORE>(p, g, a1, rd, winb, hd, a0, r, lane);
        if (wl == 0) p.stage_flags[rw0 / R] = 0u;  // the segment pass skips these 8 records
    } else if constexpr (SEG) {
        uint8_t* winw = reinterpret_cast<uint8_t*>(&win[gib][0]);
        if (mine) finish_gates<G, MODE, false, decltype(rd), 16 * WIN_CH, true, NOSTORE>(p, g, a1, rd, winb, hd, a0, r, lane,
                                                                                          winw, wsA, wsB);
        wave_lds_sync();
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        const uint64_t base = a0 & ~127ull;
        auto seg_store = [&](uint64_t dst) {
            const u32x2 x = *reinterpret_cast<const u32x2*>(winb + (dst - base));
            if constexpr (NOSTORE) asm volatile("" ::"v"(x), "v"(dst));
            else *(GMEM u32x2*)dst = x;
        };
        if constexpr (STAGE) {
            if (mine && lane == 0) stage_record(p, r, wsA != ~0ull, g, winb, hd);
            if (wl == 0) p.stage_flags[rw0 / R] = 1u;
        } else {
            if (wsA != ~0ull && lane < 8) seg_store(wsA + 8u * (uint32_t)lane);
            if (wsB != ~0ull && lane < 8) seg_store(wsB + 8u * (uint32_t)lane);
        }
    } else {
        if (mine) finish_gates<G, MODE, false, decltype(rd), 0, false, NOSTORE, (SEGF & 4) != 0>(p, g, a1, rd, winb, hd, a0, r, lane);
    }
}

// The segment pass of the staged emit (variant 97, the product's descriptor-batch emit; 94-96 and
// 80 / 81 in the experiments build): 8 lanes per record; on a wavefront of 8 records whose flag the
// staging launch set, a record with a staged entry (not ~0) loads the 64-B segment(s) holding its
// fields (default cache policy), patches the field bytes in and stores each segment whole,
// write-through and non-temporal (sc0 sc1 nt; a plain or nt store after the default-policy load stays
// dirty on chip and is written back inside the next read stream: tools/probe_wtax.hip, 0.054 against
// 0.106 ms per C2 pass).  Records anywhere in the buffer: 64-bit addresses, so the store is written as
// the instruction (global_store_dwordx2 with its cache-policy bits: a vector store).  The segments are
// the staging launch's decision (its whole-segment rule), so no two groups write one segment and no
// other write touches them.  A wavefront's 8 records (the staging launch's wavefront of 8, or part of
// one) end at once when their flag says nothing was staged.
__device__ __forceinline__ uint64_t patch_field(uint64_t x, int64_t k, uint32_t v) {
    if (k >= 0 && k < 8) x = (x & ~(0xffull << (8 * k))) | ((uint64_t)((v >> 8) & 0xffu) << (8 * k));
    if (k + 1 >= 0 && k + 1 < 8) x = (x & ~(0xffull << (8 * (k + 1)))) | ((uint64_t)(v & 0xffu) << (8 * (k + 1)));
    return x;
}

#ifdef SMOL_EXP
// (experiments build, variant 105: the first form, 8 lanes x 8 B per record, 1024-thread workgroups)
__global__ __launch_bounds__(1024) void seg_pass_kernel(KParams p) {
    const uint64_t r = (uint64_t)blockIdx.x * 128 + (threadIdx.x >> 3);
    const int l = (int)(threadIdx.x & 7);
    if (r >= p.n) return;
    if (p.stage_flags[r / 8] == 0u) return;  // (uniform over the wavefront's 8 records) nothing staged
    const uint64_t e = __builtin_nontemporal_load((const GMEM uint64_t*)(p.stage + r));
    if (e == ~0ull) return;
    const uint64_t off = p.desc ? *(const GMEM uint64_t*)((uint64_t)p.desc + 16 * r) : r * p.stride;
    const uint32_t f0 = (uint32_t)(e & 0xffu), f1 = (uint32_t)((e >> 8) & 0xffu);
    const uint32_t v0 = (uint32_t)((e >> 32) & 0xffffu), v1 = (uint32_t)(e >> 48);
    const uint64_t a0 = (uint64_t)p.buf + off;
    const uint32_t lo = min(f0 == 0xffu ? 0xffffu : f0, f1 == 0xffu ? 0xffffu : f1);
    const uint32_t hi = max(f0 == 0xffu ? 0u : f0 + 2, f1 == 0xffu ? 0u : f1 + 2);
    const uint64_t sA = (a0 + lo) & ~63ull, sB = (a0 + hi - 1) & ~63ull;
    const uint64_t wA = sA + 8u * (uint32_t)l, wB = sB + 8u * (uint32_t)l;
    // both loads before either store (stores count in vmcnt with the loads, in order)
    uint64_t xa = *(const GMEM uint64_t*)wA;
    uint64_t xb = sB != sA ? *(const GMEM uint64_t*)wB : 0ull;
    if (f0 != 0xffu) xa = patch_field(xa, (int64_t)(a0 + f0) - (int64_t)wA, v0);
    if (f1 != 0xffu) xa = patch_field(xa, (int64_t)(a0 + f1) - (int64_t)wA, v1);
    asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1 nt" ::"v"(wA), "v"(xa) : "memory");
    if (sB != sA) {
        if (f0 != 0xffu) xb = patch_field(xb, (int64_t)(a0 + f0) - (int64_t)wB, v0);
        if (f1 != 0xffu) xb = patch_field(xb, (int64_t)(a0 + f1) - (int64_t)wB, v1);
        asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1 nt" ::"v"(wB), "v"(xb) : "memory");
    }
}
#endif

// 4 lanes per record, 16 B each (late round 6: one 16-B load and one 16-B store per lane and segment
// instead of two 8-B ones, 256-thread workgroups: C3 emit 0.791 -> 0.777 ms, interleaved bench lines,
// profiles/r06_experiments/seg_pass_16b_lanes.txt)
__global__ __launch_bounds__(256) void seg_pass4_kernel(KParams p) {
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    const uint64_t r = (uint64_t)blockIdx.x * 64 + (threadIdx.x >> 2);
    const int l = (int)(threadIdx.x & 3);
    if (r >= p.n) return;
    if (p.stage_flags[r / 8] == 0u) return;
    const uint64_t e = __builtin_nontemporal_load((const GMEM uint64_t*)(p.stage + r));
    if (e == ~0ull) return;
    const uint64_t off = p.desc ? *(const GMEM uint64_t*)((uint64_t)p.desc + 16 * r) : r * p.stride;
    const uint32_t f0 = (uint32_t)(e & 0xffu), f1 = (uint32_t)((e >> 8) & 0xffu);
    const uint32_t v0 = (uint32_t)((e >> 32) & 0xffffu), v1 = (uint32_t)(e >> 48);
    const uint64_t a0 = (uint64_t)p.buf + off;
    const uint32_t lo = min(f0 == 0xffu ? 0xffffu : f0, f1 == 0xffu ? 0xffffu : f1);
    const uint32_t hi = max(f0 == 0xffu ? 0u : f0 + 2, f1 == 0xffu ? 0u : f1 + 2);
    const uint64_t sA = (a0 + lo) & ~63ull, sB = (a0 + hi - 1) & ~63ull;
    const uint64_t wA = sA + 16u * (uint32_t)l, wB = sB + 16u * (uint32_t)l;
    u32x4v xa = *(const GMEM u32x4v*)wA;
    u32x4v xb = sB != sA ? *(const GMEM u32x4v*)wB : u32x4v{0, 0, 0, 0};
    auto patch = [&](u32x4v& x, uint64_t w) {
        uint64_t q0 = (uint64_t)x.x | ((uint64_t)x.y << 32), q1 = (uint64_t)x.z | ((uint64_t)x.w << 32);
        if (f0 != 0xffu) {
            q0 = patch_field(q0, (int64_t)(a0 + f0) - (int64_t)w, v0);
            q1 = patch_field(q1, (int64_t)(a0 + f0) - (int64_t)(w + 8), v0);
        }
        if (f1 != 0xffu) {
            q0 = patch_field(q0, (int64_t)(a0 + f1) - (int64_t)w, v1);
            q1 = patch_field(q1, (int64_t)(a0 + f1) - (int64_t)(w + 8), v1);
        }
        x = u32x4v{(uint32_t)q0, (uint32_t)(q0 >> 32), (uint32_t)q1, (uint32_t)(q1 >> 32)};
    };
    patch(xa, wA);
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(wA), "v"(xa) : "memory");
    if (sB != sA) {
        patch(xb, wB);
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(wB), "v"(xb) : "memory");
    }
}

hipError_t launch_seg_pass(const KParams& p, hipStream_t s, int form) {
#ifdef SMOL_EXP
    if (form == 1) {  // the first form: 1024-thread workgroups (128 records each)
        hipLaunchKernelGGL(seg_pass_kernel, dim3((uint32_t)((p.n + 127) / 128)), dim3(1024), 0, s, p);
        return hipGetLastError();
    }
#endif
    (void)form;
    hipLaunchKernelGGL(seg_pass4_kernel, dim3((uint32_t)((p.n + 63) / 64)), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_dwalk(int mode, int variant, const KParams& p, hipStream_t s) {
#ifndef SMOL_EXP
    // the product's forms: 63 (verify / emit), 41 (emit), 60 (verify)
    if (!(variant == 63 && (mode == MODE_VERIFY || mode == MODE_EMIT)) && !(variant == 60 && mode == MODE_VERIFY) &&
        !(variant == 41 && mode == MODE_EMIT) && !(variant == 94 && mode == MODE_EMIT) && !(variant == 95 && mode == MODE_EMIT) &&
        !(variant == 96 && mode == MODE_EMIT) && !(variant == 97 && mode == MODE_EMIT))
        return hipErrorInvalidValue;
#endif
    if ((variant == 94 || variant == 95 || variant == 96 || variant == 97 || (variant >= 103 && variant <= 105) || variant == 109) &&
        mode == MODE_EMIT) {  // staged: the staging launch, then the segment pass
        if (!p.stage || !p.stage_flags || p.n > kStageChunk) return hipErrorInvalidValue;
        note_launch(KERN_DWALK, (uint32_t)variant, dwalk::G, dwalk::U);
        const uint32_t b = grid_blocks((p.n + dwalk::GPB - 1) / dwalk::GPB, kMaxGridBlocks);
        if (variant == 96)  // held to 8 wavefronts per SIMD (12 B of spills per lane; 97: 7, none)
            hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 10 | 64 | 128>), dim3(b), dim3(256), 0, s, p);
        else if (variant == 97 || variant == 105)  // (bit 256, late round 6: the wavefront's first record may stage too; 105: the first segment-pass form)
            hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 10 | 64 | 256>), dim3(b), dim3(256), 0, s, p);
#ifdef SMOL_EXP
        else if (variant == 109)  // 97 + bit 1024 (experiments build): entries (and 2-B fields) stored write-through / nt
            hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 10 | 64 | 256 | 1024>), dim3(b), dim3(256), 0, s, p);
        else if (variant == 104)  // 97 + bit 512 (experiments build): staging over gapped / shuffled layouts
            hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 10 | 64 | 256 | 512>), dim3(b), dim3(256), 0, s, p);
        else if (variant == 103)  // 97 before bit 256 (experiments build)
            hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 10 | 64>), dim3(b), dim3(256), 0, s, p);
#endif
        else if (variant == 95)  // (experiments: held to 8 wavefronts per SIMD, 64 B of spills per lane)
            hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 27 | 32>), dim3(b), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 27>), dim3(b), dim3(256), 0, s, p);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        return launch_seg_pass(p, s, variant == 105 ? 1 : 0);
    }
    const uint64_t per = (uint64_t)dwalk::GPB;
    note_launch(KERN_DWALK, (uint32_t)variant, dwalk::G, dwalk::U);
    const uint64_t span = kMaxGridBlocks * per;
    for (uint64_t i0 = 0; i0 < p.n; i0 += span) {
        KParams q = p;
        q.n = p.n - i0 < span ? p.n - i0 : span;
        if (p.desc) q.desc = p.desc + i0;
        else q.buf = p.buf + i0 * p.stride;
        if (p.status) q.status = p.status + i0;
        const uint32_t b = grid_blocks((q.n + per - 1) / per, kMaxGridBlocks);
        if (variant == 63 && mode == MODE_VERIFY)
            hipLaunchKernelGGL((dwalk_kernel<MODE_VERIFY, false, true, 2>), dim3(b), dim3(256), 0, s, q);
        else if (variant == 63)
            hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 2>), dim3(b), dim3(256), 0, s, q);
        else if (variant == 41)
            hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 10>), dim3(b), dim3(256), 0, s, q);
        else if (variant == 60 && mode == MODE_VERIFY)
            hipLaunchKernelGGL((dwalk_kernel<MODE_VERIFY, false, true>), dim3(b), dim3(256), 0, s, q);
#ifdef SMOL_EXP
        else if (variant == 60) hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true>), dim3(b), dim3(256), 0, s, q);
        else if (variant == 18) hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 6>), dim3(b), dim3(256), 0, s, q);
        else if (variant == 20) hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 4>), dim3(b), dim3(256), 0, s, q);
        else if (variant == 61) hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 1>), dim3(b), dim3(256), 0, s, q);
        else if (variant == 62) hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false, true, 3>), dim3(b), dim3(256), 0, s, q);
        else if (variant == 64 + 61) hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, true, true, 1>), dim3(b), dim3(256), 0, s, q);
        else if (mode == MODE_VERIFY) hipLaunchKernelGGL((dwalk_kernel<MODE_VERIFY, false>), dim3(b), dim3(256), 0, s, q);
        else if (variant >= 64) hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, true>), dim3(b), dim3(256), 0, s, q);
        else hipLaunchKernelGGL((dwalk_kernel<MODE_EMIT, false>), dim3(b), dim3(256), 0, s, q);
#endif
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace smolcsum
