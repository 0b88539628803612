// Fused payload copy + emit on the transposed walk's load layout (variant 49, experiments build):
// fixed-stride batches of 1024 .. 1921-byte records.  Same result as copy_kernel (csum_copy.hip):
// bit-identical to a memcpy of every payload followed by smol_csum_batch_emit.
//
// A wavefront owns 8 consecutive records, a group of 8 lanes each for the parse and the gates
// (csum_xwalk.hip's layout).  On the record's 16-B chunk grid:
// * the WINDOW (chunks 0 .. 7, the headers) is built by group j, lane i taking chunk i of record j:
//   the destination chunk and the two aligned source chunks under its payload bytes, merged with
//   byte masks, into LDS;
// * BODY chunks (8 .. nch - 2) are all payload: load instruction (s, j) covers 64 of record j's body
//   chunks, one per lane, each one dwordx4 from the chunk's first source byte rounded down to 4
//   (plus the dword after it when the source and destination 4-byte phases differ: a wave-uniform
//   test per record), shifted by a per-record constant with v_alignbyte, summed and stored whole;
// * the EDGE chunk (nch - 1, the record's last bytes and the next record's first ones) is built by
//   lane 0 of the group from two aligned source chunks and stored byte-masked.
// That layout needs every record of the wavefront to have its payload run from inside the window to
// the record's end (TCP / UDP payloads: dst_offset + len == record length, dst_offset + the
// record's 16-B phase <= 128).  A wavefront holding any other record (or a copy range that does not
// fit) takes the generic path: group j builds every chunk of record j the window's way.
// Aligned 16-B source chunks are loaded only when they overlap the payload, and a dwordx4 from a
// 4-byte-aligned address only when all of its chunk's 16 bytes are payload, so no load touches a
// page that holds none of the source range.
#include "csum_walk.h"

namespace smolcsum {

#ifdef SMOL_EXP

namespace xcopy {

constexpr int R = 8;        // records per wavefront
constexpr int G = 8;        // lanes per record (parse, gates)
constexpr int NS = 2;       // body load instructions per record (64 chunks each)
constexpr int WAVES = 4;
constexpr int GPB = WAVES * R;
constexpr int WIN = 128;    // the header window on the 16-B grid
constexpr int WIN_CH = WIN / 16;
constexpr int NOF = -(1 << 20);

// Store the bytes [lo, hi) of chunk c (chunk-relative), leaving out the 2-byte fields at f0 / f1 / f2.
__device__ __forceinline__ void store_part(gu8 dst, const u32x4& c, int lo, int hi, int f0, int f1, int f2) {
    const bool field = (f0 > -2 && f0 < 16) || (f1 > -2 && f1 < 16) || (f2 > -2 && f2 < 16);
    if (lo <= 0 && hi >= 16 && !field) {
        *(GMEM u32x4*)dst = c;
        return;
    }
    const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
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
            for (int b = 0; b < 4; ++b)
                if (keep & (0xffu << (8 * b))) dst[4 * i + b] = (uint8_t)(cw[i] >> (8 * b));
        }
    }
}

// Aligned-word sum of the chunk's bytes inside [0, s1) (pos: chunk start relative to the record).
__device__ __forceinline__ uint32_t sum_chunk(const u32x4& c, int pos, int s1, uint32_t acc) {
    if (pos >= s1 || pos + 16 <= 0) return acc;
    if (pos < 0 || pos + 16 > s1) return sum_masked_words(c, -pos, s1 - pos, acc);
    return add_words(c.x, add_words(c.y, add_words(c.z, add_words(c.w, acc))));
}

// One record's copy geometry (wave-uniform values for the fast layout).
struct Rec {
    uint64_t a0, base, sb;  // record start, its 16-B grid origin, source address of record offset 0
    uint32_t head, nch, p0, p1;
    bool bad;
};

// Chunk k of a record built the generic way: the destination chunk (unless all payload) and the two
// aligned source chunks under its payload bytes (clamped into the source range's aligned chunks).
struct Gen {
    u32x4 d, c0, c1;
};
__device__ __forceinline__ Gen gen_load(const Rec& q, uint32_t k, bool in, uint64_t dummy) {
    const int pos = (int)(16u * k) - (int)q.head;
    const int lo = (int)q.p0 - pos, hi = (int)q.p1 - pos;
    const bool pay = q.p1 > q.p0;
    const bool full = lo <= 0 && hi >= 16;
    const bool any = pay && lo < 16 && hi > 0;
    const uint64_t sk = q.sb - q.head;
    const uint64_t first = (q.sb + q.p0) & ~15ull, last = (q.sb + q.p1 - 1) & ~15ull;
    const uint64_t sA = (sk + 16ull * k) & ~15ull;
    const uint64_t a0 = sA < first ? first : sA > last ? last : sA;
    const uint64_t a1 = sA + 16 < first ? first : sA + 16 > last ? last : sA + 16;
    Gen g;
    g.d = ld16<false>((gcv4)(in && !(pay && full) ? q.base + 16ull * k : dummy));
    g.c0 = ld16<false>((gcv4)(in && any ? a0 : dummy));
    g.c1 = ld16<false>((gcv4)(in && any && (sk & 15u) ? a1 : dummy));
    return g;
}
__device__ __forceinline__ u32x4 gen_merge(const Rec& q, uint32_t k, const Gen& g) {
    const int pos = (int)(16u * k) - (int)q.head;
    const int lo = (int)q.p0 - pos, hi = (int)q.p1 - pos;
    if (!(q.p1 > q.p0 && lo < 16 && hi > 0)) return g.d;
    const u32x4 s = funnel16(g.c0, g.c1, (uint32_t)((q.sb - q.head) & 15u));
    if (lo <= 0 && hi >= 16) return s;
    u32x4 m;
    const uint32_t m0 = byte_mask(lo, hi, 0), m1 = byte_mask(lo, hi, 1);
    const uint32_t m2 = byte_mask(lo, hi, 2), m3 = byte_mask(lo, hi, 3);
    m.x = (s.x & m0) | (g.d.x & ~m0);
    m.y = (s.y & m1) | (g.d.y & ~m1);
    m.z = (s.z & m2) | (g.d.z & ~m2);
    m.w = (s.w & m3) | (g.d.w & ~m3);
    return m;
}

}  // namespace xcopy

// PERSIST (variant 50): a grid of the resident workgroups whose wavefronts step over the batch 8 records
// at a time, loading the next step's copy descriptors ahead, so that a step waits for one round
// trip (its loads) instead of two (the descriptors, then the loads that need them).
// EXPT (variants 51-53, timing only, wrong bytes): 1 source loads rounded down to 16 B instead of
// 4; 2 no body stores; 4 the C2copy descriptors computed, not loaded (src_offset 1472 r, dst 28).
// 8 (variant 54, exact): non-temporal body stores.  16 (variant 55, exact): the body chunks re-dealt
// through LDS and stored walk-shaped, each store instruction covering 128 B of each of the 8 records.
template <bool PERSIST, int EXPT = 0>
__global__ __launch_bounds__(256) void xcopy_kernel(KParams p) {
    using namespace xcopy;
    __shared__ u32x4 win[GPB][WIN_CH];
    __shared__ uint32_t spanbuf[GPB];
    __shared__ u32x4 stg[(EXPT & 16) ? WAVES : 1][(EXPT & 16) ? R : 1][64];  // EXPT 16: one half-step's body chunks
    const int wl = (int)(threadIdx.x & 63);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = wl & (G - 1);
    const int gw = wl / G;
    const int gib = wv * R + gw;
    const uint64_t dummy = (uint64_t)p.dummy;
    const uint32_t len = p.len;
    const uint64_t nwaves = PERSIST ? (uint64_t)gridDim.x * WAVES : 0;
    uint64_t tw = logical_block(p.xcd_remap) * WAVES + (uint64_t)wv;
    // the copy descriptors of step tw (lane j: record j)
    auto load_dsc = [&](uint64_t t) -> u32x4 {
        const uint64_t r0 = t * R;
        const uint32_t c = (uint32_t)(p.n - r0 < (uint64_t)R ? p.n - r0 : (uint64_t)R);
        return (uint32_t)wl < c ? *(gcv4)((uint64_t)p.copy + 16 * (r0 + (uint64_t)wl)) : u32x4{0, 0, 0, 0};
    };
    if (tw * R >= p.n) return;
    u32x4 dsc_next = load_dsc(tw);
    for (; tw * R < p.n; tw += nwaves) {
    const u32x4 dsc = dsc_next;
    if (PERSIST && (tw + nwaves) * R < p.n) dsc_next = load_dsc(tw + nwaves);
    const uint64_t rw0 = tw * R;
    const uint32_t cnt = (uint32_t)(p.n - rw0 < (uint64_t)R ? p.n - rw0 : (uint64_t)R);
    const bool mine = (uint32_t)gw < cnt;
    const uint64_t r = rw0 + (uint64_t)gw;
    Rec q;  // the group's own record (per-lane values, equal within the group)
    q.a0 = (uint64_t)p.buf + r * p.stride;
    q.base = q.a0 & ~15ull;
    q.head = (uint32_t)(q.a0 - q.base);
    q.nch = (uint32_t)(((q.a0 + len + 15) >> 4) - (q.base >> 4));
    // this group's descriptor from lane gw
    {
        const uint32_t cx = (uint32_t)__shfl((int)dsc.x, gw, 64), cy = (uint32_t)__shfl((int)dsc.y, gw, 64);
        const uint32_t cz = (uint32_t)__shfl((int)dsc.z, gw, 64), cw = (uint32_t)__shfl((int)dsc.w, gw, 64);
        q.bad = (uint64_t)cz + cw > len;
        q.p0 = q.bad ? 0u : cz;
        q.p1 = q.bad ? 0u : cz + cw;
        q.sb = q.bad ? 0ull : (uint64_t)p.src + ((uint64_t)cx | ((uint64_t)cy << 32)) - cz;
        if (EXPT & 4) {
            q.bad = false;
            q.p0 = 28;
            q.p1 = len;
            q.sb = (uint64_t)p.src + 1472ull * r - 28;
        }
    }
    const bool fast_rec = !mine || (!q.bad && q.p1 > q.p0 && q.p1 == len && q.head + q.p0 <= (uint32_t)WIN);
    const bool fast = __all(fast_rec);

    if (fast) {
        // ---- window sources (group j, lane i: chunk i) and the edge chunk's (lane 0) ----
        const Gen gwin = gen_load(q, (uint32_t)lane, mine, dummy);
        const uint32_t kedge = q.nch - 1;
        const Gen gedge = gen_load(q, kedge, mine && lane == 0, dummy);
        // ---- body: record j's chunks 8 .. nch - 2, chunk 64 s + wl of instruction (s, j) ----
        u32x4 v[NS][R];
        uint32_t vh[NS][R];
        uint32_t bsh[R], hd[R], nb[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint64_t a0 = (uint64_t)p.buf + (rw0 + (uint64_t)j) * p.stride;
            const uint32_t h = (uint32_t)(a0 & 15u);
            const uint32_t nc = (uint32_t)(((a0 + len + 15) >> 4) - (a0 >> 4));
            // source of grid byte 0: sb_j - head_j (sb_j from lane j's descriptor)
            uint64_t so = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dsc.x, j) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dsc.y, j) << 32);
            uint32_t dz = (uint32_t)__builtin_amdgcn_readlane((int)dsc.z, j);
            if (EXPT & 4) {
                so = 1472ull * (rw0 + (uint64_t)j);
                dz = 28;
            }
            const uint64_t sk = (uint64_t)p.src + so - dz - h;
            const uint64_t skA = (EXPT & 1) ? (sk & ~15ull) : (sk & ~3ull);
            bsh[j] = (uint32_t)(sk & 3u);
            hd[j] = h;
            nb[j] = (uint32_t)j < cnt ? nc - 1 : 0u;  // body chunks are [8, nb)
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const uint32_t k = (uint32_t)(64 * s + wl);
                const bool in = k >= (uint32_t)WIN_CH && k < nb[j];
                const uint64_t A = skA + 16ull * k;
                v[s][j] = ld16<false>((gcv4)(in ? A : dummy));
                vh[s][j] = 0;
                if (bsh[j] != 0) vh[s][j] = *(const GMEM uint32_t*)(in ? A + 16 : dummy);
            }
        }
        // ---- the window into LDS, the parse ----
        const u32x4 wm = gen_merge(q, (uint32_t)lane, gwin);
        if (mine) win[gib][lane] = wm;
        wave_lds_sync();
        const uint8_t* winb = reinterpret_cast<const uint8_t*>(&win[gib][0]);
        auto rd = [&](uint32_t o) -> uint32_t {
            const uint32_t x = q.head + o;
            if (x < (uint32_t)WIN) return (uint32_t)winb[x];
            if (o >= q.p0 && o < q.p1) return ld_byte_sync(q.sb + o);
            return ld_byte_sync(q.a0 + o);
        };
        Geom g = Geom{};
        if (mine) g = parse_geometry<false>(rd, len, p.kind, true);
        const bool l4 = g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED);
        const int s1 = mine && l4 ? (int)g.span_end : 0;
        // fields past the window stay out of the chunk stores (finish_gates writes them)
        int f0b = NOF, f1b = NOF, f2b = NOF;
        {
            const uint32_t fip = g.fam == 4 ? g.ip_off + 10 : NO_FIELD;
            const uint32_t fl4 = l4 ? g.l4_off + g.fo : NO_FIELD;
            const uint32_t fin = g.in_off ? g.in_off + 10 : NO_FIELD;
            auto past = [&](uint32_t f) { return f != NO_FIELD && q.head + f + 2 > (uint32_t)WIN; };
            if (mine && (past(fip) || past(fl4) || past(fin))) {
                f0b = fip != NO_FIELD ? (int)fip : NOF;
                f1b = fl4 != NO_FIELD ? (int)fl4 : NOF;
                f2b = fin != NO_FIELD ? (int)fin : NOF;
            }
        }
        if (lane == 0) spanbuf[gib] = (uint32_t)s1;
        // far fields of record j, for the body stores (rare: behind a long Hop-by-Hop header)
        const bool any_far = __any(f0b != NOF || f1b != NOF || f2b != NOF);
        wave_lds_sync();
        // ---- body: shift, sum, store ----
        uint32_t acc[R];
        if constexpr ((EXPT & 16) != 0) {
#pragma unroll
            for (int j = 0; j < R; ++j) acc[j] = 0;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    const int sj = (int)spanbuf[wv * R + j], hj = (int)hd[j];
                    const uint32_t k = (uint32_t)(64 * s + wl);
                    const bool in = k >= (uint32_t)WIN_CH && k < nb[j];
                    const u32x4 lo = v[s][j];
                    const uint32_t b = bsh[j];
                    u32x4 m;
                    m.x = __builtin_amdgcn_alignbyte(lo.y, lo.x, b);
                    m.y = __builtin_amdgcn_alignbyte(lo.z, lo.y, b);
                    m.z = __builtin_amdgcn_alignbyte(lo.w, lo.z, b);
                    m.w = __builtin_amdgcn_alignbyte(vh[s][j], lo.w, b);
                    if (in) acc[j] = sum_chunk(m, 16 * (int)k - hj, sj, acc[j]);
                    stg[wv][j][wl] = m;
                }
                wave_lds_sync();
                // lane l stores chunks 64 s + 8 i + (l % 8) of its group's record (l / 8)
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint32_t kk = (uint32_t)(8 * i + lane), k = (uint32_t)(64 * s) + kk;
                    if (mine && k >= (uint32_t)WIN_CH && k < q.nch - 1) {
                        const u32x4 m = stg[wv][gw][kk];
                        const gu8 dst = (gu8)q.base + 16u * k;
                        const int pos = 16 * (int)k - (int)q.head;
                        if (!any_far) *(GMEM u32x4*)dst = m;
                        else store_part(dst, m, 0, 16, f0b - pos, f1b - pos, f2b - pos);
                    }
                }
                wave_lds_sync();  // the staging is rewritten by the next half-step
            }
        } else
#pragma unroll
        for (int j = 0; j < R; ++j) {
            acc[j] = 0;
            const int sj = (int)spanbuf[wv * R + j], hj = (int)hd[j];
            const uint64_t base = ((uint64_t)p.buf + (rw0 + (uint64_t)j) * p.stride) & ~15ull;
            int F0 = NOF, F1 = NOF, F2 = NOF;
            if (any_far) {  // record j's far fields, from its group's lane 0
                F0 = __shfl(f0b, G * j, 64);
                F1 = __shfl(f1b, G * j, 64);
                F2 = __shfl(f2b, G * j, 64);
            }
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const uint32_t k = (uint32_t)(64 * s + wl);
                const bool in = k >= (uint32_t)WIN_CH && k < nb[j];
                const u32x4 lo = v[s][j];
                const uint32_t b = bsh[j];
                u32x4 m;
                m.x = __builtin_amdgcn_alignbyte(lo.y, lo.x, b);
                m.y = __builtin_amdgcn_alignbyte(lo.z, lo.y, b);
                m.z = __builtin_amdgcn_alignbyte(lo.w, lo.z, b);
                m.w = __builtin_amdgcn_alignbyte(vh[s][j], lo.w, b);
                const int pos = 16 * (int)k - hj;
                if (in) {
                    acc[j] = sum_chunk(m, pos, sj, acc[j]);
                    const gu8 dst = (gu8)base + 16u * k;
                    if (EXPT & 2) asm volatile("" ::"v"(m.x), "v"(m.y), "v"(m.z), "v"(m.w));
                    else if ((EXPT & 8) && !any_far) __builtin_nontemporal_store(m, (GMEM u32x4*)dst);
                    else if (!any_far) *(GMEM u32x4*)dst = m;
                    else store_part(dst, m, 0, 16, F0 - pos, F1 - pos, F2 - pos);
                }
            }
        }
        // ---- reduce-scatter of the body sums, plus the group's window and edge chunks ----
        uint32_t own = 0;
        if (mine) {
            const int posw = 16 * lane - (int)q.head;
            own = sum_chunk(wm, posw, s1, 0u);
            if (lane == 0) {
                const u32x4 em = gen_merge(q, kedge, gedge);
                const int pose = 16 * (int)kedge - (int)q.head;
                own = sum_chunk(em, pose, s1, own);
                store_part((gu8)q.base + 16u * kedge, em, -pose, (int)len - pose, f0b - pose, f1b - pose,
                           f2b - pose);
            }
        }
        // (reduce_scatter of csum_xwalk.hip, inlined: 32, 16, 8)
        uint32_t a4[4], a2[2];
        const bool up32 = (wl & 32) != 0, up16 = (wl & 16) != 0, up8 = (wl & 8) != 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            a4[i] = (up32 ? acc[i + 4] : acc[i]) + (uint32_t)__shfl_xor((int)(up32 ? acc[i] : acc[i + 4]), 32, 64);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            a2[i] = (up16 ? a4[i + 2] : a4[i]) +
                    (uint32_t)__builtin_amdgcn_ds_swizzle((int)(up16 ? a4[i] : a4[i + 2]), 0x401F);
        const uint32_t a1 = (up8 ? a2[1] : a2[0]) +
                            (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(up8 ? a2[0] : a2[1]), 0x128, 0xF, 0xF, false);
        // ---- finish: gates, fields into the window (or past it), then the window chunks ----
        if (mine) {
            finish_gates<G, MODE_COPY, false, decltype(rd), WIN>(p, g, a1 + own, rd, winb, q.head, q.a0, r, lane,
                                                                  reinterpret_cast<uint8_t*>(&win[gib][0]));
        }
        wave_lds_sync();
        if (mine) {
            const int posw = 16 * lane - (int)q.head;
            store_part((gu8)q.base + 16u * (uint32_t)lane, win[gib][lane], -posw, (int)len - posw, NOF, NOF, NOF);
        }
    } else if (mine && q.bad) {  // the copy range does not fit: record left untouched
        if (lane == 0 && p.status) ((gu8)p.status)[r] = (uint8_t)SMOL_ST_MALFORMED;
    } else if (mine) {
    // ---- generic path: group j builds every chunk of record j the window's way ----
    {
        const Gen gw0 = gen_load(q, (uint32_t)lane, lane < (int)q.nch, dummy);
        const u32x4 wm = gen_merge(q, (uint32_t)lane, gw0);
        if ((uint32_t)lane < q.nch) win[gib][lane] = wm;
    }
    wave_lds_sync();
    const uint8_t* winb = reinterpret_cast<const uint8_t*>(&win[gib][0]);
    auto rd = [&](uint32_t o) -> uint32_t {
        const uint32_t x = q.head + o;
        if (x < (uint32_t)WIN) return (uint32_t)winb[x];
        if (o >= q.p0 && o < q.p1) return ld_byte_sync(q.sb + o);
        return ld_byte_sync(q.a0 + o);
    };
    const Geom g = parse_geometry<false>(rd, len, p.kind, true);
    const bool l4 = g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED);
    const int s1 = l4 ? (int)g.span_end : 0;
    int f0b = NOF, f1b = NOF, f2b = NOF;
    {
        const uint32_t fip = g.fam == 4 ? g.ip_off + 10 : NO_FIELD;
        const uint32_t fl4 = l4 ? g.l4_off + g.fo : NO_FIELD;
        const uint32_t fin = g.in_off ? g.in_off + 10 : NO_FIELD;
        auto past = [&](uint32_t f) { return f != NO_FIELD && q.head + f + 2 > (uint32_t)WIN; };
        if (past(fip) || past(fl4) || past(fin)) {
            f0b = fip != NO_FIELD ? (int)fip : NOF;
            f1b = fl4 != NO_FIELD ? (int)fl4 : NOF;
            f2b = fin != NO_FIELD ? (int)fin : NOF;
        }
    }
    uint32_t acc = 0;
    if ((uint32_t)lane < q.nch) acc = sum_chunk(win[gib][lane], 16 * lane - (int)q.head, s1, 0u);
    for (uint32_t k0 = WIN_CH; k0 < q.nch; k0 += G) {
        const uint32_t k = k0 + (uint32_t)lane;
        const bool in = k < q.nch;
        const Gen gk = gen_load(q, in ? k : 0u, in, dummy);
        const u32x4 m = gen_merge(q, k, gk);
        if (in) {
            const int pos = (int)(16u * k) - (int)q.head;
            acc = sum_chunk(m, pos, s1, acc);
            store_part((gu8)q.base + 16u * k, m, -pos, (int)len - pos, f0b - pos, f1b - pos, f2b - pos);
        }
    }
    finish_gates<G, MODE_COPY, false, decltype(rd), WIN>(p, g, acc, rd, winb, q.head, q.a0, r, lane,
                                                          reinterpret_cast<uint8_t*>(&win[gib][0]));
    wave_lds_sync();
    if ((uint32_t)lane < q.nch) {
        const int posw = 16 * lane - (int)q.head;
        store_part((gu8)q.base + 16u * (uint32_t)lane, win[gib][lane], -posw, (int)len - posw, NOF, NOF, NOF);
    }
    }
    if (!PERSIST) break;
    wave_lds_sync();  // the windows are rewritten by the next step
    }
}

#endif  // SMOL_EXP

bool xcopy_fits(const KParams& p) {
#ifdef SMOL_EXP
    return p.desc == nullptr && p.stride >= p.len && p.len >= 1024 && p.len <= 1921 && p.stride <= (1ull << 26);
#else
    return false;
#endif
}

hipError_t launch_xcopy(int variant, const KParams& p, hipStream_t s) {
#ifdef SMOL_EXP
    const uint64_t per = (uint64_t)xcopy::GPB;
    note_launch(KERN_COPY, (uint32_t)variant, 8, 2);
    if (variant == 50) {  // persistent: the workgroups resident at once
        const uint32_t cap = resident_blocks((const void*)xcopy_kernel<true>, p.num_cu ? p.num_cu : 256u,
                                             (uint32_t)kMaxGridBlocks);
        const uint32_t b = grid_blocks((p.n + per - 1) / per, cap);
        hipLaunchKernelGGL((xcopy_kernel<true>), dim3(b), dim3(256), 0, s, p);
        return hipGetLastError();
    }
    const uint64_t span = kMaxGridBlocks * per;
    for (uint64_t i0 = 0; i0 < p.n; i0 += span) {
        KParams q = p;
        q.n = p.n - i0 < span ? p.n - i0 : span;
        q.buf = p.buf + i0 * p.stride;
        q.copy = p.copy + i0;
        if (p.status) q.status = p.status + i0;
        const uint32_t b = grid_blocks((q.n + per - 1) / per, kMaxGridBlocks);
        if (variant == 51) hipLaunchKernelGGL((xcopy_kernel<false, 1>), dim3(b), dim3(256), 0, s, q);
        else if (variant == 52) hipLaunchKernelGGL((xcopy_kernel<false, 2>), dim3(b), dim3(256), 0, s, q);
        else if (variant == 53) hipLaunchKernelGGL((xcopy_kernel<false, 4>), dim3(b), dim3(256), 0, s, q);
        else if (variant == 54) hipLaunchKernelGGL((xcopy_kernel<false, 8>), dim3(b), dim3(256), 0, s, q);
        else if (variant == 55) hipLaunchKernelGGL((xcopy_kernel<false, 16>), dim3(b), dim3(256), 0, s, q);
        else hipLaunchKernelGGL((xcopy_kernel<false>), dim3(b), dim3(256), 0, s, q);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
#else
    return hipErrorInvalidValue;
#endif
}

}  // namespace smolcsum
