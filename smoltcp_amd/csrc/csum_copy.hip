// Fused payload copy + emit, second design (variant 17): the walk kernel's MODE_COPY split by chunk
// class, so that the bulk of a record costs what a copy costs.
//
// TcpRepr::emit / UdpRepr::emit copy the payload into the packet and then fill the checksum
// (src/wire/tcp.rs:1087-1095, src/wire/udp.rs:300-308).  The result here is bit-identical to a
// memcpy of every payload followed by smol_csum_batch_emit, as in MODE_COPY of csum_walk.h, whose
// helpers (rec_at, parse_geometry, finish_gates) this kernel shares.
//
// A group of G lanes owns a record.  Its 16-B destination chunks fall into two classes:
// * BODY chunks lie past the 128-B header window and entirely inside the copy range.  A lane reads
//   the 16 source bytes from the chunk's first source byte rounded down to 4 (one dwordx4 load) and
//   the dword after them (one dword load, not issued when no record of the wavefront needs it),
//   shifts them to the destination alignment with four v_alignbyte, sums them and stores them: no
//   destination load, no mask, no neighbour exchange.  That loop is unrolled U deep, all loads
//   issued first.
// * GENERIC chunks — the window (the first 128 B of the chunk grid, which hold the headers the gates
//   parse) and any chunk past it that holds bytes outside the copy range (normally just the
//   record's last chunk) — are built from the destination chunk and two aligned source chunks with
//   byte masks.  The window, the first few other generic chunks and the first UB * G body chunks are
//   loaded in ONE round before the parse, so a C2copy record takes one round trip for its headers,
//   tail and first body chunks, then one for the rest of its body.
// Every byte of the record is written (bytes outside the copy range with their own values, so no
// line is left half-written by this kernel); the window chunks go out last from LDS, with the
// fields finish_gates patched in.  A field past the window (behind a long IPv6 Hop-by-Hop header)
// is left out of the chunk stores and written by finish_gates.
#include "csum_walk.h"

namespace smolcsum {

namespace copy2 {

// Store the bytes [lo, hi) of chunk c (chunk-relative) at dst, leaving out any byte of the fields
// starting at chunk-relative f0 / f1 / f2 (2 bytes each).
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
            for (int j = 0; j < 4; ++j)
                if (keep & (0xffu << (8 * j))) dst[4 * i + j] = (uint8_t)(cw[i] >> (8 * j));
        }
    }
}

__device__ __forceinline__ uint32_t sum_chunk(const u32x4& c, int pos, int s1, uint32_t acc) {
    // aligned-word sum of the chunk's bytes inside the record span [0, s1) (pos: chunk start
    // relative to the record start)
    if (pos >= s1 || pos + 16 <= 0) return acc;
    if (pos < 0 || pos + 16 > s1) return sum_masked_words(c, -pos, s1 - pos, acc);
    return add_words(c.x, add_words(c.y, add_words(c.z, add_words(c.w, acc))));
}

constexpr int WIN = 128;  // the header window: 16-B grid, Grid<false>
constexpr int WIN_CH = WIN / 16;
constexpr int NOF = -(1 << 20);  // "no field" for store_part

}  // namespace copy2

// LBS (variant 21): the first body round's loads are issued right after the parse, before round 1's
// chunk stores, so that waiting for them does not also wait for those stores (gfx950 counts stores
// in vmcnt, in issue order with the loads).
// NTB (experiments build): bit 0 the body chunks stored non-temporal (variant 30), bit 1 also the
// body's source chunks loaded non-temporal (variant 22); bit 2 the destination chunks of the generic
// (header / edge) chunks loaded non-temporal (variant 98, round 6: whether the 28-B header reads
// then leave L2 as 64-B requests instead of whole 128-B lines; they do not); bit 3 the body chunks
// stored write-through non-temporal, sc1 nt (variant 102, round 6; cf. variant 30's plain nt).
template <int G, int U, bool IMPLICIT, int UW0 = 0, int UB = 0, bool LBS = false, int NTB = 0>
__global__ __launch_bounds__(256) void copy_kernel(KParams p) {
    using namespace copy2;
    constexpr int GPB = 256 / G;
    // slots per lane loaded before the parse (UW0, or enough for the window plus 8 chunks past it):
    // the window, then the generic chunks past it, then the first body chunks
    constexpr int UW = UW0 > 0 ? UW0 : (WIN_CH + 8 + G - 1) / G;
    constexpr uint32_t NEX = (uint32_t)(UW * G - WIN_CH);  // chunks past the window in that round
    static_assert(G >= 8 && G <= 64 && (G & (G - 1)) == 0, "group size");
    __shared__ u32x4 win[GPB][WIN_CH];
    __shared__ Geom geo[GPB];

    const int lane = (int)(threadIdx.x % G);
    const int gib = (int)(threadIdx.x / G);
    const uint64_t ngroups = (uint64_t)gridDim.x * GPB;
    u32x4* wn = &win[gib][0];
    const uint8_t* winb = reinterpret_cast<const uint8_t*>(wn);
    const uint64_t dummy = (uint64_t)p.dummy;

    for (uint64_t r = logical_block(p.xcd_remap) * GPB + gib; r < p.n; r += ngroups) {
        const RecRef rr = rec_at<IMPLICIT, true>(p, r);
        if (rr.kind & KIND_BAD_COPY) {  // the copy range does not fit: record left untouched
            if (lane == 0 && p.status) ((gu8)p.status)[r] = (uint8_t)SMOL_ST_MALFORMED;
            continue;
        }
        const uint64_t base = rr.a0 & ~15ull;
        const uint32_t head = (uint32_t)(rr.a0 - base);
        const uint32_t nch = n_chunks<false>(rr);
        const bool pay = rr.p1 > rr.p0;
        const uint64_t sk = rr.sb - head;  // source address of grid byte 0 (payload bytes only)
        const uint64_t first = (rr.sb + rr.p0) & ~15ull, last = (rr.sb + rr.p1 - 1) & ~15ull;
        // body chunks [kb0, kb1): past the window, entirely inside the copy range
        uint32_t kb0 = pay ? (head + rr.p0 + 15) >> 4 : nch;
        kb0 = kb0 > (uint32_t)WIN_CH ? kb0 : (uint32_t)WIN_CH;
        uint32_t kb1 = pay ? (head + rr.p1) >> 4 : 0u;
        kb1 = kb1 < nch ? kb1 : nch;
        kb1 = kb1 > kb0 ? kb1 : kb0;
        // generic chunks past the window: [WIN_CH, min(kb0, nch)) then [kb1, nch)
        const uint32_t e1 = kb0 < nch ? kb0 : nch;
        const uint32_t n1 = e1 > (uint32_t)WIN_CH ? e1 - WIN_CH : 0u;
        const uint32_t n2 = nch > kb1 ? nch - kb1 : 0u;
        const uint32_t ne = n1 + n2;
        auto gen_k = [&](uint32_t e) -> uint32_t { return e < n1 ? WIN_CH + e : kb1 + (e - n1); };
        const uint32_t nb = kb1 - kb0;
        // body chunks that ride in round 1's spare slots (built there the generic way)
        // (UB > 0: none; the first UB * G body chunks are loaded the body way in round 1 instead)
        const uint32_t body1 = UB == 0 && ne < NEX ? (nb < NEX - ne ? nb : NEX - ne) : 0u;
        const uint32_t nbe = UB > 0 ? (nb < (uint32_t)(UB * G) ? nb : (uint32_t)(UB * G)) : 0u;
        // chunk of round-1 slot e past the window: generic chunks, then body chunks
        auto ext_k = [&](uint32_t e) -> uint32_t { return e < ne ? gen_k(e) : kb0 + (e - ne); };

        // a generic chunk: the destination chunk (unless it is all payload) and the two aligned
        // source chunks under its payload bytes (clamped into the source range's aligned chunks:
        // bytes outside the range are masked anyway, and no load leaves the range)
        auto gen_load = [&](uint32_t k, bool in, u32x4& d, u32x4& c0, u32x4& c1) {
            const int pos = (int)(16u * k) - (int)head;
            const int lo = (int)rr.p0 - pos, hi = (int)rr.p1 - pos;
            const bool full = lo <= 0 && hi >= 16;
            const bool any = pay && lo < 16 && hi > 0;
            d = ld16<(NTB & 4) != 0>((gcv4)(in && !(pay && full) ? base + 16ull * k : dummy));
            const uint64_t sA = (sk + 16ull * k) & ~15ull;
            const uint64_t a0 = sA < first ? first : sA > last ? last : sA;
            const uint64_t a1 = sA + 16 < first ? first : sA + 16 > last ? last : sA + 16;
            c0 = ld16<false>((gcv4)(in && any ? a0 : dummy));
            c1 = ld16<false>((gcv4)(in && any && (sk & 15u) ? a1 : dummy));
        };
        auto gen_merge = [&](uint32_t k, const u32x4& d, const u32x4& c0, const u32x4& c1) -> u32x4 {
            const int pos = (int)(16u * k) - (int)head;
            const int lo = (int)rr.p0 - pos, hi = (int)rr.p1 - pos;
            if (!(pay && lo < 16 && hi > 0)) return d;
            const u32x4 s = funnel16(c0, c1, (uint32_t)(sk & 15u));
            if (lo <= 0 && hi >= 16) return s;
            u32x4 m;
            const uint32_t m0 = byte_mask(lo, hi, 0), m1 = byte_mask(lo, hi, 1);
            const uint32_t m2 = byte_mask(lo, hi, 2), m3 = byte_mask(lo, hi, 3);
            m.x = (s.x & m0) | (d.x & ~m0);
            m.y = (s.y & m1) | (d.y & ~m1);
            m.z = (s.z & m2) | (d.z & ~m2);
            m.w = (s.w & m3) | (d.w & ~m3);
            return m;
        };

        // body chunks: U per lane per round; their loads need only the copy range, not the parse
        const uint64_t skA = sk & ~3ull;
        const uint32_t b = (uint32_t)(sk & 3u);
        // the dword after a chunk's 16 source bytes holds its last b bytes; no lane of the wavefront
        // needs it when every record it holds has b == 0 (source and destination co-aligned mod 4,
        // as in C2copy), and then those loads are not issued at all
        const bool need_hi = __any(b != 0u);
        auto body_load1 = [&](uint32_t i, u32x4& lo, uint32_t& hi) {
            const bool in = i < nb;
            const uint64_t A = skA + 16ull * (kb0 + i);
            lo = ld16<(NTB & 2) != 0>((gcv4)(in ? A : dummy));
            hi = need_hi ? *(const GMEM uint32_t*)(in && b ? A + 16 : dummy) : 0u;
        };
        auto body_load = [&](uint32_t i0, u32x4* lo, uint32_t* hi) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t i = i0 + (uint32_t)(u * G + lane);
                const bool in = i < nb;
                const uint64_t A = skA + 16ull * (kb0 + i);
                lo[u] = ld16<(NTB & 2) != 0>((gcv4)(in ? A : dummy));
                // (b == 0: that dword may lie past the source range, so it is not read)
                hi[u] = need_hi ? *(const GMEM uint32_t*)(in && b ? A + 16 : dummy) : 0u;
            }
        };
        u32x4 blo[U];
        uint32_t bhi[U];
        u32x4 elo[UB > 0 ? UB : 1];
        uint32_t ehi[UB > 0 ? UB : 1];

        // ---- round 1: the window and the first generic chunks past it ----
        u32x4 gm[UW];
        {
            u32x4 d[UW], c0[UW], c1[UW];
#pragma unroll
            for (int u = 0; u < UW; ++u) {
                const uint32_t j = (uint32_t)(u * G + lane);
                const bool w = j < (uint32_t)WIN_CH;
                const uint32_t k = w ? j : ext_k(j - WIN_CH);
                const bool in = w ? j < nch : j - WIN_CH < ne + body1;
                gen_load(k, in, d[u], c0[u], c1[u]);
            }
            if constexpr (UB > 0) {
#pragma unroll
                for (int u = 0; u < UB; ++u) body_load1((uint32_t)(u * G + lane), elo[u], ehi[u]);
            }
#pragma unroll
            for (int u = 0; u < UW; ++u) {
                const uint32_t j = (uint32_t)(u * G + lane);
                const bool w = j < (uint32_t)WIN_CH;
                const uint32_t k = w ? j : ext_k(j - WIN_CH);
                gm[u] = gen_merge(k, d[u], c0[u], c1[u]);
                if (w && j < nch) wn[j] = gm[u];
            }
        }
        wave_lds_sync();
        // record byte o: the LDS window, else global memory (payload bytes from the source)
        auto rd = [&](uint32_t o) -> uint32_t {
            const uint32_t x = head + o;
            if (x < (uint32_t)WIN) return (uint32_t)winb[x];
            if (o >= rr.p0 && o < rr.p1) return ld_byte_sync(rr.sb + o);
            return ld_byte_sync(rr.a0 + o);
        };
        {
            const Geom g0 = parse_geometry<false>(rd, rr.len, rr.kind, true);
            if (lane == 0) geo[gib] = g0;
        }
        wave_lds_sync();
        const Geom& g = geo[gib];
        const bool l4 = g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED);
        const int s1 = l4 ? (int)g.span_end : 0;
        // fields past the window stay out of the chunk stores (finish_gates writes them)
        int f0b = NOF, f1b = NOF, f2b = NOF;
        {
            const uint32_t fip = g.fam == 4 ? g.ip_off + 10 : NO_FIELD;
            const uint32_t fl4 = l4 ? g.l4_off + g.fo : NO_FIELD;
            const uint32_t fin = g.in_off ? g.in_off + 10 : NO_FIELD;
            auto past = [&](uint32_t f) { return f != NO_FIELD && head + f + 2 > (uint32_t)WIN; };
            if (past(fip) || past(fl4) || past(fin)) {
                f0b = fip != NO_FIELD ? (int)fip : NOF;
                f1b = fl4 != NO_FIELD ? (int)fl4 : NOF;
                f2b = fin != NO_FIELD ? (int)fin : NOF;
            }
        }
        const bool far = f0b != NOF || f1b != NOF || f2b != NOF;
        const int len = (int)rr.len;
        if constexpr (LBS) body_load(UB > 0 ? nbe : body1, blo, bhi);

        // ---- sum round 1; store its chunks past the window ----
        uint32_t acc = 0;
#pragma unroll
        for (int u = 0; u < UW; ++u) {
            const uint32_t j = (uint32_t)(u * G + lane);
            const bool w = j < (uint32_t)WIN_CH;
            const uint32_t k = w ? j : ext_k(j - WIN_CH);
            const bool in = w ? j < nch : j - WIN_CH < ne + body1;
            if (in) {
                const int pos = (int)(16u * k) - (int)head;
                acc = sum_chunk(gm[u], pos, s1, acc);
                if (!w) store_part((gu8)base + 16u * k, gm[u], -pos, len - pos, f0b - pos, f1b - pos, f2b - pos);
            }
        }
        // generic chunks beyond round 1 (a copy range that starts or ends far from the record's edges)
        for (uint32_t e0 = NEX; e0 < ne; e0 += G) {
            const uint32_t e = e0 + (uint32_t)lane;
            const bool in = e < ne;
            const uint32_t k = gen_k(in ? e : 0u);
            u32x4 d, c0, c1;
            gen_load(k, in, d, c0, c1);
            const u32x4 m = gen_merge(k, d, c0, c1);
            if (in) {
                const int pos = (int)(16u * k) - (int)head;
                acc = sum_chunk(m, pos, s1, acc);
                store_part((gu8)base + 16u * k, m, -pos, len - pos, f0b - pos, f1b - pos, f2b - pos);
            }
        }

        // ---- body: copy + sum ----
        auto body_proc = [&](uint32_t i, const u32x4& lo, uint32_t hi) {
            const uint32_t k = kb0 + i;
            u32x4 m;
            m.x = __builtin_amdgcn_alignbyte(lo.y, lo.x, b);
            m.y = __builtin_amdgcn_alignbyte(lo.z, lo.y, b);
            m.z = __builtin_amdgcn_alignbyte(lo.w, lo.z, b);
            m.w = __builtin_amdgcn_alignbyte(hi, lo.w, b);
            const int pos = (int)(16u * k) - (int)head;
            acc = sum_chunk(m, pos, s1, acc);
            const gu8 dst = (gu8)base + 16u * k;
            if (!far) {
                if constexpr ((NTB & 8) != 0)  // (variant 102) write-through non-temporal vector store
                    asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(dst), "v"(m) : "memory");
                else if constexpr ((NTB & 1) != 0) __builtin_nontemporal_store(m, (GMEM u32x4*)dst);
                else *(GMEM u32x4*)dst = m;
            } else store_part(dst, m, 0, 16, f0b - pos, f1b - pos, f2b - pos);
        };
        if constexpr (UB > 0) {
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                const uint32_t i = (uint32_t)(u * G + lane);
                if (i < nbe) body_proc(i, elo[u], ehi[u]);
            }
        }
        for (uint32_t i0 = UB > 0 ? nbe : body1; i0 < nb; i0 += (uint32_t)(G * U)) {
            if (!LBS || i0 != (UB > 0 ? nbe : body1)) body_load(i0, blo, bhi);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t i = i0 + (uint32_t)(u * G + lane);
                if (i < nb) body_proc(i, blo[u], bhi[u]);
            }
        }

        // ---- finish: gates, fields into the window (or past it), then the window chunks ----
        finish_gates<G, MODE_COPY, false, decltype(rd), WIN>(p, g, acc, rd, winb, head, rr.a0, r, lane,
                                                              reinterpret_cast<uint8_t*>(wn));
        wave_lds_sync();
        for (uint32_t k = (uint32_t)lane; k < (uint32_t)WIN_CH && k < nch; k += G) {
            const int pos = (int)(16u * k) - (int)head;
            store_part((gu8)base + 16u * k, wn[k], -pos, len - pos, NOF, NOF, NOF);
        }
        wave_lds_sync();  // the window is rewritten by the group's next record
    }
}

template <bool IMPLICIT, int G, int U, int UW = 0, int UB = 0, bool LBS = false, int NTB = 0>
hipError_t launch_copy2_one(const KParams& p, uint32_t max_blocks, hipStream_t s) {
    constexpr uint32_t GPB = 256 / G;
    const uint64_t want = (p.n + GPB - 1) / GPB;
    const uint32_t blocks = grid_blocks(want, max_blocks);
    note_launch(KERN_COPY, NTB == 1 ? 30 : NTB == 3 ? 22 : NTB == 4 ? 98 : NTB == 8 ? 102 : LBS ? 21 : 17, G, U);
    hipLaunchKernelGGL((copy_kernel<G, U, IMPLICIT, UW, UB, LBS, NTB>), dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

// Shapes (lanes per record x body chunks per lane per round [x generic round-1 slots per lane
// [x body round-1 slots per lane]]).  The default, 16 x 4 x 1 x 2, takes a C2copy record in two
// rounds: the window, its last chunk and 32 body chunks (loaded the body way), then the other 53.
// Measured on one MI355X (tools/exp_copy.py, profiles/r02b_experiments/): 16 x 4 x 1 x 2 0.689 ms,
// 16 x 5 x 1 x 1 0.691, 16 x 4 x 2 (body chunks in generic slots) 0.710, 16 x 3 0.743; earlier, before
// the hi-dword loads were skipped: 16 x 4 x 2 0.738, 16 x 3 0.760, 8 x 4 x 4 0.790, 8 x 6 0.837,
// 32 x 2 1.03, 64 x 2 1.73 (variant 16: 0.772).  Per-record work (parse, gates, window stores) is
// issued once per wavefront for its 64 / G records, so wide groups pay it for fewer records,
// narrow ones need more rounds.
template <bool IMPLICIT>
hipError_t launch_copy2(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    switch (shape) {
        case CFG_G8U6: return launch_copy2_one<IMPLICIT, 8, 6>(p, max_blocks, s);
        case CFG_G8U7: return launch_copy2_one<IMPLICIT, 8, 4, 4>(p, max_blocks, s);
        case CFG_G16U3: return launch_copy2_one<IMPLICIT, 16, 3>(p, max_blocks, s);
        case CFG_G16U6: return launch_copy2_one<IMPLICIT, 16, 5, 1, 1>(p, max_blocks, s);
        case CFG_G32U3: return launch_copy2_one<IMPLICIT, 16, 4, 2>(p, max_blocks, s);
        case CFG_G32U4: return launch_copy2_one<IMPLICIT, 32, 2, 1>(p, max_blocks, s);
        case CFG_G64U2:
        case CFG_G64U4: return launch_copy2_one<IMPLICIT, 64, 2>(p, max_blocks, s);
        default: return launch_copy2_one<IMPLICIT, 16, 4, 1, 2>(p, max_blocks, s);  // CFG_G16U4
    }
}

hipError_t launch_copy_v17(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    return p.desc == nullptr ? launch_copy2<true>(shape, p, max_blocks, s) : launch_copy2<false>(shape, p, max_blocks, s);
}

// variant 21 (the copy-emit default): variant 17's default shapes with the first body round's loads
// ahead of round 1's stores.  MI355X, C2copy, interleaved rounds on one box (tools/exp_copy.py,
// profiles/r04_experiments/copy_emit_lbs.jsonl): 16 x 4 x 1 x 2 0.678 ms against variant 17's 0.692;
// 16 x 5 x 1 x 1 0.711; also measured and not kept: 16 x 3 x 1 x 3 0.690, 16 x 3 x 1 x 2 0.728.
hipError_t launch_copy_v21(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    const bool im = p.desc == nullptr;
    if (shape == CFG_G16U6)
        return im ? launch_copy2_one<true, 16, 5, 1, 1, true>(p, max_blocks, s)
                  : launch_copy2_one<false, 16, 5, 1, 1, true>(p, max_blocks, s);
    return im ? launch_copy2_one<true, 16, 4, 1, 2, true>(p, max_blocks, s)
              : launch_copy2_one<false, 16, 4, 1, 2, true>(p, max_blocks, s);
}

#ifdef SMOL_EXP
// variants 30 / 22 (experiments build): variant 21 at 16 x 4 with non-temporal body stores / and
// non-temporal body source loads.
hipError_t launch_copy_nt(int var, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    const bool im = p.desc == nullptr;
    if (var == 30)
        return im ? launch_copy2_one<true, 16, 4, 1, 2, true, 1>(p, max_blocks, s)
                  : launch_copy2_one<false, 16, 4, 1, 2, true, 1>(p, max_blocks, s);
    if (var == 98)
        return im ? launch_copy2_one<true, 16, 4, 1, 2, true, 4>(p, max_blocks, s)
                  : launch_copy2_one<false, 16, 4, 1, 2, true, 4>(p, max_blocks, s);
    if (var == 102)
        return im ? launch_copy2_one<true, 16, 4, 1, 2, true, 8>(p, max_blocks, s)
                  : launch_copy2_one<false, 16, 4, 1, 2, true, 8>(p, max_blocks, s);
    return im ? launch_copy2_one<true, 16, 4, 1, 2, true, 3>(p, max_blocks, s)
              : launch_copy2_one<false, 16, 4, 1, 2, true, 3>(p, max_blocks, s);
}
#endif

}  // namespace smolcsum
