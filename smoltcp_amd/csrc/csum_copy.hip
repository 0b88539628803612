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

template <int G, int U, bool IMPLICIT, int UW0 = 0, int UB = 0>
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

    for (uint64_t r = (uint64_t)blockIdx.x * GPB + gib; r < p.n; r += ngroups) {
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
            d = ld16<false>((gcv4)(in && !(pay && full) ? base + 16ull * k : dummy));
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
            lo = ld16<false>((gcv4)(in ? A : dummy));
            hi = need_hi ? *(const GMEM uint32_t*)(in && b ? A + 16 : dummy) : 0u;
        };
        auto body_load = [&](uint32_t i0, u32x4* lo, uint32_t* hi) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t i = i0 + (uint32_t)(u * G + lane);
                const bool in = i < nb;
                const uint64_t A = skA + 16ull * (kb0 + i);
                lo[u] = ld16<false>((gcv4)(in ? A : dummy));
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
            if (!far) *(GMEM u32x4*)dst = m;
            else store_part(dst, m, 0, 16, f0b - pos, f1b - pos, f2b - pos);
        };
        if constexpr (UB > 0) {
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                const uint32_t i = (uint32_t)(u * G + lane);
                if (i < nbe) body_proc(i, elo[u], ehi[u]);
            }
        }
        for (uint32_t i0 = UB > 0 ? nbe : body1; i0 < nb; i0 += (uint32_t)(G * U)) {
            body_load(i0, blo, bhi);
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

// ---------------------------------------------------------------------------------------------
// Copy-emit, third design (variant 20): the tile split of csum_tile.hip applied to copy_kernel.
//
// A wavefront owns a TILE of T consecutive records and works on it in four phases:
//   A  lane i reads record i's descriptor and copy descriptor into LDS;
//   B  each group of G lanes copies and sums its records one after the other, exactly as
//      copy_kernel does (round 1: the 128-B window, the generic chunks past it and the first UB * G
//      body chunks; then body rounds of U * G chunks), but without any parse: it sums the record's
//      whole buffer [0, len), stores every chunk past the window, and leaves the window (with the
//      payload merged in) in the record's LDS row;
//   C  lane i parses record i from its row, takes the bytes outside the L4 span back out of the
//      sum, applies the gates and patches the fields into the row (a field past the window goes
//      to global memory after the wave's chunk stores have completed);
//   D  the groups store the window chunks from the rows.
// Parse and gates run once per lane for 64 records per instruction, instead of redundantly on the
// G lanes of each record's group (copy_kernel: ~12 % of its time).
// ---------------------------------------------------------------------------------------------
namespace ctile {

constexpr int WROW = 33;  // dwords per window row: 128 B + 4 (odd: phase C's lane-per-row reads
                          // hit distinct banks)

template <int T>
struct Lds {
    uint32_t win[T * WROW];
    uint32_t sum[T];
    uint32_t info[T * 8];  // a0 lo / hi, len, kind (| KIND_BAD_COPY), sb lo / hi, p0, p1
};

__device__ __forceinline__ uint32_t rbyte(const uint32_t* row, uint32_t x) {
    return (row[x >> 2] >> (8 * (x & 3))) & 0xffu;
}

// Aligned-word contribution of window bytes [from, to), to <= WIN.
__device__ __forceinline__ uint32_t row_sum(const uint32_t* row, uint32_t from, uint32_t to) {
    uint32_t acc = 0;
    for (uint32_t d = from >> 2; d < ((to + 3) >> 2); ++d) {
        const int lo = (int)from - (int)(4 * d), hi = (int)to - (int)(4 * d);
        acc = add_words(mask_dword(row[d], lo, hi), acc);
    }
    return acc;
}

}  // namespace ctile

template <int G, int U, bool IMPLICIT, int UB, int T>
__global__ __launch_bounds__(256) void copy_tile_kernel(KParams p) {
    using namespace copy2;
    using namespace ctile;
    constexpr int GPW = 64 / G;
    constexpr int UW = 1;                                   // round-1 generic slots per lane
    constexpr uint32_t NEX = (uint32_t)(UW * G - WIN_CH);  // of which past the window
    static_assert(G == 16 || G == 32, "group size");
    static_assert(T % GPW == 0 && T <= 64, "tile");
    __shared__ Lds<T> lds[4];
    const int wave = (int)(threadIdx.x >> 6);
    const int lane = (int)(threadIdx.x & 63);
    const int gl = lane % G;
    const int grp = lane / G;
    Lds<T>& L = lds[wave];
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    const uint64_t dummy = (uint64_t)p.dummy;

    for (uint64_t tile = (uint64_t)blockIdx.x * 4 + wave; tile * T < p.n; tile += nwaves) {
        const uint64_t r0 = tile * T;
        const uint32_t cnt = (uint32_t)((p.n - r0) < (uint64_t)T ? (p.n - r0) : (uint64_t)T);

        // ---- phase A: lane i's record and copy range ----
        if (lane < T) {
            const uint64_t r = r0 + ((uint32_t)lane < cnt ? (uint32_t)lane : 0u);
            const RecRef rr = rec_at<IMPLICIT, true>(p, r);
            uint32_t* in = &L.info[8 * lane];
            in[0] = (uint32_t)rr.a0;
            in[1] = (uint32_t)(rr.a0 >> 32);
            in[2] = (uint32_t)lane < cnt ? rr.len : 0u;
            in[3] = rr.kind;
            in[4] = (uint32_t)rr.sb;
            in[5] = (uint32_t)(rr.sb >> 32);
            in[6] = rr.p0;
            in[7] = rr.p1;
        }
        wave_lds_sync();
        auto rec = [&](int q) -> RecRef {
            const uint32_t* in = &L.info[8 * q];
            RecRef rr;
            rr.a0 = (uint64_t)in[0] | ((uint64_t)in[1] << 32);
            rr.len = in[2];
            rr.kind = in[3];
            rr.sb = (uint64_t)in[4] | ((uint64_t)in[5] << 32);
            rr.p0 = in[6];
            rr.p1 = in[7];
            return rr;
        };

        // ---- phase B: copy + sum, each group over its records ----
        for (int j = 0; j < T / GPW; ++j) {
            const int q = j * GPW + grp;
            const RecRef rr = rec(q);
            if (rr.len == 0 || (rr.kind & KIND_BAD_COPY)) {  // past the batch / left untouched
                if (gl == 0) L.sum[q] = 0;
                continue;
            }
            uint32_t* row = &L.win[q * WROW];
            const uint64_t base = rr.a0 & ~15ull;
            const uint32_t head = (uint32_t)(rr.a0 - base);
            const uint32_t nch = n_chunks<false>(rr);
            const bool pay = rr.p1 > rr.p0;
            const uint64_t sk = rr.sb - head;
            const uint64_t first = (rr.sb + rr.p0) & ~15ull, last = (rr.sb + rr.p1 - 1) & ~15ull;
            uint32_t kb0 = pay ? (head + rr.p0 + 15) >> 4 : nch;
            kb0 = kb0 > (uint32_t)WIN_CH ? kb0 : (uint32_t)WIN_CH;
            uint32_t kb1 = pay ? (head + rr.p1) >> 4 : 0u;
            kb1 = kb1 < nch ? kb1 : nch;
            kb1 = kb1 > kb0 ? kb1 : kb0;
            const uint32_t e1 = kb0 < nch ? kb0 : nch;
            const uint32_t n1 = e1 > (uint32_t)WIN_CH ? e1 - WIN_CH : 0u;
            const uint32_t n2 = nch > kb1 ? nch - kb1 : 0u;
            const uint32_t ne = n1 + n2;
            auto gen_k = [&](uint32_t e) -> uint32_t { return e < n1 ? WIN_CH + e : kb1 + (e - n1); };
            const uint32_t nb = kb1 - kb0;
            const uint32_t nbe = nb < (uint32_t)(UB * G) ? nb : (uint32_t)(UB * G);
            auto gen_load = [&](uint32_t k, bool in, u32x4& d, u32x4& c0, u32x4& c1) {
                const int pos = (int)(16u * k) - (int)head;
                const int lo = (int)rr.p0 - pos, hi = (int)rr.p1 - pos;
                const bool full = lo <= 0 && hi >= 16;
                const bool any = pay && lo < 16 && hi > 0;
                d = ld16<false>((gcv4)(in && !(pay && full) ? base + 16ull * k : dummy));
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
            const uint64_t skA = sk & ~3ull;
            const uint32_t b = (uint32_t)(sk & 3u);
            const bool need_hi = __any(b != 0u);
            const int len = (int)rr.len;
            uint32_t acc = 0;
            // round 1: the window, the first generic chunks past it, the first body chunks
            u32x4 elo[UB];
            uint32_t ehi[UB];
            {
                u32x4 d, c0, c1;
                const uint32_t jj = (uint32_t)gl;
                const bool w = jj < (uint32_t)WIN_CH;
                const uint32_t k = w ? jj : gen_k(jj - WIN_CH);
                const bool in = w ? jj < nch : jj - WIN_CH < ne;
                gen_load(k, in, d, c0, c1);
#pragma unroll
                for (int u = 0; u < UB; ++u) {
                    const uint32_t i = (uint32_t)(u * G + gl);
                    const uint64_t A = skA + 16ull * (kb0 + i);
                    elo[u] = ld16<false>((gcv4)(i < nb ? A : dummy));
                    ehi[u] = need_hi ? *(const GMEM uint32_t*)(i < nb && b ? A + 16 : dummy) : 0u;
                }
                const u32x4 m = gen_merge(k, d, c0, c1);
                if (in) {
                    const int pos = (int)(16u * k) - (int)head;
                    acc = sum_chunk(m, pos, len, acc);
                    if (w) {
                        row[4 * k] = m.x;
                        row[4 * k + 1] = m.y;
                        row[4 * k + 2] = m.z;
                        row[4 * k + 3] = m.w;
                    } else {
                        store_part((gu8)base + 16u * k, m, -pos, len - pos, NOF, NOF, NOF);
                    }
                }
            }
            // generic chunks beyond round 1
            for (uint32_t e0 = NEX; e0 < ne; e0 += G) {
                const uint32_t e = e0 + (uint32_t)gl;
                const bool in = e < ne;
                const uint32_t k = gen_k(in ? e : 0u);
                u32x4 d, c0, c1;
                gen_load(k, in, d, c0, c1);
                const u32x4 m = gen_merge(k, d, c0, c1);
                if (in) {
                    const int pos = (int)(16u * k) - (int)head;
                    acc = sum_chunk(m, pos, len, acc);
                    store_part((gu8)base + 16u * k, m, -pos, len - pos, NOF, NOF, NOF);
                }
            }
            // body: copy + sum
            auto body_proc = [&](uint32_t i, const u32x4& lo, uint32_t hi) {
                const uint32_t k = kb0 + i;
                u32x4 m;
                m.x = __builtin_amdgcn_alignbyte(lo.y, lo.x, b);
                m.y = __builtin_amdgcn_alignbyte(lo.z, lo.y, b);
                m.z = __builtin_amdgcn_alignbyte(lo.w, lo.z, b);
                m.w = __builtin_amdgcn_alignbyte(hi, lo.w, b);
                const int pos = (int)(16u * k) - (int)head;
                acc = sum_chunk(m, pos, len, acc);
                *(GMEM u32x4*)((gu8)base + 16u * k) = m;
            };
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                const uint32_t i = (uint32_t)(u * G + gl);
                if (i < nbe) body_proc(i, elo[u], ehi[u]);
            }
            for (uint32_t i0 = nbe; i0 < nb; i0 += (uint32_t)(G * U)) {
                u32x4 blo[U];
                uint32_t bhi[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t i = i0 + (uint32_t)(u * G + gl);
                    const uint64_t A = skA + 16ull * (kb0 + i);
                    blo[u] = ld16<false>((gcv4)(i < nb ? A : dummy));
                    bhi[u] = need_hi ? *(const GMEM uint32_t*)(i < nb && b ? A + 16 : dummy) : 0u;
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t i = i0 + (uint32_t)(u * G + gl);
                    if (i < nb) body_proc(i, blo[u], bhi[u]);
                }
            }
            const uint32_t tot = group_sum<G>(acc);
            if (gl == 0) L.sum[q] = tot;
        }
        wave_lds_sync();

        // ---- phase C: lane i finishes record i ----
        bool far = false;
        uint32_t far_a = 0, far_b = 0, far_c = 0;  // record offsets of fields past the window (+1; 0: none)
        uint32_t far_va = 0, far_vb = 0, far_vc = 0;
        if ((uint32_t)lane < cnt) {
            const RecRef rr = rec(lane);
            const uint64_t r = r0 + lane;
            if (rr.kind & KIND_BAD_COPY) {
                if (p.status) ((gu8)p.status)[r] = (uint8_t)SMOL_ST_MALFORMED;
            } else {
                uint32_t* row = &L.win[lane * WROW];
                uint8_t* rowb = reinterpret_cast<uint8_t*>(row);
                const uint32_t head = (uint32_t)(rr.a0 & 15u);
                const uint32_t nch = n_chunks<false>(rr);
                const uint32_t wvalid = nch * 16 < (uint32_t)WIN ? nch * 16 : (uint32_t)WIN;
                const bool odd = (rr.a0 & 1u) != 0;
                // record byte o (o < len): the row, else global memory (payload bytes from the source;
                // the others are unchanged by this kernel, fields included until phase C writes them)
                auto rd = [&](uint32_t o) -> uint32_t {
                    const uint32_t x = head + o;
                    if (x < wvalid) return rbyte(row, x);
                    if (o >= rr.p0 && o < rr.p1) return ld_byte_sync(rr.sb + o);
                    return ld_byte_sync(rr.a0 + o);
                };
                auto rsum = [&](uint32_t from, uint32_t to) -> uint32_t {  // record offsets
                    if (head + to <= wvalid) return row_sum(row, head + from, head + to);
                    uint32_t a = 0;
                    for (uint32_t o = from; o < to; ++o) a += rd(o) << (8 * ((head + o) & 1));
                    return a;
                };
                const Geom g = parse_geometry<false>(rd, rr.len, rr.kind, true);
                const bool l4 = g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED);
                uint32_t fip = MF_NONE, fl4 = MF_NONE, fin = MF_NONE, vip = 0, vl4 = 0, vin = 0;
                auto word = [&](uint32_t v) { return odd ? v : bswap16(v); };  // BE u16 at an even offset
                if (g.fam == 4) {
                    const uint32_t f0 = rd(g.ip_off + 10), f1 = rd(g.ip_off + 11);
                    const uint32_t sh = rsum(g.ip_off, g.ip_off + g.ip_hl) - (odd ? ((f0 << 8) + f1) : (f0 + (f1 << 8)));
                    const uint32_t f = fold32(sh);
                    const uint32_t hdr = odd ? f : bswap16(f);  // == checksum::data(header)
                    fip = g.ip_off + 10;
                    vip = caps_tx(p.caps_ipv4) ? (~hdr & 0xffffu) : 0u;
                }
                if (l4) {
                    const uint32_t fpos = g.l4_off + g.fo;
                    const uint32_t field = (rd(fpos) << 8) | rd(fpos + 1);
                    uint32_t s = L.sum[lane] - rsum(0, g.l4_off);
                    if (g.span_end < rr.len) s -= rsum(g.span_end, rr.len);
                    s -= word(field);
                    if (g.in_off) {  // ICMPv4 error: the embedded IPv4 header first
                        uint32_t hin = 0;
                        for (uint32_t i = 0; i < g.in_hl / 2; ++i)
                            if (i != 5) hin += (rd(g.in_off + 2 * i) << 8) | rd(g.in_off + 2 * i + 1);
                        fin = g.in_off + 10;
                        vin = caps_tx(p.caps_ipv4) ? (~fold32(hin) & 0xffffu) : 0u;
                        s = s - word((rd(fin) << 8) | rd(fin + 1)) + word(vin);
                    }
                    const uint32_t f = fold32(s);
                    const uint32_t dat = odd ? f : bswap16(f);  // == checksum::data(span)
                    const bool pseudo = g.proto == P_UDP || g.proto == P_TCP || g.proto == P_ICMP6;
                    uint32_t ph = 0;
                    if (pseudo) {
                        const uint32_t xa = fold32(rsum(g.addr_off, g.addr_off + 2 * g.addr_words));
                        const uint32_t addr = odd ? xa : bswap16(xa);
                        const uint32_t plen = g.proto == P_UDP ? (g.span_end - g.l4_off) : g.l4_len;
                        ph = fold32(addr + g.proto + (plen & 0xffffu));  // pseudo_header()
                    }
                    const uint32_t comb = pseudo ? fold32(ph + dat) : dat;  // combine()
                    uint32_t gate_caps;
                    switch (g.proto) {
                        case P_UDP: gate_caps = p.caps_udp; break;
                        case P_TCP: gate_caps = p.caps_tcp; break;
                        case P_ICMP4: gate_caps = p.caps_icmpv4; break;
                        case P_ICMP6: gate_caps = p.caps_icmpv6; break;
                        default: gate_caps = SMOL_CHECKSUM_NONE; break;  // IGMP
                    }
                    const bool fill = g.proto == P_IGMP ? true : caps_tx(gate_caps);
                    uint32_t c = ~comb & 0xffffu;
                    if (g.proto == P_UDP && c == 0) c = 0xffffu;  // udp.rs:207
                    fl4 = fpos;
                    vl4 = fill ? c : 0u;
                }
                // the fields into the row (phase D stores it), or past it: after the chunk stores
                // (a field across the window's edge: both, so that phase D's store of the window
                // chunk writes the new byte too)
                auto put = [&](uint32_t f, uint32_t v, uint32_t& fa, uint32_t& va) {
                    if (f == MF_NONE) return;
                    if (head + f < wvalid) rowb[head + f] = (uint8_t)(v >> 8);
                    if (head + f + 1 < wvalid) rowb[head + f + 1] = (uint8_t)v;
                    if (head + f + 2 > wvalid) {
                        far = true;
                        fa = f + 1;
                        va = v;
                    }
                };
                put(fip, vip, far_a, far_va);
                put(fin, vin, far_c, far_vc);
                put(fl4, vl4, far_b, far_vb);
                if (p.status) ((gu8)p.status)[r] = (uint8_t)g.st;
            }
        }
        if (__any(far)) {
            // a field past the window lies in a chunk a group stored in phase B (with its old
            // value): every store of the wave completes first, then the field goes out
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (far) {
                const uint64_t a0 = (uint64_t)L.info[8 * lane] | ((uint64_t)L.info[8 * lane + 1] << 32);
                if (far_a) store_be16((gu8)(a0 + far_a - 1), far_va);
                if (far_c) store_be16((gu8)(a0 + far_c - 1), far_vc);
                if (far_b) store_be16((gu8)(a0 + far_b - 1), far_vb);
            }
        }
        wave_lds_sync();

        // ---- phase D: the window chunks, fields patched in ----
        for (int j = 0; j < T / GPW; ++j) {
            const int q = j * GPW + grp;
            const RecRef rr = rec(q);
            if (rr.len == 0 || (rr.kind & KIND_BAD_COPY)) continue;
            const uint32_t* row = &L.win[q * WROW];
            const uint64_t base = rr.a0 & ~15ull;
            const uint32_t head = (uint32_t)(rr.a0 - base);
            const uint32_t nch = n_chunks<false>(rr);
            const uint32_t k = (uint32_t)gl;
            if (k < (uint32_t)WIN_CH && k < nch) {
                u32x4 c;
                c.x = row[4 * k];
                c.y = row[4 * k + 1];
                c.z = row[4 * k + 2];
                c.w = row[4 * k + 3];
                const int pos = (int)(16u * k) - (int)head;
                store_part((gu8)base + 16u * k, c, -pos, (int)rr.len - pos, NOF, NOF, NOF);
            }
        }
        wave_lds_sync();  // the rows are rewritten by the next tile
    }
}

template <bool IMPLICIT, int G, int U, int UB, int T>
hipError_t launch_copy_tile_one(const KParams& p, uint32_t max_blocks, hipStream_t s) {
    const uint64_t tiles = (p.n + T - 1) / T;
    const uint64_t want = (tiles + 3) / 4;
    const uint64_t cap = p.num_cu == 0 ? max_blocks : (uint64_t)0x7fffffff;  // explicit cap: persistent
    const uint32_t blocks = grid_blocks(want, cap);
    hipLaunchKernelGGL((copy_tile_kernel<G, U, IMPLICIT, UB, T>), dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

// Shapes: 16 x 4 x 2 body slots in round 1 with 32-record tiles (the default: 84 VGPRs, 5 waves per
// SIMD; 64-record tiles hold 43 KB of LDS per workgroup, 3 waves per SIMD) or 64-record tiles
// (CFG_G16U3); 32 x 2 x 1 and 16 x 5 x 1 with 32-record tiles.
template <bool IMPLICIT>
hipError_t launch_copy_tile(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    switch (shape) {
        case CFG_G16U3: return launch_copy_tile_one<IMPLICIT, 16, 4, 2, 64>(p, max_blocks, s);
        case CFG_G32U3:
        case CFG_G32U4: return launch_copy_tile_one<IMPLICIT, 32, 2, 1, 32>(p, max_blocks, s);
        case CFG_G16U6: return launch_copy_tile_one<IMPLICIT, 16, 5, 1, 32>(p, max_blocks, s);
        default: return launch_copy_tile_one<IMPLICIT, 16, 4, 2, 32>(p, max_blocks, s);
    }
}

hipError_t launch_copy_v20(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    return p.desc == nullptr ? launch_copy_tile<true>(shape, p, max_blocks, s)
                             : launch_copy_tile<false>(shape, p, max_blocks, s);
}

template <bool IMPLICIT, int G, int U, int UW = 0, int UB = 0>
hipError_t launch_copy2_one(const KParams& p, uint32_t max_blocks, hipStream_t s) {
    constexpr uint32_t GPB = 256 / G;
    const uint64_t want = (p.n + GPB - 1) / GPB;
    const uint32_t blocks = grid_blocks(want, max_blocks);
    hipLaunchKernelGGL((copy_kernel<G, U, IMPLICIT, UW, UB>), dim3(blocks), dim3(256), 0, s, p);
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

}  // namespace smolcsum
