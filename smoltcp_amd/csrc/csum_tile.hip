// Tile kernel: batched emit / verify for MI355X (gfx950).  The library's default only for emit over
// descriptor batches (C3; csum_api.cpp auto_variant); every other call runs the walk kernel.
//
// A wavefront owns a TILE of 32 or 64 consecutive records and works on it in three phases:
//
//   A  lane i reads record i's descriptor (implicit batches: pure arithmetic);
//   B  groups of G lanes stream the records' bytes: group g sums records g, g + 64/G, ... with
//      16-byte-aligned non-temporal global_load_dwordx4 (U per lane per step), one v_sad_u16 per
//      dword, a DPP row reduction per record, and store each record's aligned-word sum plus the
//      record's first 128 bytes (its header window) in LDS.  No header parsing happens here: the
//      whole record buffer [a0, a0 + len) is summed, bytes past the record end are masked;
//   C  lane i finishes record i alone: it parses the header from its LDS window, takes the bytes
//      outside the checksummed span back out of the sum (header, bytes before the record start,
//      trailing bytes past the L4 span), and applies the gate: status byte (verify) or field
//      writes (emit).  64 records per instruction instead of one record per group-instruction.
//
// The walk kernel (csum_walk.h: a group parses and finishes its own record) spent
// ~134 VALU + ~68 SALU wave-instructions per 1500-byte record (rocprofv3 SQ_INSTS_*); here
// phase B is a short straight loop and phase C is fully SIMD-parallel.
//
// Arithmetic: all sums are aligned little-endian u16 word sums of absolute addresses (exact in
// u32 below 131072 bytes).  A window byte at offset x has the parity of its absolute address, so
// a region's contribution is sum(b_x << 8*(x & 1)).  The reference's data() of a span with even
// record offset is bswap16(fold(S)) for an even record start and fold(S) for an odd one (RFC 1071
// §2(B)); see csum_device.h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csum_device.h"
#include "csum_launch.h"

namespace smolcsum {

namespace tile {

constexpr int WIN = 96;       // header window bytes per record (from the record's aligned chunk):
                              // Ethernet + IPv6 + TCP headers at any start alignment fit
constexpr int WSTRIDE = 25;   // dwords per window row in LDS: 100 B (odd), so that the 64 lanes of
                              // phase C reading dword d of their own rows hit distinct banks

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GMEM __attribute__((address_space(1)))
typedef const GMEM u32x4* gcv4;
typedef GMEM uint8_t* gu8;
typedef GMEM uint16_t* gu16;

template <int T>  // records per wavefront tile
struct WaveLds {
    uint32_t win[T * WSTRIDE];
    uint32_t sum[T];
    uint32_t info[3 * T];  // descriptor batches: record address lo / hi, length
};

struct Slot {
    uint64_t a0;
    uint32_t len, nch;  // nch: chunks of the load grid
};

__device__ __forceinline__ uint32_t ld_byte_sync(uint64_t a) {
    // one byte from global memory, waited for inside the asm (invisible to hipcc's wait
    // insertion on purpose; slow path only — header bytes outside the window)
    uint32_t x;
    asm volatile("global_load_ubyte %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(a) : "memory");
    return x;
}

template <bool NT>
__device__ __forceinline__ u32x4 ld16(gcv4 q) {
    if (NT) return __builtin_nontemporal_load(q);
    return *q;
}

__device__ __forceinline__ void store_be16(gu8 q, uint32_t v) {
    if (((uint64_t)q & 1u) == 0) {
        *(gu16)q = (uint16_t)bswap16(v);
    } else {
        q[0] = (uint8_t)(v >> 8);
        q[1] = (uint8_t)v;
    }
}

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

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Window byte x of a lane's row (x < WIN).
__device__ __forceinline__ uint32_t wbyte(const uint32_t* row, uint32_t x) {
    return (row[x >> 2] >> (8 * (x & 3))) & 0xffu;
}

// Aligned-word contribution of the window bytes [from, to) (window offsets; past WIN the bytes are
// read from global memory at base + x, base = the record's aligned chunk start).
__device__ __forceinline__ uint32_t region_sum(const uint32_t* row, uint64_t base, uint32_t from,
                                               uint32_t to) {
    uint32_t acc = 0;
    const uint32_t wto = to < (uint32_t)WIN ? to : (uint32_t)WIN;
    if (from < wto) {
        for (uint32_t d = from >> 2; d < ((wto + 3) >> 2); ++d) {
            const int lo = (int)from - (int)(4 * d), hi = (int)wto - (int)(4 * d);
            acc = add_words(mask_dword(row[d], lo, hi), acc);
        }
    }
    for (uint32_t x = from > (uint32_t)WIN ? from : (uint32_t)WIN; x < to; ++x)  // slow path
        acc += ld_byte_sync(base + x) << (8 * (x & 1));
    return acc;
}

// Phase C of one record, by one lane alone (the tile and stripe kernels): parse the header from the
// record's LDS window row (WIN bytes from its 16-byte boundary), take the bytes outside the summed
// span back out of `sum`, apply the gates, write the status byte or the fields of record r.
// `sum`: the aligned-word sum of [a0 & ~15, a0 + len) (tile); EXACT: of [a0, a0 + len) (stripe).
template <int MODE, bool EXACT>
__device__ __forceinline__ void finish_record(const KParams& p, const uint32_t* row, uint32_t sum, uint64_t my_a0,
                                              uint32_t my_len, uint32_t my_kind, uint64_t r) {
    const uint32_t head = (uint32_t)(my_a0 & 15u);
    const uint64_t base = my_a0 & ~15ull;
    const bool odd = (my_a0 & 1u) != 0;
    const uint32_t nch = my_len ? (uint32_t)(((my_a0 + my_len + 15) >> 4) - (my_a0 >> 4)) : 0u;
    const uint32_t wvalid = nch * 16 < (uint32_t)WIN ? nch * 16 : (uint32_t)WIN;  // bytes the window holds
    auto rd = [&](uint32_t o) -> uint32_t {  // record byte o (o < len)
        const uint32_t x = head + o;
        return x < wvalid ? wbyte(row, x) : ld_byte_sync(my_a0 + o);
    };
    const Geom g = parse_geometry(rd, my_len, my_kind, MODE == MODE_EMIT);
    const bool l4 = g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED);
    uint32_t st = g.st;
    uint32_t ip_valid = 1, ip_ok = 1, l4_valid = 1, l4_ok = 1, partial = 0;
    uint32_t ip_val = 0, l4_val = 0, fpos = 0, in_val = 0;
    auto rsum = [&](uint32_t from, uint32_t to) -> uint32_t {  // record offsets
        if (head + to <= wvalid) return region_sum(row, base, head + from, head + to);
        uint32_t a = 0;  // slow path: straddles or leaves the window
        for (uint32_t o = from; o < to; ++o) a += rd(o) << (8 * ((head + o) & 1));
        return a;
    };
    if (g.fam == 4) {
        uint32_t sh = rsum(g.ip_off, g.ip_off + g.ip_hl);
        if (MODE == MODE_EMIT) {
            const uint32_t f0 = rd(g.ip_off + 10), f1 = rd(g.ip_off + 11);
            sh -= odd ? ((f0 << 8) + f1) : (f0 + (f1 << 8));
        }
        const uint32_t f = fold32(sh);
        const uint32_t hdr = odd ? f : bswap16(f);  // == checksum::data(header)
        if (MODE == MODE_EMIT) {
            ip_val = caps_tx(p.caps_ipv4) ? (~hdr & 0xffffu) : 0u;
        } else {
            ip_valid = hdr == 0xffffu;
            ip_ok = caps_rx(p.caps_ipv4) ? ip_valid : 1u;
        }
    }
    if (l4) {
        fpos = g.l4_off + g.fo;
        const uint32_t field = (rd(fpos) << 8) | rd(fpos + 1);
        // L4 span sum = whole-buffer sum - [aligned start, l4_off) - [span_end, len)
        uint32_t s = sum - rsum(0, g.l4_off) - (!EXACT && head ? region_sum(row, base, 0, head) : 0u);
        if (g.span_end < my_len) s -= rsum(g.span_end, my_len);
        auto word = [&](uint32_t v) { return odd ? v : bswap16(v); };  // BE u16 at an even offset
        if (MODE == MODE_EMIT) {
            s -= word(field);
            if (g.in_off) {  // ICMPv4 error: the embedded IPv4 header first (csum_device.h)
                uint32_t hin = 0;
                for (uint32_t i = 0; i < g.in_hl / 2; ++i)
                    if (i != 5) hin += (rd(g.in_off + 2 * i) << 8) | rd(g.in_off + 2 * i + 1);
                in_val = caps_tx(p.caps_ipv4) ? (~fold32(hin) & 0xffffu) : 0u;
                const uint32_t fi = g.in_off + 10;
                s = s - word((rd(fi) << 8) | rd(fi + 1)) + word(in_val);
            }
        }
        const uint32_t f = fold32(s);
        const uint32_t dat = odd ? f : bswap16(f);  // == checksum::data(span)
        const bool pseudo = g.proto == P_UDP || g.proto == P_TCP || g.proto == P_ICMP6;
        uint32_t ph = 0;
        if (pseudo) {
            const uint32_t xa = fold32(rsum(g.addr_off, g.addr_off + 2 * g.addr_words));
            const uint32_t addr = odd ? xa : bswap16(xa);  // canonical big-endian address sum
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
        if (MODE == MODE_EMIT) {
            const bool fill = g.proto == P_IGMP ? true : caps_tx(gate_caps);
            uint32_t c = ~comb & 0xffffu;
            if (g.proto == P_UDP && c == 0) c = 0xffffu;  // udp.rs:207
            l4_val = fill ? c : 0u;
        } else {
            l4_valid = comb == 0xffffu;
            if (g.proto == P_UDP && field == 0) l4_valid = 1;  // udp.rs:138-140
            if (g.proto == P_UDP || g.proto == P_TCP) partial = ph == field;
            l4_ok = caps_rx(gate_caps) ? l4_valid : 1u;
        }
    }
    if (MODE == MODE_EMIT) {
        if (g.fam == 4) store_be16((gu8)(my_a0 + g.ip_off + 10), ip_val);
        if (g.in_off) store_be16((gu8)(my_a0 + g.in_off + 10), in_val);
        if (l4) store_be16((gu8)(my_a0 + fpos), l4_val);
        if (p.status) ((gu8)p.status)[r] = (uint8_t)st;
    } else {
        const bool mal = (st & SMOL_ST_MALFORMED) != 0;
        st |= (ip_ok ? SMOL_ST_IP_OK : 0u) | (l4_ok ? SMOL_ST_L4_OK : 0u) |
              (partial ? SMOL_ST_L4_PARTIAL : 0u) | (ip_valid ? SMOL_ST_IP_VALID : 0u) |
              (l4_valid ? SMOL_ST_L4_VALID : 0u) | ((ip_ok && l4_ok && !mal) ? SMOL_ST_ACCEPT : 0u);
        ((gu8)p.status)[r] = (uint8_t)st;
    }
}

// VAR: 0 = non-temporal record loads, 1 = plain loads (both on the record's 16-byte grid),
// 2 = non-temporal loads on the record's 128-byte line grid (see csum_walk.h: nt loads need whole
// lines; the chunks before the record are loaded and not summed).
template <int G, int U, int MODE, bool IMPLICIT, int VAR, int TILE>
__global__ __launch_bounds__(256) void csum_tile_kernel(KParams p) {
    constexpr bool NT = VAR != 1;
    constexpr uint64_t GRID = VAR == 2 ? 128 : 16;  // load-grid alignment
    constexpr int GPW = 64 / G;  // groups per wavefront
    static_assert(G >= 8 && G <= 64 && (G & (G - 1)) == 0, "group size");
    static_assert(TILE == 32 || TILE == 64, "tile");
    __shared__ WaveLds<TILE> lds[4];

    const int wave = (int)(threadIdx.x >> 6);
    const int lane = (int)(threadIdx.x & 63);
    const int gl = lane % G;   // lane within its group
    const int grp = lane / G;  // group within the wavefront
    WaveLds<TILE>& L = lds[wave];
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    const uint64_t dummy = (uint64_t)p.dummy;

    for (uint64_t tile = logical_block(p.xcd_remap) * 4 + wave; tile * TILE < p.n; tile += nwaves) {
        const uint64_t r0 = tile * TILE;
        const uint32_t cnt = (uint32_t)((p.n - r0) < (uint64_t)TILE ? (p.n - r0) : (uint64_t)TILE);

        // ---- phase A: lane i's record ----
        uint64_t my_a0 = dummy;
        uint32_t my_len = 0, my_kind = SMOL_KIND_RAW;
        if (IMPLICIT) {
            my_a0 = (uint64_t)p.buf + (r0 + lane) * p.stride;
            my_len = (uint32_t)lane < cnt ? p.len : 0u;
            my_kind = p.kind;
        } else {
            const uint64_t ri = r0 + ((uint32_t)lane < cnt ? (uint32_t)lane : 0u);
            const u32x4 d = *(gcv4)((uint64_t)p.desc + 16 * ri);
            if ((uint32_t)lane < cnt) {
                my_a0 = (uint64_t)p.buf + ((uint64_t)d.x | ((uint64_t)d.y << 32));
                my_len = d.z;
                my_kind = desc_kind(d.w);
            }
        }

        // ---- phase B: stream and sum, GPW records at a time ----
        // Slot j of this group = record q = j*GPW + grp of the tile.  The group walks its
        // (slot, step) items with the next item's loads issued before the current one is summed
        // (two register sets, the loop body instantiated twice with their roles swapped).
        if (!IMPLICIT && lane < TILE) {
            L.info[3 * lane] = (uint32_t)my_a0;
            L.info[3 * lane + 1] = (uint32_t)(my_a0 >> 32);
            L.info[3 * lane + 2] = my_len;
        }
        wave_lds_sync();
        auto slot = [&](int j) -> Slot {
            const int q = j * GPW + grp;
            Slot sl;
            if (IMPLICIT) {
                sl.a0 = (uint64_t)p.buf + (r0 + q) * p.stride;
                sl.len = (uint32_t)q < cnt ? p.len : 0u;
            } else {
                sl.a0 = (uint64_t)L.info[3 * q] | ((uint64_t)L.info[3 * q + 1] << 32);
                sl.len = L.info[3 * q + 2];
            }
            sl.nch = sl.len ? (uint32_t)(((sl.a0 + sl.len + 15) >> 4) - ((sl.a0 & ~(GRID - 1)) >> 4)) : 0u;
            return sl;
        };
        auto load = [&](u32x4 (&v)[U], const Slot& sl, uint32_t step, bool valid) {
            const uint64_t base = sl.a0 & ~(GRID - 1);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t k = step * (G * U) + u * G + gl;
                v[u] = ld16<NT>((gcv4)(valid && k < sl.nch ? base + 16ull * k : dummy));
            }
        };
        // the item after (j, step) of slot sl; false when the tile is done
        auto next = [&](int& j, uint32_t& step, Slot& sl) -> bool {
            const uint32_t nst = sl.nch ? (sl.nch + (G * U) - 1) / (G * U) : 1u;
            if (step + 1 < nst) {
                ++step;
                return true;
            }
            ++j;
            step = 0;
            if (j >= TILE / GPW) return false;
            sl = slot(j);
            return true;
        };
        uint32_t acc = 0;
        auto process = [&](const u32x4 (&v)[U], const Slot& sl, int j, uint32_t step) {
            const int q = j * GPW + grp;
            // the window holds the chunks from the record's 16-byte boundary: grid chunks k0 ..
            const uint32_t k0 = (uint32_t)((sl.a0 & (GRID - 1)) >> 4);
            if (step == 0) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t k = (uint32_t)(u * G + gl);
                    if (GRID == 16 && u > 0) break;
                    if (k >= k0 && k - k0 < (uint32_t)(WIN / 16) && k < sl.nch) {
                        uint32_t* row = &L.win[q * WSTRIDE + 4 * (k - k0)];
                        row[0] = v[u].x;
                        row[1] = v[u].y;
                        row[2] = v[u].z;
                        row[3] = v[u].w;
                    }
                }
            }
            const int endrel = (int)((uint32_t)(sl.a0 & (GRID - 1)) + sl.len);  // record end, from the grid
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t k = step * (G * U) + u * G + gl;
                u32x4 c = v[u];
                const int lim = endrel - (int)(16 * k);  // bytes of this chunk inside the record
                if (lim < 16) {                          // the record's last chunk (or none)
                    c.x = mask_dword(c.x, 0, lim);
                    c.y = mask_dword(c.y, 0, lim - 4);
                    c.z = mask_dword(c.z, 0, lim - 8);
                    c.w = mask_dword(c.w, 0, lim - 12);
                }
                if (GRID > 16 && k < k0) c = u32x4{0u, 0u, 0u, 0u};  // wholly before the record
                acc = add_words(c.x, add_words(c.y, add_words(c.z, add_words(c.w, acc))));
            }
            const uint32_t nst = sl.nch ? (sl.nch + (G * U) - 1) / (G * U) : 1u;
            if (step + 1 >= nst) {  // the record's last step
                const uint32_t tot = group_sum<G>(acc);
                if (gl == 0) L.sum[q] = tot;
                acc = 0;
            }
        };
        {
            int j = 0;
            uint32_t step = 0;
            Slot cur = slot(0);
            u32x4 va[U], vb[U];
            load(va, cur, 0, true);
            while (true) {
                int j2 = j;
                uint32_t s2 = step;
                Slot n2 = cur;
                bool more = next(j2, s2, n2);
                load(vb, n2, s2, more);
                process(va, cur, j, step);
                if (!more) break;
                j = j2;
                step = s2;
                cur = n2;
                more = next(j2, s2, n2);
                load(va, n2, s2, more);
                process(vb, cur, j, step);
                if (!more) break;
                j = j2;
                step = s2;
                cur = n2;
            }
        }
        wave_lds_sync();

        // ---- phase C: lane i finishes record i ----
        if ((uint32_t)lane < cnt) finish_record<MODE, false>(p, &L.win[lane * WSTRIDE], L.sum[lane], my_a0, my_len, my_kind, r0 + lane);
        wave_lds_sync();  // phase C's window reads complete before the next tile's phase B writes
    }
}


#ifdef SMOL_EXP
// ---------------------------------------------------------------------------------------------
// Stripe kernel (experiments build; fixed-stride emit / verify over packed records of 1024..1520
// bytes, natural grid).  Measured slower than the walk kernel: C2 verify
// 0.264-0.268 against 0.242 ms, C4 0.315 against 0.210 ms, C2 emit 0.345 against 0.316 ms fresh —
// the reads are faster, but one lane per record in phase C does the per-record work serially.
//
// A wavefront owns T = 8 consecutive records and reads their whole span (from the first record's
// 128-byte line) as wave-contiguous 1-KiB pieces, NU per lane, all in flight at once: each load
// instruction covers 8 consecutive lines of one place in the batch, where the walk kernel's covers
// one line in each of 8 records.  Read-only probe over C2's 1.5 GB (tools/probe_pol.hip,
// tools/probe_bw.hip): groups of 8 lanes over 2 steps 6.5 TB/s, one wave-wide step per record
// 7.2 TB/s, 8-record stripes 7.1 TB/s.
//
// Phase B attributes each 16-byte chunk to the record holding its FIRST byte (a piece spans at most
// two records, since stride >= 1024: the record of its first chunk and the next), keeps a running
// sum for both, and reduces a record's sum over the wavefront when the pieces leave it.  The bytes
// of a record's first chunk that follow its start (the chunk is attributed to the previous record)
// are moved back in phase C from the record's window: + its own, - its successor's (a lane shuffle).
// Bytes before the first record and past the last are masked.  Phase C is the tile kernel's.
constexpr int STRIPE_T = 8;

template <int MODE, int NU>
__global__ __launch_bounds__(256) void csum_stripe_kernel(KParams p) {
    constexpr int T = STRIPE_T;
    __shared__ WaveLds<T> lds[4];
    const int wave = (int)(threadIdx.x >> 6);
    const int lane = (int)(threadIdx.x & 63);
    WaveLds<T>& L = lds[wave];
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    const uint64_t dummy = (uint64_t)p.dummy;
    const int32_t stride = (int32_t)p.stride;  // == len (packed), 1024 .. (NU * 1024 - 127) / T

    for (uint64_t tile = logical_block(p.xcd_remap) * 4 + wave; tile * T < p.n; tile += nwaves) {
        const uint64_t r0 = tile * T;
        const uint32_t cnt = (uint32_t)((p.n - r0) < (uint64_t)T ? (p.n - r0) : (uint64_t)T);
        const uint64_t a00 = (uint64_t)p.buf + r0 * p.stride;
        const uint64_t S0 = a00 & ~127ull;
        const int32_t h0 = (int32_t)(a00 - S0);
        const int32_t end = (int32_t)cnt * stride;  // offsets relative to a00

        // ---- phase B: the stripe, all pieces in flight ----
        u32x4 v[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int32_t q = 1024 * u + 16 * lane - h0;  // the chunk's first byte, relative to a00
            v[u] = ld16<true>((gcv4)(q < end && q + 16 > 0 ? S0 + 1024ull * u + 16ull * lane : dummy));
        }
        uint32_t cur = 0, nxt = 0;  // the sums of records ja and ja + 1 (this lane's part)
        int32_t ja = h0 > 0 ? -1 : 0;       // the record of the piece's first byte (wave-uniform)
        int32_t nb = (ja + 1) * stride;     // start of record ja + 1
        auto flush = [&](int32_t jr, uint32_t x) {
            const uint32_t tot = group_sum<64>(x);
            if (lane == 0 && jr >= 0 && jr < (int32_t)cnt) L.sum[jr] = tot;
        };
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int32_t o = 1024 * u - h0;  // the piece's first byte (uniform)
            if (u > 0 && o >= nb) {           // the pieces have left record ja
                flush(ja, cur);
                cur = nxt;
                nxt = 0;
                ++ja;
                nb += stride;
            }
            const int32_t q = o + 16 * lane;
            u32x4 c = v[u];
            uint32_t x;
            if (o + 1024 > end && o < end + 16)  // the stripe's last bytes: mask past the end (uniform)
                x = add_words(mask_dword(c.x, 0, end - q), add_words(mask_dword(c.y, 0, end - q - 4),
                    add_words(mask_dword(c.z, 0, end - q - 8), add_words(mask_dword(c.w, 0, end - q - 12), 0u))));
            else
                x = add_words(c.x, add_words(c.y, add_words(c.z, add_words(c.w, 0u))));
            if (u == 0 && q < 0) x = 0;  // before the first record (attributed to record -1)
            const bool b = q >= nb;
            cur += b ? 0u : x;
            nxt += b ? x : 0u;
            // the window rows: the chunks [w, w + WIN) of the record holding the chunk's last byte,
            // w = the record's 16-byte boundary (relative to a00)
            const int32_t jw = q + 15 >= nb ? ja + 1 : ja;
            if (jw >= 0 && jw < (int32_t)cnt) {
                const int32_t w = jw * stride - (int32_t)((a00 + (uint64_t)(jw * stride)) & 15u);
                const int32_t k = q - w;
                if (k >= 0 && k < WIN) {
                    uint32_t* row = &L.win[jw * WSTRIDE + (k >> 2)];
                    row[0] = c.x;
                    row[1] = c.y;
                    row[2] = c.z;
                    row[3] = c.w;
                }
            }
        }
        flush(ja, cur);
        flush(ja + 1, nxt);
        wave_lds_sync();

        // ---- phase C: lane i finishes record i ----
        const uint64_t my_a0 = a00 + (uint64_t)lane * p.stride;
        const uint32_t* row = &L.win[(lane < T ? lane : 0) * WSTRIDE];
        const uint32_t hd = (uint32_t)(my_a0 & 15u);
        // the bytes [a0, 16-byte boundary) of this record's first chunk, summed with record i - 1
        const uint32_t xs = (lane < (int)cnt && hd) ? region_sum(row, my_a0 & ~15ull, hd, 16) : 0u;
        const uint32_t xn = (uint32_t)__shfl_down((int)xs, 1, 64);
        if ((uint32_t)lane < cnt) {
            const uint32_t sum = L.sum[lane] + xs - ((uint32_t)lane + 1 < cnt ? xn : 0u);
            finish_record<MODE, true>(p, row, sum, my_a0, p.len, p.kind, r0 + lane);
        }
        wave_lds_sync();  // phase C's window reads complete before the next tile's phase B writes
    }
}
#endif

template <int G, int U, int MODE, bool IMPLICIT, int VAR, int TILE>
static hipError_t launch_one(const KParams& p, uint32_t max_blocks, hipStream_t s) {
    auto kern = csum_tile_kernel<G, U, MODE, IMPLICIT, VAR, TILE>;
    const uint64_t tiles = (p.n + TILE - 1) / TILE;
    const uint64_t want = (tiles + 3) / 4;
    // Default: one tile per wavefront (the hardware dispatcher balances the tiles; a persistent
    // grid looping over coarse tiles measured 10-25 % slower on MI355X from tail imbalance).
    // An explicit cap (smol_csum_tool_set_max_blocks, num_cu == 0) makes the grid persistent.
    (void)kern;
    const uint64_t cap = p.num_cu == 0 ? max_blocks : (uint64_t)0x7fffffff;
    const uint32_t blocks = grid_blocks(want, cap);
    note_launch(KERN_TILE, VAR, G, U);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

template <int MODE, bool IMPLICIT, int VAR, int TILE>
static hipError_t launch_shape(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    switch (shape) {
        case CFG_G8U6:
        case CFG_G8U7: return launch_one<8, 6, MODE, IMPLICIT, VAR, TILE>(p, max_blocks, s);
        case CFG_G16U3:
        case CFG_G16U4: return launch_one<16, 3, MODE, IMPLICIT, VAR, TILE>(p, max_blocks, s);
        case CFG_G16U6: return launch_one<16, 6, MODE, IMPLICIT, VAR, TILE>(p, max_blocks, s);
        case CFG_G32U3: return launch_one<32, 3, MODE, IMPLICIT, VAR, TILE>(p, max_blocks, s);
        case CFG_G32U4: return launch_one<32, 4, MODE, IMPLICIT, VAR, TILE>(p, max_blocks, s);
        case CFG_G64U2: return launch_one<64, 2, MODE, IMPLICIT, VAR, TILE>(p, max_blocks, s);
        default: return launch_one<64, 4, MODE, IMPLICIT, VAR, TILE>(p, max_blocks, s);
    }
}

// var 2 (variant 7: nt loads on the line grid) is the product's; 0 / 1 (variants 3 / 4: nt / plain
// loads on the 16-B grid) are in the experiments build only (SMOL_EXP).
template <int MODE, int TILE>
static hipError_t launch_mode(int shape, int var, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    const bool implicit = p.desc == nullptr;
    if (var == 2) {
        return implicit ? launch_shape<MODE, true, 2, TILE>(shape, p, max_blocks, s)
                        : launch_shape<MODE, false, 2, TILE>(shape, p, max_blocks, s);
    }
#ifdef SMOL_EXP
    if (var == 1) {
        return implicit ? launch_shape<MODE, true, 1, TILE>(shape, p, max_blocks, s)
                        : launch_shape<MODE, false, 1, TILE>(shape, p, max_blocks, s);
    }
    return implicit ? launch_shape<MODE, true, 0, TILE>(shape, p, max_blocks, s)
                    : launch_shape<MODE, false, 0, TILE>(shape, p, max_blocks, s);
#else
    return hipErrorInvalidValue;
#endif
}

}  // namespace tile

// The stripe kernel serves fixed-stride batches of packed records (stride == len) of 1024 .. 1520
// bytes over a natural grid; false: not this batch.
bool stripe_fits(const KParams& p) {
#ifdef SMOL_EXP
    return p.desc == nullptr && p.len == p.stride && p.len >= 1024 && p.len <= (12 * 1024 - 127) / tile::STRIPE_T;
#else
    return false;
#endif
}

hipError_t launch_stripe(int mode, const KParams& p, hipStream_t s) {
#ifdef SMOL_EXP
    const uint64_t blocks = (p.n + 4 * tile::STRIPE_T - 1) / (4 * tile::STRIPE_T);
    const uint32_t b = grid_blocks(blocks, 0x7fffffff);
    note_launch(KERN_TILE, 42, 64, 12);
    if (mode == MODE_EMIT) hipLaunchKernelGGL((tile::csum_stripe_kernel<MODE_EMIT, 12>), dim3(b), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((tile::csum_stripe_kernel<MODE_VERIFY, 12>), dim3(b), dim3(256), 0, s, p);
    return hipGetLastError();
#else
    (void)mode, (void)p, (void)s;
    return hipErrorInvalidValue;
#endif
}

hipError_t launch_tile(int mode, int shape, int var, int tile_records, const KParams& p, uint32_t max_blocks,
                       hipStream_t s) {
    if (tile_records == 64) {
        if (mode == MODE_EMIT) return tile::launch_mode<MODE_EMIT, 64>(shape, var, p, max_blocks, s);
        return tile::launch_mode<MODE_VERIFY, 64>(shape, var, p, max_blocks, s);
    }
    if (mode == MODE_EMIT) return tile::launch_mode<MODE_EMIT, 32>(shape, var, p, max_blocks, s);
    return tile::launch_mode<MODE_VERIFY, 32>(shape, var, p, max_blocks, s);
}

}  // namespace smolcsum
