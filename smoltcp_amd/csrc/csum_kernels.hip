// Batched Internet-checksum kernels for MI355X (gfx950).
//
// One GROUP of G lanes (G = 8, 16, 32 or 64; a group never spans two wavefronts) owns one record
// at a time and walks the batch with a grid stride (persistent grid).  The record's bytes are
// read as 16-byte-ALIGNED chunks with non-temporal global_load_dwordx4 (lane-contiguous, fully
// coalesced; the data is read exactly once, so it is not kept in the caches), U chunks per lane
// per step, so a step moves G*U*16 bytes.  The next step — or the next record's first step — is
// issued before the current one is summed, into a second register set: the loop body is written
// once and instantiated twice with the two sets' roles swapped (no register copies, so the
// compiler's counted s_waitcnt vmcnt leaves the prefetch in flight).  Every load instruction is
// issued unconditionally (out-of-range chunks read a 16-byte dummy line) for the same reason:
// a load inside a branch makes hipcc fall back to vmcnt(0).  Bytes of a chunk outside the summed
// span are masked; an aligned chunk never crosses a page, so reading the few bytes around a
// record is always safe.
//
// Small groups amortise the per-record work (header parse, reductions, the finishing lane) over
// several records per wavefront: at 1500-byte records a G=16 wave finishes four records per step.
//
// The first 128 bytes of each record (8 chunks, already in registers) are copied to a per-group
// LDS window, from which every lane reads the IP/L4 header fields the gates need; L4 header bytes
// past the window (behind a long IPv6 Hop-by-Hop header) are read from global memory.  Per lane
// the protocol kernels add aligned u16 words (v_sad_u16); DPP row reductions combine the group;
// one lane finishes the record: fold, byte-swap for an odd record start (RFC 1071 §2(B)),
// pseudo-header, gate, write.
//
// See csum_device.h for the arithmetic and the reference lines each rule follows.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csum_device.h"
#include "csum_launch.h"

namespace smolcsum {

constexpr int WIN_BYTES = 128;

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
    uint32_t kind;
};

template <bool IMPLICIT>
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
        rr.kind = d.w & 0xffu;
    }
    return rr;
}

__device__ __forceinline__ uint32_t n_chunks(const RecRef& rr) {
    if (rr.len == 0) return 0;
    return (uint32_t)(((rr.a0 + rr.len + 15) >> 4) - (rr.a0 >> 4));
}

template <bool NT>
__device__ __forceinline__ u32x4 ld16(gcv4 q) {
    if (NT) return __builtin_nontemporal_load(q);
    return *q;
}

// Issue the U loads of one step.  Unconditional: chunks past the record (or a step that does
// not exist) read the dummy line instead.
template <int G, int U, bool NT>
__device__ __forceinline__ void load_step(u32x4 (&v)[U], const RecRef& rr, uint32_t nch,
                                          uint32_t step, int lane, bool valid, uint64_t dummy) {
    const uint64_t base = rr.a0 & ~15ull;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t k = step * (G * U) + u * G + lane;
        const uint64_t a = (valid && k < nch) ? base + 16ull * k : dummy;
        v[u] = ld16<NT>((gcv4)a);
    }
}

// One byte from global memory, waited for inside the asm statement.  Used only for header bytes
// outside the LDS window (behind a long IPv6 Hop-by-Hop header).  Hidden from the compiler on
// purpose: a compiler-visible conditional load here makes hipcc's wait insertion drain the
// prefetched steps with vmcnt(0) at the loop head for every record.
__device__ __forceinline__ uint32_t ld_byte_sync(uint64_t a) {
    uint32_t x;
    asm volatile("global_load_ubyte %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(a) : "memory");
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

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Store a big-endian u16 at any byte alignment.
__device__ __forceinline__ void store_be16(gu8 q, uint32_t v) {
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

// Emit patch word, one per record when the field writes are deferred to scatter_kernel:
// bits 0-15 IPv4 header checksum, 16-31 L4 checksum, 32-55 L4 field offset in the record,
// PATCH_IP / PATCH_L4 = write that field, PATCH_ETH = the IPv4 header sits behind Ethernet.
constexpr uint64_t PATCH_IP = 1ull << 56;
constexpr uint64_t PATCH_L4 = 1ull << 57;
constexpr uint64_t PATCH_ETH = 1ull << 58;

// Per-group walk state.
struct Walk {
    uint64_t r;      // current record
    RecRef cur, nxt; // current record, the group's next record (descriptor prefetched)
    uint32_t nch;    // aligned chunks of cur
    uint32_t step;   // step within cur
    Geom g;          // cur's geometry (protocol modes)
    int s1;          // end of the summed span, relative to the record start
    uint32_t acc, acc2;
};

// One step of the walk: prefetch the following step into `nx`, then sum `cv` (the current step)
// and finish the record on its last step.  Returns false when the group has no more work.
template <int G, int U, int MODE, bool IMPLICIT, bool NT, bool PF>
__device__ __forceinline__ bool walk_step(const KParams& p, Walk& w, u32x4 (&cv)[U], u32x4 (&nx)[U],
                                          int lane, uint64_t ngroups, u32x4* win) {
    const uint8_t* winb = reinterpret_cast<const uint8_t*>(win);
    const uint32_t nsteps = w.nch == 0 ? 1u : (w.nch + (G * U) - 1) / (G * U);
    const bool last = w.step + 1 >= nsteps;
    const uint64_t r2 = last ? w.r + ngroups : w.r;
    const bool have2 = r2 < p.n;
    const RecRef rec2 = last ? w.nxt : w.cur;
    const uint32_t nch2 = last ? n_chunks(w.nxt) : w.nch;
    const uint32_t step2 = last ? 0u : w.step + 1;
    if (PF) load_step<G, U, NT>(nx, rec2, nch2, step2, lane, have2, (uint64_t)p.dummy);
    // descriptor of the record after next (clamped index: an unconditional load)
    RecRef nxt2 = w.nxt;
    {
        const uint64_t r3 = r2 + ngroups < p.n ? r2 + ngroups : p.n - 1;
        const RecRef t = rec_at<IMPLICIT>(p, r3);
        if (last) nxt2 = t;
    }

    const uint32_t head = (uint32_t)(w.cur.a0 & 15u);
    // record byte o: LDS window when inside it, else global memory (long IPv6 extension chains)
    auto rd = [&](uint32_t o) -> uint32_t {
        const uint32_t x = head + o;
        return x < (uint32_t)WIN_BYTES ? (uint32_t)winb[x] : ld_byte_sync(w.cur.a0 + o);
    };
    if (w.step == 0) {
        w.acc = 0;
        w.acc2 = 0;
        if (MODE == MODE_DATA) {
            w.s1 = (int)w.cur.len;
        } else {
            if (lane < WIN_BYTES / 16 && (uint32_t)lane < w.nch) win[lane] = cv[0];
            wave_lds_sync();
            w.g = parse_geometry(rd, w.cur.len, w.cur.kind);
            // the lanes sum [0, span_end): the header part is subtracted at the end
            w.s1 = (w.g.proto != P_NONE && !(w.g.st & SMOL_ST_MALFORMED)) ? (int)w.g.span_end : 0;
        }
    }

    // ---- sum this step's chunks over [0, s1) (data: [0, len)) ----
    const int s1 = w.s1;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t k = w.step * (G * U) + u * G + lane;
        const int pos = (int)(16u * k) - (int)head;  // chunk start relative to the record
        if (k < w.nch && pos < s1) {
            const u32x4 c = cv[u];
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

    if (last) {
        const bool odd = (w.cur.a0 & 1u) != 0;
        const uint64_t r = w.r;
        if (MODE == MODE_DATA) {
            // exact little-endian word sum relative to the span start, modulo 2^32
            const uint32_t s_rel = odd ? (w.acc2 + (w.acc << 8)) : (w.acc + (w.acc2 << 8));
            const uint32_t tot = group_sum<G>(s_rel);
            if (lane == 0) ((gu16)p.out16)[r] = (uint16_t)bswap16(fold32(tot));
        } else {
            const Geom& g = w.g;
            // Header bytes [0, l4_off) that the lanes summed (taken out of the L4 sum), the IPv4
            // header's big-endian word sum and the pseudo-header address words.  All of them sit in
            // the LDS window except behind a long Hop-by-Hop header (then read from global memory).
            const bool l4 = g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED);
            const uint32_t l4_off = l4 ? g.l4_off : 0u;
            uint32_t pre = 0;  // aligned-word sum contribution of the bytes [0, l4_off)
            for (uint32_t i = lane; 2 * i < l4_off; i += G) {
                // l4_off is even: record offset 2i is the low byte of an aligned little-endian
                // word for an even record start, the high byte for an odd one
                const uint32_t e = rd(2 * i), o = rd(2 * i + 1);
                pre += odd ? ((e << 8) + o) : (e + (o << 8));
            }
            uint32_t hsum = 0, psum = 0;
            if (g.fam == 4) {
                for (uint32_t i = lane; i < g.ip_hl / 2; i += G) {
                    const uint32_t o = head + g.ip_off + 2 * i;
                    if (!(MODE == MODE_EMIT && i == 5)) hsum += (winb[o] << 8) | winb[o + 1];
                }
            }
            if (l4 && (g.proto == P_UDP || g.proto == P_TCP || g.proto == P_ICMP6)) {
                for (uint32_t i = lane; i < g.addr_words; i += G) {
                    const uint32_t o = head + g.addr_off + 2 * i;
                    psum += (winb[o] << 8) | winb[o + 1];
                }
            }
            const uint32_t tot = group_sum<G>(w.acc);
            pre = group_sum<G>(pre);
            hsum = group_sum<G>(hsum);
            psum = group_sum<G>(psum);
            if (lane == 0) {
                const gu8 wrec = (gu8)w.cur.a0;
                (void)wrec;
                uint32_t st = g.st;
                // IPv4 header: data(header) (canonical fold of the big-endian word sum)
                uint32_t ip_valid = 1, ip_ok = 1;
                uint64_t patch = 0;  // emit: the field writes of this record (see PATCH_* below)
                if (g.fam == 4) {
                    const uint32_t hdr = fold32(hsum);
                    if (MODE == MODE_EMIT) {
                        const uint32_t v = caps_tx(p.caps_ipv4) ? (~hdr & 0xffffu) : 0u;
                        patch |= (uint64_t)v | PATCH_IP | (g.ip_off ? PATCH_ETH : 0ull);
                    } else {
                        ip_valid = hdr == 0xffffu;
                        ip_ok = caps_rx(p.caps_ipv4) ? ip_valid : 1u;
                    }
                }
                uint32_t l4_valid = 1, l4_ok = 1, partial = 0;
                if (l4) {
                    const uint32_t fpos = g.l4_off + g.fo;
                    const uint32_t field = (rd(fpos) << 8) | rd(fpos + 1);
                    // aligned-word sum of the L4 span = lanes' sum of [0, span_end) minus the
                    // header bytes [0, l4_off) (exact: no u32 wrap below 131072 bytes)
                    uint32_t s = tot - pre;
                    if (MODE == MODE_EMIT) {
                        // the reference zeroes the field before summing: remove its bytes (the
                        // field offset is even: its parity is the record start's)
                        const uint32_t f0 = field >> 8, f1 = field & 0xffu;
                        s -= odd ? ((f0 << 8) + f1) : (f0 + (f1 << 8));
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
                    if (MODE == MODE_EMIT) {
                        const bool fill = g.proto == P_IGMP ? true : caps_tx(gate_caps);
                        uint32_t c = ~comb & 0xffffu;
                        if (g.proto == P_UDP && c == 0) c = 0xffffu;  // udp.rs:207
                        patch |= ((uint64_t)(fill ? c : 0u) << 16) | ((uint64_t)fpos << 32) | PATCH_L4;
                    } else {
                        l4_valid = comb == 0xffffu;
                        if (g.proto == P_UDP && field == 0) l4_valid = 1;  // udp.rs:138-140
                        if (g.proto == P_UDP || g.proto == P_TCP) partial = ph == field;
                        l4_ok = caps_rx(gate_caps) ? l4_valid : 1u;
                    }
                }
                if (MODE == MODE_EMIT) {
                    if (p.patch) {
                        // deferred: the scatter pass writes the fields after every read is done
                        ((GMEM uint64_t*)p.patch)[r] = patch;
                    } else {
                        if (patch & PATCH_IP) store_be16(wrec + g.ip_off + 10, (uint32_t)(patch & 0xffffu));
                        if (patch & PATCH_L4) store_be16(wrec + ((patch >> 32) & 0xffffffu), (uint32_t)((patch >> 16) & 0xffffu));
                    }
                    if (p.status) ((gu8)p.status)[r] = (uint8_t)st;
                } else {
                    const bool mal = (st & SMOL_ST_MALFORMED) != 0;
                    st |= (ip_ok ? SMOL_ST_IP_OK : 0u) | (l4_ok ? SMOL_ST_L4_OK : 0u) |
                          (partial ? SMOL_ST_L4_PARTIAL : 0u) | (ip_valid ? SMOL_ST_IP_VALID : 0u) |
                          (l4_valid ? SMOL_ST_L4_VALID : 0u) |
                          ((ip_ok && l4_ok && !mal) ? SMOL_ST_ACCEPT : 0u);
                    ((gu8)p.status)[r] = (uint8_t)st;
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
// VAR: 0 = non-temporal loads + register prefetch (default), 1 = plain loads + prefetch,
// 2 = non-temporal loads, no prefetch (each step loads then waits; occupancy hides latency).
template <int G, int U, int MODE, bool IMPLICIT, int VAR>
__global__ __launch_bounds__(256) void csum_kernel(KParams p) {
    constexpr bool NT = VAR != 1;
    constexpr bool PF = VAR != 2;
    constexpr int GPB = 256 / G;
    static_assert(G >= 8 && G <= 64 && (G & (G - 1)) == 0, "group size");
    __shared__ u32x4 win[GPB][WIN_BYTES / 16];

    const int lane = (int)(threadIdx.x % G);
    const int gib = (int)(threadIdx.x / G);
    const uint64_t ngroups = (uint64_t)gridDim.x * GPB;
    Walk w;
    w.r = (uint64_t)blockIdx.x * GPB + gib;
    if (w.r >= p.n) return;
    w.cur = rec_at<IMPLICIT>(p, w.r);
    w.nxt = rec_at<IMPLICIT>(p, w.r + ngroups < p.n ? w.r + ngroups : p.n - 1);
    w.nch = n_chunks(w.cur);
    w.step = 0;
    w.g = Geom{};
    w.s1 = 0;
    w.acc = w.acc2 = 0;

    u32x4 va[U];
    if (PF) {
        u32x4 vb[U];
        load_step<G, U, NT>(va, w.cur, w.nch, 0, lane, true, (uint64_t)p.dummy);
        // the body is instantiated twice with the register sets' roles swapped
        while (true) {
            if (!walk_step<G, U, MODE, IMPLICIT, NT, PF>(p, w, va, vb, lane, ngroups, &win[gib][0])) break;
            if (!walk_step<G, U, MODE, IMPLICIT, NT, PF>(p, w, vb, va, lane, ngroups, &win[gib][0])) break;
        }
    } else {
        while (true) {
            load_step<G, U, NT>(va, w.cur, w.nch, w.step, lane, true, (uint64_t)p.dummy);
            if (!walk_step<G, U, MODE, IMPLICIT, NT, PF>(p, w, va, va, lane, ngroups, &win[gib][0])) break;
        }
    }
}

// Second pass of a deferred emit: one lane per record applies the patch word.  Writing the 2-byte
// fields inside the read pass interleaves a scattered write with every 1.5 KB of streamed reads,
// which cost ~40 % of a read pass on MI355X (tools/probe_wr.hip); a compact patch array (+5 %)
// plus this write-only pass is far cheaper.
template <bool IMPLICIT>
__global__ __launch_bounds__(256) void scatter_kernel(KParams p) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < p.n; r += stride) {
        const uint64_t patch = ((const GMEM uint64_t*)p.patch)[r];
        if (!(patch & (PATCH_IP | PATCH_L4))) continue;
        uint64_t a0;
        if (IMPLICIT) {
            a0 = (uint64_t)p.buf + r * p.stride;
        } else {
            const GMEM uint64_t* d = (const GMEM uint64_t*)((uint64_t)p.desc + 16 * r);
            a0 = (uint64_t)p.buf + d[0];
        }
        if (patch & PATCH_IP) store_be16((gu8)(a0 + ((patch & PATCH_ETH) ? 24 : 10)), (uint32_t)(patch & 0xffffu));
        if (patch & PATCH_L4) store_be16((gu8)(a0 + ((patch >> 32) & 0xffffffu)), (uint32_t)((patch >> 16) & 0xffffu));
    }
}

hipError_t launch_scatter(const KParams& p, uint32_t max_blocks, hipStream_t s) {
    const uint64_t want = (p.n + 255) / 256;
    const uint32_t blocks = (uint32_t)(want < max_blocks ? want : max_blocks);
    if (p.desc) hipLaunchKernelGGL(scatter_kernel<false>, dim3(blocks), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(scatter_kernel<true>, dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Launch table
// ---------------------------------------------------------------------------------------------

template <int G, int U, int MODE, bool IMPLICIT, int VAR>
static hipError_t launch_one(const KParams& p, uint32_t max_blocks, hipStream_t s) {
    constexpr uint32_t GPB = 256 / G;
    const uint64_t want = (p.n + GPB - 1) / GPB;
    const uint32_t blocks = (uint32_t)(want < max_blocks ? want : max_blocks);
    hipLaunchKernelGGL((csum_kernel<G, U, MODE, IMPLICIT, VAR>), dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

template <int MODE, bool IMPLICIT, int VAR>
static hipError_t launch_shape(int shape, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    switch (shape) {
        case CFG_G8U6: return launch_one<8, 6, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G16U3: return launch_one<16, 3, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G16U6: return launch_one<16, 6, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G32U3: return launch_one<32, 3, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G32U4: return launch_one<32, 4, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        case CFG_G64U2: return launch_one<64, 2, MODE, IMPLICIT, VAR>(p, max_blocks, s);
        default: return launch_one<64, 4, MODE, IMPLICIT, VAR>(p, max_blocks, s);
    }
}

template <int MODE>
static hipError_t launch_mode(int shape, int var, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    const bool implicit = p.desc == nullptr;
    switch (var) {
        case 1:
            return implicit ? launch_shape<MODE, true, 1>(shape, p, max_blocks, s)
                            : launch_shape<MODE, false, 1>(shape, p, max_blocks, s);
        case 2:
            return implicit ? launch_shape<MODE, true, 2>(shape, p, max_blocks, s)
                            : launch_shape<MODE, false, 2>(shape, p, max_blocks, s);
        default:
            return implicit ? launch_shape<MODE, true, 0>(shape, p, max_blocks, s)
                            : launch_shape<MODE, false, 0>(shape, p, max_blocks, s);
    }
}

hipError_t launch_csum(int mode, int shape, int var, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    switch (mode) {
        case MODE_DATA: return launch_mode<MODE_DATA>(shape, var, p, max_blocks, s);
        case MODE_EMIT: return launch_mode<MODE_EMIT>(shape, var, p, max_blocks, s);
        default: return launch_mode<MODE_VERIFY>(shape, var, p, max_blocks, s);
    }
}

}  // namespace smolcsum
