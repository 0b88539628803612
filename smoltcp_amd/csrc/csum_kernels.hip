// Batched Internet-checksum kernels for MI355X (gfx950).
//
// One GROUP of G lanes (G = 16, 32 or 64; a group never spans two wavefronts) owns one record at
// a time and walks the batch with a grid stride (persistent grid).  The record's bytes are read
// as 16-byte-ALIGNED chunks (global_load_dwordx4, lane-contiguous, fully coalesced), U chunks per
// lane per step, so a step moves G*U*16 bytes; the next step — or the next record's first step —
// is issued before the current one is summed (register double buffer), which keeps two steps of
// HBM reads in flight per group.  Bytes of a chunk outside the summed span are masked; an
// aligned chunk never crosses a page, so reading the few bytes around a record is always safe.
//
// The first 128 bytes of each record (8 chunks, already in registers) are copied to a per-group
// LDS window, from which every lane reads the IP/L4 header fields the gates need; header bytes
// past the window (IPv6 Hop-by-Hop options) are read from global memory.  Per lane the protocol
// kernels add aligned u16 words (v_sad_u16); a group reduction and one lane finish the record:
// fold, byte-swap for an odd record start (RFC 1071 §2(B)), pseudo-header, gate, write.
//
// See csum_device.h for the arithmetic and the reference lines each rule follows.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csum_device.h"
#include "csum_launch.h"

namespace smolcsum {

constexpr int WIN_BYTES = 128;

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
        const uint4 d = *reinterpret_cast<const uint4*>(p.desc + r);
        rr.a0 = (uint64_t)p.buf + ((uint64_t)d.x | ((uint64_t)d.y << 32));
        rr.len = d.z;
        rr.kind = d.w & 0xffu;
    }
    return rr;
}

__device__ __forceinline__ uint32_t n_chunks(const RecRef& rr) {
    if (rr.len == 0) return 0;
    const uint64_t c0 = rr.a0 >> 4;
    const uint64_t c1 = (rr.a0 + rr.len + 15) >> 4;
    return (uint32_t)(c1 - c0);
}

template <int G, int U>
__device__ __forceinline__ void load_step(uint4 (&v)[U], const RecRef& rr, uint32_t nch,
                                          uint32_t step, int lane) {
    const uint4* base = reinterpret_cast<const uint4*>(rr.a0 & ~15ull);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t k = step * (G * U) + u * G + lane;
        v[u] = (k < nch) ? base[k] : make_uint4(0u, 0u, 0u, 0u);
    }
}

template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t v) {
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, G);
    return v;
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Store a big-endian u16 at any byte alignment.
__device__ __forceinline__ void store_be16(uint8_t* q, uint32_t v) {
    if (((uintptr_t)q & 1u) == 0) {
        *reinterpret_cast<uint16_t*>(q) = (uint16_t)bswap16(v);
    } else {
        q[0] = (uint8_t)(v >> 8);
        q[1] = (uint8_t)v;
    }
}

// MODE_DATA: checksum::data over [0, len).  MODE_EMIT / MODE_VERIFY: the protocol gates.
template <int G, int U, int MODE, bool IMPLICIT>
__global__ __launch_bounds__(256) void csum_kernel(KParams p) {
    constexpr int GPB = 256 / G;
    static_assert(G >= 16 && G <= 64 && (G & (G - 1)) == 0, "group size");
    __shared__ uint4 win[GPB][WIN_BYTES / 16];

    const int lane = (int)(threadIdx.x % G);
    const int gib = (int)(threadIdx.x / G);
    const uint64_t ngroups = (uint64_t)gridDim.x * GPB;
    uint64_t r = (uint64_t)blockIdx.x * GPB + gib;
    if (r >= p.n) return;

    const uint8_t* winb = reinterpret_cast<const uint8_t*>(&win[gib][0]);

    RecRef cur = rec_at<IMPLICIT>(p, r);
    RecRef nxt = {};
    if (r + ngroups < p.n) nxt = rec_at<IMPLICIT>(p, r + ngroups);
    uint32_t nch = n_chunks(cur);
    uint32_t step = 0;

    uint4 va[U], vb[U];
    load_step<G, U>(va, cur, nch, 0, lane);

    // per-record state
    Geom g = {};
    int s0 = 0, s1 = 0;        // summed span, relative to the record start
    uint32_t acc = 0, acc2 = 0; // protocol: aligned-word sum; data: even / odd byte sums

    while (true) {
        const uint32_t nsteps = nch == 0 ? 1u : (nch + (G * U) - 1) / (G * U);
        const bool last = step + 1 >= nsteps;
        const uint64_t r2 = last ? r + ngroups : r;
        const bool have2 = r2 < p.n;
        RecRef rec2 = last ? nxt : cur;
        const uint32_t nch2 = last ? n_chunks(nxt) : nch;
        const uint32_t step2 = last ? 0u : step + 1;
        if (have2) load_step<G, U>(vb, rec2, nch2, step2, lane);
        RecRef nxt2 = nxt;
        if (last && have2 && r2 + ngroups < p.n) nxt2 = rec_at<IMPLICIT>(p, r2 + ngroups);

        const uint32_t head = (uint32_t)(cur.a0 & 15u);
        if (step == 0) {
            acc = 0;
            acc2 = 0;
            if (MODE == MODE_DATA) {
                s0 = 0;
                s1 = (int)cur.len;
            } else {
                if (lane < WIN_BYTES / 16 && (uint32_t)lane < nch) win[gib][lane] = va[0];
                wave_lds_sync();
                const uint8_t* recp = reinterpret_cast<const uint8_t*>(cur.a0);
                auto rd = [&](uint32_t o) -> uint32_t {
                    const uint32_t w = head + o;
                    return w < (uint32_t)WIN_BYTES ? (uint32_t)winb[w] : (uint32_t)recp[o];
                };
                g = parse_geometry(rd, cur.len, cur.kind);
                if (g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED)) {
                    s0 = (int)g.l4_off;
                    s1 = (int)g.span_end;
                } else {
                    s0 = 0;
                    s1 = 0;
                }
            }
        }

        // ---- sum this step's chunks over [s0, s1) ----
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = step * (G * U) + u * G + lane;
            const int pos = (int)(16u * k) - (int)head;  // chunk start relative to the record
            if (k < nch && pos < s1 && pos + 16 > s0) {
                uint32_t w[4] = {va[u].x, va[u].y, va[u].z, va[u].w};
                if (pos < s0 || pos + 16 > s1) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) w[j] = mask_dword(w[j], s0 - pos - 4 * j, s1 - pos - 4 * j);
                }
                if (MODE == MODE_DATA) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        acc = add_even_bytes(w[j], acc);
                        acc2 = add_odd_bytes(w[j], acc2);
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc = add_words(w[j], acc);
                }
            }
        }

        if (last) {
            const bool odd = (cur.a0 & 1u) != 0;
            if (MODE == MODE_DATA) {
                // exact little-endian word sum relative to the span start, modulo 2^32
                const uint32_t s_rel = odd ? (acc2 + (acc << 8)) : (acc + (acc2 << 8));
                const uint32_t tot = group_sum<G>(s_rel);
                if (lane == 0) p.out16[r] = (uint16_t)bswap16(fold32(tot));
            } else {
                const uint8_t* recp = reinterpret_cast<const uint8_t*>(cur.a0);
                auto rd = [&](uint32_t o) -> uint32_t {
                    const uint32_t w = head + o;
                    return w < (uint32_t)WIN_BYTES ? (uint32_t)winb[w] : (uint32_t)recp[o];
                };
                auto be16 = [&](uint32_t o) -> uint32_t { return (rd(o) << 8) | rd(o + 1); };
                // IPv4 header words and pseudo-header address words, spread over the group
                uint32_t hsum = 0, psum = 0;
                if (g.fam == 4) {
                    for (uint32_t i = lane; i < g.ip_hl / 2; i += G)
                        if (!(MODE == MODE_EMIT && i == 5)) hsum += be16(g.ip_off + 2 * i);
                }
                const bool l4 = g.proto != P_NONE && !(g.st & SMOL_ST_MALFORMED);
                const bool pseudo = l4 && (g.proto == P_UDP || g.proto == P_TCP || g.proto == P_ICMP6);
                if (pseudo) {
                    for (uint32_t i = lane; i < g.addr_words; i += G) psum += be16(g.addr_off + 2 * i);
                }
                const uint32_t tot = group_sum<G>(acc);
                hsum = group_sum<G>(hsum);
                psum = group_sum<G>(psum);
                if (lane == 0) {
                    uint8_t* wrec = const_cast<uint8_t*>(recp);
                    uint32_t st = g.st;
                    // IPv4 header: data(header) (canonical fold of the big-endian word sum)
                    uint32_t ip_valid = 1, ip_ok = 1;
                    if (g.fam == 4) {
                        const uint32_t hdr = fold32(hsum);
                        if (MODE == MODE_EMIT) {
                            store_be16(wrec + g.ip_off + 10, caps_tx(p.caps_ipv4) ? (~hdr & 0xffffu) : 0u);
                        } else {
                            ip_valid = hdr == 0xffffu;
                            ip_ok = caps_rx(p.caps_ipv4) ? ip_valid : 1u;
                        }
                    }
                    uint32_t l4_valid = 1, l4_ok = 1, partial = 0;
                    if (l4) {
                        const uint32_t fpos = g.l4_off + g.fo;
                        const uint32_t field = be16(fpos);
                        uint32_t s = tot;
                        if (MODE == MODE_EMIT) {
                            // the reference zeroes the field before summing: remove its bytes
                            // (field offset is even relative to the record, so the parity of
                            // its absolute address is the record start's)
                            const uint32_t f0 = field >> 8, f1 = field & 0xffu;
                            s -= odd ? ((f0 << 8) + f1) : (f0 + (f1 << 8));
                        }
                        const uint32_t f = fold32(s);
                        const uint32_t dat = odd ? f : bswap16(f);  // == checksum::data(span)
                        uint32_t ph = 0, gate_caps = SMOL_CHECKSUM_NONE;
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
                            store_be16(wrec + fpos, fill ? c : 0u);
                        } else {
                            l4_valid = comb == 0xffffu;
                            if (g.proto == P_UDP && field == 0) l4_valid = 1;  // udp.rs:138-140
                            if (g.proto == P_UDP || g.proto == P_TCP) partial = ph == field;
                            l4_ok = caps_rx(gate_caps) ? l4_valid : 1u;
                        }
                    }
                    if (MODE == MODE_EMIT) {
                        if (p.status) p.status[r] = (uint8_t)st;
                    } else {
                        const bool mal = (st & SMOL_ST_MALFORMED) != 0;
                        st |= (ip_ok ? SMOL_ST_IP_OK : 0u) | (l4_ok ? SMOL_ST_L4_OK : 0u) |
                              (partial ? SMOL_ST_L4_PARTIAL : 0u) | (ip_valid ? SMOL_ST_IP_VALID : 0u) |
                              (l4_valid ? SMOL_ST_L4_VALID : 0u) |
                              ((ip_ok && l4_ok && !mal) ? SMOL_ST_ACCEPT : 0u);
                        p.status[r] = (uint8_t)st;
                    }
                }
            }
        }

        if (!have2) break;
#pragma unroll
        for (int u = 0; u < U; ++u) va[u] = vb[u];
        if (last) {
            cur = nxt;
            nxt = nxt2;
            nch = nch2;
            r = r2;
        }
        step = step2;
    }
}

// ---------------------------------------------------------------------------------------------
// Launch table
// ---------------------------------------------------------------------------------------------

template <int G, int U, int MODE, bool IMPLICIT>
static hipError_t launch_one(const KParams& p, uint32_t max_blocks, hipStream_t s) {
    constexpr uint32_t GPB = 256 / G;
    const uint64_t want = (p.n + GPB - 1) / GPB;
    const uint32_t blocks = (uint32_t)(want < max_blocks ? want : max_blocks);
    hipLaunchKernelGGL((csum_kernel<G, U, MODE, IMPLICIT>), dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

template <int MODE, bool IMPLICIT>
static hipError_t launch_cfg(int cfg, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    switch (cfg) {
        case CFG_G16U2: return launch_one<16, 2, MODE, IMPLICIT>(p, max_blocks, s);
        case CFG_G32U3: return launch_one<32, 3, MODE, IMPLICIT>(p, max_blocks, s);
        case CFG_G64U2: return launch_one<64, 2, MODE, IMPLICIT>(p, max_blocks, s);
        default: return launch_one<64, 4, MODE, IMPLICIT>(p, max_blocks, s);
    }
}

hipError_t launch_csum(int mode, int cfg, const KParams& p, uint32_t max_blocks, hipStream_t s) {
    const bool implicit = p.desc == nullptr;
    switch (mode) {
        case MODE_DATA:
            return implicit ? launch_cfg<MODE_DATA, true>(cfg, p, max_blocks, s)
                            : launch_cfg<MODE_DATA, false>(cfg, p, max_blocks, s);
        case MODE_EMIT:
            return implicit ? launch_cfg<MODE_EMIT, true>(cfg, p, max_blocks, s)
                            : launch_cfg<MODE_EMIT, false>(cfg, p, max_blocks, s);
        default:
            return implicit ? launch_cfg<MODE_VERIFY, true>(cfg, p, max_blocks, s)
                            : launch_cfg<MODE_VERIFY, false>(cfg, p, max_blocks, s);
    }
}

}  // namespace smolcsum
