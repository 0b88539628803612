// IPv4 fragment groups: smol_csum_batch_emit_frag / smol_csum_batch_verify_frag (include/smolcsum.h).
//
// Under offloaded checksums smoltcp emits a datagram that exceeds the MTU whole — its L4 checksum
// written 0 by the ignored caps — and only then cuts it into fragments, each handed to
// TxToken::consume on its own (src/iface/interface/mod.rs:1276-1331, src/iface/interface/ipv4.rs:
// 440-490).  On receive it reassembles the fragment payloads and runs the L4 gate on the whole
// payload (ipv4.rs:103-146).  A device that holds a datagram's fragments until the last one arrives
// can do both: one wavefront per group of fragments.
//
//   1. lane j parses fragment j's IPv4 header (Ipv4Packet::check_len, the reassembly key, the
//      payload range [frag_offset, frag_offset + total_len - hl)) and fills / verifies that header;
//   2. the wavefront checks the group contract: one key, non-empty payloads that cover [0, T)
//      exactly once (unique starts, one starting at 0, every end but T meets a start, lengths sum to
//      T) with exactly one last fragment (MF clear) ending at T;
//   3. the L4 header is read through the datagram map (datagram offset -> the fragment holding it);
//   4. the 64 lanes sum each fragment's payload slice as aligned 16-byte chunks (v_sad_u16, the
//      bytes outside the slice and, on emit, the checksum fields masked), and every fragment's sum
//      becomes its data() value: a payload starts at an even datagram offset (a multiple of 8), so
//      data() of the datagram is the one's-complement sum of the fragments' data() values;
//   5. lane 0 applies the same gates as finish_gates (csum_walk.h) and writes the field bytes where
//      the map puts them; every lane writes its fragments' status bytes.
//
// This is the rare path (fragmented datagrams), written for exactness, not for the HBM roofline:
// one wavefront walks a datagram's fragments one after the other.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csum_device.h"
#include "csum_launch.h"

namespace smolcsum {
namespace frag {

constexpr uint32_t MAXF = SMOL_MAX_FRAGMENTS;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GMEM __attribute__((address_space(1)))
typedef const GMEM uint8_t* gcu8;
typedef GMEM uint8_t* gu8;
typedef const GMEM u32x4* gcv4;

__device__ __forceinline__ uint32_t rb(uint64_t a) { return *(gcu8)a; }
__device__ __forceinline__ uint32_t rb16(uint64_t a) { return (rb(a) << 8) | rb(a + 1); }

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int m = 32; m; m >>= 1) v += (uint32_t)__shfl_xor((int)v, m, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int m = 32; m; m >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, m, 64));
    return v;
}
__device__ __forceinline__ bool wave_any(bool b) { return __ballot(b) != 0; }

__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Zero byte x (absolute address) of the 16-byte chunk at ca, if it lies there.
__device__ __forceinline__ void mask_byte(u32x4& c, uint64_t ca, uint64_t x) {
    if (x < ca || x >= ca + 16) return;
    const uint32_t o = (uint32_t)(x - ca), m = ~(0xffu << (8 * (o & 3)));
    switch (o >> 2) {
        case 0: c.x &= m; break;
        case 1: c.y &= m; break;
        case 2: c.z &= m; break;
        default: c.w &= m; break;
    }
}

template <int MODE, bool IMPLICIT>
__global__ __launch_bounds__(64) void frag_kernel(KParams p, const smol_csum_frag_group_t* groups, uint64_t ngroups) {
    constexpr bool EMIT = MODE == MODE_EMIT;
    __shared__ uint64_t s_addr[MAXF];  // payload start address of fragment j
    __shared__ uint32_t s_start[MAXF], s_end[MAXF];
    __shared__ uint8_t s_bits[MAXF];   // bit 0 check_len ok, 1 MF, 2 IP gate passed, 3 header valid
    const int lane = (int)threadIdx.x;

    for (uint64_t gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
        const uint64_t first = groups[gi].first;
        const uint32_t count = groups[gi].count;
        // an invalid group (outside the batch, count 0 or > SMOL_MAX_FRAGMENTS, reserved != 0) is
        // not read or written at all (include/smolcsum.h)
        if (first >= p.n || count == 0 || count > MAXF || count > p.n - first || groups[gi].reserved != 0) continue;

        // ---- 1. the fragments' IPv4 headers ----
        // record j of the group: address, length, SMOL_KIND_* (+ KIND_IPHDR_ONLY for a raw frame)
        auto rec = [&](uint32_t j, uint64_t& a0, uint32_t& len, uint32_t& kind) {
            const uint64_t r = first + j;
            if (IMPLICIT) {
                a0 = (uint64_t)p.buf + r * p.stride;
                len = p.len;
                kind = p.kind;
            } else {
                const u32x4 d = *(gcv4)((uint64_t)p.desc + 16 * r);
                a0 = (uint64_t)p.buf + ((uint64_t)d.x | ((uint64_t)d.y << 32));
                len = d.z;
                kind = desc_kind(d.w);
            }
        };
        // fragment 0's reassembly key (ipv4.rs get_key: ident, src, dst, protocol) and addresses
        uint64_t k0a = 0;
        bool k0ok = false;
        {
            uint64_t a0;
            uint32_t len, kind;
            rec(0, a0, len, kind);
            kind &= 0xffu;
            const uint32_t io = kind == SMOL_KIND_ETH ? 14u : 0u;
            if ((kind == SMOL_KIND_IP || kind == SMOL_KIND_ETH) && len >= io + 20) {
                k0a = a0 + io;
                k0ok = true;
            }
        }
        bool bad = !k0ok, raw = false;
        uint32_t T = 0, sumlen = 0, lastn = 0;
        for (uint32_t j = (uint32_t)lane; j < count; j += 64) {
            uint64_t a0;
            uint32_t len, kind;
            rec(j, a0, len, kind);
            raw = raw || (kind & KIND_IPHDR_ONLY) != 0;  // a raw socket's datagram: headers only
            kind &= 0xffu;
            uint32_t io = 0, ok = 0, hl = 0, total = 0, start = 0, end = 0, mf = 0;
            if (kind == SMOL_KIND_ETH) {
                io = 14;
                ok = len >= 14 && rb16(a0 + 12) == 0x0800u;
            } else {
                ok = kind == SMOL_KIND_IP;
            }
            const uint64_t ip = a0 + io;
            if (ok) ok = len - io >= 20 && (rb(ip) >> 4) == 4;
            if (ok) {
                hl = (rb(ip) & 0x0fu) * 4;
                total = rb16(ip + 2);
                const uint32_t lb = len - io;
                ok = !(lb < hl || hl > total || lb < total || hl < 20);  // Ipv4Packet::check_len
            }
            uint32_t bits = 0xcu;  // IP gate / header: passed unless verified and found bad
            if (ok) {
                const uint32_t fl = rb16(ip + 6);
                start = (fl & 0x1fffu) * 8;  // Ipv4Packet::frag_offset, ipv4.rs:319-322
                end = start + total - hl;
                mf = (fl >> 13) & 1u;
                bool same = k0ok && rb(ip + 9) == rb(k0a + 9) && rb16(ip + 4) == rb16(k0a + 4);
                for (uint32_t b = 12; b < 20; ++b) same = same && rb(ip + b) == rb(k0a + b);
                bad = bad || !same || end <= start;
                T = max(T, end);
                sumlen += end - start;
                lastn += mf ? 0u : 1u;
                // the fragment's own header: fill (dispatch_ipv4_frag, ipv4.rs:482-484) or verify
                uint32_t hs = 0;
                for (uint32_t w = 0; w < hl / 2; ++w)
                    if (!(EMIT && w == 5)) hs += rb16(ip + 2 * w);
                const uint32_t hdr = fold32(hs);
                if (EMIT) {
                    const uint32_t v = caps_tx(p.caps_ipv4) ? (~hdr & 0xffffu) : 0u;
                    ((gu8)ip)[10] = (uint8_t)(v >> 8);
                    ((gu8)ip)[11] = (uint8_t)v;
                } else {
                    const uint32_t valid = hdr == 0xffffu;
                    const uint32_t okg = caps_rx(p.caps_ipv4) ? valid : 1u;
                    bits = (okg ? 4u : 0u) | (valid ? 8u : 0u);
                }
            } else {
                bad = true;  // no IPv4 header checked: its IP bits stay set, the record is MALFORMED
            }
            s_addr[j] = ip + hl;
            s_start[j] = start;
            s_end[j] = end;
            s_bits[j] = (uint8_t)(bits | (mf << 1) | (ok ? 1u : 0u));
        }
        lds_sync();
        T = wave_max(T);
        sumlen = wave_sum(sumlen);
        lastn = wave_sum(lastn);
        bad = wave_any(bad);
        raw = wave_any(raw);

        // ---- 2. the group contract ----
        bool broken = bad || lastn != 1 || sumlen != T;
        uint32_t zeros = 0;
        for (uint32_t j = (uint32_t)lane; !broken && j < count; j += 64) {
            const uint32_t sj = s_start[j], ej = s_end[j];
            uint32_t starts = 0, next = 0;
            for (uint32_t i = 0; i < count; ++i) {
                starts += s_start[i] == sj;
                next += s_start[i] == ej;
            }
            zeros += sj == 0;
            if (starts != 1 || (ej != T && next != 1) || (!(s_bits[j] & 2u) && ej != T)) broken = true;
        }
        broken = wave_any(broken) || wave_sum(zeros) != 1;

        // ---- 3. the L4 header through the datagram map ----
        auto dg_addr = [&](uint32_t o) -> uint64_t {
            for (uint32_t i = 0; i < count; ++i)
                if (s_start[i] <= o && o < s_end[i]) return s_addr[i] + (o - s_start[i]);
            return 0;
        };
        auto dg = [&](uint32_t o) -> uint32_t { return rb(dg_addr(o)); };
        uint32_t proto = P_NONE, st = 0, span_end = 0, fo = 0, in_hl = 0;
        if (broken) {
            st = SMOL_ST_MALFORMED;
        } else if (raw) {
            st = SMOL_ST_UNSUPPORTED;
        } else {
            const uint32_t pr = rb(k0a + 9);
            if (pr == P_UDP) {
                fo = 6;
                const uint32_t ul = T >= 8 ? (dg(4) << 8 | dg(5)) : 0u;
                if (T < 8 || T < ul || ul < 8) st = SMOL_ST_MALFORMED;
                else if (!EMIT && (dg(2) | dg(3)) == 0) st = SMOL_ST_MALFORMED;  // udp.rs:246-248
                span_end = ul;
            } else if (pr == P_TCP) {
                fo = 16;
                const uint32_t thl = T >= 20 ? (dg(12) >> 4) * 4 : 0u;
                if (T < 20 || T < thl || thl < 20) st = SMOL_ST_MALFORMED;
                else if (!EMIT && ((dg(0) | dg(1)) == 0 || (dg(2) | dg(3)) == 0)) st = SMOL_ST_MALFORMED;  // tcp.rs:910-915
                span_end = T;
            } else if (pr == P_ICMP4 || pr == P_IGMP) {
                fo = 2;
                if (T < 8) st = SMOL_ST_MALFORMED;
                span_end = T;
                if (EMIT && pr == P_ICMP4 && T >= 28) {
                    const uint32_t t = dg(0), v = dg(8);
                    if ((t == 3 || t == 11) && (v >> 4) == 4 && (v & 0x0fu) * 4 >= 20 && 8 + (v & 0x0fu) * 4 <= T)
                        in_hl = (v & 0x0fu) * 4;
                }
            } else {
                st = SMOL_ST_UNSUPPORTED;
            }
            if (!st) proto = pr;
        }

        // ---- 4. the payload sum: data() per fragment slice, one's-complement sum over slices ----
        uint32_t l4_valid = 1, l4_ok = 1, partial = 0;
        if (proto != P_NONE) {
            const uint64_t f0 = EMIT ? dg_addr(fo) : 0, f1 = EMIT ? dg_addr(fo + 1) : 0;
            const uint64_t i0 = in_hl ? dg_addr(18) : 0, i1 = in_hl ? dg_addr(19) : 0;
            uint32_t D = 0;
            for (uint32_t j = 0; j < count; ++j) {
                const uint32_t lo = s_start[j], hi = min(s_end[j], span_end);
                if (hi <= lo) continue;
                const uint64_t A = s_addr[j], B = A + (hi - lo);
                const uint64_t base = A & ~15ull;
                const uint32_t nch = (uint32_t)(((B + 15) >> 4) - (base >> 4));
                uint32_t acc = 0;
                for (uint32_t k = (uint32_t)lane; k < nch; k += 64) {
                    const uint64_t ca = base + 16ull * k;
                    u32x4 c = *(gcv4)ca;
                    const int a = (int)((int64_t)A - (int64_t)ca), b = (int)((int64_t)B - (int64_t)ca);
                    c.x = mask_dword(c.x, a, b);
                    c.y = mask_dword(c.y, a - 4, b - 4);
                    c.z = mask_dword(c.z, a - 8, b - 8);
                    c.w = mask_dword(c.w, a - 12, b - 12);
                    if (EMIT) {  // the reference zeroes the fields before summing
                        mask_byte(c, ca, f0);
                        mask_byte(c, ca, f1);
                        if (in_hl) {
                            mask_byte(c, ca, i0);
                            mask_byte(c, ca, i1);
                        }
                    }
                    acc = add_words(c.x, add_words(c.y, add_words(c.z, add_words(c.w, acc))));
                }
                const uint32_t S = fold32(wave_sum(acc));
                D += (A & 1u) ? S : bswap16(S);  // data() of the slice (csum_device.h)
            }
            uint32_t dat = fold32(D);
            uint32_t vin = 0;
            if (EMIT && in_hl) {
                // Icmpv4Repr::emit writes the embedded IPv4 header under the same caps first
                // (icmpv4.rs:520-543); its field is a BE word at even datagram offset 18
                uint32_t hin = 0;
                for (uint32_t w = 0; w < in_hl / 2; ++w)
                    if (w != 5) hin += dg(8 + 2 * w) << 8 | dg(9 + 2 * w);
                vin = caps_tx(p.caps_ipv4) ? (~fold32(hin) & 0xffffu) : 0u;
                dat = fold32(dat + vin);
            }
            uint32_t ph = 0, psum = 0;
            const bool pseudo = proto == P_UDP || proto == P_TCP;
            if (pseudo) {
                for (uint32_t b = 12; b < 20; b += 2) psum += rb16(k0a + b);
                ph = fold32(psum + proto + ((proto == P_UDP ? span_end : T) & 0xffffu));  // pseudo_header_v4
            }
            const uint32_t comb = pseudo ? fold32(ph + dat) : dat;
            const uint32_t gate = proto == P_UDP ? p.caps_udp : proto == P_TCP ? p.caps_tcp
                                : proto == P_ICMP4 ? p.caps_icmpv4 : (uint32_t)SMOL_CHECKSUM_NONE;
            if (EMIT) {
                if (lane == 0) {
                    uint32_t c = ~comb & 0xffffu;
                    if (proto == P_UDP && c == 0) c = 0xffffu;  // udp.rs:207
                    const uint32_t v = (proto == P_IGMP || caps_tx(gate)) ? c : 0u;
                    ((gu8)f0)[0] = (uint8_t)(v >> 8);
                    ((gu8)f1)[0] = (uint8_t)v;
                    if (in_hl) {
                        ((gu8)i0)[0] = (uint8_t)(vin >> 8);
                        ((gu8)i1)[0] = (uint8_t)vin;
                    }
                }
            } else {
                const uint32_t field = dg(fo) << 8 | dg(fo + 1);
                l4_valid = comb == 0xffffu;
                if (proto == P_UDP && field == 0) l4_valid = 1;  // udp.rs:138-140
                if (pseudo) partial = ph == field;
                l4_ok = caps_rx(gate) ? l4_valid : 1u;
            }
        }

        // ---- 5. status bytes ----
        bool all_ip = true;
        if (!EMIT)
            for (uint32_t j = (uint32_t)lane; j < count; j += 64) all_ip = all_ip && (s_bits[j] & 4u);
        all_ip = !wave_any(!all_ip);
        const bool mal = (st & SMOL_ST_MALFORMED) != 0;
        for (uint32_t j = (uint32_t)lane; j < count; j += 64) {
            const uint32_t bits = s_bits[j];
            uint32_t s = (bits & 1u) ? st : (uint32_t)SMOL_ST_MALFORMED;
            if (!EMIT) {
                s = st | ((bits & 4u) ? SMOL_ST_IP_OK : 0u) | ((bits & 8u) ? SMOL_ST_IP_VALID : 0u) |
                    ((bits & 1u) ? 0u : (uint32_t)SMOL_ST_MALFORMED) |
                    (l4_ok ? SMOL_ST_L4_OK : 0u) | (l4_valid ? SMOL_ST_L4_VALID : 0u) |
                    (partial ? SMOL_ST_L4_PARTIAL : 0u) | ((all_ip && l4_ok && !mal) ? SMOL_ST_ACCEPT : 0u);
            }
            if (p.status) ((gu8)p.status)[first + j] = (uint8_t)s;
        }
        lds_sync();  // the next group's phase 1 rewrites the map
    }
}

}  // namespace frag

hipError_t launch_frag(int mode, const KParams& p, const smol_csum_frag_group_t* groups, uint64_t ngroups,
                       hipStream_t s) {
    const uint32_t blocks = grid_blocks(ngroups, kMaxGridBlocks);
    const bool implicit = p.desc == nullptr;
    if (mode == MODE_EMIT) {
        if (implicit) hipLaunchKernelGGL((frag::frag_kernel<MODE_EMIT, true>), dim3(blocks), dim3(64), 0, s, p, groups, ngroups);
        else hipLaunchKernelGGL((frag::frag_kernel<MODE_EMIT, false>), dim3(blocks), dim3(64), 0, s, p, groups, ngroups);
    } else {
        if (implicit) hipLaunchKernelGGL((frag::frag_kernel<MODE_VERIFY, true>), dim3(blocks), dim3(64), 0, s, p, groups, ngroups);
        else hipLaunchKernelGGL((frag::frag_kernel<MODE_VERIFY, false>), dim3(blocks), dim3(64), 0, s, p, groups, ngroups);
    }
    return hipGetLastError();
}

}  // namespace smolcsum
