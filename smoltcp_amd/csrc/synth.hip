// Synthetic packet batches and single-bit fault injection, generated on the device
// (tooling for tests and bench.py; see include/smolcsum_tools.h).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/smolcsum_tools.h"
#include "csum_launch.h"

namespace smolcsum {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ uint64_t rnd(uint64_t seed, uint64_t i, uint64_t k) {
    return splitmix64(seed * 0x100000001B3ull ^ (i * 0x9E3779B97F4A7C15ull) ^ (k << 56));
}

__device__ __forceinline__ int be16_byte(uint32_t v, uint32_t o) {  // o = 0 (hi) / 1 (lo)
    return (int)((o == 0 ? (v >> 8) : v) & 0xffu);
}

// Header byte of an IPv4 + (UDP|TCP) packet of total length L at offset o (relative to the
// IPv4 header), or -1 past the header.
__device__ int ipv4_l4_byte(uint32_t proto, uint64_t seed, uint64_t i, uint32_t L, uint32_t o) {
    if (o < 20) {
        switch (o) {
            case 0: return 0x45;
            case 1: return 0;
            case 2: case 3: return be16_byte(L, o - 2);
            case 4: case 5: return be16_byte((uint32_t)(i & 0xffff), o - 4);
            case 6: return 0x40;  // DF
            case 7: return 0;
            case 8: return 64;
            case 9: return (int)proto;
            case 10: case 11: return 0;
            default: {
                const uint64_t a = rnd(seed, i, 1);
                return (int)((a >> (8 * (o - 12))) & 0xff);  // src 12..15, dst 16..19
            }
        }
    }
    const uint32_t t = o - 20;
    const uint64_t pr = rnd(seed, i, 3);
    if (proto == 17) {
        if (t < 8) {
            switch (t) {
                case 0: case 1: return be16_byte((uint32_t)(pr & 0xffff), t);
                case 2: case 3: return be16_byte((uint32_t)((pr >> 16) & 0xffff) | 1u, t - 2);
                case 4: case 5: return be16_byte(L - 20, t - 4);
                default: return 0;
            }
        }
        return -1;
    }
    if (t < 20) {  // TCP
        if (t < 4) return t < 2 ? be16_byte((uint32_t)(pr & 0xffff) | 1u, t) : be16_byte((uint32_t)((pr >> 16) & 0xffff) | 1u, t - 2);
        if (t < 12) return (int)((rnd(seed, i, 4) >> (8 * (t - 4))) & 0xff);  // seq, ack
        switch (t) {
            case 12: return 0x50;  // data offset 5
            case 13: return 0x18;  // ACK | PSH
            case 14: case 15: return be16_byte((uint32_t)((pr >> 32) & 0xffff), t - 14);
            default: return 0;     // checksum, urgent pointer
        }
    }
    return -1;
}

__device__ int ipv6_l4_byte(uint64_t seed, uint64_t i, uint32_t L, uint32_t o) {
    const uint32_t kinds[3] = {6, 17, 58};
    const uint32_t nh = kinds[i % 3];
    if (o < 40) {
        switch (o) {
            case 0: return 0x60;
            case 1: case 2: case 3: return 0;
            case 4: case 5: return be16_byte(L - 40, o - 4);
            case 6: return (int)nh;
            case 7: return 64;
            default: {
                const uint32_t a = o - 8;  // 0..31: src then dst
                return (int)((rnd(seed, i, 5 + a / 8) >> (8 * (a % 8))) & 0xff);
            }
        }
    }
    const uint32_t t = o - 40;
    const uint64_t pr = rnd(seed, i, 3);
    if (nh == 17) {
        if (t >= 8) return -1;
        switch (t) {
            case 0: case 1: return be16_byte((uint32_t)(pr & 0xffff), t);
            case 2: case 3: return be16_byte((uint32_t)((pr >> 16) & 0xffff) | 1u, t - 2);
            case 4: case 5: return be16_byte(L - 40, t - 4);
            default: return 0;
        }
    }
    if (nh == 58) {
        if (t >= 8) return -1;
        switch (t) {
            case 0: return 128;  // echo request
            case 1: case 2: case 3: return 0;
            default: return (int)((pr >> (8 * t)) & 0xff);
        }
    }
    if (t >= 20) return -1;
    if (t < 4) return t < 2 ? be16_byte((uint32_t)(pr & 0xffff) | 1u, t) : be16_byte((uint32_t)((pr >> 16) & 0xffff) | 1u, t - 2);
    if (t < 12) return (int)((rnd(seed, i, 4) >> (8 * (t - 4))) & 0xff);
    switch (t) {
        case 12: return 0x50;
        case 13: return 0x18;
        case 14: case 15: return be16_byte((uint32_t)((pr >> 32) & 0xffff), t - 14);
        default: return 0;
    }
}

__device__ int header_byte(uint32_t profile, uint64_t seed, uint64_t i, uint32_t L, uint32_t o) {
    switch (profile) {
        case SMOL_SYNTH_UDP4: return ipv4_l4_byte(17, seed, i, L, o);
        case SMOL_SYNTH_TCP4: return ipv4_l4_byte(6, seed, i, L, o);
        case SMOL_SYNTH_V6MIX: return ipv6_l4_byte(seed, i, L, o);
        case SMOL_SYNTH_ETH_TCP4:
            if (o < 12) return (int)((rnd(seed, i, 9 + o / 6) >> (8 * (o % 6))) & 0xff) & (o == 0 || o == 6 ? 0xfe : 0xff);
            if (o == 12) return 0x08;
            if (o == 13) return 0x00;
            return L >= 14 ? ipv4_l4_byte(6, seed, i, L - 14, o - 14) : -1;
        default: return -1;
    }
}

// One wavefront per record; lanes store consecutive bytes (64 contiguous bytes per store).
__global__ __launch_bounds__(256) void synth_kernel(SynthParams p) {
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const int lane = threadIdx.x & 63;
    for (uint64_t i = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64; i < p.n; i += nw) {
        uint64_t off;
        uint32_t L;
        if (p.desc) {
            off = p.desc[i].offset;
            L = p.desc[i].len;
        } else {
            off = i * p.stride;
            L = p.len;
        }
        uint8_t* rec = p.buf + off;
        for (uint32_t o = lane; o < L; o += 64) {
            int b = header_byte(p.profile, p.seed, i, L, o);
            if (b < 0) {
                const uint64_t pos = off + o;
                b = (int)((splitmix64(p.seed ^ (pos >> 3) * 0xD6E8FEB86659FD93ull) >> (8 * (pos & 7))) & 0xff);
            }
            rec[o] = (uint8_t)b;
        }
    }
}

__device__ __forceinline__ uint32_t xorshift32(uint32_t& s) {  // fault_injector.rs:8-16
    uint32_t x = s;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    s = x;
    return x;
}

__global__ void corrupt_kernel(SynthParams p, uint32_t every) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j * every < p.n; j += stride) {
        const uint64_t i = j * every;
        uint64_t off;
        uint32_t L;
        if (p.desc) {
            off = p.desc[i].offset;
            L = p.desc[i].len;
        } else {
            off = i * p.stride;
            L = p.len;
        }
        if (L == 0) continue;
        uint32_t s = (uint32_t)splitmix64(p.seed ^ i) | 1u;
        const uint32_t idx = xorshift32(s) % L;            // fault_injector.rs:48
        const uint32_t bit = 1u << (xorshift32(s) % 8u);   // fault_injector.rs:49
        p.buf[off + idx] ^= (uint8_t)bit;
    }
}

hipError_t launch_synth(const SynthParams& p, uint32_t max_blocks, hipStream_t s) {
    const uint64_t want = (p.n + 3) / 4;
    const uint32_t blocks = grid_blocks(want, max_blocks);
    hipLaunchKernelGGL(synth_kernel, dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_corrupt(const SynthParams& p, uint32_t every, hipStream_t s) {
    const uint64_t cnt = (p.n + every - 1) / every;
    const uint64_t want = (cnt + 255) / 256;
    const uint32_t blocks = (uint32_t)(want < 4096 ? (want ? want : 1) : 4096);
    hipLaunchKernelGGL(corrupt_kernel, dim3(blocks), dim3(256), 0, s, p, every);
    return hipGetLastError();
}

}  // namespace smolcsum

namespace smolcsum {

// Read-only HBM streaming probe (the achievable read ceiling): each wavefront streams contiguous
// 8-KiB pieces (8 non-temporal 16-byte loads per lane in flight, lane-contiguous), grid stride over
// the pieces, then the < 8 KiB tail with a plain grid stride.  Loads are summed into a value stored
// only if it hits an impossible pattern (keeps them live).  tools/probe_bw.hip `wave_spans U8 nt`.
typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void stream_read_kernel(const uint4* p, uint64_t n16, uint32_t* sink) {
    constexpr int UNR = 8;
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint64_t w0 = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const uint64_t per = 64ull * UNR;
    const u32x4s* q = reinterpret_cast<const u32x4s*>(p);
    uint32_t acc = 0;
    for (uint64_t base = w0 * per; base + per <= n16; base += nw * per) {
        u32x4s v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = __builtin_nontemporal_load(q + base + u * 64 + lane);
#pragma unroll
        for (int u = 0; u < UNR; ++u)
            acc += __builtin_amdgcn_sad_u16(v[u].x, 0, 0) + __builtin_amdgcn_sad_u16(v[u].y, 0, 0) +
                   __builtin_amdgcn_sad_u16(v[u].z, 0, 0) + __builtin_amdgcn_sad_u16(v[u].w, 0, 0);
    }
    const uint64_t tail = n16 / per * per;
    for (uint64_t i = tail + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (uint64_t)gridDim.x * blockDim.x)
        acc += p[i].x;
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

hipError_t launch_stream_read(const uint8_t* buf, uint64_t bytes, uint32_t* sink, uint32_t max_blocks,
                              hipStream_t s) {
    hipLaunchKernelGGL(stream_read_kernel, dim3(max_blocks), dim3(256), 0, s,
                       reinterpret_cast<const uint4*>(buf), bytes / 16, sink);
    return hipGetLastError();
}

// Emit's floor probe: the read-only stream above over a batch's bytes, plus what emit writes — two
// big-endian 2-byte stores per record (one when f2 == ~0u) at record offsets f1 / f2 of records
// that start every `stride` bytes, each store issued by the wavefront that streamed the 8-KiB piece
// holding the record's first byte, right after that piece's loads (the stored value depends on
// them).  Reads every byte once at the best streaming pattern and makes exactly emit's scattered
// store events, with no parse and no gates: the time an in-place emit cannot beat
// (tools/probe_wr2.hip).
__device__ __forceinline__ void probe_store(uint8_t* buf, uint64_t bytes, uint64_t a, uint32_t v) {
    if (a + 2 <= bytes) {
        __attribute__((address_space(1))) uint8_t* g = (__attribute__((address_space(1))) uint8_t*)(buf + a);
        g[0] = (uint8_t)(v >> 8);
        g[1] = (uint8_t)v;
    }
}

__global__ __launch_bounds__(256) void field_probe_kernel(uint8_t* buf, uint64_t n16, uint64_t stride, uint32_t f1,
                                                          uint32_t f2) {
    constexpr int UNR = 8;
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint64_t w0 = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const uint64_t per = 64ull * UNR;
    const uint64_t bytes = n16 * 16;
    const u32x4s* q = reinterpret_cast<const u32x4s*>(buf);
    auto stores = [&](uint64_t lo, uint64_t hi, uint32_t acc) {  // records starting in [lo, hi)
        const uint64_t r0 = (lo + stride - 1) / stride;
        for (uint64_t r = r0 + (uint64_t)lane; r * stride < hi; r += 64) {
            probe_store(buf, bytes, r * stride + f1, acc + (uint32_t)r);
            if (f2 != ~0u) probe_store(buf, bytes, r * stride + f2, acc ^ (uint32_t)r);
        }
    };
    for (uint64_t base = w0 * per; base + per <= n16; base += nw * per) {
        u32x4s v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = __builtin_nontemporal_load(q + base + u * 64 + lane);
        uint32_t acc = 0;
#pragma unroll
        for (int u = 0; u < UNR; ++u)
            acc += __builtin_amdgcn_sad_u16(v[u].x, 0, 0) + __builtin_amdgcn_sad_u16(v[u].y, 0, 0) +
                   __builtin_amdgcn_sad_u16(v[u].z, 0, 0) + __builtin_amdgcn_sad_u16(v[u].w, 0, 0);
        stores(16 * base, 16 * (base + per), acc);
    }
    const uint64_t tail = n16 / per * per;
    if (w0 == 0 && tail < n16) {
        uint32_t acc = 0;
        for (uint64_t i = tail + (uint64_t)lane; i < n16; i += 64) acc += q[i].x;
        stores(16 * tail, bytes, acc);
    }
}

// The same probe with the store addresses given as a list (descriptor batches, whose fields do not
// sit at a fixed spacing): addrs[] ascending byte offsets of 2-byte stores, first[j] the index of the
// first address inside the 8-KiB piece j (first[] has ceil(bytes / 8 KiB) + 1 entries).
// seg64: instead, the 64-B segments holding each listed field (both of its bytes) are rewritten
// whole with the values the stream just read: each lane stores those of its 16-B chunks that lie in
// such a segment, from its registers (no reload) — the store shape of whole-segment emit.
__global__ __launch_bounds__(256) void field_probe_list_kernel(uint8_t* buf, uint64_t n16, const uint64_t* addrs,
                                                               const uint32_t* first, int seg64) {
    constexpr int UNR = 8;
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint64_t w0 = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const uint64_t per = 64ull * UNR;
    const uint64_t bytes = n16 * 16;
    const u32x4s* q = reinterpret_cast<const u32x4s*>(buf);
    typedef __attribute__((address_space(1))) u32x4s* gv4;
    auto stores = [&](uint64_t piece, uint32_t acc) {
        const uint32_t i0 = first[piece], i1 = first[piece + 1];
        for (uint32_t i = i0 + (uint32_t)lane; i < i1; i += 64) probe_store(buf, bytes, addrs[i], acc + i);
    };
    for (uint64_t base = w0 * per; base + per <= n16; base += nw * per) {
        u32x4s v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = __builtin_nontemporal_load(q + base + u * 64 + lane);
        uint32_t acc = 0;
#pragma unroll
        for (int u = 0; u < UNR; ++u)
            acc += __builtin_amdgcn_sad_u16(v[u].x, 0, 0) + __builtin_amdgcn_sad_u16(v[u].y, 0, 0) +
                   __builtin_amdgcn_sad_u16(v[u].z, 0, 0) + __builtin_amdgcn_sad_u16(v[u].w, 0, 0);
        // every piece is read, stores or not: without this the compiler sinks the loads into the
        // store loop
        asm volatile("" ::"v"(acc));
        if (seg64) {
            const uint64_t piece = base / per;
            const uint32_t i0 = first[piece], i1 = first[piece + 1];
            // a segment of this piece holds a field when one of the listed offsets (or the byte after
            // it) falls in it; the piece's offsets are few (C2: about 11 per 8 KiB)
            uint32_t hit = 0;  // bit u: chunk u of this lane lies in a field segment
            for (uint32_t i = i0; i < i1; ++i) {
                const uint64_t a = addrs[i];
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    const uint64_t sgm = (16ull * (base + u * 64 + lane)) & ~63ull;
                    if ((a & ~63ull) == sgm || ((a + 1) & ~63ull) == sgm) hit |= 1u << u;
                }
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                u32x4s x = v[u];
                asm volatile("" : "+v"(x));  // opaque: the stored values are the ones just read
                if (hit & (1u << u)) ((gv4)buf)[base + u * 64 + lane] = x;
            }
        } else {
            stores(base / per, acc);
        }
    }
    const uint64_t tail = n16 / per * per;
    if (w0 == 0 && tail < n16) {
        uint32_t acc = 0;
        for (uint64_t i = tail + (uint64_t)lane; i < n16; i += 64) acc += q[i].x;
        if (!seg64) stores(tail / per, acc);
    }
}

hipError_t launch_field_probe_list(uint8_t* buf, uint64_t bytes, const uint64_t* addrs, const uint32_t* first,
                                   int seg64, uint32_t max_blocks, hipStream_t s) {
    hipLaunchKernelGGL(field_probe_list_kernel, dim3(max_blocks), dim3(256), 0, s, buf, bytes / 16, addrs, first, seg64);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void field_scatter_kernel(uint8_t* buf, uint64_t bytes, const uint64_t* addrs,
                                                            const uint16_t* vals, uint64_t n, int nt) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = addrs[i];
    const uint32_t v = vals[i];
    if (a + 2 > bytes) return;
    __attribute__((address_space(1))) uint8_t* g = (__attribute__((address_space(1))) uint8_t*)(buf + a);
    if (nt & 14) {  // the aligned 64-B segment (bit 1), 32-B sector (bit 2) or 128-B line (bit 3) holding
                    // the field, written whole (timing probe: v repeated)
        const uint64_t sz = (nt & 2) ? 64 : (nt & 4) ? 32 : 128;
        const uint64_t s0 = a & ~(sz - 1);
        if (s0 + sz > bytes) return;
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const uint32_t w = v * 0x10001u;
        const u32x4 x = {w, w, w, w};
        for (uint64_t k = 0; k < sz / 16; ++k) *(__attribute__((address_space(1))) u32x4*)(buf + s0 + 16 * k) = x;
        return;
    }
    if (nt) {
        __builtin_nontemporal_store((uint8_t)(v >> 8), g);
        __builtin_nontemporal_store((uint8_t)v, g + 1);
    } else {
        g[0] = (uint8_t)(v >> 8);
        g[1] = (uint8_t)v;
    }
}

hipError_t launch_field_scatter(uint8_t* buf, uint64_t bytes, const uint64_t* addrs, const uint16_t* vals, uint64_t n,
                                int nt, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(field_scatter_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, buf, bytes, addrs,
                       vals, n, nt);
    return hipGetLastError();
}

// Emit's floor in emit's own store shape (round 6): the read-only stream above over the buffer, and
// every 64-B segment that holds a checksum field written back whole, with the bytes just read (nothing
// changes), by the lanes that loaded it, right after the piece's loads.  bitmap: one bit per 64-B
// segment of the buffer (bit s % 32 of word s / 32), set for the segments emit writes.  An 8-KiB piece
// is 128 segments = 4 bitmap words, read as one uniform (scalar) load; lane l's chunk of load u lies
// in segment 16 u + l / 4 of the piece.  nt: the segments stored non-temporal (emit's form for packed
// 1400-1580-B records, csum_api.cpp xwalk_auto).  The tail past the last whole piece is read, not
// written.
template <bool NT>
__global__ __launch_bounds__(256) void segment_probe_kernel(uint8_t* buf, uint64_t n16, const uint32_t* bitmap) {
    constexpr int UNR = 8;
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint64_t w0 = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const uint64_t per = 64ull * UNR;
    const u32x4s* q = reinterpret_cast<const u32x4s*>(buf);
    typedef __attribute__((address_space(1))) u32x4s* gv4;
    uint32_t acc = 0;
    for (uint64_t base = w0 * per; base + per <= n16; base += nw * per) {
        u32x4s v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = __builtin_nontemporal_load(q + base + u * 64 + lane);
        const uint64_t piece = base / per;
        uint32_t bits[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) bits[k] = bitmap[4 * piece + k];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            acc += __builtin_amdgcn_sad_u16(v[u].x, 0, 0) + __builtin_amdgcn_sad_u16(v[u].w, 0, 0);
            if ((bits[u >> 1] >> (16 * (u & 1) + lane / 4)) & 1u) {
                u32x4s x = v[u];
                asm volatile("" : "+v"(x));  // opaque: the stored values are the ones just read
                if constexpr (NT) __builtin_nontemporal_store(x, (gv4)buf + base + u * 64 + lane);
                else ((gv4)buf)[base + u * 64 + lane] = x;
            }
        }
    }
    const uint64_t tail = n16 / per * per;
    for (uint64_t i = tail + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        acc += q[i].x;
    asm volatile("" ::"v"(acc));  // keeps every load live
}

hipError_t launch_segment_probe(uint8_t* buf, uint64_t bytes, const uint32_t* bitmap, int nt, uint32_t max_blocks,
                                hipStream_t s) {
    if (nt) hipLaunchKernelGGL((segment_probe_kernel<true>), dim3(max_blocks), dim3(256), 0, s, buf, bytes / 16, bitmap);
    else hipLaunchKernelGGL((segment_probe_kernel<false>), dim3(max_blocks), dim3(256), 0, s, buf, bytes / 16, bitmap);
    return hipGetLastError();
}

hipError_t launch_field_probe(uint8_t* buf, uint64_t bytes, uint64_t stride, uint32_t f1, uint32_t f2,
                              uint32_t max_blocks, hipStream_t s) {
    hipLaunchKernelGGL(field_probe_kernel, dim3(max_blocks), dim3(256), 0, s, buf, bytes / 16, stride, f1, f2);
    return hipGetLastError();
}

}  // namespace smolcsum
