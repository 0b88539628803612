// Inline write-tax probe (round 6): what emit's field-segment writes cost when
// they land in the lines the stream itself just read, against the same writes made later.
//
// C2's geometry: n records of L bytes (default 2^20 x 1500) back to back, R = 4 TX buffers and 4 RX
// buffers taken in turn.  Every mode streams its TX buffer the way the transposed walk does (a
// wavefront owns 8 consecutive records and loads their lines as 16 non-temporal 1-KiB buffer-load
// instructions, every line once) and differs only in what it writes, and when:
//   read          nothing (the read-only reference)
//   inline        the 64-B segment(s) holding each record's two checksum fields (record offsets 10..11
//                 and 26..27: emit's 1.25 segments per record), written whole by the record's 8-lane
//                 group right after the wavefront's loads have been summed (emit's own timing);
//                 _nt / _sc: stored non-temporal (emit variant 57's form) / with sc0 sc1
//   inline_2b     two 2-B stores per record at the fields instead (emit's 2-B form)
//   deferred      read, then a separate scatter pass writing the same segments (address order);
//                 _nt / _sc / _scnt: the scatter's store policy
//   pipelined     the stream of TX buffer i writes the segments of TX buffer i - 1 (one batch later)
//   vals_rmw      the stream writes 8 B per record to a compact array; a second pass reads each
//                 segment from the buffer, patches it with them and writes it back whole
//   dense         the stream writes each record's segment(s) to consecutive 64-B slots of a side
//                 array; a second pass copies them into place (_nt: every store non-temporal)
//   scatter       the scatter pass alone (no stream; the r05 write-tax sweep's form at emit's
//                 addresses); _nt: non-temporal
// Each mode is timed alone (K passes over the TX buffers in turn) and in bench.py's step order (mode
// over TX buffer i, then a read-only pass over RX buffer i, like verify), interleaved over rounds.
// Printed per mode: ms per pass, and the write cost over the read-only reference in ps per segment.
// Standalone tool:  ./probe_wtax [n] [L] [rounds]   (results: DESIGN.md §5, profiles/r06_write_tax_inline.jsonl)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)
#define GMEM __attribute__((address_space(1)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

enum { M_READ, M_INLINE, M_INLINE_2B, M_PIPE, M_VALS, M_DENSE };
enum { SRC_CONST, SRC_RMW, SRC_DENSE };

// dense staging: record r's first slot is r + (records before r with two segments); that count is
// periodic in r with period per (= 64 / gcd(L, 64)): pre[k] for k < per, two[per] per period
struct Dense {
    uint32_t per;
    uint32_t pre[65];
};
__device__ __forceinline__ uint64_t dense_slot(const Dense& d, uint64_t r) {
    return r + (r / d.per) * d.pre[d.per] + d.pre[r % d.per];
}

__device__ __forceinline__ uint32_t sum4(const u32x4& v, uint32_t acc) {
    return __builtin_amdgcn_sad_u16(v.x, 0, __builtin_amdgcn_sad_u16(v.y, 0, __builtin_amdgcn_sad_u16(v.z, 0, __builtin_amdgcn_sad_u16(v.w, 0, acc))));
}

// the two segments (a, b; b == a when one holds both fields) of record r
__device__ __forceinline__ void segs(uint64_t r, uint32_t L, uint64_t& a, uint64_t& b) {
    a = (r * L + 10) & ~63ull;
    b = (r * L + 27) & ~63ull;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
    const uint64_t b = (uint64_t)base;
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, 0x7fffffff, 0x00020000);
}

// AUX: the store's cache policy (0 default, 2 nt, 17 sc0 sc1, 19 sc0 sc1 nt)
template <int MODE, int AUX>
__global__ __launch_bounds__(256) void stream_kernel(uint8_t* buf, uint8_t* prev, uint8_t* side, uint64_t n, uint32_t L,
                                                     uint32_t* sink, Dense dn) {
    const int wl = (int)(threadIdx.x & 63);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (uint64_t)wv;
    const uint64_t r0 = w * 8;
    if (r0 >= n) return;
    const uint64_t r1 = r0 + 8 < n ? r0 + 8 : n;
    // lines starting in [b, e): the line holding record r1's first byte belongs to the next wavefront
    const uint64_t b = ((uint64_t)buf + r0 * L) & ~127ull;
    const uint64_t e = r1 == n ? (((uint64_t)buf + n * L + 127) & ~127ull) : (((uint64_t)buf + r1 * L) & ~127ull);
    const uint32_t nb = (uint32_t)(e - b);
    const __amdgpu_buffer_rsrc_t rs = rsrc((const void*)b);
    u32x4 v[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const uint32_t o = 16u * (uint32_t)(64 * s + wl);
        v[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, o < nb ? o : 0x80000000u, 0, 2 /* nt */);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = sum4(v[s], acc);
    // a short reduction, so that each store waits for the whole wavefront's loads (as emit's does)
    acc += (uint32_t)__shfl_xor((int)acc, 32, 64);
    acc += (uint32_t)__builtin_amdgcn_ds_swizzle((int)acc, 0x401F);
    if constexpr (MODE == M_READ) {
        if (acc == 0x9E3779B9u) sink[0] = acc;
        return;
    } else {
        const int j = wl >> 3, l = wl & 7;
        const uint64_t r = r0 + (uint64_t)j;
        if (r >= r1) return;
        const u32x2 x = {acc, acc ^ (uint32_t)r};
        uint64_t sa, sb;
        segs(r, L, sa, sb);
        if constexpr (MODE == M_INLINE || MODE == M_PIPE) {
            const __amdgpu_buffer_rsrc_t ws = rsrc(MODE == M_PIPE ? prev : buf);
            __builtin_amdgcn_raw_buffer_store_b64(x, ws, (uint32_t)sa + 8 * l, 0, AUX);
            if (sb != sa) __builtin_amdgcn_raw_buffer_store_b64(x, ws, (uint32_t)sb + 8 * l, 0, AUX);
        } else if constexpr (MODE == M_INLINE_2B) {
            if (l == 0) {
                *(GMEM uint16_t*)(buf + r * L + 10) = (uint16_t)acc;
                *(GMEM uint16_t*)(buf + r * L + 26) = (uint16_t)(acc >> 16);
            }
        } else if constexpr (MODE == M_VALS) {  // 8 B per record, compact
            if (l == 0) __builtin_amdgcn_raw_buffer_store_b64(x, rsrc(side), (uint32_t)(8 * r), 0, AUX);
        } else {  // M_DENSE: the record's segment(s) in consecutive 64-B slots
            const uint64_t k = dense_slot(dn, r);
            const __amdgpu_buffer_rsrc_t ws = rsrc(side);
            __builtin_amdgcn_raw_buffer_store_b64(x, ws, (uint32_t)(64 * k) + 8 * l, 0, AUX);
            if (sb != sa) __builtin_amdgcn_raw_buffer_store_b64(x, ws, (uint32_t)(64 * k + 64) + 8 * l, 0, AUX);
        }
    }
}

// The scatter pass: 8 lanes per record write its segment(s) whole, records in address order; the data
// a constant (SRC_CONST), the segment read from the buffer and patched with the record's 8 staged
// bytes (SRC_RMW), or the staged segments (SRC_DENSE).
template <int SRC, int AUX>
__global__ __launch_bounds__(256) void scatter_kernel(uint8_t* buf, const uint8_t* side, uint64_t n, uint32_t L, Dense dn) {
    const uint64_t r = (uint64_t)blockIdx.x * 32 + (threadIdx.x >> 3);
    const int l = (int)(threadIdx.x & 7);
    if (r >= n) return;
    uint64_t sa, sb;
    segs(r, L, sa, sb);
    const __amdgpu_buffer_rsrc_t bs = rsrc(buf);
    u32x2 xa = {(uint32_t)r, 7u}, xb = xa;
    if constexpr (SRC == SRC_RMW) {
        const u32x2 val = __builtin_nontemporal_load((const GMEM u32x2*)(side + 8 * r));
        xa = __builtin_amdgcn_raw_buffer_load_b64(bs, (uint32_t)sa + 8 * l, 0, 0);
        if (sb != sa) xb = __builtin_amdgcn_raw_buffer_load_b64(bs, (uint32_t)sb + 8 * l, 0, 0);
        xa ^= val;
        xb ^= val;
    } else if constexpr (SRC == SRC_DENSE) {
        const uint64_t k = dense_slot(dn, r);
        xa = __builtin_nontemporal_load((const GMEM u32x2*)(side + 64 * k + 8 * l));
        if (sb != sa) xb = __builtin_nontemporal_load((const GMEM u32x2*)(side + 64 * k + 64 + 8 * l));
    }
    __builtin_amdgcn_raw_buffer_store_b64(xa, bs, (uint32_t)sa + 8 * l, 0, AUX);
    if (sb != sa) __builtin_amdgcn_raw_buffer_store_b64(xb, bs, (uint32_t)sb + 8 * l, 0, AUX);
}

// The same stream in the transposed walk's own shape: load instruction (s, j) covers 1 KiB of record
// j (chunks 64 s .. 64 s + 63 from its 128-B line), 2 per record, the line holding record j + 1's
// first byte loaded once, by record j + 1.  HC: the chunks of record j's field segments are loaded
// with the default cache policy (a second, exec-masked instruction), the rest non-temporal.
template <int MODE, int AUX, bool HC>
__global__ __launch_bounds__(256) void xstream_kernel(uint8_t* buf, uint8_t* side, uint64_t n, uint32_t L, uint32_t* sink) {
    const int wl = (int)(threadIdx.x & 63);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (uint64_t)wv;
    const uint64_t r0 = w * 8;
    if (r0 >= n) return;
    const uint32_t c = (uint32_t)(n - r0 < 8 ? n - r0 : 8);
    const uint64_t wbase = ((uint64_t)buf + r0 * L) & ~127ull;
    const __amdgpu_buffer_rsrc_t rs = rsrc((const void*)wbase);
    u32x4 v[2][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint64_t a0 = (uint64_t)buf + (r0 + (uint64_t)j) * L;
        const uint64_t b = a0 & ~127ull;
        const uint32_t hd = (uint32_t)(a0 - b);
        const uint32_t nch = (uint32_t)j < c ? (uint32_t)(((a0 + L + 15) >> 4) - (b >> 4)) : 0u;
        const uint32_t nload = (uint32_t)j + 1 < c ? (uint32_t)((((a0 + L) & ~127ull) - b) >> 4) : nch;
        const int soff = __builtin_amdgcn_readfirstlane((int)(uint32_t)(b - wbase));
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const uint32_t k = (uint32_t)(64 * s2 + wl);
            const uint32_t o = k < nload ? 16u * k : 0x80000000u;
            if (HC && s2 == 0) {
                const uint32_t sg = (uint32_t)wl >> 2;
                if (sg == (hd + 10) >> 6 || sg == (hd + 27) >> 6) v[s2][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, 0);
                else v[s2][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, 2);
            } else {
                v[s2][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, 2 /* nt */);
            }
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = sum4(v[1][j], sum4(v[0][j], acc));
    acc += (uint32_t)__shfl_xor((int)acc, 32, 64);
    acc += (uint32_t)__builtin_amdgcn_ds_swizzle((int)acc, 0x401F);
    if constexpr (MODE == M_READ) {
        if (acc == 0x9E3779B9u) sink[0] = acc;
        return;
    } else {
        const int j = wl >> 3, l = wl & 7;
        if ((uint32_t)j >= c) return;
        const uint64_t r = r0 + (uint64_t)j;
        const u32x2 x = {acc, acc ^ (uint32_t)r};
        uint64_t sa, sb;
        segs(r, L, sa, sb);
        if constexpr (MODE == M_INLINE) {
            const __amdgpu_buffer_rsrc_t ws = rsrc(buf);
            __builtin_amdgcn_raw_buffer_store_b64(x, ws, (uint32_t)sa + 8 * l, 0, AUX);
            if (sb != sa) __builtin_amdgcn_raw_buffer_store_b64(x, ws, (uint32_t)sb + 8 * l, 0, AUX);
        } else {  // M_VALS
            if (l == 0) __builtin_amdgcn_raw_buffer_store_b64(x, rsrc(side), (uint32_t)(8 * r), 0, AUX);
        }
    }
}

// A pass of 2-B field stores (both fields of every record, one thread per record).
template <int AUX>
__global__ __launch_bounds__(256) void scatter2b_kernel(uint8_t* buf, uint64_t n, uint32_t L) {
    const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    const __amdgpu_buffer_rsrc_t bs = rsrc(buf);
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)r, bs, (uint32_t)(r * L + 10), 0, AUX);
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(r >> 3), bs, (uint32_t)(r * L + 26), 0, AUX);
}

// The read-modify-write pass: each record's segment(s) loaded (LAUX: the load's cache policy),
// patched with the record's 8 staged bytes and stored whole (AUX); READONLY: the loads only.
template <int LAUX, int AUX, bool READONLY>
__global__ __launch_bounds__(256) void rmw_kernel(uint8_t* buf, const uint8_t* side, uint64_t n, uint32_t L, uint32_t* sink) {
    const uint64_t r = (uint64_t)blockIdx.x * 32 + (threadIdx.x >> 3);
    const int l = (int)(threadIdx.x & 7);
    if (r >= n) return;
    uint64_t sa, sb;
    segs(r, L, sa, sb);
    const __amdgpu_buffer_rsrc_t bs = rsrc(buf);
    u32x2 val = {0u, 0u};
    if (!READONLY) val = __builtin_nontemporal_load((const GMEM u32x2*)(side + 8 * r));
    u32x2 xa = __builtin_amdgcn_raw_buffer_load_b64(bs, (uint32_t)sa + 8 * l, 0, LAUX), xb = xa;
    if (sb != sa) xb = __builtin_amdgcn_raw_buffer_load_b64(bs, (uint32_t)sb + 8 * l, 0, LAUX);
    if (READONLY) {
        if ((xa.x ^ xb.y) == 0x9E3779B9u) sink[0] = 1;
        return;
    }
    xa ^= val;
    xb ^= val;
    __builtin_amdgcn_raw_buffer_store_b64(xa, bs, (uint32_t)sa + 8 * l, 0, AUX);
    if (sb != sa) __builtin_amdgcn_raw_buffer_store_b64(xb, bs, (uint32_t)sb + 8 * l, 0, AUX);
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : (1ull << 20);
    const uint32_t L = argc > 2 ? (uint32_t)strtoul(argv[2], nullptr, 0) : 1500u;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    if (L < 1024 || L > 1921 || n == 0 || n > (1ull << 24)) {
        fprintf(stderr, "probe_wtax: L must be 1024..1921 (8 records per 16 KiB), n 1..2^24\n");
        return 2;
    }
    const int NB = 4;
    const uint64_t bytes = n * L + 256;
    std::vector<uint8_t*> tx(NB), rx(NB);
    for (int i = 0; i < NB; ++i) {
        CK(hipMalloc(&tx[i], bytes));
        CK(hipMalloc(&rx[i], bytes));
        CK(hipMemset(tx[i], 0x5a + i, bytes));
        CK(hipMemset(rx[i], 0x3c + i, bytes));
    }
    uint8_t* side;
    CK(hipMalloc(&side, n * 128));
    CK(hipMemset(side, 0, n * 128));
    uint32_t* sink;
    CK(hipMalloc(&sink, 64));
    // segments written per pass
    uint64_t nseg = 0;
    for (uint64_t r = 0; r < n; ++r) nseg += ((r * L + 10) & ~63ull) == ((r * L + 27) & ~63ull) ? 1 : 2;

    Dense dn{};
    dn.per = 64;
    while (dn.per > 1 && ((uint64_t)L * (dn.per / 2)) % 64 == 0) dn.per /= 2;
    for (uint32_t k = 0; k < dn.per; ++k)
        dn.pre[k + 1] = dn.pre[k] + ((((uint64_t)k * L + 10) & ~63ull) != (((uint64_t)k * L + 27) & ~63ull) ? 1u : 0u);
    const dim3 gs((unsigned)((n + 31) / 32)), blk(256), gsc((unsigned)((n + 31) / 32));
#define STREAM(M, A, B, P) hipLaunchKernelGGL((stream_kernel<M, A>), gs, blk, 0, 0, B, P, side, n, L, sink, dn)
#define SCATTER(S, A, B) hipLaunchKernelGGL((scatter_kernel<S, A>), gsc, blk, 0, 0, B, side, n, L, dn)
    auto rd = [&](uint8_t* b) { STREAM(M_READ, 0, b, b); };
    // rmw forms: X<stream>_<B's load policy>_<B's store policy>[_<A's staging policy>]; stream x = all
    // non-temporal, h = field segments loaded with the default policy; policies: d default, n nt,
    // s sc0 sc1, w sc0 sc1 nt, 1 sc1
    const char* names[] = {"read",    "xread",   "xread_hc", "xinline_nt", "xdeferred_nt",
                           "x_d_w",   "x_n_w",   "x_d_s",    "x_n_n",      "h_d_w",
                           "h_n_w",   "h_d_s",   "h_d_1",    "h_d_w_sw",   "h_d_w_sd",
                           "h_d_n",   "scatter_nt"};
    const int NM = sizeof(names) / sizeof(names[0]);
    const int FIRST_ALONE = 16;  // modes from here on have no stream
#define XSTREAM(M, A, HC, B) hipLaunchKernelGGL((xstream_kernel<M, A, HC>), gs, blk, 0, 0, B, side, n, L, sink)
#define RMW(LA, A, RO, B) hipLaunchKernelGGL((rmw_kernel<LA, A, RO>), gsc, blk, 0, 0, B, side, n, L, sink)
    auto pass = [&](int m, int i) {
        uint8_t* b = tx[i % NB];
        switch (m) {
            case 0: rd(b); break;
            case 1: XSTREAM(M_READ, 0, false, b); break;
            case 2: XSTREAM(M_READ, 0, true, b); break;
            case 3: XSTREAM(M_INLINE, 2, false, b); break;
            case 4: XSTREAM(M_READ, 0, false, b); SCATTER(SRC_CONST, 2, b); break;
            case 5: XSTREAM(M_VALS, 2, false, b); RMW(0, 19, false, b); break;
            case 6: XSTREAM(M_VALS, 2, false, b); RMW(2, 19, false, b); break;
            case 7: XSTREAM(M_VALS, 2, false, b); RMW(0, 17, false, b); break;
            case 8: XSTREAM(M_VALS, 2, false, b); RMW(2, 2, false, b); break;
            case 9: XSTREAM(M_VALS, 2, true, b); RMW(0, 19, false, b); break;
            case 10: XSTREAM(M_VALS, 2, true, b); RMW(2, 19, false, b); break;
            case 11: XSTREAM(M_VALS, 2, true, b); RMW(0, 17, false, b); break;
            case 12: XSTREAM(M_VALS, 2, true, b); RMW(0, 16, false, b); break;
            case 13: XSTREAM(M_VALS, 19, true, b); RMW(0, 19, false, b); break;
            case 14: XSTREAM(M_VALS, 0, true, b); RMW(0, 19, false, b); break;
            case 15: XSTREAM(M_VALS, 2, true, b); RMW(0, 2, false, b); break;
            default: SCATTER(SRC_CONST, 2, b); break;
        }
    };
    hipEvent_t a, z;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&z));
    const int K = 20;
    auto timed = [&](int m, bool step) {
        for (int i = 0; i < 2 * NB; ++i) {
            pass(m, i);
            if (step) rd(rx[i % NB]);
        }
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < K; ++i) {
            pass(m, i);
            if (step) rd(rx[i % NB]);
        }
        CK(hipEventRecord(z, 0));
        CK(hipEventSynchronize(z));
        float ms;
        CK(hipEventElapsedTime(&ms, a, z));
        CK(hipGetLastError());
        return ms / K;
    };
    // clock ramp
    for (int i = 0; i < 400; ++i) rd(tx[i % NB]);
    CK(hipDeviceSynchronize());
    for (int rnd = 0; rnd < rounds; ++rnd) {
        float base[2] = {0, 0};
        for (int m = 0; m < NM; ++m)
            for (int st = 0; st < 2; ++st) {
                const float ms = timed(m, st == 1);
                if (m == 0) base[st] = ms;
                // the scatter pass alone has no stream: its cost is its own time (step form: over one read pass)
                const bool alone_scatter = m >= FIRST_ALONE;
                const double extra = m == 0 ? 0.0 : alone_scatter ? (st ? ms - base[0] : ms) : ms - base[st];
                printf("{\"round\": %d, \"mode\": \"%s\", \"form\": \"%s\", \"n\": %llu, \"L\": %u, \"segments\": %llu, "
                       "\"ms\": %.4f, \"over_read_ms\": %.4f, \"ps_per_segment\": %.1f}\n",
                       rnd, names[m], st ? "step (then a read pass over an RX buffer)" : "alone", (unsigned long long)n, L,
                       (unsigned long long)nseg, ms, extra, extra * 1e9 / (double)nseg);
                fflush(stdout);
            }
    }
    for (int i = 0; i < NB; ++i) {
        CK(hipFree(tx[i]));
        CK(hipFree(rx[i]));
    }
    CK(hipFree(side));
    CK(hipFree(sink));
    return 0;
}
