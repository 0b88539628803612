// Two-pass emit probe: does the write tax of in-place emit go away when the field stores are
// issued as a separate scatter pass with a cache policy that sends them to HBM at once, instead
// of leaving dirty lines in the Infinity Cache for the next read stream to evict?
//
// One "step" = the TX buffer's pass + the RX buffer's read-only pass (verify's stand-in), both
// 2^20 records of 1500 B, fields at record offsets 10 and 26 (C2).  Modes:
//   0  TX read-only                                  (no stores: the floor)
//   1  TX read + the two 2-B field stores in place   (today's emit, the field probe's pattern)
//   2  TX read + 4 B per record into a compact array, then a scatter pass of the 2-B stores
//   3  as 2, the scatter pass with non-temporal stores
//   4  as 2, the scatter pass with sc0 sc1 stores (system scope: written through)
//   5  as 2, the scatter pass with sc1 stores
//   6  as 2, the scatter pass with sc0 sc1 nt stores
// Standalone tool; results in DESIGN.md §5 (profiles/r03_experiments/probe_wr3.jsonl).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#define GMEM __attribute__((address_space(1)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint64_t N = 1ull << 20, L = 1500;

// Wave-contiguous 8-KiB pieces, 8 nt loads per lane in flight (stream_read_kernel); STORE 1: the
// fields of records starting in the piece in place; STORE 2: their 4-B results into `compact`.
template <int STORE>
__global__ __launch_bounds__(256) void stream(uint8_t* buf, uint64_t n16, uint32_t* compact, uint32_t* sink) {
    constexpr int UNR = 8;
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint64_t w0 = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const uint64_t per = 64ull * UNR;
    const GMEM u32x4* q = (const GMEM u32x4*)buf;
    uint32_t tot = 0;
    for (uint64_t base = w0 * per; base + per <= n16; base += nw * per) {
        u32x4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = __builtin_nontemporal_load(q + base + u * 64 + lane);
        uint32_t acc = 0;
#pragma unroll
        for (int u = 0; u < UNR; ++u)
            acc += __builtin_amdgcn_sad_u16(v[u].x, 0, 0) + __builtin_amdgcn_sad_u16(v[u].y, 0, 0) +
                   __builtin_amdgcn_sad_u16(v[u].z, 0, 0) + __builtin_amdgcn_sad_u16(v[u].w, 0, 0);
        tot += acc;
        if (STORE) {
            const uint64_t lo = 16 * base, hi = 16 * (base + per);
            for (uint64_t r = (lo + L - 1) / L + (uint64_t)lane; r * L < hi && r < N; r += 64) {
                if (STORE == 1) {
                    *(GMEM uint16_t*)(buf + r * L + 10) = (uint16_t)acc;
                    *(GMEM uint16_t*)(buf + r * L + 26) = (uint16_t)(acc >> 16);
                } else {
                    ((GMEM uint32_t*)compact)[r] = acc + (uint32_t)r;
                }
            }
        }
    }
    if (tot == 0x9E3779B9u) sink[0] = tot;
}

// The scatter pass: record r's two 2-B fields from compact[r].  POL 0 plain, 1 nt, 2 sc0 sc1,
// 3 sc1, 4 sc0 sc1 nt.
template <int POL>
__device__ __forceinline__ void st16(uint8_t* p, uint32_t v) {
    if constexpr (POL == 0) {
        *(GMEM uint16_t*)p = (uint16_t)v;
    } else if constexpr (POL == 1) {
        __builtin_nontemporal_store((uint16_t)v, (GMEM uint16_t*)p);
    } else if constexpr (POL == 2) {
        asm volatile("global_store_short %0, %1, off sc0 sc1" :: "v"(p), "v"(v) : "memory");
    } else if constexpr (POL == 3) {
        asm volatile("global_store_short %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
    } else {
        asm volatile("global_store_short %0, %1, off sc0 sc1 nt" :: "v"(p), "v"(v) : "memory");
    }
}

template <int POL>
__global__ __launch_bounds__(256) void scatter(uint8_t* buf, const uint32_t* compact) {
    const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= N) return;
    const uint32_t v = ((const GMEM uint32_t*)compact)[r];
    st16<POL>(buf + r * L + 10, v);
    st16<POL>(buf + r * L + 26, v >> 16);
}

int main() {
    uint8_t *tx, *rx;
    uint32_t *compact, *sink;
    const uint64_t bytes = N * L + 4096;
    CK(hipMalloc(&tx, bytes));
    CK(hipMalloc(&rx, bytes));
    CK(hipMalloc(&compact, N * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(tx, 0x33, bytes));
    CK(hipMemset(rx, 0x55, bytes));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const dim3 g((unsigned)prop.multiProcessorCount * 8), blk(256), gs((unsigned)(N / 256));
    const uint64_t n16 = N * L / 16;
    const char* names[] = {"TX read-only", "TX read + in-place field stores", "compact + scatter (plain)",
                           "compact + scatter (nt)", "compact + scatter (sc0 sc1)", "compact + scatter (sc1)",
                           "compact + scatter (sc0 sc1 nt)"};
    auto step = [&](int m) {
        switch (m) {
            case 0: hipLaunchKernelGGL(stream<0>, g, blk, 0, 0, tx, n16, compact, sink); break;
            case 1: hipLaunchKernelGGL(stream<1>, g, blk, 0, 0, tx, n16, compact, sink); break;
            default:
                hipLaunchKernelGGL(stream<2>, g, blk, 0, 0, tx, n16, compact, sink);
                if (m == 2) hipLaunchKernelGGL(scatter<0>, gs, blk, 0, 0, tx, compact);
                if (m == 3) hipLaunchKernelGGL(scatter<1>, gs, blk, 0, 0, tx, compact);
                if (m == 4) hipLaunchKernelGGL(scatter<2>, gs, blk, 0, 0, tx, compact);
                if (m == 5) hipLaunchKernelGGL(scatter<3>, gs, blk, 0, 0, tx, compact);
                if (m == 6) hipLaunchKernelGGL(scatter<4>, gs, blk, 0, 0, tx, compact);
        }
        hipLaunchKernelGGL(stream<0>, g, blk, 0, 0, rx, n16, compact, sink);  // verify's stand-in
    };
    hipEvent_t a, b, c;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreate(&c));
    for (int i = 0; i < 600; ++i) step(1);  // clock ramp
    CK(hipDeviceSynchronize());
    for (int rnd = 0; rnd < 4; ++rnd)
        for (int m = 0; m < 7; ++m) {
            for (int i = 0; i < 5; ++i) step(m);
            CK(hipEventRecord(a, 0));
            for (int i = 0; i < 30; ++i) step(m);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            // the TX pass alone (its kernels only), for reference
            CK(hipEventRecord(a, 0));
            for (int i = 0; i < 30; ++i) {
                if (m == 0) hipLaunchKernelGGL(stream<0>, g, blk, 0, 0, tx, n16, compact, sink);
                else if (m == 1) hipLaunchKernelGGL(stream<1>, g, blk, 0, 0, tx, n16, compact, sink);
                else {
                    hipLaunchKernelGGL(stream<2>, g, blk, 0, 0, tx, n16, compact, sink);
                    if (m == 2) hipLaunchKernelGGL(scatter<0>, gs, blk, 0, 0, tx, compact);
                    if (m == 3) hipLaunchKernelGGL(scatter<1>, gs, blk, 0, 0, tx, compact);
                    if (m == 4) hipLaunchKernelGGL(scatter<2>, gs, blk, 0, 0, tx, compact);
                    if (m == 5) hipLaunchKernelGGL(scatter<3>, gs, blk, 0, 0, tx, compact);
                    if (m == 6) hipLaunchKernelGGL(scatter<4>, gs, blk, 0, 0, tx, compact);
                }
            }
            CK(hipEventRecord(c, 0));
            CK(hipEventSynchronize(c));
            float tx_ms;
            CK(hipEventElapsedTime(&tx_ms, a, c));
            if (rnd)
                printf("{\"round\": %d, \"mode\": %d, \"what\": \"%s\", \"step_ms\": %.4f, \"tx_pass_ms\": %.4f}\n", rnd, m,
                       names[m], ms / 30, tx_ms / 30);
        }
    CK(hipFree(tx));
    CK(hipFree(rx));
    CK(hipFree(compact));
    CK(hipFree(sink));
    return 0;
}
