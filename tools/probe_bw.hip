// HBM read-streaming probe for MI355X: which load form / occupancy / in-flight depth reads a
// 1.5 GB device buffer fastest.  Standalone tool (not part of the library):
//   hipcc -O3 --offload-arch=gfx950 tools/probe_bw.hip -o tools/probe_bw && tools/probe_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldnt(const uint4* q) {
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(q));
    return make_uint4(v.x, v.y, v.z, v.w);
}

template <int UNR, bool NT>
__global__ __launch_bounds__(256) void grid_stride(const uint4* __restrict__ p, uint64_t n16, uint32_t* sink) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (; i + (UNR - 1) * stride < n16; i += UNR * stride) {
        uint4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = NT ? ldnt(p + i + u * stride) : p[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNR; ++u) acc += __builtin_amdgcn_sad_u16(v[u].x, 0, 0) + __builtin_amdgcn_sad_u16(v[u].y, 0, 0) + __builtin_amdgcn_sad_u16(v[u].z, 0, 0) + __builtin_amdgcn_sad_u16(v[u].w, 0, 0);
    }
    for (; i < n16; i += stride) acc += p[i].x;
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// Each wave owns contiguous spans of SPAN 1-KiB pieces (like a record-per-wave kernel).
template <int UNR, bool NT>
__global__ __launch_bounds__(256) void wave_spans(const uint4* __restrict__ p, uint64_t n16, uint32_t* sink) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint64_t w0 = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const uint64_t per = 64ull * UNR;  // 16-B chunks per wave step
    uint32_t acc = 0;
    for (uint64_t base = w0 * per; base + per <= n16; base += nw * per) {
        uint4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = NT ? ldnt(p + base + u * 64 + lane) : p[base + u * 64 + lane];
#pragma unroll
        for (int u = 0; u < UNR; ++u) acc += __builtin_amdgcn_sad_u16(v[u].x, 0, 0) + __builtin_amdgcn_sad_u16(v[u].y, 0, 0) + __builtin_amdgcn_sad_u16(v[u].z, 0, 0) + __builtin_amdgcn_sad_u16(v[u].w, 0, 0);
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// LDS-DMA: each wave streams 1 KiB pieces into its own LDS ring with global_load_lds_dwordx4,
// DEPTH pieces in flight, then sums them with ds_read_b128.
template <int DEPTH>
__global__ __launch_bounds__(256) void glds_ring(const uint4* __restrict__ p, uint64_t n16, uint32_t* sink) {
    __shared__ uint4 ring[4][DEPTH][64];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x / 64;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint64_t w0 = (uint64_t)blockIdx.x * 4 + w;
    const uint64_t npieces = n16 / 64;
    uint32_t acc = 0;
    uint64_t issue = w0, consume = w0;
    int slot_i = 0, slot_c = 0;
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
        if (issue < npieces) {
            __builtin_amdgcn_global_load_lds((const void*)(p + issue * 64 + lane), (__attribute__((address_space(3))) void*)&ring[w][slot_i][0], 16, 0, 0);
        }
        issue += nw;
        slot_i = (slot_i + 1) % DEPTH;
    }
    while (consume < npieces) {
        __builtin_amdgcn_s_waitcnt(0x0F70 | ((DEPTH - 1) & 0xF) | (((DEPTH - 1) >> 4) << 14));  // vmcnt(DEPTH-1)
        __builtin_amdgcn_wave_barrier();
        uint4 v = ring[w][slot_c][lane];
        acc += __builtin_amdgcn_sad_u16(v.x, 0, 0) + __builtin_amdgcn_sad_u16(v.y, 0, 0) + __builtin_amdgcn_sad_u16(v.z, 0, 0) + __builtin_amdgcn_sad_u16(v.w, 0, 0);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): slot read before it is refilled
        __builtin_amdgcn_wave_barrier();
        if (issue < npieces) {
            __builtin_amdgcn_global_load_lds((const void*)(p + issue * 64 + lane), (__attribute__((address_space(3))) void*)&ring[w][slot_c][0], 16, 0, 0);
        }
        issue += nw;
        consume += nw;
        slot_c = (slot_c + 1) % DEPTH;
    }
    __builtin_amdgcn_s_waitcnt(0);
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

template <class K>
static double time_kernel(K k, int blocks, const uint4* p, uint64_t n16, uint32_t* sink, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, p, n16, sink);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, p, n16, sink);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGetLastError());
    return ms / reps;
}

// Record-shaped access: groups of G lanes each walk one 1500-B record (G*16 B per load
// instruction per group, records back to back), like the checksum walk kernel, with the chunk
// grid aligned to 16 B or to the 128-B line.  nt / plain loads.
template <int G, int U, bool NT, bool LINE>
__global__ __launch_bounds__(256) void rec_walk(const uint8_t* __restrict__ buf, uint64_t n, uint32_t* sink) {
    const int lane = threadIdx.x % G;
    const uint64_t r = (uint64_t)blockIdx.x * (256 / G) + threadIdx.x / G;
    if (r >= n) return;
    const uint64_t a0 = (uint64_t)buf + r * 1500;
    const uint64_t base = LINE ? (a0 & ~127ull) : (a0 & ~15ull);
    const uint32_t nch = (uint32_t)(((a0 + 1500 + 15) >> 4) - (base >> 4));
    uint32_t acc = 0;
    for (uint32_t k0 = 0; k0 < nch; k0 += G * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = k0 + u * G + lane;
            const uint4* q = (const uint4*)(k < nch ? base + 16ull * k : (uint64_t)buf);
            v[u] = NT ? ldnt(q) : *q;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += __builtin_amdgcn_sad_u16(v[u].x, 0, 0) + __builtin_amdgcn_sad_u16(v[u].y, 0, 0) + __builtin_amdgcn_sad_u16(v[u].z, 0, 0) + __builtin_amdgcn_sad_u16(v[u].w, 0, 0);
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// Stripe access: each wave reads R consecutive 1500-B records as one line-aligned contiguous
// region (1 KiB per load instruction across the wave), natural grid (one stripe per wave).
// LDS=true also stages every chunk through LDS (ds_write_b128 + ds_read_b128 by another lane).
template <int R, bool NT, bool LDS>
__global__ __launch_bounds__(256) void stripe(const uint8_t* __restrict__ buf, uint64_t n, uint32_t* sink) {
    constexpr int U = (R * 1500 + 127 + 1023) / 1024;
    __shared__ uint4 st[LDS ? 4 * 64 * U : 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t r0 = ((uint64_t)blockIdx.x * 4 + wv) * R;
    if (r0 >= n) return;
    const uint64_t a0 = (uint64_t)buf + r0 * 1500;
    const uint64_t base = a0 & ~127ull;
    const uint64_t rn = r0 + R < n ? r0 + R : n;
    const uint64_t end = (uint64_t)buf + rn * 1500;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t q = base + 16ull * (u * 64 + lane);
        const uint4* pq = (const uint4*)(q < end ? q : (uint64_t)buf);
        v[u] = NT ? ldnt(pq) : *pq;
    }
    uint32_t acc = 0;
    if (LDS) {
#pragma unroll
        for (int u = 0; u < U; ++u) st[(wv * U + u) * 64 + lane] = v[u];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = st[(wv * U + u) * 64 + (lane ^ 1)];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += __builtin_amdgcn_sad_u16(v[u].x, 0, 0) + __builtin_amdgcn_sad_u16(v[u].y, 0, 0) + __builtin_amdgcn_sad_u16(v[u].z, 0, 0) + __builtin_amdgcn_sad_u16(v[u].w, 0, 0);
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const uint64_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : 1572864000ull;
    const uint64_t n16 = bytes / 16;
    uint4* p;
    uint32_t* sink;
    CK(hipMalloc(&p, n16 * 16));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(p, 0x5a, n16 * 16));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("bytes=%llu CUs=%d\n", (unsigned long long)(n16 * 16), cus);
    const int reps = 20;
    auto rep = [&](const char* name, int bpc, double ms) {
        printf("%-28s blocks/CU=%-3d %8.4f ms  %7.1f GB/s\n", name, bpc, ms, n16 * 16 / ms / 1e6);
    };
    const bool rec_only = argc > 2;  // `probe_bw BYTES rec`: only the record-shaped patterns
    for (int bpc : {2, 4, 8, 16}) {
        if (rec_only) break;
        const int blocks = cus * bpc;
        rep("grid_stride U1", bpc, time_kernel(grid_stride<1, false>, blocks, p, n16, sink, reps));
        rep("grid_stride U4", bpc, time_kernel(grid_stride<4, false>, blocks, p, n16, sink, reps));
        rep("grid_stride U8", bpc, time_kernel(grid_stride<8, false>, blocks, p, n16, sink, reps));
        rep("grid_stride U4 nt", bpc, time_kernel(grid_stride<4, true>, blocks, p, n16, sink, reps));
        rep("grid_stride U8 nt", bpc, time_kernel(grid_stride<8, true>, blocks, p, n16, sink, reps));
        rep("wave_spans U2", bpc, time_kernel(wave_spans<2, false>, blocks, p, n16, sink, reps));
        rep("wave_spans U4", bpc, time_kernel(wave_spans<4, false>, blocks, p, n16, sink, reps));
        rep("wave_spans U8", bpc, time_kernel(wave_spans<8, false>, blocks, p, n16, sink, reps));
        rep("wave_spans U4 nt", bpc, time_kernel(wave_spans<4, true>, blocks, p, n16, sink, reps));
        rep("wave_spans U8 nt", bpc, time_kernel(wave_spans<8, true>, blocks, p, n16, sink, reps));
        rep("glds_ring D4", bpc, time_kernel(glds_ring<4>, blocks, p, n16, sink, reps));
        rep("glds_ring D8", bpc, time_kernel(glds_ring<8>, blocks, p, n16, sink, reps));
    }
    {
        const uint64_t nrec = bytes / 1500;
        auto recrun = [&](const char* nm, auto kern, int G) {
            const uint64_t blocks = (nrec + 256 / G - 1) / (256 / G);
            for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, (const uint8_t*)p, nrec, sink);
            hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
            hipEventRecord(a, 0);
            for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, (const uint8_t*)p, nrec, sink);
            hipEventRecord(b, 0); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); ms /= 10;
            printf("%-28s natural grid  %8.4f ms %8.1f GB/s\n", nm, ms, nrec * 1500.0 / ms / 1e6);
        };
        recrun("rec_walk G8U6 plain 16B", rec_walk<8, 6, false, false>, 8);
        recrun("rec_walk G8U6 nt 16B", rec_walk<8, 6, true, false>, 8);
        recrun("rec_walk G8U7 plain line", rec_walk<8, 7, false, true>, 8);
        recrun("rec_walk G8U7 nt line", rec_walk<8, 7, true, true>, 8);
        recrun("rec_walk G16U3 plain 16B", rec_walk<16, 3, false, false>, 16);
        recrun("rec_walk G16U3 nt 16B", rec_walk<16, 3, true, false>, 16);
        recrun("rec_walk G16U4 nt line", rec_walk<16, 4, true, true>, 16);
        recrun("rec_walk G64U2 nt line", rec_walk<64, 2, true, true>, 64);
        recrun("rec_walk G64U2 plain 16B", rec_walk<64, 2, false, false>, 64);
        // stripes: one wave per R records, 4 R records per block (recrun's 256 / G = 4 R)
        recrun("stripe R8 nt", stripe<8, true, false>, 8);
        recrun("stripe R8 plain", stripe<8, false, false>, 8);
        recrun("stripe R8 nt LDS", stripe<8, true, true>, 8);
        recrun("stripe R16 nt", stripe<16, true, false>, 4);
        recrun("stripe R4 nt", stripe<4, true, false>, 16);
        recrun("stripe R4 nt LDS", stripe<4, true, true>, 16);
    }
    CK(hipFree(p));
        return 0;
}
