// Read-policy probe (round 5): the record-shaped walk of the verify kernel (groups of 8 lanes, one
// 1500-B record each, 7 chunks per lane per step, chunk grid on the 128-B line) over a 1.5-GB
// buffer, with global_load_dwordx4 (plain / nt) and with buffer_load_dwordx4 under every cache-policy
// combination of the aux operand (gfx950: bit 0 sc0, bit 1 nt, bit 4 sc1); `shapes`: nt loads at
// group shapes G x U of one and two steps per record.  Standalone tool:
//   hipcc -O3 --offload-arch=gfx950 tools/probe_pol.hip -o tools/probe_pol && tools/probe_pol
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// KIND 0: global plain, 1: global nt, 2: buffer load with aux AUX.  Out-of-range chunks: the dummy
// line (global) or an out-of-bounds offset (buffer: returns 0 without a memory access).
template <int KIND, int AUX, int G = 8, int U = 7>
__global__ __launch_bounds__(256) void rec_walk(const uint8_t* __restrict__ buf, uint64_t n, uint64_t bytes,
                                                uint32_t* sink) {
    const int lane = threadIdx.x % G;
    const uint64_t r = (uint64_t)blockIdx.x * (256 / G) + threadIdx.x / G;
    if (r >= n) return;
    const uint64_t off0 = r * 1500;
    const uint64_t base = off0 & ~127ull;
    const uint32_t nch = (uint32_t)(((off0 + 1500 + 15) >> 4) - (base >> 4));
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)buf >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)buf);
    const uint8_t* ub = (const uint8_t*)(((uint64_t)hi << 32) | lo);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)ub, 0, (int)0x7fffffff, 0x00020000);
    uint32_t acc = 0;
    for (uint32_t k0 = 0; k0 < nch; k0 += G * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = k0 + u * G + lane;
            if constexpr (KIND == 2) {
                const uint32_t vo = k < nch ? (uint32_t)(base + 16ull * k) : 0x7ffffff0u + 0x10u;
                v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, AUX);
            } else {
                const u32x4* q = (const u32x4*)(k < nch ? (uint64_t)buf + base + 16ull * k : (uint64_t)buf);
                const __attribute__((address_space(1))) u32x4* g = (const __attribute__((address_space(1))) u32x4*)q;
                v[u] = KIND == 1 ? __builtin_nontemporal_load(g) : *g;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc += __builtin_amdgcn_sad_u16(v[u].x, 0, 0) + __builtin_amdgcn_sad_u16(v[u].y, 0, 0) +
                   __builtin_amdgcn_sad_u16(v[u].z, 0, 0) + __builtin_amdgcn_sad_u16(v[u].w, 0, 0);
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const uint64_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : 1572864000ull;
    uint8_t* p;
    uint32_t* sink;
    CK(hipMalloc(&p, bytes + 256));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(p, 0x5a, bytes + 256));
    const uint64_t nrec = bytes / 1500;
    auto run = [&](const char* nm, auto kern, int G = 8) {
        const uint64_t blocks = (nrec + 256 / G - 1) / (256 / G);
        for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, p, nrec, bytes, sink);
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, p, nrec, bytes, sink);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= 20;
        printf("%-24s %8.4f ms %8.1f GB/s\n", nm, ms, nrec * 1500.0 / ms / 1e6);
        fflush(stdout);
    };
    const bool shapes = argc > 2;  // `probe_pol BYTES shapes`: group shapes with nt loads only
    for (int rep = 0; rep < 3 && shapes; ++rep) {
        run("nt G8U7 (2 steps)", rec_walk<1, 0, 8, 7>, 8);
        run("nt G8U14 (1 step)", rec_walk<1, 0, 8, 14>, 8);
        run("nt G16U4 (2 steps)", rec_walk<1, 0, 16, 4>, 16);
        run("nt G16U7 (1 step)", rec_walk<1, 0, 16, 7>, 16);
        run("nt G32U2 (2 steps)", rec_walk<1, 0, 32, 2>, 32);
        run("nt G32U4 (1 step)", rec_walk<1, 0, 32, 4>, 32);
        run("nt G64U1 (2 steps)", rec_walk<1, 0, 64, 1>, 64);
        run("nt G64U2 (1 step)", rec_walk<1, 0, 64, 2>, 64);
    }
    for (int rep = 0; rep < 3 && !shapes; ++rep) {
        run("global plain", rec_walk<0, 0>);
        run("global nt", rec_walk<1, 0>);
        run("buffer aux 0", rec_walk<2, 0>);
        run("buffer aux 1 (sc0)", rec_walk<2, 1>);
        run("buffer aux 2 (nt)", rec_walk<2, 2>);
        run("buffer aux 3 (sc0 nt)", rec_walk<2, 3>);
        run("buffer aux 16 (sc1)", rec_walk<2, 16>);
        run("buffer aux 17 (sc0 sc1)", rec_walk<2, 17>);
        run("buffer aux 18 (sc1 nt)", rec_walk<2, 18>);
        run("buffer aux 19 (all)", rec_walk<2, 19>);
    }
    CK(hipFree(p));
    return 0;
}
