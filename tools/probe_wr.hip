// Write-pattern probe: a 1536-B-record stream (16 lanes x 6 nt dwordx4 per record) with one of
// several per-record store patterns, to price in-place checksum-field writes.  Standalone tool.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#define GMEM __attribute__((address_space(1)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void scatter(uint8_t* buf, uint64_t n, const uint32_t* vals) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = vals[r];
        *(GMEM uint16_t*)((uint64_t)buf + r * 1536 + 10) = (uint16_t)v;
        *(GMEM uint16_t*)((uint64_t)buf + r * 1536 + 26) = (uint16_t)(v >> 16);
    }
}

// write-through variant of the scatter pass (sc0 sc1: the stores go to memory, not parked in L2)
__global__ void scatter_wt(uint8_t* buf, uint64_t n, const uint32_t* vals) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = vals[r];
        asm volatile("global_store_short %0, %1, off sc0 sc1\n\tglobal_store_short %0, %2, off offset:16 sc0 sc1"
                     :: "v"((uint64_t)buf + r * 1536 + 10), "v"(v), "v"(v >> 16) : "memory");
    }
}

// full-line scatter pass: 4 lanes per record copy the record's saved 64-B field line back
__global__ void scatter64(uint8_t* buf, uint64_t n, const uint8_t* lines) {
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < 4 * n; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = t >> 2, c = t & 3;
        const u32x4 v = *(const GMEM u32x4*)((uint64_t)lines + 16 * t);
        *(GMEM u32x4*)((uint64_t)buf + r * 1536 + 16 * c) = v;
    }
}

// re-read scatter: 4 lanes per record read the field line back from the record itself, patch the
// two fields from a 4-B compact array and write the whole line (no 64-B line copy in pass 1)
__global__ void scatter_rr(uint8_t* buf, uint64_t n, const uint32_t* vals) {
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < 4 * n; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = t >> 2, c = t & 3;
        const uint32_t v = vals[r];
        GMEM u32x4* q = (GMEM u32x4*)((uint64_t)buf + r * 1536 + 16 * c);
        u32x4 x = *q;
        if (c == 0) x.z = (x.z & 0xffff0000u) | (v & 0xffffu);
        if (c == 1) x.z = (x.z & 0xffff0000u) | (v >> 16);
        *q = x;
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void rw(uint8_t* buf, uint64_t n, uint8_t* status) {
    const int lane = threadIdx.x & 15;
    const uint64_t ng = (uint64_t)gridDim.x * 16;
    for (uint64_t r = (uint64_t)blockIdx.x * 16 + threadIdx.x / 16; r < n; r += ng) {
        const uint64_t a0 = (uint64_t)buf + r * 1536;
        u32x4 v[6];
#pragma unroll
        for (int u = 0; u < 6; ++u) v[u] = __builtin_nontemporal_load((const GMEM u32x4*)(a0 + 16 * (u * 16 + lane)));
        uint32_t acc = 0;
#pragma unroll
        for (int u = 0; u < 6; ++u) acc = __builtin_amdgcn_sad_u16(v[u].x, 0, __builtin_amdgcn_sad_u16(v[u].y, 0, __builtin_amdgcn_sad_u16(v[u].z, 0, __builtin_amdgcn_sad_u16(v[u].w, 0, acc))));
        acc += __shfl_xor(acc, 1, 16); acc += __shfl_xor(acc, 2, 16); acc += __shfl_xor(acc, 4, 16); acc += __shfl_xor(acc, 8, 16);
        if (MODE == 1 && lane == 0) { *(GMEM uint16_t*)(a0 + 10) = (uint16_t)acc; *(GMEM uint16_t*)(a0 + 26) = (uint16_t)(acc >> 16); }
        if (MODE == 2 && lane < 2) { u32x4 c = v[0]; c.x = acc; *(GMEM u32x4*)(a0 + 16 * lane) = c; }          // 32 B
        if (MODE == 3 && lane < 4) { u32x4 c = v[0]; c.x = acc; *(GMEM u32x4*)(a0 + 16 * lane) = c; }                                   // 64 B line
        if (MODE == 4 && lane < 8) { u32x4 c = v[0]; c.x = acc; *(GMEM u32x4*)(a0 + 16 * lane) = c; }                                   // 128 B
        if (MODE == 5 && lane == 0) { status[r] = (uint8_t)acc; }
        if (MODE == 6 && lane == 0) { u32x4 c = v[0]; c.x = acc; *(GMEM u32x4*)(a0) = c; }                                             // 16 B
        if (MODE == 7 && lane == 0) { __builtin_nontemporal_store((uint16_t)acc, (GMEM uint16_t*)(a0 + 10)); __builtin_nontemporal_store((uint16_t)(acc >> 16), (GMEM uint16_t*)(a0 + 26)); }
        if (MODE == 8 && lane == 0) { *(GMEM uint32_t*)((uint64_t)status + 4 * r) = acc; }   // compact 4-B array
        // cache-policy variants of the 2 x 2-B stores (gfx950 sc0/sc1/nt bits)
        if (MODE == 9 && lane == 0) { asm volatile("global_store_short %0, %1, off sc0 sc1\n\tglobal_store_short %0, %2, off offset:16 sc0 sc1" :: "v"(a0 + 10), "v"(acc), "v"(acc >> 16) : "memory"); }
        if (MODE == 10 && lane == 0) { asm volatile("global_store_short %0, %1, off sc1\n\tglobal_store_short %0, %2, off offset:16 sc1" :: "v"(a0 + 10), "v"(acc), "v"(acc >> 16) : "memory"); }
        if (MODE == 11 && lane == 0) { asm volatile("global_store_short %0, %1, off nt sc0 sc1\n\tglobal_store_short %0, %2, off offset:16 nt sc0 sc1" :: "v"(a0 + 10), "v"(acc), "v"(acc >> 16) : "memory"); }
        if (MODE == 12 && lane == 0) { asm volatile("global_store_short %0, %1, off sc0\n\tglobal_store_short %0, %2, off offset:16 sc0" :: "v"(a0 + 10), "v"(acc), "v"(acc >> 16) : "memory"); }
        // one 32-B aligned sector (two 16-B stores), write-through
        if (MODE == 13 && lane < 2) { u32x4 c = v[0]; c.x = acc; asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(a0 + 16 * lane), "v"(c) : "memory"); }
        // write density: the 2 x 2-B stores on every 2nd / 4th record only
        if (MODE == 14 && lane == 0 && (r & 1) == 0) { *(GMEM uint16_t*)(a0 + 10) = (uint16_t)acc; *(GMEM uint16_t*)(a0 + 26) = (uint16_t)(acc >> 16); }
        if (MODE == 15 && lane == 0 && (r & 3) == 0) { *(GMEM uint16_t*)(a0 + 10) = (uint16_t)acc; *(GMEM uint16_t*)(a0 + 26) = (uint16_t)(acc >> 16); }
        // 64-B line store at every 2nd record
        if (MODE == 16 && lane < 4 && (r & 1) == 0) { u32x4 c = v[0]; c.x = acc; *(GMEM u32x4*)(a0 + 16 * lane) = c; }
        // compact 64-B line array (the record's field line, patched), for a later full-line scatter
        if (MODE == 17 && lane < 4) { u32x4 c = v[0]; c.x = acc; *(GMEM u32x4*)((uint64_t)status + 64 * r + 16 * lane) = c; }
        // 64-B line store, non-temporal
        if (MODE == 18 && lane < 4) { u32x4 c = v[0]; c.x = acc; __builtin_nontemporal_store(c, (GMEM u32x4*)(a0 + 16 * lane)); }
        if (MODE == 0 && acc == 0x12345678u) status[0] = 1;
    }
}

int main() {
    const uint64_t n = 1 << 20;
    uint8_t *buf, *st;
    CK(hipMalloc(&buf, n * 1536));
    CK(hipMalloc(&st, 64 * n));
    CK(hipMemset(buf, 0x33, n * 1536));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const char* names[] = {"read only", "2 x 2-B stores", "32-B store", "64-B line store", "128-B store", "1-B status array", "16-B store", "2 x 2-B nt stores", "4-B compact array", "scatter kernel only",
                           "2x2-B sc0 sc1", "2x2-B sc1", "2x2-B nt sc0 sc1", "2x2-B sc0", "32-B sc0 sc1",
                           "2x2-B every 2nd", "2x2-B every 4th", "64-B every 2nd", "compact 64-B lines", "64-B nt line store"};
    for (int rnd = 0; rnd < 2; ++rnd)
    for (int bpc : {2, 8}) for (int m = 0; m < 20; ++m) {
        auto run = [&]() {
            switch (m) {
                case 0: hipLaunchKernelGGL(rw<0>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 1: hipLaunchKernelGGL(rw<1>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 2: hipLaunchKernelGGL(rw<2>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 3: hipLaunchKernelGGL(rw<3>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 4: hipLaunchKernelGGL(rw<4>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 5: hipLaunchKernelGGL(rw<5>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 6: hipLaunchKernelGGL(rw<6>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 7: hipLaunchKernelGGL(rw<7>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 8: hipLaunchKernelGGL(rw<8>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 10: hipLaunchKernelGGL(rw<9>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 11: hipLaunchKernelGGL(rw<10>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 12: hipLaunchKernelGGL(rw<11>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 13: hipLaunchKernelGGL(rw<12>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 14: hipLaunchKernelGGL(rw<13>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 15: hipLaunchKernelGGL(rw<14>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 16: hipLaunchKernelGGL(rw<15>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 17: hipLaunchKernelGGL(rw<16>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 18: hipLaunchKernelGGL(rw<17>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                case 19: hipLaunchKernelGGL(rw<18>, dim3(256 * bpc), dim3(256), 0, 0, buf, n, st); break;
                default: hipLaunchKernelGGL(scatter, dim3(256 * bpc), dim3(256), 0, 0, buf, n, (const uint32_t*)st); break;
            }
        };
        for (int i = 0; i < 3; ++i) run();
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < 10; ++i) run();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 10;
        if (rnd) printf("%-20s blocks/CU=%d %8.4f ms %7.1f GB/s(read)\n", names[m], bpc, ms, n * 1536 / ms / 1e6);
    }
    // Sequences like the bench step (emit on A, then verify = read-only pass on B), so that write-backs
    // leaking into the next kernel are counted.
    uint8_t* bufB;
    CK(hipMalloc(&bufB, n * 1536));
    CK(hipMemset(bufB, 0x44, n * 1536));
    const char* seqn[] = {"B read only", "A read + B read", "A 2x2B + B read", "A 64B + B read", "A compact + scatter + B read",
                          "A compact + scatter_wt + B read", "A 2x2B sc0sc1 + B read", "A compact + scatter", "A compact + scatter_wt",
                          "A compact64 + scatter64 + B read", "A compact64 + B read", "A compact64 + scatter64", "A 64B nt + B read",
                          "A compact + scatter_rr + B read", "A compact + scatter_rr"};
    for (int rnd = 0; rnd < 2; ++rnd)
    for (int q = 0; q < 15; ++q) {
        const int bpc = 2;
        auto run = [&]() {
            dim3 g(256 * bpc), b(256);
            switch (q) {
                case 0: break;
                case 1: hipLaunchKernelGGL(rw<0>, g, b, 0, 0, buf, n, st); break;
                case 2: hipLaunchKernelGGL(rw<1>, g, b, 0, 0, buf, n, st); break;
                case 3: hipLaunchKernelGGL(rw<3>, g, b, 0, 0, buf, n, st); break;
                case 4: case 7: hipLaunchKernelGGL(rw<8>, g, b, 0, 0, buf, n, st);
                        hipLaunchKernelGGL(scatter, g, b, 0, 0, buf, n, (const uint32_t*)st); break;
                case 5: case 8: hipLaunchKernelGGL(rw<8>, g, b, 0, 0, buf, n, st);
                        hipLaunchKernelGGL(scatter_wt, g, b, 0, 0, buf, n, (const uint32_t*)st); break;
                case 6: hipLaunchKernelGGL(rw<9>, g, b, 0, 0, buf, n, st); break;
                case 9: case 11: hipLaunchKernelGGL(rw<17>, g, b, 0, 0, buf, n, st);
                        hipLaunchKernelGGL(scatter64, g, b, 0, 0, buf, n, st); break;
                case 10: hipLaunchKernelGGL(rw<17>, g, b, 0, 0, buf, n, st); break;
                case 12: hipLaunchKernelGGL(rw<18>, g, b, 0, 0, buf, n, st); break;
                case 13: case 14: hipLaunchKernelGGL(rw<8>, g, b, 0, 0, buf, n, st);
                        hipLaunchKernelGGL(scatter_rr, g, b, 0, 0, buf, n, (const uint32_t*)st); break;
            }
            if (q < 7 || q == 9 || q == 10 || q == 12 || q == 13) hipLaunchKernelGGL(rw<0>, g, b, 0, 0, bufB, n, st);
        };
        for (int i = 0; i < 3; ++i) run();
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < 10; ++i) run();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 10;
        if (rnd) printf("SEQ %-34s %8.4f ms\n", seqn[q], ms);
    }
    CK(hipGetLastError());
    return 0;
}
