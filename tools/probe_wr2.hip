// Write-timing probe: does an in-place field store cost less when it follows the read of its own
// line closely?  2^20 records of 1536 B, 16 lanes x 6 non-temporal dwordx4 loads per record (the
// walk kernel's access pattern), then two 2-B stores into the record's first line, in modes:
//   0 read only
//   1 all loads at once, stores after the sum (today's emit)
//   2 the record's first 128-B line loaded LAST (after the rest has arrived and been summed, its
//     address made dependent on that sum), stores right after it
//   3 as 2, stores as one whole 64-B line (the line's bytes, patched)
//   4 scatter only: the two 2-B stores per record, no reads (stride 1536)
//   5 scatter only at stride 4608 (three times the buffer span per store)
//   6 as 1, the first line loaded with a plain (cached) load
//   7 as 1, stores as the whole first 64-B line (the line's bytes, patched)
//   8 as 1, stores as the whole first 128-B line
// Standalone tool; results in DESIGN.md §5.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#define GMEM __attribute__((address_space(1)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t sum4(const u32x4& v, uint32_t acc) {
    return __builtin_amdgcn_sad_u16(v.x, 0, __builtin_amdgcn_sad_u16(v.y, 0, __builtin_amdgcn_sad_u16(v.z, 0, __builtin_amdgcn_sad_u16(v.w, 0, acc))));
}
__device__ __forceinline__ uint32_t red16(uint32_t acc) {
    acc += __shfl_xor(acc, 1, 16); acc += __shfl_xor(acc, 2, 16); acc += __shfl_xor(acc, 4, 16); acc += __shfl_xor(acc, 8, 16);
    return acc;
}

template <int MODE>
__global__ __launch_bounds__(256) void rw(uint8_t* buf, uint64_t n, uint32_t stride) {
    const int lane = threadIdx.x & 15;
    const uint64_t r = (uint64_t)blockIdx.x * 16 + threadIdx.x / 16;
    if (r >= n) return;
    const uint64_t a0 = (uint64_t)buf + r * 1536;
    if (MODE == 4 || MODE == 5) {
        if (lane == 0) {
            const uint64_t q = (uint64_t)buf + r * stride;
            *(GMEM uint16_t*)(q + 10) = (uint16_t)r;
            *(GMEM uint16_t*)(q + 26) = (uint16_t)(r >> 16);
        }
        return;
    }
    uint32_t acc = 0;
    u32x4 head = {0, 0, 0, 0};
    if (MODE == 2 || MODE == 3) {
        u32x4 v[6];
#pragma unroll
        for (int u = 0; u < 6; ++u) {
            const int c = u * 16 + lane;
            v[u] = __builtin_nontemporal_load((const GMEM u32x4*)(a0 + 16 * (c < 8 ? 8 : c)));
        }
#pragma unroll
        for (int u = 0; u < 6; ++u)
            if (u * 16 + lane >= 8) acc = sum4(v[u], acc);
        // the first line, requested only now (its address depends on the sum)
        const uint64_t hl = a0 + 16 * (lane & 7) + (acc == 0xdeadbeefu ? 16 : 0);
        head = __builtin_nontemporal_load((const GMEM u32x4*)hl);
        if (lane < 8) acc = sum4(head, acc);
    } else {
        u32x4 v[6];
#pragma unroll
        for (int u = 0; u < 6; ++u) {
            const GMEM u32x4* q = (const GMEM u32x4*)(a0 + 16 * (u * 16 + lane));
            v[u] = (MODE == 6 && u == 0) ? *q : __builtin_nontemporal_load(q);
        }
        head = v[0];
#pragma unroll
        for (int u = 0; u < 6; ++u) acc = sum4(v[u], acc);
    }
    acc = red16(acc);
    if (MODE == 0) {
        if (acc == 0x12345678u) buf[0] = 1;
    } else if (MODE == 3 || MODE == 7 || MODE == 8) {
        if (lane < (MODE == 8 ? 8 : 4)) {
            u32x4 c = head;
            if (lane == 0) c.z = (c.z & 0xffff0000u) | (acc & 0xffffu);
            if (lane == 1) c.z = (c.z & 0xffff0000u) | (acc >> 16);
            *(GMEM u32x4*)(a0 + 16 * lane) = c;
        }
    } else if (lane == 0) {
        *(GMEM uint16_t*)(a0 + 10) = (uint16_t)acc;
        *(GMEM uint16_t*)(a0 + 26) = (uint16_t)(acc >> 16);
    }
}

int main() {
    const uint64_t n = 1 << 20;
    uint8_t* buf;
    CK(hipMalloc(&buf, 3 * n * 1536 + 4096));
    CK(hipMemset(buf, 0x33, 3 * n * 1536 + 4096));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[] = {"read only", "loads at once + 2x2B stores", "first line last + 2x2B stores",
                           "first line last + 64-B line store", "scatter only, stride 1536", "scatter only, stride 4608",
                           "first line cached + 2x2B stores", "loads at once + 64-B line store",
                           "loads at once + 128-B line store"};
    const dim3 g((unsigned)(n / 16)), blk(256);
    for (int rnd = 0; rnd < 3; ++rnd)
        for (int m = 0; m < 9; ++m) {
            auto run = [&]() {
                switch (m) {
                    case 0: hipLaunchKernelGGL(rw<0>, g, blk, 0, 0, buf, n, 1536u); break;
                    case 1: hipLaunchKernelGGL(rw<1>, g, blk, 0, 0, buf, n, 1536u); break;
                    case 2: hipLaunchKernelGGL(rw<2>, g, blk, 0, 0, buf, n, 1536u); break;
                    case 3: hipLaunchKernelGGL(rw<3>, g, blk, 0, 0, buf, n, 1536u); break;
                    case 4: hipLaunchKernelGGL(rw<4>, g, blk, 0, 0, buf, n, 1536u); break;
                    case 5: hipLaunchKernelGGL(rw<5>, g, blk, 0, 0, buf, n, 4608u); break;
                    case 6: hipLaunchKernelGGL(rw<6>, g, blk, 0, 0, buf, n, 1536u); break;
                    case 7: hipLaunchKernelGGL(rw<7>, g, blk, 0, 0, buf, n, 1536u); break;
                    default: hipLaunchKernelGGL(rw<8>, g, blk, 0, 0, buf, n, 1536u); break;
                }
            };
            for (int i = 0; i < 3; ++i) run();
            CK(hipEventRecord(a, 0));
            for (int i = 0; i < 20; ++i) run();
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ms /= 20;
            if (rnd) printf("{\"round\": %d, \"mode\": %d, \"what\": \"%s\", \"ms\": %.4f}\n", rnd, m, names[m], ms);
        }
    CK(hipFree(buf));
    return 0;
}
