// Copy-bandwidth probe: the read+write ceiling a fused copy + emit is measured against.
// hipMemcpyAsync device-to-device and wave-contiguous copy kernels (plain / non-temporal).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#define GMEM __attribute__((address_space(1)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int UNR, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void wave_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint64_t w0 = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const uint64_t per = 64ull * UNR;
    for (uint64_t base = w0 * per; base + per <= n16; base += nw * per) {
        u32x4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const GMEM u32x4* q = (const GMEM u32x4*)(src + base + u * 64 + lane);
            v[u] = NTL ? __builtin_nontemporal_load(q) : *q;
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            GMEM u32x4* q = (GMEM u32x4*)(dst + base + u * 64 + lane);
            if (NTS) __builtin_nontemporal_store(v[u], q); else *q = v[u];
        }
    }
}

// Strided copy like the C2 payloads: record r's 1472 B from src + r*1472 to dst + r*1500 + 28.
__global__ __launch_bounds__(256) void rec_copy(const uint8_t* src, uint8_t* dst, uint64_t n) {
    const int lane = threadIdx.x & 15;
    const uint64_t ng = (uint64_t)gridDim.x * 16;
    for (uint64_t r = (uint64_t)blockIdx.x * 16 + threadIdx.x / 16; r < n; r += ng) {
        const GMEM uint32_t* s = (const GMEM uint32_t*)(src + r * 1472);
        GMEM uint32_t* d = (GMEM uint32_t*)(dst + r * 1500 + 28);
        for (int i = lane; i < 368; i += 16) d[i] = s[i];
    }
}

// Same, but every byte of the destination records is written (the 28 header bytes too): no line
// is left partially dirty.
__global__ __launch_bounds__(256) void rec_copy_full(const uint8_t* src, uint8_t* dst, uint64_t n) {
    const int lane = threadIdx.x & 15;
    const uint64_t ng = (uint64_t)gridDim.x * 16;
    for (uint64_t r = (uint64_t)blockIdx.x * 16 + threadIdx.x / 16; r < n; r += ng) {
        const GMEM uint32_t* s = (const GMEM uint32_t*)(src + r * 1472);
        GMEM uint32_t* d = (GMEM uint32_t*)(dst + r * 1500);
        for (int i = lane; i < 375; i += 16) d[i] = i < 7 ? 0x01020304u : s[i - 7];
    }
}


// 16-B chunks, 8 lanes per record (natural grid: one record per group), source bytes funnel-shifted
// from two aligned 16-B loads like the fused copy-emit.  OWN_LINES: group r writes the 128-B lines
// whose first byte lies in its record, whole (every destination line written once, by one
// group); else it writes only [28, 1500) of its record, with byte stores on the two edge chunks
// (the partial lines the fused kernel leaves today).
__device__ __forceinline__ u32x4 funnel(const u32x4& lo, const u32x4& hi, uint32_t sh) {
    const uint32_t q = sh >> 2, b = sh & 3u;
    auto pick = [&](uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
        return q == 0 ? a0 : q == 1 ? a1 : q == 2 ? a2 : a3;
    };
    const uint32_t x0 = pick(lo.x, lo.y, lo.z, lo.w), x1 = pick(lo.y, lo.z, lo.w, hi.x);
    const uint32_t x2 = pick(lo.z, lo.w, hi.x, hi.y), x3 = pick(lo.w, hi.x, hi.y, hi.z);
    const uint32_t x4 = pick(hi.x, hi.y, hi.z, hi.w);
    u32x4 r;
    r.x = __builtin_amdgcn_alignbyte(x1, x0, b);
    r.y = __builtin_amdgcn_alignbyte(x2, x1, b);
    r.z = __builtin_amdgcn_alignbyte(x3, x2, b);
    r.w = __builtin_amdgcn_alignbyte(x4, x3, b);
    return r;
}

template <bool OWN_LINES>
__global__ __launch_bounds__(256) void rec_copy16(const uint8_t* src, uint8_t* dst, uint64_t n) {
    const int lane = threadIdx.x & 7;
    const uint64_t r = (uint64_t)blockIdx.x * 32 + threadIdx.x / 8;
    if (r == 0 || r >= n) return;  // record 0's chunk grid would start before the source
    const uint64_t d0 = (uint64_t)dst + r * 1500, d1 = d0 + 1500;
    const uint64_t lo = OWN_LINES ? (r == 0 ? d0 : (d0 + 127) & ~127ull) : d0 + 28;
    const uint64_t hi = OWN_LINES ? (r + 1 == n ? d1 : (d1 + 127) & ~127ull) : d1;
    const uint64_t c0 = lo & ~15ull;
    const uint32_t nch = (uint32_t)((hi - c0 + 15) >> 4);
    const int64_t sdelta = (int64_t)((uint64_t)src + r * 1472) - (int64_t)(d0 + 28);  // src = dst + sdelta
    for (uint32_t k0 = 0; k0 < nch; k0 += 32) {
        u32x4 a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t k = k0 + u * 8 + lane;
            const uint64_t c = c0 + 16ull * (k < nch ? k : 0);
            const uint64_t sa = (uint64_t)((int64_t)c + sdelta);
            a[u] = *(const GMEM u32x4*)(sa & ~15ull);
            b[u] = *(const GMEM u32x4*)((sa & ~15ull) + 16);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t k = k0 + u * 8 + lane;
            if (k >= nch) continue;
            const uint64_t c = c0 + 16ull * k;
            const uint64_t sa = (uint64_t)((int64_t)c + sdelta);
            const u32x4 v = funnel(a[u], b[u], (uint32_t)(sa & 15u));
            if (c >= lo && c + 16 <= hi) {
                *(GMEM u32x4*)c = v;
            } else {
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                for (int j = 0; j < 16; ++j)
                    if (c + j >= lo && c + j < hi) *(GMEM uint8_t*)(c + j) = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
            }
        }
    }
}

// copy_kernel's body path in isolation: 16 lanes per record, aligned 16-B destination chunks, the
// source read from the chunk's first source byte rounded down to 4 (one unaligned dwordx4 load; the
// C2 sources are co-aligned mod 4 with the payload, so the v_alignbyte shift is 0 here).
// HDR: 0 = the group writes the 128-B lines whose first byte lies in its record, whole (as
// rec_copy16 OWN_LINES); 1 = only [28, 1500) (the header bytes are never written: partial lines);
// 2 = [28, 1500), then the record's 28 header bytes after the payload (copy_kernel's order: every
// line ends up whole, its two parts written by two groups at different times); 3 = the header bytes
// first, then the payload.
template <int HDR>
__global__ __launch_bounds__(256) void rec_copy_u4(const uint8_t* src, uint8_t* dst, uint64_t n) {
    const int lane = threadIdx.x & 15;
    const uint64_t r = (uint64_t)blockIdx.x * 16 + threadIdx.x / 16;
    if (r == 0 || r >= n) return;
    const uint64_t d0 = (uint64_t)dst + r * 1500, d1 = d0 + 1500;
    const uint64_t lo = HDR == 0 ? (d0 + 127) & ~127ull : d0 + 28;
    const uint64_t hi = HDR == 0 ? (r + 1 == n ? d1 : (d1 + 127) & ~127ull) : d1;
    const uint64_t c0 = lo & ~15ull;
    const uint32_t nch = (uint32_t)((hi - c0 + 15) >> 4);
    const int64_t sdelta = (int64_t)((uint64_t)src + r * 1472) - (int64_t)(d0 + 28);
    auto header = [&]() {  // 28 header bytes (a constant pattern), dword or byte stores
        if (lane < 7) {
            const uint64_t a = d0 + 4 * lane;
            if ((a & 3u) == 0) *(GMEM uint32_t*)a = 0x45000000u + lane;
            else for (int j = 0; j < 4; ++j) *(GMEM uint8_t*)(a + j) = (uint8_t)(lane + j);
        }
    };
    if (HDR == 3) header();
    for (uint32_t k0 = 0; k0 < nch; k0 += 64) {
        u32x4 a[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t k = k0 + u * 16 + lane;
            const uint64_t c = c0 + 16ull * (k < nch ? k : 0);
            const uint64_t sa = (uint64_t)((int64_t)c + sdelta);
            a[u] = *(const GMEM u32x4*)(sa & ~3ull);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t k = k0 + u * 16 + lane;
            if (k >= nch) continue;
            const uint64_t c = c0 + 16ull * k;
            const uint64_t sa = (uint64_t)((int64_t)c + sdelta);
            const uint32_t bb = (uint32_t)(sa & 3u);
            u32x4 v;
            v.x = __builtin_amdgcn_alignbyte(a[u].y, a[u].x, bb);
            v.y = __builtin_amdgcn_alignbyte(a[u].z, a[u].y, bb);
            v.z = __builtin_amdgcn_alignbyte(a[u].w, a[u].z, bb);
            v.w = __builtin_amdgcn_alignbyte(a[u].w, a[u].w, bb);
            if (c >= lo && c + 16 <= hi) {
                *(GMEM u32x4*)c = v;
            } else {
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                for (int j = 0; j < 16; ++j)
                    if (c + j >= lo && c + j < hi) *(GMEM uint8_t*)(c + j) = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
            }
        }
    }
    if (HDR == 2) header();
}

// 8 lanes per record: each lane loads ALIGNED 16-B source chunks (the C2 source records are 16-B
// aligned, 1472 = 92 x 16) and stores each one UNALIGNED at its destination (dst + r*1500 + 28 +
// 16k, misaligned by (r*1500 + 28) % 16): no funnel shift at all.  FULL: the 28 header bytes are
// written too (two overlapping unaligned 16-B stores), so no line is left partially written.
template <bool FULL>
__global__ __launch_bounds__(256) void rec_copy_unal(const uint8_t* src, uint8_t* dst, uint64_t n) {
    const int lane = threadIdx.x & 7;
    const uint64_t r = (uint64_t)blockIdx.x * 32 + threadIdx.x / 8;
    if (r >= n) return;
    const uint64_t s0 = (uint64_t)src + r * 1472, d0 = (uint64_t)dst + r * 1500;
#pragma unroll
    for (int k0 = 0; k0 < 96; k0 += 32) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + u * 8 + lane;
            v[u] = *(const GMEM u32x4*)(s0 + 16ull * (k < 92 ? k : 91));
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + u * 8 + lane;
            if (k < 92) *(GMEM u32x4*)(d0 + 28 + 16ull * k) = v[u];
        }
    }
    if (FULL && lane < 2) {
        const u32x4 h = {0x45000000u, 0x01020304u, 0x05060708u, 0x090a0b0cu};
        *(GMEM u32x4*)(d0 + 12 * lane) = h;
    }
}

__global__ void check_unal(const uint8_t* src, const uint8_t* dst, uint64_t n, uint32_t* bad) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    for (int i = 0; i < 1472; ++i)
        if (dst[r * 1500 + 28 + i] != src[r * 1472 + i]) { atomicAdd(bad, 1u); return; }
}

int main() {
    const uint64_t bytes = 1500ull << 20;
    uint8_t *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto fn) {
        for (int i = 0; i < 3; ++i) fn();
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 10; ++i) fn();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 10;
        printf("%-36s %8.4f ms  %7.1f GB/s (read+write)\n", name, ms, 2.0 * bytes / ms / 1e6);
    };
    const uint64_t n16 = bytes / 16;
    {  // clock ramp (bench.py --ramp-ms): ~300 ms of copies before anything is timed
        for (int i = 0; i < 600; ++i) CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0));
        CK(hipDeviceSynchronize());
    }
    timeit("hipMemcpyAsync D2D", [&] { CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0)); });
    for (int bpc : {2, 4, 8}) {
        char nm[64];
        snprintf(nm, sizeof nm, "wave_copy U4 plain bpc=%d", bpc);
        timeit(nm, [&] { hipLaunchKernelGGL((wave_copy<4, false, false>), dim3(256 * bpc), dim3(256), 0, 0, (const u32x4*)a, (u32x4*)b, n16); });
        snprintf(nm, sizeof nm, "wave_copy U4 ntload bpc=%d", bpc);
        timeit(nm, [&] { hipLaunchKernelGGL((wave_copy<4, true, false>), dim3(256 * bpc), dim3(256), 0, 0, (const u32x4*)a, (u32x4*)b, n16); });
        snprintf(nm, sizeof nm, "wave_copy U4 nt both bpc=%d", bpc);
        timeit(nm, [&] { hipLaunchKernelGGL((wave_copy<4, true, true>), dim3(256 * bpc), dim3(256), 0, 0, (const u32x4*)a, (u32x4*)b, n16); });
        snprintf(nm, sizeof nm, "wave_copy U4 ntstore bpc=%d", bpc);
        timeit(nm, [&] { hipLaunchKernelGGL((wave_copy<4, false, true>), dim3(256 * bpc), dim3(256), 0, 0, (const u32x4*)a, (u32x4*)b, n16); });
    }
    const uint64_t n = 1ull << 20;
    timeit("rec_copy 1472 B -> stride 1500 (+28)", [&] { hipLaunchKernelGGL(rec_copy, dim3(256 * 8), dim3(256), 0, 0, a, b, n); });
    timeit("rec_copy_full 1500 B (all bytes)", [&] { hipLaunchKernelGGL(rec_copy_full, dim3(256 * 8), dim3(256), 0, 0, a, b, n); });
    timeit("rec_copy16 own lines (whole lines)", [&] { hipLaunchKernelGGL(rec_copy16<true>, dim3(n / 32), dim3(256), 0, 0, a, b, n); });
    timeit("rec_copy16 [28,1500) (partial edges)", [&] { hipLaunchKernelGGL(rec_copy16<false>, dim3(n / 32), dim3(256), 0, 0, a, b, n); });
    timeit("rec_copy_u4 own lines (copy_kernel body)", [&] { hipLaunchKernelGGL(rec_copy_u4<0>, dim3(n / 16), dim3(256), 0, 0, a, b, n); });
    timeit("rec_copy_u4 [28,1500) (partial edges)", [&] { hipLaunchKernelGGL(rec_copy_u4<1>, dim3(n / 16), dim3(256), 0, 0, a, b, n); });
    timeit("rec_copy_u4 payload, then header", [&] { hipLaunchKernelGGL(rec_copy_u4<2>, dim3(n / 16), dim3(256), 0, 0, a, b, n); });
    timeit("rec_copy_u4 header, then payload", [&] { hipLaunchKernelGGL(rec_copy_u4<3>, dim3(n / 16), dim3(256), 0, 0, a, b, n); });
    timeit("rec_copy_unal [28,1500) unaligned 16-B stores", [&] { hipLaunchKernelGGL(rec_copy_unal<false>, dim3(n / 32), dim3(256), 0, 0, a, b, n); });
    timeit("rec_copy_unal all bytes (unaligned)", [&] { hipLaunchKernelGGL(rec_copy_unal<true>, dim3(n / 32), dim3(256), 0, 0, a, b, n); });
    {  // the unaligned stores land where they should (a source with distinct bytes)
        uint8_t* h = (uint8_t*)malloc(n * 1472);
        for (uint64_t i = 0; i < n * 1472; ++i) h[i] = (uint8_t)(i * 2654435761u >> 13);
        CK(hipMemcpy(a, h, n * 1472, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(rec_copy_unal<false>, dim3(n / 32), dim3(256), 0, 0, a, b, n);
        uint32_t* bad; CK(hipMalloc(&bad, 4)); CK(hipMemset(bad, 0, 4));
        hipLaunchKernelGGL(check_unal, dim3(n / 256), dim3(256), 0, 0, a, b, n, bad);
        uint32_t hb = 0; CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
        printf("rec_copy_unal check: %u of %llu records differ\n", hb, (unsigned long long)n);
        free(h);
    }
    CK(hipGetLastError());
    return 0;
}
