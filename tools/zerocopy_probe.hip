// tools/zerocopy_probe.hip — can the coding kernels stream host memory
// directly (zero-copy over PCIe) instead of staging through HBM?  Not
// product code.  Measures, on hipHostRegister'ed malloc memory:
//   dma_h2d / dma_d2h    hipMemcpyAsync rates (pinned)
//   zc_read              kernel reading host memory (16 B per lane)
//   zc_xor 10->4         the RS(10,4) stream shape: 10 host chunks read,
//                        4 host chunks written, per stripe
//   small-call latency   one 4 KiB-chunk RS(8,2) stripe: launch + sync,
//                        zero-copy vs H2D + kernel + D2H
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/zerocopy_probe.hip -o tools/zerocopy_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void rd(const u32x4 *p, uint64_t n, u32x4 *sink) {
    u32x4 a{0, 0, 0, 0};
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256)
        a ^= __builtin_nontemporal_load(p + i);
    if (a.x == 0x12345678u) sink[0] = a;
}

// stripes of K chunks of cs bytes (host), outputs R chunks (host)
template <int K, int R>
__global__ __launch_bounds__(256) void xk(const uint8_t *src, uint8_t *dst, uint64_t cs, uint32_t tiles) {
    const uint32_t s = blockIdx.x / tiles, t = blockIdx.x % tiles;
    const uint64_t off = (uint64_t(t) * 256 + threadIdx.x) * 16;
    if (off >= cs) return;
    const uint8_t *sb = src + uint64_t(s) * K * cs + off;
    uint8_t *db = dst + uint64_t(s) * R * cs + off;
    u32x4 d[K];
#pragma unroll
    for (int j = 0; j < K; ++j) d[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(sb + j * cs));
#pragma unroll
    for (int i = 0; i < R; ++i) {
        u32x4 a = d[i];
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (j != i) a ^= d[j];
        __builtin_nontemporal_store(a, reinterpret_cast<u32x4 *>(db + i * cs));
    }
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const uint64_t cs = 1 << 20, S = 64, K = 10, R = 4;
    const uint64_t sb = S * K * cs, db = S * R * cs;
    uint8_t *hs = static_cast<uint8_t *>(aligned_alloc(4096, sb));
    uint8_t *hd = static_cast<uint8_t *>(aligned_alloc(4096, db));
    memset(hs, 0x5a, sb);
    memset(hd, 0, db);
    CHECK(hipHostRegister(hs, sb, hipHostRegisterMapped));
    CHECK(hipHostRegister(hd, db, hipHostRegisterMapped));
    uint8_t *ds, *dd;
    CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&ds), hs, 0));
    CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&dd), hd, 0));
    printf("host %p -> device %p (same VA: %d)\n", (void *)hs, (void *)ds, hs == ds);
    uint8_t *gs, *gd;
    u32x4 *sink;
    CHECK(hipMalloc(&gs, sb));
    CHECK(hipMalloc(&gd, db));
    CHECK(hipMalloc(&sink, 16));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timeit = [&](auto fn, int reps) {
        fn();
        CHECK(hipStreamSynchronize(st));
        CHECK(hipEventRecord(e0, st));
        for (int i = 0; i < reps; ++i) fn();
        CHECK(hipEventRecord(e1, st));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        return ms / reps;
    };
    float t;
    t = timeit([&] { CHECK(hipMemcpyAsync(gs, hs, sb, hipMemcpyHostToDevice, st)); }, 3);
    printf("dma_h2d        %8.3f ms  %6.1f GB/s\n", t, sb / t / 1e6);
    t = timeit([&] { CHECK(hipMemcpyAsync(hd, gd, db, hipMemcpyDeviceToHost, st)); }, 3);
    printf("dma_d2h        %8.3f ms  %6.1f GB/s\n", t, db / t / 1e6);
    for (int grid : {1024, 4096, 16384}) {
        t = timeit([&] { hipLaunchKernelGGL(rd, dim3(grid), dim3(256), 0, st, (const u32x4 *)ds, sb / 16, sink); }, 3);
        printf("zc_read g%-5d %8.3f ms  %6.1f GB/s\n", grid, t, sb / t / 1e6);
    }
    const uint32_t tiles = cs / 16 / 256;
    t = timeit([&] { hipLaunchKernelGGL((xk<10, 4>), dim3(S * tiles), dim3(256), 0, st, ds, dd, cs, tiles); }, 3);
    printf("zc_xor 10->4   %8.3f ms  %6.1f GB/s data (%.1f GB/s PCIe both ways)\n", t, sb / t / 1e6, (sb + db) / t / 1e6);
    t = timeit([&] {
        CHECK(hipMemcpyAsync(gs, hs, sb, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL((xk<10, 4>), dim3(S * tiles), dim3(256), 0, st, gs, gd, cs, tiles);
        CHECK(hipMemcpyAsync(hd, gd, db, hipMemcpyDeviceToHost, st));
    }, 3);
    printf("staged 10->4   %8.3f ms  %6.1f GB/s data (serial H2D, kernel, D2H)\n", t, sb / t / 1e6);
    // small-call latency: one RS(8,2) 4 KiB stripe, host wall clock per call
    {
        const uint64_t c4 = 4096;
        const uint32_t t4 = 1;
        const int n = 2000;
        double a = now();
        for (int i = 0; i < n; ++i) {
            hipLaunchKernelGGL((xk<8, 2>), dim3(t4), dim3(256), 0, st, ds, dd, c4, t4);
            CHECK(hipStreamSynchronize(st));
        }
        double zc = (now() - a) / n * 1e6;
        a = now();
        for (int i = 0; i < n; ++i) {
            CHECK(hipMemcpyAsync(gs, hs, 8 * c4, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL((xk<8, 2>), dim3(t4), dim3(256), 0, st, gs, gd, c4, t4);
            CHECK(hipMemcpyAsync(hd, gd, 2 * c4, hipMemcpyDeviceToHost, st));
            CHECK(hipStreamSynchronize(st));
        }
        double stg = (now() - a) / n * 1e6;
        printf("small call RS(8,2) 4 KiB: zero-copy %.1f us, staged %.1f us per call\n", zc, stg);
    }
    // correctness of the zero-copy output for stripe 0, chunk 0
    CHECK(hipStreamSynchronize(st));
    printf("check: %s\n", hd[0] == (0x5a ^ 0x5a ^ 0x5a ^ 0x5a ^ 0x5a ^ 0x5a ^ 0x5a ^ 0x5a) ? "ok" : "mismatch");
    return 0;
}
