// tools/stream_probe.hip — what HBM3E rate does this part sustain for
// streams of different read/write mixes?  The coding kernels read k chunks
// and write m (RS(10,4): 10 reads : 4 writes); this prices the mix itself
// with no arithmetic, so the ceiling quoted in DESIGN.md §4 is measured, not
// assumed.  Not part of the product.
//
// Every kernel: one 16-byte non-temporal unit per lane per stream, one-wave
// blocks over 1 KiB column tiles of [stripe][chunk] buffers (the product's
// split-layout shape), resident waves capped through dynamic LDS.
//   R reads, W writes per tile: (R, W) in {(1,0), (0,1), (1,1), (2,1), (10,4), (8,2)}
// Read-only tiles fold their data into one dword per wave that is stored only
// if it matches an impossible value (keeps the loads live, no write traffic).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Imemec_amd/csrc tools/stream_probe.hip -o tools/stream_probe
//   ./tools/stream_probe [gib=8] [rounds=5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "stream_common.hpp"

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

using namespace mec::detail;

template <int R, int W>
__global__ __launch_bounds__(64) void k_stream(const uint8_t *src, uint8_t *dst, uint64_t cs, uint32_t tiles,
                                               uint32_t *sink) {
    const uint32_t stripe = blockIdx.x / tiles, t = blockIdx.x % tiles;
    const uint64_t off = uint64_t(t) * 1024 + threadIdx.x * 16;
    u32x4 acc{0, 0, 0, 0};
    if constexpr (R > 0) {
        const uint8_t *s = src + uint64_t(stripe) * R * cs + off;
        u32x4 x[R];
#pragma unroll
        for (int j = 0; j < R; ++j) x[j] = ld_nt<u32x4>(s + j * cs);
#pragma unroll
        for (int j = 0; j < R; ++j) acc ^= x[j];
    } else {
        acc = u32x4{stripe, t, threadIdx.x, 0x4D454D45u};
    }
    if constexpr (W > 0) {
        uint8_t *d = dst + uint64_t(stripe) * W * cs + off;
#pragma unroll
        for (int i = 0; i < W; ++i) st_nt<u32x4>(d + i * cs, acc + u32x4{uint32_t(i), 0, 0, 0});
    } else {
        const uint32_t v = acc.x ^ acc.y ^ acc.z ^ acc.w;
        if (v == 0x9E3779B9u && threadIdx.x == 0) sink[0] = v;  // keeps the loads live
    }
}

static size_t cap_lds(uint32_t wpc) {
    if (!wpc) return 0;
    const size_t per = (160u << 10) / wpc / 512 * 512;
    return per > 512 ? per - 512 : 0;
}

struct Buf {
    uint8_t *src, *dst;
    uint32_t *sink;
};

typedef void (*Fn)(const Buf &, uint64_t cs, uint32_t stripes, uint32_t wpc, hipStream_t);

template <int R, int W>
void run(const Buf &b, uint64_t cs, uint32_t stripes, uint32_t wpc, hipStream_t s) {
    const uint32_t tiles = uint32_t(cs / 1024);
    hipLaunchKernelGGL((k_stream<R, W>), dim3(stripes * tiles), dim3(64), cap_lds(wpc), s, b.src, b.dst, cs, tiles,
                       b.sink);
}

struct Shape {
    const char *name;
    int r, w;
    Fn fn;
};

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 8.0;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t cs = 1 << 20;
    const Shape shapes[] = {
        {"read-only 1R", 1, 0, run<1, 0>},     {"read-only 10R", 10, 0, run<10, 0>}, {"write-only 1W", 0, 1, run<0, 1>},
        {"write-only 4W", 0, 4, run<0, 4>},    {"copy 1R1W", 1, 1, run<1, 1>},     {"xor 2R1W", 2, 1, run<2, 1>},
        {"rs(8,2) 8R2W", 8, 2, run<8, 2>},     {"rs(10,4) 10R4W", 10, 4, run<10, 4>},
    };
    const uint32_t caps[] = {0, 8, 12, 16, 24};
    Buf b{};
    const uint64_t total = uint64_t(gib * double(1ull << 30));
    CHECK(hipMalloc(&b.src, total));
    CHECK(hipMalloc(&b.dst, total));
    CHECK(hipMalloc(&b.sink, 64));
    CHECK(hipMemset(b.src, 0x5a, total));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    printf("1 MiB chunks, ~%.1f GiB moved per launch, one-wave blocks, median of %d rounds x 5 launches\n", gib,
           rounds);
    for (const Shape &sh : shapes) {
        // stripes so that reads + writes ~= gib, each side within its buffer
        const uint32_t per = uint32_t(sh.r + sh.w);
        const uint32_t stripes = uint32_t(total / (per * cs));
        const double bytes = double(stripes) * per * cs;
        std::vector<std::vector<float>> ms(sizeof(caps) / sizeof(caps[0]));
        for (int r = 0; r < rounds; ++r)
            for (size_t c = 0; c < ms.size(); ++c) {
                sh.fn(b, cs, stripes, caps[c], st);
                CHECK(hipEventRecord(e0, st));
                for (int i = 0; i < 5; ++i) sh.fn(b, cs, stripes, caps[c], st);
                CHECK(hipEventRecord(e1, st));
                CHECK(hipEventSynchronize(e1));
                float t = 0;
                CHECK(hipEventElapsedTime(&t, e0, e1));
                ms[c].push_back(t / 5);
            }
        printf("  %-16s", sh.name);
        for (size_t c = 0; c < ms.size(); ++c) {
            std::sort(ms[c].begin(), ms[c].end());
            const double med = ms[c][ms[c].size() / 2];
            printf("  w%-2u %6.1f GB/s %5.1f %%", caps[c], bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12 * 100);
        }
        printf("\n");
    }
    return 0;
}
