// tools/layout_bench.hip — HBM layout study for the 10-read / 4-write
// stripe stream (RS(10,4), 1 MiB chunks, 4096 stripes).  Not product code.
//
// Same XOR-only kernel (one 16-B unit per lane, nt loads/stores, 256-thread
// blocks, tiles of a stripe on consecutive blocks) over several placements
// of the 14 chunks, interleaved in one process:
//   split         data [S][10][C], parity [S][4][C] in two allocations
//   inplace       one [S][14][C] buffer, read chunks 0..9, write 10..13
//   inplace+pad   stripe stride 14C + pad
//   chunkpad      chunk stride C + pad inside the stripe
//   xcd           inplace, block id swizzled so each XCD owns whole stripes
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/layout_bench.hip -o tools/layout_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e = (x);                                                                       \
        if (e != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));     \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int K = 10, R = 4;
constexpr uint64_t CS = 1 << 20;
constexpr uint32_t TILES = CS / 16 / 256;

struct P {
    const uint8_t *src;
    uint8_t *dst;
    uint64_t sss, scs, dss, dcs;
    uint32_t stripes, swz, win, winx;
};

__global__ __launch_bounds__(256) void xork(const P p) {
    uint32_t b = blockIdx.x;
    if (p.swz) {  // runs of swz consecutive logical blocks stay on one XCD (b % 8)
        const uint32_t L = p.swz, q = b / 8;
        b = (q / L) * (8 * L) + (b % 8) * L + q % L;
    }
    if (p.win) {  // p.win windows of the grid in flight at once
        const uint32_t W = p.win, per = gridDim.x / W;
        if (p.winx) {  // window chosen by XCD-ish bits (b % W)
            b = (b % W) * per + b / W;
        } else {  // window chosen by bits 3.. (each XCD visits every window)
            const uint32_t w = (b / 8) % W, rest = (b % 8) + 8 * (b / (8 * W));
            b = w * per + rest;
        }
    }
    const uint32_t stripe = b / TILES, tile = b % TILES;
    const uint64_t off = (uint64_t(tile) * 256 + threadIdx.x) * 16;
    const uint8_t *sb = p.src + stripe * p.sss + off;
    uint8_t *db = p.dst + stripe * p.dss + off;
    u32x4 d[K];
#pragma unroll
    for (int j = 0; j < K; ++j) d[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(sb + j * p.scs));
#pragma unroll
    for (int i = 0; i < R; ++i) {
        u32x4 a = d[i];
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (j != i) a ^= d[j] + u32x4{uint32_t(i), 0, 0, 0};
        __builtin_nontemporal_store(a, reinterpret_cast<u32x4 *>(db + i * p.dcs));
    }
}

int main(int argc, char **argv) {
    const uint32_t S = argc > 1 ? atoi(argv[1]) : 4096;
    const int rounds = argc > 2 ? atoi(argv[2]) : 4;
    const uint64_t pad = 2 << 20;  // max stripe pad tried (inplace+2M)
    const uint64_t big = uint64_t(S) * (14 * CS + pad) + 64 * pad;
    uint8_t *buf, *par;
    CHECK(hipMalloc(&buf, big));
    CHECK(hipMalloc(&par, uint64_t(S) * R * CS));
    CHECK(hipMemset(buf, 0x5a, big));
    struct V {
        const char *name;
        P p;
    };
    std::vector<V> vs;
    auto inplace = [&](uint64_t spad, uint64_t cpad, uint32_t swz) {
        P p;
        p.src = buf;
        p.scs = CS + cpad;
        p.sss = 14 * p.scs + spad;
        p.dst = buf + 10 * p.scs;
        p.dcs = p.scs;
        p.dss = p.sss;
        p.stripes = S;
        p.swz = swz;
        p.win = p.winx = 0;
        return p;
    };
    vs.push_back({"split", P{buf, par, 10 * CS, CS, 4 * CS, CS, S, 0, 0, 0}});
    vs.push_back({"inplace", inplace(0, 0, 0)});
    vs.push_back({"inplace+1M(=15C)", inplace(CS, 0, 0)});
    vs.push_back({"inplace+2M(=16C)", inplace(2 * CS, 0, 0)});
    const uint32_t runs[] = {S * TILES / 8};
    static char names[32][48];
    int ni = 0;
    for (uint32_t L : runs) {
        snprintf(names[ni], 48, "inplace run%u", L);
        vs.push_back({names[ni++], inplace(0, 0, L)});
        snprintf(names[ni], 48, "split run%u", L);
        vs.push_back({names[ni++], P{buf, par, 10 * CS, CS, 4 * CS, CS, S, L, 0, 0}});
    }
    static char wn[32][48];
    int wi = 0;
    for (uint32_t W : {2u, 4u, 8u, 16u, 32u})
        for (uint32_t x : {0u, 1u}) {
            P a = inplace(0, 0, 0);
            a.win = W;
            a.winx = x;
            snprintf(wn[wi], 48, "inplace win%u%s", W, x ? " (b%W)" : " (b/8%W)");
            vs.push_back({wn[wi++], a});
            P c{buf, par, 10 * CS, CS, 4 * CS, CS, S, 0, W, x};
            snprintf(wn[wi], 48, "split win%u%s", W, x ? " (b%W)" : " (b/8%W)");
            vs.push_back({wn[wi++], c});
        }
    vs.push_back({"split (src stride 14C)", P{buf, par, 14 * CS, CS, 4 * CS, CS, S, 0, 0, 0}});
    vs.push_back({"split (dst stride 14C)", P{buf, buf + 10 * CS, 10 * CS, CS, 14 * CS, CS, S, 0, 0, 0}});
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<float> best(vs.size(), 1e30f);
    for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
            hipLaunchKernelGGL(xork, dim3(S * TILES), dim3(256), 0, 0, vs[v].p);
            CHECK(hipEventRecord(e0, 0));
            for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(xork, dim3(S * TILES), dim3(256), 0, 0, vs[v].p);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            best[v] = std::min(best[v], ms / 3);
        }
    const double bytes = double(S) * 14 * CS;
    for (size_t v = 0; v < vs.size(); ++v)
        printf("%-24s %8.3f ms %8.1f GB/s %5.1f%%\n", vs[v].name, best[v], bytes / best[v] / 1e6,
               bytes / best[v] / 1e6 / 80.0);
    return 0;
}
