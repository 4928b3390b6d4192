// tools/tile_probe.hip — memory-pattern probe for wide codes on small chunks
// (ISA-L Cauchy(20,8)@4 KiB at 75.5 %, its XOR twin 75.9 %).
//
// Same bytes as a split encode ([stripe][ns][chunk] in, [stripe][nd][chunk]
// out), arithmetic reduced to one XOR per source and output, so only the
// access pattern varies: U 16-byte units per lane 1 KiB apart (a wave covers
// U KiB of every chunk of its stripe), 64- or 256-thread blocks, a wave cap
// per CU through dynamic LDS, XCD runs on or off.  Prints one JSON line per
// arm: % of 8 TB/s on (ns + nd) * chunk bytes per stripe.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/tile_probe.hip -o tools/tile_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *a, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(a), 0, int(bytes), 0x00020000);
}

// One wave codes U KiB of every chunk of one stripe (tile t of the stripe);
// a 256-thread block is four such waves on four consecutive tiles.
template <int NS, int ND, int U>
__global__ __launch_bounds__(256) void probe(const uint8_t *src, uint8_t *dst, uint32_t chunk, uint32_t tiles,
                                             uint32_t nwaves, uint32_t xcd) {
    extern __shared__ uint32_t lds_pad[];
    const uint32_t wpb = blockDim.x >> 6;
    uint32_t bid = blockIdx.x;
    if (xcd) {
        const uint32_t per = gridDim.x >> 3;
        if (bid < per * 8u) bid = (bid & 7u) * per + (bid >> 3);
    }
    const uint32_t w = bid * wpb + (threadIdx.x >> 6);
    if (w >= nwaves) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t stripe = w / tiles, tile = w - stripe * tiles;
    const uint32_t off = tile * (U * 1024u) + lane * 16u;
    const uint8_t *s0 = src + size_t(stripe) * NS * chunk;
    uint8_t *d0 = dst + size_t(stripe) * ND * chunk;
    u32x4 acc[ND][U];
#pragma unroll
    for (int r = 0; r < ND; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) acc[r][u] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(s0 + size_t(j) * chunk, chunk), off + u * 1024u, 0, 2);
#pragma unroll
        for (int r = 0; r < ND; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) acc[r][u] ^= x[u] + uint32_t(r);
    }
#pragma unroll
    for (int r = 0; r < ND; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(acc[r][u], rsrc(d0 + size_t(r) * chunk, chunk), off + u * 1024u, 0, 18);
    if (lane == 64u) lds_pad[0] = 0;  // keeps the dynamic LDS allocation
}

template <int NS, int ND, int U>
static void arm(const uint8_t *src, uint8_t *dst, uint32_t chunk, uint32_t stripes, int block, int cap, int xcd,
                const char *name) {
    const uint32_t tiles = chunk / (U * 1024u);
    const uint32_t nwaves = stripes * tiles;
    const uint32_t wpb = uint32_t(block / 64);
    const uint32_t grid = (nwaves + wpb - 1) / wpb;
    // waves per CU <= cap: each block takes 160 KiB * wpb / cap of LDS
    size_t lds = cap > 0 ? (160u * 1024u * wpb) / uint32_t(cap) : 0;
    if (lds > 65536) lds = 65536;
    lds &= ~size_t(255);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 5; ++i)
        probe<NS, ND, U><<<grid, block, lds>>>(src, dst, chunk, tiles, nwaves, uint32_t(xcd));
    CK(hipGetLastError());
    const int iters = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i)
        probe<NS, ND, U><<<grid, block, lds>>>(src, dst, chunk, tiles, nwaves, uint32_t(xcd));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= iters;
    const double bytes = double(stripes) * (NS + ND) * chunk;
    std::printf("{\"shape\": \"%s\", \"ns\": %d, \"nd\": %d, \"chunk\": %u, \"stripes\": %u, \"units\": %d, \"block\": %d, "
                "\"cap\": %d, \"xcd\": %d, \"ms\": %.4f, \"frac\": %.4f}\n",
                name, NS, ND, chunk, stripes, U, block, cap, xcd, ms, bytes / (ms * 1e-3) / 8e12);
    std::fflush(stdout);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

template <int NS, int ND>
static void shape(uint32_t chunk, uint32_t stripes, const char *name, const std::vector<int> &caps) {
    uint8_t *src, *dst;
    CK(hipMalloc(&src, size_t(stripes) * NS * chunk));
    CK(hipMalloc(&dst, size_t(stripes) * ND * chunk));
    CK(hipMemset(src, 0x5a, size_t(stripes) * NS * chunk));
    for (int rep = 0; rep < 2; ++rep)
        for (int cap : caps)
            for (int xcd = 0; xcd < 2; ++xcd) {
                arm<NS, ND, 1>(src, dst, chunk, stripes, 64, cap, xcd, name);
                arm<NS, ND, 1>(src, dst, chunk, stripes, 256, cap, xcd, name);
                arm<NS, ND, 2>(src, dst, chunk, stripes, 64, cap, xcd, name);
                if (chunk >= 4096) arm<NS, ND, 4>(src, dst, chunk, stripes, 64, cap, xcd, name);
            }
    CK(hipFree(src));
    CK(hipFree(dst));
}

int main(int argc, char **argv) {
    const int which = argc > 1 ? std::atoi(argv[1]) : 0;
    const std::vector<int> caps = {4, 6, 8, 12, 0};
    if (which == 0 || which == 1) shape<20, 8>(4096, 65536, "20+8@4K", caps);
    if (which == 0 || which == 2) shape<16, 8>(4096, 65536, "16+8@4K", caps);
    if (which == 0 || which == 3) shape<8, 2>(4096, 65536, "8+2@4K", caps);
    if (which == 0 || which == 4) shape<10, 4>(1048576, 1024, "10+4@1M", caps);
    return 0;
}
