// tools/smallchunk_bench.hip — variant study for small-chunk byte-wise
// encodes (BASELINE configs[3]: RS(8,2), 4 KiB chunks, 65536 stripes).
//
// Not part of the product.  Same arithmetic as gf8_kernel.hpp (v_perm
// tables in LDS, 3-input XOR folding, Vandermonde row/column 0 as XORs),
// timed interleaved in one process, varying only the work decomposition:
//   base      one 16-B unit per thread, one tile per block (the product)
//   uN        N units per thread (all loads issued before any math)
//   pB        persistent grid of B blocks per CU, grid-stride over tiles,
//             tables staged once per block, next tile prefetched
//   xor       the base decomposition with XOR-only math (memory ceiling of
//             the access pattern)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Imemec_amd/csrc tools/smallchunk_bench.hip -o tools/smallchunk_bench
//   ./tools/smallchunk_bench [k=8] [m=2] [chunk=4096] [stripes=65536] [rounds=7]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gf8_kernel.hpp"

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

using namespace mec;
using namespace mec::detail;

constexpr int KMAX = 16, RMAX = 4;

struct Args {
    const uint8_t *src;
    uint8_t *dst;
    uint64_t sss, dss, cs;
    uint32_t units, tps, total_tiles;  // units per chunk, tiles per stripe, tiles
    Gf8Coef coef[RMAX][KMAX];
};

template <int K, int R>
__device__ __forceinline__ void stage(const Args &a, uint32_t *tab, int bt) {
    for (int t = threadIdx.x; t < R * K; t += bt) {
        const Gf8Coef c = a.coef[t / K][t % K];
        tab[t * 8 + 0] = c.t0;
        tab[t * 8 + 1] = c.t1;
        tab[t * 8 + 2] = c.u0;
        tab[t * 8 + 3] = c.u1;
        tab[t * 8 + 4] = c.v;
    }
    __syncthreads();
}

// U units per thread of tile `tile`: loads, math, stores.
template <int K, int R, int BT, int U, bool XOR>
__device__ __forceinline__ void do_tile(const Args &a, const uint32_t *tab, uint32_t tile) {
    const uint32_t stripe = tile / a.tps;
    const uint32_t u0 = (tile - stripe * a.tps) * (BT * U) + threadIdx.x;
    const uint8_t *sb = a.src + stripe * a.sss;
    uint8_t *db = a.dst + stripe * a.dss;
    u32x4 d[U][K];
#pragma unroll
    for (int r = 0; r < U; ++r) {
        const uint32_t u = u0 + r * BT;
        if (u < a.units) {
#pragma unroll
            for (int j = 0; j < K; ++j) d[r][j] = ld_nt<u32x4>(sb + j * a.cs + uint64_t(u) * 16);
        }
    }
#pragma unroll
    for (int r = 0; r < U; ++r) {
        const uint32_t u = u0 + r * BT;
        if (u >= a.units) continue;
        u32x4 acc[R];
#pragma unroll
        for (int i = 0; i < R; ++i) acc[i] = u32x4{0, 0, 0, 0};
        if (XOR) {
#pragma unroll
            for (int j = 0; j < K; ++j)
#pragma unroll
                for (int i = 0; i < R; ++i) acc[i] ^= d[r][j];
        } else {
            gf8_apply<K, R, kGf8Vand>(d[r], acc, tab + opaque_zero());
        }
#pragma unroll
        for (int i = 0; i < R; ++i) st_nt<u32x4>(db + i * a.cs + uint64_t(u) * 16, acc[i]);
    }
}

template <int K, int R, int BT, int U, bool XOR>
__global__ __launch_bounds__(BT) void k_tiled(const Args a) {
    __shared__ uint32_t tab[R * K * 8];
    stage<K, R>(a, tab, BT);
    do_tile<K, R, BT, U, XOR>(a, tab, blockIdx.x);
}

template <int K, int R, int BT, int U>
__global__ __launch_bounds__(BT) void k_persist(const Args a) {
    __shared__ uint32_t tab[R * K * 8];
    stage<K, R>(a, tab, BT);
    for (uint32_t tile = blockIdx.x; tile < a.total_tiles; tile += gridDim.x) do_tile<K, R, BT, U, false>(a, tab, tile);
}

__global__ void fill_kernel(uint64_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t z = 0x4D454D4543ull + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

struct Variant {
    std::string name;
    void (*launch)(const Args &, uint32_t units, hipStream_t, int cus);
};

// WPC > 0: cap the resident waves per CU at WPC by giving every block a
// share of the 160 KiB LDS (the kernels use only the small coefficient table).
template <int K, int R, int BT, int U, bool XOR, int WPC = 0>
void launch_tiled(const Args &a0, uint32_t units, hipStream_t s, int) {
    Args a = a0;
    a.tps = (units + BT * U - 1) / (BT * U);
    const uint64_t stripes = a.total_tiles;  // holds the stripe count on entry
    a.total_tiles = uint32_t(stripes * a.tps);
    size_t lds = 0;
    if (WPC > 0) {
        const int blocks = std::max(1, WPC / (BT / 64));
        lds = (160 * 1024) / blocks - R * K * 32 - 256;
    }
    hipLaunchKernelGGL((k_tiled<K, R, BT, U, XOR>), dim3(a.total_tiles), dim3(BT), lds, s, a);
}

template <int K, int R, int BT, int U, int PER_CU>
void launch_persist(const Args &a0, uint32_t units, hipStream_t s, int cus) {
    Args a = a0;
    a.tps = (units + BT * U - 1) / (BT * U);
    const uint64_t stripes = a.total_tiles;
    a.total_tiles = uint32_t(stripes * a.tps);
    const uint32_t grid = std::min<uint32_t>(a.total_tiles, uint32_t(cus * PER_CU));
    hipLaunchKernelGGL((k_persist<K, R, BT, U>), dim3(grid), dim3(BT), 0, s, a);
}

// GF(2^8) multiply, poly 0x11d (host)
static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) p ^= a;
        const bool hi = a & 0x80;
        a <<= 1;
        if (hi) a ^= 0x1d;
        b >>= 1;
    }
    return p;
}

template <int K, int R>
std::vector<Variant> variants() {
    return {
        {"base(64x1)", launch_tiled<K, R, 64, 1, false>},
        {"xor(64x1)", launch_tiled<K, R, 64, 1, true>},
        {"256x1", launch_tiled<K, R, 256, 1, false>},
        {"u2(64x2)", launch_tiled<K, R, 64, 2, false>},
        {"u4(64x4)", launch_tiled<K, R, 64, 4, false>},
        {"u4(256x4)", launch_tiled<K, R, 256, 4, false>},
        {"64x1/w8", launch_tiled<K, R, 64, 1, false, 8>},
        {"64x1/w12", launch_tiled<K, R, 64, 1, false, 12>},
        {"64x1/w16", launch_tiled<K, R, 64, 1, false, 16>},
        {"64x1/w20", launch_tiled<K, R, 64, 1, false, 20>},
        {"64x1/w24", launch_tiled<K, R, 64, 1, false, 24>},
        {"64x1/w32", launch_tiled<K, R, 64, 1, false, 32>},
        {"256x1/w8", launch_tiled<K, R, 256, 1, false, 8>},
        {"256x1/w12", launch_tiled<K, R, 256, 1, false, 12>},
        {"256x1/w16", launch_tiled<K, R, 256, 1, false, 16>},
        {"256x1/w24", launch_tiled<K, R, 256, 1, false, 24>},
        {"xor64/w12", launch_tiled<K, R, 64, 1, true, 12>},
        {"xor64/w16", launch_tiled<K, R, 64, 1, true, 16>},
    };
}

template <int K, int R>
int run(uint64_t cs, uint32_t stripes, int rounds) {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    uint8_t *src, *dst;
    const uint64_t sbytes = uint64_t(stripes) * K * cs, dbytes = uint64_t(stripes) * R * cs;
    CHECK(hipMalloc(&src, sbytes));
    CHECK(hipMalloc(&dst, dbytes));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, nullptr, reinterpret_cast<uint64_t *>(src), sbytes / 8);
    CHECK(hipDeviceSynchronize());
    // Jerasure-like Vandermonde coefficients: row 0 and column 0 all ones
    uint8_t A[RMAX][KMAX];
    for (int i = 0; i < R; ++i)
        for (int j = 0; j < K; ++j) A[i][j] = (i == 0 || j == 0) ? 1 : uint8_t(3 + 7 * i + 13 * j);
    Args a{};
    a.src = src;
    a.dst = dst;
    a.cs = cs;
    a.sss = K * cs;
    a.dss = R * cs;
    a.units = uint32_t(cs / 16);
    a.total_tiles = stripes;
    for (int i = 0; i < R; ++i)
        for (int j = 0; j < K; ++j) a.coef[i][j] = gf8_coef(A[i][j]);
    auto vs = variants<K, R>();
    std::vector<std::vector<float>> ms(vs.size());
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // reference output of the base variant for a correctness check
    const uint64_t cbytes = std::min<uint64_t>(dbytes, 64ull << 20);  // compared prefix
    std::vector<uint8_t> ref(cbytes), got(cbytes);
    for (size_t v = 0; v < vs.size(); ++v) {
        CHECK(hipMemsetAsync(dst, 0, dbytes, s));
        vs[v].launch(a, a.units, s, cus);
        CHECK(hipStreamSynchronize(s));
        CHECK(hipMemcpy(v == 0 ? ref.data() : got.data(), dst, cbytes, hipMemcpyDeviceToHost));
        if (v > 0 && vs[v].name.rfind("xor", 0) != 0 && got != ref) printf("MISMATCH %s\n", vs[v].name.c_str());
    }
    // spot-check the base output against a host computation (stripe 0 and last)
    for (uint32_t st : {0u, uint32_t(cbytes / (R * cs)) - 1}) {
        std::vector<uint8_t> h(K * cs);
        CHECK(hipMemcpy(h.data(), src + uint64_t(st) * K * cs, K * cs, hipMemcpyDeviceToHost));
        for (int i = 0; i < R; ++i)
            for (uint64_t b = 0; b < cs; ++b) {
                uint8_t p = 0;
                for (int j = 0; j < K; ++j) p ^= gmul(A[i][j], h[j * cs + b]);
                if (p != ref[(uint64_t(st) * R + i) * cs + b]) {
                    printf("BASE WRONG at stripe %u row %d byte %llu\n", st, i, (unsigned long long)b);
                    return 1;
                }
            }
    }
    const double bytes = double(sbytes + dbytes);
    for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
            for (int w = 0; w < 3; ++w) vs[v].launch(a, a.units, s, cus);
            CHECK(hipEventRecord(e0, s));
            const int reps = 10;
            for (int w = 0; w < reps; ++w) vs[v].launch(a, a.units, s, cus);
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float t = 0;
            CHECK(hipEventElapsedTime(&t, e0, e1));
            ms[v].push_back(t / reps);
        }
    printf("RS(%d,%d) chunk %llu, %u stripes, %.3f GB per launch, %d CUs\n", K, R, (unsigned long long)cs, stripes,
           bytes / 1e9, cus);
    for (size_t v = 0; v < vs.size(); ++v) {
        std::vector<float> t = ms[v];
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2], best = t[0];
        printf("  %-12s median %8.1f us  %6.1f %% of 8 TB/s   (best %6.1f %%)\n", vs[v].name.c_str(), med * 1e3,
               bytes / (med * 1e-3) / 8e12 * 100, bytes / (best * 1e-3) / 8e12 * 100);
    }
    CHECK(hipFree(src));
    CHECK(hipFree(dst));
    return 0;
}

int main(int argc, char **argv) {
    const int k = argc > 1 ? atoi(argv[1]) : 8, m = argc > 2 ? atoi(argv[2]) : 2;
    const uint64_t cs = argc > 3 ? strtoull(argv[3], nullptr, 10) : 4096;
    const uint32_t stripes = argc > 4 ? atoi(argv[4]) : 65536;
    const int rounds = argc > 5 ? atoi(argv[5]) : 7;
    if (k == 8 && m == 2) return run<8, 2>(cs, stripes, rounds);
    if (k == 4 && m == 2) return run<4, 2>(cs, stripes, rounds);
    if (k == 10 && m == 4) return run<10, 4>(cs, stripes, rounds);
    if (k == 12 && m == 2) return run<12, 2>(cs, stripes, rounds);
    fprintf(stderr, "unsupported k,m\n");
    return 2;
}
