// tools/ldsdma_probe.hip — does streaming the sources through LDS-DMA
// (global_load_lds_dwordx4) raise the HBM stream ceiling that libmec's
// kernels sit at?    Not part of the product.
//
// Two shapes, each timed interleaved (medians of rounds):
//   xor     d = a ^ b over 3 x GiB buffers (mec_xor's stream: 2 reads, 1 write)
//   rs104   10 sources -> 4 outputs of XORs over [stripe][chunk] buffers
//           (RS(10,4) encode's traffic with XOR-only math)
// and three loaders:
//   direct   one unit per lane, non-temporal dwordx4 loads to VGPRs (the
//            product's form), one-wave blocks, the product's wave cap
//   glds     persistent one-wave blocks; each wave streams its tiles through
//            a private ring of DEPTH LDS slots filled by
//            global_load_lds_dwordx4 (a wave-instruction moves 1 KiB), waits
//            with a counted vmcnt, reads back with ds_read_b128
//   glds-nt  the same with the non-temporal cache policy on the DMA
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Imemec_amd/csrc tools/ldsdma_probe.hip -o tools/ldsdma_probe
//   ./tools/ldsdma_probe [gib=8] [rounds=5]
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

typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

// one 16-byte-per-lane DMA: 1 KiB per wave-instruction into LDS at `l`
// (wave-uniform base; lane i lands at l + 16 i)
template <int AUX>
__device__ __forceinline__ void glds16(const uint8_t *g, void *l) {
    __builtin_amdgcn_global_load_lds((gvoid *)(g), (lvoid *)(l), 16, 0, AUX);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- direct loads (the product's form) --------------------------------------
template <int K, int R>
__global__ __launch_bounds__(64) void k_direct(const uint8_t *src, uint8_t *dst, uint64_t cs, uint32_t tiles) {
    const uint32_t stripe = blockIdx.x / tiles, t = blockIdx.x % tiles;
    const uint64_t off = uint64_t(t) * 1024 + threadIdx.x * 16;
    const uint8_t *s = src + uint64_t(stripe) * K * cs + off;
    uint8_t *d = dst + uint64_t(stripe) * R * cs + off;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld_nt<u32x4>(s + j * cs);
#pragma unroll
    for (int i = 0; i < R; ++i) {
        u32x4 acc = x[0];
#pragma unroll
        for (int j = 1; j < K; ++j) acc ^= (i + j) & 1 ? x[j] : (x[j] >> 1);
        st_nt<u32x4>(d + i * cs, acc);
    }
}

// ---- LDS-DMA ring ------------------------------------------------------------
// A wave owns work items w = wave, wave + nwaves, ...; item = (stripe, 1 KiB
// column tile).  Ring slot q holds the K source tiles of one item.  Per
// iteration: wait for the item's K DMAs (counted: the later items' DMAs and
// stores may stay in flight), read, compute, store, refill the slot with the
// item DEPTH ahead.
template <int K, int R, int DEPTH, int AUX>
__global__ __launch_bounds__(64) void k_glds(const uint8_t *src, uint8_t *dst, uint64_t cs, uint32_t tiles,
                                             uint32_t items) {
    extern __shared__ u32x4 ring[];  // [DEPTH][K][64]
    const uint32_t lane = threadIdx.x;
    const uint32_t nw = gridDim.x;
    auto issue = [&](uint32_t item, int q) {
        const uint32_t stripe = item / tiles, t = item % tiles;
        const uint8_t *s = src + uint64_t(stripe) * K * cs + uint64_t(t) * 1024 + lane * 16;
#pragma unroll
        for (int j = 0; j < K; ++j) glds16<AUX>(s + j * cs, &ring[(q * K + j) * 64]);
    };
#pragma unroll
    for (int q = 0; q < DEPTH; ++q) {
        const uint32_t item = blockIdx.x + q * nw;
        if (item < items) issue(item, q);
    }
    uint32_t n = 0;
    for (uint32_t item = blockIdx.x; item < items; item += nw, ++n) {
        const int q = int(n % DEPTH);
        // ops issued after this item's K DMAs: per later iteration R stores
        // + K DMAs; waiting for (DEPTH - 1) * K outstanding is safe either way
        wait_vm<(DEPTH - 1) * K>();
        u32x4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = ring[(q * K + j) * 64 + lane];
        const uint32_t stripe = item / tiles, t = item % tiles;
        uint8_t *d = dst + uint64_t(stripe) * R * cs + uint64_t(t) * 1024 + lane * 16;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            u32x4 acc = x[0];
#pragma unroll
            for (int j = 1; j < K; ++j) acc ^= (i + j) & 1 ? x[j] : (x[j] >> 1);
            st_nt<u32x4>(d + i * cs, acc);
        }
        // the slot's LDS reads must finish before the DMA overwrites it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint32_t next = item + DEPTH * nw;
        if (next < items) issue(next, q);
    }
    wait_vm<0>();
}

__global__ void fill_kernel(uint64_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t z = 0x4D454D4543ull + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

struct Shape {
    uint8_t *src, *dst;
    uint64_t cs;
    uint32_t stripes, tiles;
    int cus;
};

typedef void (*Fn)(const Shape &, uint32_t arg, hipStream_t);

static size_t cap_lds(uint32_t wpc, size_t used) {
    if (!wpc) return used;
    const size_t per = (160u << 10) / wpc / 512 * 512;
    return std::max(per > 512 ? per - 512 : 0, used);
}

template <int K, int R>
void run_direct(const Shape &s, uint32_t wpc, hipStream_t st) {
    hipLaunchKernelGGL((k_direct<K, R>), dim3(s.stripes * s.tiles), dim3(64), cap_lds(wpc, 0), st, s.src, s.dst,
                       s.cs, s.tiles);
}

template <int K, int R, int DEPTH, int AUX>
void run_glds(const Shape &s, uint32_t wpc, hipStream_t st) {
    const size_t ring = size_t(DEPTH) * K * 1024;
    const uint32_t items = s.stripes * s.tiles;
    const uint32_t grid = std::min<uint32_t>(items, uint32_t(s.cus) * wpc);
    hipLaunchKernelGGL((k_glds<K, R, DEPTH, AUX>), dim3(grid), dim3(64), cap_lds(wpc, ring), st, s.src, s.dst, s.cs,
                       s.tiles, items);
}

struct Variant {
    std::string name;
    Fn fn;
    uint32_t arg;
};

template <int K, int R>
int shape(const char *label, uint64_t cs, double gib, int rounds, int cus) {
    const uint64_t per = uint64_t(K + R) * cs;
    const uint32_t stripes = uint32_t(gib * double(1ull << 30) / double(per));
    Shape s{};
    s.cs = cs;
    s.stripes = stripes;
    s.tiles = uint32_t(cs / 1024);
    s.cus = cus;
    const uint64_t sb = uint64_t(stripes) * K * cs, db = uint64_t(stripes) * R * cs;
    CHECK(hipMalloc(&s.src, sb));
    CHECK(hipMalloc(&s.dst, db));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, nullptr, reinterpret_cast<uint64_t *>(s.src), sb / 8);
    CHECK(hipDeviceSynchronize());
    std::vector<Variant> vs = {
        {"direct/w12", run_direct<K, R>, 12},
        {"direct/w16", run_direct<K, R>, 16},
        {"direct/w0", run_direct<K, R>, 0},
        {"glds d2/w8", run_glds<K, R, 2, 0>, 8},
        {"glds d2/w16", run_glds<K, R, 2, 0>, 16},
        {"glds d3/w8", run_glds<K, R, 3, 0>, 8},
        {"glds d3/w12", run_glds<K, R, 3, 0>, 12},
        {"glds-nt d2/w8", run_glds<K, R, 2, 2>, 8},
        {"glds-nt d2/w16", run_glds<K, R, 2, 2>, 16},
        {"glds-nt d3/w8", run_glds<K, R, 3, 2>, 8},
        {"glds-nt d3/w12", run_glds<K, R, 3, 2>, 12},
    };
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    // every variant writes the same bytes as the first
    const uint64_t cmp = std::min<uint64_t>(db, 64ull << 20);
    std::vector<uint8_t> ref(cmp), got(cmp);
    for (size_t v = 0; v < vs.size(); ++v) {
        CHECK(hipMemsetAsync(s.dst, 0, db, st));
        vs[v].fn(s, vs[v].arg, st);
        CHECK(hipStreamSynchronize(st));
        CHECK(hipMemcpy(v ? got.data() : ref.data(), s.dst, cmp, hipMemcpyDeviceToHost));
        if (v && got != ref) {
            printf("MISMATCH %s\n", vs[v].name.c_str());
            return 1;
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ms(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
            vs[v].fn(s, vs[v].arg, st);
            CHECK(hipEventRecord(e0, st));
            for (int i = 0; i < 5; ++i) vs[v].fn(s, vs[v].arg, st);
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float t = 0;
            CHECK(hipEventElapsedTime(&t, e0, e1));
            ms[v].push_back(t / 5);
        }
    const double bytes = double(sb + db);
    printf("%s: K=%d R=%d chunk %llu, %u stripes, %.2f GB per launch\n", label, K, R, (unsigned long long)cs, stripes,
           bytes / 1e9);
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(ms[v].begin(), ms[v].end());
        const double med = ms[v][ms[v].size() / 2];
        printf("  %-16s median %9.1f us  %7.1f GB/s  %5.1f %% of 8 TB/s\n", vs[v].name.c_str(), med * 1e3,
               bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12 * 100);
    }
    CHECK(hipFree(s.src));
    CHECK(hipFree(s.dst));
    return 0;
}

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 8.0;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    int rc = shape<2, 1>("xor", 1 << 20, gib, rounds, cus);
    if (!rc) rc = shape<10, 4>("rs104", 1 << 20, gib, rounds, cus);
    return rc;
}
