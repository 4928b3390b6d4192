// tools/microbench.hip — variant study for the RS(10,4) 1 MiB encode stream.
//
// Not part of the product.  Times, interleaved in one process (rule 24),
// kernels that share the gf8 access pattern (10 chunk reads + 4 chunk
// writes per 16-B unit) but differ in arithmetic, cache policy, units per
// thread and block size, plus plain read / write / copy ceilings.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench.hip -o tools/microbench
//   ./tools/microbench [stripes=4096] [rounds=5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int K = 10, R = 4;
constexpr uint64_t CS = 1 << 20;

struct Coef {
    uint32_t t0, t1, u0, u1, v;
};
struct Args {
    const uint8_t *src;
    uint8_t *dst;
    uint32_t units, tiles, upt;
    Coef coef[R][K];
};

enum Mode { kFull = 0, kXorOnly = 1 };

__device__ __forceinline__ uint32_t gmul(const Coef &c, uint32_t x) {
    uint32_t s0 = x & 0x07070707u, s1 = (x >> 3) & 0x07070707u, s2 = (x >> 6) & 0x03030303u;
    return __builtin_amdgcn_perm(c.t1, c.t0, s0) ^ __builtin_amdgcn_perm(c.u1, c.u0, s1) ^
           __builtin_amdgcn_perm(c.v, c.v, s2);
}

template <int MODE, bool NTL, bool NTS, int BS>
__global__ __launch_bounds__(BS) void enc(const Args a) {
    const uint32_t stripe = blockIdx.x / a.tiles, tile = blockIdx.x - stripe * a.tiles;
    const uint8_t *sb = a.src + uint64_t(stripe) * K * CS;
    uint8_t *db = a.dst + uint64_t(stripe) * R * CS;
    const uint32_t ub = tile * a.upt * BS + threadIdx.x;
    for (uint32_t r = 0; r < a.upt; ++r) {
        uint32_t u = ub + r * BS;
        if (u >= a.units) return;
        uint64_t off = uint64_t(u) * 16;
        u32x4 d[K], acc[R];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const u32x4 *p = reinterpret_cast<const u32x4 *>(sb + j * CS + off);
            d[j] = NTL ? __builtin_nontemporal_load(p) : *p;
        }
#pragma unroll
        for (int i = 0; i < R; ++i) acc[i] = u32x4{0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
            for (int i = 0; i < R; ++i) {
                if (MODE == kXorOnly) {
                    acc[i] ^= d[j];
                } else {
                    acc[i].x ^= gmul(a.coef[i][j], d[j].x);
                    acc[i].y ^= gmul(a.coef[i][j], d[j].y);
                    acc[i].z ^= gmul(a.coef[i][j], d[j].z);
                    acc[i].w ^= gmul(a.coef[i][j], d[j].w);
                }
            }
#pragma unroll
        for (int i = 0; i < R; ++i) {
            u32x4 *p = reinterpret_cast<u32x4 *>(db + i * CS + off);
            if (NTS)
                __builtin_nontemporal_store(acc[i], p);
            else
                *p = acc[i];
        }
    }
}


// Variant: coefficient tables staged in LDS, read back by broadcast into
// VGPRs (no SGPR pressure, no constant-bus copies).  ONES: 0 = none,
// 1 = compile-time row0/col0 ones skip, 2 = runtime mask skip.
template <int ONES, bool NTL, bool NTS, int BS, bool PF, bool OPQ = false>
__global__ __launch_bounds__(BS) void enc_lds(const Args a, uint64_t ones_mask) {
    __shared__ uint32_t tab[R * K * 8];
    for (int i = threadIdx.x; i < R * K; i += BS) {
        const Coef c = a.coef[i / K][i % K];
        tab[i * 8 + 0] = c.t0; tab[i * 8 + 1] = c.t1; tab[i * 8 + 2] = c.u0; tab[i * 8 + 3] = c.u1; tab[i * 8 + 4] = c.v;
    }
    __syncthreads();
    const uint32_t stripe = blockIdx.x / a.tiles, tile = blockIdx.x - stripe * a.tiles;
    const uint8_t *sb = a.src + uint64_t(stripe) * K * CS;
    uint8_t *db = a.dst + uint64_t(stripe) * R * CS;
    const uint32_t ub = tile * a.upt * BS + threadIdx.x;
    u32x4 d[K];
    auto load = [&](uint32_t u) {
        uint64_t off = uint64_t(u) * 16;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const u32x4 *p = reinterpret_cast<const u32x4 *>(sb + j * CS + off);
            d[j] = NTL ? __builtin_nontemporal_load(p) : *p;
        }
    };
    if (ub >= a.units) return;
    load(ub);
    for (uint32_t r = 0; r < a.upt; ++r) {
        uint32_t u = ub + r * BS;
        if (u >= a.units) return;
        uint64_t off = uint64_t(u) * 16;
        u32x4 cur[K];
#pragma unroll
        for (int j = 0; j < K; ++j) cur[j] = d[j];
        if (PF && r + 1 < a.upt && u + BS < a.units) load(u + BS);
        u32x4 acc[R];
#pragma unroll
        for (int i = 0; i < R; ++i) acc[i] = u32x4{0, 0, 0, 0};
        int z = 0;
        if (OPQ) asm volatile("s_mov_b32 %0, 0" : "=s"(z));
        const uint32_t *tb = tab + z;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const u32x4 x = cur[j];
            const u32x4 s0 = x & 0x07070707u, s1 = (x >> 3) & 0x07070707u, s2 = (x >> 6) & 0x03030303u;
#pragma unroll
            for (int i = 0; i < R; ++i) {
                bool one = ONES == 1 ? (i == 0 || j == 0) : ONES == 2 ? ((ones_mask >> (i * K + j)) & 1) : false;
                if (one) { acc[i] ^= x; continue; }
                const u32x4 t = *reinterpret_cast<const u32x4 *>(&tb[(i * K + j) * 8]);
                const uint32_t v = tb[(i * K + j) * 8 + 4];
                acc[i].x ^= __builtin_amdgcn_perm(t.y, t.x, s0.x) ^ __builtin_amdgcn_perm(t.w, t.z, s1.x) ^ __builtin_amdgcn_perm(v, v, s2.x);
                acc[i].y ^= __builtin_amdgcn_perm(t.y, t.x, s0.y) ^ __builtin_amdgcn_perm(t.w, t.z, s1.y) ^ __builtin_amdgcn_perm(v, v, s2.y);
                acc[i].z ^= __builtin_amdgcn_perm(t.y, t.x, s0.z) ^ __builtin_amdgcn_perm(t.w, t.z, s1.z) ^ __builtin_amdgcn_perm(v, v, s2.z);
                acc[i].w ^= __builtin_amdgcn_perm(t.y, t.x, s0.w) ^ __builtin_amdgcn_perm(t.w, t.z, s1.w) ^ __builtin_amdgcn_perm(v, v, s2.w);
            }
            if (OPQ) __builtin_amdgcn_sched_barrier(0);
        }
        if (!PF && r + 1 < a.upt && u + BS < a.units) load(u + BS);
#pragma unroll
        for (int i = 0; i < R; ++i) {
            u32x4 *p = reinterpret_cast<u32x4 *>(db + i * CS + off);
            if (NTS) __builtin_nontemporal_store(acc[i], p); else *p = acc[i];
        }
    }
}

__global__ void read_only(const u32x4 *src, uint64_t n, uint32_t *sink) {
    u32x4 acc{0, 0, 0, 0};
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
        acc ^= src[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}
__global__ void write_only(u32x4 *dst, uint64_t n) {
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
        dst[i] = u32x4{uint32_t(i), 1, 2, 3};
}
__global__ void copy_k(const u32x4 *src, u32x4 *dst, uint64_t n) {
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
        dst[i] = src[i];
}

struct Variant {
    std::string name;
    void (*launch)(const Args &, uint32_t stripes, hipStream_t);
    double bytes;
    uint32_t upt;
};

template <int MODE, bool NTL, bool NTS, int BS>
void launch_enc(const Args &a0, uint32_t stripes, hipStream_t s) {
    Args a = a0;
    a.tiles = (a.units + a.upt * BS - 1) / (a.upt * BS);
    hipLaunchKernelGGL((enc<MODE, NTL, NTS, BS>), dim3(stripes * a.tiles), dim3(BS), 0, s, a);
}


template <int ONES, bool NTL, bool NTS, int BS, bool PF, bool OPQ = false>
void launch_lds(const Args &a0, uint32_t stripes, hipStream_t s) {
    Args a = a0;
    a.tiles = (a.units + a.upt * BS - 1) / (a.upt * BS);
    uint64_t mask = 0;
    for (int i = 0; i < R; ++i) for (int j = 0; j < K; ++j) if (i == 0 || j == 0) mask |= 1ull << (i * K + j);
    hipLaunchKernelGGL((enc_lds<ONES, NTL, NTS, BS, PF, OPQ>), dim3(stripes * a.tiles), dim3(BS), 0, s, a, mask);
}

int main(int argc, char **argv) {
    uint32_t stripes = argc > 1 ? atoi(argv[1]) : 4096;
    int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t dbytes = uint64_t(stripes) * K * CS, pbytes = uint64_t(stripes) * R * CS;
    uint8_t *src, *dst;
    uint32_t *sink;
    CHECK(hipMalloc(&src, dbytes));
    CHECK(hipMalloc(&dst, pbytes));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(src, 0x5a, dbytes));
    // random-ish data so DVFS sees real bit flips
    {
        std::vector<uint32_t> h(1 << 20);
        uint64_t x = 88172645463325252ull;
        for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = uint32_t(x); }
        for (uint64_t off = 0; off < dbytes; off += h.size() * 4)
            CHECK(hipMemcpy(src + off, h.data(), std::min<uint64_t>(h.size() * 4, dbytes - off), hipMemcpyHostToDevice));
    }
    Args a;
    a.src = src;
    a.dst = dst;
    a.units = CS / 16;
    for (int i = 0; i < R; ++i)
        for (int j = 0; j < K; ++j) a.coef[i][j] = Coef{0x03020100u + i, 0x07060504u + j, 0x18100800u, 0x38302820u, 0xc0804000u};
    const double alg = double(dbytes + pbytes);
    std::vector<Variant> vs = {
        {"full ntboth upt4 (old)", launch_enc<kFull, true, true, 256>, alg, 4},
        {"lds nt upt1 opq", launch_lds<0, true, true, 256, false, true>, alg, 1},
        {"lds nt ones-rt upt1 opq", launch_lds<2, true, true, 256, false, true>, alg, 1},
        {"lds nt ones-rt upt4 opq", launch_lds<2, true, true, 256, false, true>, alg, 4},
        {"lds nt ones-ct upt4 opq", launch_lds<1, true, true, 256, false, true>, alg, 4},
        {"lds nt ones-rt upt4 pf opq", launch_lds<2, true, true, 256, true, true>, alg, 4},
        {"lds nt upt1", launch_lds<0, true, true, 256, false>, alg, 1},
        {"lds nt upt4", launch_lds<0, true, true, 256, false>, alg, 4},
        {"lds nt ones-ct upt1", launch_lds<1, true, true, 256, false>, alg, 1},
        {"lds nt ones-rt upt1", launch_lds<2, true, true, 256, false>, alg, 1},
        {"lds nt ones-rt upt4", launch_lds<2, true, true, 256, false>, alg, 4},
        {"lds nt ones-rt upt4 pf", launch_lds<2, true, true, 256, true>, alg, 4},
        {"lds nt ones-rt upt8 pf", launch_lds<2, true, true, 256, true>, alg, 8},
        {"lds ones-rt upt1 (no nt)", launch_lds<2, false, false, 256, false>, alg, 1},
        {"lds nt ones-rt upt1 bs512", launch_lds<2, true, true, 512, false>, alg, 1},
        {"lds nt ones-rt upt2 bs128", launch_lds<2, true, true, 128, false>, alg, 2},
        {"xor-only ntboth upt4", launch_enc<kXorOnly, true, true, 256>, alg, 4},
        {"xor-only ntboth upt1", launch_enc<kXorOnly, true, true, 256>, alg, 1},
    };
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size() + 3);
    const uint64_t n16 = dbytes / 16, p16 = pbytes / 16;
    for (int rd = 0; rd < rounds; ++rd) {
        for (size_t v = 0; v < vs.size(); ++v) {
            a.upt = vs[v].upt;
            vs[v].launch(a, stripes, s);  // warm
            CHECK(hipEventRecord(e0, s));
            for (int it = 0; it < 3; ++it) vs[v].launch(a, stripes, s);
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / 3);
        }
        float ms;
        CHECK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(read_only, dim3(256 * 32), dim3(256), 0, s, (const u32x4 *)src, n16, sink);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        t[vs.size()].push_back(ms);
        CHECK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(write_only, dim3(256 * 32), dim3(256), 0, s, (u32x4 *)dst, p16);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        t[vs.size() + 1].push_back(ms);
        CHECK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(copy_k, dim3(256 * 32), dim3(256), 0, s, (const u32x4 *)src, (u32x4 *)(src + dbytes / 2),
                           n16 / 2);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        t[vs.size() + 2].push_back(ms);
    }
    auto report = [&](const char *name, std::vector<float> &v, double bytes) {
        std::sort(v.begin(), v.end());
        printf("%-26s median %8.3f ms  min %8.3f ms  %7.1f GB/s (%.1f%% of 8 TB/s)\n", name, v[v.size() / 2], v[0],
               bytes / (v[v.size() / 2] * 1e-3) / 1e9, 100 * bytes / (v[v.size() / 2] * 1e-3) / 8e12);
    };
    for (size_t v = 0; v < vs.size(); ++v) report(vs[v].name.c_str(), t[v], vs[v].bytes);
    report("read-only (data)", t[vs.size()], double(dbytes));
    report("write-only (parity)", t[vs.size() + 1], double(pbytes));
    report("copy 1:1 (data/2)", t[vs.size() + 2], double(dbytes));
    return 0;
}
