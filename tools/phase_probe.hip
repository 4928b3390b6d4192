// tools/phase_probe.hip — does separating reads from writes in time, chip
// wide, raise the rate of a mixed read/write stream?  Not part of the
// product.
//
// The RS(10,4)-shaped XOR stream (10 reads : 4 writes) runs at ~84 % of
// 8 TB/s on this part while read-only streams reach ~90 % and write-only
// ~86 % (tools/stream_probe.hip): mixing costs ~4-5 %.  Here a persistent
// grid of one-wave blocks works in cycles of a fixed period P on the
// chip-wide constant clock (s_memrealtime, 100 MHz): during the read window
// of a cycle every wave reads its next T tiles (10 x 1 KiB each), folds them
// and parks the 4 x 1 KiB results per tile in LDS; during the write window
// it streams the parked results out.  No atomics, no barriers: the windows
// are absolute clock ranges, so all CUs switch together.
//   free    the same batching with no waiting (each wave alternates at its
//           own pace): separates "batched per wave" from "phased chip wide";
//   phased  the clock windows, P = bytes per cycle / (f x 8 TB/s) for a few
//           target fractions f, read share of the window rs.
// Output of every arm is checked against the plain one-tile-per-lane
// kernel.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Imemec_amd/csrc tools/phase_probe.hip -o tools/phase_probe
//   ./tools/phase_probe [rounds=5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

constexpr int K = 10, R = 4;
constexpr uint64_t CS = 1 << 20;            // chunk bytes
constexpr uint32_t TPS = uint32_t(CS / 1024);  // 1 KiB tiles per chunk

// plain reference kernel: one 1 KiB tile per one-wave block
__global__ __launch_bounds__(64) void k_plain(const uint8_t *src, uint8_t *dst) {
    const uint32_t stripe = blockIdx.x / TPS, t = blockIdx.x % TPS;
    const uint64_t off = uint64_t(t) * 1024 + threadIdx.x * 16;
    const uint8_t *s = src + uint64_t(stripe) * K * CS + off;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld_nt<u32x4>(s + j * CS);
    u32x4 acc = x[0];
#pragma unroll
    for (int j = 1; j < K; ++j) acc ^= x[j];
    uint8_t *d = dst + uint64_t(stripe) * R * CS + off;
#pragma unroll
    for (int i = 0; i < R; ++i) st_nt<u32x4>(d + i * CS, acc + u32x4{uint32_t(i), 0, 0, 0});
}

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

// never waits more than 10 ms (a wrong start time cannot hang the grid)
__device__ __forceinline__ void wait_until(uint64_t t) {
    const uint64_t cap = now() + 1000000;
    while (now() < t && now() < cap) __builtin_amdgcn_s_sleep(2);
}

// Persistent: nw waves (one per block), tile g of cycle c for wave w and
// slot q: g = (c * T + q) * nw + w, so at every step the waves cover nw
// consecutive tiles (same XCD affinity as the plain grid when nw % 8 == 0).
// PHASED: read window [base + c*P, base + c*P + PR), write window up to
// base + (c+1)*P; base = the first multiple of P after the kernel started
// (computed per wave from the clock, so every wave agrees).
template <int T, bool PHASED>
__global__ __launch_bounds__(64) void k_phase(const uint8_t *src, uint8_t *dst, uint32_t tiles, uint32_t nw,
                                              uint64_t P, uint64_t PR, uint64_t t_start) {
    extern __shared__ u32x4 park[];  // [T][R][64] per block (one wave)
    const uint32_t w = blockIdx.x, lane = threadIdx.x;
    const uint32_t cycles = (tiles + T * nw - 1) / (T * nw);
    const uint64_t base = (t_start / P + 1) * P;
    for (uint32_t c = 0; c < cycles; ++c) {
        if constexpr (PHASED) wait_until(base + uint64_t(c) * P);
        // all T tiles' loads in flight at once (T x 10 KiB per wave)
        u32x4 x[T][K];
#pragma unroll
        for (int q = 0; q < T; ++q) {
            uint32_t g = (c * T + q) * nw + w;
            if (g >= tiles) g = tiles - 1;  // re-read the last tile, parked but never stored
            const uint32_t stripe = g / TPS, t = g % TPS;
            const uint8_t *s = src + uint64_t(stripe) * K * CS + uint64_t(t) * 1024 + lane * 16;
#pragma unroll
            for (int j = 0; j < K; ++j) x[q][j] = ld_nt<u32x4>(s + j * CS);
        }
#pragma unroll
        for (int q = 0; q < T; ++q) {
            u32x4 acc = x[q][0];
#pragma unroll
            for (int j = 1; j < K; ++j) acc ^= x[q][j];
#pragma unroll
            for (int i = 0; i < R; ++i) park[(q * R + i) * 64 + lane] = acc + u32x4{uint32_t(i), 0, 0, 0};
        }
        if constexpr (PHASED) wait_until(base + uint64_t(c) * P + PR);
#pragma unroll
        for (int q = 0; q < T; ++q) {
            const uint32_t g = (c * T + q) * nw + w;
            if (g >= tiles) break;
            const uint32_t stripe = g / TPS, t = g % TPS;
            uint8_t *d = dst + uint64_t(stripe) * R * CS + uint64_t(t) * 1024 + lane * 16;
#pragma unroll
            for (int i = 0; i < R; ++i) st_nt<u32x4>(d + i * CS, park[(q * R + i) * 64 + lane]);
        }
    }
}

// host clock read on the device: one tiny kernel, so t_start is close to
// the launch that follows it on the same stream
__global__ void k_clock(uint64_t *out) {
    if (threadIdx.x == 0) out[0] = now();
}

struct Arm {
    char name[64];
    int T;
    bool phased;
    uint32_t wpc;
    double f, rs;  // target fraction of 8 TB/s and read share of a cycle
};

template <int T, bool PH>
static void launch_phase(const uint8_t *src, uint8_t *dst, uint32_t tiles, uint32_t nw, uint64_t P, uint64_t PR,
                         uint64_t ts, hipStream_t s) {
    const size_t lds = size_t(T) * R * 64 * 16;
    hipLaunchKernelGGL((k_phase<T, PH>), dim3(nw), dim3(64), lds, s, src, dst, tiles, nw, P, PR, ts);
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const uint32_t stripes = 584;  // ~8 GiB moved per launch
    const uint32_t tiles = stripes * TPS;
    const double bytes = double(stripes) * (K + R) * CS;
    uint8_t *src, *dst, *ref;
    uint64_t *clk;
    CHECK(hipMalloc(&src, size_t(stripes) * K * CS));
    CHECK(hipMalloc(&dst, size_t(stripes) * R * CS));
    CHECK(hipMalloc(&ref, size_t(stripes) * R * CS));
    CHECK(hipMalloc(&clk, 64));
    {
        std::vector<uint32_t> h(size_t(stripes) * K * CS / 4);
        uint32_t x = 0x2468ACE1u;
        for (auto &v : h) v = (x = x * 1664525u + 1013904223u);
        CHECK(hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    hipLaunchKernelGGL(k_plain, dim3(tiles), dim3(64), 0, st, src, ref);
    CHECK(hipStreamSynchronize(st));

    std::vector<Arm> arms;
    // LDS per one-wave block = T x 4 KiB: T = 4 fits 8 waves per CU
    for (int T : {2, 4})
        for (uint32_t wpc : {4u, 8u, 12u}) {
            if (T == 4 && wpc > 8) continue;
            Arm a{};
            snprintf(a.name, sizeof a.name, "free   T%d wpc%u", T, wpc);
            a.T = T, a.phased = false, a.wpc = wpc;
            arms.push_back(a);
            for (double f : {0.78, 0.82, 0.86})
                for (double rs : {0.70, 0.74}) {
                    Arm b = a;
                    snprintf(b.name, sizeof b.name, "phased T%d wpc%u f%.2f rs%.2f", T, wpc, f, rs);
                    b.phased = true, b.f = f, b.rs = rs;
                    arms.push_back(b);
                }
        }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto run = [&](const Arm &a) {
        const uint32_t nw = uint32_t(cus) * a.wpc;
        const double cyc_bytes = double(nw) * a.T * (K + R) * 1024.0;
        const uint64_t P = uint64_t(cyc_bytes / (a.f * 8e12) * 1e8) + 1;  // 100 MHz ticks
        const uint64_t PR = uint64_t(double(P) * a.rs);
        hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, st, clk);
        uint64_t ts = 0;
        if (a.phased) {  // the launch's own start time, read on the device
            CHECK(hipStreamSynchronize(st));
            CHECK(hipMemcpy(&ts, clk, 8, hipMemcpyDeviceToHost));
            ts += 2000;  // 20 us: the launch below starts after this
        }
        if (a.T == 2 && a.phased) launch_phase<2, true>(src, dst, tiles, nw, P, PR, ts, st);
        if (a.T == 2 && !a.phased) launch_phase<2, false>(src, dst, tiles, nw, 1, 0, 0, st);
        if (a.T == 4 && a.phased) launch_phase<4, true>(src, dst, tiles, nw, P, PR, ts, st);
        if (a.T == 4 && !a.phased) launch_phase<4, false>(src, dst, tiles, nw, 1, 0, 0, st);
    };
    // correctness, every arm
    const size_t dbytes = size_t(stripes) * R * CS;
    std::vector<uint8_t> hr(dbytes), hd(dbytes);
    CHECK(hipMemcpy(hr.data(), ref, dbytes, hipMemcpyDeviceToHost));
    for (const Arm &a : arms) {
        CHECK(hipMemset(dst, 0, dbytes));
        run(a);
        CHECK(hipStreamSynchronize(st));
        CHECK(hipMemcpy(hd.data(), dst, dbytes, hipMemcpyDeviceToHost));
        if (memcmp(hr.data(), hd.data(), dbytes) != 0) {
            printf("MISMATCH %s\n", a.name);
            return 1;
        }
    }
    printf("all %zu arms bit-exact vs the plain kernel; %u CUs, %.2f GB per launch, median of %d rounds\n", arms.size(),
           cus, bytes / 1e9, rounds);
    fflush(stdout);
    std::vector<std::vector<float>> ms(arms.size() + 1);
    for (int r = 0; r < rounds; ++r) {
        for (size_t i = 0; i <= arms.size(); ++i) {
            // one launch per timing: phased arms need their own start time
            if (i == arms.size())
                hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, st, clk);
            else if (arms[i].phased)
                run(arms[i]);  // warm
            CHECK(hipStreamSynchronize(st));
            if (i == arms.size()) {
                CHECK(hipEventRecord(e0, st));
                hipLaunchKernelGGL(k_plain, dim3(tiles), dim3(64), 0, st, src, dst);
                CHECK(hipEventRecord(e1, st));
            } else {
                // the clock kernel + copy run before e0 for phased arms
                const Arm &a = arms[i];
                const uint32_t nw = uint32_t(cus) * a.wpc;
                const double cyc_bytes = double(nw) * a.T * (K + R) * 1024.0;
                const uint64_t P = uint64_t(cyc_bytes / (a.f * 8e12) * 1e8) + 1;
                const uint64_t PR = uint64_t(double(P) * a.rs);
                uint64_t ts = 0;
                if (a.phased) {
                    hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, st, clk);
                    CHECK(hipStreamSynchronize(st));
                    CHECK(hipMemcpy(&ts, clk, 8, hipMemcpyDeviceToHost));
                    ts += 2000;
                }
                CHECK(hipEventRecord(e0, st));
                if (a.T == 2 && a.phased) launch_phase<2, true>(src, dst, tiles, nw, P, PR, ts, st);
                if (a.T == 2 && !a.phased) launch_phase<2, false>(src, dst, tiles, nw, 1, 0, 0, st);
                if (a.T == 4 && a.phased) launch_phase<4, true>(src, dst, tiles, nw, P, PR, ts, st);
                if (a.T == 4 && !a.phased) launch_phase<4, false>(src, dst, tiles, nw, 1, 0, 0, st);
                CHECK(hipEventRecord(e1, st));
            }
            CHECK(hipEventSynchronize(e1));
            float t = 0;
            CHECK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t);
        }
        printf("round %d done\n", r);
        fflush(stdout);
    }
    auto report = [&](const char *name, std::vector<float> &v) {
        std::sort(v.begin(), v.end());
        const double med = v[v.size() / 2];
        printf("  %-36s %7.3f ms %7.1f GB/s %5.1f %%\n", name, med, bytes / (med * 1e-3) / 1e9,
               bytes / (med * 1e-3) / 8e12 * 100);
    };
    report("plain (one tile per block, uncapped)", ms[arms.size()]);
    for (size_t i = 0; i < arms.size(); ++i) report(arms[i].name, ms[i]);
    return 0;
}
