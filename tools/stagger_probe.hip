// stagger_probe.hip — experiment: why does the split
// Vandermonde encode outrun its arithmetic-free twin while the in-place
// decode (configs[2]) only ties its twin?  Hypothesis: the encode's
// arithmetic spaces a wave's store burst away from its load burst, and the
// DRAM stream prefers that spacing.  This probe runs the product's own
// gf8_kernel body (gf8_kernel.hpp: same loads, gf8_apply, stores, block
// order, stripe map and wave cap as libmec's launch) with two extra
// compile-time knobs, over the configs[2] layout (RS(10,4) 1 MiB,
// [stripe][14][chunk], erasures {0,1,2,3} rebuilt in place from chunks
// 4..13) and the configs[1] split layout:
//   SLEEP  s_sleep(SLEEP) between the arithmetic and the stores (0 = none)
//   REV    stores in reverse row order
// Timing only (outputs are not checked: any dense 4 x 10 matrix costs the
// same); each arm best of 5 launches, arms interleaved over `rounds`.
//
//   stagger_probe [stripes=4096] [rounds=2] [arm,arm,...]
// (the arm list selects and orders arms: under rocprofv3 --pmc every arm is
// 6 dispatches of probe_kernel, one untimed then 5 timed, in list order;
// tools/stagger_pmc.py sums the counters per arm)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gf8_kernel.hpp"
#include "mec.h"

using namespace mec;
using namespace mec::detail;

template <int K, int R, int S, int BT, int SLEEP, bool REV>
__global__ __launch_bounds__(BT) void probe_kernel(const Gf8Params<K, R> p) {
    __shared__ uint32_t tab[R * K * 8];
    for (int t = threadIdx.x; t < R * K; t += BT) {
        const Gf8Coef c = p.coef[t / K][t % K];
        tab[t * 8 + 0] = c.t0;
        tab[t * 8 + 1] = c.t1;
        tab[t * 8 + 2] = c.u0;
        tab[t * 8 + 3] = c.u1;
        tab[t * 8 + 4] = c.v;
    }
    __syncthreads();
    const uint32_t bid = block_order(p.win);
    uint32_t stripe, tile;
    stripe_tile(bid, p.tiles, p.nstr, p.sgroup, p.srun, stripe, tile);
    const uint32_t u = tile * BT + threadIdx.x;
    if (u >= p.units) return;
    const uint32_t off = u * 16;
    u32x4 d[K];
#pragma unroll
    for (int j = 0; j < K; ++j)
        d[j] = buf_ld<u32x4>(chunk_rsrc(uint64_t(uintptr_t(p.src + int64_t(stripe) * p.sss + p.src_off[j])), p.chunk),
                             off, true);
    __amdgpu_buffer_rsrc_t dr[R];
#pragma unroll
    for (int i = 0; i < R; ++i) dr[i] = chunk_rsrc(uint64_t(uintptr_t(p.dst + int64_t(stripe) * p.dss + p.dst_off[i])), p.chunk);
    u32x4 acc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = u32x4{0, 0, 0, 0};
    gf8_apply<K, R, S>(d, acc, tab + opaque_zero());
    if constexpr (SLEEP > 0) __builtin_amdgcn_s_sleep(SLEEP);
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int i = REV ? R - 1 - q : q;
        buf_st(acc[i], dr[i], off);
    }
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

constexpr int K = 10, R = 4;
constexpr uint64_t CS = 1 << 20;

struct Arm {
    const char *name;
    bool in_place;
    int s;       // kGf8Dense / kGf8Vand / kGf8Xor
    int sleep;
    bool rev;
    int cap = 0;  // waves per CU; 0 = the product's rule (gf8_target_waves)
};

template <int S, int BT, int SLEEP, bool REV>
void launch(dim3 grid, uint32_t lds, const Gf8Params<K, R> &p) {
    hipLaunchKernelGGL((probe_kernel<K, R, S, BT, SLEEP, REV>), grid, dim3(BT), lds, 0, p);
}

template <int S, int BT>
void launch_s(int sleep, bool rev, dim3 grid, uint32_t lds, const Gf8Params<K, R> &p) {
    switch (sleep * 2 + (rev ? 1 : 0)) {
        case 0: launch<S, BT, 0, false>(grid, lds, p); break;
        case 1: launch<S, BT, 0, true>(grid, lds, p); break;
        case 4: launch<S, BT, 2, false>(grid, lds, p); break;
        case 16: launch<S, BT, 8, false>(grid, lds, p); break;
        case 32: launch<S, BT, 16, false>(grid, lds, p); break;
        case 48: launch<S, BT, 24, false>(grid, lds, p); break;
        case 64: launch<S, BT, 32, false>(grid, lds, p); break;
        case 65: launch<S, BT, 32, true>(grid, lds, p); break;
        case 96: launch<S, BT, 48, false>(grid, lds, p); break;
        case 128: launch<S, BT, 64, false>(grid, lds, p); break;
        default: fprintf(stderr, "arm not instantiated\n"); exit(2);
    }
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 4096;
    const int rounds = argc > 2 ? atoi(argv[2]) : 2;
    CK(hipSetDevice(0));
    uint8_t *stripe = nullptr, *data = nullptr, *par = nullptr;
    CK(hipMalloc((void **)&stripe, size_t(n) * (K + R) * CS));
    CK(hipMalloc((void **)&data, size_t(n) * K * CS));
    CK(hipMalloc((void **)&par, size_t(n) * R * CS));
    mec_fill_random(stripe, size_t(n) * (K + R) * CS, 1, 0, nullptr);
    mec_fill_random(data, size_t(n) * K * CS, 2, 0, nullptr);
    CK(hipDeviceSynchronize());
    // a dense decode-like matrix and the Vandermonde RS(10,4) parity rows
    const uint8_t vand[R][K] = {{1, 1, 1, 1, 1, 1, 1, 1, 1, 1},
                                {1, 147, 138, 73, 93, 161, 103, 58, 99, 178},
                                {1, 103, 156, 151, 123, 187, 166, 175, 244, 83},
                                {1, 220, 166, 123, 82, 143, 245, 40, 167, 122}};
    std::vector<Arm> arms = {
        {"inplace_dec", true, kGf8Dense, 0, false},          {"inplace_dec_rev", true, kGf8Dense, 0, true},
        {"inplace_dec_sleep16", true, kGf8Dense, 16, false}, {"inplace_dec_sleep24", true, kGf8Dense, 24, false},
        {"inplace_dec_sleep32", true, kGf8Dense, 32, false}, {"inplace_dec_sleep48", true, kGf8Dense, 48, false},
        {"inplace_dec_rev_sleep32", true, kGf8Dense, 32, true},
        {"inplace_dec_cap12", true, kGf8Dense, 0, false, 12}, {"inplace_dec_cap14", true, kGf8Dense, 0, false, 14},
        {"inplace_dec_cap12_sleep32", true, kGf8Dense, 32, false, 12},
        {"inplace_twin", true, kGf8Xor, 0, false},           {"inplace_vand", true, kGf8Vand, 0, false},
        {"inplace_vand_cap16", true, kGf8Vand, 0, false, 16},
        {"split_enc", false, kGf8Vand, 0, false},             {"split_enc_cap16", false, kGf8Vand, 0, false, 16},
        {"split_twin", false, kGf8Xor, 0, false},             {"split_twin_cap12", false, kGf8Xor, 0, false, 12},
        {"split_dense", false, kGf8Dense, 0, false},          {"split_dense_cap12", false, kGf8Dense, 0, false, 12},
    };
    if (argc > 3) {
        std::vector<Arm> pick;
        std::string list = argv[3];
        size_t at = 0;
        while (at <= list.size()) {
            const size_t e = std::min(list.find(',', at), list.size());
            const std::string name = list.substr(at, e - at);
            bool found = false;
            for (const Arm &a : arms)
                if (name == a.name) {
                    pick.push_back(a);
                    found = true;
                }
            if (!found) {
                fprintf(stderr, "unknown arm %s\n", name.c_str());
                return 2;
            }
            at = e + 1;
        }
        arms = pick;
    }
    const double alg = double(n) * (K + R) * CS;
    for (int rd = 0; rd < rounds; ++rd) {
        for (const Arm &a : arms) {
            Gf8Params<K, R> p{};
            const bool ip = a.in_place;
            p.sss = ip ? int64_t(K + R) * CS : int64_t(K) * CS;
            p.dss = ip ? int64_t(K + R) * CS : int64_t(R) * CS;
            p.chunk = uint32_t(CS);
            p.accumulate = 0;
            for (int j = 0; j < K; ++j) p.src_off[j] = ip ? int64_t(R + j) * CS : int64_t(j) * CS;  // survivors 4..13
            for (int i = 0; i < R; ++i) p.dst_off[i] = int64_t(i) * CS;
            for (int i = 0; i < R; ++i)
                for (int j = 0; j < K; ++j)
                    p.coef[i][j] = gf8_coef(a.s == kGf8Vand ? vand[i][j] : uint8_t(17 + 31 * i + 7 * j));
            p.src = ip ? stripe : data;
            p.dst = ip ? stripe : par;
            // the product's launch rules (gf8_kernel.hpp run_gf8)
            p.win = launch_windows(p.src, int64_t(n) * p.sss, p.dst, int64_t(n) * p.dss);
            const uint32_t bt = block_threads(true, p.win, false);  // 1 MiB stride: 4-wave blocks in place
            const Geometry g = geometry(CS / 16, bt);
            p.units = g.units;
            p.tiles = g.tiles;
            p.nstr = n;
            p.s0 = 0;
            p.sgroup = stripe_group(CS, g.tiles, p.win > 1 ? n / p.win : n, p.win > 1, false, p.srun);
            const bool dense = a.s != kGf8Vand;
            const uint32_t lds =
                occupancy_lds(bt, bt, R * K * 32, a.cap ? uint32_t(a.cap) : gf8_target_waves(K, R, ip, dense, false));
            const dim3 grid(n * g.tiles);
            auto go = [&] {
                if (bt == kWaveBlock) {
                    if (a.s == kGf8Dense) launch_s<kGf8Dense, kWaveBlock>(a.sleep, a.rev, grid, lds, p);
                    else if (a.s == kGf8Vand) launch_s<kGf8Vand, kWaveBlock>(a.sleep, a.rev, grid, lds, p);
                    else launch_s<kGf8Xor, kWaveBlock>(a.sleep, a.rev, grid, lds, p);
                } else {
                    if (a.s == kGf8Dense) launch_s<kGf8Dense, kThreads>(a.sleep, a.rev, grid, lds, p);
                    else if (a.s == kGf8Vand) launch_s<kGf8Vand, kThreads>(a.sleep, a.rev, grid, lds, p);
                    else launch_s<kGf8Xor, kThreads>(a.sleep, a.rev, grid, lds, p);
                }
            };
            go();
            CK(hipDeviceSynchronize());
            float best = 1e30f;
            for (int r = 0; r < 5; ++r) {
                hipEvent_t e0, e1;
                CK(hipEventCreate(&e0));
                CK(hipEventCreate(&e1));
                CK(hipEventRecord(e0, 0));
                go();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
                CK(hipEventDestroy(e0));
                CK(hipEventDestroy(e1));
            }
            printf("{\"round\": %d, \"arm\": \"%s\", \"win\": %u, \"block\": %u, \"lds\": %u, \"ms\": %.4f, \"frac\": %.4f}\n",
                   rd, a.name, p.win, bt, lds, best, alg / (best * 1e-3) / 8e12);
            fflush(stdout);
        }
    }
    CK(hipFree(stripe));
    CK(hipFree(data));
    CK(hipFree(par));
    return 0;
}
