// tools/align_probe.hip — what do 8-byte-aligned chunks (MemEC's ChunkPool
// slots: an 8-byte ChunkIdentifier header before every chunk,
// chunk_pool.cc:22-55, so consecutive slots alternate between 8 and 0 mod
// 16) cost a 10R4W stream, and does realigning the lanes win it back?
// Not part of the product.
//
// Every kernel: RS(10,4)-shaped XOR stream (10 reads, 4 writes per 16-byte
// unit), data and parity chunks in separate ChunkPool-like slabs
// (slot = hdr + chunk), non-temporal 16-byte accesses, resident waves
// capped through dynamic LDS.  Modes:
//   direct   each lane loads/stores its 16 bytes wherever they are (what
//            the product's gathered kernels do today);
//   realign  every access 16-byte aligned: a lane loads the aligned block
//            under its unit and takes the bytes past the misalignment from
//            the next lane (ds_bpermute), lane 63 loads one extra block;
//            stores are shifted the other way, the wave's first and last
//            lanes store their partial pieces as dwords;
//   aligned  hdr = 16 (every chunk 16-byte aligned), direct accesses: the
//            target.
// Each realign run is checked byte for byte (headers included) against the
// direct run of the same layout.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Imemec_amd/csrc tools/align_probe.hip -o tools/align_probe
//   ./tools/align_probe [gib=8] [rounds=5]
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

__device__ __forceinline__ uint32_t from_lane(uint32_t v, uint32_t src_lane) {
    return uint32_t(__builtin_amdgcn_ds_bpermute(int(src_lane * 4), int(v)));
}

// bytes [a, 16) of b followed by bytes [0, a) of n (a uniform, multiple of 4)
__device__ __forceinline__ u32x4 funnel(const u32x4 &b, const u32x4 &n, uint32_t a) {
    switch (a) {
        case 4: return u32x4{b.y, b.z, b.w, n.x};
        case 8: return u32x4{b.z, b.w, n.x, n.y};
        case 12: return u32x4{b.w, n.x, n.y, n.z};
        default: return b;
    }
}

template <int MODE>
__device__ __forceinline__ u32x4 load_unit(const uint8_t *chunk, uint64_t off, uint32_t lane) {
    if constexpr (MODE == 0) {
        return ld_nt<u32x4>(chunk + off);
    } else {
        const uint32_t a = uint32_t(reinterpret_cast<uintptr_t>(chunk)) & 15u;
        const uint8_t *ab = chunk - a + off;
        const u32x4 b = ld_nt<u32x4>(ab);
        if (a == 0) return b;
        u32x4 e{0, 0, 0, 0};
        if (lane == 63) e = ld_nt<u32x4>(ab + 16);
        const uint32_t nl = (lane + 1) & 63;
        u32x4 n{from_lane(b.x, nl), from_lane(b.y, nl), from_lane(b.z, nl), 0u};
        if (lane == 63) n = e;
        return funnel(b, n, a);
    }
}

template <int MODE>
__device__ __forceinline__ void store_unit(uint8_t *chunk, uint64_t off, uint32_t lane, const u32x4 &v) {
    if constexpr (MODE == 0) {
        st_nt<u32x4>(chunk + off, v);
    } else {
        const uint32_t a = uint32_t(reinterpret_cast<uintptr_t>(chunk)) & 15u;
        if (a == 0) {
            st_nt<u32x4>(chunk + off, v);
            return;
        }
        const uint32_t pl = (lane + 63) & 63;
        const u32x4 p{0u, from_lane(v.y, pl), from_lane(v.z, pl), from_lane(v.w, pl)};
        // aligned block under the unit: the previous lane's last a bytes,
        // then this lane's first 16 - a
        const u32x4 x = funnel(p, v, 16 - a);
        uint8_t *ab = chunk - a + off;
        if (lane != 0) st_nt<u32x4>(ab, x);
        const uint32_t nd = a / 4;
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
        if (lane == 0)  // this lane's first 16 - a bytes, from the chunk's own offset
            for (uint32_t q = 0; q < 4 - nd; ++q) __builtin_nontemporal_store(w[q], reinterpret_cast<uint32_t *>(chunk + off) + q);
        if (lane == 63)  // its last a bytes, at the start of the next aligned block
            for (uint32_t q = 0; q < nd; ++q)
                __builtin_nontemporal_store(w[4 - nd + q], reinterpret_cast<uint32_t *>(ab + 16) + q);
    }
}

template <int MODE, int BT>
__global__ __launch_bounds__(BT) void k_align(const uint8_t *src, uint8_t *dst, uint64_t cs, uint64_t slot,
                                              uint32_t hdr, uint32_t tiles) {
    const uint32_t stripe = blockIdx.x / tiles, t = blockIdx.x % tiles;
    const uint64_t off = uint64_t(t) * BT * 16 + threadIdx.x * 16;
    const uint32_t lane = threadIdx.x & 63;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = load_unit<MODE>(src + (uint64_t(stripe) * K + j) * slot + hdr, off, lane);
    u32x4 acc = x[0];
#pragma unroll
    for (int j = 1; j < K; ++j) acc ^= x[j];
#pragma unroll
    for (int i = 0; i < R; ++i)
        store_unit<MODE>(dst + (uint64_t(stripe) * R + i) * slot + hdr, off, lane, acc + u32x4{uint32_t(i), 0, 0, 0});
}

static size_t cap_lds(uint32_t wpc, uint32_t bt) {
    if (!wpc) return 0;
    const uint32_t blocks = std::max<uint32_t>(1, wpc / (bt / 64));
    const size_t per = (160u << 10) / blocks / 512 * 512;
    return per > 512 ? per - 512 : 0;
}

struct Arm {
    const char *name;
    int mode, bt;
    uint32_t hdr, wpc;
};

template <int MODE, int BT>
void launch(const uint8_t *src, uint8_t *dst, uint64_t cs, uint32_t hdr, uint32_t stripes, uint32_t wpc,
            hipStream_t s) {
    const uint32_t tiles = uint32_t(cs / (BT * 16));
    hipLaunchKernelGGL((k_align<MODE, BT>), dim3(stripes * tiles), dim3(BT), cap_lds(wpc, BT), s, src, dst, cs,
                       cs + hdr, hdr, tiles);
}

static void run(const Arm &a, const uint8_t *src, uint8_t *dst, uint64_t cs, uint32_t stripes, hipStream_t s) {
    if (a.mode == 0 && a.bt == 64) launch<0, 64>(src, dst, cs, a.hdr, stripes, a.wpc, s);
    if (a.mode == 0 && a.bt == 256) launch<0, 256>(src, dst, cs, a.hdr, stripes, a.wpc, s);
    if (a.mode == 1 && a.bt == 64) launch<1, 64>(src, dst, cs, a.hdr, stripes, a.wpc, s);
    if (a.mode == 1 && a.bt == 256) launch<1, 256>(src, dst, cs, a.hdr, stripes, a.wpc, s);
}

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 8.0;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const Arm arms[] = {
        {"aligned  hdr16 b64 w16", 0, 64, 16, 16},  {"aligned  hdr16 b256 w12", 0, 256, 16, 12},
        {"direct   hdr8  b64 w16", 0, 64, 8, 16},   {"direct   hdr8  b256 w12", 0, 256, 8, 12},
        {"direct   hdr8  b256 w0", 0, 256, 8, 0},   {"realign  hdr8  b64 w16", 1, 64, 8, 16},
        {"realign  hdr8  b64 w12", 1, 64, 8, 12},   {"realign  hdr8  b256 w12", 1, 256, 8, 12},
        {"realign  hdr4  b64 w16", 1, 64, 4, 16},   {"realign  hdr12 b64 w16", 1, 64, 12, 16},
        {"aligned  hdr64 b64 w16", 0, 64, 64, 16},  {"aligned  hdr64 b256 w12", 0, 256, 64, 12},
        {"aligned  hdr128 b64 w16", 0, 64, 128, 16}, {"aligned  hdr128 b256 w12", 0, 256, 128, 12},
        {"aligned  hdr256 b64 w16", 0, 64, 256, 16}, {"aligned  hdr256 b256 w12", 0, 256, 256, 12},
        {"aligned  hdr1024 b64 w16", 0, 64, 1024, 16}, {"aligned  hdr1024 b256 w12", 0, 256, 1024, 12},
        {"aligned  hdr0 b64 w16", 0, 64, 0, 16},    {"aligned  hdr0 b256 w12", 0, 256, 0, 12},
    };
    const int na = sizeof(arms) / sizeof(arms[0]);
    for (uint64_t cs : {uint64_t(1) << 20, uint64_t(64) << 10, uint64_t(16) << 10}) {
        const uint64_t total = uint64_t(gib * double(1ull << 30));
        const uint32_t stripes = uint32_t(total / ((K + R) * (cs + 1024)));
        const uint64_t sbytes = uint64_t(stripes) * K * (cs + 1024) + 64, dbytes = uint64_t(stripes) * R * (cs + 1024) + 64;
        uint8_t *src, *dst, *ref;
        CHECK(hipMalloc(&src, sbytes));
        CHECK(hipMalloc(&dst, dbytes));
        CHECK(hipMalloc(&ref, dbytes));
        {  // non-constant source bytes so a wrong shift shows
            std::vector<uint32_t> h(sbytes / 4);
            uint32_t x = 0x12345678u;
            for (auto &v : h) v = (x = x * 1664525u + 1013904223u);
            CHECK(hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        }
        hipStream_t st;
        CHECK(hipStreamCreate(&st));
        // correctness: each realign arm vs the direct run of the same header
        std::vector<uint8_t> hr(dbytes), hd(dbytes);
        for (int i = 0; i < na; ++i) {
            if (arms[i].mode != 1) continue;
            CHECK(hipMemset(ref, 0xA5, dbytes));
            CHECK(hipMemset(dst, 0xA5, dbytes));
            run(Arm{"", 0, 256, arms[i].hdr, 0}, src, ref, cs, stripes, st);
            run(arms[i], src, dst, cs, stripes, st);
            CHECK(hipStreamSynchronize(st));
            CHECK(hipMemcpy(hr.data(), ref, dbytes, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(hd.data(), dst, dbytes, hipMemcpyDeviceToHost));
            const bool ok = memcmp(hr.data(), hd.data(), dbytes) == 0;
            printf("check %-26s cs=%7llu %s\n", arms[i].name, (unsigned long long)cs, ok ? "bit-exact" : "MISMATCH");
            if (!ok) return 1;
        }
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        const double bytes = double(stripes) * (K + R) * cs;
        std::vector<std::vector<float>> ms(na);
        for (int r = 0; r < rounds; ++r)
            for (int i = 0; i < na; ++i) {
                run(arms[i], src, dst, cs, stripes, st);
                CHECK(hipEventRecord(e0, st));
                for (int q = 0; q < 5; ++q) run(arms[i], src, dst, cs, stripes, st);
                CHECK(hipEventRecord(e1, st));
                CHECK(hipEventSynchronize(e1));
                float t = 0;
                CHECK(hipEventElapsedTime(&t, e0, e1));
                ms[i].push_back(t / 5);
            }
        printf("chunk %llu B, %u stripes, %.2f GB algorithmic per launch, median of %d x 5\n", (unsigned long long)cs,
               stripes, bytes / 1e9, rounds);
        for (int i = 0; i < na; ++i) {
            std::sort(ms[i].begin(), ms[i].end());
            const double med = ms[i][ms[i].size() / 2];
            printf("  %-28s %7.1f GB/s %5.1f %%\n", arms[i].name, bytes / (med * 1e-3) / 1e9,
                   bytes / (med * 1e-3) / 8e12 * 100);
        }
        fflush(stdout);
        CHECK(hipFree(src));
        CHECK(hipFree(dst));
        CHECK(hipFree(ref));
        CHECK(hipStreamDestroy(st));
    }
    return 0;
}
