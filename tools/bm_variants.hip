// tools/bm_variants.hip — variant study for the bitmatrix (Cauchy-RS)
// kernel on small chunks, in place on [stripe][k+m][chunk] (the layout of
// tools/perf_sweep.py, where CRS at 8-32 KiB with k >= 8 runs 66-71 %).
//
// Not part of the product.  Same arithmetic as bm_kernel.hpp (a lane keeps
// its R*W output slices in registers, SGPR masks, one v_bitop3 per
// (output, input) dword), timed interleaved in one process, varying:
//   D    source chunks in flight per wave (2 = the product: current + next)
//   xor  XOR-only math (memory ceiling of the same access pattern)
//   BT   threads per block (64 / 256), WPC resident-wave cap via LDS
//   split  separate data / parity buffers instead of in place
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Imemec_amd/csrc tools/bm_variants.hip -o tools/bm_variants
//   ./tools/bm_variants [k=12] [m=2] [chunk=8192] [gib=2] [rounds=7]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "bm_kernel.hpp"

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

using namespace mec::detail;

constexpr int KMAX = 16;

struct VArgs {
    const uint8_t *src;
    uint8_t *dst;
    uint64_t sss, dss, packet;
    uint32_t units, tiles, k, win;
    int64_t src_off[KMAX];
    int64_t dst_off[4];
    uint8_t mask[KMAX][32];
};

template <typename V, bool NT>
__device__ __forceinline__ V ldv(const uint8_t *p) {
    if constexpr (NT) return ld_nt<V>(p);
    return *reinterpret_cast<const V *>(p);
}
template <typename V, bool NT>
__device__ __forceinline__ void stv(uint8_t *p, V v) {
    if constexpr (NT) st_nt<V>(p, v);
    else *reinterpret_cast<V *>(p) = v;
}

// XCD-aware window split: block b runs on XCD b % 8; the window split is
// applied to rows of 8 consecutive blocks, so block b keeps b % 8 as its
// position inside the row (and, for 1 KiB tiles of 8 KiB-multiple chunks,
// as the KiB slot of every address it touches).
__device__ __forceinline__ uint32_t xcd_order(uint32_t win) {
    const uint32_t b = blockIdx.x;
    const uint32_t rows = gridDim.x / 8;
    if (win <= 1 || b >= rows * 8) return b;
    const uint32_t r = b / 8, x = b % 8;
    const uint32_t per = rows / win;
    const uint32_t r2 = r < per * win ? (r % win) * per + r / win : r;
    return r2 * 8 + x;
}

// MAP 0: lane u owns bytes [16u, 16u+16) of every packet (the product);
// MAP 1 (XOR-only ceiling study): a wave owns 64*16*W contiguous bytes of
// each chunk, unit x of lane l at wave_base + x*1024 + 16l.
template <int VW>
struct VecOf {
    typedef u32x4 type;
};
template <>
struct VecOf<2> {
    typedef u32x2 type;
};
template <>
struct VecOf<1> {
    typedef uint32_t type;
};

template <int W, int R, int BT, int D, bool XOR, int MAP = 0, bool NT = true, int VW = 4, int XO = 0>
__global__ __launch_bounds__(BT) void k_bm(const VArgs p) {
    typedef typename VecOf<VW>::type vec;
    constexpr int ROWS = R * W;
    const uint32_t bid = XO ? xcd_order(p.win) : block_order(p.win);
    const uint32_t stripe = bid / p.tiles;
    const uint32_t u = (bid - stripe * p.tiles) * BT + threadIdx.x;
    if (u >= p.units) return;
    const uint64_t off = MAP == 0 ? uint64_t(u) * (4 * VW) : uint64_t(u / 64) * (1024 * W) + (u % 64) * 16;
    const uint64_t pstride = MAP == 0 ? p.packet : 1024;
    const uint8_t *sb = p.src + int64_t(stripe) * p.sss + off;
    uint8_t *db = p.dst + int64_t(stripe) * p.dss + off;
    vec acc[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r] = vec(0);
    vec buf[D][W];
#pragma unroll
    for (int q = 0; q < D; ++q)
        if (q < int(p.k))
#pragma unroll
            for (int x = 0; x < W; ++x) buf[q][x] = ldv<vec, NT>(sb + p.src_off[q] + uint64_t(x) * pstride);
    for (uint32_t j0 = 0; j0 < p.k; j0 += D) {
#pragma unroll
        for (int q = 0; q < D; ++q) {
            const uint32_t j = j0 + q;
            if (j < p.k) {
                if (XOR) {
#pragma unroll
                    for (int r = 0; r < ROWS; ++r) acc[r] ^= buf[q][r % W];
                } else {
                    bm_combine<W, ROWS, vec>(buf[q], acc, p.mask[j]);
                }
                if (j + D < p.k)
#pragma unroll
                    for (int x = 0; x < W; ++x) buf[q][x] = ldv<vec, NT>(sb + p.src_off[j + D] + uint64_t(x) * pstride);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
        for (int l = 0; l < W; ++l) stv<vec, NT>(db + p.dst_off[i] + uint64_t(l) * pstride, acc[i * W + l]);
}

// gf8 (byte-wise RS) access pattern, XOR-only: lane owns one 16-B unit of
// the chunk, all K source loads in flight at once, R stores.
template <int K, int R, int BT, int ROT = 0, int XO = 0>
__global__ __launch_bounds__(BT) void k_gf8xor(const VArgs p, uint32_t cunits, uint32_t ctiles) {
    const uint32_t bid = XO ? xcd_order(p.win) : block_order(p.win);
    const uint32_t stripe = bid / ctiles;
    // ROT: tile t of stripe s handled by block (t - s*ROT) mod tiles, so an
    // XCD no longer sees one fixed KiB slot of every chunk
    const uint32_t t0 = bid - stripe * ctiles;
    uint32_t u;
    if (ROT == 9) {
        // slot-affine 4-wave blocks: wave w of block q covers the 1 KiB tile
        // ((q / 8) * (BT / 64) + w) * 8 + q % 8, so every wave of a block
        // (one XCD) touches the same KiB slot mod 8 KiB
        const uint32_t wv = threadIdx.x / 64, ln = threadIdx.x % 64;
        u = (((t0 / 8) * (BT / 64) + wv) * 8 + t0 % 8) * 64 + ln;
    } else {
        u = ((t0 + stripe * ROT) % ctiles) * BT + threadIdx.x;
    }
    if (u >= cunits) return;
    const uint8_t *sb = p.src + int64_t(stripe) * p.sss + uint64_t(u) * 16;
    uint8_t *db = p.dst + int64_t(stripe) * p.dss + uint64_t(u) * 16;
    u32x4 d[K];
#pragma unroll
    for (int j = 0; j < K; ++j) d[j] = ld_nt<u32x4>(sb + p.src_off[j]);
    u32x4 acc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        acc[i] = d[0];
#pragma unroll
        for (int j = 1; j < K; ++j) acc[i] ^= (j + i) & 1 ? d[j] : (d[j] << 1);
    }
#pragma unroll
    for (int i = 0; i < R; ++i) st_nt<u32x4>(db + p.dst_off[i], acc[i]);
}

__global__ void fill_kernel(uint64_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t z = 0x4D454D4543ull + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

struct Layout {
    uint8_t *src, *dst;
    uint64_t sss, dss;
    int64_t src_off[KMAX], dst_off[4];
    uint32_t win;
};

typedef void (*LaunchFn)(const VArgs &, uint32_t stripes, uint32_t wpc, hipStream_t);

template <int W, int R, int BT, int D, bool XOR, int MAP = 0, bool NT = true, int VW = 4, int XO = 0>
void launch(const VArgs &a0, uint32_t stripes, uint32_t wpc, hipStream_t s) {
    VArgs a = a0;
    a.units = uint32_t(a.packet / (4 * VW));
    a.tiles = (a.units + BT - 1) / BT;
    size_t lds = 0;
    if (wpc > 0) {
        const uint32_t act = std::min<uint32_t>(BT, a.units);
        const uint32_t per = (act + 63) / 64;
        const uint32_t blocks = std::max<uint32_t>(1, (wpc + per - 1) / per);
        const uint32_t pb = (160u << 10) / blocks / 512 * 512;
        lds = pb > 1024 ? pb - 1024 : 0;
    }
    hipLaunchKernelGGL((k_bm<W, R, BT, D, XOR, MAP, NT, VW, XO>), dim3(stripes * a.tiles), dim3(BT), lds, s, a);
}

template <int K, int R, int BT, int ROT = 0, int XO = 0>
void launch_gf8xor(const VArgs &a, uint32_t stripes, uint32_t wpc, hipStream_t s) {
    // chunk bytes = W * packet; recovered from the first two source offsets
    const uint64_t chunk = uint64_t(a.src_off[1] - a.src_off[0]);
    const uint32_t units = uint32_t(chunk / 16), tiles = (units + BT - 1) / BT;
    size_t lds = 0;
    if (wpc > 0) {
        const uint32_t per = (std::min<uint32_t>(BT, units) + 63) / 64;
        const uint32_t blocks = std::max<uint32_t>(1, (wpc + per - 1) / per);
        const uint32_t pb = (160u << 10) / blocks / 512 * 512;
        lds = pb > 1024 ? pb - 1024 : 0;
    }
    hipLaunchKernelGGL((k_gf8xor<K, R, BT, ROT, XO>), dim3(stripes * tiles), dim3(BT), lds, s, a, units, tiles);
}

struct Variant {
    std::string name;
    LaunchFn fn;
    uint32_t wpc;
    bool split, xr;
    uint32_t win = 0;  // 0: the layout's default (2 in place, 1 split)
};

template <int W, int R, int KG>
std::vector<Variant> variants() {
    std::vector<Variant> v;
    if (getenv("BMV_SET") && atoi(getenv("BMV_SET")) == 7) {
        for (uint32_t win : {1u, 2u}) {
            for (uint32_t wpc : {8u, 16u}) {
                const std::string sfx = "/w" + std::to_string(wpc) + "/win" + std::to_string(win);
                v.push_back({"gf8xor.64" + sfx, launch_gf8xor<KG, R, 64>, wpc, false, true, win});
                v.push_back({"gf8xor.64.xo" + sfx, launch_gf8xor<KG, R, 64, 0, 1>, wpc, false, true, win});
                v.push_back({"gf8xor.256" + sfx, launch_gf8xor<KG, R, 256>, wpc, false, true, win});
                v.push_back({"gf8xor.256.slot" + sfx, launch_gf8xor<KG, R, 256, 9, 0>, wpc, false, true, win});
                v.push_back({"gf8xor.256.slot.xo" + sfx, launch_gf8xor<KG, R, 256, 9, 1>, wpc, false, true, win});
            }
        }
        v.push_back({"gf8xor.256/w16/split", launch_gf8xor<KG, R, 256>, 16, true, true});
        v.push_back({"gf8xor.256.slot/w16/split", launch_gf8xor<KG, R, 256, 9, 0>, 16, true, true});
        return v;
    }
    if (getenv("BMV_SET") && atoi(getenv("BMV_SET")) == 6) {
        for (uint32_t win : {1u, 2u, 4u}) {
            const std::string sfx = "/win" + std::to_string(win);
            v.push_back({"gf8xor.64/w8" + sfx, launch_gf8xor<KG, R, 64>, 8, false, true, win});
            v.push_back({"gf8xor.64.xo/w8" + sfx, launch_gf8xor<KG, R, 64, 0, 1>, 8, false, true, win});
            v.push_back({"d2.64.v4/w8" + sfx, launch<W, R, 64, 2, false>, 8, false, false, win});
            v.push_back({"d2.64.v4.xo/w8" + sfx, launch<W, R, 64, 2, false, 0, true, 4, 1>, 8, false, false, win});
            v.push_back({"d2.64.v2/w12" + sfx, launch<W, R, 64, 2, false, 0, true, 2>, 12, false, false, win});
            v.push_back({"d2.64.v2.xo/w12" + sfx, launch<W, R, 64, 2, false, 0, true, 2, 1>, 12, false, false, win});
        }
        v.push_back({"gf8xor.64/w8/split", launch_gf8xor<KG, R, 64>, 8, true, true});
        v.push_back({"d2.64.v2/w12/split", launch<W, R, 64, 2, false, 0, true, 2>, 12, true, false});
        v.push_back({"d2.64.v2.xo/w12/split", launch<W, R, 64, 2, false, 0, true, 2, 1>, 12, true, false});
        return v;
    }
    if (getenv("BMV_SET") && atoi(getenv("BMV_SET")) == 5) {
        for (uint32_t wpc : {8u, 12u}) {
            const std::string sfx = "/w" + std::to_string(wpc);
            v.push_back({"gf8xor.64" + sfx, launch_gf8xor<KG, R, 64>, wpc, false, true});
            v.push_back({"gf8xor.64.rot1" + sfx, launch_gf8xor<KG, R, 64, 1>, wpc, false, true});
            v.push_back({"gf8xor.64.rot3" + sfx, launch_gf8xor<KG, R, 64, 3>, wpc, false, true});
            v.push_back({"gf8xor.256" + sfx, launch_gf8xor<KG, R, 256>, wpc, false, true});
            v.push_back({"d2.64.v2" + sfx, launch<W, R, 64, 2, false, 0, true, 2>, wpc, false, false});
            v.push_back({"gf8xor.64.rot1/split" + sfx, launch_gf8xor<KG, R, 64, 1>, wpc, true, true});
            v.push_back({"gf8xor.64/split" + sfx, launch_gf8xor<KG, R, 64>, wpc, true, true});
        }
        return v;
    }
    if (getenv("BMV_SET") && atoi(getenv("BMV_SET")) == 4) {
        for (uint32_t wpc : {8u, 12u, 16u}) {
            const std::string sfx = "/w" + std::to_string(wpc);
            v.push_back({"d2.64.v4" + sfx, launch<W, R, 64, 2, false>, wpc, false, false});
            v.push_back({"d2.64.v2" + sfx, launch<W, R, 64, 2, false, 0, true, 2>, wpc, false, false});
            v.push_back({"d16.64.v2" + sfx, launch<W, R, 64, 16, false, 0, true, 2>, wpc, false, false});
            v.push_back({"d16.64.v4" + sfx, launch<W, R, 64, 16, false, 0, true, 4>, wpc, false, false});
            v.push_back({"d16.256.v2" + sfx, launch<W, R, 256, 16, false, 0, true, 2>, wpc, false, false});
            v.push_back({"gf8xor.64" + sfx, launch_gf8xor<KG, R, 64>, wpc, false, true});
            v.push_back({"gf8xor.256" + sfx, launch_gf8xor<KG, R, 256>, wpc, false, true});
        }
        v.push_back({"gf8xor.64/w0", launch_gf8xor<KG, R, 64>, 0, false, true});
        v.push_back({"d2.64.v2/w12/split", launch<W, R, 64, 2, false, 0, true, 2>, 12, true, false});
        v.push_back({"d16.64.v2/w12/split", launch<W, R, 64, 16, false, 0, true, 2>, 12, true, false});
        v.push_back({"gf8xor.64/w12/split", launch_gf8xor<KG, R, 64>, 12, true, true});
        return v;
    }
    if (getenv("BMV_SET") && atoi(getenv("BMV_SET")) == 3) {
        for (uint32_t wpc : {0u, 8u, 16u}) {
            const std::string sfx = "/w" + std::to_string(wpc);
            v.push_back({"d2.64.v4" + sfx, launch<W, R, 64, 2, false>, wpc, false, false});
            v.push_back({"d2.64.v2" + sfx, launch<W, R, 64, 2, false, 0, true, 2>, wpc, false, false});
            v.push_back({"d2.64.v1" + sfx, launch<W, R, 64, 2, false, 0, true, 1>, wpc, false, false});
            v.push_back({"d4.64.v1" + sfx, launch<W, R, 64, 4, false, 0, true, 1>, wpc, false, false});
            v.push_back({"d2.256.v2" + sfx, launch<W, R, 256, 2, false, 0, true, 2>, wpc, false, false});
            v.push_back({"xor2.64.v2" + sfx, launch<W, R, 64, 2, true, 0, true, 2>, wpc, false, true});
            v.push_back({"xor2.64.v1" + sfx, launch<W, R, 64, 2, true, 0, true, 1>, wpc, false, true});
        }
        v.push_back({"d2.64.v4/w8/split", launch<W, R, 64, 2, false>, 8, true, false});
        v.push_back({"d2.64.v2/w8/split", launch<W, R, 64, 2, false, 0, true, 2>, 8, true, false});
        v.push_back({"d2.64.v1/w8/split", launch<W, R, 64, 2, false, 0, true, 1>, 8, true, false});
        return v;
    }
    if (getenv("BMV_SET") && atoi(getenv("BMV_SET")) == 2) {
        for (uint32_t win : {1u, 2u, 4u, 8u}) {
            const std::string sfx = "/win" + std::to_string(win);
            v.push_back({"d2.64/w8" + sfx, launch<W, R, 64, 2, false>, 8, false, false, win});
            v.push_back({"d2.256/w8" + sfx, launch<W, R, 256, 2, false>, 8, false, false, win});
            v.push_back({"xor2.64/w8" + sfx, launch<W, R, 64, 2, true>, 8, false, true, win});
            v.push_back({"xorC.64/w8" + sfx, launch<W, R, 64, 2, true, 1>, 8, false, true, win});
            v.push_back({"d2.64c/w8" + sfx, launch<W, R, 64, 2, false, 0, false>, 8, false, false, win});
        }
        v.push_back({"xor2.64/w8/split", launch<W, R, 64, 2, true>, 8, true, true});
        v.push_back({"xorC.64/w8/split", launch<W, R, 64, 2, true, 1>, 8, true, true});
        return v;
    }
    for (int split = 0; split < 2; ++split)
        for (uint32_t wpc : {0u, 8u, 12u}) {
            const std::string sfx = std::string(split ? "/split" : "") + "/w" + std::to_string(wpc);
            v.push_back({"d2.256" + sfx, launch<W, R, 256, 2, false>, wpc, bool(split), false});
            v.push_back({"d2.64" + sfx, launch<W, R, 64, 2, false>, wpc, bool(split), false});
            v.push_back({"d3.64" + sfx, launch<W, R, 64, 3, false>, wpc, bool(split), false});
            v.push_back({"d4.64" + sfx, launch<W, R, 64, 4, false>, wpc, bool(split), false});
            v.push_back({"d4.256" + sfx, launch<W, R, 256, 4, false>, wpc, bool(split), false});
            v.push_back({"xor2.64" + sfx, launch<W, R, 64, 2, true>, wpc, bool(split), true});
            v.push_back({"xor4.64" + sfx, launch<W, R, 64, 4, true>, wpc, bool(split), true});
        }
    return v;
}

template <int W, int R, int KG>
int run(int k, uint64_t cs, double gib, int rounds) {
    const int m = R;
    const uint64_t packet = cs / W;
    if (packet % 16) {
        fprintf(stderr, "packet must be a multiple of 16\n");
        return 2;
    }
    const uint32_t stripes = uint32_t(gib * double(1ull << 30) / double((k + m) * cs));
    uint8_t *st, *data, *par;
    const uint64_t sbytes = uint64_t(stripes) * (k + m) * cs;
    CHECK(hipMalloc(&st, sbytes));
    CHECK(hipMalloc(&data, uint64_t(stripes) * k * cs));
    CHECK(hipMalloc(&par, uint64_t(stripes) * m * cs));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, nullptr, reinterpret_cast<uint64_t *>(st), sbytes / 8);
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, nullptr, reinterpret_cast<uint64_t *>(data),
                       uint64_t(stripes) * k * cs / 8);
    CHECK(hipDeviceSynchronize());
    VArgs a{};
    a.packet = packet;
    a.units = uint32_t(packet / 16);
    a.k = uint32_t(k);
    srand(7);
    for (int j = 0; j < k; ++j)
        for (int r = 0; r < R * W; ++r) a.mask[j][r] = uint8_t(rand() & ((1 << W) - 1));
    auto set_layout = [&](bool split) {
        if (split) {
            a.src = data;
            a.dst = par;
            a.sss = uint64_t(k) * cs;
            a.dss = uint64_t(m) * cs;
            for (int j = 0; j < k; ++j) a.src_off[j] = int64_t(j) * cs;
            for (int i = 0; i < m; ++i) a.dst_off[i] = int64_t(i) * cs;
            a.win = 1;
        } else {
            a.src = st;
            a.dst = st;
            a.sss = a.dss = uint64_t(k + m) * cs;
            for (int j = 0; j < k; ++j) a.src_off[j] = int64_t(j) * cs;
            for (int i = 0; i < m; ++i) a.dst_off[i] = int64_t(k + i) * cs;
            a.win = 2;
        }
    };
    auto vs = variants<W, R, KG>();
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    // correctness: every non-xor in-place variant reproduces a host computation of stripe 0 and the last
    for (const Variant &v : vs) {
        if (v.xr || v.split) continue;
        set_layout(false);
        v.fn(a, stripes, v.wpc, s);
        CHECK(hipStreamSynchronize(s));
        for (uint32_t sidx : {0u, stripes - 1}) {
            std::vector<uint8_t> h((k + m) * cs);
            CHECK(hipMemcpy(h.data(), st + uint64_t(sidx) * (k + m) * cs, (k + m) * cs, hipMemcpyDeviceToHost));
            for (int i = 0; i < R; ++i)
                for (int l = 0; l < W; ++l)
                    for (uint64_t b = 0; b < packet; ++b) {
                        uint8_t x = 0;
                        for (int j = 0; j < k; ++j)
                            for (int q = 0; q < W; ++q)
                                if ((a.mask[j][i * W + l] >> q) & 1) x ^= h[j * cs + q * packet + b];
                        if (x != h[(k + i) * cs + l * packet + b]) {
                            printf("WRONG %s stripe %u row %d packet %d byte %llu\n", v.name.c_str(), sidx, i, l,
                                   (unsigned long long)b);
                            return 1;
                        }
                    }
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ms(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            set_layout(vs[i].split);
            if (vs[i].win) a.win = vs[i].win;
            for (int w = 0; w < 2; ++w) vs[i].fn(a, stripes, vs[i].wpc, s);
            CHECK(hipEventRecord(e0, s));
            const int reps = 8;
            for (int w = 0; w < reps; ++w) vs[i].fn(a, stripes, vs[i].wpc, s);
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float t = 0;
            CHECK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t / reps);
        }
    const double bytes = double(stripes) * (k + m) * cs;
    printf("CRS(%d,%d) w=%d chunk %llu, %u stripes, %.3f GB per launch\n", k, m, W, (unsigned long long)cs, stripes,
           bytes / 1e9);
    for (size_t i = 0; i < vs.size(); ++i) {
        std::vector<float> t = ms[i];
        std::sort(t.begin(), t.end());
        printf("  %-18s median %8.1f us  %6.1f %%\n", vs[i].name.c_str(), t[t.size() / 2] * 1e3,
               bytes / (t[t.size() / 2] * 1e-3) / 8e12 * 100);
    }
    CHECK(hipFree(st));
    CHECK(hipFree(data));
    CHECK(hipFree(par));
    return 0;
}

int main(int argc, char **argv) {
    const int k = argc > 1 ? atoi(argv[1]) : 12, m = argc > 2 ? atoi(argv[2]) : 2;
    const uint64_t cs = argc > 3 ? strtoull(argv[3], nullptr, 10) : 8192;
    const double gib = argc > 4 ? atof(argv[4]) : 2.0;
    const int rounds = argc > 5 ? atoi(argv[5]) : 7;
    if (k < 1 || k > KMAX) return 2;
    int w = 1;
    while ((1 << w) < k + m) ++w;
    if (w < 3) w = 3;
    if (w == 4 && m == 2 && k == 12) return run<4, 2, 12>(k, cs, gib, rounds);
    if (w == 4 && m == 2 && k == 8) return run<4, 2, 8>(k, cs, gib, rounds);
    if (w == 4 && m == 4 && k == 12) return run<4, 4, 12>(k, cs, gib, rounds);
    fprintf(stderr, "unsupported (w=%d, m=%d)\n", w, m);
    return 2;
}
