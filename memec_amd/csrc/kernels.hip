// kernels.hip — libmec's CDNA4 (gfx950) kernels.
//
// Every kernel is a streaming pass over HBM: each lane owns one 16-byte
// column slice ("unit") of a stripe and touches it in every chunk it reads
// or writes, so a wave moves 1 KiB contiguous per chunk per instruction and
// no byte is read twice.  The arithmetic is chosen to stay under the HBM
// time (SURVEY §7 "hard parts"):
//
//  * gf8_kernel — GF(2^8) matrix apply, byte-wise (Jerasure RS, ISA-L RS and
//    Cauchy; replaces gf_w8_table_multiply_region, gf_w8.c:1033-1056 and
//    ISA-L's gf_Nvect_dot_prod_*).  A product c*x is linear in x's bits, so
//    a byte is split into bit fields 0-2 | 3-5 | 6-7 and each field indexes
//    a <= 8-entry table of c*(field) with one v_perm_b32 (4 bytes per
//    instruction).  Per (coefficient, dword): 3 v_perm + 3 v_xor.
//  * bm_kernel  — bitmatrix packet XOR (Jerasure Cauchy-RS; replaces
//    jerasure_do_scheduled_operations, jerasure.c:1162-1185).  Masks are
//    kernel arguments (SGPRs); each (output packet, input packet) pair is an
//    AND with a 0/-1 mask and an XOR.
//  * xor_kernel — region XOR (Coding::bitwiseXOR, coding.cc:88-118).
//  * fill_kernel — splitmix64 fill for synthetic stripes.
#include <array>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <utility>

#include "gf_math.hpp"
#include "kernels.hpp"
#include "knobs.hpp"
#include "bm_kernel.hpp"
#include "gf8_kernel.hpp"
#include "gather_kernel.hpp"
#include "stream_common.hpp"

namespace mec {
namespace detail {
template <int K, int R>
hipError_t run_gf8(const Gf8Launch &L, hipStream_t stream);
template <int W, int R>
hipError_t run_bm(const BmLaunch &L, hipStream_t stream);
template <int K, int R>
hipError_t run_gf8_gather(const GatherLaunch &L, hipStream_t stream);
template <int W, int R>
hipError_t run_bm_gather(const GatherLaunch &L, hipStream_t stream);
// instantiated in gf8_r*.hip, gg8_r*.hip, bm_w*.hip and gbm.hip, never here
MEC_FOR_K(MEC_GF8_EXT, 1) MEC_FOR_K(MEC_GF8_EXT, 2) MEC_FOR_K(MEC_GF8_EXT, 3) MEC_FOR_K(MEC_GF8_EXT, 4)
MEC_FOR_K(MEC_GFM_EXT, 3) MEC_FOR_K(MEC_GFM_EXT, 4) MEC_FOR_K8(MEC_GFM_EXT)
MEC_FOR_K(MEC_GG8_EXT, 1) MEC_FOR_K(MEC_GG8_EXT, 2) MEC_FOR_K(MEC_GG8_EXT, 3) MEC_FOR_K(MEC_GG8_EXT, 4)
MEC_FOR_W(MEC_FOR_R8, MEC_BM_EXT)
MEC_FOR_W(MEC_FOR_R8, MEC_GBM_EXT)

// Gathered tails: the < unit remainder of each region, one thread per
// stripe, any k / rows / w, reading the descriptor blob directly.
__global__ __launch_bounds__(kThreads) void gather_tail_kernel(const GatherParams p, uint32_t n_stripes, uint32_t rows,
                                                               uint32_t w, uint64_t off, uint32_t n, uint32_t bitmatrix) {
    const uint32_t s = blockIdx.x * kThreads + threadIdx.x;
    if (s >= n_stripes) return;
    const uint32_t di = gather_desc(p, s);
    if (di == kSkipStripe) return;
    const uint32_t *D = p.desc + size_t(di) * p.desc_dw;
    const uint32_t sel_dw = bitmatrix ? 0 : 8, dsel_dw = bitmatrix ? 8 : 16;
    const uint64_t *srow = p.stab + uint64_t(s) * p.sstride;
    const uint64_t *drow = p.dtab + uint64_t(s) * p.dstride;
    auto src = [&](uint32_t j, uint64_t extra) -> u32x4 {
        const uint64_t a = srow[(D[sel_dw + j / 4] >> (8 * (j % 4))) & 0xffu];
        return a ? load_partial(reinterpret_cast<const uint8_t *>(a) + off + extra, n) : u32x4{0, 0, 0, 0};
    };
    MEC_DASSERT(rows <= (bitmatrix ? uint32_t(kBmGatherRows) : uint32_t(kMaxRows)));
    for (uint32_t i = 0; i < rows; ++i) {
        const uint32_t sel = (D[dsel_dw + i / 4] >> (8 * (i % 4))) & 0xffu;
        MEC_DASSERT(sel == kNoRow || sel < p.dstride);
        if (sel == kNoRow || !drow[sel]) continue;
        uint8_t *q0 = reinterpret_cast<uint8_t *>(drow[sel]) + off;
        if (!bitmatrix) {
            u32x4 acc = p.accumulate ? load_partial(q0, n) : u32x4{0, 0, 0, 0};
            for (uint32_t j = 0; j < p.k; ++j) {
                const u32x4 x = src(j, 0);
                const uint32_t *t = D + kGf8DescHead + (i * p.k + j) * 8;
                const Gf8Coef c{t[0], t[1], t[2], t[3], t[4]};
                acc ^= u32x4{gf8_mul(c, x.x), gf8_mul(c, x.y), gf8_mul(c, x.z), gf8_mul(c, x.w)};
            }
            store_partial(q0, acc, n);
        } else {
            for (uint32_t l = 0; l < w; ++l) {
                uint8_t *q = q0 + uint64_t(l) * p.packet;
                u32x4 acc = p.accumulate ? load_partial(q, n) : u32x4{0, 0, 0, 0};
                for (uint32_t j = 0; j < p.k; ++j) {
                    const uint32_t r = i * w + l;
                    const uint32_t mb = (D[kBmDescHead + j * 2 * w + r / 4] >> (8 * (r % 4))) & 0xffu;
                    for (uint32_t x = 0; x < w; ++x)
                        if ((mb >> x) & 1u) acc ^= src(j, uint64_t(x) * p.packet);
                }
                store_partial(q, acc, n);
            }
        }
    }
}

hipError_t launch_gather_tail(const GatherLaunch &L, bool bitmatrix, uint64_t off, hipStream_t stream) {
    Geometry g{};
    GatherParams p = gather_params(L, g);
    const uint32_t n = uint32_t(L.len - off);
    hipLaunchKernelGGL(gather_tail_kernel, dim3((L.n_stripes + kThreads - 1) / kThreads), dim3(kThreads), 0, stream, p,
                       L.n_stripes, uint32_t(L.rows), uint32_t(L.w), off, n, bitmatrix ? 1u : 0u);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Tails: the < 16-byte (gf8) / < unit (bitmatrix) remainder of each region,
// one thread per stripe.  Only launched for sizes that are not multiples of
// the vector unit.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void gf8_tail_kernel(const Gf8TailParams p) {
    const uint32_t s = blockIdx.x * kThreads + threadIdx.x;
    if (s >= p.n_stripes) return;
    const uint8_t *sb = p.stab ? nullptr : p.src + int64_t(s) * p.sss + p.off;
    uint8_t *db = p.stab ? nullptr : p.dst + int64_t(s) * p.dss + p.off;
    for (uint32_t i = 0; i < p.rows; ++i) {
        uint8_t *q = db ? db + p.dst_off[i] : reinterpret_cast<uint8_t *>(p.dtab[uint64_t(s) * p.dstride + p.dst_off[i]]);
        if (!q) continue;
        if (!db) q += p.off;
        u32x4 acc = p.accumulate ? load_partial(q, p.n) : u32x4{0, 0, 0, 0};
        for (uint32_t j = 0; j < p.k; ++j) {
            const uint8_t *a =
                sb ? sb + p.src_off[j] : reinterpret_cast<const uint8_t *>(p.stab[uint64_t(s) * p.sstride + p.src_off[j]]);
            if (!a) continue;
            if (!sb) a += p.off;
            const u32x4 x = load_partial(a, p.n);
            const Gf8Coef c = p.coef[i][j];
            acc ^= u32x4{gf8_mul(c, x.x), gf8_mul(c, x.y), gf8_mul(c, x.z), gf8_mul(c, x.w)};
        }
        store_partial(q, acc, p.n);
    }
}

hipError_t launch_gf8_tail(const Gf8Launch &L, uint64_t off, hipStream_t stream) {
    Gf8TailParams p;
    p.src = L.src;
    p.dst = L.dst;
    p.sss = L.src_stripe_stride;
    p.dss = L.dst_stripe_stride;
    p.stab = L.stab;
    p.dtab = L.dtab;
    p.sstride = L.sstride;
    p.dstride = L.dstride;
    p.off = off;
    p.n = uint32_t(L.len - off);
    p.k = uint32_t(L.k);
    p.rows = uint32_t(L.rows);
    p.n_stripes = L.n_stripes;
    p.accumulate = L.accumulate ? 1u : 0u;
    p.pad = 0;
    for (int j = 0; j < kMaxSrc; ++j) p.src_off[j] = L.src_off[j];
    for (int i = 0; i < kMaxRows; ++i) {
        p.dst_off[i] = L.dst_off[i];
        for (int j = 0; j < kMaxSrc; ++j) p.coef[i][j] = L.coef[i][j];
    }
    hipLaunchKernelGGL(gf8_tail_kernel, dim3((L.n_stripes + kThreads - 1) / kThreads), dim3(kThreads), 0, stream, p);
    return hipGetLastError();
}

struct BmTailParams {
    const uint8_t *src;
    uint8_t *dst;
    int64_t sss, dss;
    const uint64_t *stab, *dtab;
    uint32_t sstride, dstride;
    uint64_t packet, off;
    uint32_t n, k, rows, w, n_stripes, accumulate;
    int64_t src_off[kMaxSrc];
    int64_t dst_off[kMaxBmOut];
    uint8_t mask[kMaxSrc][kMaxBmRows];
};

__global__ __launch_bounds__(kThreads) void bm_tail_kernel(const BmTailParams p) {
    const uint32_t s = blockIdx.x * kThreads + threadIdx.x;
    if (s >= p.n_stripes) return;
    const uint8_t *sb = p.stab ? nullptr : p.src + int64_t(s) * p.sss + p.off;
    uint8_t *db = p.stab ? nullptr : p.dst + int64_t(s) * p.dss + p.off;
    for (uint32_t i = 0; i < p.rows; ++i)
        for (uint32_t l = 0; l < p.w; ++l) {
            uint8_t *q0 = db ? db + p.dst_off[i] : reinterpret_cast<uint8_t *>(p.dtab[uint64_t(s) * p.dstride + p.dst_off[i]]);
            if (!q0) continue;
            uint8_t *q = q0 + (db ? 0 : p.off) + uint64_t(l) * p.packet;
            u32x4 acc = p.accumulate ? load_partial(q, p.n) : u32x4{0, 0, 0, 0};
            for (uint32_t j = 0; j < p.k; ++j) {
                const uint8_t *a = sb ? sb + p.src_off[j]
                                      : reinterpret_cast<const uint8_t *>(p.stab[uint64_t(s) * p.sstride + p.src_off[j]]);
                if (!a) continue;
                if (!sb) a += p.off;
                const uint32_t mb = p.mask[j][i * p.w + l];
                for (uint32_t x = 0; x < p.w; ++x)
                    if ((mb >> x) & 1u) acc ^= load_partial(a + uint64_t(x) * p.packet, p.n);
            }
            store_partial(q, acc, p.n);
        }
}

hipError_t launch_bm_tail(const BmLaunch &L, uint64_t off, hipStream_t stream) {
    BmTailParams p;
    p.src = L.src;
    p.dst = L.dst;
    p.sss = L.src_stripe_stride;
    p.dss = L.dst_stripe_stride;
    p.stab = L.stab;
    p.dtab = L.dtab;
    p.sstride = L.sstride;
    p.dstride = L.dstride;
    p.packet = L.packet;
    p.off = off;
    p.n = uint32_t(L.packet - off);
    p.k = uint32_t(L.k);
    p.rows = uint32_t(L.rows);
    p.w = uint32_t(L.w);
    p.n_stripes = L.n_stripes;
    p.accumulate = L.accumulate ? 1u : 0u;
    for (int j = 0; j < kMaxSrc; ++j) p.src_off[j] = L.src_off[j];
    for (int i = 0; i < kMaxBmOut; ++i) p.dst_off[i] = L.dst_off[i];
    for (int j = 0; j < kMaxSrc; ++j)
        for (int r = 0; r < kMaxBmRows; ++r) p.mask[j][r] = L.mask[j][r];
    hipLaunchKernelGGL(bm_tail_kernel, dim3((L.n_stripes + kThreads - 1) / kThreads), dim3(kThreads), 0, stream, p);
    return hipGetLastError();
}

}  // namespace detail

using namespace detail;

Gf8Coef gf8_coef(uint8_t c) {
    const Field &f = Field::get(8);
    auto pack = [&](unsigned a, unsigned b, unsigned cc, unsigned d) {
        return uint32_t(f.mul(c, a)) | uint32_t(f.mul(c, b)) << 8 | uint32_t(f.mul(c, cc)) << 16 |
               uint32_t(f.mul(c, d)) << 24;
    };
    Gf8Coef r;
    r.t0 = pack(0, 1, 2, 3);
    r.t1 = pack(4, 5, 6, 7);
    r.u0 = pack(0, 8, 16, 24);
    r.u1 = pack(32, 40, 48, 56);
    r.v = pack(0, 64, 128, 192);
    return r;
}

namespace {

using Gf8Fn = hipError_t (*)(const Gf8Launch &, hipStream_t);

template <size_t... I>
constexpr std::array<Gf8Fn, sizeof...(I)> make_gf8_table(std::index_sequence<I...>) {
    return {{&run_gf8<int(I / kMaxRows) + 1, int(I % kMaxRows) + 1>...}};
}
const auto kGf8Table = make_gf8_table(std::make_index_sequence<kMaxK * kMaxRows>{});

using Gf8MgFn = hipError_t (*)(const Gf8MgLaunch &, hipStream_t);

template <size_t... I>
constexpr std::array<Gf8MgFn, sizeof...(I)> make_gfm_table(std::index_sequence<I...>) {
    return {{&run_gf8_mg<int(I / 2) + 1, int(I % 2) + 3>...}};
}
const auto kGfmTable = make_gfm_table(std::make_index_sequence<kMaxK * 2>{});

template <size_t... I>
constexpr std::array<Gf8MgFn, sizeof...(I)> make_gfm8_table(std::index_sequence<I...>) {
    return {{&run_gf8_mg<int(I) + kMg8MinK, 8>...}};
}
const auto kGfm8Table = make_gfm8_table(std::make_index_sequence<kMg8MaxK - kMg8MinK + 1>{});

using BmFn = hipError_t (*)(const BmLaunch &, hipStream_t);

template <size_t... I>
constexpr std::array<BmFn, sizeof...(I)> make_bm_table(std::index_sequence<I...>) {
    return {{&run_bm<int(I / kMaxBmOut) + 1, int(I % kMaxBmOut) + 1>...}};
}
const auto kBmTable = make_bm_table(std::make_index_sequence<8 * kMaxBmOut>{});

using GatherFn = hipError_t (*)(const GatherLaunch &, hipStream_t);

template <size_t... I>
constexpr std::array<GatherFn, sizeof...(I)> make_gg8_table(std::index_sequence<I...>) {
    return {{&run_gf8_gather<int(I / kMaxRows) + 1, int(I % kMaxRows) + 1>...}};
}
const auto kGg8Table = make_gg8_table(std::make_index_sequence<kMaxK * kMaxRows>{});

template <size_t... I>
constexpr std::array<GatherFn, sizeof...(I)> make_gbm_table(std::index_sequence<I...>) {
    return {{&run_bm_gather<int(I / kBmGatherRows) + 1, int(I % kBmGatherRows) + 1>...}};
}
const auto kGbmTable = make_gbm_table(std::make_index_sequence<8 * kBmGatherRows>{});

// ---------------------------------------------------------------------------
// XOR and fill
// ---------------------------------------------------------------------------
// One 16-byte unit per lane over the whole region (grid-stride only past
// 16 GiB), non-temporal: a plain 2-read / 1-write HBM stream, also the
// bench's on-box streaming ceiling.  dst may alias a or b (parity ^= delta).
template <int BT>
__global__ __launch_bounds__(BT) void xor_kernel(uint8_t *dst, const uint8_t *a, const uint8_t *b, uint64_t len) {
    // each block's BT x 16-byte span as three buffer resources (uniform
    // bases, 32-bit lane offsets), as the coding kernels stream
    const uint64_t stride = uint64_t(gridDim.x) * BT * 16;
    for (uint64_t base = uint64_t(blockIdx.x) * BT * 16; base < len; base += stride) {
        const uint64_t span = std::min<uint64_t>(len - base, uint64_t(BT) * 16);
        const uint32_t off = threadIdx.x * 16;
        if (off + 16 <= span) {
            const auto ra = chunk_rsrc(uint64_t(uintptr_t(a + base)), uint32_t(span));
            const auto rb = chunk_rsrc(uint64_t(uintptr_t(b + base)), uint32_t(span));
            const auto rd = chunk_rsrc(uint64_t(uintptr_t(dst + base)), uint32_t(span));
            buf_st(buf_ld<u32x4>(ra, off, true) ^ buf_ld<u32x4>(rb, off, true), rd, off);
        } else if (off < span) {
            const uint32_t n = uint32_t(span - off);
            store_partial(dst + base + off, load_partial(a + base + off, n) ^ load_partial(b + base + off, n), n);
        }
    }
}

__device__ __forceinline__ uint64_t splitmix(uint64_t seed, uint64_t q) {
    uint64_t z = seed + (q + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(kThreads) void fill_kernel(uint8_t *dst, uint64_t len, uint64_t seed,
                                                        uint64_t word_offset) {
    const uint64_t stride = uint64_t(gridDim.x) * kThreads * 16;
    for (uint64_t off = (uint64_t(blockIdx.x) * kThreads + threadIdx.x) * 16; off < len; off += stride) {
        const uint64_t q = word_offset + off / 8;
        const uint64_t a = splitmix(seed, q), b = splitmix(seed, q + 1);
        const u32x4 v{uint32_t(a), uint32_t(a >> 32), uint32_t(b), uint32_t(b >> 32)};
        if (off + 16 <= len)
            *reinterpret_cast<u32x4 *>(dst + off) = v;
        else
            store_partial(dst + off, v, uint32_t(len - off));
    }
}

uint32_t stream_blocks(uint64_t len) {
    uint64_t b = (len + uint64_t(kThreads) * 16 - 1) / (uint64_t(kThreads) * 16);
    return uint32_t(std::min<uint64_t>(std::max<uint64_t>(b, 1), 256 * 16));
}

}  // namespace

hipError_t launch_gf8(const Gf8Launch &L, hipStream_t stream) {
    if (L.k < 1 || L.k > kMaxK || L.rows < 1 || L.rows > kMaxRows) return hipErrorInvalidValue;
    if (L.len == 0 || L.n_stripes == 0) return hipSuccess;
    if (L.len / 16 > uint64_t(UINT32_MAX)) return hipErrorInvalidValue;
    return kGf8Table[size_t(L.k - 1) * kMaxRows + size_t(L.rows - 1)](L, stream);
}

hipError_t launch_gf8_mg(const Gf8MgLaunch &L, hipStream_t stream) {
    if (L.k < 1 || L.k > kMaxK || L.rows <= kMaxRows || L.rows > kMaxSrc || !L.tabs || L.len % 16) return hipErrorInvalidValue;
    if (L.len == 0 || L.n_stripes == 0) return hipSuccess;
    if (L.len / 16 > uint64_t(UINT32_MAX)) return hipErrorInvalidValue;
    // every group's rows index the kernel's kMaxSrc dst_off slots
    if (L.group_rows < 1 || ((L.rows + L.group_rows - 1) / L.group_rows) * L.group_rows > kMaxSrc)
        return hipErrorInvalidValue;
    if (L.group_rows == 8) {
        if (L.k < kMg8MinK || L.k > kMg8MaxK) return hipErrorInvalidValue;
        return kGfm8Table[size_t(L.k - kMg8MinK)](L, stream);
    }
    if (L.group_rows != 3 && L.group_rows != 4) return hipErrorInvalidValue;
    return kGfmTable[size_t(L.k - 1) * 2 + size_t(L.group_rows - 3)](L, stream);
}

void gf8_mg_tables(const uint8_t *coef, int rows, int k, int R, std::vector<uint32_t> &out) {
    const int groups = (rows + R - 1) / R;
    out.assign(size_t(groups) * R * k * 8, 0u);
    for (int r = 0; r < rows; ++r)
        for (int j = 0; j < k; ++j) {
            const Gf8Coef c = gf8_coef(coef[size_t(r) * k + j]);
            uint32_t *t = &out[(size_t(r) * k + j) * 8];
            t[0] = c.t0;
            t[1] = c.t1;
            t[2] = c.u0;
            t[3] = c.u1;
            t[4] = c.v;
        }
}

hipError_t launch_bm(const BmLaunch &L, hipStream_t stream) {
    if (L.k < 1 || L.k > kMaxK || L.rows < 1 || L.rows > kMaxBmOut || L.w < 1 || L.w > 8)
        return hipErrorInvalidValue;
    if (L.packet == 0 || L.n_stripes == 0) return hipSuccess;
    return kBmTable[size_t(L.w - 1) * kMaxBmOut + size_t(L.rows - 1)](L, stream);
}

hipError_t launch_gf8_gather(const GatherLaunch &L, hipStream_t stream) {
    if (L.k < 1 || L.k > kMaxK || L.rows < 1 || L.rows > kMaxRows || !L.stab || !L.dtab || !L.desc)
        return hipErrorInvalidValue;
    if (L.len == 0 || L.n_stripes == 0) return hipSuccess;
    if (L.len / 16 > uint64_t(UINT32_MAX)) return hipErrorInvalidValue;
    return kGg8Table[size_t(L.k - 1) * kMaxRows + size_t(L.rows - 1)](L, stream);
}

hipError_t launch_bm_gather(const GatherLaunch &L, hipStream_t stream) {
    if (L.k < 1 || L.k > kMaxK || L.rows < 1 || L.rows > kBmGatherRows || L.w < 1 || L.w > 8 || !L.stab ||
        !L.dtab || !L.desc)
        return hipErrorInvalidValue;
    if (L.len == 0 || L.n_stripes == 0) return hipSuccess;
    return kGbmTable[size_t(L.w - 1) * kBmGatherRows + size_t(L.rows - 1)](L, stream);
}

hipError_t launch_xor(uint8_t *dst, const uint8_t *a, const uint8_t *b, uint64_t len, hipStream_t stream) {
    if (len == 0) return hipSuccess;
    const KernelPlan pl = plan_xor(len);
    if (!pl.ok) return hipErrorInvalidValue;
    const dim3 grid(uint32_t(pl.grid));
    if (pl.bt == kWaveBlock)
        hipLaunchKernelGGL((xor_kernel<kWaveBlock>), grid, dim3(pl.bt), pl.lds_dynamic, stream, dst, a, b, len);
    else
        hipLaunchKernelGGL((xor_kernel<kThreads>), grid, dim3(pl.bt), pl.lds_dynamic, stream, dst, a, b, len);
    return hipGetLastError();
}

// 32-bit slab offsets -> chunk pointers (mec_*_batch32): entry e becomes
// base + (off << shift), or 0 (NULL) for kNullOff.  Four entries per lane:
// one 16-byte load, two 16-byte stores; the rest one at a time.
__global__ __launch_bounds__(kThreads) void expand_rows_kernel(const uint32_t *in, uint64_t *out, uint64_t base,
                                                               uint32_t shift, uint64_t n) {
    const uint64_t q = uint64_t(blockIdx.x) * kThreads + threadIdx.x, e = q * 4;
    auto one = [&](uint32_t o) -> uint64_t { return o == kNullOff ? 0 : base + (uint64_t(o) << shift); };
    if (e + 4 <= n) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(in + e);
        reinterpret_cast<u64x2 *>(out + e)[0] = u64x2{one(v.x), one(v.y)};
        reinterpret_cast<u64x2 *>(out + e)[1] = u64x2{one(v.z), one(v.w)};
    } else {
        for (uint64_t i = e; i < n; ++i) out[i] = one(in[i]);
    }
}

hipError_t launch_expand_rows(const uint32_t *in, uint64_t *out, uint64_t base, uint32_t shift, uint64_t n,
                              hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n + 4ull * kThreads - 1) / (4ull * kThreads);
    if (blocks >= (uint64_t(1) << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(expand_rows_kernel, dim3(uint32_t(blocks)), dim3(kThreads), 0, stream, in, out, base, shift, n);
    return hipGetLastError();
}

hipError_t launch_fill(uint8_t *dst, uint64_t len, uint64_t seed, uint64_t word_offset, hipStream_t stream) {
    if (len == 0) return hipSuccess;
    hipLaunchKernelGGL(fill_kernel, dim3(stream_blocks(len)), dim3(kThreads), 0, stream, dst, len, seed,
                       word_offset);
    return hipGetLastError();
}

}  // namespace mec
