// bm_kernel.hpp — bitmatrix packet XOR (Jerasure Cauchy-RS).  Instantiated
// per field width in bm_w{lo,hi}.hip.
//
// A chunk is w packets of chunk/w bytes (cauchycoding.cc:80).  Output packet
// r = i*w + l is the XOR of the source packets (j, x) whose bit is set in
// the (m*w) x (k*w) bitmatrix — exactly what the reference's schedule
// computes (jerasure_do_scheduled_operations, jerasure.c:1162-1185) without
// materialising intermediate packets: each lane keeps its R*W output slices
// in registers and streams the k*w source slices through once.  The bits
// are kernel arguments expanded to 0/~0 masks in SGPRs, so every (output,
// input) pair is one v_bitop3_b32 (acc ^ (d & m)) per dword; the next
// source chunk is loaded while the current one is being combined.
#pragma once

#include "stream_common.hpp"

namespace mec {
namespace detail {

template <int VW>
struct VecT;
template <>
struct VecT<4> {
    typedef u32x4 type;
};
template <>
struct VecT<2> {
    typedef u32x2 type;
};

// (d & m) ^ acc, one v_bitop3_b32 per dword (truth table over
// src0 = 0xF0, src1 = 0xCC, src2 = 0xAA: (0xF0 & 0xCC) ^ 0xAA = 0x6A).
__device__ __forceinline__ uint32_t and_xor(uint32_t d, uint32_t m, uint32_t acc) {
    return uint32_t(__builtin_amdgcn_bitop3_b32(d, m, acc, 0x6A));
}
__device__ __forceinline__ u32x4 and_xor(u32x4 d, uint32_t m, u32x4 acc) {
    return u32x4{and_xor(d.x, m, acc.x), and_xor(d.y, m, acc.y), and_xor(d.z, m, acc.z), and_xor(d.w, m, acc.w)};
}
__device__ __forceinline__ u32x2 and_xor(u32x2 d, uint32_t m, u32x2 acc) {
    return u32x2{and_xor(d.x, m, acc.x), and_xor(d.y, m, acc.y)};
}

template <int W, int R>
struct BmParams {
    const uint8_t *src;
    uint8_t *dst;
    int64_t sss, dss;
    const uint64_t *stab, *dtab;  // gather mode, as Gf8Params
    uint32_t sstride, dstride, chunk, s0;
    uint64_t packet;
    uint32_t units, tiles, k, accumulate, win, pad;
    uint32_t nstr, sgroup, srun, skew;  // stripe-group map and tile skew (stream_common.hpp stripe_tile)
    int64_t src_off[kMaxSrc];
    int64_t dst_off[R];
    uint8_t mask[kMaxSrc][R * W];
};

template <int W>
constexpr int bm_vw() {
    return W <= 4 ? 4 : 2;
}

// acc[r] ^= AND of source packet x with the 0 / ~0 mask of bit x of the
// (uniform) mask byte mb[r]: one v_bitop3_b32 per dword.
template <int W, int ROWS, typename vec>
__device__ __forceinline__ void bm_combine(const vec (&d)[W], vec (&acc)[ROWS], const uint8_t *mb) {
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
        const uint32_t b = mb[r];
#pragma unroll
        for (int x = 0; x < W; ++x) {
            // 0 / ~0 from a kernel-argument bit (SALU); acc ^= d & m is one
            // v_bitop3_b32 per dword on gfx950.
            const uint32_t m = 0u - ((b >> x) & 1u);
            acc[r] = and_xor(d[x], m, acc[r]);
        }
    }
}

template <int W, int R, bool G, int BT, int VW = bm_vw<W>()>
__global__ __launch_bounds__(BT) void bm_kernel(const BmParams<W, R> p) {
    constexpr int ROWS = R * W;
    typedef typename VecT<VW>::type vec;
    const uint32_t bid = block_order(p.win);
    uint32_t stripe, tile;
    stripe_tile(bid, p.tiles, p.nstr, p.sgroup, p.srun, p.skew, stripe, tile);
    uint32_t u = tile * BT + threadIdx.x;
    if constexpr (G) {
        if (!gather_unit<BT>(tile, p.units, u)) return;
    } else if (u >= p.units) {
        return;
    }
    vec acc[ROWS];
    vec d[W], nx[W];
    if constexpr (G) {
        const uint32_t off = u * (4 * VW);
        const uint32_t pk = uint32_t(p.packet);
        const uint64_t s = p.s0 + stripe;
        // the stripe's pointer row, one vector load (stream_common.hpp row_fetch)
        static_assert(R <= 32, "pointer row lanes");
        const uint64_t row = row_fetch(p.stab + s * p.sstride, p.src_off, p.k, p.dtab + s * p.dstride, p.dst_off, R);
        __amdgpu_buffer_rsrc_t dr[R];
#pragma unroll
        for (int i = 0; i < R; ++i) dr[i] = chunk_rsrc(row_entry(row, 32u + i), p.chunk);
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
            for (int l = 0; l < W; ++l) acc[i * W + l] = p.accumulate ? buf_ld<vec>(dr[i], off + l * pk, true) : vec(0);
        {
            const __amdgpu_buffer_rsrc_t sr = chunk_rsrc(row_entry(row, 0), p.chunk);
#pragma unroll
            for (int x = 0; x < W; ++x) d[x] = buf_ld<vec>(sr, off + x * pk, true);
        }
        for (uint32_t j = 0; j < p.k; ++j) {
            if (j + 1 < p.k) {
                const __amdgpu_buffer_rsrc_t sr = chunk_rsrc(row_entry(row, j + 1), p.chunk);
#pragma unroll
                for (int x = 0; x < W; ++x) nx[x] = buf_ld<vec>(sr, off + x * pk, true);
            }
            bm_combine<W, ROWS, vec>(d, acc, p.mask[j]);
#pragma unroll
            for (int x = 0; x < W; ++x) d[x] = nx[x];
        }
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
            for (int l = 0; l < W; ++l) buf_st(acc[i * W + l], dr[i], off + l * pk);
    } else {  // strided: chunk bases uniform per block, buffer resources as above
        const uint32_t off = u * (4 * VW);
        const uint32_t pk = uint32_t(p.packet);
        const uint8_t *sb = p.src + int64_t(stripe) * p.sss;
        uint8_t *db = p.dst + int64_t(stripe) * p.dss;
        __amdgpu_buffer_rsrc_t dr[R];
#pragma unroll
        for (int i = 0; i < R; ++i) dr[i] = chunk_rsrc(uint64_t(uintptr_t(db + p.dst_off[i])), p.chunk);
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
            for (int l = 0; l < W; ++l) acc[i * W + l] = p.accumulate ? buf_ld<vec>(dr[i], off + l * pk, true) : vec(0);
        {
            const __amdgpu_buffer_rsrc_t sr = chunk_rsrc(uint64_t(uintptr_t(sb + p.src_off[0])), p.chunk);
#pragma unroll
            for (int x = 0; x < W; ++x) d[x] = buf_ld<vec>(sr, off + x * pk, true);
        }
        for (uint32_t j = 0; j < p.k; ++j) {
            if (j + 1 < p.k) {
                const __amdgpu_buffer_rsrc_t sr = chunk_rsrc(uint64_t(uintptr_t(sb + p.src_off[j + 1])), p.chunk);
#pragma unroll
                for (int x = 0; x < W; ++x) nx[x] = buf_ld<vec>(sr, off + x * pk, true);
            }
            bm_combine<W, ROWS, vec>(d, acc, p.mask[j]);
#pragma unroll
            for (int x = 0; x < W; ++x) d[x] = nx[x];
        }
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
            for (int l = 0; l < W; ++l) buf_st(acc[i * W + l], dr[i], off + l * pk);
    }
}

hipError_t launch_bm_tail(const BmLaunch &L, uint64_t off, hipStream_t stream);

template <int W, int R, int VW>
hipError_t run_bm_vw(const BmLaunch &L, hipStream_t stream) {
    constexpr int UB = 4 * VW;
    BmParams<W, R> p;
    p.sss = L.src_stripe_stride;
    p.dss = L.dst_stripe_stride;
    p.packet = L.packet;
    p.k = uint32_t(L.k);
    p.stab = L.stab;
    p.dtab = L.dtab;
    p.sstride = L.sstride;
    p.dstride = L.dstride;
    p.chunk = uint32_t(L.packet * uint64_t(L.w));
    p.accumulate = L.accumulate ? 1u : 0u;
    p.pad = 0;
    p.skew = 0;
    for (int j = 0; j < kMaxSrc; ++j) p.src_off[j] = j < L.k ? L.src_off[j] : 0;
    for (int i = 0; i < R; ++i) p.dst_off[i] = L.dst_off[i];
    for (int j = 0; j < kMaxSrc; ++j)
        for (int r = 0; r < R * W; ++r) p.mask[j][r] = j < L.k ? L.mask[j][r] : 0;
    for (uint32_t s0 = 0; s0 < L.n_stripes;) {
        const KernelPlan pl = plan_bm(L, s0);
        if (!pl.ok || pl.k != L.k || pl.rows != R || pl.vw != uint32_t(VW)) return hipErrorInvalidValue;
        if (pl.geo.units == 0) break;
        p.units = pl.geo.units;
        p.tiles = pl.geo.tiles;
        p.s0 = s0;
        p.win = pl.win;
        p.nstr = L.stab ? 0 : pl.ns;
        p.sgroup = pl.sgroup;
        p.srun = pl.srun;
        p.skew = pl.skew;
        p.src = L.stab ? nullptr : L.src + int64_t(s0) * L.src_stripe_stride;
        p.dst = L.stab ? nullptr : L.dst + int64_t(s0) * L.dst_stripe_stride;
        const dim3 grid(uint32_t(pl.grid)), block(pl.bt);
        if (L.stab) {
            if (pl.bt == kWaveBlock)
                hipLaunchKernelGGL((bm_kernel<W, R, true, kWaveBlock, VW>), grid, block, pl.lds_dynamic, stream, p);
            else
                hipLaunchKernelGGL((bm_kernel<W, R, true, kThreads, VW>), grid, block, pl.lds_dynamic, stream, p);
        } else {
            if (pl.bt == kWaveBlock)
                hipLaunchKernelGGL((bm_kernel<W, R, false, kWaveBlock, VW>), grid, block, pl.lds_dynamic, stream, p);
            else
                hipLaunchKernelGGL((bm_kernel<W, R, false, kThreads, VW>), grid, block, pl.lds_dynamic, stream, p);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        s0 += pl.ns;
    }
    if (L.packet % UB) return launch_bm_tail(L, uint64_t(L.packet / UB) * UB, stream);
    return hipSuccess;
}

// Lane width from the plan (bm_lane_bytes for strided launches; gathered
// launches keep the default width).
template <int W, int R>
hipError_t run_bm(const BmLaunch &L, hipStream_t stream) {
    if constexpr (bm_vw<W>() == 4) {
        if (L.n_stripes && plan_bm(L, 0).vw == 2) return run_bm_vw<W, R, 2>(L, stream);
    }
    return run_bm_vw<W, R, bm_vw<W>()>(L, stream);
}

#define MEC_BM_ONE(W, R) template hipError_t run_bm<W, R>(const BmLaunch &, hipStream_t);
#define MEC_BM_EXT(W, R) extern template hipError_t run_bm<W, R>(const BmLaunch &, hipStream_t);
#define MEC_FOR_R4(X, W) X(W, 1) X(W, 2) X(W, 3) X(W, 4)
#define MEC_FOR_R8(X, W) MEC_FOR_R4(X, W) X(W, 5) X(W, 6) X(W, 7) X(W, 8)
#define MEC_FOR_W(F, X) F(X, 1) F(X, 2) F(X, 3) F(X, 4) F(X, 5) F(X, 6) F(X, 7) F(X, 8)
// strided and gathered launches take up to kMaxBmOut = 8 outputs (R = 1..8)
#define MEC_BM_INSTANTIATE_W(W) MEC_FOR_R8(MEC_BM_ONE, W)

}  // namespace detail
}  // namespace mec
