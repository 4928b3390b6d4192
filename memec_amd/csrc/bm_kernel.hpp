// bm_kernel.hpp — bitmatrix packet XOR (Jerasure Cauchy-RS).  Instantiated
// per field width in bm_w{lo,hi}.hip.
//
// A chunk is w packets of chunk/w bytes (cauchycoding.cc:80).  Output packet
// r = i*w + l is the XOR of the source packets (j, x) whose bit is set in
// the (m*w) x (k*w) bitmatrix, i.e. exactly what the reference's schedule
// computes (jerasure_do_scheduled_operations, jerasure.c:1162-1185) without
// materialising intermediate packets: each lane keeps its m*w output slices
// in registers and streams the k*w source slices through once.
#pragma once

#include "stream_common.hpp"

namespace mec {
namespace detail {

// ---------------------------------------------------------------------------
// Bitmatrix packet XOR (Cauchy-RS)
// ---------------------------------------------------------------------------
template <int W, int R, int VW>
struct BmParams {
    const uint8_t *src;
    uint8_t *dst;
    int64_t sss, dss;
    uint64_t packet;
    uint32_t units, tiles, upt, accumulate, k;
    int64_t src_off[kMaxSrc];
    int64_t dst_off[R];
    uint8_t mask[kMaxSrc][R * W];
};

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

template <int VW>
__device__ inline typename VecT<VW>::type vload_partial(const uint8_t *p, uint32_t n);
template <>
__device__ inline u32x4 vload_partial<4>(const uint8_t *p, uint32_t n) { return load_partial(p, n); }
template <>
__device__ inline u32x2 vload_partial<2>(const uint8_t *p, uint32_t n) {
    u32x4 v = load_partial(p, n);
    return u32x2{v.x, v.y};
}
__device__ inline void vstore_partial(uint8_t *p, u32x4 v, uint32_t n) { store_partial(p, v, n); }
__device__ inline void vstore_partial(uint8_t *p, u32x2 v, uint32_t n) { store_partial(p, u32x4{v.x, v.y, 0, 0}, n); }

template <int W, int R, int VW, bool FULL>
__device__ __forceinline__ void bm_unit(const BmParams<W, R, VW> &p, const uint8_t *sb, uint8_t *db,
                                        uint64_t off, uint32_t n) {
    typedef typename VecT<VW>::type vec;
    constexpr int ROWS = R * W;
    vec acc[ROWS];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
        for (int l = 0; l < W; ++l) {
            const uint8_t *q = db + p.dst_off[i] + uint64_t(l) * p.packet + off;
            if (p.accumulate)
                acc[i * W + l] = FULL ? *reinterpret_cast<const vec *>(q) : vload_partial<VW>(q, n);
            else
                acc[i * W + l] = vec(0);
        }
    for (uint32_t j = 0; j < p.k; ++j) {
        vec d[W];
        const uint8_t *s = sb + p.src_off[j] + off;
#pragma unroll
        for (int x = 0; x < W; ++x)
            d[x] = FULL ? *reinterpret_cast<const vec *>(s + uint64_t(x) * p.packet)
                        : vload_partial<VW>(s + uint64_t(x) * p.packet, n);
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const uint32_t mb = p.mask[j][r];
#pragma unroll
            for (int x = 0; x < W; ++x) {
                const uint32_t m = 0u - ((mb >> x) & 1u);
                acc[r] ^= d[x] & m;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
        for (int l = 0; l < W; ++l) {
            uint8_t *q = db + p.dst_off[i] + uint64_t(l) * p.packet + off;
            if (FULL)
                *reinterpret_cast<vec *>(q) = acc[i * W + l];
            else
                vstore_partial(q, acc[i * W + l], n);
        }
}

template <int W, int R, int VW>
__global__ __launch_bounds__(kThreads) void bm_kernel(const BmParams<W, R, VW> p) {
    constexpr uint32_t UB = 4 * VW;
    const uint32_t stripe = blockIdx.x / p.tiles;
    const uint32_t tile = blockIdx.x - stripe * p.tiles;
    const uint8_t *sb = p.src + int64_t(stripe) * p.sss;
    uint8_t *db = p.dst + int64_t(stripe) * p.dss;
    const uint32_t ubase = tile * p.upt * kThreads + threadIdx.x;
    for (uint32_t r = 0; r < p.upt; ++r) {
        const uint32_t u = ubase + r * kThreads;
        if (u >= p.units) return;
        const uint64_t off = uint64_t(u) * UB;
        if (off + UB <= p.packet)
            bm_unit<W, R, VW, true>(p, sb, db, off, UB);
        else
            bm_unit<W, R, VW, false>(p, sb, db, off, uint32_t(p.packet - off));
    }
}

template <int W, int R>
hipError_t run_bm(const BmLaunch &L, hipStream_t stream) {
    constexpr int VW = W <= 4 ? 4 : 2;
    BmParams<W, R, VW> p;
    p.sss = L.src_stripe_stride;
    p.dss = L.dst_stripe_stride;
    p.packet = L.packet;
    p.k = uint32_t(L.k);
    const Geometry g = geometry((L.packet + 4 * VW - 1) / (4 * VW));
    p.units = g.units;
    p.tiles = g.tiles;
    p.upt = g.upt;
    p.accumulate = L.accumulate ? 1u : 0u;
    for (int j = 0; j < kMaxSrc; ++j) p.src_off[j] = j < L.k ? L.src_off[j] : 0;
    for (int i = 0; i < R; ++i) p.dst_off[i] = L.dst_off[i];
    for (int j = 0; j < kMaxSrc; ++j)
        for (int r = 0; r < R * W; ++r) p.mask[j][r] = j < L.k ? L.mask[j][r] : 0;
    for (uint32_t s0 = 0; s0 < L.n_stripes; s0 += g.max_stripes_per_launch) {
        const uint32_t ns = std::min(L.n_stripes - s0, g.max_stripes_per_launch);
        p.src = L.src + int64_t(s0) * L.src_stripe_stride;
        p.dst = L.dst + int64_t(s0) * L.dst_stripe_stride;
        hipLaunchKernelGGL((bm_kernel<W, R, VW>), dim3(ns * g.tiles), dim3(kThreads), 0, stream, p);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}


#define MEC_BM_INSTANTIATE_W(W) \
    template hipError_t run_bm<W, 1>(const BmLaunch &, hipStream_t); \
    template hipError_t run_bm<W, 2>(const BmLaunch &, hipStream_t); \
    template hipError_t run_bm<W, 3>(const BmLaunch &, hipStream_t); \
    template hipError_t run_bm<W, 4>(const BmLaunch &, hipStream_t);

}  // namespace detail
}  // namespace mec
