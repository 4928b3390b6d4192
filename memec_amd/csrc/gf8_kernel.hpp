// gf8_kernel.hpp — GF(2^8) byte-wise matrix apply (Jerasure RS, ISA-L RS /
// Cauchy).  Instantiated per row count in gf8_r{1..4}.hip.
//
// A product c*x is linear in the bits of x, so each byte is split into bit
// fields 0-2 | 3-5 | 6-7 and every field indexes a <= 8-entry table of
// c*(field << shift) with one v_perm_b32, four bytes per instruction:
// 3 v_perm + 3 v_xor per (coefficient, dword).  Replaces the scalar
// multtable[s][c] byte loop (gf_w8.c:1047-1050) and ISA-L's PSHUFB nibble
// kernels (gf_vect_dot_prod_sse.asm:215-230).
#pragma once

#include "stream_common.hpp"

namespace mec {
namespace detail {

// ---------------------------------------------------------------------------
// GF(2^8) byte-wise matrix apply
// ---------------------------------------------------------------------------
template <int K, int R>
struct Gf8Params {
    const uint8_t *src;
    uint8_t *dst;
    int64_t sss, dss;
    uint64_t len;
    uint32_t units, tiles, upt, accumulate;
    int64_t src_off[K];
    int64_t dst_off[R];
    Gf8Coef coef[R][K];
};

__device__ __forceinline__ uint32_t gf8_mul(const Gf8Coef &c, uint32_t s0, uint32_t s1, uint32_t s2) {
    return __builtin_amdgcn_perm(c.t1, c.t0, s0) ^ __builtin_amdgcn_perm(c.u1, c.u0, s1) ^
           __builtin_amdgcn_perm(c.v, c.v, s2);
}

template <int K, int R>
__device__ __forceinline__ void gf8_combine(const Gf8Params<K, R> &p, const u32x4 (&d)[K], u32x4 (&acc)[R]) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const u32x4 x = d[j];
        const u32x4 s0 = x & 0x07070707u;
        const u32x4 s1 = (x >> 3) & 0x07070707u;
        const u32x4 s2 = (x >> 6) & 0x03030303u;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const Gf8Coef &c = p.coef[i][j];
            acc[i].x ^= gf8_mul(c, s0.x, s1.x, s2.x);
            acc[i].y ^= gf8_mul(c, s0.y, s1.y, s2.y);
            acc[i].z ^= gf8_mul(c, s0.z, s1.z, s2.z);
            acc[i].w ^= gf8_mul(c, s0.w, s1.w, s2.w);
        }
    }
}

template <int K, int R>
__global__ __launch_bounds__(kThreads) void gf8_kernel(const Gf8Params<K, R> p) {
    const uint32_t stripe = blockIdx.x / p.tiles;
    const uint32_t tile = blockIdx.x - stripe * p.tiles;
    const uint8_t *sb = p.src + int64_t(stripe) * p.sss;
    uint8_t *db = p.dst + int64_t(stripe) * p.dss;
    const uint32_t ubase = tile * p.upt * kThreads + threadIdx.x;
    for (uint32_t r = 0; r < p.upt; ++r) {
        const uint32_t u = ubase + r * kThreads;
        if (u >= p.units) return;
        const uint64_t off = uint64_t(u) * 16;
        u32x4 d[K], acc[R];
        if (off + 16 <= p.len) {
#pragma unroll
            for (int j = 0; j < K; ++j) d[j] = *reinterpret_cast<const u32x4 *>(sb + p.src_off[j] + off);
#pragma unroll
            for (int i = 0; i < R; ++i)
                acc[i] = p.accumulate ? *reinterpret_cast<const u32x4 *>(db + p.dst_off[i] + off) : u32x4{0, 0, 0, 0};
            gf8_combine(p, d, acc);
#pragma unroll
            for (int i = 0; i < R; ++i) *reinterpret_cast<u32x4 *>(db + p.dst_off[i] + off) = acc[i];
        } else {
            const uint32_t n = uint32_t(p.len - off);
#pragma unroll
            for (int j = 0; j < K; ++j) d[j] = load_partial(sb + p.src_off[j] + off, n);
#pragma unroll
            for (int i = 0; i < R; ++i)
                acc[i] = p.accumulate ? load_partial(db + p.dst_off[i] + off, n) : u32x4{0, 0, 0, 0};
            gf8_combine(p, d, acc);
#pragma unroll
            for (int i = 0; i < R; ++i) store_partial(db + p.dst_off[i] + off, acc[i], n);
        }
    }
}

template <int K, int R>
hipError_t run_gf8(const Gf8Launch &L, hipStream_t stream) {
    Gf8Params<K, R> p;
    p.sss = L.src_stripe_stride;
    p.dss = L.dst_stripe_stride;
    p.len = L.len;
    const Geometry g = geometry((L.len + 15) / 16);
    p.units = g.units;
    p.tiles = g.tiles;
    p.upt = g.upt;
    p.accumulate = L.accumulate ? 1u : 0u;
    for (int j = 0; j < K; ++j) p.src_off[j] = L.src_off[j];
    for (int i = 0; i < R; ++i) p.dst_off[i] = L.dst_off[i];
    for (int i = 0; i < R; ++i)
        for (int j = 0; j < K; ++j) p.coef[i][j] = L.coef[i][j];
    for (uint32_t s0 = 0; s0 < L.n_stripes; s0 += g.max_stripes_per_launch) {
        const uint32_t ns = std::min(L.n_stripes - s0, g.max_stripes_per_launch);
        p.src = L.src + int64_t(s0) * L.src_stripe_stride;
        p.dst = L.dst + int64_t(s0) * L.dst_stripe_stride;
        hipLaunchKernelGGL((gf8_kernel<K, R>), dim3(ns * g.tiles), dim3(kThreads), 0, stream, p);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}


#define MEC_GF8_INSTANTIATE_K(R) \
    template hipError_t run_gf8<1, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<2, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<3, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<4, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<5, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<6, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<7, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<8, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<9, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<10, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<11, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<12, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<13, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<14, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<15, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<16, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<17, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<18, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<19, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<20, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<21, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<22, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<23, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<24, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<25, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<26, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<27, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<28, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<29, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<30, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<31, R>(const Gf8Launch &, hipStream_t); \
    template hipError_t run_gf8<32, R>(const Gf8Launch &, hipStream_t);

}  // namespace detail
}  // namespace mec
