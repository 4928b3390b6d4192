// gather_kernel.hpp — descriptor-driven gathered variants of the gf8 and
// bitmatrix kernels, for the pointer-array batches (mec_encode_batch,
// mec_decode_batch, mec_encode_update_batch).
//
// A block serves one (stripe, 256-unit tile) as in the strided kernels.  It
// finds its chunks through two device tables of chunk pointers (the
// caller's Chunk* rows, uploaded as they are) and its linear map through a
// descriptor: the stripe's erasure pattern (decode) or delta column
// (update) selects one, so every pattern in a batch shares one launch.
// A block's table entries are fetched once, cooperatively, into LDS and
// read back as wave-uniform SGPR values; each chunk is then a buffer
// resource (32-bit offsets, range-checked).  A NULL source pointer is an
// all-zero chunk (Coding::zeros, coding.cc:14-16): its resource has zero
// records, so it is not read; a NULL output is not written, the same way.
#pragma once

#include "bm_kernel.hpp"
#include "gf8_kernel.hpp"
#include "stream_common.hpp"

namespace mec {
namespace detail {

struct GatherParams {
    const uint64_t *stab;
    const uint64_t *dtab;
    const uint32_t *desc;  // descriptor blobs (layout in kernels.hpp), desc_dw dwords apart
    const uint16_t *pat;
    uint64_t packet;  // bitmatrix packet bytes
    uint32_t chunk;   // bytes per chunk (buffer range)
    uint32_t desc_dw;
    uint32_t sstride, dstride;
    uint32_t s0, units, tiles, k, accumulate;
    // gf8: row groups coded in this launch from one read of the sources;
    // group g's descriptor of map d at desc + (g * group_maps + d) * desc_dw
    uint32_t groups, group_maps;
};

__device__ __forceinline__ uint32_t gather_desc(const GatherParams &p, uint32_t s) {
    return p.pat ? uint32_t(p.pat[s]) : 0u;
}


// Block prologue of both gathered kernels, three dependent latencies: the
// stripe's descriptor index; the descriptor's first NDW dwords, one dword
// per thread, into LDS; the stripe's source and output pointers (wave 0
// and wave 1, selected by the descriptor) into LDS.
template <int NDW, int KMAX, int R>
__device__ __forceinline__ bool gather_prologue(const GatherParams &p, uint32_t s, uint32_t k, uint32_t *dsc,
                                                uint64_t *ptr, int sel_dw, int dsel_dw) {
    const uint32_t di = gather_desc(p, s);
    if (di == kSkipStripe) return false;
    MEC_DASSERT(p.group_maps == 0 || di < p.group_maps);
    const uint32_t *D = p.desc + size_t(di) * p.desc_dw;
    constexpr int NI = (NDW + kThreads - 1) / kThreads;
    uint32_t v[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int q = int(threadIdx.x) + i * kThreads;
        v[i] = q < NDW ? D[q] : 0u;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int q = int(threadIdx.x) + i * kThreads;
        if (q < NDW) dsc[q] = v[i];
    }
    __syncthreads();
    const int t = threadIdx.x;
    if (t < int(k)) {
        const uint32_t sel = (dsc[sel_dw + t / 4] >> (8 * (t % 4))) & 0xffu;
        MEC_DASSERT(sel < p.sstride);
        ptr[t] = p.stab[uint64_t(s) * p.sstride + sel];
    } else if (t >= 64 && t < 64 + R) {
        const uint32_t sel = (dsc[dsel_dw + (t - 64) / 4] >> (8 * ((t - 64) % 4))) & 0xffu;
        MEC_DASSERT(sel == kNoRow || sel < p.dstride);
        ptr[KMAX + t - 64] = sel == kNoRow ? 0 : p.dtab[uint64_t(s) * p.dstride + sel];
    }
    __syncthreads();
    return true;
}

// MG = false: one row group per launch (m <= 4; the kernel before round 4).
// MG = true (R = 4 only): every row group of the descriptors in one launch,
// the k sources read once (m > 4) — a separate instantiation because the
// group loop's barriers keep lanes past the chunk alive and cost ~20-30
// VGPRs, which the common m <= 4 launches should not pay.
template <int K, int R, bool MG>
__global__ __launch_bounds__(kThreads) void gf8_gather_kernel(const GatherParams p) {
    constexpr int NDW = kGf8DescHead + R * K * 8;
    __shared__ uint32_t dsc[NDW];
    __shared__ uint64_t ptr[K + R];
    const uint32_t local = blockIdx.x / p.tiles;
    const uint32_t s = p.s0 + local;
    if (!gather_prologue<NDW, K, R>(p, s, K, dsc, ptr, 8, 16)) return;
    const uint32_t u = (blockIdx.x - local * p.tiles) * kThreads + threadIdx.x;
    if constexpr (!MG) {
        if (u >= p.units) return;
        const uint32_t off = u * 16;
        u32x4 d[K];
#pragma unroll
        for (int j = 0; j < K; ++j) d[j] = buf_ld<u32x4>(chunk_rsrc(uniform64(ptr[j]), p.chunk), off, true);
        __amdgpu_buffer_rsrc_t dr[R];
#pragma unroll
        for (int i = 0; i < R; ++i) dr[i] = chunk_rsrc(uniform64(ptr[K + i]), p.chunk);
        u32x4 acc[R];
#pragma unroll
        for (int i = 0; i < R; ++i) acc[i] = p.accumulate ? buf_ld<u32x4>(dr[i], off, true) : u32x4{0, 0, 0, 0};
        gf8_apply<K, R, kGf8Dense>(d, acc, dsc + kGf8DescHead + opaque_zero());
#pragma unroll
        for (int i = 0; i < R; ++i) buf_st(acc[i], dr[i], off);
    } else {
        // lanes past the chunk stay for the group barriers, without memory ops
        const bool live = u < p.units;
        const uint32_t off = live ? u * 16 : 0u;
        u32x4 d[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
            d[j] = live ? buf_ld<u32x4>(chunk_rsrc(uniform64(ptr[j]), p.chunk), off, true) : u32x4{0, 0, 0, 0};
        for (uint32_t g = 0;;) {  // uniform
            __amdgpu_buffer_rsrc_t dr[R];
#pragma unroll
            for (int i = 0; i < R; ++i) dr[i] = chunk_rsrc(live ? uniform64(ptr[K + i]) : 0, p.chunk);
            u32x4 acc[R];
#pragma unroll
            for (int i = 0; i < R; ++i) acc[i] = p.accumulate ? buf_ld<u32x4>(dr[i], off, true) : u32x4{0, 0, 0, 0};
            gf8_apply<K, R, kGf8Dense>(d, acc, dsc + kGf8DescHead + opaque_zero());
#pragma unroll
            for (int i = 0; i < R; ++i) buf_st(acc[i], dr[i], off);
            if (++g >= p.groups) break;
            // next group: its descriptor (output rows, tables), its output pointers
            __syncthreads();
            const uint32_t *D = p.desc + (size_t(g) * p.group_maps + gather_desc(p, s)) * p.desc_dw;
            for (int q = threadIdx.x; q < NDW; q += kThreads) dsc[q] = D[q];
            __syncthreads();
            if (threadIdx.x < R) {
                const uint32_t sel = (dsc[16] >> (8 * threadIdx.x)) & 0xffu;
                MEC_DASSERT(sel == kNoRow || sel < p.dstride);
                ptr[K + threadIdx.x] = sel == kNoRow ? 0 : p.dtab[uint64_t(s) * p.dstride + sel];
            }
            __syncthreads();
            // the sources "change" (an empty asm): their bit fields are not
            // hoisted out of the group loop (as gf8_mg_kernel)
#pragma unroll
            for (int j = 0; j < K; ++j) asm volatile("" : "+v"(d[j]));
        }
    }
}

template <int W, int R>
__global__ __launch_bounds__(kThreads) void bm_gather_kernel(const GatherParams p) {
    constexpr int VW = bm_vw<W>();
    constexpr int UB = 4 * VW;
    constexpr int ROWS = R * W;
    constexpr int MW = (ROWS + 3) / 4;  // mask dwords used per source (of W stored)
    constexpr int MS = 2 * W;  // mask dwords per source (kBmGatherRows rows of W bytes)
    constexpr int NDW = kBmDescHead + kMaxSrc * MS;
    typedef typename VecT<VW>::type vec;
    __shared__ uint32_t dsc[NDW];
    __shared__ uint64_t ptr[kMaxSrc + R];
    const uint32_t local = blockIdx.x / p.tiles;
    const uint32_t k = p.k;
    if (!gather_prologue<NDW, kMaxSrc, R>(p, p.s0 + local, k, dsc, ptr, 0, 8)) return;
    const uint32_t u = (blockIdx.x - local * p.tiles) * kThreads + threadIdx.x;
    if (u >= p.units) return;
    const uint32_t off = u * UB;
    const uint32_t pk = uint32_t(p.packet);
    __amdgpu_buffer_rsrc_t dr[R];
#pragma unroll
    for (int i = 0; i < R; ++i) dr[i] = chunk_rsrc(uniform64(ptr[kMaxSrc + i]), p.chunk);
    vec acc[ROWS];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
        for (int l = 0; l < W; ++l) acc[i * W + l] = p.accumulate ? buf_ld<vec>(dr[i], off + l * pk, true) : vec(0);
    vec d[W], nx[W];
    {
        const __amdgpu_buffer_rsrc_t sr = chunk_rsrc(uniform64(ptr[0]), p.chunk);
#pragma unroll
        for (int x = 0; x < W; ++x) d[x] = buf_ld<vec>(sr, off + x * pk, true);
    }
    const uint32_t *mt = dsc + kBmDescHead + opaque_zero();
    for (uint32_t j = 0; j < k; ++j) {
        if (j + 1 < k) {
            const __amdgpu_buffer_rsrc_t sr = chunk_rsrc(uniform64(ptr[j + 1]), p.chunk);
#pragma unroll
            for (int x = 0; x < W; ++x) nx[x] = buf_ld<vec>(sr, off + x * pk, true);
        }
        uint32_t mw[MW];
#pragma unroll
        for (int q = 0; q < MW; ++q) mw[q] = uniform32(mt[j * MS + q]);
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const uint32_t mb = (mw[r / 4] >> (8 * (r % 4))) & 0xffu;
#pragma unroll
            for (int x = 0; x < W; ++x) {
                const uint32_t m = 0u - ((mb >> x) & 1u);
                acc[r] = and_xor(d[x], m, acc[r]);
            }
        }
#pragma unroll
        for (int x = 0; x < W; ++x) d[x] = nx[x];
    }
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
        for (int l = 0; l < W; ++l) buf_st(acc[i * W + l], dr[i], off + l * pk);
}

hipError_t launch_gather_tail(const GatherLaunch &L, bool bitmatrix, uint64_t off, hipStream_t stream);

inline GatherParams gather_params(const GatherLaunch &L, const Geometry &g) {
    GatherParams p;
    p.stab = L.stab;
    p.dtab = L.dtab;
    p.desc = static_cast<const uint32_t *>(L.desc);
    p.desc_dw = L.desc_dw;
    p.pat = L.pat;
    p.packet = L.w ? L.len : 0;
    p.chunk = uint32_t(L.w ? L.len * uint64_t(L.w) : L.len);
    p.sstride = L.sstride;
    p.dstride = L.dstride;
    p.s0 = 0;
    p.units = g.units;
    p.tiles = g.tiles;
    p.k = uint32_t(L.k);
    p.accumulate = L.accumulate ? 1u : 0u;
    p.groups = L.groups ? L.groups : 1u;
    p.group_maps = L.group_maps;
    return p;
}

template <int K, int R>
hipError_t run_gf8_gather(const GatherLaunch &L, hipStream_t stream) {
    uint32_t units = 0;
    for (uint32_t s0 = 0; s0 < L.n_stripes;) {
        const KernelPlan pl = plan_gf8_gather(L, s0);
        if (!pl.ok || pl.k != K || pl.rows != R) return hipErrorInvalidValue;
        units = pl.geo.units;
        if (units == 0) break;
        GatherParams p = gather_params(L, pl.geo);
        p.s0 = s0;
        const dim3 grid(uint32_t(pl.grid)), block(kThreads);
        if constexpr (R == kMaxRows) {
            if (p.groups > 1)
                hipLaunchKernelGGL((gf8_gather_kernel<K, R, true>), grid, block, 0, stream, p);
            else
                hipLaunchKernelGGL((gf8_gather_kernel<K, R, false>), grid, block, 0, stream, p);
        } else {
            hipLaunchKernelGGL((gf8_gather_kernel<K, R, false>), grid, block, 0, stream, p);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        s0 += pl.ns;
    }
    if (L.len % 16)  // the tail, one launch per row group
        for (uint32_t grp = 0; grp < std::max(1u, L.groups); ++grp) {
            GatherLaunch Lg = L;
            Lg.desc = static_cast<const uint8_t *>(L.desc) + size_t(grp) * L.group_maps * L.desc_dw * sizeof(uint32_t);
            Lg.groups = 1;
            hipError_t e = launch_gather_tail(Lg, false, uint64_t(L.len / 16) * 16, stream);
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}

template <int W, int R>
hipError_t run_bm_gather(const GatherLaunch &L, hipStream_t stream) {
    constexpr int UB = 4 * bm_vw<W>();
    for (uint32_t s0 = 0; s0 < L.n_stripes;) {
        const KernelPlan pl = plan_bm_gather(L, s0);
        if (!pl.ok || pl.rows != R || pl.vw * 4 != uint32_t(UB)) return hipErrorInvalidValue;
        if (pl.geo.units == 0) break;
        GatherParams p = gather_params(L, pl.geo);
        p.s0 = s0;
        hipLaunchKernelGGL((bm_gather_kernel<W, R>), dim3(uint32_t(pl.grid)), dim3(kThreads), 0, stream, p);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        s0 += pl.ns;
    }
    if (L.len % UB) return launch_gather_tail(L, true, uint64_t(L.len / UB) * UB, stream);
    return hipSuccess;
}

#define MEC_GG8_ONE(K, R) template hipError_t run_gf8_gather<K, R>(const GatherLaunch &, hipStream_t);
#define MEC_GG8_EXT(K, R) extern template hipError_t run_gf8_gather<K, R>(const GatherLaunch &, hipStream_t);
#define MEC_GG8_INSTANTIATE_LO(R) MEC_FOR_K_LO(MEC_GG8_ONE, R)
#define MEC_GG8_INSTANTIATE_HI(R) MEC_FOR_K_HI(MEC_GG8_ONE, R)
#define MEC_GBM_ONE(W, R) template hipError_t run_bm_gather<W, R>(const GatherLaunch &, hipStream_t);
#define MEC_GBM_EXT(W, R) extern template hipError_t run_bm_gather<W, R>(const GatherLaunch &, hipStream_t);
#define MEC_GBM_INSTANTIATE_W(W) MEC_FOR_R8(MEC_GBM_ONE, W)

}  // namespace detail
}  // namespace mec
