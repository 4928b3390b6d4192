// gf8_kernel.hpp — GF(2^8) byte-wise matrix apply (Jerasure RS, ISA-L RS /
// Cauchy).  Instantiated per row count in gf8_r{1..4}.hip.
//
// Arithmetic: c*x is linear in the bits of x, so every byte is split into
// bit fields 0-2 | 3-5 | 6-7 and each field indexes a <= 8-entry table of
// c*(field << shift) with one v_perm_b32, four bytes per instruction:
// 3 v_perm + 2 v_bitop3 per (coefficient, dword).  Coefficient 1 is a plain
// XOR and coefficient 0 is skipped (uniform branches on kernel-argument
// masks).  Replaces the scalar multtable[s][c] byte loop
// (gf_w8.c:1047-1050) and ISA-L's PSHUFB nibble kernels
// (gf_vect_dot_prod_sse.asm:215-230).
//
// Memory: each lane owns one 16-byte column slice of one stripe: K
// non-temporal dwordx4 loads (one per source chunk, a wave reads 1 KiB
// contiguous per chunk), R non-temporal dwordx4 stores.  The permute tables
// live in LDS (R*K*32 bytes) and are read by broadcast right before use.
#pragma once

#include <vector>

#include "knobs.hpp"
#include "stream_common.hpp"

namespace mec {
namespace detail {

template <int K, int R>
struct Gf8Params {
    const uint8_t *src;
    uint8_t *dst;
    int64_t sss, dss;
    // gather mode (G): source j of stripe s is chunk pointer
    // stab[s * sstride + src_off[j]], output i is dtab[s * dstride + dst_off[i]]
    const uint64_t *stab, *dtab;
    uint32_t sstride, dstride, chunk, s0;
    uint32_t units, tiles, accumulate, win;
    uint32_t nstr, sgroup, srun, skew;  // stripes in this launch, stripe group and run, tile skew (stripe_tile)
    uint32_t xcd;                       // gathered: blocks b, b + 8, ... (one XCD) take one contiguous run (plan_gf8)
    int64_t src_off[K];
    int64_t dst_off[R];
    Gf8Coef coef[R][K];
};

// a ^ b ^ c ^ d in two gfx950 v_bitop3_b32 (truth table 0x96 = 3-input XOR;
// hipcc does not fuse XOR chains on its own).
__device__ __forceinline__ uint32_t xor4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const uint32_t t = uint32_t(__builtin_amdgcn_bitop3_b32(a, b, c, 0x96));
    return uint32_t(__builtin_amdgcn_bitop3_b32(t, d, 0u, 0x96));
}

__device__ __forceinline__ uint32_t gf8_mul(const Gf8Coef &c, uint32_t x) {
    return __builtin_amdgcn_perm(c.t1, c.t0, x & 0x07070707u) ^
           __builtin_amdgcn_perm(c.u1, c.u0, (x >> 3) & 0x07070707u) ^
           __builtin_amdgcn_perm(c.v, c.v, (x >> 6) & 0x03030303u);
}

// 3-input XOR of 16-byte vectors: one v_bitop3_b32 per dword.
__device__ __forceinline__ u32x4 xor3(const u32x4 &a, const u32x4 &b, const u32x4 &c) {
    return u32x4{uint32_t(__builtin_amdgcn_bitop3_b32(a.x, b.x, c.x, 0x96)),
                 uint32_t(__builtin_amdgcn_bitop3_b32(a.y, b.y, c.y, 0x96)),
                 uint32_t(__builtin_amdgcn_bitop3_b32(a.z, b.z, c.z, 0x96)),
                 uint32_t(__builtin_amdgcn_bitop3_b32(a.w, b.w, c.w, 0x96))};
}

// Matrix structure a launch is specialised for (chosen on the host from the
// coefficients, so the kernel has no data-dependent branches; constants in
// launch_plan.hpp):
//   kGf8Dense — every coefficient through its permute tables (a 0 / 1
//               coefficient's tables give 0 / x, so any matrix is exact);
//   kGf8Vand  — row 0 and column 0 all ones (Jerasure's Vandermonde
//               distribution rows, reed_sol.c:269-297, and ISA-L's
//               gf_gen_rs_matrix parity rows, ec_base.c:62-79): those
//               entries are plain XORs, the rest through tables.
//   kGf8Xor   — measurement twin (mec_set_probe): every product replaced by
//               a plain XOR, same loads, stores and launch shape; the
//               outputs are not codes.
//   kGf8Col0  — column 0 all ones only: the row groups after the first of a
//               Vandermonde matrix with more than one group (gf8_mg_kernel).

// acc[i] ^= sum_j coef(i, j) * d[j] for one 16-byte unit.  TB = the LDS
// permute tables (8 dwords per coefficient b = i*K + j: t0 t1 u0 u1 v).
// Every product contributes 1 (unit) or 3 (v_perm) terms to its row; the
// terms are folded into the row accumulator two at a time with 3-input
// XORs, carrying an odd one over to the next source (the `has` flags are
// compile-time constants once the loops are unrolled), so a table product
// costs 3 v_perm + 1.5 v_bitop3 per dword and a unit one 0.5 v_bitop3.
template <int K, int R, int S>
__device__ __forceinline__ void gf8_apply(const u32x4 (&d)[K], u32x4 (&acc)[R], const uint32_t *tb) {
    if constexpr (S == kGf8Xor) {
        u32x4 x = d[0];
#pragma unroll
        for (int j = 1; j + 1 < K; j += 2) x = xor3(x, d[j], d[j + 1]);
        if constexpr (K % 2 == 0) x ^= d[K - 1];
#pragma unroll
        for (int i = 0; i < R; ++i) acc[i] ^= x;
        return;
    }
    u32x4 pend[R];
    bool has[R];
#pragma unroll
    for (int i = 0; i < R; ++i) has[i] = false;
    auto put = [&](int i, const u32x4 &t) {
        if (has[i]) {
            acc[i] = xor3(acc[i], pend[i], t);
            has[i] = false;
        } else {
            pend[i] = t;
            has[i] = true;
        }
    };
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const u32x4 x = d[j];
        if ((S == kGf8Vand || S == kGf8Col0) && j == 0) {
#pragma unroll
            for (int i = 0; i < R; ++i) put(i, x);
            continue;
        }
        const u32x4 s0 = x & 0x07070707u;
        const u32x4 s1 = (x >> 3) & 0x07070707u;
        const u32x4 s2 = (x >> 6) & 0x03030303u;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            if (S == kGf8Vand && i == 0) {
                put(0, x);
                continue;
            }
            const int b = i * K + j;
            const u32x4 t = *reinterpret_cast<const u32x4 *>(tb + b * 8);
            const uint32_t v = tb[b * 8 + 4];
            put(i, u32x4{__builtin_amdgcn_perm(t.y, t.x, s0.x), __builtin_amdgcn_perm(t.y, t.x, s0.y),
                         __builtin_amdgcn_perm(t.y, t.x, s0.z), __builtin_amdgcn_perm(t.y, t.x, s0.w)});
            put(i, u32x4{__builtin_amdgcn_perm(t.w, t.z, s1.x), __builtin_amdgcn_perm(t.w, t.z, s1.y),
                         __builtin_amdgcn_perm(t.w, t.z, s1.z), __builtin_amdgcn_perm(t.w, t.z, s1.w)});
            put(i, u32x4{__builtin_amdgcn_perm(v, v, s2.x), __builtin_amdgcn_perm(v, v, s2.y),
                         __builtin_amdgcn_perm(v, v, s2.z), __builtin_amdgcn_perm(v, v, s2.w)});
        }
    }
#pragma unroll
    for (int i = 0; i < R; ++i)
        if (has[i]) acc[i] ^= pend[i];
}

// G = gather: chunk addresses come from per-stripe pointer rows (the
// caller's Chunk* arrays) instead of base + stripe * stride + offset; the
// map stays in kernel arguments, so a block's only extra latency is one
// batch of scalar loads of its pointers.
//
// U = 2 (gathered one-wave blocks only, MEC_GU): a lane codes units u and
// u + 64 of its stripe's 2 KiB tile, the wave's loads 1 KiB contiguous per
// chunk each, one pointer-row fetch per 2 KiB; the planner uses it only
// where every tile is whole (units % 128 == 0), so no lane is past the
// chunk and none redoes another's unit.
template <int K, int R, bool G, int S, int BT, int U = 1>
__global__ __launch_bounds__(BT) void gf8_kernel(const Gf8Params<K, R> p) {
    static_assert(U == 1 || (G && BT == 64 && U == 2), "two units per lane: gathered one-wave blocks");
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
    uint32_t bid = block_order(p.win);
    if (G && p.xcd) {  // blocks are dealt round-robin over the 8 XCDs: each XCD takes one run, so a stripe's tiles share an L2
        const uint32_t per = gridDim.x >> 3;
        if (bid < per * 8u) bid = (bid & 7u) * per + (bid >> 3);
    }
    uint32_t stripe, tile;
    stripe_tile(bid, p.tiles, p.nstr, p.sgroup, p.srun, p.skew, stripe, tile);
    uint32_t u = tile * BT * U + threadIdx.x;
    if constexpr (U == 2) {
        if (u >= p.units) return;  // whole tiles: the wave is in or out
    } else if constexpr (G) {
        if (!gather_unit<BT>(tile, p.units, u)) return;
    } else if (u >= p.units) {
        return;
    }
    // Every chunk is a buffer resource (SGPR base, 32-bit lane offsets) in
    // both modes: strided chunk bases are uniform per block too, and the
    // same non-temporal stream runs 2-3 points faster through buffer
    // instructions than through 64-bit flat addresses at the product's
    // wave caps (tools/policy_probe.hip, profiles/r02/policy/).
    const uint32_t off = u * 16;
    // chunk addresses (uniform): source j / output i of this stripe
    const uint64_t gs = p.s0 + stripe;
    static_assert(K <= 32 && R <= 32, "pointer row lanes (row_fetch)");
    const uint64_t row = G ? row_fetch(p.stab + gs * p.sstride, p.src_off, K, p.dtab + gs * p.dstride, p.dst_off, R) : 0;
    auto src_at = [&](int j) -> uint64_t {
        if constexpr (G) return row_entry(row, uint32_t(j));
        else return uint64_t(uintptr_t(p.src + int64_t(stripe) * p.sss + p.src_off[j]));
    };
    auto dst_at = [&](int i) -> uint64_t {
        if constexpr (G) return row_entry(row, 32u + uint32_t(i));
        else return uint64_t(uintptr_t(p.dst + int64_t(stripe) * p.dss + p.dst_off[i]));
    };
    u32x4 d[K];
    [[maybe_unused]] u32x4 d2[U == 2 ? K : 1];
#pragma unroll
    for (int j = 0; j < K; ++j) d[j] = buf_ld<u32x4>(chunk_rsrc(src_at(j), p.chunk), off, true);
    if constexpr (U == 2) {
#pragma unroll
        for (int j = 0; j < K; ++j) d2[j] = buf_ld<u32x4>(chunk_rsrc(src_at(j), p.chunk), off + 1024u, true);
    }
    __amdgpu_buffer_rsrc_t dr[R];
#pragma unroll
    for (int i = 0; i < R; ++i) dr[i] = chunk_rsrc(dst_at(i), p.chunk);
    u32x4 acc[R];
    // read-modify-write of the outputs (delta updates) is streamed too
    // (non-temporal: RS(10,4) update 70.9 -> 73.9 %)
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = p.accumulate ? buf_ld<u32x4>(dr[i], off, true) : u32x4{0, 0, 0, 0};
    gf8_apply<K, R, S>(d, acc, tab + opaque_zero());
#pragma unroll
    for (int i = 0; i < R; ++i) buf_st(acc[i], dr[i], off);
    if constexpr (U == 2) {
        u32x4 acc2[R];
#pragma unroll
        for (int i = 0; i < R; ++i) acc2[i] = p.accumulate ? buf_ld<u32x4>(dr[i], off + 1024u, true) : u32x4{0, 0, 0, 0};
        gf8_apply<K, R, S>(d2, acc2, tab + opaque_zero());
#pragma unroll
        for (int i = 0; i < R; ++i) buf_st(acc2[i], dr[i], off + 1024u);
    }
}

// Write-batched in-place decode (A/B, MEC_WBATCH=T):
// a 256-thread block codes T consecutive 4 KiB tiles of one stripe, keeping
// every tile's outputs in registers, and stores them only after the last
// tile's sources are in: each output chunk then receives one T x 4 KiB
// burst per block instead of T separate 4 KiB ones between the survivors'
// reads.  configs[2]'s in-place decode loses 3-5 points to the split layout
// inside the DRAM channels (§5.3); this changes the write pattern, not the
// read one.  Instantiated for the shape it tests (K = 10, R = 4, dense).
template <int K, int R, int S, int T>
__global__ __launch_bounds__(kThreads) void gf8_wb_kernel(const Gf8Params<K, R> p) {
    __shared__ uint32_t tab[R * K * 8];
    for (int t = threadIdx.x; t < R * K; t += kThreads) {
        const Gf8Coef c = p.coef[t / K][t % K];
        tab[t * 8 + 0] = c.t0;
        tab[t * 8 + 1] = c.t1;
        tab[t * 8 + 2] = c.u0;
        tab[t * 8 + 3] = c.u1;
        tab[t * 8 + 4] = c.v;
    }
    __syncthreads();
    const uint32_t bid = block_order(p.win);
    uint32_t stripe, st;
    stripe_tile(bid, p.tiles, p.nstr, p.sgroup, p.srun, p.skew, stripe, st);  // p.tiles: groups of T tiles
    const uint8_t *sb = p.src + int64_t(stripe) * p.sss;
    uint8_t *db = p.dst + int64_t(stripe) * p.dss;
    __amdgpu_buffer_rsrc_t dr[R];
#pragma unroll
    for (int i = 0; i < R; ++i) dr[i] = chunk_rsrc(uint64_t(uintptr_t(db + p.dst_off[i])), p.chunk);
    u32x4 acc[T][R];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const uint32_t off = ((st * T + t) * kThreads + threadIdx.x) * 16;  // host: units % (T x 256) == 0
        u32x4 d[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
            d[j] = buf_ld<u32x4>(chunk_rsrc(uint64_t(uintptr_t(sb + p.src_off[j])), p.chunk), off, true);
#pragma unroll
        for (int i = 0; i < R; ++i) acc[t][i] = u32x4{0, 0, 0, 0};
        gf8_apply<K, R, S>(d, acc[t], tab + opaque_zero());
    }
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
        for (int t = 0; t < T; ++t) buf_st(acc[t][i], dr[i], ((st * T + t) * kThreads + threadIdx.x) * 16);
}
// K = 10, R = 4, dense, T = 2 / 4 (gf8_r4lo.hip); false elsewhere
template <int K, int R>
bool launch_gf8_wb(const KernelPlan &pl, Gf8Params<K, R> p, int T, hipStream_t stream);

// More than 4 outputs (m > 4: RS(16,8), ISA-L RS(12,8), decodes of > 4
// erasures) in ONE pass over the sources: a lane loads its K source units
// once and codes `groups` row groups of R outputs from the same registers,
// one group at a time (the register footprint of an R-row launch), so the
// sources are read once however many outputs there are — the 4-row launches
// before re-read them ceil(m / 4) times (RS(16,8): 1.67x the algorithmic
// bytes).  The groups' permute tables (groups x R x K x 8 dwords, row r of
// group g at (g * R + r) * K * 8) come from a device copy (gf8_mg_tables)
// into dynamic LDS; rows past the last output are padding (dst_off < 0: no
// store).  S = kGf8Vand: group 0 has row 0 and column 0 all ones, the others
// column 0 (Jerasure / ISA-L RS parity rows); kGf8Dense otherwise.  One-wave
// blocks, strided layouts only (pointer batches split rows in groups of 4).
// G = gather (pointer batches with one map for every stripe): source j /
// output r of stripe s are the chunk pointers stab[s * sstride + src_off[j]]
// / dtab[s * dstride + dst_off[r]] (as gf8_kernel's gather mode).
template <int K>
struct Gf8MgParams {
    const uint8_t *src;
    uint8_t *dst;
    int64_t sss, dss;
    const uint64_t *stab, *dtab;
    uint64_t s0;
    uint32_t sstride, dstride;
    const uint32_t *tabs;  // device: groups x R x K x 8 dwords
    uint32_t chunk, units, tiles, accumulate, win, nstr, sgroup, srun, groups, skew;
    int64_t src_off[K];
    int64_t dst_off[kMaxSrc];  // groups x R rows; < 0 = padding
};

template <int K, int R, int S, bool G>
__global__ __launch_bounds__(kWaveBlock) void gf8_mg_kernel(const Gf8MgParams<K> p) {
    extern __shared__ uint32_t mtab[];
    const uint32_t ntab = p.groups * R * K * 8;
    MEC_DASSERT(p.groups * R <= uint32_t(kMaxSrc));
    for (uint32_t t = threadIdx.x; t < ntab; t += kWaveBlock) mtab[t] = p.tabs[t];
    __syncthreads();
    const uint32_t bid = block_order(p.win);
    uint32_t stripe, tile;
    stripe_tile(bid, p.tiles, p.nstr, p.sgroup, p.srun, p.skew, stripe, tile);
    uint32_t u = tile * kWaveBlock + threadIdx.x;
    if constexpr (G) {
        if (!gather_unit<kWaveBlock>(tile, p.units, u)) return;
    } else if (u >= p.units) {
        return;
    }
    const uint32_t off = u * 16;
    const uint64_t gs = p.s0 + stripe;
    static_assert(K <= 32, "pointer row lanes (row_fetch)");
    const uint64_t row =
        G ? row_fetch(p.stab + gs * p.sstride, p.src_off, K, p.dtab + gs * p.dstride, p.dst_off, p.groups * R) : 0;
    u32x4 d[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        MEC_DASSERT(!G || (p.src_off[j] >= 0 && p.src_off[j] < int64_t(p.sstride)));
        const uint64_t a = G ? row_entry(row, uint32_t(j))
                             : uint64_t(uintptr_t(p.src + int64_t(stripe) * p.sss + p.src_off[j]));
        d[j] = buf_ld<u32x4>(chunk_rsrc(a, p.chunk), off, true);
    }
    uint8_t *db = G ? nullptr : p.dst + int64_t(stripe) * p.dss;
    auto group = [&](uint32_t g, auto apply) {
        __amdgpu_buffer_rsrc_t dr[R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            MEC_DASSERT(g * R + i < uint32_t(kMaxSrc));
            MEC_DASSERT(!G || p.dst_off[g * R + i] < int64_t(p.dstride));
            const int64_t o = p.dst_off[g * R + i];
            const uint64_t a = o < 0 ? 0 : G ? row_entry(row, 32u + g * R + uint32_t(i)) : uint64_t(uintptr_t(db + o));
            dr[i] = chunk_rsrc(a, p.chunk);
        }
        u32x4 acc[R];
#pragma unroll
        for (int i = 0; i < R; ++i) acc[i] = p.accumulate ? buf_ld<u32x4>(dr[i], off, true) : u32x4{0, 0, 0, 0};
        apply(acc, mtab + g * (R * K * 8) + opaque_zero());
#pragma unroll
        for (int i = 0; i < R; ++i) buf_st(acc[i], dr[i], off);
    };
    // group 0 (row 0 all ones for kGf8Vand), then the rest; the sources
    // "change" before every group (an empty asm), so the compiler cannot
    // hoist their bit fields out of the loop (3 x K x 4 more live VGPRs:
    // K = 17 ran at 256 VGPRs, occupancy 1)
    group(0, [&](u32x4 (&acc)[R], const uint32_t *tb) { gf8_apply<K, R, S>(d, acc, tb); });
    for (uint32_t g = 1; g < p.groups; ++g) {  // uniform
#pragma unroll
        for (int j = 0; j < K; ++j) asm volatile("" : "+v"(d[j]));
        group(g, [&](u32x4 (&acc)[R], const uint32_t *tb) {
            gf8_apply<K, R, S == kGf8Vand ? kGf8Col0 : kGf8Dense>(d, acc, tb);
        });
    }
}

template <int K, int R>
hipError_t run_gf8_mg(const Gf8MgLaunch &L, hipStream_t stream);

// The < 16-byte remainder of each region (chunk sizes that are not a
// multiple of 16): one thread per stripe, any K and row count.
struct Gf8TailParams {
    const uint8_t *src;
    uint8_t *dst;
    int64_t sss, dss;
    const uint64_t *stab, *dtab;
    uint32_t sstride, dstride;
    uint64_t off;
    uint32_t n, k, rows, n_stripes, accumulate, pad;
    int64_t src_off[kMaxSrc];
    int64_t dst_off[kMaxRows];
    Gf8Coef coef[kMaxRows][kMaxSrc];
};

hipError_t launch_gf8_tail(const Gf8Launch &L, uint64_t off, hipStream_t stream);

// Launch one plan (launch_plan.cpp plan_gf8) with its kernel instantiation.
template <int K, int R, bool G, int S>
void launch_gf8_plan(const KernelPlan &pl, const Gf8Params<K, R> &p, hipStream_t stream) {
    const dim3 grid(uint32_t(pl.grid)), block(pl.bt);
    if constexpr (G) {
        if (pl.gu == 2 && pl.bt == kWaveBlock) {
            hipLaunchKernelGGL((gf8_kernel<K, R, G, S, kWaveBlock, 2>), grid, block, pl.lds_dynamic, stream, p);
            return;
        }
    }
    if (pl.bt == kWaveBlock)
        hipLaunchKernelGGL((gf8_kernel<K, R, G, S, kWaveBlock>), grid, block, pl.lds_dynamic, stream, p);
    else
        hipLaunchKernelGGL((gf8_kernel<K, R, G, S, kThreads>), grid, block, pl.lds_dynamic, stream, p);
}

template <int K, int R>
hipError_t run_gf8(const Gf8Launch &L, hipStream_t stream) {
    Gf8Params<K, R> p;
    p.sss = L.src_stripe_stride;
    p.dss = L.dst_stripe_stride;
    p.stab = L.stab;
    p.dtab = L.dtab;
    p.sstride = L.sstride;
    p.dstride = L.dstride;
    p.chunk = uint32_t(L.len);
    p.accumulate = L.accumulate ? 1u : 0u;
    for (int j = 0; j < K; ++j) p.src_off[j] = L.src_off[j];
    for (int i = 0; i < R; ++i) p.dst_off[i] = L.dst_off[i];
    for (int i = 0; i < R; ++i)
        for (int j = 0; j < K; ++j) p.coef[i][j] = L.coef[i][j];
    uint32_t units = 0;
    for (uint32_t s0 = 0; s0 < L.n_stripes;) {
        const KernelPlan pl = plan_gf8(L, s0);
        if (!pl.ok || pl.k != K || pl.rows != R) return hipErrorInvalidValue;
        units = pl.geo.units;
        if (units == 0) break;
        p.units = pl.geo.units;
        p.tiles = pl.geo.tiles;
        p.s0 = s0;
        p.win = pl.win;
        p.nstr = L.stab ? 0 : pl.ns;
        p.sgroup = pl.sgroup;
        p.srun = pl.srun;
        p.skew = pl.skew;
        p.xcd = pl.xcd;
        p.src = L.stab ? nullptr : L.src + int64_t(s0) * L.src_stripe_stride;
        p.dst = L.stab ? nullptr : L.dst + int64_t(s0) * L.dst_stripe_stride;
        const int64_t wb = knob(kKnobWbatch);
        if (wb > 0 && !L.stab && !L.accumulate && pl.structure == kGf8Dense && pl.win > 1 && pl.bt == kThreads &&
            pl.sgroup == 0 && pl.skew == 0 && pl.geo.units % (uint32_t(wb) * kThreads) == 0 &&
            launch_gf8_wb<K, R>(pl, p, int(wb), stream)) {
            // the write-batched A/B form took the launch
        } else if (L.stab) {
            if (pl.structure == kGf8Vand) launch_gf8_plan<K, R, true, kGf8Vand>(pl, p, stream);
            else launch_gf8_plan<K, R, true, kGf8Dense>(pl, p, stream);
        } else if (pl.structure == kGf8Xor) {
            launch_gf8_plan<K, R, false, kGf8Xor>(pl, p, stream);
        } else if (pl.structure == kGf8Vand) {
            launch_gf8_plan<K, R, false, kGf8Vand>(pl, p, stream);
        } else {
            launch_gf8_plan<K, R, false, kGf8Dense>(pl, p, stream);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        s0 += pl.ns;
    }
    if (L.len % 16) return launch_gf8_tail(L, uint64_t(L.len / 16) * 16, stream);
    return hipSuccess;
}

template <int K, int R>
hipError_t run_gf8_mg(const Gf8MgLaunch &L, hipStream_t stream) {
    Gf8MgParams<K> p;
    p.sss = L.src_stripe_stride;
    p.dss = L.dst_stripe_stride;
    p.tabs = L.tabs;
    p.stab = L.stab;
    p.dtab = L.dtab;
    p.sstride = L.sstride;
    p.dstride = L.dstride;
    p.chunk = uint32_t(L.len);
    p.accumulate = L.accumulate ? 1u : 0u;
    p.skew = 0;
    for (int j = 0; j < K; ++j) p.src_off[j] = L.src_off[j];
    for (uint32_t s0 = 0; s0 < L.n_stripes;) {
        const KernelPlan pl = plan_gf8_mg(L, s0);
        // the plan bounds groups x R by the kernel's kMaxSrc output slots
        if (!pl.ok || pl.k != K || pl.rows != R || pl.groups * uint32_t(R) > uint32_t(kMaxSrc))
            return hipErrorInvalidValue;
        if (pl.geo.units == 0) break;
        p.groups = pl.groups;
        for (int r = 0; r < kMaxSrc; ++r) p.dst_off[r] = r < L.rows ? L.dst_off[r] : -1;
        p.units = pl.geo.units;
        p.tiles = pl.geo.tiles;
        p.s0 = s0;
        p.win = pl.win;
        p.nstr = L.stab ? 0 : pl.ns;
        p.sgroup = pl.sgroup;
        p.srun = pl.srun;
        p.skew = pl.skew;
        // pointer rows: no layout to window or group over
        p.src = L.stab ? nullptr : L.src + int64_t(s0) * L.src_stripe_stride;
        p.dst = L.stab ? nullptr : L.dst + int64_t(s0) * L.dst_stripe_stride;
        const dim3 grid(uint32_t(pl.grid)), block(kWaveBlock);
        const uint32_t lds = pl.lds_dynamic;
        if (L.stab) {
            if (L.vand)
                hipLaunchKernelGGL((gf8_mg_kernel<K, R, kGf8Vand, true>), grid, block, lds, stream, p);
            else
                hipLaunchKernelGGL((gf8_mg_kernel<K, R, kGf8Dense, true>), grid, block, lds, stream, p);
        } else if (L.vand) {
            hipLaunchKernelGGL((gf8_mg_kernel<K, R, kGf8Vand, false>), grid, block, lds, stream, p);
        } else {
            hipLaunchKernelGGL((gf8_mg_kernel<K, R, kGf8Dense, false>), grid, block, lds, stream, p);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        s0 += pl.ns;
    }
    return hipSuccess;
}

// the write-batched A/B form exists for (10, 4) only (gf8_r4lo.hip)
template <int K, int R>
bool launch_gf8_wb(const KernelPlan &, Gf8Params<K, R>, int, hipStream_t) {
    return false;
}
template <>
bool launch_gf8_wb<10, 4>(const KernelPlan &pl, Gf8Params<10, 4> p, int T, hipStream_t stream);

#define MEC_GF8_ONE(K, R) template hipError_t run_gf8<K, R>(const Gf8Launch &, hipStream_t);
#define MEC_GF8_EXT(K, R) extern template hipError_t run_gf8<K, R>(const Gf8Launch &, hipStream_t);
#define MEC_GF8_INSTANTIATE_LO(R) MEC_FOR_K_LO(MEC_GF8_ONE, R)
#define MEC_GF8_INSTANTIATE_HI(R) MEC_FOR_K_HI(MEC_GF8_ONE, R)
#define MEC_GFM_ONE(K, R) template hipError_t run_gf8_mg<K, R>(const Gf8MgLaunch &, hipStream_t);
#define MEC_GFM_EXT(K, R) extern template hipError_t run_gf8_mg<K, R>(const Gf8MgLaunch &, hipStream_t);
// the 8-row group instantiations, K = kMg8MinK..kMg8MaxK
#define MEC_FOR_K8(X) \
    X(12, 8) X(13, 8) X(14, 8) X(15, 8) X(16, 8) X(17, 8) X(18, 8) X(19, 8) X(20, 8)
static_assert(kMg8MinK == 12 && kMg8MaxK == 20, "MEC_FOR_K8 lists K = 12..20");

}  // namespace detail
}  // namespace mec
