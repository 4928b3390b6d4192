// stream_common.hpp — device helpers shared by libmec's streaming kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "kernels.hpp"
#include "launch_plan.hpp"

namespace mec {
namespace detail {

// Bounds checks on runtime-indexed kernel-argument arrays, descriptor
// selectors and pointer-row entries.  Compiled in only by the bounds build
// (make -C memec_amd bounds: -DMEC_DEVICE_BOUNDS, memec_amd/bounds/libmec.so,
// loaded with MEMEC_LIBMEC), where a violated index aborts the kernel with
// a message before it forms an address; the release build has none.
#ifdef MEC_DEVICE_BOUNDS
#define MEC_DASSERT(c)                                                                     \
    do {                                                                                   \
        if (!(c)) {                                                                        \
            printf("libmec bounds check failed: %s:%d: %s\n", __FILE__, __LINE__, #c);    \
            __builtin_trap();                                                              \
        }                                                                                  \
    } while (0)
#else
#define MEC_DASSERT(c) ((void)0)
#endif

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Streamed-once data: non-temporal loads/stores keep the stripe bytes from
// displacing anything in L2 / the Infinity Cache (measured +2-4 % on the
// RS(10,4) stream, tools/microbench.hip).
template <typename V>
__device__ __forceinline__ V ld_nt(const uint8_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const V *>(p));
}
template <typename V>
__device__ __forceinline__ void st_nt(uint8_t *p, V v) {
    __builtin_nontemporal_store(v, reinterpret_cast<V *>(p));
}

// One chunk as a buffer resource: a NULL chunk gets zero records, so its
// loads return 0 and its stores are dropped by the range check — no
// branches around the memory operations.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t chunk_rsrc(uint64_t a, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(a), 0, a ? int(bytes) : 0, 0x00020000);
}
constexpr int kAuxNT = 2;  // non-temporal (streamed once)
template <typename V>
__device__ __forceinline__ V buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t off, bool nt);
template <>
__device__ __forceinline__ u32x4 buf_ld<u32x4>(__amdgpu_buffer_rsrc_t r, uint32_t off, bool nt) {
    return nt ? __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxNT) : __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
template <>
__device__ __forceinline__ u32x2 buf_ld<u32x2>(__amdgpu_buffer_rsrc_t r, uint32_t off, bool nt) {
    return nt ? __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kAuxNT) : __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
}
// Stores: non-temporal + sc1 (the line leaves the XCD's L2 instead of
// staying in it): the in-place RS(10,4)-shaped stream +0.7-1.4 points at
// 12-20 waves per CU, split layouts unchanged (tools/policy_probe.hip,
// profiles/r02/policy/policy_probe_inplace.log).
constexpr int kAuxStore = 2 | 16;
__device__ __forceinline__ void buf_st(u32x4 v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxStore);
}
__device__ __forceinline__ void buf_st(u32x2 v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, kAuxStore);
}

// An SGPR zero the compiler cannot see through: offsetting the LDS table
// base by it stops LLVM from hoisting every table read to the top of the
// kernel (which cost 200+ VGPRs and 2x time in tools/microbench.hip).
__device__ __forceinline__ int opaque_zero() {
    int z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    return z;
}

// Block order.  Blocks are handed out in blockIdx order, so with the
// identity map every resident block works inside one narrow address window
// (a few consecutive stripes).  When the outputs are interleaved with the
// inputs in that window (in-place decode of a [stripe][k+m][chunk] buffer,
// parity written next to its data) the stream loses 6-8 % of HBM
// throughput; splitting the grid into `win` windows far apart, taken
// round-robin by consecutive block ids, recovers it (tools/layout_bench.hip,
// tools/win_ab.py, profiles/r01/layout: RS(10,4) 1 MiB in-place decode
// 73.4 % -> 79.5 % of 8 TB/s with 2 windows).  Separate input and output
// buffers are already two windows: there a second split costs 4 % (RS(10,4)
// encode 78.9 % -> 74.6 %), so they keep the identity order (win = 1).
__device__ __forceinline__ uint32_t block_order(uint32_t win) {
    const uint32_t b = blockIdx.x;
    if (win <= 1) return b;
    const uint32_t per = gridDim.x / win;
    return b < per * win ? (b % win) * per + b / win : b;
}

// Stripe groups.  With the identity map the resident blocks of a launch
// cover a few thousand consecutive tiles, i.e. only the first one to three
// stripes of 1 MiB chunks and less than one stripe of larger ones, every
// wave reading its k chunks at the same offset, chunk-size bytes apart;
// RS(10,4) encode runs 84 % of 8 TB/s at 64 KiB chunks, 81 % at 1 MiB, 72 %
// at 4 MiB and 57 % at 16 MiB for the same bytes (tools/stride_probe.py,
// tools/sgroup_ab.py).  A group map
// walks `group` stripes at a time: consecutive blocks take 8 consecutive
// tiles (so block id mod 8, the XCD, still fixes the tile mod 8, as in the
// identity map), then the next stripe of the group, and only after every
// stripe of the group the next 8 tiles.  group = 0 keeps the identity map;
// tiles % run == 0 and run % 8 == 0 whenever group != 0 (host side,
// stripe_group; `run` consecutive tiles per stripe visit, default 8).
// skew (identity map only; MEC_TILE_SKEW, an experiment on the in-place
// decodes): stripe s starts its tiles at s * skew mod
// tiles, so neighbouring stripes' resident blocks sit at different column
// offsets (a rotation per stripe: still a bijection).
__device__ __forceinline__ void stripe_tile(uint32_t bid, uint32_t tiles, uint32_t ns, uint32_t group, uint32_t run,
                                            uint32_t skew, uint32_t &stripe, uint32_t &tile) {
    if (group == 0) {
        stripe = bid / tiles;
        tile = bid - stripe * tiles;
        if (skew) tile = uint32_t((uint64_t(tile) + uint64_t(stripe) * skew) % tiles);
        return;
    }
    const uint32_t per = group * tiles;
    const uint32_t g = bid / per, r = bid - g * per;
    const uint32_t gl = ns - g * group < group ? ns - g * group : group;
    const uint32_t q = r / run, sl = q % gl;
    stripe = g * group + sl;
    tile = (q / gl) * run + (r - q * run);
}
// Template instantiation lists: X(K, R) for every source count a launch can
// have (k + m <= 32 with m >= 1, so K <= kMaxK), split in two halves so the
// units build in parallel; kernels.hip declares the same lists `extern` so
// its dispatch tables do not instantiate a second copy.
#define MEC_FOR_K_LO(X, R) \
    X(1, R) X(2, R) X(3, R) X(4, R) X(5, R) X(6, R) X(7, R) X(8, R) X(9, R) X(10, R) X(11, R) X(12, R) X(13, R) X(14, R) X(15, R) X(16, R)
#define MEC_FOR_K_HI(X, R) \
    X(17, R) X(18, R) X(19, R) X(20, R) X(21, R) X(22, R) X(23, R) X(24, R) X(25, R) X(26, R) X(27, R) X(28, R) X(29, R) X(30, R) X(31, R)
#define MEC_FOR_K(X, R) MEC_FOR_K_LO(X, R) MEC_FOR_K_HI(X, R)

// Uniform 64-bit / 32-bit values (read back from LDS or memory) into SGPRs.
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(v));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(v >> 32));
    return uint64_t(hi) << 32 | lo;
}
__device__ __forceinline__ uint32_t uniform32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Pointer rows of gathered launches.  A wave fetches its stripe's row in ONE
// vector load — lane j < ns source j's entry, lane 32 + i output i's, the
// rest 0 — and each use reads its entry back from that lane (v_readlane,
// lane index uniform).  An entry read as a scalar load at its use made the
// compiler wait on each in turn before that chunk's loads could issue: ten
// dependent round trips per block before RS(10,4)'s last source load left,
// sixteen for the bit-sliced RS(16,8) (one-map RS(16,8) batches 71.7 ->
// 78-80 % with the row in one load, profiles/r05/vrow/vrow_ab_box13.jsonl).
// so / do_: the entry numbers (Gf8Params::src_off / dst_off in gather mode).
template <int NS, int ND>
__device__ __forceinline__ uint64_t row_fetch(const uint64_t *srow, const int64_t (&so)[NS], uint32_t ns,
                                              const uint64_t *drow, const int64_t (&do_)[ND], uint32_t nd) {
    // each lane picks its entry number from the (scalar) kernel arguments
    // by compare-and-select: no per-lane read of the argument block
    const uint32_t l = threadIdx.x & 63u;
    const uint64_t *e = nullptr;
#pragma unroll
    for (int j = 0; j < NS && j < 32; ++j)
        if (uint32_t(j) < ns && l == uint32_t(j)) e = srow + so[j];
#pragma unroll
    for (int i = 0; i < ND && i < 32; ++i)
        if (uint32_t(i) < nd && l == 32u + i && do_[i] >= 0) e = drow + do_[i];
    return e ? *e : 0;
}
// A gathered lane past the launch's last unit must not leave before the
// row's v_readlanes (a lane that left no longer holds its entry): a wave
// wholly past it leaves (uniform), a partial wave's extra lanes redo the last
// unit — the same loads, and the same bytes stored to the same place in the
// same instruction as the unit's own lane, read-modify-write included.
// Returns false for a wave that leaves; u = the lane's unit.
template <int BT>
__device__ __forceinline__ bool gather_unit(uint32_t tile, uint32_t units, uint32_t &u) {
    const uint32_t u0 = tile * BT + (threadIdx.x & ~63u);
    if (u0 >= units) return false;
    u = min(u0 + (threadIdx.x & 63u), units - 1u);
    return true;
}
__device__ __forceinline__ uint64_t row_entry(uint64_t row, uint32_t lane) {
    const uint32_t lo = __builtin_amdgcn_readlane(int(uint32_t(row)), int(lane));
    const uint32_t hi = __builtin_amdgcn_readlane(int(uint32_t(row >> 32)), int(lane));
    return uint64_t(hi) << 32 | lo;
}

// ---------------------------------------------------------------------------
// partial (tail) units: < 16 bytes at the end of a region
// ---------------------------------------------------------------------------
__device__ inline u32x4 load_partial(const uint8_t *p, uint32_t n) {
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t i = 0; i < n; ++i) w[i >> 2] |= uint32_t(p[i]) << (8 * (i & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ inline void store_partial(uint8_t *p, u32x4 v, uint32_t n) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (uint32_t i = 0; i < n; ++i) p[i] = uint8_t(w[i >> 2] >> (8 * (i & 3)));
}

}  // namespace detail
}  // namespace mec
