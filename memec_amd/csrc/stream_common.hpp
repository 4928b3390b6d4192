// stream_common.hpp — device helpers shared by libmec's streaming kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "kernels.hpp"

namespace mec {
namespace detail {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kThreads = 256;

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
__device__ __forceinline__ void stripe_tile(uint32_t bid, uint32_t tiles, uint32_t ns, uint32_t group, uint32_t run,
                                            uint32_t &stripe, uint32_t &tile) {
    if (group == 0) {
        stripe = bid / tiles;
        tile = bid - stripe * tiles;
        return;
    }
    const uint32_t per = group * tiles;
    const uint32_t g = bid / per, r = bid - g * per;
    const uint32_t gl = ns - g * group < group ? ns - g * group : group;
    const uint32_t q = r / run, sl = q % gl;
    stripe = g * group + sl;
    tile = (q / gl) * run + (r - q * run);
}
// Host: stripes per group for a strided launch of `tiles` blocks per stripe
// (0 = identity) and the run length.  MEC_SGROUP=<n>[:<run>] overrides
// (experiments flip it).  (Round 3's experiment-only maps — every eighth
// tile per XCD, a stripe permutation — measured worse and were removed from
// the product kernels)
uint32_t stripe_group(uint64_t chunk, uint32_t tiles, uint32_t n_stripes, bool in_place, bool bitmatrix,
                      uint32_t &run);

// Host: windows for a strided launch — 2 when the output region lies inside
// the input region's stripe span (one allocation, interleaved), else 1.
// MEC_WINDOWS=<n> overrides (layout experiments).
uint32_t launch_windows(const void *src, int64_t src_span, const void *dst, int64_t dst_span);
// Host: windows of a strided bitmatrix launch — launch_windows, except that
// in-place launches of tiny stripes (chunks <= 1 KiB; <= 2 KiB with <= 2
// outputs and k >= 8) run as split layouts do (1 window, which also picks
// one-wave blocks and the split wave caps; kernels.hip).
uint32_t bm_windows(const void *src, int64_t src_span, const void *dst, int64_t dst_span, uint64_t chunk, int rows,
                    int k);

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

// Launch geometry of the streaming kernels: one full unit per thread
// (measured faster than looping 2-16 units per thread), `tiles` blocks of
// kThreads per stripe, grid split so grid * block stays < 2^31 work-items.
struct Geometry {
    uint32_t units, tiles, max_stripes_per_launch;
};

inline Geometry geometry(uint64_t full_units, uint32_t threads = kThreads) {
    Geometry g;
    g.units = uint32_t(full_units);
    g.tiles = uint32_t((full_units + threads - 1) / threads);
    if (g.tiles == 0) g.tiles = 1;
    g.max_stripes_per_launch = uint32_t(((1ull << 31) / threads) / g.tiles);
    if (g.max_stripes_per_launch == 0) g.max_stripes_per_launch = 1;
    return g;
}

// Threads per block of the gf8 / bitmatrix kernels.  One-wave blocks when
// outputs are written away from the inputs (split data / parity, delta
// updates): consecutive 1 KiB column slices then go to different XCDs, and
// RS(10,4)@1 MiB encode gains 1 %, RS(10,4) update 2.3 %, RS(8,2)@4 KiB
// 2 %.  In-place layouts (win > 1) keep 4-wave blocks: one-wave blocks lose
// 1.4 % (RS) to 5 % (CRS) on in-place decode
// (profiles/r01/layout/block_ab*.log) — at RS(10,4)@1 MiB and
// CRS(12,4)@64 KiB.  The chunk-size sweeps (tools/block_ab_sizes.py,
// profiles/r01/layout/block_ab_sizes.log, block_ab_cauchy.log) find
// in-place layouts where one-wave blocks win instead (`wave_in_place`):
//   gf8 (byte-wise) with stripes under kWaveBlockSpan bytes: RS(4,2) /
//     RS(10,4) in-place decode at 4 KiB-256 KiB chunks, +2-7 points —
//     except stripe strides of exactly 512 KiB and 1 MiB, which keep
//     4-wave blocks (run_gf8; profiles/r02/wpc/win_pow2.log);
//   bitmatrix with chunks of kBmWaveChunk or more: CRS(12,4) / CRS(4,2)
//     in-place decode at 256 KiB-2 MiB, +1-9 points (64 KiB keeps 4 waves:
//     -6 points with one).
// Returns kWaveBlock or kThreads (a kernel template argument, so the
// 256-thread code is unchanged); MEC_BLOCK=64|256 overrides it per strided
// launch (gathered launches always use kThreads: their kernels are only
// instantiated for it).
constexpr int kWaveBlock = 64;
constexpr int64_t kWaveBlockSpan = int64_t(8) << 20;
constexpr uint64_t kBmWaveChunk = uint64_t(256) << 10;
uint32_t block_threads(bool strided, uint32_t win, bool wave_in_place = false);
// Single-map gathered gf8 launches (pointer tables) over device memory:
// line-aligned (128-byte) chunks take one-wave blocks with 16 resident waves
// per CU, others (8-byte ChunkPool headers, or 16-byte-aligned slots off the
// line grid: each wave's 1 KiB straddles an extra line) 4-wave blocks with 12; host memory and unknown layouts keep
// 4-wave blocks, uncapped (tools/gather_ab.py, profiles/r02/host/
// gather_ab2.log: +2-6 % aligned, +3-7 % unaligned at 64 KiB-1 MiB).
// Experiment knobs MEC_GBLOCK=64|256 and MEC_GWPC=<waves> (0 = no cap).
uint32_t gathered_block_threads(uint8_t gshape);
uint32_t gathered_lds(uint32_t bt, uint32_t static_lds, uint8_t gshape);

// Resident waves per CU of a streaming launch, capped through the LDS each
// block reserves (the kernels themselves use only their small coefficient
// tables).  More waves than the memory system can keep streaming cost HBM
// throughput: uncapped, the gf8 kernels run 79-84 % of 8 TB/s wherever
// their VGPR budget puts occupancy, capped at the right count 82-87 %
// (tools/wpc_ab.py, profiles/r02/wpc/).  The right count falls as a wave's
// own in-flight reads grow and rises with its output streams:
//   gf8 (all K source loads of a wave in flight at once)
//     split outputs, Vandermonde:      ceil_even(64 / K + R), 6..20; with
//                                      R = 4 at least min(ceil_even(K / 2 + 1), 16)
//     split outputs, dense (decode_split, ISA-L Cauchy encode):
//                          max(split count, min(ceil_even(64 / K + 2R), 16))
//     read-modify-write (update):      ceil_even(36 / R),      6..20
//     in place, dense (decode):        ceil_even(64 / K + 2R), 12..24
//     in place, Vandermonde (encode):  ceil_even(64 / K + R),  10..16
//   bitmatrix (one source, W packets, prefetched one ahead), 16-byte
//     slices: 3R, 6..16; 8-byte slices at w <= 4 (half the bytes in
//     flight per wave): 6R, 6..16 split, 6..12 in place
// in active waves (waves that own units; a block of small packets can have
// idle ones).  MEC_WPC=<n> overrides (0 = no cap): experiments flip it.
uint32_t gf8_target_waves(int k, int rows, bool in_place, bool dense, bool accumulate);
// Bytes per lane per packet of a strided bitmatrix launch (16 or 8; w > 4
// always 8).  A lane of the bitmatrix kernel reads the same slice of all w
// packets of a chunk, so a wave touches w 1 KiB address slots (mod 8 KiB)
// per chunk where a byte-wise wave touches one.  Blocks go to the 8 XCDs
// round-robin, and an in-place stream whose XCDs each touch one slot runs
// at 78-80 % of 8 TB/s, 72-74 % when each XCD touches four or eight (the
// same XOR-only kernel with its tiles rotated per stripe); the bitmatrix
// layout of packets under 8 KiB cannot be made slot-affine, so in-place CRS
// at 2-16 KiB chunks stays near that 72-74 % (tools/bm_variants.hip,
// profiles/r02/xcd/).  8-byte slices halve each wave's footprint, with the
// resident waves doubled to keep the bytes in flight (tools/bm_small_ab.py):
//   split layouts (encode, update): 8 bytes at every chunk size, +2-4
//     points (CRS(12,4)@64 KiB encode 80.7 -> 83.3 %);
//   in place: 8 bytes for chunks <= 8 KiB, or <= 32 KiB with <= 2 output
//     rows (+1-3 points; 16 bytes stay ahead above that, -5 to -9 points
//     at 256 KiB with 8).
// MEC_BM_VW=2|4 overrides (dwords per lane).
uint32_t bm_lane_bytes(int w, int rows, uint64_t chunk, bool in_place);
uint32_t bm_target_waves(int rows, int w, int vw, bool in_place);
// Dynamic LDS bytes per block of `bt` threads (`active` of them owning
// units, `static_lds` bytes of static LDS) so that about `waves` active waves
// share a CU; 0 = no cap.
uint32_t occupancy_lds(uint32_t bt, uint32_t active, uint32_t static_lds, uint32_t waves);

}  // namespace detail
}  // namespace mec
