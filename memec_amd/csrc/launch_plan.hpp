// launch_plan.hpp — host-side launch planning of libmec's streaming kernels.
//
// Every strided, one-pass, bitmatrix, gathered and XOR launch takes its
// shape from one function here: threads per block, the dynamic LDS that
// caps resident waves, block windows, the stripe-group map, lane width and
// row groups.  The .hip launchers only fill kernel arguments from a plan and
// launch it, so the planner — host C++ with no device code — is what
// tests/cpp/launch_plan_check.cc runs on the CPU against the invariants each
// kernel relies on (rows per group x groups <= 32 kernel-argument slots, LDS
// <= 160 KiB per block, only instantiated templates, 32-bit lane offsets)
// for every accepted value of every MEC_* knob.  A plan the planner cannot
// make valid has ok = false and the launcher returns hipErrorInvalidValue
// instead of launching.
#pragma once

#include <cstdint>

#include "kernels.hpp"

namespace mec {
namespace detail {

constexpr int kThreads = 256;
constexpr int kWaveBlock = 64;
constexpr int64_t kWaveBlockSpan = int64_t(8) << 20;
constexpr uint64_t kBmWaveChunk = uint64_t(256) << 10;
constexpr uint32_t kLdsPerCu = 160u << 10;  // gfx950: one block may take all of it
// In-place strided launches rotate stripe s's tiles by s * kTileSkew
// (DESIGN §5.3); 0 keeps the identity order.
constexpr int64_t kTileSkew = 0;
// Bit-sliced launches of at most this many blocks per stripe take XCD runs
// (plan_bs): gathered, strided.
constexpr uint32_t kBsXcdTiles = 32;
constexpr uint32_t kBsXcdStridedTiles = 2;

// Matrix structure a gf8 launch is specialised for (gf8_kernel.hpp).
constexpr int kGf8Dense = 0;
constexpr int kGf8Vand = 1;
constexpr int kGf8Xor = 2;
constexpr int kGf8Col0 = 3;

// Host side: the structure a coefficient block qualifies for (kGf8Vand:
// row 0 and column 0 all ones, else kGf8Dense).
int gf8_structure(const Gf8Coef (*coef)[kMaxSrc], int k, int rows);

// Launch geometry of the streaming kernels: one full unit per thread
// (measured faster than looping 2-16 units per thread), `tiles` blocks of
// `threads` per stripe, grid split so grid * block stays < 2^31 work-items.
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

// One launch (or one sub-launch of a strided batch: stripes [s0, s0 + ns)).
struct KernelPlan {
    bool ok = false;
    const char *why = "";    // reason when !ok
    int k = 0, rows = 0;     // the instantiation's source count K and rows R
    uint32_t groups = 1;     // row groups coded from one read of the sources
    int structure = kGf8Dense;
    uint32_t bt = 0;         // threads per block
    uint32_t vw = 4;         // dwords per lane (bitmatrix 2 or 4; byte-wise 4)
    uint32_t lds_static = 0, lds_dynamic = 0;
    uint32_t win = 1, sgroup = 0, srun = 8;
    uint32_t skew = 0;       // per-stripe tile rotation (identity map, in place; MEC_TILE_SKEW)
    uint32_t tpb = 1;        // tiles per block (bit-sliced kernels: geo.tiles = blocks per stripe)
    uint32_t xcd = 0;        // bit-sliced: blocks b, b + 8, ... (one XCD) take one run of the launch's blocks
    uint32_t gu = 1;         // one-map gathered gf8, one-wave blocks: 16-byte units per lane (64 apart)
    Geometry geo{};
    uint32_t ns = 0;         // stripes in this launch
    uint64_t grid = 0;       // blocks
};

// ---- the rules ---------------------------------------------------------------
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
// Rows per group of a one-pass launch of `rows` outputs over k sources
// (gf8_mg_rows, kernels.hpp), MEC_MG_ROWS applied only where the groups fit
// the kernel's kMaxSrc output slots and the template exists.
int mg_group_rows(int rows, int k, bool vand);

// ---- plans ------------------------------------------------------------------
// gf8_kernel: strided sub-launch of stripes [s0, s0 + ns), or a gathered
// one (L.stab).  `structure` is the kernel the launcher picks.
KernelPlan plan_gf8(const Gf8Launch &L, uint32_t s0);
// gf8_mg_kernel (L.group_rows rows per group).
KernelPlan plan_gf8_mg(const Gf8MgLaunch &L, uint32_t s0);
// bm_kernel.
KernelPlan plan_bm(const BmLaunch &L, uint32_t s0);
// gf8_gather_kernel / bm_gather_kernel (one launch per max_stripes chunk).
KernelPlan plan_gf8_gather(const GatherLaunch &L, uint32_t s0);
KernelPlan plan_bm_gather(const GatherLaunch &L, uint32_t s0);
// The run-time compiled bit-sliced kernel (jit.cpp): one-wave blocks over
// 2 KiB tiles of every chunk.
KernelPlan plan_bs(const BsLaunch &L, uint32_t s0);
// Tiles per block of a gathered bit-sliced kernel built now: MEC_BS_TPB, or 1.
uint32_t bs_gather_tpb();
// Resident waves per CU of a bit-sliced launch (plan_bs).
// Bytes in flight per CU the split dense bit-sliced launches are capped to.
constexpr uint32_t kBsInflightKiB = 144;
uint32_t bs_target_waves(bool in_place, bool vand, bool gather, int k, int rows, uint32_t tiles);
// xor_kernel over len bytes.
KernelPlan plan_xor(uint64_t len);

// Static LDS of the kernels (bytes), as their __shared__ declarations.
constexpr uint32_t gf8_static_lds(int k, int rows) { return uint32_t(rows * k * 8 * 4); }
constexpr uint32_t gf8_gather_static_lds(int k, int rows) {
    return uint32_t((kGf8DescHead + rows * k * 8) * 4 + (k + rows) * 8);
}
constexpr uint32_t bm_gather_static_lds(int w, int rows) {
    return uint32_t((kBmDescHead + kMaxSrc * 2 * w) * 4 + (kMaxSrc + rows) * 8);
}

}  // namespace detail
}  // namespace mec
