// kernels.hpp — host-side launch descriptors for libmec's HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace mec {

constexpr int kMaxSrc = 32;   // k + m <= 32 (RS_N_MAX)
constexpr int kMaxK = 31;     // sources of one launch: k <= 31 (m >= 1)
constexpr int kMaxRows = 4;   // outputs per launch; more are split into groups (gf8: see gf8_mg_kernel)
constexpr int kMaxBmOut = 8;  // outputs per strided bitmatrix launch (m > 8 splits)
constexpr int kMaxBmRows = kMaxBmOut * 8;  // its output packets (outputs x w)

// One GF(2^8) coefficient c as the three byte-permute tables used on the
// device: bits 0-2 of a byte index {t1:t0} = c*{0..7}; bits 3-5 index
// {u1:u0} = c*{0,8,..,56}; bits 6-7 index v = c*{0,64,128,192}.
struct Gf8Coef {
    uint32_t t0, t1, u0, u1, v;
};
Gf8Coef gf8_coef(uint8_t c);

// Chunk addressing: strided (src + s * src_stripe_stride + src_off[j]), or,
// when stab != nullptr (device arrays of chunk pointers, one row per
// stripe), gathered: source j = stab[s * sstride + src_off[j]], output r =
// dtab[s * dstride + dst_off[r]] (0 = all-zero source / unwanted output).

// out[r] (^)= sum_j coef[r][j] * src[j]  over GF(2^8), byte-wise.
struct Gf8Launch {
    const uint8_t *src;
    uint8_t *dst;
    int64_t src_stripe_stride, dst_stripe_stride;
    const uint64_t *stab, *dtab;
    uint32_t sstride, dstride;
    int64_t src_off[kMaxSrc];
    int64_t dst_off[kMaxRows];
    int k, rows;
    uint64_t len;          // bytes per chunk region
    uint32_t n_stripes;
    bool accumulate;       // XOR into dst instead of overwriting
    // pointer tables over device memory: 1 = every sampled chunk 16-byte
    // aligned, 2 = some are not (MemEC's 8-byte ChunkPool headers); 0 =
    // unknown / host memory (gathered_block_threads)
    uint8_t gshape;
    // measurement twin (mec_set_probe): strided launches run the same
    // kernel with every product a plain XOR (kGf8Xor); outputs are not codes
    bool probe;
    Gf8Coef coef[kMaxRows][kMaxSrc];
};

// Bitmatrix (packet) form: chunk = w packets of `packet` bytes; output
// packet (r = i*w + l) (^)= XOR over (j, x) with bit x of mask[j][r] of
// source j packet x.
struct BmLaunch {
    const uint8_t *src;
    uint8_t *dst;
    int64_t src_stripe_stride, dst_stripe_stride;
    const uint64_t *stab, *dtab;
    uint32_t sstride, dstride;
    int64_t src_off[kMaxSrc];
    int64_t dst_off[kMaxBmOut];
    int k, rows, w;        // rows = output chunks (each w packets), <= kMaxBmOut = 8 (strided and gathered)
    uint64_t packet;
    uint32_t n_stripes;
    bool accumulate;
    uint8_t gshape;        // as Gf8Launch::gshape
    uint8_t mask[kMaxSrc][kMaxBmRows];
};

// ---- gathered launches (pointer-array batches) -------------------------------
// A stripe's chunks are found through device tables of chunk pointers (one
// row per stripe, as server/ holds Chunk* arrays) and its linear map through
// a descriptor in device memory, so stripes with different erasure patterns
// (decode) or delta columns (update) share one launch.
constexpr uint8_t kNoRow = 0xFF;
constexpr uint16_t kSkipStripe = 0xFFFF;

// Descriptor blobs (uint32 words), one per map, desc_dw words apart:
//  gf8 (K sources, 4 rows): [0..3] ones bits, [4..7] zeros bits (bit i*K+j),
//      [8..15] ssel bytes, [16] dsel bytes (kNoRow = no output), then at
//      kGf8DescHead + (i*K + j)*8 the v_perm tables t0 t1 u0 u1 v of
//      coefficient (i, j);  desc_dw = kGf8DescHead + 4*K*8.
//  bitmatrix (K sources, width w, up to kMaxBmOut = 8 rows): [0..7] ssel
//      bytes, [8..9] dsel bytes, then at kBmDescHead + j*2w + q the mask
//      bytes 4q..4q+3 of source j (byte i*w + l: bit x set <=> packet x
//      feeds output i packet l); desc_dw = kBmDescHead + kMaxSrc*2w.
constexpr int kGf8DescHead = 32;
constexpr int kBmDescHead = 16;
constexpr int kBmGatherRows = 8;  // outputs per gathered bitmatrix launch (= kMaxBmOut)

struct GatherLaunch {
    const uint64_t *stab;  // source pointer rows: stripe s at stab + s * sstride (0 = all-zero chunk)
    const uint64_t *dtab;  // output pointer rows (0 = output not wanted)
    uint32_t sstride, dstride;
    const void *desc;      // descriptor blobs of this row group (device)
    uint32_t desc_dw;      // dwords per descriptor
    const uint16_t *pat;   // per-stripe descriptor index, kSkipStripe = no work; nullptr = desc 0
    uint32_t n_stripes;
    int k, rows;           // sources per stripe, output rows of this launch
    int w;                 // bitmatrix field width
    uint64_t len;          // gf8: bytes per chunk; bitmatrix: packet bytes
    bool accumulate;       // XOR into outputs
    // gf8 only: row groups of kMaxRows coded in one launch (0/1 = this
    // group only); group g's descriptors at desc + g * group_maps * desc_dw
    uint32_t groups, group_maps;
};

// Host side of a multi-group launch: rows (> kMaxRows) outputs at dst_off,
// coef[r * k + j], in groups of group_rows (gf8_mg_rows); the permute tables
// in device memory (tabs, from gf8_mg_tables for the same coef and
// group_rows).
struct Gf8MgLaunch {
    const uint8_t *src;
    uint8_t *dst;
    int64_t src_stripe_stride, dst_stripe_stride;
    // pointer batches (one map for every stripe): chunk pointers at
    // stab[s * sstride + src_off[j]], dtab[s * dstride + dst_off[r]]
    // (device-readable); src / dst unused then
    const uint64_t *stab, *dtab;
    uint32_t sstride, dstride;
    int64_t src_off[kMaxSrc];
    int64_t dst_off[kMaxSrc];
    int k, rows, group_rows;
    uint64_t len;
    uint32_t n_stripes;
    bool accumulate, vand;
    const uint32_t *tabs;
};
// 8-row groups are instantiated for these source counts.
constexpr int kMg8MinK = 12, kMg8MaxK = 20;
// Rows per group.  Groups of 8 when the rows split into whole groups of 8
// and the sources are many: each source's bit fields are extracted once per
// group, so 8-row groups halve that work against two groups of 4, at 160-230
// VGPRs instead of 130-150 (one wave less per SIMD).  Measured at 64 KiB
// chunks (tools/wide_r8_probe.hip, profiles/r04/probes/wide_r8_probe_box*.log,
// groups of 4 -> 8): RS(16,8) 63.5 -> 69.0 %, RS(20,8) 61.9 -> 62.4, dense
// ISA-L Cauchy(12,8) 63.2 -> 65.2, Cauchy(20,8) 55.3 -> 56.4, Cauchy(16,8)
// and RS(24,8) even; Vandermonde K = 10 and 12 (whose first group skips row
// 0's products) lose 0.5-3 points.  Otherwise 3 or 4, whichever pads fewer
// rows (5 -> 3+2, 6 -> 3+3, 7 -> 4+3, 8 -> 4+4, 9 -> 3+3+3).
inline int gf8_mg_rows(int rows, int k, bool vand) {
    if (rows % 8 == 0 && k <= kMg8MaxK && (k >= 16 || (!vand && k >= kMg8MinK))) return 8;
    const int g4 = (rows + 3) / 4, g3 = (rows + 2) / 3;
    return g4 * 4 - rows <= g3 * 3 - rows ? 4 : 3;
}
// The permute-table image for coef (rows x k) at R rows per group: groups x
// R x k x 8 dwords, padding rows zero.
void gf8_mg_tables(const uint8_t *coef, int rows, int k, int R, std::vector<uint32_t> &out);

// Run-time compiled bit-sliced launch (jit.cpp, bitslice.hpp): rows > 4
// byte-wise outputs of a chunk that is a multiple of 16 bytes, strided or
// gathered addressing as Gf8MgLaunch.
struct BsLaunch {
    const uint8_t *src;
    uint8_t *dst;
    int64_t src_stripe_stride, dst_stripe_stride;
    const uint64_t *stab, *dtab;
    uint32_t sstride, dstride;
    int64_t src_off[kMaxSrc];
    int64_t dst_off[kMaxSrc];
    int k, rows;
    uint64_t len;
    uint32_t n_stripes;
    uint32_t tpb;  // gathered: 2 KiB tiles per block the kernel was built for (0 = MEC_BS_TPB / rule)
    bool vand;     // row 0 and column 0 all ones (the Vandermonde-structured encodes): the wave cap (plan_bs)
};

hipError_t launch_gf8(const Gf8Launch &L, hipStream_t stream);
hipError_t launch_gf8_mg(const Gf8MgLaunch &L, hipStream_t stream);
hipError_t launch_gf8_gather(const GatherLaunch &L, hipStream_t stream);
hipError_t launch_bm_gather(const GatherLaunch &L, hipStream_t stream);
hipError_t launch_bm(const BmLaunch &L, hipStream_t stream);
hipError_t launch_xor(uint8_t *dst, const uint8_t *a, const uint8_t *b, uint64_t len, hipStream_t stream);
hipError_t launch_fill(uint8_t *dst, uint64_t len, uint64_t seed, uint64_t word_offset, hipStream_t stream);
// 32-bit slab offsets (mec_*_batch32) expanded into chunk pointers on the
// device: out[e] = in[e] == kNullOff ? 0 : base + (in[e] << shift).  in must
// be 16-byte aligned.
constexpr uint32_t kNullOff = 0xFFFFFFFFu;
hipError_t launch_expand_rows(const uint32_t *in, uint64_t *out, uint64_t base, uint32_t shift, uint64_t n,
                              hipStream_t stream);

}  // namespace mec
