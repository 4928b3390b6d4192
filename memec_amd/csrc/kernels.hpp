// kernels.hpp — host-side launch descriptors for libmec's HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mec {

constexpr int kMaxSrc = 32;   // k <= 32 (RS_N_MAX)
constexpr int kMaxRows = 4;   // outputs per launch; more are split into groups
constexpr int kMaxBmRows = 32;

// One GF(2^8) coefficient c as the three byte-permute tables used on the
// device: bits 0-2 of a byte index {t1:t0} = c*{0..7}; bits 3-5 index
// {u1:u0} = c*{0,8,..,56}; bits 6-7 index v = c*{0,64,128,192}.
struct Gf8Coef {
    uint32_t t0, t1, u0, u1, v;
};
Gf8Coef gf8_coef(uint8_t c);

// Chunk addressing of a launch.  Strided: source j of stripe s is
// src + s * src_stripe_stride + src_off[j] (dst likewise).  Gather (tab !=
// nullptr, a device array): stripe s's chunk pointers are the row
// tab[s * tab_stride ...]: sources at [0, k), outputs at [tab_dst, tab_dst +
// rows); src / dst / strides / offsets are then unused.

// out[r] (^)= sum_j coef[r][j] * src[j]  over GF(2^8), byte-wise.
struct Gf8Launch {
    const uint8_t *src;
    uint8_t *dst;
    int64_t src_stripe_stride, dst_stripe_stride;
    const uint64_t *tab;
    uint32_t tab_stride, tab_dst;
    int64_t src_off[kMaxSrc];
    int64_t dst_off[kMaxRows];
    int k, rows;
    uint64_t len;          // bytes per chunk region
    uint32_t n_stripes;
    bool accumulate;       // XOR into dst instead of overwriting
    Gf8Coef coef[kMaxRows][kMaxSrc];
};

// Bitmatrix (packet) form: chunk = w packets of `packet` bytes; output
// packet (r = i*w + l) (^)= XOR over (j, x) with bit x of mask[j][r] of
// source j packet x.
struct BmLaunch {
    const uint8_t *src;
    uint8_t *dst;
    int64_t src_stripe_stride, dst_stripe_stride;
    const uint64_t *tab;
    uint32_t tab_stride, tab_dst;
    int64_t src_off[kMaxSrc];
    int64_t dst_off[kMaxRows];
    int k, rows, w;        // rows = output chunks (each w packets)
    uint64_t packet;
    uint32_t n_stripes;
    bool accumulate;
    uint8_t mask[kMaxSrc][kMaxBmRows];
};

hipError_t launch_gf8(const Gf8Launch &L, hipStream_t stream);
hipError_t launch_bm(const BmLaunch &L, hipStream_t stream);
hipError_t launch_xor(uint8_t *dst, const uint8_t *a, const uint8_t *b, uint64_t len, hipStream_t stream);
hipError_t launch_fill(uint8_t *dst, uint64_t len, uint64_t seed, uint64_t word_offset, hipStream_t stream);

}  // namespace mec
