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

// Launch geometry shared by the streaming kernels: `units` per stripe,
// each thread takes `upt` units spaced kThreads apart (so a wave's 64
// lanes stay contiguous), `tiles` blocks per stripe.
struct Geometry {
    uint32_t units, upt, tiles, max_stripes_per_launch;
};

inline Geometry geometry(uint64_t units) {
    Geometry g;
    g.units = uint32_t(units);
    g.upt = units >= 16 * kThreads ? 4 : 1;
    g.tiles = uint32_t((units + uint64_t(g.upt) * kThreads - 1) / (uint64_t(g.upt) * kThreads));
    if (g.tiles == 0) g.tiles = 1;
    // keep grid * block under 2^32 work-items
    g.max_stripes_per_launch = uint32_t(((1ull << 31) / kThreads) / g.tiles);
    if (g.max_stripes_per_launch == 0) g.max_stripes_per_launch = 1;
    return g;
}

}  // namespace detail
}  // namespace mec
