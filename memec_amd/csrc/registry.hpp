// registry.hpp — the zero-copy registry's range arithmetic (hostmem.cpp),
// host code only, so tests/cpp/registry_check.cc checks it on the CPU.
//
// Registered host ranges are kept sorted by begin and pairwise disjoint.  A
// new range that overlaps an existing one is refused:
// with overlaps allowed, a slab freed without mec_host_unregister left a
// stale range, and a later slab that started below it and extended across
// it had the addresses inside the stale range translated to the old
// mapping (lookup takes the range with the greatest begin <= the address).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace mec {
namespace reg {

struct Range {
    uintptr_t begin, end, dev;
};

enum class Insert { kOk, kEmpty, kWraps, kOverlap };

// The range [b, b + len) may join v (sorted, disjoint): not empty, no
// address wrap, disjoint from every member.  `hit` = the overlapped member.
inline Insert can_insert(const std::vector<Range> &v, uintptr_t b, size_t len, Range *hit = nullptr) {
    if (len == 0) return Insert::kEmpty;
    if (b + len < b) return Insert::kWraps;
    const uintptr_t e = b + len;
    // the first member that ends after b is the only candidate below e
    auto it = std::upper_bound(v.begin(), v.end(), b, [](uintptr_t x, const Range &g) { return x < g.end; });
    if (it != v.end() && it->begin < e) {
        if (hit) *hit = *it;
        return Insert::kOverlap;
    }
    return Insert::kOk;
}

// v with [b, b + len) -> dev added, sorted (can_insert must have said kOk).
inline std::vector<Range> with(const std::vector<Range> &v, uintptr_t b, size_t len, uintptr_t dev) {
    std::vector<Range> r;
    r.reserve(v.size() + 1);
    auto it = std::lower_bound(v.begin(), v.end(), b, [](const Range &g, uintptr_t x) { return g.begin < x; });
    r.insert(r.end(), v.begin(), it);
    r.push_back(Range{b, b + len, dev});
    r.insert(r.end(), it, v.end());
    return r;
}

// v without the range that begins at b; `found` says whether there was one.
inline std::vector<Range> without(const std::vector<Range> &v, uintptr_t b, bool &found) {
    std::vector<Range> r;
    r.reserve(v.size());
    found = false;
    for (const Range &g : v) {
        if (g.begin == b) found = true;
        else r.push_back(g);
    }
    return r;
}

// Device address of [a, a + len) when it lies inside one member.
inline bool lookup(const std::vector<Range> &v, uintptr_t a, size_t len, uint64_t &dev) {
    auto it = std::upper_bound(v.begin(), v.end(), a, [](uintptr_t x, const Range &g) { return x < g.begin; });
    if (it == v.begin()) return false;
    --it;
    if (a < it->begin || a + len < a || a + len > it->end) return false;
    dev = uint64_t(it->dev + (a - it->begin));
    return true;
}

}  // namespace reg
}  // namespace mec
