// knobs.cpp — experiment overrides, read from the environment once (see
// knobs.hpp), every value validated against its knob's accepted set.
#include "knobs.hpp"

#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace mec {
namespace detail {
namespace {

// Accepted values.  Wave caps: 0 (no cap) .. 32 waves per CU (the gfx950
// limit); windows 1..16; MEC_SGROUP groups 0..64 stripes (0 / 1 = identity
// map) with runs of 8..1024 tiles in steps of 8 (stripe_tile's contract).
constexpr KnobSpec kSpecs[] = {
    {"MEC_SGROUP", kKnobSgroup, 0, 64, {}, 0, 0},
    {"MEC_WINDOWS", kKnobWindows, 1, 16, {}, 0},
    {"MEC_BLOCK", kKnobBlock, 64, 256, {64, 256}, 2},
    {"MEC_GBLOCK", kKnobGblock, 64, 256, {64, 256}, 2},
    {"MEC_GWPC", kKnobGwpc, 0, 32, {}, 0},
    {"MEC_BM_VW", kKnobBmVw, 2, 4, {2, 4}, 2},
    {"MEC_WPC", kKnobWpc, 0, 32, {}, 0},
    {"MEC_COPY_THREADS", kKnobCopyThreads, 1, 64, {}, 0},
    {"MEC_WIDE", kKnobWide, 0, 1, {}, 0},
    {"MEC_MG_ROWS", kKnobMgRows, 3, 8, {3, 4, 8}, 3},
    {"MEC_BITSLICE", kKnobBitslice, 0, 3, {}, 0},
    {"MEC_BS_WAVES", kKnobBsWaves, 0, 8, {}, 0},
    {"MEC_BS_PREFETCH", kKnobBsPrefetch, 0, 31, {}, 0},
    {"MEC_BS_TPB", kKnobBsTpb, 0, 64, {}, 0},
    {"MEC_TILE_SKEW", kKnobTileSkew, 0, 1024, {}, 0, 8},
    {"MEC_BS_FENCE", kKnobBsFence, 0, 1, {}, 0, 0},
    {"MEC_BS_XCD", kKnobBsXcd, 0, 1, {}, 0, 0},
    {"MEC_BS_VROW", kKnobBsVrow, 0, 1, {}, 0, 0},
    {"MEC_WBATCH", kKnobWbatch, 0, 4, {0, 2, 4}, 3, 0},
    {"MEC_TAB_WAIT", kKnobTabWait, 0, 1, {}, 0, 0},
    {"MEC_GXCD", kKnobGxcd, 0, 1, {}, 0, 0},
    {"MEC_GU", kKnobGu, 1, 2, {}, 0, 0},
};
// every knob but MEC_SGROUP's run half has its own variable
static_assert(sizeof(kSpecs) / sizeof(kSpecs[0]) == kKnobCount - 1, "a knob whose variable is never read");

// A whole decimal integer (optionally signed), nothing else.
bool parse_int(const char *s, const char *end, int64_t &out) {
    if (s == end) return false;
    char buf[32];
    const size_t n = size_t(end - s);
    if (n >= sizeof buf) return false;
    std::memcpy(buf, s, n);
    buf[n] = 0;
    char *e = nullptr;
    errno = 0;
    const long long v = std::strtoll(buf, &e, 10);
    if (errno || e != buf + n) return false;
    out = int64_t(v);
    return true;
}

bool accepted(const KnobSpec &s, int64_t v) {
    if (v < s.lo || v > s.hi) return false;
    if (s.step > 1 && (v - s.lo) % s.step != 0) return false;
    if (s.nset == 0) return true;
    for (int i = 0; i < s.nset; ++i)
        if (s.set[i] == v) return true;
    return false;
}

struct Knobs {
    std::atomic<int64_t> v[kKnobCount];
    Knobs() {
        for (auto &x : v) x.store(kKnobUnset, std::memory_order_relaxed);
        for (const KnobSpec &s : kSpecs) {
            const char *e = std::getenv(s.name);
            if (e && apply(s, e) != KnobStatus::kOk)
                std::fprintf(stderr, "libmec: %s=%s is not an accepted value; the built-in rule applies\n", s.name, e);
        }
    }
    KnobStatus apply(const KnobSpec &s, const char *value) {
        auto put = [&](Knob k, int64_t x) { v[k].store(x, std::memory_order_relaxed); };
        if (!value) {
            put(s.knob, kKnobUnset);
            if (s.knob == kKnobSgroup) put(kKnobSrun, kKnobUnset);
            return KnobStatus::kOk;
        }
        const char *end = value + std::strlen(value);
        if (s.knob == kKnobSgroup) {
            const char *c = std::strchr(value, ':');
            int64_t g = 0, r = kKnobUnset;
            if (!parse_int(value, c ? c : end, g) || !accepted(s, g)) return KnobStatus::kInvalid;
            if (c && (!parse_int(c + 1, end, r) || r < 8 || r > kSrunMax || r % 8 != 0)) return KnobStatus::kInvalid;
            put(kKnobSgroup, g);
            put(kKnobSrun, r);
            return KnobStatus::kOk;
        }
        int64_t x = 0;
        if (!parse_int(value, end, x) || !accepted(s, x)) return KnobStatus::kInvalid;
        put(s.knob, x);
        return KnobStatus::kOk;
    }
};

Knobs &knobs() {
    static Knobs k;
    return k;
}

}  // namespace

const KnobSpec *knob_specs(int &n) {
    n = int(sizeof(kSpecs) / sizeof(kSpecs[0]));
    return kSpecs;
}

int64_t knob(Knob k) { return knobs().v[k].load(std::memory_order_relaxed); }

KnobStatus set_knob(const char *name, const char *value) {
    if (!name) return KnobStatus::kUnknown;
    for (const KnobSpec &s : kSpecs)
        if (!std::strcmp(name, s.name)) return knobs().apply(s, value);
    return KnobStatus::kUnknown;
}

}  // namespace detail
}  // namespace mec
