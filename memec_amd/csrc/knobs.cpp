// knobs.cpp — experiment overrides, read from the environment once (see
// knobs.hpp).
#include "knobs.hpp"

#include <atomic>
#include <cstdlib>
#include <cstring>

namespace mec {
namespace detail {
namespace {

// every knob's variable (the environment is read for each, once)
constexpr const char *kEnvNames[] = {"MEC_SGROUP", "MEC_WINDOWS",      "MEC_BLOCK", "MEC_GBLOCK",  "MEC_GWPC",
                                     "MEC_BM_VW",  "MEC_WPC",          "MEC_COPY_THREADS", "MEC_WIDE",
                                     "MEC_MG_ROWS"};
// MEC_SGROUP sets two knobs (group and run), every other name one
static_assert(sizeof(kEnvNames) / sizeof(kEnvNames[0]) == kKnobCount - 1, "a knob whose variable is never read");

struct Knobs {
    std::atomic<int64_t> v[kKnobCount];
    Knobs() {
        for (auto &x : v) x.store(kKnobUnset, std::memory_order_relaxed);
        for (const char *n : kEnvNames) apply(n, std::getenv(n));
    }
    bool apply(const char *name, const char *value) {
        auto put = [&](Knob k, int64_t x) { v[k].store(x, std::memory_order_relaxed); };
        const bool unset = value == nullptr;
        const int64_t num = unset ? kKnobUnset : int64_t(std::atoll(value));
        if (!std::strcmp(name, "MEC_SGROUP")) {
            if (unset) {
                put(kKnobSgroup, kKnobUnset);
                put(kKnobSrun, kKnobUnset);
            } else {
                put(kKnobSgroup, num);
                const char *c = std::strchr(value, ':');
                put(kKnobSrun, c ? int64_t(std::atoll(c + 1)) : kKnobUnset);
            }
            return true;
        }
        static const struct {
            const char *name;
            Knob k;
        } kPlain[] = {{"MEC_WINDOWS", kKnobWindows}, {"MEC_BLOCK", kKnobBlock},   {"MEC_GBLOCK", kKnobGblock},
                      {"MEC_GWPC", kKnobGwpc},       {"MEC_BM_VW", kKnobBmVw},     {"MEC_WPC", kKnobWpc},
                      {"MEC_COPY_THREADS", kKnobCopyThreads}, {"MEC_WIDE", kKnobWide},
                      {"MEC_MG_ROWS", kKnobMgRows}};
        for (const auto &p : kPlain)
            if (!std::strcmp(name, p.name)) {
                put(p.k, num);
                return true;
            }
        return false;
    }
};

Knobs &knobs() {
    static Knobs k;
    return k;
}

}  // namespace

int64_t knob(Knob k) { return knobs().v[k].load(std::memory_order_relaxed); }

bool set_knob(const char *name, const char *value) { return name && knobs().apply(name, value); }

}  // namespace detail
}  // namespace mec
