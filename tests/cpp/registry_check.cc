// registry_check.cc — the zero-copy registry's range rules
// (memec_amd/csrc/registry.hpp, used by hostmem.cpp): overlapping ranges
// refused, re-registration refused, unregister by begin only, lookups
// inside exactly one range, against a brute-force model over random
// register / unregister / lookup sequences.  Host code only.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>

#include "registry.hpp"

using mec::reg::Insert;
using mec::reg::Range;

static int fails = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);     \
            if (++fails > 20) std::exit(1);                             \
        }                                                               \
    } while (0)

int main() {
    // the named cases
    std::vector<Range> v;
    CHECK(mec::reg::can_insert(v, 0x1000, 0) == Insert::kEmpty);
    CHECK(mec::reg::can_insert(v, ~uintptr_t(0) - 4, 16) == Insert::kWraps);
    v = mec::reg::with(v, 0x10000, 0x1000, 0x90000);
    CHECK(mec::reg::can_insert(v, 0x10000, 0x1000) == Insert::kOverlap);  // re-register
    CHECK(mec::reg::can_insert(v, 0x10800, 0x10) == Insert::kOverlap);    // inside
    CHECK(mec::reg::can_insert(v, 0xF000, 0x1001) == Insert::kOverlap);   // starts below, extends across
    CHECK(mec::reg::can_insert(v, 0xF000, 0x1000) == Insert::kOk);        // ends where it begins
    CHECK(mec::reg::can_insert(v, 0x11000, 0x1000) == Insert::kOk);       // begins where it ends
    Range hit{};
    CHECK(mec::reg::can_insert(v, 0x8000, 0x100000, &hit) == Insert::kOverlap && hit.begin == 0x10000);
    uint64_t d = 0;
    CHECK(mec::reg::lookup(v, 0x10008, 0x800, d) && d == 0x90008);
    CHECK(!mec::reg::lookup(v, 0x10808, 0x800, d));  // runs past the end
    CHECK(!mec::reg::lookup(v, 0xFFF8, 0x10, d));
    bool found = false;
    std::vector<Range> w = mec::reg::without(v, 0x10008, found);
    CHECK(!found && w.size() == 1);
    w = mec::reg::without(v, 0x10000, found);
    CHECK(found && w.empty());

    // random sequences against a model: address space of 4096 cells of 64 B
    std::mt19937_64 rng(7);
    size_t ops = 0;
    for (int trial = 0; trial < 200; ++trial) {
        std::vector<Range> r;
        std::map<uintptr_t, Range> model;  // begin -> range
        auto owner = [&](uintptr_t a) -> const Range * {
            for (auto &kv : model)
                if (a >= kv.second.begin && a < kv.second.end) return &kv.second;
            return nullptr;
        };
        for (int step = 0; step < 400; ++step, ++ops) {
            const int op = int(rng() % 3);
            const uintptr_t b = 0x100000 + (rng() % 4096) * 64, len = 64 * (1 + rng() % 64);
            if (op == 0) {
                bool overlap = false;
                for (auto &kv : model) overlap |= b < kv.second.end && kv.second.begin < b + len;
                const Insert got = mec::reg::can_insert(r, b, len);
                CHECK((got == Insert::kOverlap) == overlap && (got == Insert::kOk) == !overlap);
                if (got == Insert::kOk) {
                    const uintptr_t dev = 0x7000000000ull + b * 3;
                    r = mec::reg::with(r, b, len, dev);
                    model[b] = Range{b, b + len, dev};
                }
            } else if (op == 1 && !model.empty()) {
                auto it = model.begin();
                std::advance(it, rng() % model.size());
                const uintptr_t key = (rng() % 4) ? it->first : it->first + 64;
                bool f = false;
                r = mec::reg::without(r, key, f);
                CHECK(f == (model.count(key) == 1));
                model.erase(key);
            } else {
                const uintptr_t a = 0x100000 + rng() % (4096 * 64 + 4096), n = 1 + rng() % 4096;
                const Range *o = owner(a);
                const bool inside = o && a + n <= o->end;
                uint64_t dv = 0;
                const bool got = mec::reg::lookup(r, a, n, dv);
                CHECK(got == inside);
                if (got && inside) CHECK(dv == o->dev + (a - o->begin));
            }
            for (size_t i = 1; i < r.size(); ++i) CHECK(r[i - 1].end <= r[i].begin);
            CHECK(r.size() == model.size());
        }
    }
    if (fails) return 1;
    std::printf("ok %zu\n", ops);
    return 0;
}
