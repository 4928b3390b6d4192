// launch_plan_check.cc — CPU check of libmec's launch planner
// (memec_amd/csrc/launch_plan.cpp) under every accepted value of every MEC_*
// launch knob: each plan the launchers would issue must satisfy the
// invariants its kernel relies on.  No device is touched: chunk addresses are
// synthetic (never dereferenced), only their layout (split or in place)
// matters to the planner.
//
//   * gf8_mg_kernel: groups x rows per group <= kMaxSrc (its dst_off[] slots;
//     the round-4 MEC_MG_ROWS=3 path gave 11 x 3 = 33 for 31 rows), rows per
//     group in {3, 4, 8}, 8 only for K = kMg8MinK..kMg8MaxK (the
//     instantiated templates, chosen for their VGPR budget);
//   * gf8 R <= 4, bitmatrix R <= 8 and w <= 8, gathered multi-group launches
//     only with 4 rows per group and at most kMaxSrc rows;
//   * blocks of 64 or 256 threads (the instantiated block sizes), static +
//     dynamic LDS <= 160 KiB, grid x block < 2^31 work-items, lane byte
//     offsets within 32 bits, stripe-group runs that tile the stripe;
//   * the sub-launches of a strided batch cover every stripe exactly once;
//   * a legal call always gets a plan (the planner falls back to the
//     built-in rule instead of refusing it).
// Prints "ok <plans checked>" or the first violations, exit status 1.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "knobs.hpp"
#include "launch_plan.hpp"

using namespace mec;
using namespace mec::detail;

static long g_plans = 0, g_bad = 0;
static std::string g_ctx;

static void bad(const char *what, const KernelPlan &p) {
    if (g_bad++ < 20)
        std::printf("VIOLATION %s [%s] k=%d rows=%d groups=%u bt=%u lds=%u+%u grid=%llu win=%u sgroup=%u run=%u why=%s\n",
                    what, g_ctx.c_str(), p.k, p.rows, p.groups, p.bt, p.lds_static, p.lds_dynamic,
                    (unsigned long long)p.grid, p.win, p.sgroup, p.srun, p.why);
}

static void common(const KernelPlan &p, uint64_t lane_span) {
    ++g_plans;
    if (!p.ok) return bad("legal call refused", p);
    if (p.bt != uint32_t(kWaveBlock) && p.bt != uint32_t(kThreads)) bad("block size not instantiated", p);
    if (uint64_t(p.lds_static) + p.lds_dynamic > kLdsPerCu) bad("LDS over 160 KiB", p);
    if (p.grid == 0 || p.grid * p.bt >= (uint64_t(1) << 31) + 1) bad("grid x block past 2^31", p);
    if (lane_span > (uint64_t(1) << 32)) bad("lane offsets past 32 bits", p);
    if (p.win < 1) bad("no window", p);
    if (p.sgroup != 0 && (p.srun == 0 || p.srun % 8 || p.geo.tiles % p.srun)) bad("stripe-group run", p);
    if (p.skew != 0 && (p.sgroup != 0 || p.skew >= p.geo.tiles)) bad("tile skew off the identity map", p);
}

// Synthetic layouts: split (sources and outputs in separate regions) or in
// place (outputs inside the sources' stripe span).
struct Layout {
    const uint8_t *src;
    uint8_t *dst;
    int64_t sss, dss;
};
static Layout layout(bool in_place, uint64_t chunk, int k, int rows) {
    const uintptr_t base = uintptr_t(1) << 40;
    Layout l;
    if (in_place) {
        l.src = reinterpret_cast<const uint8_t *>(base);
        l.dst = reinterpret_cast<uint8_t *>(base + uintptr_t(k) * chunk);
        l.sss = l.dss = int64_t(k + rows) * int64_t(chunk);
    } else {
        l.src = reinterpret_cast<const uint8_t *>(base);
        l.dst = reinterpret_cast<uint8_t *>(base + (uintptr_t(1) << 39));
        l.sss = int64_t(k) * int64_t(chunk);
        l.dss = int64_t(rows) * int64_t(chunk);
    }
    return l;
}

static Gf8Coef coef_of(bool one) {
    Gf8Coef c{};
    c.t0 = one ? 0x03020100u : 0x11223344u;
    return c;
}

static const uint64_t kChunks[] = {16, 48, 1024, 4096, 4112, 65536, 256u << 10, 1u << 20, 2u << 20, 16u << 20};
static const uint32_t kStripes[] = {1, 7, 4096, 65536};

static void check_gf8(int k, int rows, uint64_t chunk, uint32_t n, bool in_place, bool vand, bool acc, bool probe,
                      bool gather) {
    Gf8Launch L{};
    const Layout ly = layout(in_place, chunk, k, rows);
    L.src = ly.src;
    L.dst = ly.dst;
    L.src_stripe_stride = ly.sss;
    L.dst_stripe_stride = ly.dss;
    static const uint64_t tab[1] = {0};
    if (gather) {
        L.stab = L.dtab = tab;
        L.sstride = L.dstride = uint32_t(k + rows);
        L.gshape = uint8_t(n % 3);
    }
    L.k = k;
    L.rows = rows;
    L.len = chunk;
    L.n_stripes = n;
    L.accumulate = acc;
    L.probe = probe;
    for (int i = 0; i < rows; ++i)
        for (int j = 0; j < k; ++j) L.coef[i][j] = coef_of(vand && (i == 0 || j == 0));
    uint64_t covered = 0;
    for (uint32_t s0 = 0; s0 < n;) {
        const KernelPlan p = plan_gf8(L, s0);
        common(p, uint64_t(p.geo.units) * 16);
        if (!p.ok || p.ns == 0) break;
        if (p.rows > kMaxRows || p.k > kMaxK) bad("gf8 template not instantiated", p);
        covered += p.ns;
        s0 += p.ns;
    }
    if (covered != n) {
        KernelPlan z;
        bad("sub-launches do not cover the batch", z);
    }
}

static void check_mg(int k, int rows, uint64_t chunk, uint32_t n, bool in_place, bool vand, bool acc, bool gather) {
    Gf8MgLaunch L{};
    const Layout ly = layout(in_place, chunk, k, rows);
    L.src = ly.src;
    L.dst = ly.dst;
    L.src_stripe_stride = ly.sss;
    L.dst_stripe_stride = ly.dss;
    static const uint64_t tab[1] = {0};
    static const uint32_t tabs[1] = {0};
    if (gather) {
        L.stab = L.dtab = tab;
        L.sstride = L.dstride = uint32_t(k + rows);
    }
    L.k = k;
    L.rows = rows;
    L.len = chunk;
    L.n_stripes = n;
    L.accumulate = acc;
    L.vand = vand;
    L.tabs = tabs;
    L.group_rows = mg_group_rows(rows, k, vand);
    uint64_t covered = 0;
    for (uint32_t s0 = 0; s0 < n;) {
        const KernelPlan p = plan_gf8_mg(L, s0);
        common(p, uint64_t(p.geo.units) * 16);
        if (!p.ok || p.ns == 0) break;
        if (p.groups * uint32_t(p.rows) > uint32_t(kMaxSrc)) bad("groups x rows past the kernel's dst_off[] slots", p);
        if (p.rows != 3 && p.rows != 4 && p.rows != 8) bad("rows per group not instantiated", p);
        if (p.rows == 8 && (p.k < kMg8MinK || p.k > kMg8MaxK)) bad("8-row groups outside K = 12..20", p);
        if (p.groups * uint32_t(p.rows) < uint32_t(rows)) bad("groups do not cover the rows", p);
        if (p.bt != uint32_t(kWaveBlock)) bad("one-pass kernel is one-wave blocks only", p);
        covered += p.ns;
        s0 += p.ns;
    }
    if (covered != n) {
        KernelPlan z;
        bad("sub-launches do not cover the batch", z);
    }
}

static void check_bs(int k, int rows, uint64_t chunk, uint32_t n, bool in_place, bool gather, bool vand) {
    BsLaunch L{};
    L.vand = vand;
    const Layout ly = layout(in_place, chunk, k, rows);
    L.src = ly.src;
    L.dst = ly.dst;
    L.src_stripe_stride = ly.sss;
    L.dst_stripe_stride = ly.dss;
    static const uint64_t tab[1] = {0};
    if (gather) {
        L.stab = L.dtab = tab;
        L.sstride = L.dstride = uint32_t(k + rows);
    }
    L.k = k;
    L.rows = rows;
    L.len = chunk;
    L.n_stripes = n;
    uint64_t covered = 0;
    for (uint32_t s0 = 0; s0 < n;) {
        const KernelPlan p = plan_bs(L, s0);
        common(p, uint64_t(p.geo.tiles) * p.tpb * 2048);
        if (!p.ok || p.ns == 0) break;
        if (p.bt != uint32_t(kWaveBlock)) bad("bit-sliced kernels are one-wave blocks", p);
        if (knob(kKnobWpc) == kKnobUnset && p.lds_dynamic == 0) bad("bit-sliced launches are capped", p);
        if (knob(kKnobWpc) == kKnobUnset && p.lds_dynamic * bs_target_waves(p.win > 1, vand, gather, k, rows, p.geo.tiles) > kLdsPerCu)
            bad("bit-sliced wave cap reserves more than a CU's LDS", p);
        if (p.xcd && p.win > 1) bad("XCD runs on a windowed launch", p);
        if (knob(kKnobBsXcd) == kKnobUnset &&
            p.xcd != uint32_t(p.win <= 1 && p.geo.tiles <= (gather ? kBsXcdTiles : kBsXcdStridedTiles)))
            bad("XCD runs outside the rule (<= kBsXcdTiles / kBsXcdStridedTiles blocks per stripe)", p);
        if (p.tpb < 1 || uint64_t(p.geo.tiles) * p.tpb * 2048 < chunk) bad("tiles do not cover the chunk", p);
        if (uint64_t(p.geo.tiles - 1) * p.tpb * 2048 >= chunk) bad("a block with no tile", p);
        covered += p.ns;
        s0 += p.ns;
    }
    if (covered != n) {
        KernelPlan z;
        bad("sub-launches do not cover the batch", z);
    }
}

static void check_bm(int k, int rows, int w, uint64_t packet, uint32_t n, bool in_place, bool acc, bool gather) {
    BmLaunch L{};
    const Layout ly = layout(in_place, packet * uint64_t(w), k, rows);
    L.src = ly.src;
    L.dst = ly.dst;
    L.src_stripe_stride = ly.sss;
    L.dst_stripe_stride = ly.dss;
    static const uint64_t tab[1] = {0};
    if (gather) {
        L.stab = L.dtab = tab;
        L.sstride = L.dstride = uint32_t(k + rows);
        L.gshape = uint8_t(n % 3);
    }
    L.k = k;
    L.rows = rows;
    L.w = w;
    L.packet = packet;
    L.n_stripes = n;
    L.accumulate = acc;
    uint64_t covered = 0;
    for (uint32_t s0 = 0; s0 < n;) {
        const KernelPlan p = plan_bm(L, s0);
        common(p, uint64_t(w - 1) * packet + uint64_t(p.geo.units) * 4 * p.vw);
        if (!p.ok || p.ns == 0) break;
        if (p.rows > kMaxBmOut) bad("bitmatrix rows past 8", p);
        if (p.vw != 2 && p.vw != 4) bad("lane width", p);
        if (w > 4 && p.vw != 2) bad("w > 4 takes 8-byte lanes only", p);
        if (gather) {  // gathered: 8-byte lanes for w > 4, forced, or chunks of at most 4 KiB
            const int64_t e = knob(kKnobBmVw);
            const uint32_t want = w > 4 || e == 2 || (e == kKnobUnset && packet * uint64_t(w) <= 4096) ? 2u : 4u;
            if (p.vw != want) bad("gathered bm launches use the rule's lane width", p);
        }
        covered += p.ns;
        s0 += p.ns;
    }
    if (covered != n) {
        KernelPlan z;
        bad("sub-launches do not cover the batch", z);
    }
}

static void check_gather(int k, int rows, int w, uint64_t len, uint32_t n, uint32_t groups) {
    GatherLaunch L{};
    static const uint64_t tab[1] = {0};
    static const uint32_t desc[1] = {0};
    L.stab = L.dtab = tab;
    L.desc = desc;
    L.sstride = L.dstride = uint32_t(k + rows * groups);
    L.n_stripes = n;
    L.k = k;
    L.rows = rows;
    L.w = w;
    L.len = len;
    L.groups = groups;
    L.group_maps = 1;
    for (uint32_t s0 = 0; s0 < n;) {
        const KernelPlan p = w ? plan_bm_gather(L, s0) : plan_gf8_gather(L, s0);
        common(p, w ? uint64_t(w - 1) * len + uint64_t(p.geo.units) * 4 * p.vw : uint64_t(p.geo.units) * 16);
        if (!p.ok || p.ns == 0) break;
        if (!w && p.groups > 1 && p.rows != kMaxRows) bad("multi-group gathered gf8 launch with R != 4", p);
        if (!w && p.groups * uint32_t(kMaxRows) > uint32_t(kMaxSrc)) bad("gathered row groups past 32 rows", p);
        s0 += p.ns;
    }
}

// One pass over every launch shape under the current knobs.
static void sweep() {
    for (uint64_t chunk : kChunks)
        for (uint32_t n : kStripes) {
            if (chunk * n > (uint64_t(64) << 30)) continue;
            for (int k = 1; k <= kMaxK; k += (k < 12 ? 1 : 3))
                for (bool ip : {false, true})
                    for (bool vand : {false, true}) {
                        for (int rows = 1; rows <= kMaxRows && k + rows <= kMaxSrc; ++rows) {
                            check_gf8(k, rows, chunk, n, ip, vand, false, false, false);
                            check_gf8(k, rows, chunk, n, ip, vand, true, false, false);
                            if (!ip) check_gf8(k, rows, chunk, n, ip, vand, false, true, false);
                            check_gf8(k, rows, chunk, n, ip, vand, false, false, true);
                        }
                        if (chunk % 16 == 0)
                            for (int rows = kMaxRows + 1; k + rows <= kMaxSrc; ++rows) {
                                check_bs(k, rows, chunk, n, ip, (rows + int(vand)) % 2 == 0, vand);
                                check_mg(k, rows, chunk, n, ip, vand, false, false);
                                check_mg(k, rows, chunk, n, ip, vand, true, false);
                                check_mg(k, rows, chunk, n, ip, vand, false, true);
                            }
                    }
            for (int w = 1; w <= 8; ++w) {
                if (chunk % uint64_t(w)) continue;
                for (int k = 1; k <= kMaxK; k += (k < 8 ? 1 : 5))
                    for (int rows = 1; rows <= kMaxBmOut && k + rows <= kMaxSrc; ++rows)
                        for (bool ip : {false, true}) {
                            check_bm(k, rows, w, chunk / w, n, ip, false, false);
                            check_bm(k, rows, w, chunk / w, n, ip, true, false);
                            check_bm(k, rows, w, chunk / w, n, ip, false, true);
                        }
            }
            for (int k = 1; k <= kMaxK; k += 5) {
                for (int rows = 1; rows <= kMaxRows && k + rows <= kMaxSrc; ++rows) check_gather(k, rows, 0, chunk, n, 1);
                for (uint32_t g = 2; k + 4 * int(g) <= kMaxSrc + 3; ++g) check_gather(k, 4, 0, chunk, n, g);
                for (int w = 1; w <= 8; ++w)
                    for (int rows = 1; rows <= kBmGatherRows && k + rows <= kMaxSrc; ++rows)
                        if (chunk % uint64_t(w) == 0) check_gather(k, rows, w, chunk / w, n, 1);
            }
        }
    for (uint64_t len : {uint64_t(1), uint64_t(17), uint64_t(1) << 20, uint64_t(24) << 30, uint64_t(80) << 30}) {
        const KernelPlan p = plan_xor(len);
        common(p, uint64_t(p.bt) * 16);
    }
}

// Every accepted value of one knob (from its spec), plus unset.
static std::vector<std::string> values_of(const KnobSpec &s) {
    std::vector<std::string> v;
    if (s.nset) {
        for (int i = 0; i < s.nset; ++i) v.push_back(std::to_string(s.set[i]));
    } else {
        for (int64_t x = s.lo; x <= s.hi; x += s.step > 1 ? s.step : 1) v.push_back(std::to_string(x));
    }
    if (s.knob == kKnobSgroup) {  // with run lengths
        std::vector<std::string> r;
        for (const std::string &g : v)
            for (const char *run : {"", ":8", ":16", ":64", ":1024"}) r.push_back(g + run);
        v = r;
    }
    return v;
}

int main(int argc, char **argv) {
    const bool quick = argc > 1 && !std::strcmp(argv[1], "--quick");
    int nspec = 0;
    const KnobSpec *specs = knob_specs(nspec);
    g_ctx = "built-in rules";
    sweep();
    for (int i = 0; i < nspec; ++i) {
        const KnobSpec &s = specs[i];
        if (s.knob == kKnobCopyThreads) continue;  // host copy threads: no launch shape
        const std::vector<std::string> vals = values_of(s);
        for (size_t vi = 0; vi < vals.size(); ++vi) {
            // the whole sweep for the knobs that shape every launch, a
            // sample of values for the wide-range ones under --quick
            if (quick && vals.size() > 8 && vi % 4 != 0 && vi + 1 != vals.size()) continue;
            if (set_knob(s.name, vals[vi].c_str()) != KnobStatus::kOk) {
                std::printf("VIOLATION %s=%s refused but listed as accepted\n", s.name, vals[vi].c_str());
                return 1;
            }
            g_ctx = std::string(s.name) + "=" + vals[vi];
            sweep();
        }
        set_knob(s.name, nullptr);
    }
    // knob combinations the experiments use together
    const char *combos[][2][2] = {{{"MEC_MG_ROWS", "3"}, {"MEC_WPC", "32"}},
                                  {{"MEC_BLOCK", "256"}, {"MEC_WPC", "1"}},
                                  {{"MEC_BLOCK", "64"}, {"MEC_WINDOWS", "16"}},
                                  {{"MEC_GBLOCK", "64"}, {"MEC_GWPC", "1"}},
                                  {{"MEC_SGROUP", "64:1024"}, {"MEC_WINDOWS", "3"}}};
    for (auto &c : combos) {
        set_knob(c[0][0], c[0][1]);
        set_knob(c[1][0], c[1][1]);
        g_ctx = std::string(c[0][0]) + "=" + c[0][1] + " " + c[1][0] + "=" + c[1][1];
        sweep();
        set_knob(c[0][0], nullptr);
        set_knob(c[1][0], nullptr);
    }
    // values outside the accepted sets are refused
    const char *refused[][2] = {{"MEC_MG_ROWS", "5"}, {"MEC_MG_ROWS", "2"}, {"MEC_BLOCK", "128"}, {"MEC_WPC", "33"},
                                {"MEC_WPC", "-1"},   {"MEC_WINDOWS", "0"}, {"MEC_SGROUP", "4:7"}, {"MEC_SGROUP", "bad"},
                                {"MEC_BM_VW", "3"},  {"MEC_WIDE", "2"},    {"MEC_WPC", "12x"},
                                {"MEC_TILE_SKEW", "12"}, {"MEC_TILE_SKEW", "2048"}};
    for (auto &r : refused)
        if (set_knob(r[0], r[1]) != KnobStatus::kInvalid) {
            std::printf("VIOLATION %s=%s accepted\n", r[0], r[1]);
            return 1;
        }
    if (g_bad) {
        std::printf("FAILED %ld of %ld plans\n", g_bad, g_plans);
        return 1;
    }
    std::printf("ok %ld\n", g_plans);
    return 0;
}
