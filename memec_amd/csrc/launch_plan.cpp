// launch_plan.cpp — launch shapes of libmec's streaming kernels (see
// launch_plan.hpp).  Host code only: the rules below were each measured on
// the MI355X (the evidence is cited at each), and the plan_* functions
// assemble them per launch exactly as the launchers in gf8_kernel.hpp,
// bm_kernel.hpp, gather_kernel.hpp and kernels.hip use them.
#include "launch_plan.hpp"

#include <algorithm>
#include <cmath>

#include "knobs.hpp"

namespace mec {
namespace detail {

uint32_t stripe_group(uint64_t chunk, uint32_t tiles, uint32_t n_stripes, bool in_place, bool bitmatrix,
                      uint32_t &run) {
    const int64_t kg = knob(kKnobSgroup), kr = knob(kKnobSrun);  // experiments (mec_set_knob)
    run = 8;
    // chunks of 2 MiB or more: 16 stripes, runs of 8 tiles
    // (tools/sgroup_ab.py, profiles/r02/sgroup/; RS(10,4) split encode 2 MiB
    // 75.7 -> 78.8-80.0 %, 4 MiB 72.4 -> 77.2, 8 MiB 67.1 -> 79.2, 16 MiB
    // 57.4 -> 80.1; in-place decode 2 MiB 76.6 -> 78.5, 4 MiB 57.5 -> 76.0,
    // 8 MiB 59.0 -> 78.1); at 256 KiB-1 MiB every group costs 1-10 points.
    // Not for the bitmatrix kernel, whose lanes already read w packets a
    // packet apart: CRS(12,4) 2 MiB encode 76.4 -> 72.8 %, decode 72.2 ->
    // 68.7 with the same map (profiles/r02/sgroup/sgroup_ab_crs.log)
    (void)in_place;
    uint32_t g = (!bitmatrix && chunk >= (uint64_t(2) << 20)) ? 16u : 0u;
    if (kg != kKnobUnset) {
        g = uint32_t(std::max<int64_t>(kg, 0));
        if (kr != kKnobUnset) run = uint32_t(std::max<int64_t>(kr, 0));
    }
    if (g <= 1 || run == 0 || run % 8 != 0 || tiles % run != 0 || n_stripes < 2) return 0;
    return std::min(g, n_stripes);
}

uint32_t launch_windows(const void *src, int64_t src_span, const void *dst, int64_t dst_span) {
    const int64_t forced = knob(kKnobWindows);  // experiments (mec_set_knob)
    if (forced > 0) return uint32_t(forced);
    const int64_t a0 = int64_t(reinterpret_cast<uintptr_t>(src)), b0 = int64_t(reinterpret_cast<uintptr_t>(dst));
    const int64_t a1 = a0 + std::max<int64_t>(src_span, 0), b1 = b0 + std::max<int64_t>(dst_span, 0);
    return (b0 < a1 && a0 < b1) ? 2u : 1u;
}

uint32_t bm_windows(const void *src, int64_t src_span, const void *dst, int64_t dst_span, uint64_t chunk, int rows,
                    int k) {
    const uint32_t w = launch_windows(src, src_span, dst, dst_span);
    if (w <= 1 || knob(kKnobWindows) != kKnobUnset) return w;
    // tiny in-place stripes take the split-layout launch: identity order,
    // one-wave blocks, split caps (tools/bm_small_ab.py MEC_WINDOWS=1 arm,
    // profiles/r03/bm_small_win1_ab_{1,2}.log, two rounds): 1 KiB chunks
    // +2-16 points for every (k, m) tried, 2 KiB with <= 2 outputs and
    // k >= 8 +0.6-2.5; 2 KiB with 4 outputs or k <= 6 and 4 KiB lose 0.5-4
    const bool tiny = chunk <= 1024 || (chunk <= 2048 && rows <= 2 && k >= 8);
    return tiny ? 1u : w;
}

uint32_t block_threads(bool strided, uint32_t win, bool wave_in_place) {
    // gathered (pointer-table) launches are instantiated for kThreads only
    if (!strided) return uint32_t(kThreads);
    const int64_t forced = knob(kKnobBlock);  // experiments (mec_set_knob)
    if (forced == kWaveBlock || forced == kThreads) return uint32_t(forced);
    if (win == 1) return uint32_t(kWaveBlock);
    return wave_in_place ? uint32_t(kWaveBlock) : uint32_t(kThreads);
}

uint32_t gathered_block_threads(uint8_t gshape) {
    const int64_t e = knob(kKnobGblock);  // experiments (mec_set_knob)
    if (e != kKnobUnset) return e == kWaveBlock ? uint32_t(kWaveBlock) : uint32_t(kThreads);
    return gshape == 1 ? uint32_t(kWaveBlock) : uint32_t(kThreads);
}

namespace {
// Dynamic LDS per block so that about `waves` active waves share a CU (each
// block has `per` active waves); 0 when no LDS is left to reserve.
uint32_t lds_for_waves(uint32_t per, uint32_t static_lds, uint32_t waves) {
    constexpr uint32_t kGranule = 512;
    const uint32_t blocks = std::max<uint32_t>(1, (waves + per - 1) / per);
    const uint32_t per_block = kLdsPerCu / blocks / kGranule * kGranule;
    const uint32_t used = (static_lds + kGranule - 1) / kGranule * kGranule;
    return per_block > used + kGranule ? per_block - used - kGranule : 0;
}
uint32_t ceil_even(double x) { return 2u * uint32_t(std::ceil(x / 2.0)); }
uint32_t clampw(uint32_t w, uint32_t lo, uint32_t hi) { return std::min(hi, std::max(lo, w)); }
}  // namespace

uint32_t gathered_lds(uint32_t bt, uint32_t static_lds, uint8_t gshape) {
    const int64_t e = knob(kKnobGwpc);  // experiments (mec_set_knob)
    const int64_t w = e != kKnobUnset ? e : (gshape == 1 ? 16 : gshape == 2 ? 12 : 0);
    if (w <= 0) return 0;
    return lds_for_waves(std::max<uint32_t>(1, bt / 64), static_lds, uint32_t(w));
}

uint32_t gf8_target_waves(int k, int rows, bool in_place, bool dense, bool accumulate) {
    // read-modify-write of the outputs (delta updates, K = 1): each wave
    // also loads its R outputs; R = 2 / 3 / 4 want 16-18 / 12 / 10-12
    // waves (tools/bm_small_ab.py update, profiles/r02/gf8/update_caps.log:
    // RS(10,4)@1 MiB update 81.7 -> 84.1 %)
    if (accumulate && !in_place) return clampw(ceil_even(36.0 / std::max(1, rows)), 6, 20);
    const double w = 64.0 / std::max(1, k) + (in_place ? 2.0 : 1.0) * rows;
    // split layouts: a dense matrix (decode into separate output chunks,
    // ISA-L Cauchy encode) computes ~30 % longer per wave than the
    // Vandermonde encode, so it wants more waves to keep as many reads in
    // flight: ceil_even(64/K + 2R), at most 16, never below the split
    // count (tools/split_cap_ab.py, tools/split_rule_ab.py,
    // profiles/r03/gf8/split_*.log: RS(10,4)@1 MiB decode_split 80.3 ->
    // 83.5 %, (12,4)@64 KiB 75.4 -> 83.1, (16,4)@256 KiB 70.5 -> 80.0,
    // (20,4)@16 KiB 68.9 -> 80.6; 20 waves cost (4,2)@4 KiB 1.1-1.8)
    // Wide stripes with 4 output rows want more waves than 64/K + R gives,
    // since a wave's K x R products keep it computing longer: at least
    // ceil_even(K/2 + 1), at most 16 (tools/enc_cap_ab.py,
    // profiles/r03/gf8/enc_cap_ab.log, enc_rule_ab*.log: RS and ISA-L RS
    // (16,4)@256 KiB encode +1.0-1.9 points, (20,4)@16 KiB +4.0, (24,4)@64
    // KiB +5.1-5.8, (28,4)@4 KiB +4.1; k <= 12 unchanged).  Two rows lose
    // 1-3 points with the same floor ((18,2), (22,2), (30,2)), so they keep
    // the plain count.
    const uint32_t floor_wide = rows >= 4 ? std::min(ceil_even(0.5 * k + 1.0), 16u) : 0u;
    const uint32_t split = clampw(std::max(ceil_even(w), floor_wide), 6, 20);
    if (!in_place && dense)
        return std::max(split, std::min(ceil_even(64.0 / std::max(1, k) + 2.0 * rows), 16u));
    if (!in_place) return split;
    // a dense (decode) matrix keeps each wave busy longer than the
    // Vandermonde encode shortcut: at least 12 waves (RS(12,2) in-place
    // decode at 128-256 KiB chunks 71 -> 76 %, RS(14,2) +1-2 points;
    // profiles/r02/gf8/rs_inplace_ab.log, profiles/r02/wpc/wpc_pow2_strides.log)
    if (dense) return clampw(std::max(ceil_even(w), 12u), 8, 24);
    // the lighter Vandermonde encode in place wants the split count, 10..16
    // (RS(10,4)@1 MiB 76.7 -> 79.5 %, RS(6,2)@256 KiB 81 -> 86 %;
    // profiles/r02/gf8/rs104_valu_probe.log, rs_inplace_ab.log)
    return clampw(ceil_even(64.0 / std::max(1, k) + rows), 10, 16);
}

uint32_t bm_lane_bytes(int w, int rows, uint64_t chunk, bool in_place) {
    if (w > 4) return 8;
    const int64_t e = knob(kKnobBmVw);  // experiments (mec_set_knob)
    if (e != kKnobUnset) return e == 2 ? 8 : 16;
    if (!in_place) return 8;
    return (chunk <= (8u << 10) || (rows <= 2 && chunk <= (32u << 10))) ? 8 : 16;
}

uint32_t bm_target_waves(int rows, int w, int vw, bool in_place) {
    // more than 4 outputs (wide codes): no cap — such a wave keeps rows x w
    // packet slices and computes long enough that the caps below starve the
    // stream (Cauchy(10,6)@64 KiB encode 74.6 -> 79.3 %, its in-place
    // decode unchanged, Cauchy(8,5)@16 KiB +2.8, Cauchy(20,8) equal;
    // tools/wide_ab.py, profiles/r04/wide/bm_wpc_ab*.jsonl)
    if (rows > 4) return 0;
    // w > 4 always runs 8-byte slices of twice as many packets: the
    // 16-byte rule's bytes in flight per wave
    if (vw >= 4 || w > 4) return clampw(uint32_t(3 * rows), 6, 16);
    return in_place ? clampw(uint32_t(6 * rows), 6, 12) : clampw(uint32_t(6 * rows), 6, 16);
}

uint32_t occupancy_lds(uint32_t bt, uint32_t active, uint32_t static_lds, uint32_t waves) {
    const int64_t e = knob(kKnobWpc);  // experiments (mec_set_knob)
    const bool forced = e != kKnobUnset;
    if (forced) waves = uint32_t(std::max<int64_t>(0, e));
    // a block with less than one wave's worth of units streams too little
    // per wave for a cap to pay (CRS at 2 KiB chunks: 75 % uncapped, 51 %
    // capped, profiles/r02/sweep)
    if (waves == 0 || (!forced && active < 64)) return 0;
    const uint32_t act = std::min(bt, std::max<uint32_t>(active, 1));
    return lds_for_waves(std::max<uint32_t>(1, (act + 63) / 64), static_lds, waves);
}

int gf8_structure(const Gf8Coef (*coef)[kMaxSrc], int k, int rows) {
    const uint32_t one = 0x03020100u;  // t0 of coefficient 1 (identity on bits 0-2)
    bool vand = true;
    for (int j = 0; j < k && vand; ++j) vand = coef[0][j].t0 == one;
    for (int i = 0; i < rows && vand; ++i) vand = coef[i][0].t0 == one;
    return vand ? kGf8Vand : kGf8Dense;
}

int mg_group_rows(int rows, int k, bool vand) {
    const int R = gf8_mg_rows(rows, k, vand);
    const int64_t kr = knob(kKnobMgRows);  // experiments (mec_set_knob)
    const bool made = kr == 3 || kr == 4 || (kr == 8 && k >= kMg8MinK && k <= kMg8MaxK);
    // the forced count only where its groups fit the kernel's kMaxSrc
    // output slots: 31 rows in groups of 3 would be 11 groups, 33 slots
    // (round 4: gf8_mg_kernel read dst_off[32] past its kernel arguments)
    if (made && (rows + int(kr) - 1) / int(kr) * int(kr) <= kMaxSrc) return int(kr);
    return R;
}

namespace {
bool fail_plan(KernelPlan &p, const char *why) {
    p.ok = false;
    p.why = why;
    return false;
}
// The checks every launch shares: block size, LDS, grid, 32-bit offsets.
bool common_ok(KernelPlan &p, uint64_t lane_span_bytes) {
    if (p.bt != uint32_t(kWaveBlock) && p.bt != uint32_t(kThreads)) return fail_plan(p, "block size not instantiated");
    if (uint64_t(p.lds_static) + p.lds_dynamic > kLdsPerCu) return fail_plan(p, "LDS over 160 KiB per block");
    if (p.grid == 0 || p.grid > (uint64_t(1) << 31) / p.bt) return fail_plan(p, "grid past 2^31 work-items");
    if (lane_span_bytes > (uint64_t(1) << 32)) return fail_plan(p, "lane offsets past 32 bits");
    if (p.win < 1) return fail_plan(p, "no block window");
    if (p.sgroup != 0 && (p.srun == 0 || p.srun % 8 != 0 || p.geo.tiles % p.srun != 0))
        return fail_plan(p, "stripe-group run does not tile the stripe");
    p.ok = true;
    p.why = "";
    return true;
}
uint32_t sub_stripes(const Geometry &g, uint32_t n, uint32_t s0) { return std::min(n - s0, g.max_stripes_per_launch); }
// Per-stripe tile rotation of identity-map strided launches
// (stream_common.hpp stripe_tile): in place, kTileSkew tiles; split
// layouts none.  MEC_TILE_SKEW=<n> forces n (0 = none) on either.
uint32_t tile_skew(bool in_place, uint32_t sgroup, uint32_t tiles) {
    const int64_t k = knob(kKnobTileSkew);
    const int64_t v = k != kKnobUnset ? k : in_place ? kTileSkew : 0;
    if (sgroup != 0 || v <= 0 || tiles == 0) return 0;
    return uint32_t(uint64_t(v) % tiles);
}
}  // namespace

KernelPlan plan_gf8(const Gf8Launch &L, uint32_t s0) {
    KernelPlan p;
    p.k = L.k;
    p.rows = L.rows;
    if (L.k < 1 || L.k > kMaxK || L.rows < 1 || L.rows > kMaxRows) return fail_plan(p, "K or R not instantiated"), p;
    if (L.len / 16 > uint64_t(UINT32_MAX)) return fail_plan(p, "chunk too large"), p;
    // block size from the whole launch's layout (sub-launches share it)
    // one-wave blocks in place for stripe strides under kWaveBlockSpan,
    // except strides of exactly 512 KiB and 1 MiB: there one-wave blocks
    // decode at 62-71 % of 8 TB/s and 4-wave blocks at 77-82 %
    // (tools/wpc_ab.py WPC_VAR=MEC_BLOCK, profiles/r02/wpc/win_pow2.log);
    // other powers of two favour one-wave blocks like any stride (16 KiB:
    // 69 -> 82 %, 2 MiB / 4 MiB +1-4; profiles/r02/gf8/rs_inplace_ab.log)
    const int64_t sss = L.src_stripe_stride;
    const bool wave_ok = sss >= 0 && sss < kWaveBlockSpan && sss != (int64_t(512) << 10) && sss != (int64_t(1) << 20);
    p.bt = L.stab ? gathered_block_threads(L.gshape)
                  : block_threads(true, launch_windows(L.src, int64_t(L.n_stripes) * L.src_stripe_stride, L.dst,
                                                       int64_t(L.n_stripes) * L.dst_stripe_stride),
                                  wave_ok);
    // one-wave one-map gathered blocks take two units per lane (a 2 KiB
    // tile, one pointer-row fetch per 2 KiB of every chunk) where a wave's
    // 1 KiB per chunk is at most 6 KiB (k + rows <= 6) and the tiles are
    // whole (no lane past the chunk).  Interleaved A/B at 4 KiB-64 KiB
    // (tools/wide_ab.py, profiles/r06/batch/gu_ab_r06s.jsonl,
    // gu_sweep_r06s.jsonl): RS(2,2) 66 -> 78 %, RS(3,2) 72 -> 76, RS(4,1)
    // 76 -> 82, RS(4,2) 75-78 -> 80-82; at 7 KiB and more per wave it
    // loses (RS(5,2), RS(4,3), RS(4,4) 0-3 points, RS(8,2) / RS(10,4)
    // 4-15).  MEC_GU=1|2 forces it.
    const int64_t gk = L.stab && p.bt == uint32_t(kWaveBlock) ? knob(kKnobGu) : int64_t(1);
    const bool gu_rule = L.stab && p.bt == uint32_t(kWaveBlock) && L.k + L.rows <= 6;
    p.gu = (gk == 2 || (gk == kKnobUnset && gu_rule)) && (L.len / 16) % (2 * kWaveBlock) == 0 ? 2u : 1u;
    p.geo = geometry(L.len / 16, p.bt * p.gu);
    p.ns = sub_stripes(p.geo, L.n_stripes, s0);
    p.grid = uint64_t(p.ns) * p.geo.tiles;
    p.lds_static = gf8_static_lds(L.k, L.rows);
    const bool vand = gf8_structure(L.coef, L.k, L.rows) == kGf8Vand;
    p.structure = vand ? kGf8Vand : kGf8Dense;
    if (L.stab) {
        p.lds_dynamic = gathered_lds(p.bt, uint32_t(L.rows * L.k * 32), L.gshape);
        // block windows (the in-place layouts' block order, §4.3) for
        // decode batches — outputs addressed through the sources' own rows —
        // of <= 2 outputs on <= 4 KiB chunks: one-map RS(8,2)@4 KiB decode
        // batches 74.5-76.2 -> 78.7-80.8 % of 8 TB/s at 65536 and 262144
        // stripes; RS(4,2) and ISA-L RS(6,3) at 4 KiB within +-1 point, and
        // more outputs or larger chunks lose (RS(10,4)@1 MiB -3)
        // (tools/wide_ab.py, profiles/r06/batch/gwin_ab_r06s.jsonl).
        // MEC_WINDOWS=<n> forces n.
        const int64_t wk = knob(kKnobWindows);
        const bool dec_rows = L.stab == L.dtab && L.sstride == L.dstride;
        p.win = wk != kKnobUnset ? uint32_t(wk) : dec_rows && L.rows <= 2 && L.len <= 4096 ? 2u : 1u;
        // XCD runs (A/B, MEC_GXCD; default off until measured)
        const int64_t xk = knob(kKnobGxcd);
        p.xcd = xk == 1 ? 1u : 0u;
    } else {
        const uint8_t *src = L.src + int64_t(s0) * L.src_stripe_stride;
        const uint8_t *dst = L.dst + int64_t(s0) * L.dst_stripe_stride;
        p.win = launch_windows(src, int64_t(p.ns) * L.src_stripe_stride, dst, int64_t(p.ns) * L.dst_stripe_stride);
        p.sgroup = stripe_group(L.len, p.geo.tiles, p.win > 1 ? p.ns / p.win : p.ns, p.win > 1, false, p.srun);
        p.skew = tile_skew(p.win > 1, p.sgroup, p.geo.tiles);
        const bool in_place = p.win > 1;
        p.lds_dynamic = occupancy_lds(p.bt, p.bt, uint32_t(L.rows * L.k * 32),
                                      gf8_target_waves(L.k, L.rows, in_place, !vand, L.accumulate));
        if (L.probe) p.structure = kGf8Xor;
    }
    common_ok(p, uint64_t(p.geo.units) * 16);
    return p;
}

KernelPlan plan_gf8_mg(const Gf8MgLaunch &L, uint32_t s0) {
    KernelPlan p;
    const int R = L.group_rows;
    p.k = L.k;
    p.rows = R;
    p.structure = L.vand ? kGf8Vand : kGf8Dense;
    if (L.k < 1 || L.k > kMaxK) return fail_plan(p, "K not instantiated"), p;
    if (L.rows <= kMaxRows || L.rows > kMaxSrc) return fail_plan(p, "one-pass launches take 5..32 rows"), p;
    if (R == 8 ? (L.k < kMg8MinK || L.k > kMg8MaxK) : (R != 3 && R != 4))
        return fail_plan(p, "rows per group not instantiated for this K"), p;
    if (!L.tabs || L.len % 16) return fail_plan(p, "no tables, or a chunk with a tail"), p;
    if (L.len / 16 > uint64_t(UINT32_MAX)) return fail_plan(p, "chunk too large"), p;
    p.groups = uint32_t((L.rows + R - 1) / R);
    if (p.groups * uint32_t(R) > uint32_t(kMaxSrc)) return fail_plan(p, "row groups past the kernel's 32 output slots"), p;
    p.bt = kWaveBlock;
    p.geo = geometry(L.len / 16, kWaveBlock);
    p.ns = sub_stripes(p.geo, L.n_stripes, s0);
    p.grid = uint64_t(p.ns) * p.geo.tiles;
    if (!L.stab) {
        const uint8_t *src = L.src + int64_t(s0) * L.src_stripe_stride;
        const uint8_t *dst = L.dst + int64_t(s0) * L.dst_stripe_stride;
        p.win = launch_windows(src, int64_t(p.ns) * L.src_stripe_stride, dst, int64_t(p.ns) * L.dst_stripe_stride);
        p.sgroup = stripe_group(L.len, p.geo.tiles, p.win > 1 ? p.ns / p.win : p.ns, p.win > 1, false, p.srun);
        p.skew = tile_skew(p.win > 1, p.sgroup, p.geo.tiles);
    }
    // the tables are the block's LDS, and no wave cap: the caps of the
    // <= 4-row launches (gf8_target_waves) starve these longer-computing
    // waves — uncapped, RS(10,6)@256 KiB 67.2 -> 72.3 %, RS(8,5)@16 KiB
    // 63.6 -> 66.5, ISA-L RS(12,8) 65.8 -> 67.2, the rest within 0.3
    // (tools/wide_ab.py, profiles/r04/wide/mg_wpc_ab*.jsonl); MEC_WPC
    // still forces one (experiments)
    const uint32_t tab_bytes = p.groups * uint32_t(R) * uint32_t(L.k) * 32;
    p.lds_dynamic = std::max(occupancy_lds(kWaveBlock, kWaveBlock, 0, 0), tab_bytes);
    common_ok(p, uint64_t(p.geo.units) * 16);
    return p;
}

KernelPlan plan_bm(const BmLaunch &L, uint32_t s0) {
    KernelPlan p;
    p.k = L.k;
    p.rows = L.rows;
    if (L.k < 1 || L.k > kMaxK || L.rows < 1 || L.rows > kMaxBmOut || L.w < 1 || L.w > 8)
        return fail_plan(p, "K, R or w not instantiated"), p;
    const uint64_t cb = L.packet * uint64_t(L.w);
    if (cb > uint64_t(UINT32_MAX)) return fail_plan(p, "chunk too large"), p;
    const int R = L.rows;
    // lane width: 8 bytes for w > 4 and gathered launches' default, else
    // bm_lane_bytes (strided)
    p.vw = L.w <= 4 ? 4 : 2;
    if (p.vw == 4 && !L.stab) {
        const bool in_place = bm_windows(L.src, int64_t(L.n_stripes) * L.src_stripe_stride, L.dst,
                                         int64_t(L.n_stripes) * L.dst_stripe_stride, cb, R, L.k) > 1;
        if (bm_lane_bytes(L.w, R, cb, in_place) == 8) p.vw = 2;
    } else if (p.vw == 4) {
        // gathered: 8-byte lanes on chunks of at most 4 KiB (CRS(4,2)@4 KiB
        // batches 73.4-73.7 -> 75.2-76.4 %, CRS(8,2) 72.6-72.9 -> 73.5-73.7,
        // CRS(4,2) decode batches +0.5-1; CRS(12,4)@64 KiB encode batches
        // lose 1 point with them, so larger chunks keep 16 bytes;
        // tools/wide_ab.py, profiles/r06/batch/bm_vw_ab_r06s.jsonl).
        // MEC_BM_VW=2|4 forces either.
        const int64_t e = knob(kKnobBmVw);
        if (e == 2 || (e == kKnobUnset && cb <= 4096)) p.vw = 2;
    }
    // gathered: aligned chunks keep the default shape (one-wave blocks cost
    // the bitmatrix kernel 3.5 % on aligned decode batches), unaligned ones
    // take the capped 4-wave shape (+1-3 %; profiles/r02/host/gather_ab_bm.log);
    // aligned chunks of at most 4 KiB take one-wave blocks, 16 waves per CU,
    // as the byte-wise gathered kernels do (with 8-byte lanes: CRS(8,2)@4 KiB
    // batches 73.2-74.0 -> 77.4 %, CRS(4,2) decode batches 68.3 -> 72.6;
    // tools/wide_ab.py, profiles/r06/batch/bm_gb_ab_r06s.jsonl)
    const uint8_t gshape = L.gshape == 1 && cb > 4096 ? 0 : L.gshape;
    // one-wave blocks in place: chunks of kBmWaveChunk or more, and
    // 16-32 KiB chunks with <= 2 output rows and k >= 6 (8-byte lanes, 12
    // waves per CU; CRS(6,2) / (8,2) / (12,2) in place +1-5 points,
    // CRS(4,2), CRS(12,4), 8 KiB and >= 64 KiB chunks lose;
    // profiles/r02/bmshape/)
    const bool wave_ip = cb >= kBmWaveChunk || (R <= 2 && L.k >= 6 && cb >= (16u << 10) && cb <= (32u << 10));
    p.bt = L.stab ? gathered_block_threads(gshape)
                  : block_threads(true, bm_windows(L.src, int64_t(L.n_stripes) * L.src_stripe_stride, L.dst,
                                                   int64_t(L.n_stripes) * L.dst_stripe_stride, cb, R, L.k),
                                  wave_ip);
    const uint32_t ub = 4 * p.vw;
    p.geo = geometry(L.packet / ub, p.bt);
    p.ns = sub_stripes(p.geo, L.n_stripes, s0);
    p.grid = uint64_t(p.ns) * p.geo.tiles;
    if (L.stab) {
        p.lds_dynamic = gathered_lds(p.bt, 0, gshape);
    } else {
        const uint8_t *src = L.src + int64_t(s0) * L.src_stripe_stride;
        const uint8_t *dst = L.dst + int64_t(s0) * L.dst_stripe_stride;
        p.win = bm_windows(src, int64_t(p.ns) * L.src_stripe_stride, dst, int64_t(p.ns) * L.dst_stripe_stride, cb, R, L.k);
        p.sgroup = stripe_group(cb, p.geo.tiles, p.win > 1 ? p.ns / p.win : p.ns, p.win > 1, true, p.srun);
        p.skew = tile_skew(p.win > 1, p.sgroup, p.geo.tiles);
        const bool in_place = p.win > 1;
        p.lds_dynamic = occupancy_lds(p.bt, std::min<uint32_t>(p.bt, p.geo.units), 0,
                                      bm_target_waves(R, L.w, int(p.vw), in_place));
    }
    // the last packet's lane slices end inside the chunk: (w - 1) packets
    // plus one packet's units
    common_ok(p, uint64_t(L.w - 1) * L.packet + uint64_t(p.geo.units) * ub);
    return p;
}

KernelPlan plan_gf8_gather(const GatherLaunch &L, uint32_t s0) {
    KernelPlan p;
    p.k = L.k;
    p.rows = L.rows;
    p.groups = L.groups ? L.groups : 1u;
    if (L.k < 1 || L.k > kMaxK || L.rows < 1 || L.rows > kMaxRows || !L.stab || !L.dtab || !L.desc)
        return fail_plan(p, "K or R not instantiated, or no tables"), p;
    if (p.groups > 1 && L.rows != kMaxRows) return fail_plan(p, "multi-group gathered launches run 4 rows per group"), p;
    if (p.groups * uint32_t(kMaxRows) > uint32_t(kMaxSrc)) return fail_plan(p, "more row groups than outputs"), p;
    if (L.len / 16 > uint64_t(UINT32_MAX)) return fail_plan(p, "chunk too large"), p;
    p.bt = kThreads;
    p.geo = geometry(L.len / 16);
    p.ns = sub_stripes(p.geo, L.n_stripes, s0);
    p.grid = uint64_t(p.ns) * p.geo.tiles;
    p.lds_static = gf8_gather_static_lds(L.k, L.rows);
    common_ok(p, uint64_t(p.geo.units) * 16);
    return p;
}

KernelPlan plan_bm_gather(const GatherLaunch &L, uint32_t s0) {
    KernelPlan p;
    p.k = L.k;
    p.rows = L.rows;
    if (L.k < 1 || L.k > kMaxK || L.rows < 1 || L.rows > kBmGatherRows || L.w < 1 || L.w > 8 || !L.stab ||
        !L.dtab || !L.desc)
        return fail_plan(p, "K, R or w not instantiated, or no tables"), p;
    const uint64_t cb = L.len * uint64_t(L.w);
    if (cb > uint64_t(UINT32_MAX)) return fail_plan(p, "chunk too large"), p;
    p.vw = L.w <= 4 ? 4 : 2;
    p.bt = kThreads;
    p.geo = geometry(L.len / (4 * p.vw));
    p.ns = sub_stripes(p.geo, L.n_stripes, s0);
    p.grid = uint64_t(p.ns) * p.geo.tiles;
    p.lds_static = bm_gather_static_lds(L.w, L.rows);
    common_ok(p, uint64_t(L.w - 1) * L.len + uint64_t(p.geo.units) * 4 * p.vw);
    return p;
}

uint32_t bs_target_waves(bool in_place, bool vand, bool gather, int k, int rows, uint32_t tiles) {
    // A strided bit-sliced wave streams 2 KiB of every one of its 13-28
    // chunks (32-56 KiB), 4 sources ahead; uncapped, the VGPR budget puts 12
    // such waves on a CU and the memory side queues them into lower
    // throughput (RS(16,8)@64 KiB encode 71.6-73.8 % of 8 TB/s).  Capped
    // (tools/wide_ab.py bsw<n> arms, three rounds on two boxes,
    // profiles/r05/wide_cap_box8.jsonl, wide_cap_box9.jsonl): split
    // Vandermonde encodes run best at 5 waves per CU (RS(16,8) 79.6-80.1,
    // RS(10,6)@256 KiB 78.9-79.9, RS(8,5)@16 KiB 82.8-83.4, RS(4,12)@1 MiB
    // 81.8, ISA-L RS(12,8) 80.1-80.7), split dense ones at 6 (ISA-L
    // Cauchy(12,6) 80.6-80.7, 69 at 5; Cauchy(20,8)@4 KiB 69.2-69.9 and
    // (4,12) 75.2-76.2 would take 5 but the cliff of (12,6) rules it out),
    // in-place decodes at 8 (RS(10,6) 78.7 against 74.5 uncapped and 58 at
    // 4-5; RS(16,8) 77.9-78.2 against 77.1).  Gathered launches at 6 once
    // their pointer row is one vector load and each XCD takes a run of
    // stripes (bitslice.hpp vrow / xcd): RS(16,8) batch 79.1-81.7, ISA-L
    // RS(12,8) 80.7-80.8, RS(10,6)@256 KiB 76.1-79.4, the 8-erasure batch
    // decode 78.7-78.8, at 5 waves 1.5-5 points lower
    // (profiles/r05/vrow/vrow_cap_ab_box14.jsonl); with a scalar load per entry the
    // compiler waited on each, and any cap cost them 10-37 points.  MEC_WPC
    // overrides.  In-place decodes of >= 8 erasures on <= 64 KiB chunks take
    // 6 too: RS(16,8)@64 KiB 78.2 -> 79.8-80.0, ISA-L RS(12,8) 78.5 -> 80.6,
    // RS(16,8)@4 KiB 70.9 -> 73.2, while 6-erasure decodes lose 4-5 points at
    // 6 (RS(10,6), ISA-L Cauchy(12,6)) and so does RS(4,12)@1 MiB's decode
    // of 12 (profiles/r05/vrow/ipcap_ab_box20.jsonl, vrow_cap_ab_box14.jsonl).
    //
    // Round 6: split dense launches by the bytes a
    // wave keeps in flight — 2 KiB of each of the (at most 4) sources it
    // loads ahead plus 2 KiB of each output — against kBsInflightKiB per
    // CU: (12,6) 20 KiB and (20,8) 24 KiB keep 6 waves, (4,12) 32 KiB takes
    // 4.  Interleaved A/B, one box (profiles/r06/wide/wcap_r06d.jsonl; % of
    // 8 TB/s at 4 / 5 / 6 waves, default): ISA-L Cauchy(4,12)@1 MiB 78.8 /
    // 78.7 / 75.2 (round-5 rule 74.4-74.7); Cauchy(12,6)@64 KiB 68.8 / 68.9 /
    // 81.9; Cauchy(20,8)@4 KiB 74.0 / 73.7 / 75.5.
    if (gather) return 6;
    if (in_place) return rows >= 8 && tiles <= kBsXcdTiles ? 6 : 8;
    if (vand) return 5;
    const uint32_t kib = 2u * uint32_t(std::min(k, 4) + rows);
    return clampw(kBsInflightKiB / kib, 4, 6);
}

uint32_t bs_gather_tpb() {
    const int64_t kt = knob(kKnobBsTpb);
    return kt != kKnobUnset && kt > 0 ? uint32_t(kt) : 1u;
}

KernelPlan plan_bs(const BsLaunch &L, uint32_t s0) {
    KernelPlan p;
    p.k = L.k;
    p.rows = L.rows;
    if (L.k < 1 || L.rows <= kMaxRows || L.k + L.rows > kMaxSrc) return fail_plan(p, "bit-sliced launches take 5..31 rows"), p;
    if (L.len == 0 || L.len % 16 || L.len > (uint64_t(1) << 32) - 2048) return fail_plan(p, "chunk size"), p;
    p.bt = kWaveBlock;
    // 2 KiB tiles (each lane two 16-byte units 1 KiB apart), tpb of them
    // per block.  Strided blocks take one; gathered ones the count their
    // kernel was built for (jit.cpp: 1, straight-line like the strided
    // kernel, unless MEC_BS_TPB asks for a loop over several tiles per
    // pointer-row read — which measured slower, §4.7).
    const uint32_t tiles = uint32_t((L.len + 2047) / 2048);
    p.tpb = !L.stab ? 1u : L.tpb ? L.tpb : bs_gather_tpb();
    p.tpb = std::min(p.tpb, tiles);
    p.geo.units = uint32_t(L.len / 16);
    p.geo.tiles = (tiles + p.tpb - 1) / p.tpb;
    p.geo.max_stripes_per_launch = std::max<uint32_t>(1, uint32_t(((uint64_t(1) << 31) / kWaveBlock) / p.geo.tiles));
    p.ns = sub_stripes(p.geo, L.n_stripes, s0);
    p.grid = uint64_t(p.ns) * p.geo.tiles;
    if (!L.stab) {
        const uint8_t *src = L.src + int64_t(s0) * L.src_stripe_stride;
        const uint8_t *dst = L.dst + int64_t(s0) * L.dst_stripe_stride;
        p.win = launch_windows(src, int64_t(p.ns) * L.src_stripe_stride, dst, int64_t(p.ns) * L.dst_stripe_stride);
    }
    p.lds_dynamic = occupancy_lds(kWaveBlock, kWaveBlock, 0,
                                  bs_target_waves(p.win > 1, L.vand, L.stab != nullptr, L.k, L.rows, p.geo.tiles));
    // XCD runs: blocks are dealt round-robin over the 8 XCDs, so a stripe's
    // blocks land on all eight and each XCD's L2 fetches its pointer row.
    // Gathered launches of <= kBsXcdTiles blocks per stripe give each XCD a
    // contiguous run instead (three boxes, profiles/r05/vrow/: the 8-erasure
    // RS(16,8)@64 KiB batch decode +2.1-3.2 points, RS(16,8) batch encode
    // +1.2 on average, ISA-L RS(12,8) -0.4); with more tiles per stripe the
    // row is already shared (RS(10,6)@256 KiB -1.2 to -4.5).  Strided
    // launches take them only at <= kBsXcdStridedTiles blocks per stripe
    // (4 KiB chunks: ISA-L Cauchy(20,8) 69.4-71.0 -> 78.0-78.7; at 64 KiB
    // -2 to +1, at 256 KiB - 1 MiB -4.5 to -7).  MEC_BS_XCD forces it
    // either way (never on windowed in-place launches).
    const int64_t xk = knob(kKnobBsXcd);
    const uint32_t xt = L.stab ? kBsXcdTiles : kBsXcdStridedTiles;
    p.xcd = p.win > 1 ? 0u : xk != kKnobUnset ? uint32_t(xk != 0) : uint32_t(p.geo.tiles <= xt);
    common_ok(p, uint64_t(p.geo.tiles) * p.tpb * 2048);
    return p;
}

KernelPlan plan_xor(uint64_t len) {
    KernelPlan p;
    // one-wave blocks over 1 KiB tiles unless MEC_BLOCK=256, like the
    // split-layout coding launches; 2 source streams + 1 output per lane:
    // the gf8 split-layout cap
    p.bt = block_threads(true, 1, false);
    const uint64_t units = (len + 15) / 16, blocks = (units + p.bt - 1) / p.bt;
    p.lds_dynamic = occupancy_lds(p.bt, p.bt, 0, gf8_target_waves(2, 1, false, false, false));
    p.grid = std::max<uint64_t>(1, std::min<uint64_t>({blocks, uint64_t(1) << 24, (uint64_t(1) << 31) / p.bt}));
    p.ns = 1;
    // grid-stride past 16 GiB: each block's span is one buffer resource
    common_ok(p, uint64_t(p.bt) * 16);
    return p;
}

}  // namespace detail
}  // namespace mec
