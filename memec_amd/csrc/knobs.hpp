// knobs.hpp — launch-shape experiment overrides.
//
// Each knob is read from its environment variable ONCE (first use, a C++11
// thread-safe static) and held in an atomic; mec_set_knob() changes it at
// run time.  No launch path calls getenv, so the library never races a
// caller's setenv/putenv, and an experiment flips a knob between launches
// through the API instead of the environment.
//
// Every value is validated where it enters (knob_spec): a value outside a
// knob's accepted set is refused by mec_set_knob (MEC_EINVAL) and ignored,
// with a warning, when it comes from the environment, so a launch never sees
// it.  Combinations that depend on the launch (MEC_MG_ROWS against the row
// count, wave caps against the LDS a block already uses) are resolved by the
// launch planner (launch_plan.cpp), which falls back to the built-in rule
// rather than issue a launch outside its invariants.
#pragma once

#include <cstdint>

namespace mec {
namespace detail {

enum Knob : int {
    kKnobSgroup = 0,  // MEC_SGROUP=<group>[:<run>]
    kKnobSrun,        //   ... its run length
    kKnobWindows,     // MEC_WINDOWS=<n>
    kKnobBlock,       // MEC_BLOCK=64|256
    kKnobGblock,      // MEC_GBLOCK=64|256
    kKnobGwpc,        // MEC_GWPC=<waves> (0 = no cap)
    kKnobBmVw,        // MEC_BM_VW=2|4
    kKnobWpc,         // MEC_WPC=<waves> (0 = no cap)
    kKnobCopyThreads, // MEC_COPY_THREADS=<n>
    kKnobWide,        // MEC_WIDE=0: > 4 outputs as 4-row launches (A/B of gf8_mg_kernel)
    kKnobMgRows,      // MEC_MG_ROWS=3|4|8: rows per group of gf8_mg_kernel
    kKnobBitslice,    // MEC_BITSLICE=0|1|2|3: wide codes' run-time compiled kernels off / async (default) / sync / sync, every wide launch
    kKnobBsWaves,     // MEC_BS_WAVES=<n>: those kernels compiled for at least n waves per SIMD (0 = compiler's choice)
    kKnobBsPrefetch,  // MEC_BS_PREFETCH=<n>: ... with at most n sources' loads ahead of the combine (unset: 4; 0 = all first)
    kKnobBsTpb,       // MEC_BS_TPB=<n>: 2 KiB tiles per block of the gathered ones (0 = rule: 1, straight-line)
    kKnobTileSkew,    // MEC_TILE_SKEW=<tiles>: strided identity-map launches rotate stripe s's tiles by s * n (0 = none; unset = rule)
    kKnobBsFence,     // MEC_BS_FENCE=0|1: bit-sliced kernels compiled with scheduling fences between sources (unset: gathered ones)
    kKnobBsXcd,       // MEC_BS_XCD=0|1: bit-sliced launches deal each XCD a contiguous run of stripes (unset: rule, plan_bs)
    kKnobBsVrow,      // MEC_BS_VROW=0|1: gathered ones fetch the pointer row in one vector load (unset: rule, 1) or per entry
    kKnobWbatch,      // MEC_WBATCH=0|2|4: in-place dense RS(10,4)-shaped decodes write T tiles' outputs per block in one burst (A/B, gf8_wb_kernel)
    kKnobTabWait,     // MEC_TAB_WAIT=0|1: a device batch's launch waits for its pointer-table copy on the device (0) or, while its stream is busy, on the host (1; unset: rule, 1)
    kKnobGxcd,        // MEC_GXCD=0|1: one-map gathered gf8 launches deal each XCD a contiguous run of blocks (unset: rule, plan_gf8)
    kKnobGu,          // MEC_GU=1|2: 16-byte units per lane of one-wave one-map gathered gf8 launches (unset: rule, plan_gf8: 2 for k + rows <= 6)
    kKnobCount
};
constexpr int64_t kKnobUnset = INT64_MIN;

// Accepted values of one knob: lo..hi in steps of `step` (0 = 1), and when
// `set` is non-empty only the values it lists.
struct KnobSpec {
    const char *name;  // environment variable
    Knob knob;
    int64_t lo, hi;
    int64_t set[4];
    int nset;
    int64_t step;
};
// The table (knobs.cpp); MEC_SGROUP's run half is checked with it.
const KnobSpec *knob_specs(int &n);
// Accepted range of MEC_SGROUP's run (a multiple of 8).
constexpr int64_t kSrunMax = 1024;

// Current value, or kKnobUnset.
int64_t knob(Knob k);
// name: the environment variable's name ("MEC_WPC", ...); value: the same
// syntax as the variable, NULL = unset.
enum class KnobStatus { kOk, kUnknown, kInvalid };
KnobStatus set_knob(const char *name, const char *value);

}  // namespace detail
}  // namespace mec
