// gf8_r4lo.hip — GF(2^8) kernel instantiations with 4 output row(s), K = 1..16.
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
template <>
bool launch_gf8_wb<10, 4>(const KernelPlan &pl, Gf8Params<10, 4> p, int T, hipStream_t stream) {
    if (T != 2 && T != 4) return false;
    p.tiles = pl.geo.tiles / uint32_t(T);
    const dim3 grid(uint32_t(pl.grid / uint64_t(T))), block(kThreads);
    if (T == 2) hipLaunchKernelGGL((gf8_wb_kernel<10, 4, kGf8Dense, 2>), grid, block, pl.lds_dynamic, stream, p);
    else hipLaunchKernelGGL((gf8_wb_kernel<10, 4, kGf8Dense, 4>), grid, block, pl.lds_dynamic, stream, p);
    return true;
}
MEC_GF8_INSTANTIATE_LO(4)
}  // namespace detail
}  // namespace mec
