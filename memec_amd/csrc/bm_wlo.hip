// bm_wlo.hip — bitmatrix kernel instantiations, w = 1..4.
#include "bm_kernel.hpp"

namespace mec {
namespace detail {
MEC_BM_INSTANTIATE_W(1)
MEC_BM_INSTANTIATE_W(2)
MEC_BM_INSTANTIATE_W(3)
MEC_BM_INSTANTIATE_W(4)
}  // namespace detail
}  // namespace mec
