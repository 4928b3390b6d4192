// gbm.hip — gathered bitmatrix kernel instantiations, w = 1..8.
#include "gather_kernel.hpp"

namespace mec {
namespace detail {
MEC_GBM_INSTANTIATE_W(1)
MEC_GBM_INSTANTIATE_W(2)
MEC_GBM_INSTANTIATE_W(3)
MEC_GBM_INSTANTIATE_W(4)
MEC_GBM_INSTANTIATE_W(5)
MEC_GBM_INSTANTIATE_W(6)
MEC_GBM_INSTANTIATE_W(7)
MEC_GBM_INSTANTIATE_W(8)
}  // namespace detail
}  // namespace mec
