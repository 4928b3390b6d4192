// bm_whi.hip — bitmatrix kernel instantiations, w = 5..8.
#include "bm_kernel.hpp"

namespace mec {
namespace detail {
MEC_BM_INSTANTIATE_W(5)
MEC_BM_INSTANTIATE_W(6)
MEC_BM_INSTANTIATE_W(7)
MEC_BM_INSTANTIATE_W(8)
}  // namespace detail
}  // namespace mec
