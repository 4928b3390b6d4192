// gg8_r3lo.hip — gathered GF(2^8) kernel instantiations, 3 output row(s), K = 1..16.
#include "gather_kernel.hpp"

namespace mec {
namespace detail {
MEC_GG8_INSTANTIATE_LO(3)
}  // namespace detail
}  // namespace mec
