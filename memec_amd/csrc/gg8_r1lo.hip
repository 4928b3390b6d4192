// gg8_r1lo.hip — gathered GF(2^8) kernel instantiations, 1 output row(s), K = 1..16.
#include "gather_kernel.hpp"

namespace mec {
namespace detail {
MEC_GG8_INSTANTIATE_LO(1)
}  // namespace detail
}  // namespace mec
