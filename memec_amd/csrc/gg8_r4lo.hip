// gg8_r4lo.hip — gathered GF(2^8) kernel instantiations, 4 output row(s), K = 1..16.
#include "gather_kernel.hpp"

namespace mec {
namespace detail {
MEC_GG8_INSTANTIATE_LO(4)
}  // namespace detail
}  // namespace mec
