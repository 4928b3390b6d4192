// gg8_r1hi.hip — gathered GF(2^8) kernel instantiations, 1 output row(s), K = 17..32.
#include "gather_kernel.hpp"

namespace mec {
namespace detail {
MEC_GG8_INSTANTIATE_HI(1)
}  // namespace detail
}  // namespace mec
