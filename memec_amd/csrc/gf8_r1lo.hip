// gf8_r1lo.hip — GF(2^8) kernel instantiations with 1 output row(s), K = 1..16.
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
MEC_GF8_INSTANTIATE_LO(1)
}  // namespace detail
}  // namespace mec
