// gf8_r3lo.hip — GF(2^8) kernel instantiations with 3 output row(s), K = 1..16.
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
MEC_GF8_INSTANTIATE_LO(3)
}  // namespace detail
}  // namespace mec
