// gf8_r4lo.hip — GF(2^8) kernel instantiations with 4 output row(s), K = 1..16.
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
MEC_GF8_INSTANTIATE_LO(4)
}  // namespace detail
}  // namespace mec
