// gf8_r4hi.hip — GF(2^8) kernel instantiations with 4 output row(s), K = 17..32.
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
MEC_GF8_INSTANTIATE_HI(4)
}  // namespace detail
}  // namespace mec
