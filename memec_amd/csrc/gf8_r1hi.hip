// gf8_r1hi.hip — GF(2^8) kernel instantiations with 1 output row(s), K = 17..32.
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
MEC_GF8_INSTANTIATE_HI(1)
}  // namespace detail
}  // namespace mec
