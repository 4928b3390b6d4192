// gf8_r2hi.hip — GF(2^8) kernel instantiations with 2 output row(s), K = 17..32.
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
MEC_GF8_INSTANTIATE_HI(2)
}  // namespace detail
}  // namespace mec
