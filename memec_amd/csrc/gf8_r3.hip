// gf8_r3.hip — GF(2^8) kernel instantiations with 3 output row(s).
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
MEC_GF8_INSTANTIATE_K(3)
}  // namespace detail
}  // namespace mec
