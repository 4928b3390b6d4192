// gf8_r1.hip — GF(2^8) kernel instantiations with 1 output row(s).
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
MEC_GF8_INSTANTIATE_K(1)
}  // namespace detail
}  // namespace mec
