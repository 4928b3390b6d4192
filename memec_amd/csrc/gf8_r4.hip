// gf8_r4.hip — GF(2^8) kernel instantiations with 4 output row(s).
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
MEC_GF8_INSTANTIATE_K(4)
}  // namespace detail
}  // namespace mec
