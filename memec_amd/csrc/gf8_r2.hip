// gf8_r2.hip — GF(2^8) kernel instantiations with 2 output row(s).
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
MEC_GF8_INSTANTIATE_K(2)
}  // namespace detail
}  // namespace mec
