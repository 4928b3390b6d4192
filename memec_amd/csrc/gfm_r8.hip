// gfm_r8.hip — multi-group GF(2^8) kernel instantiations with 8-row groups
// (gf8_mg_kernel, K = kMg8MinK..kMg8MaxK; gf8_mg_rows picks them).
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
MEC_FOR_K8(MEC_GFM_ONE)
}  // namespace detail
}  // namespace mec
