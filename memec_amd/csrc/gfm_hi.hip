// gfm_hi.hip — multi-group GF(2^8) kernel instantiations (m > 4 outputs in one
// pass, gf8_mg_kernel), 3 and 4 rows per group, K = 17..31.
#include "gf8_kernel.hpp"

namespace mec {
namespace detail {
MEC_FOR_K_HI(MEC_GFM_ONE, 3)
MEC_FOR_K_HI(MEC_GFM_ONE, 4)
}  // namespace detail
}  // namespace mec
