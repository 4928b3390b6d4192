// cauchycoding.cc — CauchyCoding (common/coding/cauchycoding.cc:20-39):
// Jerasure cauchy_good_general_coding_matrix as a w-packet bitmatrix, or
// ISA-L gf_gen_cauchy1_matrix with -DUSE_ISAL.
#include "cauchycoding.hh"

CauchyCoding::CauchyCoding(uint32_t k, uint32_t m, uint32_t chunkSize)
#ifdef USE_ISAL
    : GpuMatrixCoding(MEC_ISAL_CAUCHY, "Cauchy coding", k, m, chunkSize)
#else
    : GpuMatrixCoding(MEC_CAUCHY_GOOD, "Cauchy coding", k, m, chunkSize)
#endif
{
}
