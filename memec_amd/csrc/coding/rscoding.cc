// rscoding.cc — RSCoding (common/coding/rscoding.cc:20-43): Jerasure
// reed_sol_vandermonde_coding_matrix over GF(2^8), or ISA-L
// gf_gen_rs_matrix with -DUSE_ISAL.
#include "rscoding.hh"

RSCoding::RSCoding(uint32_t k, uint32_t m, uint32_t chunkSize)
#ifdef USE_ISAL
    : GpuMatrixCoding(MEC_ISAL_RS, "RS coding", k, m, chunkSize)
#else
    : GpuMatrixCoding(MEC_RS_VANDERMONDE, "RS coding", k, m, chunkSize)
#endif
{
}
