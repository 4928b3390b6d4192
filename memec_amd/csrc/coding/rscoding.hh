// rscoding.hh — RS (Vandermonde) coding on the MI355X.  Same class name and
// constructor as common/coding/rscoding.hh:7-43.
#ifndef MEMEC_AMD_RSCODING_HH
#define MEMEC_AMD_RSCODING_HH

#include "gpu_coding.hh"

#define RS_N_MAX (32)

class RSCoding : public GpuMatrixCoding {
public:
    RSCoding(uint32_t k = 0, uint32_t m = 0, uint32_t chunkSize = 0);
};

#endif
