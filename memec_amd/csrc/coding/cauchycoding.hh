// cauchycoding.hh — Cauchy-RS coding on the MI355X.  Same class name and
// constructor as common/coding/cauchycoding.hh:7-46.
#ifndef MEMEC_AMD_CAUCHYCODING_HH
#define MEMEC_AMD_CAUCHYCODING_HH

#include "gpu_coding.hh"

#define CRS_N_MAX (32)

class CauchyCoding : public GpuMatrixCoding {
public:
    CauchyCoding(uint32_t k = 0, uint32_t m = 0, uint32_t chunkSize = 0);
};

#endif
