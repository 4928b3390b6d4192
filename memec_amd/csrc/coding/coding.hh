// coding.hh — MemEC's coding plugin surface (common/coding/coding.hh:9-61),
// kept signature-for-signature so server/ links it unchanged.  RSCoding and
// CauchyCoding forward to libmec (include/mec.h): the chunks stay where the
// caller keeps them (host memory), the arithmetic runs on the MI355X.
#ifndef MEMEC_AMD_CODING_HH
#define MEMEC_AMD_CODING_HH

#include <stdint.h>

#include "boundary.hh"
#include "coding_params.hh"

class Coding {
public:
    CodingScheme scheme;
    static Chunk *zeros;

    virtual ~Coding();
    // Write parity number `index` (1-based) of the stripe data[0..k-1] into
    // parity's data area.  data[j] may be Coding::zeros.  startOff/endOff
    // are stripe-global byte offsets; they select columns only in the ISA-L
    // build (rscoding.cc:81-89), as in the reference.
    virtual void encode(Chunk **data, Chunk *parity, uint32_t index, uint32_t startOff = 0,
                        uint32_t endOff = 0) = 0;
    // Rebuild, in place, every chunk whose bit is clear in bitmap.  False iff
    // more than m chunks are missing (or the device call failed).
    virtual bool decode(Chunk **chunks, BitmaskArray *bitmap) = 0;

    static Coding *instantiate(CodingScheme scheme, CodingParams &params, uint32_t chunkSize);
    static void destroy(Coding *coding);

    static char *bitwiseXOR(char *dst, char *srcA, char *srcB, uint32_t len);
    static Chunk *bitwiseXOR(Chunk *dst, Chunk *srcA, Chunk *srcB, uint32_t size);

    static uint32_t forceSeal(Coding *coding, Chunk **chunks, Chunk *tmpParityChunk, bool **sealIndicator,
                              uint32_t dataChunkCount, uint32_t parityChunkCount);
};

#endif
