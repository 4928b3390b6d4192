// gpu_coding.hh — shared implementation of RSCoding / CauchyCoding over a
// libmec context.  One instance is shared by every server worker thread
// (server.cc:107, worker.cc:128-137); libmec is reentrant (per-call staging
// lanes, read-only matrices, a locked plan cache).
#ifndef MEMEC_AMD_GPU_CODING_HH
#define MEMEC_AMD_GPU_CODING_HH

#include "coding.hh"
#include "mec.h"

class GpuMatrixCoding : public Coding {
public:
    ~GpuMatrixCoding();
    void encode(Chunk **dataChunks, Chunk *parityChunk, uint32_t index, uint32_t startOff = 0,
                uint32_t endOff = 0);
    bool decode(Chunk **chunks, BitmaskArray *chunkStatus);

    uint32_t k() const { return _k; }
    uint32_t m() const { return _m; }
    mec_ctx *context() const { return _ctx; }

protected:
    // family: MEC_RS_VANDERMONDE / MEC_CAUCHY_GOOD, or the ISA-L matrices when
    // the adapter is built with -DUSE_ISAL (the reference's switch, Makefile:3).
    GpuMatrixCoding(int family, const char *name, uint32_t k, uint32_t m, uint32_t chunkSize);

private:
    void encode_failed(int rc) const;

    const char *_name;
    int _family;
    uint32_t _k, _m, _chunkSize;
    mec_ctx *_ctx;
};

#endif
