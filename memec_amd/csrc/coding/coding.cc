// coding.cc — Coding factory and static helpers (common/coding/coding.cc).
#include "boundary_ds.hh"

#include <stdio.h>
#include <string.h>

#include "cauchycoding.hh"
#include "rscoding.hh"

#ifdef MEMEC_TREE
#include "raid0coding.hh"
#include "raid1coding.hh"
#include "raid5coding.hh"
#include "rdpcoding.hh"
#include "evenoddcoding.hh"
#else
uint32_t ChunkUtil::chunkSize;
uint32_t ChunkUtil::dataChunkCount;
#endif

Chunk *Coding::zeros;

Coding::~Coding() {}

// coding.cc:12-54.  Also records the scheme, which the reference never
// assigns (Appendix B #1), so destroy() is well defined.
Coding *Coding::instantiate(CodingScheme scheme, CodingParams &params, uint32_t chunkSize) {
    ChunkUtil::chunkSize = chunkSize;
    TempChunkPool tempChunkPool;
    Coding::zeros = tempChunkPool.alloc();

    Coding *coding = 0;
    switch (scheme) {
        case CS_RS:
            coding = new RSCoding(params.getK(), params.getM(), chunkSize);
            break;
        case CS_CAUCHY:
            coding = new CauchyCoding(params.getK(), params.getM(), chunkSize);
            break;
#ifdef MEMEC_TREE
        // The XOR codes are outside the accelerated path; the reference
        // implementations are kept as they are.
        case CS_RAID0: {
            RAID0Coding *c = new RAID0Coding();
            c->init(params.getN());
            coding = c;
            break;
        }
        case CS_RAID1: {
            RAID1Coding *c = new RAID1Coding();
            c->init(params.getN());
            coding = c;
            break;
        }
        case CS_RAID5: {
            RAID5Coding *c = new RAID5Coding();
            c->init(params.getN());
            coding = c;
            break;
        }
        case CS_RDP:
            coding = new RDPCoding(params.getK(), chunkSize);
            break;
        case CS_EVENODD:
            coding = new EvenOddCoding(params.getK(), chunkSize);
            break;
#endif
        default:
            fprintf(stderr, "[ERROR] Coding::instantiate(): Coding scheme is not yet implemented.\n");
            return 0;
    }
    coding->scheme = scheme;
    return coding;
}

void Coding::destroy(Coding *coding) {
    if (!coding) return;
    delete coding;  // virtual destructor
    if (Coding::zeros) {
        free(Coding::zeros);
        Coding::zeros = 0;
    }
}

// coding.cc:88-108: dst = a ^ b, 64-bit words then bytes.  Host memory: the
// server applies parity deltas to chunks it holds in its own buffers.
char *Coding::bitwiseXOR(char *dst, char *srcA, char *srcB, uint32_t len) {
    uint32_t i = 0;
    for (; i + 8 <= len; i += 8) {
        uint64_t a, b;
        memcpy(&a, srcA + i, 8);
        memcpy(&b, srcB + i, 8);
        a ^= b;
        memcpy(dst + i, &a, 8);
    }
    for (; i < len; i++) dst[i] = srcA[i] ^ srcB[i];
    return dst;
}

Chunk *Coding::bitwiseXOR(Chunk *dst, Chunk *srcA, Chunk *srcB, uint32_t size) {
    Coding::bitwiseXOR(ChunkUtil::getData(dst), ChunkUtil::getData(srcA), ChunkUtil::getData(srcB), size);
    return dst;
}

// coding.cc:120-185, unchanged caller-level logic.  It passes the 0-based
// parity loop index as encode()'s 1-based `index` (Appendix B #11); that is
// the caller's behaviour and is kept as is — encode() honours its contract.
uint32_t Coding::forceSeal(Coding *coding, Chunk **chunks, Chunk *tmpParityChunk, bool **sealIndicator,
                           uint32_t dataChunkCount, uint32_t parityChunkCount) {
    Chunk **tmpChunks = new Chunk *[dataChunkCount];
    bool *trueSealIndicator = sealIndicator[parityChunkCount];
    uint32_t fixed = 0;

    for (uint32_t j = 0; j < dataChunkCount; j++) {
        uint32_t count = 0, total = 0;
        char indicator = -1;
        for (uint32_t i = 0; i < parityChunkCount; i++) {
            if (!chunks[i + dataChunkCount]) continue;
            total++;
            if (sealIndicator[i][j]) count++;
            indicator = sealIndicator[i][j];
        }
        if ((count == 0 || count == total) && indicator != trueSealIndicator[j]) {
            chunks[j] = Coding::zeros;
            trueSealIndicator[j] = false;
        }
    }
    for (uint32_t i = 0; i < parityChunkCount; i++) {
        if (!chunks[i + dataChunkCount]) continue;
        for (uint32_t j = 0; j < dataChunkCount; j++) {
            if (sealIndicator[i][j] == trueSealIndicator[j]) continue;
            for (uint32_t x = 0; x < dataChunkCount; x++) tmpChunks[x] = (x == j) ? chunks[j] : Coding::zeros;
            ChunkUtil::clear(tmpParityChunk);
            coding->encode(tmpChunks, tmpParityChunk, i, 0, ChunkUtil::chunkSize);
            char *parity = ChunkUtil::getData(chunks[i + dataChunkCount]);
            Coding::bitwiseXOR(parity, parity, ChunkUtil::getData(tmpParityChunk), ChunkUtil::chunkSize);
            sealIndicator[i][j] = true;
            fixed++;
        }
    }
    delete[] tmpChunks;
    return fixed;
}
