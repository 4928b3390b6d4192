// boundary.hh — the MemEC boundary types the Coding plugin touches
// (SURVEY §8 a14).  Inside a MemEC tree (MEMEC_TREE: detected below, or
// defined) the real headers are used; standalone builds (tests, the
// GPU box) get these equivalents with the same layout and semantics:
//   Chunk        char*: [8-byte ChunkIdentifier][chunkSize data bytes]
//                (common/ds/chunk.hh:11-31)
//   ChunkUtil    getData = chunk + 8, clear, chunkSize (chunk_util.hh:131-307)
//   TempChunkPool  zeroed malloc'd chunk (chunk_pool.hh:38-53)
//   BitmaskArray check(i) = bit i of entry 0 (bitmask_array.cc:6-62)
#ifndef MEMEC_AMD_CODING_BOUNDARY_HH
#define MEMEC_AMD_CODING_BOUNDARY_HH

// Inside a MemEC tree the adapter sits in common/coding/ next to ../ds/:
// detect that, so the reference's own code (server/, the coding tests)
// compiles against the adapter headers with its unchanged flags.
#if !defined(MEMEC_TREE) && defined(__has_include)
#if __has_include("../ds/chunk_util.hh")
#define MEMEC_TREE 1
#endif
#endif

#ifdef MEMEC_TREE
// As the reference's coding.hh:4-7: only chunk.hh and bitmask_array.hh
// here — ds/chunk_util.hh includes coding/coding.hh itself, so the
// adapter's .cc files include chunk_util.hh / chunk_pool.hh (boundary_ds.hh).
#include "../ds/bitmask_array.hh"
#include "../ds/chunk.hh"
#else
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef char *Chunk;
#define CHUNK_IDENTIFIER_SIZE 8

class ChunkUtil {
public:
    static uint32_t chunkSize;
    static uint32_t dataChunkCount;
    static inline void init(uint32_t cs, uint32_t dataCount) {
        chunkSize = cs;
        dataChunkCount = dataCount;
    }
    static inline char *getData(Chunk *chunk) { return ((char *)chunk) + CHUNK_IDENTIFIER_SIZE; }
    static inline void clear(Chunk *chunk) { memset((char *)chunk, 0, CHUNK_IDENTIFIER_SIZE + chunkSize); }
    static inline void copy(Chunk *chunk, uint32_t offset, char *src, uint32_t n) {
        memcpy(getData(chunk) + offset, src, n);
    }
};

class TempChunkPool {
public:
    Chunk *alloc(uint32_t = 0, uint32_t = 0, uint32_t = 0) {
        Chunk *c = (Chunk *)malloc(CHUNK_IDENTIFIER_SIZE + ChunkUtil::chunkSize);
        if (c) ChunkUtil::clear(c);
        return c;
    }
    void free(Chunk *chunk) { ::free((char *)chunk); }
};

class BitmaskArray {
public:
    BitmaskArray(size_t size, size_t count) : size_(size) {
        size_t bits = size * count;
        words_ = (bits + 63) / 64;
        masks_ = (uint64_t *)calloc(words_ ? words_ : 1, sizeof(uint64_t));
    }
    ~BitmaskArray() { ::free(masks_); }
    void set(size_t entry, size_t bit) { at(entry, bit) |= one(entry, bit); }
    void unset(size_t entry, size_t bit) { at(entry, bit) &= ~one(entry, bit); }
    bool check(size_t entry, size_t bit) { return at(entry, bit) & one(entry, bit); }
    void set(size_t bit) { set(0, bit); }
    void unset(size_t bit) { unset(0, bit); }
    bool check(size_t bit) { return check(0, bit); }

private:
    BitmaskArray(const BitmaskArray &);
    uint64_t &at(size_t e, size_t b) { return masks_[(e * size_ + b) >> 6]; }
    uint64_t one(size_t e, size_t b) const { return uint64_t(1) << ((e * size_ + b) & 63); }
    size_t size_, words_;
    uint64_t *masks_;
};
#endif

#endif
